"""Attention-mask contract at the drop-in boundary (model/attention.py:65/117/171:
`attn_weights += attention_mask`).

Every additive mask the reference accepts — anything broadcastable to (B, H, Tq, Tk) — is
expanded to the kernels' dense layout before a launch: (B, Tq, Tk) when it is the same for
every head, (B, H, Tq, Tk) when it is per head (mask_heads = H in the C ABI); shapes the
reference would reject raise; `None` raises TypeError as `attn_weights += None` does.  CPU
tests cover the host-side resolution; the GPU test runs the broadcast shapes, per-head ones
included, through the HIP kernels against the oracle.
"""
import pytest
import torch

from oracle import sca_oracle as O
from tests.golden_util import close, rel_err

PARITY_TOL = 1e-3


def _resolve(mask, causal=False, B=3, Tq=5, Tk=7, H=4):
    from scattennet_amd.attention import _resolve_mask
    return _resolve_mask(mask, causal, B, Tq, Tk, torch.device("cpu"), H)


@pytest.mark.parametrize("shape", [(3, 1, 5, 7), (1, 1, 5, 7), (3, 1, 1, 7), (5, 7), (7,), (1, 5, 1), ()])
def test_broadcast_masks_expand_to_dense(shape):
    m = torch.randn(shape)
    kv, am, plus = _resolve(m)
    assert kv is None and not plus
    assert am.shape == (3, 5, 7) and am.is_contiguous() and am.dtype == torch.float32
    want = m.reshape((1,) * (4 - m.dim()) + tuple(m.shape)).expand(3, 1, 5, 7)[:, 0]
    assert torch.equal(am, want)


@pytest.mark.parametrize("shape", [(3, 4, 5, 7), (1, 4, 5, 7), (3, 4, 1, 7), (4, 1, 1)])
def test_per_head_masks_expand_to_dense(shape):
    m = torch.randn(shape)
    kv, am, plus = _resolve(m)
    assert kv is None and not plus
    assert am.shape == (3, 4, 5, 7) and am.is_contiguous()
    assert torch.equal(am, m.reshape((1,) * (4 - m.dim()) + tuple(m.shape)).expand(3, 4, 5, 7))


@pytest.mark.parametrize("shape", [(3, 2, 5, 7), (2, 1, 5, 7), (3, 1, 4, 7), (5, 6), (1, 3, 1, 5, 7)])
def test_non_broadcastable_masks_raise(shape):
    with pytest.raises(ValueError):
        _resolve(torch.zeros(shape))


def test_none_mask_raises_type_error():
    with pytest.raises(TypeError):
        _resolve(None)


def test_key_padding_mask_shape_checked():
    from scattennet_amd.utils import key_padding_mask
    kv, am, plus = _resolve(key_padding_mask(torch.ones(3, 7, dtype=torch.long), causal=True), causal=True)
    assert kv.shape == (3, 7) and am is None and plus
    with pytest.raises(ValueError):
        _resolve(key_padding_mask(torch.ones(2, 7, dtype=torch.long)))


def test_bool_and_int_masks_add_like_the_reference():
    m = torch.tensor([[True, False, True, True, False, True, True]])
    _, am, _ = _resolve(m)
    assert torch.equal(am[0, 0], m[0].float())


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["self", "causal", "cross"])
@pytest.mark.parametrize("form", ["B1TT", "11TT", "B11T", "TT", "BHTT", "1HTT"])
def test_gpu_broadcast_masks_vs_oracle(kind, form):
    import scattennet_amd as S
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda:0")
    B, Tq, d, H = 3, 48, 64, 4
    Tk = 40 if kind == "cross" else Tq
    torch.manual_seed(17 * len(kind) + len(form))
    cls = {"self": S.SelfAttention, "causal": S.SelfCausalAttention, "cross": S.CrossAttention}[kind]
    m = cls(d, H)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) / (p.shape[-1] ** 0.5 if p.dim() == 2 else 10.0))
    m = m.to(dev)
    shape = {"B1TT": (B, 1, Tq, Tk), "11TT": (1, 1, Tq, Tk), "B11T": (B, 1, 1, Tk), "TT": (Tq, Tk),
             "BHTT": (B, H, Tq, Tk), "1HTT": (1, H, Tq, Tk)}[form]
    # additive masks in the reference's vocabulary: finfo.min on dropped keys, small offsets elsewhere
    am = torch.randn(shape) * 0.5
    drop = torch.rand(shape) < 0.3
    am = am.masked_fill(drop, O.FMIN)
    x, kv = torch.randn(B, Tq, d), torch.randn(B, Tk, d)
    xg, kvg = x.to(dev).requires_grad_(True), kv.to(dev).requires_grad_(True)
    out = m(xg, kvg, am.to(dev)) if kind == "cross" else m(xg, am.to(dev))
    gout = torch.randn(out.shape)
    out.backward(gout.to(dev))

    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    xr, kvr = x.clone().requires_grad_(True), kv.clone().requires_grad_(True)
    ref = O.attention({"a." + k: v for k, v in p.items()}, "a", xr, kvr if kind == "cross" else xr, am, H, kind)
    assert rel_err(out, ref) < PARITY_TOL
    (ref * gout).sum().backward()
    assert rel_err(xg.grad, xr.grad) < PARITY_TOL
    if kind == "cross":
        assert rel_err(kvg.grad, kvr.grad) < PARITY_TOL
    gscale = max(float(v.grad.abs().max()) for v in p.values())
    named = dict(m.named_parameters())
    for k, v in p.items():
        assert close(named[k].grad.cpu(), v.grad, PARITY_TOL, gscale), (k, rel_err(named[k].grad.cpu(), v.grad))


@pytest.mark.gpu
def test_gpu_none_mask_raises():
    import scattennet_amd as S
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    m = S.SelfAttention(64, 4).cuda()
    with pytest.raises(TypeError):
        m(torch.randn(2, 8, 64, device="cuda"), None)


# ---- the key-validity predicate (model/utils.py:8-12, 19-23): keep a key only where the fp32
# mask value is exactly 1 — 1.0 - mask is masked wherever it is non-zero ----
ODD_VALUES = [1.0, 2.0, 0.5, 0.0, -1.0, 1.0, 3.0, 1.0]


def test_key_valid_predicate_matches_the_reference_masks():
    """The traced / host form of the predicate against the oracle's restatement of
    create_attention_mask: a key is kept exactly where the additive mask is 0."""
    from scattennet_amd.ops import key_valid_vector
    for dtype in (torch.float32, torch.float64, torch.int64, torch.int32, torch.float16, torch.bfloat16):
        m = torch.tensor([ODD_VALUES, ODD_VALUES[::-1]]).to(dtype)
        kv = key_valid_vector(m)
        want = (O.additive_key_mask(m)[:, 0, 0] == 0).float()
        assert torch.equal(kv, want), dtype
    nan = torch.tensor([[1.0, float("nan"), 1.0]])
    assert torch.equal(key_valid_vector(nan), torch.tensor([[1.0, 0.0, 1.0]]))
    assert torch.equal(key_valid_vector(torch.tensor([[True, False]])), torch.tensor([[1.0, 0.0]]))


@pytest.mark.gpu
def test_gpu_key_valid_kernel_every_dtype():
    """sca_key_valid (one launch, no ATen) against the reference predicate for every mask dtype."""
    from scattennet_amd.ops import key_valid_vector
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    g = torch.Generator().manual_seed(3)
    vals = torch.tensor([1.0, 2.0, 0.5, 0.0, -1.0, 3.0, 1.0 + 2 ** -20])
    m = vals[torch.randint(0, len(vals), (5, 301), generator=g)]
    m[:, ::3] = 1.0
    for dtype in (torch.float32, torch.float64, torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8,
                  torch.bool, torch.float16, torch.bfloat16):
        md = m.to(dtype)
        want = (O.additive_key_mask(md)[:, 0, 0] == 0).float()
        got = key_valid_vector(md.cuda())
        assert torch.equal(got.cpu(), want), dtype
    assert key_valid_vector(torch.empty(0, 4, dtype=torch.long, device="cuda")).shape == (0, 4)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.int64, torch.float32])
def test_gpu_sca_stack_with_non_binary_mask_vs_oracle(dtype):
    """The SCA stack fed a (B, T) mask holding 2, 0.5, -1 besides 0 / 1: keys are kept only
    where the mask is 1, as the reference's mask builders decide (model/utils.py:3-28)."""
    import scattennet_amd as S
    from scattennet_amd import workloads as W
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda:0")
    torch.manual_seed(5)
    B, T, d, H = 3, 40, 64, 4
    cfg = W.model_cfg(d, H, 2, maxpos=T)
    sca = S.SeparativeCoordinateAttention(cfg).eval()
    vals = torch.tensor([1.0, 1.0, 1.0, 2.0, 0.5, 0.0, -1.0])
    mask = vals[torch.randint(0, len(vals), (B, T))]
    mask[0, :5] = 1.0
    mask[1] = 2.0  # every key of clip 1 masked: uniform attention, as in the reference
    if dtype == torch.int64:
        mask = mask.round().to(torch.int64)  # 0.5 -> 0 (masked), 2 / -1 kept as such
    x, y = torch.randn(B, T, d), torch.randn(B, T, d)
    p = {k: v.detach().clone().requires_grad_(True) for k, v in sca.state_dict().items()}
    sca = sca.to(dev)
    xg, yg = x.to(dev).requires_grad_(True), y.to(dev).requires_grad_(True)
    out = sca(xg, yg, mask.to(dev))
    gout = torch.randn(out.shape)
    out.backward(gout.to(dev))
    xr, yr = x.clone().requires_grad_(True), y.clone().requires_grad_(True)
    ref = O.sca({"s." + k: v for k, v in p.items()}, "s", xr, yr, mask, cfg)
    assert rel_err(out, ref) < PARITY_TOL
    (ref * gout).sum().backward()
    assert rel_err(xg.grad, xr.grad) < PARITY_TOL and rel_err(yg.grad, yr.grad) < PARITY_TOL
    gscale = max(float(v.grad.abs().max()) for v in p.values() if v.grad is not None)
    named = dict(sca.named_parameters())
    for k, v in p.items():
        if v.grad is not None:
            assert close(named[k].grad.cpu(), v.grad, PARITY_TOL, gscale), (k, rel_err(named[k].grad.cpu(), v.grad))
    # and the result differs from treating every non-zero as "keep" (the old predicate)
    ref_nz = O.sca({"s." + k: v.detach() for k, v in p.items()}, "s", x, y, (mask != 0).long(), cfg)
    assert rel_err(ref_nz, ref.detach()) > 1e-2
