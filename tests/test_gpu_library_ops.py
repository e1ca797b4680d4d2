"""torch.library registrations (scattennet_amd/library.py): the operators
torch.ops.scatten.* against the CPU oracle / torch references, forward and autograd, plus a
CPU-side check that they are registered with fake (meta) implementations."""
import pytest
import torch

from oracle import sca_oracle as O
from tests.golden_util import rel_err

PARITY_TOL = 1e-3


def test_ops_registered_with_fake_impls():
    import scattennet_amd  # noqa: F401
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        q = torch.empty(2, 8, 32)
        o, sm, sl = torch.ops.scatten.masked_attention(q, q, q, None, 2)
        assert o.shape == q.shape and sm.shape == (2 * 2 * 8,)
        y, m, r = torch.ops.scatten.layer_norm(q, torch.empty(32), torch.empty(32), 1e-5)
        assert y.shape == q.shape and m.shape == (16,)
        kp = torch.empty(2, 5, 10, 2)
        assert torch.ops.scatten.normalize_keypoints(kp, torch.empty(2), torch.empty(3), torch.empty(4)).shape == kp.shape


def test_ops_reject_cpu_tensors():
    import scattennet_amd  # noqa: F401
    q = torch.randn(2, 8, 32)
    with pytest.raises(RuntimeError):
        torch.ops.scatten.masked_attention(q, q, q, None, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_masked_attention_op_vs_torch(causal):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import scattennet_amd  # noqa: F401
    torch.manual_seed(5)
    B, T, H, hd = 3, 70, 4, 16
    d = H * hd
    q, k, v = (torch.randn(B, T, d) for _ in range(3))
    mask = torch.ones(B, T, dtype=torch.long)
    mask[1, 30:] = 0
    mask[2, :] = 0
    dev = "cuda"
    qg, kg, vg = (t.to(dev).requires_grad_(True) for t in (q, k, v))
    o = torch.ops.scatten.masked_attention(qg, kg, vg, (mask != 0).float().to(dev), H, causal, causal)[0]
    g = torch.randn(B, T, d)
    o.backward(g.to(dev))
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    am = O.additive_causal_mask(mask) if causal else O.additive_key_mask(mask, tgt_len=T)

    def split(t):
        return t.view(B, T, H, hd).transpose(1, 2)
    s = split(qr) @ split(kr).transpose(-1, -2)
    if causal:
        s = s.masked_fill(~torch.ones(T, T, dtype=torch.bool).tril(), float("-inf"))
    ref = (torch.softmax(s + am, dim=-1) @ split(vr)).transpose(1, 2).reshape(B, T, d)
    assert rel_err(o, ref) < PARITY_TOL
    (ref * g).sum().backward()
    for got, want in ((qg, qr), (kg, kr), (vg, vr)):
        assert rel_err(got.grad, want.grad) < PARITY_TOL


@pytest.mark.gpu
def test_layer_norm_and_normalize_ops():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import numpy as np
    import scattennet_amd  # noqa: F401
    torch.manual_seed(6)
    x, w, b = torch.randn(37, 256), torch.randn(256), torch.randn(256)
    xg, wg, bg = (t.cuda().requires_grad_(True) for t in (x, w, b))
    y = torch.ops.scatten.layer_norm(xg, wg, bg, 1e-5)[0]
    g = torch.randn(37, 256)
    y.backward(g.cuda())
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    ref = torch.nn.functional.layer_norm(xr, (256,), wr, br, 1e-5)
    (ref * g).sum().backward()
    assert rel_err(y, ref) < PARITY_TOL
    for got, want in ((xg, xr), (wg, wr), (bg, br)):
        assert rel_err(got.grad, want.grad) < PARITY_TOL
    parts = [list(range(3)), list(range(3, 9))]
    kp = np.random.default_rng(0).uniform(0, 1, size=(2, 4, 9, 2)).astype(np.float32)
    off = torch.tensor([0, 3, 9], dtype=torch.int32, device="cuda")
    idx = torch.arange(9, dtype=torch.int32, device="cuda")
    got = torch.ops.scatten.normalize_keypoints(torch.from_numpy(kp).cuda(), torch.tensor([4, 2], device="cuda"),
                                               off, idx)
    want = np.stack([O.normalize_keypoints(kp[0], parts), np.concatenate([O.normalize_keypoints(kp[1, :2], parts),
                                                                          np.zeros_like(kp[1, 2:])])])
    np.testing.assert_allclose(got.cpu().numpy(), want, rtol=1e-5, atol=1e-6)


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.gpu
def test_block_ops_opcheck():
    """torch.library.opcheck (schema, fake tensors, autograd registration) of every block
    operator on real device tensors."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import scattennet_amd  # noqa: F401
    dev = "cuda"
    torch.manual_seed(3)
    B, T, d, H, F = 2, 24, 64, 4, 128

    def r(*s, g=True):
        return (torch.randn(*s, device=dev) * 0.3).requires_grad_(g)
    x, kv = r(B, T, d), r(B, 17, d)
    p8 = [r(d, d), r(d)] * 3 + [r(d, d), r(d)]
    kvalid = torch.ones(B, T, device=dev)
    kvalid[1, 20:] = 0
    kv17 = torch.ones(B, 17, device=dev)
    tests = "test_schema", "test_faketensor", "test_autograd_registration"
    S = torch.ops.scatten
    torch.library.opcheck(S.attention_block, (x, None, p8, r(d), r(d), kvalid, None, "self", H, 0.25, False, True,
                                              1e-5), test_utils=tests)
    torch.library.opcheck(S.attention_block, (x, kv, p8, None, None, kv17, None, "cross", H, 0.25, False, True, -1.0),
                          test_utils=tests)
    torch.library.opcheck(S.feed_forward, (x, [r(F, d), r(F), r(d, F), r(d)], r(d), r(d), True, 1e-5),
                          test_utils=tests)
    # d_model 256: the LayerNorms fused into the GEMM launches
    D = 256
    x2 = r(B, T, D)
    p8w = [r(D, D), r(D)] * 4
    torch.library.opcheck(S.attention_block, (x2, None, p8w, r(D), r(D), kvalid, None, "causal", 16, 0.25, True, True,
                                              1e-5), test_utils=tests)
    torch.library.opcheck(S.feed_forward, (x2, [r(2 * D, D), r(2 * D), r(D, 2 * D), r(D)], r(D), r(D), True, 1e-5),
                          test_utils=tests)
    torch.library.opcheck(S.linear, (x, r(F, d), r(F), None, True), test_utils=tests)
    torch.library.opcheck(S.layer_norm_ex, (x, r(T + 2, d), None, r(d), r(d), 1e-5, False), test_utils=tests)
    torch.library.opcheck(S.layer_norm_ex, (x, None, r(B, T, d), r(d), r(d), 1e-5, True), test_utils=tests)
    torch.library.opcheck(S.maxpool_t, (r(B, T, d),), test_utils=tests)
    torch.library.opcheck(S.clip_matmul, (r(B, 8, d), r(B, 12, d), True), test_utils=tests)
    torch.library.opcheck(S.softmax_rows, (r(B, 8, 12),), test_utils=tests)
    kp = torch.rand(B, T, 9, 2, device=dev)
    torch.library.opcheck(S.coordinate_mapping, (kp, torch.tensor([0, 3, 5, 8], dtype=torch.int32, device=dev),
                                                 r(d, 4), r(d), r(d, 4), r(d)), test_utils=tests)


@pytest.mark.gpu
def test_compiled_sca_stack_matches_eager():
    """The drop-in SCA stack under torch.compile (aot_eager, one graph of scatten operators,
    one stream per launch) against the eager grouped launches: outputs and every gradient."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import scattennet_amd as S
    from scattennet_amd import workloads as W
    torch.manual_seed(4)
    d, H, T, B = 256, 16, 64, 3
    cfg = W.model_cfg(d, H, 2, maxpos=T)
    sca = S.SeparativeCoordinateAttention(cfg).eval().cuda()
    x0, y0 = torch.randn(B, T, d, device="cuda"), torch.randn(B, T, d, device="cuda")
    mask = torch.ones(B, T, dtype=torch.long, device="cuda")
    mask[1, 40:] = 0
    gout = torch.randn(B, T, d, device="cuda")

    def run(fn):
        for p in sca.parameters():
            p.grad = None
        x, y = x0.clone().requires_grad_(True), y0.clone().requires_grad_(True)
        out = fn(x, y)
        (out * gout).sum().backward()
        torch.cuda.synchronize()
        return out.detach(), x.grad, y.grad, {k: p.grad.clone() for k, p in sca.named_parameters()}

    want = run(lambda a, b: sca(a, b, mask))
    torch._dynamo.reset()
    got = run(torch.compile(lambda a, b: sca(a, b, mask), backend="aot_eager", fullgraph=True))
    torch._dynamo.reset()
    assert _rel(got[0], want[0]) < 1e-4
    assert _rel(got[1], want[1]) < 1e-4 and _rel(got[2], want[2]) < 1e-4
    for k in want[3]:  # (k_proj.bias: analytically zero, compared at the noise level)
        assert float((got[3][k] - want[3][k]).abs().max()) <= 1e-4 * float(want[3][k].abs().max()) + 1e-6, k


@pytest.mark.gpu
@pytest.mark.parametrize("off,n", [(0, 0), (0, 1), (1, 3), (3, 7), (0, 4096), (1, 4096 * 33 + 5), (2, 258 * 256 * 4)])
def test_sca_zero_writes_exactly_its_range(off, n):
    """sca_zero: p[0 .. n) = 0 at any 4-byte alignment (scalar head / tail around float4 stores),
    nothing outside it touched — the position-table gradient's buffer in the captured step."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from scattennet_amd import _lib as L
    buf = torch.full((off + n + 9,), float("nan"), device="cuda")
    assert L.lib().sca_zero(buf.data_ptr() + 4 * off, n, L.stream_handle()) == 0
    torch.cuda.synchronize()
    assert torch.equal(buf[off:off + n], torch.zeros(n, device="cuda"))
    assert torch.isnan(buf[:off]).all() and torch.isnan(buf[off + n:]).all()
