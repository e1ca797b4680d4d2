"""GPU parity of the fused attention kernels beyond the golden fixtures' shapes: every head
size the kernels are built for (16 / 32 / 64 / 128) and the head sizes between them (zero-padded to
the next kernel size, ops._padded_hd: the reference's modules take any d_model / num_heads),
frame counts that are not multiples of the 64-row
blocks, cross attention with Tq != Tk, hd 32 beyond one 256-key block (the fused key-block
backward), all three mask kinds with ragged and fully padded clips — the drop-in modules against the CPU oracle (oracle/sca_oracle.py:attention), forward
and all gradients within the north-star 1e-3.
"""
import pytest
import torch

from oracle import sca_oracle as O
from tests.golden_util import close, rel_err

PARITY_TOL = 1e-3

CASES = [  # kind, B, Tq, Tk, d, H
    ("self", 3, 100, 100, 64, 1),     # hd 64, T not a multiple of 64
    ("causal", 3, 130, 130, 64, 2),   # hd 32, three key blocks, partial diagonal block
    ("causal", 2, 64, 64, 128, 2),    # hd 64
    ("cross", 3, 70, 45, 64, 4),      # hd 16, Tq != Tk
    ("cross", 2, 33, 129, 128, 4),    # hd 32, Tk > Tq
    ("self", 2, 1, 1, 64, 4),         # single frame
    # hd 16 with Tq, Tk <= 256: the fused single-launch backward (sca_attn_bwd_fused)
    ("self", 3, 256, 256, 256, 16),   # the production shape (BASELINE config 2)
    ("causal", 3, 256, 256, 256, 16),
    ("cross", 3, 256, 256, 256, 16),
    ("causal", 3, 130, 130, 64, 4),   # partial last query block and key tile
    ("self", 3, 200, 200, 32, 2),
    ("cross", 2, 17, 250, 64, 4),
    # hd 32 at any length: the fused backward over 256-key blocks + the dQ partial reduction
    ("self", 2, 600, 600, 64, 2),     # three key blocks, the last partial
    ("causal", 2, 520, 520, 64, 2),   # key blocks see only the queries after their first key
    ("cross", 2, 300, 530, 64, 2),    # Tk > 256, Tq != Tk
    ("causal", 1, 1024, 1024, 512, 16),  # BASELINE config 5's attention shape
    # head sizes between the kernel sizes: zero-padded heads
    ("self", 2, 70, 70, 48, 6),       # hd 8 -> 16
    ("causal", 2, 90, 90, 48, 4),     # hd 12 -> 16
    ("causal", 2, 64, 64, 36, 6),     # hd 6 -> 16
    ("cross", 2, 40, 65, 72, 3),      # hd 24 -> 32
    ("self", 2, 50, 50, 120, 3),      # hd 40 -> 64
    # hd 128 (single-buffered LDS images) and sizes padded to it
    ("self", 2, 100, 100, 256, 2),    # hd 128
    ("causal", 2, 130, 130, 256, 2),  # hd 128, partial diagonal block
    ("cross", 2, 40, 90, 384, 3),     # hd 128, Tq != Tk
    ("self", 2, 50, 50, 192, 2),      # hd 96 -> 128
    ("causal", 2, 70, 70, 160, 2),    # hd 80 -> 128
    # head sizes over 128: scores / P V through the grouped GEMM, the row-softmax kernel
    ("self", 2, 100, 100, 512, 2),    # hd 256
    ("causal", 2, 70, 70, 600, 3),    # hd 200 (K not a multiple of 32: element-wise GEMM form)
    ("cross", 2, 40, 90, 288, 1),     # hd 288, Tq != Tk
    # d_model not a multiple of 4 (element-wise GEMM loads; heads padded to 16)
    ("self", 2, 40, 40, 30, 5),       # hd 6
    ("cross", 2, 30, 50, 42, 3),      # hd 14
    ("causal", 2, 33, 33, 21, 3),     # hd 7
]


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [1, 0])
@pytest.mark.parametrize("kind,B,Tq,Tk,d,H", CASES)
def test_attention_shapes_vs_oracle(kind, B, Tq, Tk, d, H, fused):
    import scattennet_amd as S
    from scattennet_amd import _lib as L
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from scattennet_amd import ops
    if not fused and (d // H > 128 or ops._padded_hd(d // H) not in (16, 32)):
        pytest.skip("the fused backward only exists for hd 16 and 32")
    L.lib().sca_attn_bwd_fused(fused)
    try:
        _run_case(S, kind, B, Tq, Tk, d, H)
    finally:
        L.lib().sca_attn_bwd_fused(1)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["self", "causal", "cross"])
def test_large_head_materialised_masks_vs_oracle(kind):
    """hd 256 with the reference's own materialised masks (create_attention_mask /
    create_causal_attention_mask semantics: the additive-mask path of the GEMM route)."""
    import scattennet_amd as S
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    _run_case(S, kind, 2, 48, 48 if kind != "cross" else 64, 512, 2, materialised=True)


def _run_case(S, kind, B, Tq, Tk, d, H, materialised=False):
    dev = torch.device("cuda:0")
    torch.manual_seed(Tq * 7 + Tk)
    cls = {"self": S.SelfAttention, "causal": S.SelfCausalAttention, "cross": S.CrossAttention}[kind]
    m = cls(d, H)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) / (p.shape[-1] ** 0.5 if p.dim() == 2 else 10.0))
    m = m.to(dev)
    x = torch.randn(B, Tq, d)
    kv = torch.randn(B, Tk, d)
    lens = [Tk, max(Tk // 2, 1), 0][:B]  # full, half, fully padded clip
    mask = torch.ones(B, Tk, dtype=torch.long)
    for b, n in enumerate(lens):
        mask[b, n:] = 0
    xg, kvg = x.to(dev).requires_grad_(True), kv.to(dev).requires_grad_(True)
    if materialised:
        if kind == "causal":
            am_dev = S.create_causal_attention_mask(mask.to(dev), (B, Tq), xg)
        else:
            am_dev = S.create_attention_mask(mask.to(dev), torch.float32, tgt_len=Tq)
        out = m(xg, kvg, am_dev) if kind == "cross" else m(xg, am_dev)
    elif kind == "cross":
        out = m(xg, kvg, S.key_padding_mask(mask.to(dev)))
    else:
        out = m(xg, S.key_padding_mask(mask.to(dev), causal=(kind == "causal")))
    gout = torch.randn(out.shape)
    out.backward(gout.to(dev))

    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    xr, kvr = x.clone().requires_grad_(True), kv.clone().requires_grad_(True)
    if kind == "causal":
        am = O.additive_causal_mask(mask)
    else:
        am = O.additive_key_mask(mask, tgt_len=Tq)
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
