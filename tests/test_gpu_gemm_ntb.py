"""The 128x128 register-staged NT / NN kernel (gemm_ntb_kernel, variants 41 / 42) at kernel level.

C = epilogue(A B^T) for A [M, K], B [N, K] — the nn.Linear forward of attention.py:41-44,74 and
layers.py:94-108 — through the C ABI (sca_gemm_variant), against a float64 product and against
the 64x64 LDS-DMA kernel (variant 20) on the same problem: M and N not multiples of 128, the
bias / post-scale / residual epilogue, GELU with its pre-activation output, ACCUM, dropout
(the same mask as variant 20: mask bits compared exactly), and the hand-over to variant 20
when K is not a multiple of 64 or split-K is asked for.
"""
import pytest
import torch

TOL = 2e-5


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _operands(shapes, K, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return [(torch.randn(M, K, generator=g).cuda(), torch.randn(N, K, generator=g).cuda(),
             torch.randn(N, generator=g).cuda(), torch.randn(M, N, generator=g).cuda()) for M, N in shapes]


def _run(ops_, L, ops, tile, epi=0, gelu=False, drop=None, accum_base=None):
    outs, auxs, probs = [], [], []
    for i, (A, B, bias, res) in enumerate(ops_):
        M, K = A.shape
        N = B.shape[0]
        C = accum_base[i].clone() if accum_base is not None else torch.full((M, N), float("nan"), device="cuda")
        aux = torch.full((M, N), float("nan"), device="cuda") if gelu else None
        probs.append(ops._prob([ops._seg(A, B, K, K, K, 0.75)], C, M, N, N, bias=bias, post_scale=1.5, resid=res,
                               ldr=N, epi=epi | (L.EPI_GELU if gelu else 0) | (L.EPI_ACCUM if accum_base is not None
                                                                                   else 0),
                               aux_out=aux, ldo=N, drop=drop))
        outs.append(C)
        auxs.append(aux)
    ops.gemm(L.GEMM_NT, probs, tile=tile)
    torch.cuda.synchronize()
    return outs, auxs


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [41, 42, 44, 45])
def test_ntb_matches_float64(tile):
    from scattennet_amd import _lib as L, ops
    xs = _operands([(200, 132), (256, 384), (64, 4)], 192, seed=tile)
    outs, _ = _run(xs, L, ops, tile)
    for (A, B, bias, res), C in zip(xs, outs):
        ref = (0.75 * (A.double() @ B.double().t()) + bias.double()) * 1.5 + res.double()
        assert _rel(C, ref) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [41, 42, 44, 45])
def test_ntb_gelu_accum_and_dropout_match_variant_20(tile):
    from scattennet_amd import _lib as L, ops
    xs = _operands([(300, 260), (128, 128)], 256, seed=7)
    for kw in (dict(gelu=True), dict(accum_base=[torch.randn(300, 260).cuda(), torch.randn(128, 128).cuda()]),
               dict(drop=(12345, 0.3))):
        ref_c, ref_a = _run(xs, L, ops, 20, **kw)
        got_c, got_a = _run(xs, L, ops, tile, **kw)
        for r, g in zip(ref_c, got_c):
            assert _rel(g, r) < TOL, kw.keys()
            if "drop" in kw:  # the identical mask: zero exactly where variant 20 dropped
                assert torch.equal(r == 0, g == 0)
        for r, g in zip(ref_a, got_a):
            if r is not None:
                assert _rel(g, r) < TOL


@pytest.mark.gpu
def test_ntb_hands_over_when_ineligible():
    """K % 64 != 0, or split-K: variant 41 runs as variant 20 (same results)."""
    from scattennet_amd import _lib as L, ops
    xs = _operands([(132, 68)], 96, seed=3)
    assert ops._gemm_kernel_name(L.GEMM_NT, [ops._prob([ops._seg(xs[0][0], xs[0][1], 96, 96, 96)], xs[0][3], 132, 68,
                                                       68)], 41) == "gemm_glds_kernel<0, 3>"
    outs, _ = _run(xs, L, ops, 41)
    A, B, bias, res = xs[0]
    ref = (0.75 * (A.double() @ B.double().t()) + bias.double()) * 1.5 + res.double()
    assert _rel(outs[0], ref) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("layout_name", ["NT", "NN"])
@pytest.mark.parametrize("tile", [41, 42, 44, 45])
def test_ntb_segments_nt_and_nn(layout_name, tile):
    """Three segments (the dX = dQ Wq + dK Wk + dV Wv form) of different K, NT and NN (B [K][N],
    transposed into the LDS image), M / N not multiples of 128, against float64 and against the
    LDS-DMA kernel."""
    from scattennet_amd import _lib as L, ops
    layout = getattr(L, "GEMM_" + layout_name)
    g = torch.Generator(device="cpu").manual_seed(11 + tile)
    M, N = 260, 196
    segs, ref = [], torch.zeros(M, N, dtype=torch.float64)
    keep = []
    for K in (64, 192, 128):
        A = torch.randn(M, K, generator=g).cuda()
        B = torch.randn(N, K, generator=g).cuda() if layout_name == "NT" else torch.randn(K, N, generator=g).cuda()
        keep += [A, B]
        segs.append(ops._seg(A, B, K, K if layout_name == "NT" else N, K, 0.5))
        ref += 0.5 * (A.double().cpu() @ (B.double().cpu().t() if layout_name == "NT" else B.double().cpu()))
    bias = torch.randn(N, generator=g).cuda()
    outs = {}
    for t in (tile, 20 if layout_name == "NT" else 21):
        C = torch.full((M, N), float("nan"), device="cuda")
        ops.gemm(layout, [ops._prob(segs, C, M, N, N, bias=bias)], tile=t)
        torch.cuda.synchronize()
        outs[t] = C
    ref = ref + bias.double().cpu()
    assert _rel(outs[tile].cpu(), ref) < TOL
    assert _rel(outs[tile], outs[20 if layout_name == "NT" else 21]) < TOL


@pytest.mark.gpu
def test_gelu_epilogue_against_exact_erf():
    """The GEMM epilogues' GELU (branch-free erf, common.h erf_ep) against float64 erf-GELU
    over pre-activations spanning the whole useful range: max |err| <= 4e-7 * max(1, |z|)
    (the erf fit's 3.9e-7 plus fp32 rounding), and GELU' (the DGELU epilogue) likewise."""
    import math
    from scattennet_amd import _lib as L, ops
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = "cuda"
    M, N, K = 256, 256, 64
    z = torch.linspace(-9.0, 9.0, M * N, dtype=torch.float64).reshape(M, N)
    # z = A B^T with A = z, B = identity blocks: one segment of K = N (an exact product)
    A = z.float().to(dev)
    B = torch.eye(N, device=dev)
    C = torch.empty(M, N, device=dev)
    aux = torch.empty(M, N, device=dev)
    p = ops._prob([ops._seg(A, B, N, N, N)], C, M, N, N, epi=L.EPI_GELU, aux_out=aux, ldo=N)
    ops.gemm(L.GEMM_NT, [p])
    torch.cuda.synchronize()
    zf = A.double().cpu()
    want = 0.5 * zf * (1 + torch.special.erf(zf / math.sqrt(2.0)))
    err = (C.double().cpu() - want).abs() / zf.abs().clamp_min(1.0)
    assert float(err.max()) <= 4e-7, float(err.max())
    assert torch.equal(aux.cpu(), A.cpu())  # the pre-activation kept for the backward
    # DGELU: dY * gelu'(z)
    dY = torch.ones(M, N, device=dev)
    D = torch.empty(M, N, device=dev)
    q = ops._prob([ops._seg(dY, B, N, N, N)], D, M, N, N, epi=L.EPI_DGELU, aux=A, ldx=N)
    ops.gemm(L.GEMM_NT, [q])
    torch.cuda.synchronize()
    cdf = 0.5 * (1 + torch.special.erf(zf / math.sqrt(2.0)))
    pdf = torch.exp(-0.5 * zf * zf) / math.sqrt(2 * math.pi)
    gwant = cdf + zf * pdf
    gerr = (D.double().cpu() - gwant).abs() / zf.abs().clamp_min(1.0)
    assert float(gerr.max()) <= 1e-6, float(gerr.max())
