"""GPU parity of the fused GEMM + post-LN LayerNorm launch (sca_gemm_ln).

* the C ABI directly against a float64 torch restatement of the same epilogue
  (v = resid + (A W^T + b) * post_scale, y = LayerNorm(v) * gamma + beta), ragged M;
* the blocks that use it at d_model = 256 (both CoordinateAttention kinds and
  CoordinatesMerge, keypoint_module.py:61-80, 97-115) against the CPU oracle, with the fused
  path on and off, forward and every gradient within the north-star 1e-3.
"""
import pytest
import torch

from oracle import sca_oracle as O
from tests.golden_util import close, rel_err

PARITY_TOL = 1e-3

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("M,K,N", [(8192, 256, 256), (2048, 768, 256), (100, 64, 256), (33, 32, 256),
                                   (8192, 512, 512), (2048, 2048, 512), (100, 64, 512), (33, 32, 512)])
def test_gemm_ln_c_abi_vs_float64(M, K, N):
    """N = 512 (cfg5's d_model): two 256-column halves of one slice sequence, one LayerNorm
    over the 512-wide row."""
    _need_gpu()
    from scattennet_amd import _lib as L, ops
    dev = torch.device("cuda:0")
    torch.manual_seed(M + K + N)
    A, W = torch.randn(M, K, device=dev), torch.randn(N, K, device=dev) / K ** 0.5
    bias, resid = torch.randn(N, device=dev), torch.randn(M, N, device=dev)
    gam, bet = torch.randn(N, device=dev), torch.randn(N, device=dev)
    v, y = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    prob = ops._prob([ops._seg(A, W, K, K, K)], v, M, N, N, bias=bias, post_scale=0.75, resid=resid, ldr=N)
    ops.gemm_ln([prob], [L.GemmLnProblem(gam.data_ptr(), bet.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                         rstd.data_ptr())], 1e-5)
    torch.cuda.synchronize()
    v64 = resid.double().cpu() + (A.double().cpu() @ W.double().cpu().T + bias.double().cpu()) * 0.75
    y64 = torch.nn.functional.layer_norm(v64, (N,), gam.double().cpu(), bet.double().cpu(), 1e-5)
    assert rel_err(v.cpu(), v64) < 1e-5
    assert rel_err(y.cpu(), y64) < 1e-4
    assert rel_err(mean.cpu(), v64.mean(-1)) < 1e-4
    assert rel_err(rstd.cpu(), 1.0 / (v64.var(-1, unbiased=False) + 1e-5).sqrt()) < 1e-4


@pytest.mark.parametrize("K", [768, 256])
def test_gemm_ln_grouped_row_tiles(K):
    """Four problems of 2048 rows: K = 768 takes the 32-row tile (a workgroup per CU at 32
    rows), K = 256 the 16-row tile (sca_gemm_ln's heuristic) — both against float64."""
    _need_gpu()
    from scattennet_amd import _lib as L, ops
    dev = torch.device("cuda:0")
    torch.manual_seed(K)
    M, N, G = 2048, 256, 4
    probs, lns, keep = [], [], []
    for g in range(G):
        A, W = torch.randn(M, K, device=dev), torch.randn(N, K, device=dev) / K ** 0.5
        b, r = torch.randn(N, device=dev), torch.randn(M, N, device=dev)
        gam, bet = torch.randn(N, device=dev), torch.randn(N, device=dev)
        v, y = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
        mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
        probs.append(ops._prob([ops._seg(A, W, K, K, K)], v, M, N, N, bias=b, resid=r, ldr=N))
        lns.append(L.GemmLnProblem(gam.data_ptr(), bet.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr()))
        keep.append((A, W, b, r, gam, bet, v, y, mean, rstd))  # every buffer alive until the launch ran
    ops.gemm_ln(probs, lns, 1e-5)
    torch.cuda.synchronize()
    for A, W, b, r, gam, bet, v, y, _, _ in keep:
        v64 = r.double().cpu() + A.double().cpu() @ W.double().cpu().T + b.double().cpu()
        y64 = torch.nn.functional.layer_norm(v64, (N,), gam.double().cpu(), bet.double().cpu(), 1e-5)
        assert rel_err(v.cpu(), v64) < 1e-5
        assert rel_err(y.cpu(), y64) < 1e-4


def _chain_pass(L, W, bias, C, scale, aux=None):
    gelu = aux is not None
    return L.ChainPass(W.data_ptr(), W.stride(0), bias.data_ptr() if bias is not None else None, scale,
                       L.EPI_GELU if gelu else 0, C.data_ptr(), C.stride(0), aux.data_ptr() if gelu else None,
                       aux.stride(0) if gelu else 0)


@pytest.mark.parametrize("G,M,K,npass,gelu", [(4, 2048, 256, 3, True), (4, 2048, 768, 3, False),
                                              (2, 1000, 256, 1, True), (1, 33, 32, 2, False)])
def test_gemm_ln_chained_passes_vs_float64(G, M, K, npass, gelu):
    """Chained NT passes on the LayerNorm output (an FFN's fc1 with GELU, or q / k / v)
    written in the same launch: out_p = epi((y W_p^T + b_p) * s_p) from 256-row blocks of one
    [256 * npass, 256] weight, against float64; ragged M, one to three passes."""
    _need_gpu()
    from scattennet_amd import _lib as L, ops
    dev = torch.device("cuda:0")
    torch.manual_seed(G * M + K + npass)
    N = 256
    probs, lns, keep = [], [], []
    for g in range(G):
        A, W = torch.randn(M, K, device=dev), torch.randn(N, K, device=dev) / K ** 0.5
        b, r = torch.randn(N, device=dev), torch.randn(M, N, device=dev)
        gam, bet = torch.randn(N, device=dev), torch.randn(N, device=dev)
        v, y = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
        mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
        W2, b2 = torch.randn(N * npass, N, device=dev) / N ** 0.5, torch.randn(N * npass, device=dev)
        out = torch.full((M, N * npass), float("nan"), device=dev)
        aux = torch.full((M, N * npass), float("nan"), device=dev) if gelu else None
        scales = [0.25 * (p + 1) for p in range(npass)]
        passes = [_chain_pass(L, W2[p * N:(p + 1) * N], b2[p * N:(p + 1) * N] if p != 1 else None,
                              out[:, p * N:], scales[p], aux[:, p * N:] if gelu else None) for p in range(npass)]
        passes += [L.ChainPass()] * (3 - npass)
        probs.append(ops._prob([ops._seg(A, W, K, K, K)], v, M, N, N, bias=b, resid=r, ldr=N))
        lns.append(L.GemmLnProblem(gam.data_ptr(), bet.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                   npass, (L.ChainPass * 3)(*passes)))
        keep.append((A, W, b, r, gam, bet, v, y, W2, b2, out, aux, scales, mean, rstd))  # alive until it ran
    ops.gemm_ln(probs, lns, 1e-5)
    torch.cuda.synchronize()
    for A, W, b, r, gam, bet, v, y, W2, b2, out, aux, scales, _, _ in keep:
        v64 = r.double().cpu() + A.double().cpu() @ W.double().cpu().T + b.double().cpu()
        y64 = torch.nn.functional.layer_norm(v64, (N,), gam.double().cpu(), bet.double().cpu(), 1e-5)
        assert rel_err(v.cpu(), v64) < 1e-5
        assert rel_err(y.cpu(), y64) < 1e-4
        for p in range(npass):
            bp = b2[p * N:(p + 1) * N].double().cpu() if p != 1 else 0.0
            pre = (y64 @ W2[p * N:(p + 1) * N].double().cpu().T + bp) * scales[p]
            want = torch.nn.functional.gelu(pre) if gelu else pre
            assert rel_err(out[:, p * N:(p + 1) * N].cpu(), want) < 1e-4, p
            if gelu:
                assert rel_err(aux[:, p * N:(p + 1) * N].cpu(), pre) < 1e-4, p


def test_gemm_ln_rejects_other_widths():
    _need_gpu()
    from scattennet_amd import _lib as L, ops
    dev = torch.device("cuda:0")
    A, W = torch.randn(64, 64, device=dev), torch.randn(128, 64, device=dev)
    v = torch.empty(64, 128, device=dev)
    g = torch.ones(128, device=dev)
    prob = ops._prob([ops._seg(A, W, 64, 64, 64)], v, 64, 128, 128)
    with pytest.raises(ValueError):
        ops.gemm_ln([prob], [L.GemmLnProblem(g.data_ptr(), g.data_ptr(), v.data_ptr(), g.data_ptr(),
                                             g.data_ptr())], 1e-5)


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("block", ["self", "causal", "merge"])
def test_blocks_d256_vs_oracle(block, fused):
    _need_gpu()
    import scattennet_amd as S
    from scattennet_amd import ops
    from scattennet_amd.workloads import model_cfg
    dev = torch.device("cuda:0")
    torch.manual_seed(11)
    B, T, d, H = 3, 72, 256, 16
    cfg = model_cfg(d, H, 1)
    m = S.CoordinatesMerge(cfg) if block == "merge" else \
        S.CoordinateAttention(cfg, "self_attn" if block == "self" else "causal_attn")
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) / (p.shape[-1] ** 0.5 if p.dim() == 2 else 4.0))
    m = m.to(dev)
    x, kv = torch.randn(B, T, d), torch.randn(B, T, d)
    mask = torch.ones(B, T, dtype=torch.long)
    mask[1, 40:] = 0
    mask[2, :] = 0
    causal = block == "causal"
    am = S.key_padding_mask(mask.to(dev), causal=causal)
    xg, kvg = x.to(dev).requires_grad_(True), kv.to(dev).requires_grad_(True)
    old = ops._FUSE_LN
    ops._FUSE_LN = fused
    try:
        out = m(xg, kvg, am) if block == "merge" else m(xg, am)
        gout = torch.randn(out.shape)
        out.backward(gout.to(dev))
        torch.cuda.synchronize()
    finally:
        ops._FUSE_LN = old
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    xr, kvr = x.clone().requires_grad_(True), kv.clone().requires_grad_(True)
    pp = {"b." + k: v for k, v in p.items()}
    if block == "merge":
        ref = O.coordinates_merge(pp, "b", xr, kvr, O.additive_key_mask(mask, tgt_len=T), H)
    else:
        amr = O.additive_causal_mask(mask) if causal else O.additive_key_mask(mask, tgt_len=T)
        ref = O.coordinate_attention(pp, "b", xr, amr, H, "causal_attn" if causal else "self_attn")
    assert rel_err(out, ref) < PARITY_TOL
    (ref * gout).sum().backward()
    assert rel_err(xg.grad, xr.grad) < PARITY_TOL
    if block == "merge":
        assert rel_err(kvg.grad, kvr.grad) < PARITY_TOL
    gscale = max(float(v.grad.abs().max()) for v in p.values() if v.grad is not None)
    named = dict(m.named_parameters())
    for k, v in p.items():
        if v.grad is not None:
            assert close(named[k].grad.cpu(), v.grad, PARITY_TOL, gscale), (k, rel_err(named[k].grad.cpu(), v.grad))


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("splitk", [1, 3, 4])
def test_weight_gradient_gemm_mixed_shapes(splitk, fused, monkeypatch):
    """The TN (weight-gradient) split-K GEMM with problems of different shapes in one launch
    (fc1 768x256 and fc2 256x768 weight gradients, bias colsums fused) vs float64 — the slab
    combine in the same launch (last arriver, sca_gemm_splitk_fused) and as a second launch;
    repeated launches on the same counters (they must be left zero) and a ragged
    (100 x 36, K = 1000) problem."""
    _need_gpu()
    from scattennet_amd import _lib as L, ops
    monkeypatch.setattr(ops, "_SPLITK_FUSED", fused)
    dev = torch.device("cuda:0")
    torch.manual_seed(splitk)
    Mr = 2048
    shapes = [(768, 256), (256, 768), (256, 256), (64, 32)]
    probs, keep, wsz = [], [], 0
    for (n_out, n_in) in shapes:
        dY, X = torch.randn(Mr, n_out, device=dev), torch.randn(Mr, n_in, device=dev)
        dW, db = torch.empty(n_out, n_in, device=dev), torch.empty(n_out, device=dev)
        probs.append(ops._prob([ops._seg(dY, X, n_out, n_in, Mr, 0.5)], dW, n_out, n_in, n_in,
                               bias_grad=db, bias_grad_scale=2.0))
        keep.append((dY, X, dW, db))
        wsz += splitk * (n_out * n_in + n_out)
    ws = torch.empty(wsz, device=dev) if splitk > 1 else None
    for _ in range(3):  # the same counters / workspace three times
        for _, _, dW, db in keep:
            dW.fill_(float("nan"))
            db.fill_(float("nan"))
        ops.gemm(L.GEMM_TN, probs, splitk=splitk, ws=ws)
        torch.cuda.synchronize()
        for dY, X, dW, db in keep:
            ref = 0.5 * dY.double().cpu().T @ X.double().cpu()
            assert rel_err(dW.cpu(), ref) < 1e-5
            assert rel_err(db.cpu(), dY.double().cpu().sum(0)) < 1e-5
    if fused and ops._CNT:
        for ring, _ in ops._CNT.values():
            assert int(ring.abs().sum()) == 0  # every tile counter reset by its last arriver
    # a ragged problem: rows / columns not multiples of the 64x64 tile, uneven K chunks
    dY, X = torch.randn(1000, 100, device=dev), torch.randn(1000, 36, device=dev)
    dW, db = torch.empty(100, 36, device=dev), torch.empty(100, device=dev)
    p = ops._prob([ops._seg(dY, X, 100, 36, 1000)], dW, 100, 36, 36, bias_grad=db)
    ws2 = torch.empty(splitk * (100 * 36 + 100), device=dev) if splitk > 1 else None
    ops.gemm(L.GEMM_TN, [p], splitk=splitk, ws=ws2)
    torch.cuda.synchronize()
    assert rel_err(dW.cpu(), dY.double().cpu().T @ X.double().cpu()) < 1e-5
    assert rel_err(db.cpu(), dY.double().cpu().sum(0)) < 1e-5


@pytest.mark.parametrize("chain", [True, False])
def test_sca_stack_chained_projections_vs_oracle(chain, monkeypatch):
    """A two-layer SeparativeCoordinateAttention at d_model 256 (keypoint_module.py:153-198)
    with the next op's projections chained into each fused GEMM + LayerNorm launch (every
    FFN's fc1; self layer 1's and causal layer 1's q / k / v) against the CPU oracle, forward
    and every gradient; with the chain the forward issues 4 stand-alone NT GEMM launches
    (self / causal layer 0 q/k/v, the two merges' q + k/v) instead of 10."""
    _need_gpu()
    import scattennet_amd as S
    from scattennet_amd import _lib as L, ops
    from scattennet_amd.workloads import model_cfg
    monkeypatch.setattr(ops, "_CHAIN_NEXT", chain)
    monkeypatch.setattr(ops, "_CHAIN_MIN_TILES", 0)  # chain even at this test's 8 row tiles
    dev = torch.device("cuda:0")
    torch.manual_seed(21)
    B, T, d, H = 3, 80, 256, 16
    cfg = model_cfg(d, H, 2, maxpos=T)
    m = S.SeparativeCoordinateAttention(cfg)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) / (p.shape[-1] ** 0.5 if p.dim() == 2 else 4.0))
    m = m.to(dev)
    x, y = torch.randn(B, T, d), torch.randn(B, T, d)
    mask = torch.ones(B, T, dtype=torch.long)
    mask[1, 50:] = 0
    mask[2, 1:] = 0
    xg, yg = x.to(dev).requires_grad_(True), y.to(dev).requires_grad_(True)
    gout = torch.randn(B, T, d)
    prof = ops.LaunchProfiler()
    with prof:
        out = m(xg, yg, mask.to(dev))
    out.backward(gout.to(dev))
    torch.cuda.synchronize()
    nt = prof.launches(*ops.GEMM_KERNELS[L.GEMM_NT])
    assert nt == (4 if chain else 10), nt
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    xr, yr = x.clone().requires_grad_(True), y.clone().requires_grad_(True)
    ref = O.sca(p, "", xr, yr, mask, cfg)
    assert rel_err(out, ref) < PARITY_TOL
    (ref * gout).sum().backward()
    assert rel_err(xg.grad, xr.grad) < PARITY_TOL
    assert rel_err(yg.grad, yr.grad) < PARITY_TOL
    gscale = max(float(v.grad.abs().max()) for v in p.values() if v.grad is not None)
    named = dict(m.named_parameters())
    for k, v in p.items():
        if v.grad is not None:
            assert close(named[k].grad.cpu(), v.grad, PARITY_TOL, gscale), (k, rel_err(named[k].grad.cpu(), v.grad))
