"""GPU parity of the NN input-gradient GEMM + LayerNorm backward launch (sca_gemm_lnb).

* the C ABI directly against a float64 restatement (C = resid + sum_s A_s B_s, then
  aten's layer_norm backward of the LayerNorm whose output C is the gradient of), 1-3
  segments, ragged M, the dgamma / dbeta partials summed;
* the hand-off between post-LN blocks: two chained CoordinateAttention (self) blocks at
  d_model 256 — the second block's input-gradient GEMM runs the first block's last
  LayerNorm backward (and each block's FFN runs its attention LayerNorm backward) — against
  the CPU oracle, forward and every gradient; and the same chain with a second consumer of
  the first block's output, where the producer must NOT take the hand-off (autograd sums
  the two consumers' gradients first).
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


@pytest.mark.parametrize("chain", ["none", "wo", "dgelu3", "ld2"])
@pytest.mark.parametrize("M,Ks", [(2048, (768,)), (2048, (256, 256, 256)), (1000, (256,)), (33, (32, 64))])
def test_gemm_lnb_c_abi_vs_float64(M, Ks, chain):
    """chain: none; "wo": dout = dx Wo (one pass, the attention out-projection input
    gradient); "dgelu3": dout = (dx W2) * gelu'(aux) over three 256-column passes (the FFN's
    dz); "ld2": two passes with row stride 640 (ldw > 256 npass)."""
    _need_gpu()
    from scattennet_amd import _lib as L, ops
    dev = torch.device("cuda:0")
    torch.manual_seed(M + sum(Ks))
    N = 256
    segs, c64 = [], torch.zeros(M, N, dtype=torch.float64)
    keep = []
    for K in Ks:
        A, B = torch.randn(M, K, device=dev), torch.randn(K, N, device=dev) / K ** 0.5
        keep += [A, B]
        segs.append(ops._seg(A, B, K, N, K))
        c64 += A.double().cpu() @ B.double().cpu()
    resid = torch.randn(M, N, device=dev)
    c64 += resid.double().cpu()
    x = torch.randn(M, N, device=dev) * 2 + 0.5
    gam = torch.randn(N, device=dev)
    mean = x.mean(-1)
    rstd = 1.0 / (x.var(-1, unbiased=False) + 1e-5).sqrt()
    C, dx = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
    nblk = L.lib().sca_gemm_lnb_blocks(M)
    part = torch.empty(2 * nblk * N, device=dev)
    prob = ops._prob(segs, C, M, N, N, resid=resid, ldr=N)
    npass, ldw = {"none": (0, 0), "wo": (1, 256), "dgelu3": (3, 768), "ld2": (2, 640)}[chain]
    wo = torch.randn(N, max(ldw, N), device=dev) / N ** 0.5
    dout = torch.full((M, max(ldw, N)), float("nan"), device=dev)
    aux = torch.randn(M, max(ldw, N), device=dev) if chain == "dgelu3" else None
    on = chain != "none"
    lnp = L.GemmLnbProblem(x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gam.data_ptr(), dx.data_ptr(),
                           part.data_ptr(), wo.data_ptr() if on else None, dout.data_ptr() if on else None,
                           aux.data_ptr() if aux is not None else None, npass if chain != "wo" else 0,
                           ldw if chain == "ld2" else 0)
    arr, larr = (L.GemmProblem * 1)(prob), (L.GemmLnbProblem * 1)(lnp)
    L.check(L.lib().sca_gemm_lnb(1, arr, larr, L.stream_handle()), "sca_gemm_lnb")
    torch.cuda.synchronize()
    # float64 restatement of aten's layer_norm backward with dL/dy = C
    x64 = x.double().cpu().requires_grad_(True)
    g64, b64 = gam.double().cpu().requires_grad_(True), torch.zeros(N, dtype=torch.float64, requires_grad=True)
    y64 = torch.nn.functional.layer_norm(x64, (N,), g64, b64, 1e-5)
    y64.backward(c64)
    assert rel_err(C.cpu(), c64) < 1e-5
    assert rel_err(dx.cpu(), x64.grad) < 1e-4
    pg = part[:nblk * N].view(nblk, N).sum(0).cpu()
    pb = part[nblk * N:].view(nblk, N).sum(0).cpu()
    assert rel_err(pg, g64.grad) < 1e-4
    assert rel_err(pb, b64.grad) < 1e-4
    if on:  # the chained GEMM: dout = dx Wo (* gelu'(aux))
        n = 256 * npass
        want = x64.grad @ wo.double().cpu()[:, :n]
        if aux is not None:
            z = aux.double().cpu()[:, :n].requires_grad_(True)
            torch.nn.functional.gelu(z).backward(torch.ones_like(z))
            want = want * z.grad
        assert rel_err(dout.cpu()[:, :n], want) < 1e-4
        if chain == "ld2":
            assert torch.isnan(dout[:, n:]).all()  # columns past the passes untouched


@pytest.mark.parametrize("tab", [False, True])
@pytest.mark.parametrize("M,Ks", [(2048, (2048,)), (2048, (512, 512, 512)), (1000, (512,)), (33, (32, 64))])
def test_gemm_lnb_n512_vs_float64(M, Ks, tab):
    """d_model 512 (cfg5): two 256-column halves of one slice sequence (segments walked once
    per half), the LayerNorm backward over the 512-wide row, dgamma / dbeta partials of 512
    columns; `tab`: the position-table mode (LN input x + P[t + 2], the embedding LayerNorm)."""
    _need_gpu()
    from scattennet_amd import _lib as L, ops
    dev = torch.device("cuda:0")
    torch.manual_seed(M + sum(Ks) + tab)
    N, T = 512, 50
    segs, c64, keep = [], torch.zeros(M, N, dtype=torch.float64), []
    for K in Ks:
        A, B = torch.randn(M, K, device=dev), torch.randn(K, N, device=dev) / K ** 0.5
        keep += [A, B]
        segs.append(ops._seg(A, B, K, N, K))
        c64 += A.double().cpu() @ B.double().cpu()
    resid = torch.randn(M, N, device=dev)
    c64 += resid.double().cpu()
    x = torch.randn(M, N, device=dev) * 2 + 0.5
    P = torch.randn(T + 2, N, device=dev) if tab else None
    xin = x + P[2:][torch.arange(M, device=dev) % T] if tab else x
    gam = torch.randn(N, device=dev)
    mean = xin.mean(-1)
    rstd = 1.0 / (xin.var(-1, unbiased=False) + 1e-5).sqrt()
    C, dx = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
    nblk = L.lib().sca_gemm_lnb_blocks(M)
    part = torch.empty(2 * nblk * N, device=dev)
    prob = ops._prob(segs, C, M, N, N, resid=resid, ldr=N)
    lnp = L.GemmLnbProblem(x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gam.data_ptr(), dx.data_ptr(),
                           part.data_ptr(), None, None, None, 0, 0, P.data_ptr() if tab else None, T if tab else 0)
    arr, larr = (L.GemmProblem * 1)(prob), (L.GemmLnbProblem * 1)(lnp)
    L.check(L.lib().sca_gemm_lnb(1, arr, larr, L.stream_handle()), "sca_gemm_lnb")
    torch.cuda.synchronize()
    x64 = xin.double().cpu().requires_grad_(True)
    g64, b64 = gam.double().cpu().requires_grad_(True), torch.zeros(N, dtype=torch.float64, requires_grad=True)
    torch.nn.functional.layer_norm(x64, (N,), g64, b64, 1e-5).backward(c64)
    assert rel_err(C.cpu(), c64) < 1e-5
    assert rel_err(dx.cpu(), x64.grad) < 1e-4
    assert rel_err(part[:nblk * N].view(nblk, N).sum(0).cpu(), g64.grad) < 1e-4
    assert rel_err(part[nblk * N:].view(nblk, N).sum(0).cpu(), b64.grad) < 1e-4


def test_gemm_lnb_n512_rejects_chain():
    """The chained GEMM (dout = dx Wo) exists for d_model 256 only."""
    _need_gpu()
    from scattennet_amd import _lib as L, ops
    dev = torch.device("cuda:0")
    M, N = 64, 512
    A, B, C = torch.randn(M, 64, device=dev), torch.randn(64, N, device=dev), torch.empty(M, N, device=dev)
    prob = ops._prob([ops._seg(A, B, 64, N, 64)], C, M, N, N)
    t = torch.empty(M, N, device=dev)
    lnp = L.GemmLnbProblem(t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(),
                           t.data_ptr(), t.data_ptr(), None, 1, 0)
    with pytest.raises(ValueError):
        L.check(L.lib().sca_gemm_lnb(1, (L.GemmProblem * 1)(prob), (L.GemmLnbProblem * 1)(lnp),
                                     L.stream_handle()), "sca_gemm_lnb")


def test_gemm_lnb_rejects_bad_shapes():
    _need_gpu()
    from scattennet_amd import _lib as L, ops
    dev = torch.device("cuda:0")
    A, B, C = torch.randn(64, 48, device=dev), torch.randn(48, 256, device=dev), torch.empty(64, 256, device=dev)
    prob = ops._prob([ops._seg(A, B, 48, 256, 48)], C, 64, 256, 256)  # K = 48: not a multiple of 32
    t = torch.empty(64, 256, device=dev)
    lnp = L.GemmLnbProblem(t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr())
    with pytest.raises(ValueError):
        L.check(L.lib().sca_gemm_lnb(1, (L.GemmProblem * 1)(prob), (L.GemmLnbProblem * 1)(lnp),
                                     L.stream_handle()), "sca_gemm_lnb")


@pytest.mark.parametrize("dz", [True, False])
@pytest.mark.parametrize("second_consumer", [False, True])
def test_chained_blocks_hand_off_layer_norm_backward(second_consumer, dz, monkeypatch):
    """... and with `dz` block 0's FFN dz = (dL/dv W2) * gelu'(z) rides in block 1's
    gemm_lnb launch too (one NN launch fewer) unless a second consumer blocks the hand-off."""
    _need_gpu()
    import scattennet_amd as S
    from scattennet_amd import _lib as L, ops, workloads as W
    monkeypatch.setattr(ops, "_CHAIN_DZ", dz)
    dev = torch.device("cuda:0")
    torch.manual_seed(5)
    B, T, d, H = 3, 96, 256, 16
    cfg = W.model_cfg(d, H, 1, maxpos=T)
    blocks = [S.CoordinateAttention(cfg, "self_attn"), S.CoordinateAttention(cfg, "self_attn")]
    g = torch.Generator().manual_seed(7)
    with torch.no_grad():
        for blk in blocks:
            for name, p in blk.named_parameters():
                p.copy_(torch.randn(p.shape, generator=g) / (p.shape[-1] ** 0.5) if p.dim() == 2
                        else (1.0 if name.endswith("weight") else 0.0) + 0.1 * torch.randn(p.shape, generator=g))
    blocks = [b.to(dev) for b in blocks]
    x = torch.randn(B, T, d, generator=g)
    mask = torch.ones(B, T, dtype=torch.long)
    mask[1, 60:] = 0
    mask[2, 1:] = 0
    g1, g2 = torch.randn(B, T, d, generator=g), torch.randn(B, T, d, generator=g)
    xg = x.to(dev).requires_grad_(True)
    kpm = S.key_padding_mask(mask.to(dev))
    prof = ops.LaunchProfiler()
    with prof:
        h1 = blocks[0](xg, kpm)
        h2 = blocks[1](h1, kpm)
        loss = (h2 * g1.to(dev)).sum()
        if second_consumer:
            loss = loss + (h1 * g2.to(dev)).sum()
        loss.backward()
    torch.cuda.synchronize()
    # hand-offs: block 1's FFN -> its attention LN; block 1's attention -> block 0's last LN;
    # block 0's FFN -> its attention LN (block 0's attention input x has no fused producer)
    assert prof.launches("gemm_lnb_kernel<1,") == 3
    # NN launches: block 0's attention dX (no fused producer), block 1's FFN dz (its output has
    # no fused consumer) and block 0's FFN dz unless block 1's launch chained it
    nn = prof.launches(*ops.GEMM_KERNELS[L.GEMM_NN])
    assert nn == (2 if dz and not second_consumer else 3), nn

    ps = [{k: v.detach().cpu().clone().requires_grad_(True) for k, v in blk.state_dict().items()} for blk in blocks]
    xr = x.clone().requires_grad_(True)
    am = O.additive_key_mask(mask)
    r1 = O.coordinate_attention({"b." + k: v for k, v in ps[0].items()}, "b", xr, am, H, "self_attn")
    r2 = O.coordinate_attention({"b." + k: v for k, v in ps[1].items()}, "b", r1, am, H, "self_attn")
    ref = (r2 * g1).sum() + ((r1 * g2).sum() if second_consumer else 0.0)
    assert rel_err(h2, r2) < PARITY_TOL
    ref.backward()
    assert rel_err(xg.grad, xr.grad) < PARITY_TOL
    for blk, p in zip(blocks, ps):
        gscale = max(float(v.grad.abs().max()) for v in p.values())
        named = dict(blk.named_parameters())
        for k, v in p.items():
            assert close(named[k].grad.cpu(), v.grad, PARITY_TOL, gscale), (k, rel_err(named[k].grad.cpu(), v.grad))
