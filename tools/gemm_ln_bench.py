"""Microbenchmark of the fused GEMM + LayerNorm launch (sca_gemm_ln) against the unfused
pair (sca_gemm + sca_layernorm_fwd) at the workload's out-projection and fc2 shapes, each
graph-captured (`iters` launches per replay).

    python tools/gemm_ln_bench.py [--iters 30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import _lib as L, ops  # noqa: E402


def case(G, M, K, N=256):
    dev = "cuda"
    A = [torch.randn(M, K, device=dev) for _ in range(G)]
    W = [torch.randn(N, K, device=dev) / K ** 0.5 for _ in range(G)]
    b = [torch.randn(N, device=dev) for _ in range(G)]
    r = [torch.randn(M, N, device=dev) for _ in range(G)]
    gam = [torch.ones(N, device=dev) for _ in range(G)]
    bet = [torch.zeros(N, device=dev) for _ in range(G)]
    v = [torch.empty(M, N, device=dev) for _ in range(G)]
    y = [torch.empty(M, N, device=dev) for _ in range(G)]
    mean = [torch.empty(M, device=dev) for _ in range(G)]
    rstd = [torch.empty(M, device=dev) for _ in range(G)]
    probs = [ops._prob([ops._seg(A[g], W[g], K, K, K)], v[g], M, N, N, bias=b[g], resid=r[g], ldr=N)
             for g in range(G)]
    lns = [L.GemmLnProblem(gam[g].data_ptr(), bet[g].data_ptr(), y[g].data_ptr(), mean[g].data_ptr(),
                           rstd[g].data_ptr()) for g in range(G)]

    def fused():
        ops.gemm_ln(probs, lns, 1e-5)

    def split():
        ops.gemm(L.GEMM_NT, probs)
        arr = (L.LnFwdProblem * G)(*[L.LnFwdProblem(v[g].data_ptr(), None, gam[g].data_ptr(), bet[g].data_ptr(),
                                                     None, y[g].data_ptr(), mean[g].data_ptr(), rstd[g].data_ptr(),
                                                     0, 0, 0.0) for g in range(G)])
        L.check(L.lib().sca_layernorm_fwd(G, arr, M, N, M, 0, 1e-5, L.stream_handle()), "ln")

    # the next op's projection (fc1: 768 wide, bias + GELU) chained into the launch, vs the
    # fused launch followed by a stand-alone NT GEMM
    W1 = [torch.randn(768, N, device=dev) / N ** 0.5 for _ in range(G)]
    b1 = [torch.randn(768, device=dev) for _ in range(G)]
    z = [torch.empty(M, 768, device=dev) for _ in range(G)]
    act = [torch.empty(M, 768, device=dev) for _ in range(G)]
    nxt = ops.NextProjections([[(W1[g], b1[g], 1.0, True)] for g in range(G)])

    def chained():
        ops.gemm_ln(probs, ops._chain_lns(nxt, G, M, v[0], gam, bet, y, mean, rstd), 1e-5)

    def unchained():
        ops.gemm_ln(probs, lns, 1e-5)
        ops.gemm(L.GEMM_NT, [ops._prob([ops._seg(y[g], W1[g], N, N, N)], act[g], M, 768, 768, bias=b1[g],
                                       epi=L.EPI_GELU, aux_out=z[g], ldo=768) for g in range(G)])

    keep = (A, W, b, r, gam, bet, v, y, mean, rstd, W1, b1, z, act)
    return dict(name=f"{G}x(M={M}, N={N}, K={K})", fused=fused, split=split, flops=2.0 * G * M * N * K, keep=keep,
                chained=chained, unchained=unchained, cflops=2.0 * G * M * N * (K + 768))


def timed(fn, iters):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    for c in [case(4, 2048, 256), case(4, 2048, 768), case(1, 2048, 256)]:
        c["fused"]()
        c["split"]()
        torch.cuda.synchronize()
        tf, ts = timed(c["fused"], args.iters), timed(c["split"], args.iters)
        print(f"{c['name']:28s} fused {tf:7.2f} us ({c['flops'] / tf / 1e6:6.1f} TFLOP/s)   "
              f"gemm+ln {ts:7.2f} us")
        c["chained"]()
        torch.cuda.synchronize()
        tc, tu = timed(c["chained"], args.iters), timed(c["unchained"], args.iters)
        print(f"{'':28s} + fc1 chained {tc:7.2f} us ({c['cflops'] / tc / 1e6:6.1f} TFLOP/s)   "
              f"fused + NT GEMM {tu:7.2f} us")


if __name__ == "__main__":
    main()
