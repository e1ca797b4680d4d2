"""Stand-alone LayerNorm forward / backward launches (sca_layernorm_fwd / _bwd + the affine
reduction) at the config-2 and config-5 shapes, graph-captured, with the bytes each moves.

    python tools/ln_bench.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import _lib as L, ops  # noqa: E402

KEEP = []


def graph_time(fn, iters):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    KEEP.append(g)
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def case(G, rows, N, iters):
    dev = "cuda"
    x = [torch.randn(rows, N, device=dev) for _ in range(G)]
    dy = [torch.randn(rows, N, device=dev) for _ in range(G)]
    gam = [torch.randn(N, device=dev) for _ in range(G)]
    bet = [torch.randn(N, device=dev) for _ in range(G)]
    y = [torch.empty(rows, N, device=dev) for _ in range(G)]
    mean = [torch.empty(rows, device=dev) for _ in range(G)]
    rstd = [torch.empty(rows, device=dev) for _ in range(G)]
    KEEP.append((x, dy, gam, bet, y, mean, rstd))
    arr = (L.LnFwdProblem * G)(*[L.LnFwdProblem(x[g].data_ptr(), None, gam[g].data_ptr(), bet[g].data_ptr(),
                                                 None, y[g].data_ptr(), mean[g].data_ptr(), rstd[g].data_ptr(),
                                                 0, 0, 0.0) for g in range(G)])

    def fwd():
        L.check(L.lib().sca_layernorm_fwd(G, arr, rows, N, rows, 0, 1e-5, L.stream_handle()), "ln fwd")

    def bwd():
        out = ops._ln_bwd(dy, x, gam, mean, rstd)
        KEEP.append(out)

    def bwd_main():  # without the affine reduction
        out = ops._ln_bwd(dy, x, gam, mean, rstd, defer_affine=True)
        KEEP.append(out)

    tf = graph_time(fwd, iters)
    tb = graph_time(bwd, iters)
    tm = graph_time(bwd_main, iters)
    mb = G * rows * N * 4 / 1e6
    print(f"{G}x({rows}, {N})  fwd {tf:7.2f} us ({2 * mb / tf:5.2f} TB/s)   bwd+affine {tb:7.2f} us   "
          f"bwd {tm:7.2f} us ({3 * mb / tm:5.2f} TB/s over x, dy, dx)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    for G, rows, N in [(4, 2048, 256), (4, 8192, 512), (8, 8192, 512)]:
        case(G, rows, N, args.iters)


if __name__ == "__main__":
    main()
