"""NT / NN GEMMs and the fused GEMM + LayerNorm against the library (torch.bmm / baddbmm ->
hipBLASLt, F.layer_norm) at the step shapes of configs 2 and 5.  Ours: the launcher's default
kernel choice, graph-captured (`iters` launches per replay; every operand kept alive for the
whole run).  Library: back-to-back eager launches (no host gaps at these kernel lengths) on the
problems stacked into one tensor (the stacking copies are not timed).

    python tools/nt_library_compare.py [--iters 20]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

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


def eager_time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def gemm_case(lay, G, M, N, K):
    dev = "cuda"
    A = [torch.randn(M, K, device=dev) for _ in range(G)]
    if lay == "NT":
        B = [torch.randn(N, K, device=dev) / K ** 0.5 for _ in range(G)]
        probs_seg = lambda g: ops._seg(A[g], B[g], K, K, K)  # noqa: E731
        Bt = torch.stack(B).transpose(1, 2)
    else:
        B = [torch.randn(K, N, device=dev) / K ** 0.5 for _ in range(G)]
        probs_seg = lambda g: ops._seg(A[g], B[g], K, N, K)  # noqa: E731
        Bt = torch.stack(B)
    C = [torch.empty(M, N, device=dev) for _ in range(G)]
    probs = [ops._prob([probs_seg(g)], C[g], M, N, N) for g in range(G)]
    At = torch.stack(A)
    KEEP.append((A, B, C, probs, At, Bt))
    ours = lambda: ops.gemm(L.GEMM_NT if lay == "NT" else L.GEMM_NN, probs)  # noqa: E731
    lib = lambda: torch.bmm(At, Bt)  # noqa: E731
    ours()
    ref = lib()
    torch.cuda.synchronize()
    err = float((torch.stack(C) - ref).abs().max() / ref.abs().max())
    name = ops._gemm_kernel_name(L.GEMM_NT if lay == "NT" else L.GEMM_NN, probs, 0).split("(")[0]
    return ours, lib, 2.0 * G * M * N * K, err, name


def ln_case(G, M, N, K):
    """v = A W^T + b + r, y = LayerNorm(v): sca_gemm_ln vs baddbmm + layer_norm."""
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
    At, Wt = torch.stack(A), torch.stack(W).transpose(1, 2)
    Rb = torch.stack(r) + torch.stack(b)[:, None, :]
    KEEP.append((A, W, b, r, gam, bet, v, y, mean, rstd, probs, lns, At, Wt, Rb))
    ours = lambda: ops.gemm_ln(probs, lns, 1e-5)  # noqa: E731
    lib = lambda: F.layer_norm(torch.baddbmm(Rb, At, Wt), (N,))  # noqa: E731
    ours()
    ref = lib()
    torch.cuda.synchronize()
    err = float((torch.stack(y) - ref).abs().max() / ref.abs().max())
    return ours, lib, 2.0 * G * M * N * K, err, "gemm_ln" + ("_reg" if ops._ln_reg(probs) else "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="", help="run the cases whose name starts with this")
    args = ap.parse_args()
    torch.manual_seed(0)
    peak = 157.3
    cases = [
        ("cfg2 NT qkv", gemm_case, ("NT", 12, 2048, 256, 256)),
        ("cfg2 NT fc1", gemm_case, ("NT", 4, 2048, 768, 256)),
        ("cfg2 NT fc2", gemm_case, ("NT", 4, 2048, 256, 768)),
        ("cfg2 NN dX qkv", gemm_case, ("NN", 4, 2048, 256, 768)),
        ("cfg2 NN dX fc2", gemm_case, ("NN", 4, 2048, 768, 256)),
        ("cfg2 GEMM+LN fc2", ln_case, (4, 2048, 256, 768)),
        ("cfg2 GEMM+LN out", ln_case, (4, 2048, 256, 256)),
        ("cfg5 NT qkv", gemm_case, ("NT", 12, 8192, 512, 512)),
        ("cfg5 NT fc1", gemm_case, ("NT", 4, 8192, 1536, 512)),
        ("cfg5 NT fc2", gemm_case, ("NT", 4, 8192, 512, 1536)),
        ("cfg5 NN dX qkv", gemm_case, ("NN", 4, 8192, 512, 1536)),
        ("cfg5 NN dX fc2", gemm_case, ("NN", 4, 8192, 1536, 512)),
        ("cfg5 GEMM+LN fc2", ln_case, (4, 8192, 512, 1536)),
    ]
    print(f"{'case':18s} {'ours kernel':28s} {'ours us':>8s} {'frac':>6s} {'library us':>10s} {'frac':>6s}  rel err")
    for name, mk, a in cases:
        if not name.startswith(args.only):
            continue
        ours, lib, flops, err, kname = mk(*a)
        to, tl = graph_time(ours, args.iters), eager_time(lib, args.iters)
        print(f"{name:18s} {kname:28s} {to:8.2f} {flops / to / 1e6 / peak:6.3f} {tl:10.2f} "
              f"{flops / tl / 1e6 / peak:6.3f}  {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
