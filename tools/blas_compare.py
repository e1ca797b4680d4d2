"""Diagnostic: the library fp32 GEMM (torch.bmm -> hipBLASLt / rocBLAS) against this repo's
grouped MFMA GEMM at the cfg2 weight-gradient / input-gradient shapes.

    python tools/blas_compare.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import _lib as L, ops  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    dev = "cuda"
    torch.manual_seed(0)
    # (name, G, M_out, N_out, K, layout): TN = dW[M_out, N_out] = dY^T X over K rows
    cases = [("TN qkv+o dW", 16, 256, 256, 2048, "TN"), ("TN fc1 dW", 4, 1024, 256, 2048, "TN"),
             ("TN fc2 dW", 4, 256, 1024, 2048, "TN"), ("NN dX qkv", 4, 2048, 256, 768, "NN"),
             ("NN dX fc2", 4, 2048, 1024, 256, "NN"), ("NT fc1", 4, 2048, 1024, 256, "NT")]
    for name, G, M, N, K, lay in cases:
        flops = 2.0 * G * M * N * K
        if lay == "TN":
            A = [torch.randn(K, M, device=dev) for _ in range(G)]
            B = [torch.randn(K, N, device=dev) for _ in range(G)]
            At, Bt = torch.stack(A), torch.stack(B)
            blas = lambda: torch.bmm(At.transpose(1, 2), Bt)  # noqa: E731
            C = [torch.empty(M, N, device=dev) for _ in range(G)]
            probs = [ops._prob([ops._seg(A[g], B[g], M, N, K)], C[g], M, N, N) for g in range(G)]
            sk = ops._splitk_for(K, G * ((M + 63) // 64) * ((N + 63) // 64))
            ws = torch.empty(G * sk * (M * N + M), device=dev) if sk > 1 else None
            ours = lambda: ops.gemm(L.GEMM_TN, probs, splitk=sk, ws=ws)  # noqa: E731
        elif lay == "NN":
            A = [torch.randn(M, K, device=dev) for _ in range(G)]
            B = [torch.randn(K, N, device=dev) for _ in range(G)]
            At, Bt = torch.stack(A), torch.stack(B)
            blas = lambda: torch.bmm(At, Bt)  # noqa: E731
            C = [torch.empty(M, N, device=dev) for _ in range(G)]
            probs = [ops._prob([ops._seg(A[g], B[g], K, N, K)], C[g], M, N, N) for g in range(G)]
            ours = lambda: ops.gemm(L.GEMM_NN, probs)  # noqa: E731
        else:
            A = [torch.randn(M, K, device=dev) for _ in range(G)]
            B = [torch.randn(N, K, device=dev) for _ in range(G)]
            At, Bt = torch.stack(A), torch.stack(B)
            blas = lambda: torch.bmm(At, Bt.transpose(1, 2))  # noqa: E731
            C = [torch.empty(M, N, device=dev) for _ in range(G)]
            probs = [ops._prob([ops._seg(A[g], B[g], K, K, K)], C[g], M, N, N) for g in range(G)]
            ours = lambda: ops.gemm(L.GEMM_NT, probs)  # noqa: E731
        tb, to = timeit(blas), timeit(ours)
        ref = blas()
        got = torch.stack(C)
        err = float((got - ref).abs().max() / ref.abs().max())
        print(f"{name:14s} G={G:2d} {M}x{N}x{K}: blas {tb:7.1f} us {flops / tb / 1e6:6.1f} TF   "
              f"ours {to:7.1f} us {flops / to / 1e6:6.1f} TF   rel err {err:.1e}")


if __name__ == "__main__":
    main()
