"""Time sca_gemm_lnb (NN dX GEMM + LayerNorm backward in one launch) against the two launches
it replaces (NN sca_gemm + sca_layernorm_bwd) at the SCA shapes: 4 x (2048 x 256), K = 768 as
one segment (FFN dx = dz W1) or three of 256 (attention dX = dq Wq + dk Wk + dv Wv).
    python tools/lnb_bench.py [--iters 50] [--chains]

--chains: the attention-dX launch (K = 3 x 256) alone and with its chained pass(es) — the
out-projection (dO = dv Wo, 1 pass) and the FFN's (dz = (dv W2) gelu'(z), 3 passes) — so
that a chained pass's cost shows beside the main loop's.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import _lib as L, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--sweep", action="store_true", help="K = 32 .. 1536 (one segment): fixed cost vs slope")
    ap.add_argument("--chains", action="store_true", help="no chain / out-projection chain / FFN chain")
    a = ap.parse_args()
    if a.chains:
        return chains(a)
    dev = "cuda"
    M, N, G = 2048, 256, 4
    for Ks in (((32,), (256,), (512,), (768,), (1536,)) if a.sweep else ((768,), (256, 256, 256))):
        keep, probs, lnp = [], [], []
        for _ in range(G):
            segs = []
            for K in Ks:
                A, B = torch.randn(M, K, device=dev), torch.randn(K, N, device=dev)
                keep += [A, B]
                segs.append(ops._seg(A, B, K, N, K))
            C, r = torch.empty(M, N, device=dev), torch.randn(M, N, device=dev)
            keep += [C, r]
            probs.append(ops._prob(segs, C, M, N, N, resid=r, ldr=N))
            lnp.append(ops.LnSaved(torch.randn(M, N, device=dev), torch.zeros(M, device=dev),
                                   torch.ones(M, device=dev), torch.ones(N, device=dev)))
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        ops.gemm_lnb(probs, lnp)
        with torch.cuda.graph(g1):
            for _ in range(a.iters):
                ops.gemm_lnb(probs, lnp)
        Cs = [torch.empty(M, N, device=dev) for _ in range(G)]
        with torch.cuda.graph(g2):
            for _ in range(a.iters):
                ops.gemm(L.GEMM_NN, probs)
                ops._ln_bwd(Cs, [o.v for o in lnp], [o.gamma for o in lnp], [o.mean for o in lnp],
                            [o.rstd for o in lnp])
        flops = 2.0 * M * N * sum(Ks) * G
        for name, g in (("gemm_lnb", g1), ("gemm+ln_bwd", g2)):
            best = 1e9
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1e3 / a.iters)
            print(f"K={'+'.join(map(str, Ks)):12s} {name:12s} {best:7.2f} us  {flops / best / 1e6:6.1f} TFLOP/s")


def chains(a):
    dev = "cuda"
    M, N, G, Ks = 2048, 256, 4, (256, 256, 256)
    for chain in ("none", "attn", "ffn"):
        keep, probs, lnp = [], [], []
        for _ in range(G):
            segs = []
            for K in Ks:
                A, B = torch.randn(M, K, device=dev), torch.randn(K, N, device=dev) / 16
                keep += [A, B]
                segs.append(ops._seg(A, B, K, N, K))
            C, r = torch.empty(M, N, device=dev), torch.randn(M, N, device=dev)
            keep += [C, r]
            probs.append(ops._prob(segs, C, M, N, N, resid=r, ldr=N))
            n2 = {"none": 0, "attn": 256, "ffn": 768}[chain]
            wo = torch.randn(N, n2, device=dev) / 16 if n2 else None
            aux = torch.randn(M, n2, device=dev) if chain == "ffn" else None
            keep += [wo, aux]
            lnp.append(ops.LnSaved(torch.randn(M, N, device=dev), torch.zeros(M, device=dev),
                                   torch.ones(M, device=dev), torch.ones(N, device=dev), wo=wo, aux=aux))
        g = torch.cuda.CUDAGraph()
        ops.gemm_lnb(probs, lnp)
        with torch.cuda.graph(g):
            for _ in range(a.iters):
                ops.gemm_lnb(probs, lnp)
        flops = 2.0 * M * N * (sum(Ks) + {"none": 0, "attn": 256, "ffn": 768}[chain]) * G
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / a.iters)
        print(f"chain={chain:5s} {best:7.2f} us  {flops / best / 1e6:6.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
