"""Microbenchmark of the grouped fp32-MFMA GEMM at the SCA workload's shapes, per tile
config (sca_gemm_tile_override), interleaved in one process.  Checks each result against a
float64 host product first.

    python tools/gemm_bench.py [--iters 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import _lib as L, ops  # noqa: E402

TILES = {1: "64x64", 5: "64s1", 7: "128x64w8", 20: "G64s3", 21: "G64s2", 22: "G64s4", 41: "NTB128i", 42: "NTB128", 44: "NTB128il", 45: "NTB64il"}


def make_case(name, layout, shapes, splitk=1, segs=1):
    """shapes: list of (M, N, K) per problem (K per segment)."""
    dev = "cuda"
    probs, keep, refs = [], [], []
    for (M, N, K) in shapes:
        C = torch.empty(M, N, device=dev)
        seglist = []
        ref = torch.zeros(M, N, dtype=torch.float64)
        for _ in range(segs):
            if layout == L.GEMM_NT:
                A, B = torch.randn(M, K, device=dev), torch.randn(N, K, device=dev)
                seglist.append(ops._seg(A, B, K, K, K))
                ref += A.double().cpu() @ B.double().cpu().T
            elif layout == L.GEMM_NN:
                A, B = torch.randn(M, K, device=dev), torch.randn(K, N, device=dev)
                seglist.append(ops._seg(A, B, K, N, K))
                ref += A.double().cpu() @ B.double().cpu()
            else:
                A, B = torch.randn(K, M, device=dev), torch.randn(K, N, device=dev)
                seglist.append(ops._seg(A, B, M, N, K))
                ref += A.double().cpu().T @ B.double().cpu()
            keep += [A, B]
        probs.append(ops._prob(seglist, C, M, N, N))
        keep.append(C)
        refs.append((C, ref))
    flops = sum(2.0 * M * N * K * segs for (M, N, K) in shapes)
    ws = None
    if splitk > 1:
        M, N, _ = shapes[0]
        ws = torch.empty(len(shapes) * splitk * (M * N + M), device=dev)
    return dict(name=name, layout=layout, probs=probs, keep=keep, refs=refs, flops=flops, splitk=splitk, ws=ws)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--lib", default=None, help="alternative build of the library (ablation experiments)")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--cases", default="", help="comma-separated substrings selecting cases")
    ap.add_argument("--tiles", default="", help="comma-separated tile ids")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--kscan", action="store_true", help="fixed-cost probe: NT 4x/12x(2048,256,K) over K")
    ap.add_argument("--cfg5", action="store_true", help="config 5's NT / NN shapes (B x T = 8192 rows, d 512)")
    args = ap.parse_args()
    if args.lib:
        L.LIB_PATH = os.path.abspath(args.lib)
    M = 2048
    d, F = 256, 768
    cases = [
        make_case("NT qkv 12x(2048,256,256)", L.GEMM_NT, [(M, d, d)] * 12),
        make_case("NT out 4x(2048,256,256)", L.GEMM_NT, [(M, d, d)] * 4),
        make_case("NT ffn1 4x(2048,768,256)", L.GEMM_NT, [(M, F, d)] * 4),
        make_case("NT ffn2 4x(2048,256,768)", L.GEMM_NT, [(M, d, F)] * 4),
        make_case("NN dx-qkv 4x(2048,256,3x256)", L.GEMM_NN, [(M, d, d)] * 4, segs=3),
        make_case("NN dffn1 4x(2048,768,256)", L.GEMM_NN, [(M, F, d)] * 4),
        make_case("NN dffn2 4x(2048,256,768)", L.GEMM_NN, [(M, d, F)] * 4),
        make_case("TN dW 12x(256,256,2048) sk4", L.GEMM_TN, [(d, d, M)] * 12, splitk=4),
        make_case("TN dW 12x(256,256,2048) sk2", L.GEMM_TN, [(d, d, M)] * 12, splitk=2),
        make_case("NT as-dW 12x(256,256,2048) sk4", L.GEMM_NT, [(d, d, M)] * 12, splitk=4),
        make_case("TN dW 12x(256,256,2048) sk1", L.GEMM_TN, [(d, d, M)] * 12, splitk=1),
        make_case("TN dW 16x(256,256,2048) sk1", L.GEMM_TN, [(d, d, M)] * 16, splitk=1),
        make_case("TN dW 16x(256,256,2048) sk3", L.GEMM_TN, [(d, d, M)] * 16, splitk=3),
        make_case("TN dW 16x(256,256,2048) sk2", L.GEMM_TN, [(d, d, M)] * 16, splitk=2),
        make_case("TN dW12 8x(mixed,2048) sk1", L.GEMM_TN, [(d, F, M)] * 4 + [(F, d, M)] * 4, splitk=1),
        make_case("TN dW2 4x(256,768,2048) sk4", L.GEMM_TN, [(d, F, M)] * 4, splitk=4),
        make_case("TN dW2 4x(256,768,2048) sk2", L.GEMM_TN, [(d, F, M)] * 4, splitk=2),
        # steady-state main loop (long K): 512 and 1536 64x64 tiles
        make_case("NT longK 4x(2048,256,4096)", L.GEMM_NT, [(M, d, 4096)] * 4),
        make_case("NT longK 12x(2048,256,2048)", L.GEMM_NT, [(M, d, 2048)] * 12),
    ]
    if args.cfg5:
        M5, d5, F5 = 8192, 512, 1536
        cases = [make_case("NT5 qkv 12x(8192,512,512)", L.GEMM_NT, [(M5, d5, d5)] * 12),
                 make_case("NT5 ffn1 4x(8192,1536,512)", L.GEMM_NT, [(M5, F5, d5)] * 4),
                 make_case("NT5 ffn2 4x(8192,512,1536)", L.GEMM_NT, [(M5, d5, F5)] * 4),
                 make_case("NN5 dffn1 4x(8192,512,1536)", L.GEMM_NN, [(M5, d5, F5)] * 4),
                 make_case("NN5 dffn2 4x(8192,1536,512)", L.GEMM_NN, [(M5, F5, d5)] * 4),
                 make_case("NN5 dx-qkv 4x(8192,512,3x512)", L.GEMM_NN, [(M5, d5, d5)] * 4, segs=3)] + cases
    if args.kscan:
        cases = [make_case(f"NT kscan {n}x(2048,256,{k})", L.GEMM_NT, [(M, d, k)] * n)
                 for n in (4, 12) for k in (32, 64, 128, 256, 512, 1024)]
    if args.cases:
        cases = [c for c in cases if any(k in c["name"] for k in args.cases.split(","))]
    if args.tiles:
        for k in list(TILES):
            if str(k) not in args.tiles.split(","):
                del TILES[k]
    lib = L.lib()

    def valid(layout, t):  # variant ids of one layout only (41 / 42: NT) are skipped elsewhere
        return lib.sca_gemm_tile_override(layout, t) == 0

    for c in cases:
        for t in TILES:
            if not valid(c["layout"], t):
                continue
            ops.gemm(c["layout"], c["probs"], c["splitk"], c["ws"])
            torch.cuda.synchronize()
            for C, ref in ([] if args.no_check else c["refs"]):
                err = float((C.double().cpu() - ref).abs().max() / ref.abs().max())
                assert err < 1e-5, (c["name"], TILES[t], err)
    print(f"{'case':34s} " + " ".join(f"{v:>9s}" for v in TILES.values()) + "   (TFLOP/s)")
    res = {}
    graphs = {}
    for c in cases:  # capture `iters` launches per (case, tile): times the GPU, not the Python launcher
        for t in TILES:
            if not valid(c["layout"], t):
                continue
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(args.iters):
                    ops.gemm(c["layout"], c["probs"], c["splitk"], c["ws"])
            graphs[(c["name"], t)] = g
    for rnd in range(args.rounds):
        for c in cases:
            for t in TILES:
                g = graphs.get((c["name"], t))
                if g is None:
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                tf = c["flops"] * args.iters / (e0.elapsed_time(e1) / 1e3) / 1e12
                res.setdefault((c["name"], t), []).append(tf)
    for c in cases:
        print(f"{c['name']:34s} " + " ".join(f"{max(res[(c['name'], t)]):9.1f}" if (c['name'], t) in res
                                              else f"{'-':>9s}" for t in TILES))
    for lay in range(3):
        lib.sca_gemm_tile_override(lay, 0)


if __name__ == "__main__":
    main()
