"""Microbenchmark of the weight-gradient (TN) GEMM launches of a config-2 step, per kernel
tile and split-K, interleaved in one process; every variant is first checked against a
float64 host product (dW and the fused bias gradient).

    python tools/tn_bench.py [--iters 20] [--rounds 3] [--tiles 21,36,37] [--splits 1,2,3,4]

Shapes (per step: 12 + 16 launches): the attention blocks' q/k/v/o of 4 streams =
16 x (256 x 256, K = 2048); the FFN fc1 4 x (768 x 256) and fc2 4 x (256 x 768), K = 2048.
Tiles: 21 = gemm_glds_kernel<TN, 2> (64x64 LDS-DMA, 4 waves), 36 / 37 = gemm_tnk_kernel<3 / 4, 1>
(the k-split outer-product kernel, 3- / 4-stage ring)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import _lib as L, ops  # noqa: E402

NAMES = {1: "reg64", 5: "reg64s1", 7: "reg128x64", 20: "glds64s3", 21: "glds64", 22: "glds64s4", 36: "TNKs3", 37: "TNKs4"}
TILE_BM = {1: (64, 64), 5: (64, 64), 7: (128, 64), 20: (64, 64), 21: (64, 64), 22: (64, 64), 36: (64, 64), 37: (64, 64)}


def make_case(name, shapes, Mr=2048):
    dev = "cuda"
    items = []
    for (n_out, n_in) in shapes:
        dY, X = torch.randn(Mr, n_out, device=dev), torch.randn(Mr, n_in, device=dev)
        dW, db = torch.empty(n_out, n_in, device=dev), torch.empty(n_out, device=dev)
        items.append((dY, X, dW, db))
    flops = sum(2.0 * Mr * a * b for a, b in shapes)
    return dict(name=name, items=items, flops=flops, Mr=Mr)


def probs_for(c):
    return [ops._prob([ops._seg(dY, X, dW.shape[0], dW.shape[1], c["Mr"])], dW, dW.shape[0], dW.shape[1],
                      dW.shape[1], bias_grad=db) for dY, X, dW, db in c["items"]]


def run(c, sk):
    ws = c.setdefault("ws", {}).get(sk)
    if sk > 1 and ws is None:
        n = sum(sk * (dW.numel() + dW.shape[0]) for _, _, dW, _ in c["items"])
        ws = c["ws"][sk] = torch.empty(n, device="cuda")
    ops.gemm(L.GEMM_TN, c["probs"], splitk=sk, ws=ws)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tiles", default="21,36,37")
    ap.add_argument("--splits", default="1,2,3,4,6")
    args = ap.parse_args()
    tiles = [int(t) for t in args.tiles.split(",")]
    splits = [int(s) for s in args.splits.split(",")]
    cases = [make_case("attn 16x(256,256)", [(256, 256)] * 16), make_case("fc1 4x(768,256)", [(768, 256)] * 4),
             make_case("fc2 4x(256,768)", [(256, 768)] * 4)]
    lib = L.lib()
    for c in cases:
        c["probs"] = probs_for(c)
        c["ref"] = [(dY.double().cpu().T @ X.double().cpu(), dY.double().cpu().sum(0)) for dY, X, _, _ in c["items"]]
    variants = []
    for c in cases:
        for t in tiles:
            bm, bn = TILE_BM[t]
            ntile = sum(-(-dW.shape[0] // bm) * -(-dW.shape[1] // bn) for _, _, dW, _ in c["items"])
            for sk in splits:
                if c["Mr"] // sk < 256 and sk > 1:
                    continue
                lib.sca_gemm_tile_override(L.GEMM_TN, t)
                for _, _, dW, db in c["items"]:
                    dW.fill_(float("nan"))
                    db.fill_(float("nan"))
                run(c, sk)
                torch.cuda.synchronize()
                for (_, _, dW, db), (rw, rb) in zip(c["items"], c["ref"]):
                    ew = float((dW.double().cpu() - rw).abs().max() / rw.abs().max())
                    eb = float((db.double().cpu() - rb).abs().max() / rb.abs().max())
                    if t not in (40, 41, 42, 43):  # 40, 41: the no-DMA timing probes computes garbage by design
                        assert ew < 1e-5 and eb < 1e-5, (c["name"], t, sk, ew, eb)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(args.iters):
                        run(c, sk)
                variants.append((c, t, sk, ntile * sk, g))
    lib.sca_gemm_tile_override(L.GEMM_TN, 0)
    res = {}
    for _ in range(args.rounds):
        for (c, t, sk, nwg, g) in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            res.setdefault((c["name"], t, sk), []).append(us)
    for (c, t, sk, nwg, g) in variants:
        us = min(res[(c["name"], t, sk)])
        print(f"{c['name']:20s} {NAMES[t]:10s} sk={sk}  wg={nwg:5d}  {us:8.2f} us  {c['flops'] / us / 1e6:7.1f} TFLOP/s "
              f"({c['flops'] / us / 1e6 / 157.3:.3f})", flush=True)


if __name__ == "__main__":
    main()
