"""Weight-gradient (TN) GEMM shapes of configs 2, 3 and 5: this library's k-split kernel (tile 36,
the launcher's choice for these launches) at split-K 2 / 3 against the library GEMM (torch.bmm -> hipBLASLt, no bias gradient).  Our launches are checked against
float64 first and timed as graph replays of --iters launches; the library (--library, its own
process) eagerly, back-to-back; best of --rounds.  Round 5's stream-K kernels were measured with
this tool (profiles/r05_tn/) and removed.  (Round 5's stream-K kernels were measured with this tool: profiles/r05_tn/.)

    python tools/tn_library_compare.py [--iters 20] [--rounds 3] [--only cfg2,cfg3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import _lib as L, ops  # noqa: E402

PEAK = 157.3
SPLITS = (1, 2, 3, 4, 5, 6, 8)  # --splits
TNB_TILES = (38, 39, 40, 43)  # --tnb-tiles
KSPLIT_TILES = (36, 46)  # --ksplit-tiles
KSPLIT_SPLITS = (2, 3, 4)  # --ksplit-splits
LIBRARY = False  # --library: the hipBLASLt timings only, eagerly, in a process that captures no graph


def case(name, shapes, K):
    items = []
    for (M, N) in shapes:
        dY, X = torch.randn(K, M, device="cuda"), torch.randn(K, N, device="cuda")
        items.append((dY, X, torch.empty(M, N, device="cuda"), torch.empty(M, device="cuda")))
    return dict(name=name, items=items, flops=sum(2.0 * K * M * N for M, N in shapes), K=K)


def probs(c):
    return [ops._prob([ops._seg(dY, X, dW.shape[0], dW.shape[1], c["K"])], dW, dW.shape[0], dW.shape[1], dW.shape[1],
                      bias_grad=db) for dY, X, dW, db in c["items"]]


def variants(c):
    P = probs(c)
    out = []
    tiles = sum(-(-dW.shape[0] // 64) * -(-dW.shape[1] // 64) for _, _, dW, _ in c["items"])
    for sk in KSPLIT_SPLITS:
        ws = torch.empty(sum(sk * (dW.numel() + dW.shape[0]) for _, _, dW, _ in c["items"]), device="cuda")
        for tl in KSPLIT_TILES:
            out.append((f"ksplit{tl} sk={sk} wg={tiles * sk}", lambda sk=sk, ws=ws, tl=tl: ops.gemm(
                L.GEMM_TN, P, splitk=sk, ws=ws, tile=tl)))
    t128 = sum(-(-dW.shape[0] // 128) * -(-dW.shape[1] // 128) for _, _, dW, _ in c["items"])
    for sk in SPLITS:
        if c["K"] // sk < 256 and sk > 1:
            continue
        ws = torch.empty(sum(sk * (dW.numel() + dW.shape[0]) for _, _, dW, _ in c["items"]), device="cuda")
        for tl in TNB_TILES:
            if not tl:
                continue
            out.append((f"tnb{tl} sk={sk} wg={t128 * sk}", lambda sk=sk, ws=ws, tl=tl: ops.gemm(
                L.GEMM_TN, P, splitk=sk, ws=ws, tile=tl)))
    if LIBRARY and len({dW.shape for _, _, dW, _ in c["items"]}) == 1:
        out.clear()
        A = torch.stack([dY for dY, _, _, _ in c["items"]])
        B = torch.stack([X for _, X, _, _ in c["items"]])
        C = torch.empty(len(c["items"]), A.shape[2], B.shape[2], device="cuda")
        out.append(("hipBLASLt bmm (no bias)", lambda: torch.bmm(A.transpose(1, 2), B, out=C)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--library", action="store_true",
                    help="time only torch.bmm (hipBLASLt), eagerly; without it, only this library's kernels "
                         "(graphs): the two never share a process — round 5 saw two illegal-address faults in "
                         "processes that mixed hipBLASLt calls with graph replays (profiles/r05_tn/)")
    ap.add_argument("--only", default="", help="comma-separated substrings of case names to run")
    ap.add_argument("--profile", default="", help="run the variants whose names contain this, eagerly, "
                                                   "--iters times each, for rocprofv3 counter passes "
                                                   "(tools/tn_pmc2.py)")
    ap.add_argument("--splits", default="1,2,3,4,5,6,8", help="split-K values of the 128x128 kernels")
    ap.add_argument("--tnb-tiles", default="38,39,40,43", help="variant ids of the 128x128 kernel")
    ap.add_argument("--ksplit-tiles", default="36,46", help="variant ids of the 64x64 k-split kernel")
    ap.add_argument("--ksplit-splits", default="2,3,4", help="split-K values of the 64x64 k-split kernels")
    args = ap.parse_args()
    global LIBRARY, SPLITS, TNB_TILES, KSPLIT_TILES, KSPLIT_SPLITS
    KSPLIT_TILES = tuple(int(x) for x in args.ksplit_tiles.split(",") if x)
    KSPLIT_SPLITS = tuple(int(x) for x in args.ksplit_splits.split(",") if x)
    SPLITS = tuple(int(x) for x in args.splits.split(",") if int(x) > 0)
    TNB_TILES = tuple(int(x) for x in args.tnb_tiles.split(","))
    LIBRARY = args.library
    torch.manual_seed(0)
    cases = [case("cfg2 attn 16x(256,256)", [(256, 256)] * 16, 2048),
             case("cfg2 fc1 4x(768,256)", [(768, 256)] * 4, 2048),
             case("cfg2 fc2 4x(256,768)", [(256, 768)] * 4, 2048),
             case("cfg3 attn 12x(256,256)", [(256, 256)] * 12, 2048),
             case("cfg3 res0 6x(256,256)", [(256, 256)] * 6, 2048),
             case("cfg3 res1 6x(256,256)", [(256, 256)] * 6, 1024),
             case("cfg3 res2 3x(512,512)", [(512, 512)] * 3, 1024),
             case("cfg3 res3 6x(512,512)", [(512, 512)] * 6, 512),
             case("cfg3 fusion se 3x(1024,512)", [(1024, 512)] * 3, 512),
             case("cfg3 fusion inv 1x(3072,1024)", [(3072, 1024)], 512),
             case("cfg5 attn 16x(512,512)", [(512, 512)] * 16, 8192),
             case("cfg5 fc1 4x(1536,512)", [(1536, 512)] * 4, 8192)]
    runs = []
    keep = []
    if args.only:
        cases = [c for c in cases if any(o in c["name"] for o in args.only.split(","))]
    if args.profile:
        for c in cases:
            for name, fn in variants(c):
                if any(p in name for p in args.profile.split(",")):
                    for _ in range(args.iters):
                        fn()
                    torch.cuda.synchronize()
                    print("profiled", c["name"], name, flush=True)
        return
    print("checking + capturing", flush=True)
    for c in cases:
        print(" ", c["name"], flush=True)
        ref = [(dY.double().t() @ X.double(), dY.double().sum(0)) for dY, X, _, _ in c["items"]]
        for name, fn in variants(c):
            for _, _, dW, db in c["items"]:
                dW.fill_(float("nan"))
                db.fill_(float("nan"))
            fn()
            torch.cuda.synchronize()
            if "bmm" not in name:
                for (_, _, dW, db), (rw, rb) in zip(c["items"], ref):
                    ew = float((dW.double() - rw).abs().max() / rw.abs().max())
                    eb = float((db.double() - rb).abs().max() / rb.abs().max())
                    assert ew < 2e-5 and eb < 2e-5, (c["name"], name, ew, eb)
            for ring, _ in ops._CNT.values():  # every tile counter back at zero
                assert int(ring.abs().sum()) == 0, (c["name"], name, "tile counters left non-zero")
            if "bmm" in name:  # the library eagerly (not captured): launches back to back
                runs.append((c, name, fn))
                continue
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(args.iters):
                    fn()
            # the graph bakes in the addresses of the variant's split-K workspace, which only the
            # lambda holds: keep it alive (every later torch.cuda.graph() capture starts with
            # empty_cache(), which hands freed blocks back to the driver, and a replay into them
            # faults — the cause of round 5's two "illegal address" faults in this tool)
            keep.append(fn)
            runs.append((c, name, g))
    best = {}
    print("timing", flush=True)
    for c, name, g in runs:  # one checked replay each first: a fault names its variant
        print(" ", c["name"], name, flush=True)
        g.replay() if isinstance(g, torch.cuda.CUDAGraph) else g()
        torch.cuda.synchronize()
    for _ in range(args.rounds):
        for c, name, g in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if isinstance(g, torch.cuda.CUDAGraph):
                g.replay()
            else:
                for _ in range(args.iters):
                    g()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            k = (c["name"], name)
            best[k] = min(best.get(k, 1e30), us)
    for c, name, _ in runs:
        us = best[(c["name"], name)]
        tf = c["flops"] / us / 1e6
        print(f"{c['name']:24s} {name:28s} {us:8.2f} us {tf:7.1f} TFLOP/s ({tf / PEAK:.3f})", flush=True)


if __name__ == "__main__":
    main()
