"""Where a short-K GEMM launch's time goes: per-workgroup s_memrealtime stamps (100 MHz) of
the diagnostic build (make -C scattennet_amd/csrc stamps -> libscatten_hip_stamps.so) at
entry, first K-slice landed, main loop done, epilogue stored.  One launch per case after
warm-up, alone on the GPU.

    python tools/gemm_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import _lib as L, ops  # noqa: E402

L.LIB_PATH = os.path.join(os.path.dirname(L.LIB_PATH), "libscatten_hip_stamps.so")
from tools.gemm_bench import make_case  # noqa: E402


def main():
    lib = L.lib()
    lib.sca_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    M, d, F = 2048, 256, 768
    cases = [
        make_case("NT out 4x(2048,256,256)", L.GEMM_NT, [(M, d, d)] * 4),
        make_case("NT qkv 12x(2048,256,256)", L.GEMM_NT, [(M, d, d)] * 12),
        make_case("NT ffn2 4x(2048,256,768)", L.GEMM_NT, [(M, d, F)] * 4),
        make_case("NN dffn1 4x(2048,768,256)", L.GEMM_NN, [(M, F, d)] * 4),
        make_case("TN dW 16x(256,256,2048) sk3", L.GEMM_TN, [(d, d, M)] * 16, splitk=3),
        make_case("TN dW 16x(256,256,2048) sk1", L.GEMM_TN, [(d, d, M)] * 16, splitk=1),
    ]
    lib.sca_gemm_clk.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for c in cases:
        for _ in range(3):
            ops.gemm(c["layout"], c["probs"], c["splitk"], c["ws"])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.sca_gemm_partial(c["layout"], len(c["probs"]), (L.GemmProblem * len(c["probs"]))(*c["probs"]),
                             c["splitk"], L.ptr(c["ws"]), L.stream_handle())
        e1.record()
        torch.cuda.synchronize()
        nwg = sum(((p.M + 63) // 64) * ((p.N + 63) // 64) for p in c["probs"]) * c["splitk"]
        if c["layout"] != L.GEMM_TN:
            nwg = max(((p.N + 63) // 64) for p in c["probs"]) * max(((p.M + 63) // 64) for p in c["probs"]) * \
                len(c["probs"]) * c["splitk"]
        buf = np.zeros((nwg, 5), dtype=np.uint64)
        assert lib.sca_gemm_stamps(buf.ctypes.data, nwg) == 0
        clk = np.zeros((nwg, 2), dtype=np.uint64)
        assert lib.sca_gemm_clk(clk.ctypes.data, nwg) == 0
        st = buf[:, :4].astype(np.int64)
        ok = st[:, 2] > 0
        ghz = (clk[ok, 1].astype(np.float64) - clk[ok, 0]) / ((st[ok, 2] - st[ok, 0]) / 100.0) / 1e3
        st = st[ok]
        st[:, 3] = np.where(st[:, 3] > 0, st[:, 3], st[:, 2])  # split-K slabs: no epilogue stamp
        t0 = st[:, 0].min()
        us = (st - t0) / 100.0  # 100 MHz ticks -> us
        first, loop, epi = us[:, 1] - us[:, 0], us[:, 2] - us[:, 1], us[:, 3] - us[:, 2]
        print(f"{c['name']:30s} wgs={len(st):5d} event {e0.elapsed_time(e1) * 1e3:6.1f} us | span "
              f"{us[:, 3].max():6.1f} | entry ramp {us[:, 0].max():5.1f} (p50 {np.median(us[:, 0]):5.1f}) | "
              f"first-slice p50 {np.median(first):4.1f} max {first.max():4.1f} | loop p50 {np.median(loop):5.1f} "
              f"max {loop.max():5.1f} | epilogue p50 {np.median(epi):4.1f} max {epi.max():4.1f} | "
              f"last start {us[:, 0].max():5.1f} first end {us[:, 3].min():5.1f} | in-kernel clock p50 "
              f"{np.median(ghz):.2f} GHz")


if __name__ == "__main__":
    main()
