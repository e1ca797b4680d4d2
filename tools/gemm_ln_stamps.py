"""Where a fused GEMM + LayerNorm launch's time goes (diagnostic stamps build, make -C
scattennet_amd/csrc stamps): per-workgroup s_memrealtime at entry, main loop done, LayerNorm
done, first chained pass done, end — for the workload's out-projection + fc1-chain and
fc2 + qkv-chain launches (4 streams x 2048 rows, 32-row tiles).

    python tools/gemm_ln_stamps.py [other_stamps_build.so]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import _lib as L, ops  # noqa: E402

# the stamps build (or, A/B, another stamps build given as the first argument)
L.LIB_PATH = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(L.LIB_PATH), "libscatten_hip_stamps.so")


def run_case(name, G, M, K, passes):
    dev = "cuda"
    N = 256
    A = [torch.randn(M, K, device=dev) for _ in range(G)]
    W = [torch.randn(N, K, device=dev) / K ** 0.5 for _ in range(G)]
    b = [torch.randn(N, device=dev) for _ in range(G)]
    r = [torch.randn(M, N, device=dev) for _ in range(G)]
    gam = [torch.ones(N, device=dev) for _ in range(G)]
    bet = [torch.zeros(N, device=dev) for _ in range(G)]
    v, y = [torch.empty(M, N, device=dev) for _ in range(G)], [torch.empty(M, N, device=dev) for _ in range(G)]
    mean, rstd = [torch.empty(M, device=dev) for _ in range(G)], [torch.empty(M, device=dev) for _ in range(G)]
    probs = [ops._prob([ops._seg(A[g], W[g], K, K, K)], v[g], M, N, N, bias=b[g], resid=r[g], ldr=N)
             for g in range(G)]
    specs = [[(torch.randn(256 * (3 if gelu else 1), N, device=dev) / 16, torch.randn(256 * (3 if gelu else 1),
               device=dev), 1.0, gelu) for gelu in passes] for _ in range(G)]
    nxt = ops.NextProjections(specs)
    lns = ops._chain_lns(nxt, G, M, v[0], gam, bet, y, mean, rstd)
    for _ in range(3):
        ops.gemm_ln(probs, lns, 1e-5)
    torch.cuda.synchronize()
    ops.gemm_ln(probs, lns, 1e-5)
    torch.cuda.synchronize()
    nwg = G * M // 32
    buf = np.zeros((nwg, 5), dtype=np.uint64)
    L.lib().sca_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.lib().sca_gemm_stamps(buf.ctypes.data, nwg) == 0
    st = buf.astype(np.int64)
    t0 = st[:, 0].min()
    us = (st - t0) / 100.0
    ph = {"main loop": us[:, 1] - us[:, 0], "LayerNorm": us[:, 2] - us[:, 1], "pass 1": us[:, 3] - us[:, 2],
          "rest of passes": us[:, 4] - us[:, 3]}
    print(f"{name}: span {us[:, 4].max():.1f} us, entry ramp max {us[:, 0].max():.1f} | " +
          " | ".join(f"{k} p50 {np.median(x):.2f} max {x.max():.2f}" for k, x in ph.items()), flush=True)


def main():
    run_case("out-proj K=256 + fc1 (GELU, 768)", 4, 2048, 256, [True])
    run_case("fc2 K=768 + q/k/v (3 x 256)", 4, 2048, 768, [False, False, False])


if __name__ == "__main__":
    main()
