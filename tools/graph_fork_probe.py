"""When do forked branches of a captured hipGraph run?  A chain of N matmuls on the capture
stream; MODE "one": after chain kernel F a side stream forks and runs S matmuls; MODE "each":
after every chain kernel i >= F a side kernel forks (event recorded before chain kernel i+1 is
captured: the side kernel is child 1, as the weight gradients of ops.weight_grads), all side
kernels on one side stream; joined at the end.  Run under rocprofv3 --kernel-trace and read the
start times (the last replay is printed).

    python tools/graph_fork_probe.py MODE N F S
"""
import os
import sys

os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "2")
import torch  # noqa: E402

MODE = sys.argv[1] if len(sys.argv) > 1 else "each"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 40
F = int(sys.argv[3]) if len(sys.argv) > 3 else 2
S = int(sys.argv[4]) if len(sys.argv) > 4 else 1
dev = torch.device("cuda", 0)
a = torch.randn(2048, 2048, device=dev)
w = torch.randn(2048, 2048, device=dev) / 45
b = torch.randn(1024, 1024, device=dev)
w2 = torch.randn(1024, 1024, device=dev) / 32
side = torch.cuda.Stream()
if MODE.startswith("lib") or MODE == "mmlib":
    # our kernels: the chain = fused GEMM + LayerNorm launches (1 workgroup / CU, 147 KB LDS), the
    # side = k-split weight-gradient launches (tools/gemm_ln_bench.py / the step's shapes)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from scattennet_amd import _lib as L, ops  # noqa: E402
    G, M, K = 4, 2048, 768
    A = [torch.randn(M, K, device=dev) for _ in range(G)]
    W = [torch.randn(256, K, device=dev) / K ** 0.5 for _ in range(G)]
    gam = [torch.ones(256, device=dev) for _ in range(G)]
    bet = [torch.zeros(256, device=dev) for _ in range(G)]
    v = [torch.empty(M, 256, device=dev) for _ in range(G)]
    yv = [torch.empty(M, 256, device=dev) for _ in range(G)]
    mean = [torch.empty(M, device=dev) for _ in range(G)]
    rstd = [torch.empty(M, device=dev) for _ in range(G)]
    probs = [ops._prob([ops._seg(A[g], W[g], K, K, K)], v[g], M, 256, 256) for g in range(G)]
    lns = [L.GemmLnProblem(gam[g].data_ptr(), bet[g].data_ptr(), yv[g].data_ptr(), mean[g].data_ptr(),
                           rstd[g].data_ptr()) for g in range(G)]
    dY = [torch.randn(M, 256, device=dev) for _ in range(16)]
    X = [torch.randn(M, 256, device=dev) for _ in range(16)]
    dW = [torch.empty(256, 256, device=dev) for _ in range(16)]
    tprobs = [ops._prob([ops._seg(dY[i], X[i], 256, 256, M)], dW[i], 256, 256, 256) for i in range(16)]
    ws = torch.empty(2 * 16 * (256 * 256 + 256), device=dev)

    def chain_op(x):
        ops.gemm_ln(probs, lns, 1e-5)
        return x

    SIDE_TILE = 36 if MODE == "lib" else 0  # lib: k-split kernel (70 KB LDS); lib32: LDS-DMA 64x64 (32 KB)

    def side_op(y):
        ops.gemm(L.GEMM_TN, tprobs, splitk=2, ws=ws, tile=SIDE_TILE)
        return y


def step():
    x = a
    main = torch.cuda.current_stream()
    ys = []
    for i in range(N):
        if MODE in ("each", "lib", "lib32", "libmm", "mmlib") and i > F:
            ev = torch.cuda.Event()
            ev.record()
        x = chain_op(x) if MODE.startswith("lib") else torch.mm(x, w)  # libmm: our chain, torch.mm side
        if (MODE == "one" and i == F) or (MODE in ("each", "lib", "lib32", "libmm", "mmlib") and i > F):
            if MODE == "one":
                ev = torch.cuda.Event()
                ev.record()
            side.wait_event(ev)
            with torch.cuda.stream(side):
                y = b
                for _ in range(S):
                    y = side_op(y) if (MODE.startswith("lib") and MODE != "libmm") or MODE == "mmlib" \
                        else torch.mm(y, w2)
                ys.append(y)
    main.wait_stream(side)
    return x, ys


s0 = torch.cuda.Stream()
s0.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s0):
    step()
torch.cuda.current_stream().wait_stream(s0)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = step()
for _ in range(10):
    g.replay()
torch.cuda.synchronize()
print("done", MODE, N, F, S)
