"""Host cost of launching the captured step: time N graph.replay() calls without a sync
(host submission) against the time until the GPU is done (config 2 unless --workload).

    python tools/replay_probe.py [--workload cfg2] [--n 20] ["ops._EARLY_FORK=False" ...]
"""
import os
import sys
import time

os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "2")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import keypoint_module, ops, workloads as W  # noqa: E402

args = [a for a in sys.argv[1:] if "=" in a and not a.startswith("--")]
for stmt in args:
    exec(stmt, {"ops": ops, "keypoint_module": keypoint_module})
wl = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "cfg2"
n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 20
dev = torch.device("cuda", 0)
w = W.WORKLOADS[wl]
model = W.build_encoder(w, dev, seed=0) if w.get("fusion") else W.build_streams(w, dev, seed=0, init="reference")
kp, mask, gout = W.synthetic_batch(w, dev, seed=1)
go = [gout[g].contiguous() for g in range(gout.shape[0])]
params = list(model.parameters())


def fwd_bwd():
    outs = model(kp, mask)
    outs = outs[:1] if w.get("fusion") else outs
    torch.autograd.backward(outs, go)


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        for p in params:
            p.grad = None
        fwd_bwd()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
for p in params:
    p.grad = None
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    fwd_bwd()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
if "--sync" in sys.argv:  # one replay at a time: GPU time per step with the whole replay submitted up front
    for rnd in range(3):
        ts = []
        for _ in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        print(f"{wl} {' '.join(args)}: synced replays, GPU {ts[n // 2]:.3f} ms/step (min {ts[0]:.3f})", flush=True)
    sys.exit(0)
for rnd in range(3):
    t0 = time.perf_counter()
    per = []
    for _ in range(n):
        a = time.perf_counter()
        g.replay()
        per.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    per.sort()
    print(f"{wl} {' '.join(args)}: host submit {1e3 * (t1 - t0) / n:.3f} ms/replay (median {1e3 * per[n // 2]:.3f}, "
          f"first {1e3 * per[0]:.3f}), GPU done {1e3 * (t2 - t0) / n:.3f} ms/step", flush=True)
