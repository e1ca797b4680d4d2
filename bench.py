"""Benchmark: clips/s forward+backward of the SCA hot path on MI355X (BASELINE.json metric).

Workload (BASELINE config 2, the metric's configuration): four keypoint streams
(body/left/right/face = 6/21/21/31 of K=79 joints) sliced out of one (B=8, T=256, 79, 2)
synthetic keypoint batch, each through coordinate mapping + the 4-layer SCA stack
(d=256, 16 heads, ff 768), forward + backward of every parameter.  One "step" = one such
fwd+bwd over the batch; with N > 1 GPUs each rank runs its own 8 clips (weak scaling) and
the step includes the RCCL gradient all-reduce.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg2] [--no-graph]

--gpus N > 1 without a launcher (WORLD_SIZE unset): this process starts N rank processes of
the same command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their
environment, one GPU each) and exits with their status; it never touches the GPU itself.
Under torch.distributed.run (WORLD_SIZE set) --gpus must agree with WORLD_SIZE.
SCA_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices round-robin).

Prints ONE JSON line on rank 0 (contract in the build instructions), including:
  roofline      the dominant kernel's algorithmic FLOP rate (HIP events around each of its
                launches in an instrumented eager step after the timed region) vs fp32 MFMA peak
  cpu_baseline  the CPU oracle (plain PyTorch fp32 restatement) timed on this host's cores
                on a bounded sample of the same workload (rank 0, N = 1 only)
"""
import argparse
import json
import os
import sys
import time

# HIP graph executor: spread the captured step over 2 hardware queues instead of the
# runtime's default (4): fewer cross-queue hand-offs on the critical path while the
# weight-gradient side streams still overlap — +1.3 % at config 2 (tools/graph_env_sweep.sh,
# 3 alternations: 1598 vs 1577 clips/s; 1 queue -1.6 %, 3 queues +0.2 %).  Read by the HIP
# runtime at initialisation, so set before the first GPU call; an explicit setting wins.
# With the data-parallel path (N > 1, or SCA_DP_FORCE) one more queue: the bucket all-reduces'
# RCCL nodes are the second children of weight-gradient nodes (dp.GradBuckets defers their
# fork), which the executor would put on the critical chain's queue with only two
# (SCA_DP_GRAPH_QUEUES overrides).
_dp_env = int(os.environ.get("WORLD_SIZE", "1")) > 1 or os.environ.get("SCA_DP_FORCE", "0") != "0"
_GQ_USER = "DEBUG_HIP_FORCE_GRAPH_QUEUES" in os.environ
os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", os.environ.get("SCA_DP_GRAPH_QUEUES", "3") if _dp_env else "2")

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from scattennet_amd import ops, workloads as W  # noqa: E402
from scattennet_amd.dp import GradBuckets, gathered_mean  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA == fp32 vector peak
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default: WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfg2", choices=sorted(W.WORKLOADS))
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one captured hipGraph")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU-oracle baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dropout", type=float, default=0.0,
                    help="train-mode dropout p for every block (the yaml's 0.2 = the secondary run)")
    return ap.parse_args()


def spawn_ranks(n):
    """Start n rank processes of this bench command and wait for them (the parent imports torch
    but makes no GPU call: torch.cuda.device_count() does not initialise the device).  Returns
    the first non-zero exit status, else 0."""
    import signal
    import socket
    import subprocess
    backend = os.environ.get("SCA_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and ndev < n:
        raise SystemExit(f"bench.py --gpus {n}: only {ndev} GPU(s) visible; RCCL needs one GPU per rank "
                         "(SCA_DIST_BACKEND=gloo rehearses several ranks per GPU)")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    base = dict(os.environ)
    if not _GQ_USER:
        base.pop("DEBUG_HIP_FORCE_GRAPH_QUEUES", None)  # each rank picks its own (the DP count)
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    status = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            rc = p.poll()
            if rc is None:
                continue
            pending.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                for q in pending:  # one rank failed: the others would wait in a collective
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return status


def main(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if os.environ.get("SCA_DIST_BACKEND", "nccl") != "nccl":  # rehearsal: ranks may share a GPU
        local %= max(1, ndev)
    # SCA_DP_FORCE=1 (under torch.distributed.run): the data-parallel path at world size 1 —
    # rehearses the captured bucketed RCCL all-reduces on a one-GPU box
    use_dp = world > 1 or ("MASTER_ADDR" in os.environ and os.environ.get("SCA_DP_FORCE", "0") != "0")
    if use_dp:
        torch.cuda.set_device(local)
        backend = os.environ.get("SCA_DIST_BACKEND", "nccl")  # nccl == RCCL; gloo: rehearse N>1 on one GPU
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    w = W.WORKLOADS[args.workload]

    fusion = bool(w.get("fusion"))
    model = W.build_encoder(w, dev, seed=0) if fusion else W.build_streams(w, dev, seed=0, init="reference")
    if args.dropout > 0:  # secondary run: the yaml's dropout (keypoint_module / layers / fusion)
        from scattennet_amd import (CoordinateAttention, CoordinatesFusion, CoordinatesMerge, FeedForward,
                                    SeparativeCoordinateAttention)
        for m in model.modules():
            if isinstance(m, (CoordinateAttention, CoordinatesMerge, FeedForward, SeparativeCoordinateAttention)):
                m.dropout = args.dropout
            elif isinstance(m, CoordinatesFusion):
                m.drop_rate = args.dropout
    if world > 1:  # identical initial weights on every rank
        for p in model.parameters():
            dist.broadcast(p.data, 0)
    kp, mask, gout = W.synthetic_batch(w, dev, seed=1 + rank)
    grads_out = [gout[g].contiguous() for g in range(gout.shape[0])]
    params = [p for p in model.parameters()]
    # data parallel: gradients land in ~25 MB flat buckets whose RCCL all-reduces are issued
    # from the backward as each bucket fills (captured into the step's hipGraph); gloo
    # rehearsals all-reduce the buckets after the step instead (reducer.sync)
    reducer = GradBuckets(params, world) if use_dp else None

    def fwd_bwd():
        if args.dropout > 0:
            ops.advance_dropout()  # device-side step counter: fresh masks on every graph replay
        outs = model(kp, mask)
        outs = outs[:1] if fusion else outs  # config 3: the loss seed sits on the fusion output
        torch.autograd.backward(outs, grads_out)

    def sync():
        if reducer is not None:
            reducer.sync()

    def step():
        fwd_bwd()
        sync()

    # warm-up (also builds the library's lazy state) on a side stream, as graph capture requires
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(max(1, args.warmup)):
            for p in params:
                p.grad = None
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    # the captured graph holds forward + backward (~200 HIP launches) and, with RCCL, the
    # bucketed gradient all-reduces overlapped with the backward
    graph = None
    if not args.no_graph:
        for p in params:
            p.grad = None
        if reducer is not None:
            reducer.quiesce()  # no eager RCCL work left for the watchdog to poll during capture
        graph = torch.cuda.CUDAGraph()
        # thread-local capture mode with RCCL: ProcessGroupNCCL's watchdog thread queries the
        # warm-up steps' events while the step is captured (tools/dp_capture_diag.py)
        with torch.cuda.graph(graph, capture_error_mode="thread_local" if reducer is not None else "global"):
            ops.fork_ledger_begin()  # every stream forked in the step must join the capture origin
            fwd_bwd()
            ops.fork_ledger_end()
        for _ in range(2):
            graph.replay()
            sync()
        torch.cuda.synchronize()

    marks = []

    def run(k):
        for _ in range(k):
            if graph is not None:
                graph.replay()
                sync()
            else:
                for p in params:
                    p.grad = None
                step()
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            marks.append(ev)

    if use_dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    start = torch.cuda.Event(enable_timing=True)
    start.record()
    run(args.steps)
    torch.cuda.synchronize()
    if use_dp:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if use_dp:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = 1000.0 * elapsed / args.steps
    per_step = sorted(a.elapsed_time(b) for a, b in zip([start] + marks[:-1], marks))
    ms_median = per_step[len(per_step) // 2]
    clips = w["B"] * world * args.steps / elapsed
    step_flops = W.flops_per_step(w)

    # ---- data parallel: the averaged buckets checked once against an eager gather-and-mean ----
    dp_check = None
    if reducer is not None and reducer.collective and args.dropout == 0:
        dp_check = check_allreduce(reducer, graph, fwd_bwd, sync, params)

    # ---- dominant-kernel roofline: one instrumented eager step (HIP events per launch) ----
    prof = ops.LaunchProfiler()
    with prof:
        for p in params:
            p.grad = None
        step()
    torch.cuda.synchronize()
    # the dominant kernel: the top row by time per step of the committed rocprofv3 profile of
    # this workload when that profile was measured on the current sources (so `kernel`,
    # `frac` and `traffic` all come from one profile), else the eager HIP-event ranking
    stats = prof.stats()
    ranked = committed_ranking(args, stats)
    kname = ranked[0] if ranked else prof.dominant()[0]
    kstat = stats[kname]
    achieved = kstat["flops"] / kstat["seconds"] / 1e12 if kstat["seconds"] > 0 else 0.0
    roofline = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 3), "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                "frac_source": "HIP events around each launch of the kernel in an instrumented eager step",
                "kernel_source": ("top kernel by time per step of the committed rocprofv3 profile" if ranked else
                                  "top kernel by HIP-event time in the instrumented eager step"),
                "launches": kstat["launches"], "avg_launch_us": round(1e6 * kstat["seconds"] / kstat["launches"], 2),
                "flops_per_launch": kstat["flops"] / kstat["launches"],
                "step_achieved": round(step_flops / (ms / 1e3) / 1e12, 3),
                "step_frac": round(step_flops / (ms / 1e3) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)}
    roofline.update(committed_profile(args, kname, roofline["flops_per_launch"]))

    rp = roofline.pop("_rocprof", None)
    if rp is not None:  # the profiler's figure leads; the in-bench HIP-event one beside it
        roofline["event_achieved"], roofline["event_frac"] = roofline["achieved"], roofline["frac"]
        roofline["achieved"], roofline["frac"] = rp
        roofline["frac_source"] = roofline["rocprof_source"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not fusion and args.dropout == 0:
        cpu = cpu_baseline(w, model, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "clips/sec fwd+bwd, (B=8,T=256,K=79,d=256) at 1/2/4/8 MI355X",
            "value": round(clips, 2), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic (U[0,1) keypoints, MSCA_Net init)",
            "config": {"workload": f"{args.workload}: " + describe(w), "clips_per_gpu": w["B"], "frames": w["T"],
                       "joints": w["K_all"], "streams": w["groups"], "d_model": w["d"], "heads": w["H"],
                       "layers": w["L"], "dropout": args.dropout, "hipgraph": graph is not None,
                       "parallelism": f"dp{world}", "devices": min(world, max(1, ndev))},
            "ms_per_step_median": round(ms_median, 4),
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if reducer is not None:
            line["config"]["grad_allreduce"] = {
                "backend": dist.get_backend(), "buckets_mb": [round(b / 2 ** 20, 2) for b in reducer.bucket_sizes()],
                "overlapped": reducer.overlap, "in_graph": reducer.overlap and graph is not None,
                "fallback_params": len(reducer.last_fallback)}
            if dp_check is not None:
                line["config"]["grad_allreduce"].update(dp_check)
        print(json.dumps(line), flush=True)
    if use_dp:
        reducer.close()
        dist.destroy_process_group()


def check_allreduce(reducer, graph, fwd_bwd, sync, params):
    """Once, after the timed region: the averaged gradient buckets of one step (a graph replay,
    or an eager step) against an eager all_gather of every rank's LOCAL gradients of the same
    step, summed in rank order and divided by the world size (dp.gathered_mean).  The local
    gradients come from the same step run with the reducer's collectives off (the kernels are
    deterministic, so they are the gradients the replay fed its all-reduces)."""
    if graph is not None:
        graph.replay()
    else:
        for p in params:
            p.grad = None
        fwd_bwd()
    sync()
    torch.cuda.synchronize()
    averaged = reducer.flat.clone()
    reducer.collective = False
    try:
        for p in params:
            p.grad = None
        fwd_bwd()
        torch.cuda.synchronize()
        local = reducer.flat.clone()
    finally:
        reducer.collective = True
    ref = gathered_mean(local)
    diff = float((averaged - ref).abs().max())
    scale = float(ref.abs().max())
    spread = float((local - ref).abs().max())  # how far this rank's own gradients are from the mean
    return {"check_max_abs": diff, "check_rel": diff / scale if scale > 0 else 0.0,
            "check_local_vs_mean_max_abs": spread,
            "check": "captured AVG buckets vs eager all_gather + mean of the ranks' local gradients, one step "
                     "after the timed region"}


def _kstats_name(raw):
    return raw.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def committed_ranking(args, stats):
    """Kernels of the committed profile of this workload (fresh digest only) that the eager
    profiler also timed with algorithmic FLOPs, by total time (= time per step: every kernel
    of the step runs once per profiled step), largest first."""
    import csv
    from scattennet_amd import _lib
    d = os.path.join(ROOT, "profiles", "latest")
    mpath = os.path.join(d, f"{args.workload}_meta.json")
    if args.dropout != 0 or not os.path.exists(mpath):
        return []
    if json.load(open(mpath)).get("source_digest") != _lib.source_digest():
        return []
    rows = [(float(r["TotalDurationNs"]), _kstats_name(r["Name"]))
            for r in csv.DictReader(open(os.path.join(d, f"{args.workload}_kstats.csv")))]
    return [n for _, n in sorted(rows, reverse=True) if n in stats and stats[n]["flops"] > 0]


def committed_profile(args, kname, flops_per_launch):
    """The dominant kernel's figures from the committed rocprofv3 profile of THIS workload
    (profiles/latest/<workload>_*: tools/promote_profile.py), used only when it was measured
    on the current library sources (source digest) — then `frac` / `achieved` are the
    profiler's (average kernel-trace duration, graph replays of the same bench command) and
    the HIP-event figures stay beside them as event_*; `traffic` = PMC HBM bytes per launch
    (FETCH_SIZE doubled + WRITE_SIZE, separate passes)."""
    import csv
    from scattennet_amd import _lib
    d = os.path.join(ROOT, "profiles", "latest")
    wl = args.workload
    mpath = os.path.join(d, f"{wl}_meta.json")
    if args.dropout != 0 or not os.path.exists(mpath):
        return {}
    meta = json.load(open(mpath))
    if meta.get("source_digest") != _lib.source_digest():
        return {"profile": f"profiles/latest/{wl}_* is stale (sources {meta.get('source_digest')}, "
                           f"build {_lib.source_digest()}): not reported"}
    out = {"profile_digest": meta["source_digest"]}
    kpath = os.path.join(d, f"{wl}_kstats.csv")
    for r in csv.DictReader(open(kpath)):
        if _kstats_name(r["Name"]) == kname:
            avg_s = float(r["AverageNs"]) * 1e-9
            tf = flops_per_launch / avg_s / 1e12
            out.update({"event_achieved": None, "event_frac": None})
            out["rocprof_avg_launch_us"] = round(avg_s * 1e6, 2)
            out["rocprof_source"] = f"profiles/latest/{wl}_kstats.csv (rocprofv3 --kernel-trace --stats)"
            out["_rocprof"] = (round(tf, 3), round(tf / FP32_MFMA_PEAK_TFLOPS, 4))
    upath = os.path.join(d, f"{wl}_util.json")
    if os.path.exists(upath):  # the kernel's MFMA busy share (SQ counters, the kernel alone)
        for r in json.load(open(upath)):
            if r["kernel"] == kname and r.get("mfma_busy") is not None:
                out["mfma_busy"] = round(r["mfma_busy"], 4)
                out["mfma_busy_source"] = (f"profiles/latest/{wl}_util.json (rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES / "
                                           "(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), counter pass: the kernel alone)")
    tpath = os.path.join(d, f"{wl}_traffic.json")
    if os.path.exists(tpath):
        tr = json.load(open(tpath)).get(kname)
        if tr:
            out["traffic"] = round(tr["bytes_per_launch"])
            out["traffic_source"] = f"profiles/latest/{wl}_traffic.json (rocprofv3 PMC, bytes per launch)"
    return out


def describe(w):
    if w.get("fusion"):
        return (f"full encoder: {len(w['groups'])} streams (mapping + {w['L']}x SCA + residual "
                f"{w['residual_blocks']}) + CoordinatesFusion {w['in_fusion']}->{w['out_fusion']}, "
                f"B={w['B']} T={w['T']} K={w['K_all']} d={w['d']} H={w['H']}, fwd+bwd all params")
    return (f"{len(w['groups'])}-stream SCA (mapping + {w['L']}x self / causal / cross-merge), "
            f"B={w['B']} T={w['T']} K={w['K_all']} d={w['d']} H={w['H']}, fwd+bwd all params")


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _time_oracle(w, plist, groups, cfg, B, iters, warm=1):
    """Median seconds of `iters` oracle fwd+bwd steps over the first B clips (after `warm`)."""
    from oracle import sca_oracle as O
    kp, mask, gout = W.synthetic_batch(dict(w, B=B), "cpu", seed=1)
    times = []
    for i in range(warm + iters):
        t0 = time.perf_counter()
        outs = O.multi_stream_sca(plist, kp, mask, groups, cfg)
        torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])
        dt = time.perf_counter() - t0
        for p in plist:
            for v in p.values():
                v.grad = None
        if i >= warm:
            times.append(dt)
    times.sort()
    return times[len(times) // 2]


def _time_cfg1(iters, warm=2):
    """Median seconds of the config-1 x-stream fwd+bwd (oracle.x_stream) on this host."""
    from oracle import sca_oracle as O
    w1 = W.WORKLOADS["cfg1"]
    mod = W.build_streams(w1, "cpu", seed=0, init="reference").streams[0]
    p = {k: v.detach().clone().requires_grad_(True) for k, v in mod.state_dict().items()}
    cfg = W.model_cfg(w1["d"], w1["H"], w1["L"], maxpos=w1["maxpos"])
    kp, mask, _ = W.synthetic_batch(w1, "cpu", seed=1)
    g = torch.randn(w1["B"], w1["T"], w1["d"], generator=torch.Generator().manual_seed(1))
    times = []
    for i in range(warm + iters):
        t0 = time.perf_counter()
        (O.x_stream(p, "", kp, mask, cfg) * g).sum().backward()
        times.append(time.perf_counter() - t0)
        for v in p.values():
            v.grad = None
    times = sorted(times[warm:])
    return times[len(times) // 2]


def cpu_baseline(w, model, budget_s):
    """The CPU oracle (oracle/sca_oracle.py, pinned to the reference's golden vectors) timed
    on this host (BASELINE.md CPU-baseline plan): same workload and weights, 1 warm-up then
    the median of >= 3 fwd+bwd steps on all the box's threads; a 1-thread run on a 1-clip
    sample; config 1 (x-stream, B=2 T=64 K=27 d=64) at both thread counts.  About 15-20 s
    of CPU time in all (`budget_s` is kept for the command line; the sample sizes are fixed)."""
    threads = os.cpu_count() or 1
    # the GPU box reports the whole machine; use the box's CPU share (OMP_NUM_THREADS = 16)
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", "16")))
    cfg = W.model_cfg(w["d"], w["H"], w["L"], maxpos=w["maxpos"])
    groups = W.split_groups(w["groups"])
    plist = [{k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
             for m in model.streams]
    torch.set_num_threads(threads)
    t_full = _time_oracle(w, plist, groups, cfg, w["B"], iters=3)
    torch.set_num_threads(1)
    t_one = _time_oracle(w, plist, groups, cfg, 1, iters=3)
    c1_one = _time_cfg1(iters=9)
    torch.set_num_threads(threads)
    c1_full = _time_cfg1(iters=9)
    w1 = W.WORKLOADS["cfg1"]
    return {"value": round(w["B"] / t_full, 3), "unit": "clips/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(),
            "sample": f"median of 3 fwd+bwd steps of the full workload (B={w['B']}) on the CPU oracle after 1 warm-up, "
                      f"{threads} threads ({t_full:.2f} s/step)",
            "one_thread": {"value": round(1 / t_one, 3), "unit": "clips/s", "cores": 1,
                           "sample": f"median of 3 fwd+bwd steps of 1 clip of the same workload ({t_one:.2f} s/step)"},
            "cfg1": {"value": round(w1["B"] / c1_full, 2), "one_thread": round(w1["B"] / c1_one, 2), "unit": "clips/s",
                     "sample": "BASELINE config 1: x-stream (mapping + 4 self layers), B=2 T=64 K=27 d=64 H=4, median "
                               f"of 9 fwd+bwd steps ({1e3 * c1_full:.1f} ms at {threads} threads, "
                               f"{1e3 * c1_one:.1f} ms at 1)"}}


if __name__ == "__main__":
    _args = parse()
    _ws = os.environ.get("WORLD_SIZE")
    if _ws is None and (_args.gpus or 1) > 1:
        sys.exit(spawn_ranks(_args.gpus))
    if _ws is not None and _args.gpus is not None and _args.gpus != int(_ws):
        raise SystemExit(f"bench.py: --gpus {_args.gpus} disagrees with WORLD_SIZE={_ws}")
    main(_args)
