"""Diagnose hipGraph capture of RCCL collectives (world size 1) on the one-GPU box.

  python tools/dp_capture_diag.py <variant>

variants (each in its own process; the driver script stops at the first failure):
  plain      all_reduce of a tensor captured on the capture stream itself
  forked     all_reduce issued on a second stream forked from / joined into the capture stream
             (no kernel of its own before the collective)
  kernel     a kernel on the forked stream before and after the all_reduce
  nojoinnode a kernel before the all_reduce, none after (the side stream joins through the
             collective's completion event)
  mainwait   a kernel before the all_reduce; the capture stream itself waits for the collective
  origin     a kernel on a forked stream joined back first; the collective is issued from and
             waited on the capture stream
  reducer    scattennet_amd.dp.GradBuckets over a small 4-stream SCA step (global capture mode)
  reducer_tl the same with capture_error_mode="thread_local"
  watchdog_race   (round 5) the round-4 abort, made deterministic: an eager async all_reduce
             (on ProcessGroupNCCL's internal stream), then at once a thread_local capture that
             issues an async all_reduce (the same internal stream joins the capture) and sleeps
             0.5 s inside the capture, so the watchdog's next poll of the eager work's end event
             falls while that event's stream is capturing.  Expected: hipErrorCapturedEvent
             from the watchdog thread -> terminate -> SIGABRT.  Run it LAST in a call.
  watchdog_fixed  the same timing with dp.GradBuckets' stream discipline: eager collectives in
             the synchronous form on an eager communication stream, the captured one in the
             synchronous form on a capture-only stream forked from / joined into the origin.
             Expected: capture, instantiate and replay pass (this also shows that the
             synchronous form runs on the current stream: on the internal stream it would race
             exactly like watchdog_race).
"""
import time
import os
import sys

import torch
import torch.distributed as dist


def reducer(variant):
    """The bench's pattern: the bucketed reducer's all-reduces issued from the backward
    (autograd's device thread) during capture of a small 4-stream SCA step."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["SCA_DP_FORCE"] = "1"
    from scattennet_amd import workloads as W
    from scattennet_amd.dp import GradBuckets
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29434", rank=0, world_size=1, device_id=dev)
    w = dict(W.WORKLOADS["cfg2"], B=4, T=128)
    model = W.build_streams(w, dev, seed=2, init="random")
    kp, mask, gout = W.synthetic_batch(w, dev, seed=3, ragged=True)
    red = GradBuckets(model.parameters(), bucket_mb=6)
    params = list(model.parameters())

    def step():
        outs = model(kp, mask)
        torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])

    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
            for p in params:
                p.grad = None
            step()
            print("eager step", i, "buckets", red.bucket_sizes(), flush=True)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for p in params:
        p.grad = None
    g = torch.cuda.CUDAGraph()
    mode = "thread_local" if variant == "reducer_tl" else "global"
    with torch.cuda.graph(g, capture_error_mode=mode):
        step()
        print("  .. backward captured", flush=True)
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("replayed", variant, float(params[0].grad.abs().sum()), flush=True)
    red.close()
    dist.destroy_process_group()


def watchdog(variant):
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29435", rank=0, world_size=1, device_id=dev)
    x = torch.ones(1 << 20, device=dev)
    eager_s, cap_s = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    for i in range(3):  # eager works for the watchdog to track; the last one issued just before capture
        if variant == "watchdog_race":
            dist.all_reduce(x, async_op=True).wait()
        else:
            eager_s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(eager_s):
                dist.all_reduce(x)
            torch.cuda.current_stream().wait_stream(eager_s)
    torch.cuda.synchronize()
    print("eager collectives done", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        main_s = torch.cuda.current_stream()
        x.mul_(2.0)
        if variant == "watchdog_race":
            dist.all_reduce(x, async_op=True).wait()
        else:
            cap_s.wait_stream(main_s)
            with torch.cuda.stream(cap_s):
                dist.all_reduce(x)
            main_s.wait_stream(cap_s)
        print("  .. collective captured; sleeping inside the capture", flush=True)
        time.sleep(0.5)  # >= 4 watchdog polls while the collective's stream is capturing
        x.mul_(0.5)
    print("captured", flush=True)
    x.fill_(3.0)
    g.replay()
    torch.cuda.synchronize()
    print("replayed", variant, float(x[0]), "(expect 3.0)", flush=True)
    time.sleep(0.5)  # let the watchdog poll again after the replay
    dist.destroy_process_group()
    print("ok", variant, flush=True)


def main(variant):
    if variant.startswith("reducer"):
        return reducer(variant)
    if variant.startswith("watchdog"):
        return watchdog(variant)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29433", rank=0, world_size=1, device_id=dev)
    x = torch.ones(1 << 20, device=dev)
    y = torch.zeros(1 << 20, device=dev)
    dist.all_reduce(x)  # warm the communicator outside capture
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph()

    def mark(m):
        print("  ..", m, flush=True)

    with torch.cuda.graph(g):
        main_s = torch.cuda.current_stream()
        x.mul_(2.0)
        if variant == "plain":
            dist.all_reduce(x)
        elif variant == "origin":
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                y.copy_(x)
            main_s.wait_stream(side)
            mark("side kernel joined")
            w = dist.all_reduce(y, async_op=True)
            mark("all_reduce issued from the origin stream")
            w.wait()
            mark("origin waited")
        else:
            side.wait_stream(main_s)
            mark("forked")
            with torch.cuda.stream(side):
                if variant != "forked":
                    y.copy_(x)
                    mark("side kernel")
                w = dist.all_reduce(y if variant != "forked" else x, async_op=True)
                mark("all_reduce issued")
                if variant != "mainwait":
                    w.wait()
                    mark("side waited")
                if variant in ("forked", "kernel"):
                    x.add_(1.0)
                    mark("side kernel after")
            if variant == "mainwait":
                w.wait()
                mark("main waited")
            main_s.wait_stream(side)
            mark("joined")
        x.mul_(0.5)
        mark("capture body done")
    print("captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("replayed", variant, float(x[0]), float(y[0]), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
