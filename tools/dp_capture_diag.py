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
"""
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


def main(variant):
    if variant.startswith("reducer"):
        return reducer(variant)
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
