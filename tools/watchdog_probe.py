"""Diagnostic (one GPU, RCCL world 1): when does ProcessGroupNCCL's watchdog thread retire an
eager collective's work?  The watchdog keeps a copy of every eager work (holding its output
tensors) in its list and polls its end event until it completes, then erases it; a CUDA
graph capture that starts while such works are listed races the watchdog's event queries.
This prints the storage use count of an all-reduced tensor over time: a drop back to the
baseline after synchronize() marks the watchdog's retirement of the work (the condition
GradBuckets.quiesce waits for).

    python tools/watchdog_probe.py
"""
import os
import time

import torch
import torch.distributed as dist


def uses(t):
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{29500 + os.getpid() % 400}", rank=0,
                            world_size=1, device_id=dev)
    t = torch.ones(1 << 20, device=dev)
    for trial in range(3):
        base = uses(t)
        w = dist.all_reduce(t, async_op=True)
        after_issue = uses(t)
        w.wait()
        after_wait = uses(t)
        del w
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        seen = [(0.0, uses(t))]
        while time.perf_counter() - t0 < 1.0:
            u = uses(t)
            if u != seen[-1][1]:
                seen.append((round(1e3 * (time.perf_counter() - t0), 2), u))
            time.sleep(0.001)
        print(f"trial {trial}: base {base}, after issue {after_issue}, after wait {after_wait}, "
              f"after sync (ms, uses): {seen}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
