"""Rank program for tests/test_dp.py (launched by torch.distributed.run, gloo on CPU)."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import sca_oracle as O  # noqa: E402
from scattennet_amd import workloads as W  # noqa: E402
from scattennet_amd.dp import GradAllReduce  # noqa: E402

WL = dict(B=4, T=16, K_all=27, groups=[6, 21], d=32, H=2, L=1, residual=False, maxpos=32)


def grads(model, kp, mask, gout):
    cfg = W.model_cfg(WL["d"], WL["H"], WL["L"], maxpos=WL["maxpos"])
    groups = W.split_groups(WL["groups"])
    plist = [dict(m.named_parameters()) for m in model.streams]
    outs = O.multi_stream_sca(plist, kp, mask, groups, cfg)
    torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])


def main(out_path):
    torch.set_num_threads(1)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    model = W.build_streams(WL, "cpu", seed=3, init="random")
    kp, mask, gout = W.synthetic_batch(WL, "cpu", seed=5, ragged=True)
    sl = slice(rank * WL["B"] // world, (rank + 1) * WL["B"] // world)
    grads(model, kp[sl], mask[sl], gout[:, sl])
    GradAllReduce(model.parameters(), world)()
    if rank == 0:
        torch.save({k: (p.grad * world).clone() for k, p in model.named_parameters() if p.grad is not None},
                   out_path)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
