"""Batch-sharded data parallelism over RCCL.

The reference initialises an NCCL process group but never wraps the model in DDP nor
all-reduces a gradient (utils.py:237-265, main.py:132-133), so this is the
north-star's new functionality: one process per GPU, each running its own clips through the
HIP path, and ONE coalesced fp32 all-reduce of all gradients per step over RCCL/xGMI
(torch.distributed backend "nccl" is RCCL on ROCm).  The 4-stream SCA has 25.8 M
parameters: one 103 MB bucket, which RCCL splits over its channels / all 7 xGMI links.

Oracle: the averaged all-reduced gradient times the world size equals the single-process
gradient of the whole global batch (sum loss) — tests/test_dp.py checks it with `gloo`.
Parameters that never receive a gradient (the ResidualNetwork long shortcuts) are reduced
as zeros and left without a .grad, as in the reference.
"""
import torch
import torch.distributed as dist


class GradAllReduce:
    """Average the gradients of `params` over all ranks with one coalesced all-reduce.

    Flatten (one cat launch), all-reduce, scatter back (one multi-tensor copy launch); the
    set of parameters holding a gradient is structural (identical on every rank)."""

    def __init__(self, params, world=None, average=True):
        self.params = [p for p in params if p.requires_grad]
        self.world = world if world is not None else (dist.get_world_size() if dist.is_initialized() else 1)
        self.average = average
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, device=self.params[0].device, dtype=torch.float32)

    def __call__(self):
        if self.world == 1:
            return
        grads = [p.grad for p in self.params if p.grad is not None]
        if not grads:
            return
        n = sum(g.numel() for g in grads)
        flat = self.flat[:n]
        torch.cat([g.reshape(-1) for g in grads], out=flat)
        dist.all_reduce(flat)
        if self.average:
            flat.mul_(1.0 / self.world)
        views, o = [], 0
        for g in grads:
            views.append(flat[o:o + g.numel()].view_as(g))
            o += g.numel()
        torch._foreach_copy_(grads, views)
