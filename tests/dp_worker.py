"""Rank programs for tests/test_dp.py (launched by torch.distributed.run, gloo on CPU).

mode "oracle": the per-rank gradients come from the CPU oracle (plain autograd, no gradient
  sink): the reducer's fallback path (one flattened all-reduce of .grad).
mode "sink":   the per-rank gradients are written through the ops gradient-sink protocol
  (ops.param_grad_empty / ops.params_produced) by a small stack of CPU Linear functions
  that stand in for the HIP ops: discovery step, then bucketed steps whose all-reduces are
  issued as buckets fill (overlap on), a parameter used twice (fallback), a parameter that
  never gets a gradient, and an accumulation step (.grad already set).
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import sca_oracle as O  # noqa: E402
from scattennet_amd import ops, workloads as W  # noqa: E402
from scattennet_amd.dp import GradAllReduce, GradBuckets  # noqa: E402

WL = dict(B=4, T=16, K_all=27, groups=[6, 21], d=32, H=2, L=1, residual=False, maxpos=32)


def grads(model, kp, mask, gout):
    cfg = W.model_cfg(WL["d"], WL["H"], WL["L"], maxpos=WL["maxpos"])
    groups = W.split_groups(WL["groups"])
    plist = [dict(m.named_parameters()) for m in model.streams]
    outs = O.multi_stream_sca(plist, kp, mask, groups, cfg)
    torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])


class SinkLinear(torch.autograd.Function):
    """y = x W^T + b whose parameter gradients go through the ops sink, like the HIP ops."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.b = b
        return x @ w.t() + b

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dw = ops.param_grad_empty(w)
        torch.matmul(dy.t(), x, out=dw)
        db = ops.param_grad_empty(ctx.b)
        torch.sum(dy, 0, out=db)
        ops.params_produced([w, ctx.b])
        return dy @ w, dw, db


def sink_model(seed=0):
    g = torch.Generator().manual_seed(seed)
    dims = [16, 64, 48, 32, 8]
    ps = []
    for a, b in zip(dims[:-1], dims[1:]):
        ps.append(torch.nn.Parameter(torch.randn(b, a, generator=g) / a ** 0.5))
        ps.append(torch.nn.Parameter(torch.randn(b, generator=g) * 0.1))
    unused = torch.nn.Parameter(torch.randn(5, generator=g))  # never receives a gradient
    return ps, unused


def sink_forward(ps, x):
    h = x
    for i in range(0, len(ps), 2):
        if i == 2:  # the second layer is applied twice: autograd adds its two gradient pieces
            h = SinkLinear.apply(h, ps[i], ps[i + 1]) + 0.5 * SinkLinear.apply(h, ps[i], ps[i + 1])
        else:
            h = SinkLinear.apply(h, ps[i], ps[i + 1])
        h = torch.tanh(h)
    return h


def sink_data(step):
    g = torch.Generator().manual_seed(100 + step)
    x = torch.randn(8, 16, generator=g)
    gy = torch.randn(8, 8, generator=g)
    return x, gy


def main_oracle(out_path):
    rank, world = dist.get_rank(), dist.get_world_size()
    model = W.build_streams(WL, "cpu", seed=3, init="random")
    kp, mask, gout = W.synthetic_batch(WL, "cpu", seed=5, ragged=True)
    sl = slice(rank * WL["B"] // world, (rank + 1) * WL["B"] // world)
    grads(model, kp[sl], mask[sl], gout[:, sl])
    red = GradAllReduce(model.parameters(), world)
    red()
    red.close()
    if rank == 0:
        torch.save({k: (p.grad * world).clone() for k, p in model.named_parameters() if p.grad is not None},
                   out_path)


def main_sink(out_path):
    rank, world = dist.get_rank(), dist.get_world_size()
    ps, unused = sink_model()
    red = GradBuckets(ps + [unused], world, bucket_mb=1024 * 4 / 2 ** 20, overlap=True)  # 1K-float buckets
    results = {}
    for step in range(3):
        x, gy = sink_data(step)
        sl = slice(rank * 8 // world, (rank + 1) * 8 // world)
        if step < 2:
            for p in ps:
                p.grad = None
        # step 2 accumulates onto step 1's (already averaged) gradients: the fallback path
        y = sink_forward(ps, x[sl])
        y.backward(gy[sl])
        red.sync()
        results[f"step{step}"] = [p.grad.clone() for p in ps]
        results[f"step{step}_slot"] = [red.flat is not None and i in red.slot and
                                       p.grad.data_ptr() == red.flat[red.slot[i][0]:].data_ptr()
                                       for i, p in enumerate(ps)]
    results["buckets"] = red.bucket_sizes()
    results["unused_grad_none"] = unused.grad is None
    red.close()
    if rank == 0:
        torch.save(results, out_path)


def main_sink_raise(out_path):
    """Discovery and a bucketed step, then a backward that raises at its very end (a hook on
    the input: every bucket's all-reduce is already issued, the finish callback never runs),
    then a clean bucketed step: its gradients must be exact."""
    rank, world = dist.get_rank(), dist.get_world_size()
    ps, unused = sink_model()
    red = GradBuckets(ps + [unused], world, bucket_mb=1024 * 4 / 2 ** 20, overlap=True)
    sl = slice(rank * 8 // world, (rank + 1) * 8 // world)
    for step in range(2):
        x, gy = sink_data(step)
        for p in ps:
            p.grad = None
        sink_forward(ps, x[sl]).backward(gy[sl])
        red.sync()

    def boom(_):
        raise RuntimeError("boom")

    x, gy = sink_data(5)
    xs = x[sl].clone().requires_grad_(True)
    xs.register_hook(boom)
    for p in ps:
        p.grad = None
    raised = False
    try:
        sink_forward(ps, xs).backward(gy[sl])
    except RuntimeError:
        raised = True
    x, gy = sink_data(2)
    for p in ps:
        p.grad = None
    sink_forward(ps, x[sl]).backward(gy[sl])
    red.sync()
    results = {"raised": raised, "after": [p.grad.clone() for p in ps]}
    red.close()
    if rank == 0:
        torch.save(results, out_path)


if __name__ == "__main__":
    torch.set_num_threads(1)
    dist.init_process_group("gloo")
    {"sink": main_sink, "sink_raise": main_sink_raise}.get(sys.argv[2], main_oracle)(sys.argv[1])
    dist.barrier()
    dist.destroy_process_group()
