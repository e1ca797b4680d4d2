"""Data parallelism on the HIP path (BASELINE config 4), in one process.

* Batch additivity: the config-2 model (4 streams, d 256, L 4) on two 8-clip halves through
  the HIP kernels — the sum of the halves' gradients equals the full 16-clip HIP gradient
  and the CPU oracle's, within the north-star 1e-3.  This is exactly what the all-reduce of
  an 8-GPU x 8-clip run relies on (config 4: B = 64 = 8 x 8).
* The bucketed reducer (scattennet_amd.dp.GradBuckets) at world size 1 over RCCL, with the
  collectives forced on (SCA_DP_FORCE): discovery step, eager bucketed step, then the step
  captured into a hipGraph WITH the bucket all-reduces and replayed — gradients identical to
  the plain (no-DP) HIP gradients, `.grad` views of the flat buckets.
"""
import os

import pytest
import torch

from oracle import sca_oracle as O
from tests.golden_util import close, rel_err

PARITY_TOL = 1e-3


def _cfg2(B):
    from scattennet_amd import workloads as W
    return dict(W.WORKLOADS["cfg2"], B=B)


def _grads(model, kp, mask, gout):
    for p in model.parameters():
        p.grad = None
    outs = model(kp, mask)
    torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])
    torch.cuda.synchronize()
    return {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}


@pytest.mark.gpu
def test_half_batch_gradients_sum_to_full_batch():
    from scattennet_amd import workloads as W
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda:0")
    w16 = _cfg2(16)
    model = W.build_streams(w16, dev, seed=4, init="random")
    kp, mask, gout = W.synthetic_batch(w16, dev, seed=9, ragged=False)
    g = torch.Generator().manual_seed(21)
    lens = torch.randint(1, w16["T"] + 1, (16,), generator=g)
    lens[3], lens[11] = w16["T"], 1
    mask = (torch.arange(w16["T"])[None] < lens[:, None]).long().to(dev)
    full = _grads(model, kp, mask, gout)
    h0 = _grads(model, kp[:8], mask[:8], gout[:, :8].contiguous())
    h1 = _grads(model, kp[8:], mask[8:], gout[:, 8:].contiguous())
    assert set(full) == set(h0) == set(h1)
    gscale = max(float(v.abs().max()) for v in full.values())
    for k in full:
        s = h0[k] + h1[k]
        assert close(s.cpu(), full[k].cpu(), PARITY_TOL, gscale), (k, rel_err(s, full[k]))

    # ... and the oracle's full-batch gradient (every stream, every parameter)
    cfg = W.model_cfg(w16["d"], w16["H"], w16["L"], maxpos=w16["maxpos"])
    groups = W.split_groups(w16["groups"])
    plist = [{k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
             for m in model.streams]
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    outs = O.multi_stream_sca(plist, kp.cpu(), mask.cpu(), groups, cfg)
    torch.autograd.backward(outs, [gout[i].cpu() for i in range(len(outs))])
    ref = {f"streams.{s}.{k}": v.grad for s, p in enumerate(plist) for k, v in p.items() if v.grad is not None}
    rscale = max(float(v.abs().max()) for v in ref.values())
    for k, v in ref.items():
        s = (h0[k] + h1[k]).cpu()
        assert close(s, v, PARITY_TOL, rscale), (k, rel_err(s, v))


@pytest.mark.gpu
def test_bucketed_reducer_captured_rccl_world1(monkeypatch):
    """At world size 1 the all-reduce is an identity and the 1/world pre-scale is x1, so a
    missing or late wait of the communication stream on a producing stream would go unseen:
    the collective is wrapped so that it DOUBLES its bucket on the communication stream
    before reducing it — every gradient must then come out exactly 2x the plain HIP one, in
    the eager step and in the graph replay (a bucket reduced before its last gradient
    landed would not be doubled).

    The capture also sleeps 0.35 s before it ends: ProcessGroupNCCL's watchdog (100-ms polls)
    then certainly queries the eager steps' collectives while the captured collectives'
    stream is capturing — the round-4 SIGABRT (hipErrorCapturedEvent in the watchdog) unless
    the eager and the captured collectives live on disjoint streams (dp.GradBuckets)."""
    import time
    import warnings

    import torch.distributed as dist

    from scattennet_amd import ops, workloads as W
    from scattennet_amd.dp import GradBuckets
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda:0")
    w = dict(W.WORKLOADS["cfg2"], B=4, T=128)
    model = W.build_streams(w, dev, seed=2, init="random")
    kp, mask, gout = W.synthetic_batch(w, dev, seed=3, ragged=True)
    ref = _grads(model, kp, mask, gout)  # plain HIP gradients, no sink

    monkeypatch.setenv("SCA_DP_FORCE", "1")
    init_here = not dist.is_initialized()
    if init_here:
        port = 29400 + os.getpid() % 500
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=dev)
    real_all_reduce = dist.all_reduce

    def doubling_all_reduce(t, *a, **k):  # on the stream the reducer issues from
        t.mul_(2.0)
        return real_all_reduce(t, *a, **k)

    monkeypatch.setattr(dist, "all_reduce", doubling_all_reduce)
    red = GradBuckets(model.parameters(), bucket_mb=6)
    try:
        assert red.collective and red.overlap
        params = list(model.parameters())
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # discovery step, then a bucketed eager step
                for p in params:
                    p.grad = None
                outs = model(kp, mask)
                torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        assert len(red.plan) >= 2
        eager = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
        for p in params:
            p.grad = None
        # drop the eager step's autograd graph: its AccumulateGrad nodes (bound to stream s)
        # would otherwise be reused by the captured backward — an unrecorded fork into s
        del outs
        red.quiesce()
        graph = torch.cuda.CUDAGraph()
        with warnings.catch_warnings():
            warnings.filterwarnings("error", message=".*AccumulateGrad.*")
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):  # RCCL watchdog thread
                led = ops.fork_ledger_begin()
                outs = model(kp, mask)
                torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])
                ops.fork_ledger_end()  # every fork (side streams, branch, RCCL) joined into the origin
                time.sleep(0.35)  # >= 3 watchdog polls inside the capture
        assert led.last_fork and any("RCCL" in n for n in led.names.values())
        for p in params:  # poison the buckets: the replay must rewrite every planned gradient
            if p.grad is not None:
                p.grad.fill_(float("nan"))
        graph.replay()
        graph.replay()
        torch.cuda.synchronize()
        replay = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
        flat0 = red.flat.data_ptr()
        views = [p.grad.data_ptr() - flat0 for i, p in enumerate(params) if i in red.slot]
        assert all(0 <= v < red.flat.numel() * 4 for v in views)
        assert set(ref) == set(eager) == set(replay)
        for k in ref:
            assert torch.equal(eager[k], 2.0 * ref[k]), k
            assert torch.equal(replay[k], 2.0 * ref[k]), k
        assert red.last_fallback == []
    finally:
        red.close()
        ops.set_grad_sink(None)
        if init_here:
            dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(400)  # the oracle's full 64-clip encoder step on the host (~1-2 min)
def test_cfg4_eight_shards_sum_to_full_batch(monkeypatch):
    """BASELINE config 4's shape in one process: the config-3 encoder (3 streams + residual +
    fusion) at B = 64 = 8 shards x 8 clips.  The eight shards' HIP gradients summed equal
    the full 64-clip HIP gradient and the (tie-aware) oracle's full-batch gradient, within
    the north-star 1e-3 — what the 8-GPU all-reduce of config 4 computes."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    # the same kernels for the 8- and the 64-clip launches (the launchers pick 16-row GEMM +
    # LayerNorm tiles and no chained next-op passes below 256 row tiles): the shards then
    # compute every clip's forward exactly as the full batch does, so no ReLU / max-pool
    # rounding tie can resolve differently between the two and the sums compare at rounding
    # level
    from scattennet_amd import ops
    ops.gemm_ln_force_rows(32)
    try:
        _cfg4_shards(monkeypatch)
    finally:
        ops.gemm_ln_force_rows(0)


def _cfg4_shards(monkeypatch):
    from scattennet_amd import ops, workloads as W
    from tests.test_gpu_scale import hip_encoder_step, tie_aware_encoder_oracle
    monkeypatch.setattr(ops, "_CHAIN_MIN_TILES", 0)  # chained next-op passes at 8 clips too
    dev = torch.device("cuda:0")
    w = dict(W.WORKLOADS["cfg3"], B=64)
    enc = W.build_encoder(w, dev, seed=8, init="random").eval()
    kp, mask, gout = W.synthetic_batch(w, dev, seed=12, ragged=False)
    g = torch.Generator().manual_seed(22)
    lens = torch.randint(1, w["T"] + 1, (64,), generator=g)
    lens[5], lens[40], lens[63] = w["T"], 1, 0
    mask = (torch.arange(w["T"])[None] < lens[:, None]).long().to(dev)
    named = dict(enc.named_parameters())
    for p in enc.parameters():
        p.grad = None
    fuse, pool_inputs, relu_outputs = hip_encoder_step(enc, kp, mask, gout[0], monkeypatch)
    full = {k: p.grad.detach().clone() for k, p in named.items() if p.grad is not None}
    shard_sum = {}
    for s in range(8):
        for p in enc.parameters():
            p.grad = None
        sl = slice(8 * s, 8 * s + 8)
        out = enc(kp[sl], mask[sl])[0]
        out.backward(gout[0, sl].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(out, fuse[sl]), (s, rel_err(out, fuse[sl]))  # the same per-clip forward
        for k, p in named.items():
            if p.grad is not None:
                shard_sum[k] = shard_sum[k] + p.grad if k in shard_sum else p.grad.detach().clone()
    assert set(full) == set(shard_sum)
    gscale = max(float(v.abs().max()) for v in full.values())
    for k in full:
        assert close(shard_sum[k].cpu(), full[k].cpu(), PARITY_TOL, gscale), (k, rel_err(shard_sum[k], full[k]))
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref, grads, stats = tie_aware_encoder_oracle(enc, w, kp, mask, gout[0], pool_inputs, relu_outputs, monkeypatch)
    print("cfg4 shape (cfg3 at B = 64) ties:", stats)
    assert rel_err(fuse, ref) < PARITY_TOL
    rscale = max(float(v.abs().max()) for v in grads.values())
    for k, v in grads.items():
        assert close(shard_sum[k].cpu(), v, PARITY_TOL, rscale), (k, rel_err(shard_sum[k].cpu(), v))


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["nccl", "gloo"])
def test_bucketed_reducer_averages_two_ranks(monkeypatch, backend):
    """The overlapped reducer's averaging at world size 2, driven through the RCCL branch of
    dp.GradBuckets._launch with a stand-in second rank: every bucket all-reduce issued by the
    reducer receives the other rank's bucket (its local gradients of a different batch, at
    the same offsets) — AVG: (mine + other) / 2; with the gloo backend (no AVG) the reducer
    must pre-scale by 1/2 and ask for SUM.  The result must be the mean of the two ranks'
    local gradients, bucket by bucket, bitwise."""
    import torch.distributed as dist

    from scattennet_amd import ops, workloads as W
    from scattennet_amd.dp import GradBuckets
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda:0")
    w = dict(W.WORKLOADS["cfg2"], B=2, T=64)
    model = W.build_streams(w, dev, seed=6, init="random")
    kp_a, mask_a, gout_a = W.synthetic_batch(w, dev, seed=31, ragged=True)
    kp_b, mask_b, gout_b = W.synthetic_batch(w, dev, seed=32, ragged=True)
    init_here = not dist.is_initialized()
    if init_here:
        port = 29900 + os.getpid() % 90
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    red = GradBuckets(model.parameters(), world=2, bucket_mb=4, overlap=True)
    red.backend = backend
    params = list(model.parameters())

    def step(kp, mask, gout):
        for p in params:
            p.grad = None
        outs = model(kp, mask)
        torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])
        red.sync()
        torch.cuda.synchronize()
        return red.flat.clone()

    try:
        red.collective = False
        step(kp_a, mask_a, gout_a)  # discovery step (builds the plan)
        local_a = step(kp_a, mask_a, gout_a)
        local_b = step(kp_b, mask_b, gout_b)
        red.collective = True
        ops_seen = []
        real = dist.all_reduce

        def second_rank(t, op=dist.ReduceOp.SUM, **k):
            o = (t.data_ptr() - red.flat.data_ptr()) // 4
            other = local_b[o:o + t.numel()]
            ops_seen.append((op, o, t.numel()))
            if op == dist.ReduceOp.AVG:
                t.add_(other).mul_(0.5)
            else:  # the other rank pre-scaled its bucket as this one did
                t.add_(other * 0.5)
            return real(t, op=dist.ReduceOp.SUM, **k)  # world 1: identity

        monkeypatch.setattr(dist, "all_reduce", second_rank)
        got = step(kp_a, mask_a, gout_a)
        want_op = dist.ReduceOp.AVG if backend == "nccl" else dist.ReduceOp.SUM
        assert len(ops_seen) == len(red.plan) and all(op == want_op for op, _, _ in ops_seen), ops_seen
        assert sorted(o for _, o, _ in ops_seen) == [o for o, _, _ in red.plan]
        want = (local_a + local_b) * 0.5 if backend == "nccl" else local_a * 0.5 + local_b * 0.5
        for o, n, _ in red.plan:
            assert torch.equal(got[o:o + n], want[o:o + n]), o
        assert not torch.equal(local_a, local_b)
    finally:
        red.close()
        ops.set_grad_sink(None)
        if init_here:
            dist.destroy_process_group()
