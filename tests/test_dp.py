"""Multi-process data parallelism (world size 2, gloo on CPU): the bucketed gradient reducer
used by bench.py (scattennet_amd.dp.GradBuckets) reproduces the single-process gradient of the
whole global batch.  Ranks are launched exactly like the driver launches bench.py
(torch.distributed.run, 127.0.0.1).  The per-rank compute is CPU code: the collective logic is
what is under test (tests/test_gpu_dp.py covers the HIP path)."""
import os
import subprocess
import sys

import torch

from tests import dp_worker as DW

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(out, mode):
    port = str(29500 + (os.getpid() + {"sink": 7, "sink_raise": 13}.get(mode, 0)) % 2000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.join(ROOT, "tests", "dp_worker.py"),
           str(out), mode]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(out, weights_only=True)


def test_grad_allreduce_matches_full_batch(tmp_path):
    """Fallback path: gradients computed outside the ops sites, one flattened all-reduce."""
    got = _launch(tmp_path / "g.pt", "oracle")
    model = DW.W.build_streams(DW.WL, "cpu", seed=3, init="random")
    kp, mask, gout = DW.W.synthetic_batch(DW.WL, "cpu", seed=5, ragged=True)
    DW.grads(model, kp, mask, gout)
    ref = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    assert set(got) == set(ref)
    for k in ref:
        scale = float(ref[k].abs().max()) + 1e-6
        assert float((got[k] - ref[k]).abs().max()) / scale < 1e-4, k


def test_bucketed_reducer_matches_full_batch(tmp_path):
    """Sink path: discovery step, bucketed overlapped steps, a twice-used parameter (fallback),
    an unused parameter (no .grad), and an accumulation step."""
    got = _launch(tmp_path / "s.pt", "sink")
    ps, unused = DW.sink_model()
    ref = {}
    for step in range(3):
        x, gy = DW.sink_data(step)
        if step < 2:
            for p in ps:
                p.grad = None
        y = DW.sink_forward(ps, x)  # no sink installed here: plain autograd, whole batch
        # mean over the 2 ranks == average of the per-rank sums; step 2 accumulates onto step
        # 1's averaged .grad and the reducer averages the sums as a whole: step-1 avg + step-2 avg
        y.backward(gy / 2)
        ref[f"step{step}"] = [p.grad.clone() for p in ps]
    for step in range(3):
        for i, (a, b) in enumerate(zip(got[f"step{step}"], ref[f"step{step}"])):
            assert float((a - b).abs().max()) <= 1e-5 * (float(b.abs().max()) + 1e-6), (step, i)
    # planned parameters' .grad are views of the flat buckets; the twice-used layer is not planned
    assert got["step1_slot"] == [True, True, False, False, True, True, True, True]
    assert not any(got["step0_slot"])  # discovery step: plain allocations
    assert len(got["buckets"]) >= 2 and got["unused_grad_none"]


def test_bucketed_reducer_recovers_from_a_raised_backward(tmp_path):
    """A backward that raised before the reducer's finish (its all-reduces issued, never
    joined) is drained at the next backward's first sink call; the next step is exact."""
    got = _launch(tmp_path / "r.pt", "sink_raise")
    assert got["raised"]
    ps, _ = DW.sink_model()
    x, gy = DW.sink_data(2)
    y = DW.sink_forward(ps, x)
    y.backward(gy / 2)
    for i, (a, p) in enumerate(zip(got["after"], ps)):
        b = p.grad
        assert float((a - b).abs().max()) <= 1e-5 * (float(b.abs().max()) + 1e-6), i
