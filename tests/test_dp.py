"""Multi-process data parallelism (world size 2, gloo on CPU): the gradient all-reduce used by
bench.py (scattennet_amd.dp.GradAllReduce) reproduces the single-process gradient of the whole
global batch.  Ranks are launched exactly like the driver launches bench.py
(torch.distributed.run, 127.0.0.1); the per-rank compute is the CPU oracle — the collective
logic is what is under test (the HIP path needs a GPU)."""
import os
import subprocess
import sys

import torch

from tests import dp_worker as DW

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_grad_allreduce_matches_full_batch(tmp_path):
    out = tmp_path / "g.pt"
    port = str(29500 + os.getpid() % 2000)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.join(ROOT, "tests", "dp_worker.py"), str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    got = torch.load(out, weights_only=True)
    model = DW.W.build_streams(DW.WL, "cpu", seed=3, init="random")
    kp, mask, gout = DW.W.synthetic_batch(DW.WL, "cpu", seed=5, ragged=True)
    DW.grads(model, kp, mask, gout)
    ref = {k: p.grad for k, p in model.named_parameters() if p.grad is not None}
    assert set(got) == set(ref)
    for k in ref:
        scale = float(ref[k].abs().max()) + 1e-6
        assert float((got[k] - ref[k]).abs().max()) / scale < 1e-4, k
