"""A backward that raises before its final callbacks (a user hook throwing at its very end, after
every weight-gradient section) must not poison the next one: the side-stream join and the
deferred LayerNorm affine reductions are keyed by the autograd graph task (ops._queue_join,
ops._affine_defer), so the next backward queues its own join / flush and drops the failed
one's pending reductions.  Checked bitwise against a clean backward (the kernels are
deterministic)."""
import pytest
import torch

from scattennet_amd import workloads as W

pytestmark = pytest.mark.gpu


def test_backward_after_a_raised_backward():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    dev = torch.device("cuda:0")
    w = dict(W.WORKLOADS["cfg2"], B=2)
    model = W.build_streams(w, dev, seed=3, init="random")
    kp, mask, gout = W.synthetic_batch(w, dev, seed=5, ragged=True)

    def run(x):
        outs = model(x, mask)
        torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])

    run(kp)
    torch.cuda.synchronize()
    ref = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    assert ref
    model.zero_grad(set_to_none=True)

    kp_bad = kp.clone().requires_grad_(True)  # its gradient is the backward's last product

    def boom(_):
        raise RuntimeError("boom")

    kp_bad.register_hook(boom)
    with pytest.raises(RuntimeError, match="boom"):
        run(kp_bad)
    torch.cuda.synchronize()
    model.zero_grad(set_to_none=True)

    run(kp)
    torch.cuda.synchronize()
    got = {n: p.grad for n, p in model.named_parameters() if p.grad is not None}
    assert set(got) == set(ref)
    for n, g in got.items():
        assert torch.equal(g, ref[n]), n
