"""sca_sum_tensors and the FanOut op (ops.fan_out): the gradient of a tensor read by several
ops summed in one grouped launch equals autograd's pairwise sum (keypoint_module.py:181-187:
the final x-stream map read by every merge layer)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fan_out_gradient_sum():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from scattennet_amd import ops
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(5, 7, 12, generator=g).to(dev).requires_grad_(True) for _ in range(3)]
    ws = [[torch.randn(5, 7, 12, generator=g).to(dev) for _ in range(3)] for _ in range(4)]
    outs = ops.fan_out(xs, 4)
    loss = sum((o * w).sum() for i in range(4) for o, w in zip(outs[i], ws[i]))
    loss.backward()
    for gi, x in enumerate(xs):
        want = sum(ws[i][gi] for i in range(4))
        assert torch.allclose(x.grad, want, rtol=0, atol=1e-6), gi
    # a consumer that never runs backward (no gradient for that alias) is skipped
    ys = [torch.randn(33, generator=g).to(dev).requires_grad_(True)]
    o = ops.fan_out(ys, 3)
    (o[0][0] * 2.0).sum().backward()
    assert torch.allclose(ys[0].grad, torch.full_like(ys[0], 2.0))


def test_sum_tensors_fixed_order():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from scattennet_amd import ops
    dev = torch.device("cuda:0")
    ins = [torch.randn(1001, device=dev) for _ in range(8)]
    out = torch.empty_like(ins[0])
    ops.sum_tensors([(out, ins)])
    want = ins[0].clone()
    for t in ins[1:]:
        want += t
    assert torch.equal(out, want)  # left to right, bit for bit
