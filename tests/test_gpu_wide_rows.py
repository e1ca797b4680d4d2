"""Row kernels beyond 1024 columns (rowops.hip ln_*_wide_kernel / softmax_*_wide_kernel): the
reference's nn.LayerNorm and softmax take any width (model/residual.py:31-38,
keypoint_module.py:66-72, fusion.py:52-53), so widths over the register kernels' 1024 run a
row-looping kernel.  Forward and every gradient against torch's fp32 CPU ops within the
north-star 1e-3 (floating-point kernels: a torch fp32 reference of the same op)."""
import pytest
import torch

from tests.golden_util import rel_err

PARITY_TOL = 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1100, 2048, 3001])
def test_layer_norm_wide(N):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import scattennet_amd  # noqa: F401
    torch.manual_seed(N)
    x, w, b = torch.randn(37, N) * 2 + 0.5, torch.randn(N), torch.randn(N)
    xg, wg, bg = (t.cuda().requires_grad_(True) for t in (x, w, b))
    y = torch.ops.scatten.layer_norm(xg, wg, bg, 1e-5)[0]
    g = torch.randn(37, N)
    y.backward(g.cuda())
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    ref = torch.nn.functional.layer_norm(xr, (N,), wr, br, 1e-5)
    (ref * g).sum().backward()
    assert rel_err(y, ref) < PARITY_TOL
    for got, want in ((xg, xr), (wg, wr), (bg, br)):
        assert rel_err(got.grad, want.grad) < PARITY_TOL


@pytest.mark.gpu
def test_layer_norm_ex_wide_post_relu():
    """y = ReLU(LayerNorm(x) * gamma + beta + post) at N = 1280 (a wide ResidualBlock)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import scattennet_amd  # noqa: F401
    torch.manual_seed(7)
    B, T, N = 2, 21, 1280
    x, post, w, b = torch.randn(B, T, N), torch.randn(B, T, N), torch.randn(N), torch.randn(N)
    xg, pg, wg, bg = (t.cuda().requires_grad_(True) for t in (x, post, w, b))
    y = torch.ops.scatten.layer_norm_ex(xg, None, pg, wg, bg, 1e-5, True)
    y = y[0] if isinstance(y, (tuple, list)) else y
    g = torch.randn(B, T, N)
    y.backward(g.cuda())
    xr, pr, wr, br = (t.clone().requires_grad_(True) for t in (x, post, w, b))
    ref = torch.relu(torch.nn.functional.layer_norm(xr, (N,), wr, br, 1e-5) + pr)
    (ref * g).sum().backward()
    assert rel_err(y, ref) < PARITY_TOL
    for got, want in ((xg, xr), (pg, pr), (wg, wr), (bg, br)):
        assert rel_err(got.grad, want.grad) < PARITY_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1500, 4100])
def test_softmax_rows_wide(N):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    import scattennet_amd  # noqa: F401
    torch.manual_seed(N)
    x = torch.randn(3, 5, N) * 3
    xg = x.cuda().requires_grad_(True)
    y = torch.ops.scatten.softmax_rows(xg)
    g = torch.randn(3, 5, N)
    y.backward(g.cuda())
    xr = x.clone().requires_grad_(True)
    ref = torch.softmax(xr, dim=-1)
    (ref * g).sum().backward()
    assert rel_err(y, ref) < PARITY_TOL
    assert rel_err(xg.grad, xr.grad) < PARITY_TOL
