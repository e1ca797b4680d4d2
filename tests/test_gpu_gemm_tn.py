"""Weight-gradient (TN) GEMM kernels at kernel level, against a float64 product on the GPU.

dW = alpha * dY^T X (dY [K, M], X [K, N]) and the fused bias gradient
db = bias_grad_scale * alpha * colsum(dY) — the nn.Linear weight / bias gradients of
attention.py:41-44,49-51,74 and layers.py:94-108 — through the C ABI (sca_gemm_variant):
the k-split kernel (tiles 36 / 37, 3- / 4-stage ring) at split-K 1 / 2 / 3 with the fused
(in-launch) and the two-launch combine, M and N not multiples of 64, bias on and off, alpha
and bias scale; the ACCUM epilogue; bitwise determinism; and the fallback to the
register-staged kernel when K is not a multiple of 32.
"""
import pytest
import torch

TOL = 2e-5


def _rel(a, b):
    return float((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _case(shapes, K, seed, bias=True, dev="cuda"):
    g = torch.Generator(device="cpu").manual_seed(seed)
    items = []
    for (M, N) in shapes:
        dY = torch.randn(K, M, generator=g).to(dev)
        X = torch.randn(K, N, generator=g).to(dev)
        dW = torch.full((M, N), float("nan"), device=dev)
        db = torch.full((M,), float("nan"), device=dev) if bias else None
        items.append((dY, X, dW, db))
    return items


def _probs(items, alpha=1.0, bscale=1.0, accum=False):
    from scattennet_amd import _lib as L, ops
    out = []
    for dY, X, dW, db in items:
        K, M = dY.shape
        N = X.shape[1]
        out.append(ops._prob([ops._seg(dY, X, M, N, K, alpha)], dW, M, N, N, bias_grad=db, bias_grad_scale=bscale,
                             epi=L.EPI_ACCUM if accum else 0))
    return out


def _check(items, alpha=1.0, bscale=1.0, base=None):
    for idx, (dY, X, dW, db) in enumerate(items):
        ref = alpha * (dY.double().t() @ X.double())
        if base is not None:
            ref = ref + base[idx].double()
        assert _rel(dW, ref) < TOL, (idx, _rel(dW, ref))
        if db is not None:
            rb = alpha * bscale * dY.double().sum(0)
            assert _rel(db, rb) < TOL, (idx, _rel(db, rb))


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [36, 37, 38, 39, 40, 43, 46])
@pytest.mark.parametrize("splitk,fused", [(1, False), (2, False), (2, True), (3, True), (5, True)])
def test_ksplit_kernel_matches_float64(tile, splitk, fused):
    """gemm_tnk_kernel (tiles 36 / 37) and gemm_tnb_kernel (38): M not a multiple of 64 / 128,
    bias on and off, split-K with the in-launch (fused) and the two-launch combine; split 5 of
    K = 1024 leaves the last split empty for tile 38 (64-row chunks: 256 x 4)."""
    from scattennet_amd import _lib as L, ops
    items = _case([(100, 68), (256, 256)], 1024, seed=tile + splitk) + _case([(64, 132)], 1024, seed=3, bias=False)
    probs = _probs(items, alpha=2.0, bscale=0.25)
    ws = torch.empty(sum(splitk * (p.M * p.N + p.M) for p in probs), device="cuda") if splitk > 1 else None
    saved = ops._SPLITK_FUSED
    ops._SPLITK_FUSED = fused
    try:
        ops.gemm(L.GEMM_TN, probs, splitk=splitk, ws=ws, tile=tile)
    finally:
        ops._SPLITK_FUSED = saved
    torch.cuda.synchronize()
    _check(items, alpha=2.0, bscale=0.25)


@pytest.mark.gpu
def test_ksplit_tile_falls_back_when_k_is_ragged():
    """K % 32 != 0: tile 36 is not eligible and the launcher takes the register-staged kernel."""
    from scattennet_amd import _lib as L, ops
    items = _case([(64, 64), (36, 100)], 200, seed=4)
    ops.gemm(L.GEMM_TN, _probs(items), splitk=1, tile=36)
    torch.cuda.synchronize()
    _check(items)




def _ksplit(items, tile=36, splitk=2, **kw):
    from scattennet_amd import _lib as L, ops
    probs = _probs(items, **kw)
    ws = torch.empty(sum(splitk * (p.M * p.N + p.M) for p in probs), device="cuda") if splitk > 1 else None
    ops.gemm(L.GEMM_TN, probs, splitk=splitk, ws=ws, tile=tile)
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_tnb_tile_falls_back_when_k_is_not_a_multiple_of_64():
    """K % 64 != 0 (K % 32 == 0): tile 38 hands over to the k-split kernel."""
    from scattennet_amd import ops
    items = _case([(128, 128), (100, 36)], 992, seed=6)
    probs = _probs(items)
    assert ops._gemm_kernel_name(2, probs, 38) == "gemm_tnk_kernel<3, 1, false>"
    _ksplit(items, tile=38, splitk=2)
    _check(items)


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [36, 38, 39, 43, 46])
def test_ksplit_bias_off_and_accumulate(tile):
    items = _case([(128, 192)] * 3, 512, seed=5, bias=False)
    base = [torch.randn(128, 192, device="cuda") for _ in items]
    for (_, _, dW, _), b in zip(items, base):
        dW.copy_(b)
    _ksplit(items, tile=tile, accum=True)
    _check(items, base=base)


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [36, 38, 39, 43, 46])
def test_ksplit_is_deterministic(tile):
    """The split-K slabs are summed in slice order whichever split arrives last."""
    items = _case([(256, 256)] * 6, 2048, seed=9)
    outs = []
    for _ in range(2):
        _ksplit(items, tile=tile, splitk=3)
        outs.append([(dW.clone(), db.clone()) for _, _, dW, db in items])
    for (a, b), (c, d) in zip(*outs):
        assert torch.equal(a, c) and torch.equal(b, d)


@pytest.mark.gpu
@pytest.mark.parametrize("splitk", [1, 2, 4])
def test_mixed_shape_launch_flat_grid(splitk):
    """One variant-46 launch holding problems of different shapes (an FFN's fc1 and fc2 weight
    gradients, 768 x 256 and 256 x 768, and a few odd ones): the flat grid of each problem's
    own tiles x splits, with the in-launch split-K combine, against float64."""
    from scattennet_amd import _lib as L, ops
    shapes = [(192, 64), (64, 192)] * 6 + [(100, 68), (68, 100), (256, 256), (40, 36)]
    items = _case(shapes, 512, seed=40 + splitk)
    probs = _probs(items, alpha=0.5, bscale=2.0)
    ws = torch.empty(sum(splitk * (p.M * p.N + p.M) for p in probs), device="cuda") if splitk > 1 else None
    ops.gemm(L.GEMM_TN, probs, splitk=splitk, ws=ws, tile=46)
    torch.cuda.synchronize()
    _check(items, alpha=0.5, bscale=2.0)
