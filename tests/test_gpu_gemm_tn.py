"""Weight-gradient (TN) GEMM kernels at kernel level, against a float64 product on the GPU.

dW = alpha * dY^T X (dY [K, M], X [K, N]) and the fused bias gradient
db = bias_grad_scale * alpha * colsum(dY) — the nn.Linear weight / bias gradients of
attention.py:41-44,49-51,74 and layers.py:94-108 — through the C ABI:
* sca_gemm_tn_streamk (the stream-K kernel): the config-2/5 shapes, ragged M / N, bias on / off,
  alpha and bias scale, the ACCUM epilogue, workgroup counts from 1 to more than the blocks,
  4- and 8-slice blocks (tiles split into many pieces combined in-launch), determinism, a
  captured graph replayed twice, and the refusal of shapes it cannot take;
* sca_gemm_variant: the k-split kernel (tiles 36 / 37, 3- / 4-stage ring) at split-K 1 / 2 / 3 with the fused
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


def _streamk(items, nwg=0, spb=0, **kw):
    from scattennet_amd import ops
    ops.gemm_tn_streamk(_probs(items, **kw), nwg=nwg, spb=spb)
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("name,shapes,K", [
    ("attn 16x(256,256)", [(256, 256)] * 16, 2048),
    ("fc1 4x(768,256)", [(768, 256)] * 4, 2048),
    ("fc2 4x(256,768)", [(256, 768)] * 4, 2048),
    ("cfg5 attn 4x(512,512)", [(512, 512)] * 4, 8192),
    ("ragged", [(100, 36), (4, 260), (132, 68)], 384),
])
def test_streamk_matches_float64(name, shapes, K):
    items = _case(shapes, K, seed=len(name))
    _streamk(items)
    _check(items)


@pytest.mark.gpu
@pytest.mark.parametrize("nwg", [1, 3, 7, 37, 256, 100000])
@pytest.mark.parametrize("spb", [4, 8])
def test_streamk_pieces_any_workgroup_count(nwg, spb):
    """Every split of the block range: one workgroup for all tiles, prime counts (tiles cut into
    uneven pieces, pieces spanning several workgroups), more workgroups than blocks."""
    items = _case([(192, 128), (68, 260), (256, 64)], 1024, seed=nwg + spb)
    _streamk(items, nwg=nwg, spb=spb, alpha=0.5, bscale=3.0)
    _check(items, alpha=0.5, bscale=3.0)


@pytest.mark.gpu
def test_streamk_bias_off_and_accumulate():
    items = _case([(128, 192)] * 3, 512, seed=5, bias=False)
    base = [torch.randn(128, 192, device="cuda") for _ in items]
    for (_, _, dW, _), b in zip(items, base):
        dW.copy_(b)
    _streamk(items, nwg=5, accum=True)
    _check(items, base=base)


@pytest.mark.gpu
def test_streamk_is_deterministic():
    items = _case([(256, 256)] * 6, 2048, seed=9)
    outs = []
    for _ in range(2):
        _streamk(items, nwg=97)
        outs.append([(dW.clone(), db.clone()) for _, _, dW, db in items])
    for (a, b), (c, d) in zip(*outs):
        assert torch.equal(a, c) and torch.equal(b, d)


@pytest.mark.gpu
def test_streamk_refuses_unsupported_shapes():
    from scattennet_amd import _lib as L, ops
    items = _case([(64, 64)], 96, seed=1)  # K not a multiple of 128
    with pytest.raises(ValueError):
        ops.gemm_tn_streamk(_probs(items))
    assert not ops.tn_streamk_ok(items[0][0], items[0][1], items[0][2])
    items = _case([(66, 64)], 256, seed=1)  # M not a multiple of 4
    with pytest.raises(ValueError):
        ops.gemm_tn_streamk(_probs(items))
    assert L.lib().sca_gemm_tn_streamk(1, (L.GemmProblem * 1)(*_probs(_case([(64, 64)], 256, 1))), 0, 5,
                                       None, None, None) == 1  # bad slices_per_block / pointers


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [36, 37])
@pytest.mark.parametrize("splitk,fused", [(1, False), (2, False), (2, True), (3, True)])
def test_ksplit_kernel_matches_float64(tile, splitk, fused):
    """gemm_tnk_kernel (tiles 36 / 37): M not a multiple of 64, bias on and off, split-K with the
    in-launch (fused) and the two-launch combine."""
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
def test_ksplit_bias_off_and_accumulate():
    items = _case([(128, 192)] * 3, 512, seed=5, bias=False)
    base = [torch.randn(128, 192, device="cuda") for _ in items]
    for (_, _, dW, _), b in zip(items, base):
        dW.copy_(b)
    _ksplit(items, accum=True)
    _check(items, base=base)


@pytest.mark.gpu
def test_ksplit_is_deterministic():
    """The split-K slabs are summed in slice order whichever split arrives last."""
    items = _case([(256, 256)] * 6, 2048, seed=9)
    outs = []
    for _ in range(2):
        _ksplit(items, splitk=3)
        outs.append([(dW.clone(), db.clone()) for _, _, dW, db in items])
    for (a, b), (c, d) in zip(*outs):
        assert torch.equal(a, c) and torch.equal(b, d)


@pytest.mark.gpu
def test_streamk_in_captured_graph():
    """Captured (as in the bench step) and replayed: several launches back to back on fresh
    workspace from the graph pool and counters from the ring, replayed twice."""
    from scattennet_amd import ops
    items = _case([(256, 256)] * 4 + [(768, 256)], 2048, seed=12)
    items2 = _case([(256, 768)] * 2, 1024, seed=13)
    p1, p2 = _probs(items), _probs(items2, alpha=0.5)
    ops.gemm_tn_streamk(p1)  # warm (lazy state) outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(3):
            ops.gemm_tn_streamk(p1)
            ops.gemm_tn_streamk(p2, nwg=37)
    for _, _, dW, db in items + items2:
        dW.fill_(float("nan"))
        db.fill_(float("nan"))
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    _check(items)
    _check(items2, alpha=0.5)
    for ring, _ in ops._CNT.values():
        assert int(ring.abs().sum()) == 0
