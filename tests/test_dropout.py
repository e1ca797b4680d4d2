"""Training-mode dropout (p > 0): the counter-based mask of include/scatten.h (sca_dropout),
fused into the GEMM / LayerNorm epilogues and applied elementwise in the backward.

torch's Philox stream cannot be reproduced outside ATen, so parity is defined on the HIP
path's own mask: the oracle (oracle/sca_oracle.py: dropout_mask / Drop) regenerates it from
the seeds the HIP path drew, in the reference's call order, and every output and gradient
must then match within the north-star 1e-3.  The mask itself is pinned by a scalar
restatement and by its keep-rate statistics (CPU tests).
"""
import numpy as np
import pytest
import torch

from oracle import sca_oracle as O
from tests.golden_util import close, load, rel_err

PARITY_TOL = 1e-3


# --------------------------------------------------------------------------- the mask (CPU)
def _mix_scalar(x):
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    return x ^ (x >> 16)


def _keep_scalar(seed, e, p):
    key = _mix_scalar((seed & 0xFFFFFFFF) ^ _mix_scalar(((seed >> 32) + 0x9E3779B9) & 0xFFFFFFFF))
    thr = int(np.float32(p) * np.float32(4294967296.0))
    return _mix_scalar(_mix_scalar(e ^ key) + key) >= thr


def test_mask_matches_scalar_restatement():
    for seed in (0, 1, 0x123456789ABCDEF, 2 ** 63 - 1):
        m = O.dropout_mask(seed, (7, 13), 0.2).reshape(-1)
        assert [bool(v) for v in m] == [_keep_scalar(seed, e, 0.2) for e in range(91)]


@pytest.mark.parametrize("p", [0.1, 0.2, 0.5])
def test_mask_keep_rate_and_independence(p):
    a = O.dropout_mask(11, (1000, 1000), p)
    b = O.dropout_mask(12, (1000, 1000), p)
    assert abs(a.float().mean().item() - (1 - p)) < 2e-3
    # two seeds: independent masks (agreement rate of two Bernoulli(1-p))
    agree = (a == b).float().mean().item()
    assert abs(agree - ((1 - p) ** 2 + p ** 2)) < 3e-3
    # no row/column structure
    assert a.float().mean(0).std().item() < 0.05 and a.float().mean(1).std().item() < 0.05


def test_dropout_scales_kept_values():
    x = torch.randn(64, 33)
    y = O.dropout(x, 5, 0.25)
    keep = O.dropout_mask(5, (64, 33), 0.25)
    assert torch.equal(y[~keep], torch.zeros_like(y[~keep]))
    assert torch.allclose(y[keep], x[keep] / 0.75)


# --------------------------------------------------------------------------- HIP path (GPU)
class SeedLog:
    """Deterministic seed source for ops.dropout_seeds that records every draw."""

    def __init__(self, seed=2024):
        self.rng = np.random.default_rng(seed)
        self.draws = []

    def __call__(self, n):
        d = [int(v) for v in self.rng.integers(0, 2 ** 63 - 1, size=n, dtype=np.int64)]
        self.draws.append(d)
        return d

    def stream(self, g):
        return [d[g] for d in self.draws]


@pytest.fixture
def seedlog():
    from scattennet_amd import ops
    log = SeedLog()
    if torch.cuda.is_available():  # the oracle replays raw seeds: device step counter at 0
        ops.dropout_counter().zero_()
    ops._SEED_SOURCE = log
    yield log
    ops._SEED_SOURCE = None


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda:0")


def _grads_close(module, ref_params, tol=PARITY_TOL):
    grads = {k: v.grad for k, v in ref_params.items() if v.grad is not None}
    gscale = max(float(g.abs().max()) for g in grads.values())
    named = dict(module.named_parameters())
    for k, g in grads.items():
        assert named[k].grad is not None, k
        assert close(named[k].grad.cpu(), g, tol, gscale), (k, rel_err(named[k].grad.cpu(), g))


def _ref_params(module):
    return {k: v.detach().cpu().clone().requires_grad_(True) for k, v in module.state_dict().items()}


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols", [(512, 256), (37, 19), (1, 3)])
def test_sca_dropout_kernel_matches_oracle_mask(rows, cols):
    from scattennet_amd import ops
    dev = _dev()
    x = torch.randn(rows, cols, device=dev)
    y = torch.empty_like(x)
    ops.dropout_apply([(x, y, 987654321)], 0.2)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), O.dropout(x.cpu(), 987654321, 0.2))


@pytest.mark.gpu
def test_feed_forward_train_dropout(seedlog):
    import scattennet_amd as S
    dev = _dev()
    torch.manual_seed(0)
    m = S.FeedForward(64, 192, 0.2).to(dev).train()
    x = torch.randn(2, 40, 64, device=dev, requires_grad=True)
    out = m(x)
    g = torch.randn_like(out)
    out.backward(g)
    p = _ref_params(m)
    xr = x.detach().cpu().requires_grad_(True)
    ref = O.feed_forward({"m." + k: v for k, v in p.items()}, "m", xr, O.Drop(0.2, seedlog.stream(0)))
    assert rel_err(out, ref) < PARITY_TOL
    (ref * g.cpu()).sum().backward()
    assert rel_err(x.grad, xr.grad) < PARITY_TOL
    _grads_close(m, p)
    assert 0.7 < float((out != 0).float().mean()) < 0.9  # ~80% kept


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["self_attn", "causal_attn"])
def test_coordinate_attention_train_dropout(kind, seedlog):
    import scattennet_amd as S
    dev = _dev()
    fx = load("coordattn_" + kind)
    cfg = dict(fx["meta"]["cfg"], dropout=0.2)
    m = S.CoordinateAttention(cfg, kind)
    m.load_state_dict(fx["param"])
    m = m.to(dev).train()
    x = fx["in"]["coord_embed"].to(dev).requires_grad_(True)
    mask = fx["in"]["mask"].to(dev)
    out = m(x, S.key_padding_mask(mask, causal=(kind == "causal_attn")))
    out.backward(fx["gout"].to(dev))
    p = _ref_params(m)
    xr = fx["in"]["coord_embed"].clone().requires_grad_(True)
    am = O.additive_causal_mask(fx["in"]["mask"]) if kind == "causal_attn" else O.additive_key_mask(fx["in"]["mask"])
    ref = O.coordinate_attention(p, "", xr, am, cfg["attention_heads"], kind, O.Drop(0.2, seedlog.stream(0)))
    assert rel_err(out, ref) < PARITY_TOL
    (ref * fx["gout"]).sum().backward()
    assert rel_err(x.grad, xr.grad) < PARITY_TOL
    _grads_close(m, p)


@pytest.mark.gpu
def test_sca_stack_train_dropout(seedlog):
    """A3 embedding dropout + every block's dropout, L = 2, against the oracle."""
    import scattennet_amd as S
    dev = _dev()
    fx = load("sca_L2")
    cfg = dict(fx["meta"]["cfg"], dropout=0.2)
    m = S.SeparativeCoordinateAttention(cfg)
    m.load_state_dict(fx["param"])
    m = m.to(dev).train()
    xe = fx["in"]["x_embed"].to(dev).requires_grad_(True)
    ye = fx["in"]["y_embed"].to(dev).requires_grad_(True)
    out = m(xe, ye, fx["in"]["mask"].to(dev))
    out.backward(fx["gout"].to(dev))
    p = _ref_params(m)
    xr = fx["in"]["x_embed"].clone().requires_grad_(True)
    yr = fx["in"]["y_embed"].clone().requires_grad_(True)
    ref = O.sca(p, "", xr, yr, fx["in"]["mask"], cfg, drop=O.Drop(0.2, seedlog.stream(0)))
    assert rel_err(out, ref) < PARITY_TOL
    (ref * fx["gout"]).sum().backward()
    assert rel_err(xe.grad, xr.grad) < PARITY_TOL and rel_err(ye.grad, yr.grad) < PARITY_TOL
    _grads_close(m, p)


@pytest.mark.gpu
@pytest.mark.parametrize("d,H,L", [(64, 4, 2), (256, 16, 1)])  # d 256: GEMM + LayerNorm launches, fused bwd
def test_grouped_streams_train_dropout(seedlog, d, H, L):
    """Two streams in one grouped launch: each stream gets its own masks."""
    from scattennet_amd import workloads as W
    dev = _dev()
    w = dict(W.WORKLOADS["cfg1"], groups=[12, 15], B=2, T=32, d=d, H=H, L=L, maxpos=32)
    import scattennet_amd as S
    model = W.build_streams(w, dev, seed=3, init="random")
    for sub in model.modules():  # the block dropouts (cfg["dropout"]); attention_dropout stays 0
        if isinstance(sub, (S.CoordinateAttention, S.CoordinatesMerge, S.FeedForward,
                            S.SeparativeCoordinateAttention)):
            sub.dropout = 0.2
    model.train()
    kp, mask, gout = W.synthetic_batch(w, dev, seed=5, ragged=True)
    outs = model(kp, mask)
    torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])
    cfg = dict(W.model_cfg(w["d"], w["H"], w["L"], maxpos=w["maxpos"]), dropout=0.2)
    groups = W.split_groups(w["groups"])
    assert all(len(d) == 2 and d[0] != d[1] for d in seedlog.draws)  # one mask per stream
    for g, mod in enumerate(model.streams):
        p = _ref_params(mod)
        ref = O.multi_stream_sca([p], kp.cpu(), mask.cpu(), [groups[g]], cfg,
                                 drops=[O.Drop(0.2, seedlog.stream(g))])[0]
        assert rel_err(outs[g], ref) < PARITY_TOL, g
        (ref * gout[g].cpu()).sum().backward()
        _grads_close(mod, p)


@pytest.mark.gpu
def test_fusion_train_dropout(seedlog):
    import scattennet_amd as S
    dev = _dev()
    fx = load("fusion")
    m = S.CoordinatesFusion(fx["meta"]["in"], fx["meta"]["out"], 0.2)
    m.load_state_dict(fx["param"])
    m = m.to(dev).train()
    ins = {k: fx["in"][k].to(dev).requires_grad_(True) for k in ("left", "right", "body")}
    out = m(ins["left"], ins["right"], ins["body"])
    out.backward(fx["gout"].to(dev))
    p = _ref_params(m)
    refs = {k: fx["in"][k].clone().requires_grad_(True) for k in ("left", "right", "body")}
    ref = O.coordinates_fusion(p, "", refs["left"], refs["right"], refs["body"], drop=O.Drop(0.2, seedlog.stream(0)))
    assert rel_err(out, ref) < PARITY_TOL
    (ref * fx["gout"]).sum().backward()
    for k in ins:
        assert rel_err(ins[k].grad, refs[k].grad) < PARITY_TOL, k
    _grads_close(m, p)


@pytest.mark.gpu
def test_graph_replays_draw_fresh_masks():
    """Seeds are frozen in a captured graph's kernel arguments; the device step counter
    (ops.advance_dropout, captured) still gives every replay new masks."""
    import scattennet_amd as S
    from scattennet_amd import ops
    dev = _dev()
    m = S.FeedForward(64, 192, 0.2).to(dev).train()
    x = torch.randn(2, 40, 64, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.advance_dropout()
        m(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.advance_dropout()
        y = m(x)
    g.replay()
    a = (y == 0).clone()
    g.replay()
    b = (y == 0).clone()
    torch.cuda.synchronize()
    assert 0.1 < float(a.float().mean()) < 0.3 and not torch.equal(a, b)


# --------------------------------------------------------------------------- attention dropout
@pytest.mark.gpu
@pytest.mark.parametrize("kind,B,Tq,Tk,d,H,explicit", [
    ("self", 2, 96, 96, 64, 4, False),      # hd 16: the fused single-launch backward
    ("causal", 2, 80, 80, 64, 4, False),
    ("cross", 2, 48, 70, 64, 4, False),
    ("self", 2, 300, 300, 64, 2, False),    # hd 32 beyond one key block: the key-block backward
    ("causal", 2, 270, 270, 64, 2, False),
    ("self", 2, 70, 70, 128, 2, False),     # hd 64: split dq / dkdv kernels
    ("cross", 2, 40, 50, 64, 4, True),      # a materialised additive mask: the general path
    ("self", 2, 40, 40, 320, 2, False),     # hd 160 > 128: GEMM + row-softmax path, sca_dropout on P
    ("causal", 2, 36, 36, 256, 1, False),   # hd 256
    ("cross", 2, 30, 44, 320, 2, True),
])
def test_attention_probability_dropout(kind, B, Tq, Tk, d, H, explicit, seedlog):
    """attention.py:67-69 / 119-121 / 173-175: F.dropout on the softmax probabilities in
    training mode — forward (O from the dropped probabilities, statistics of the undropped
    ones) and every gradient against the oracle replaying the HIP path's seed."""
    import scattennet_amd as S
    dev = _dev()
    torch.manual_seed(Tq + Tk)
    cls = {"self": S.SelfAttention, "causal": S.SelfCausalAttention, "cross": S.CrossAttention}[kind]
    m = cls(d, H, dropout=0.3)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) / (p.shape[-1] ** 0.5 if p.dim() == 2 else 10.0))
    m = m.to(dev).train()
    x, kv = torch.randn(B, Tq, d), torch.randn(B, Tk, d)
    mask = torch.ones(B, Tk, dtype=torch.long)
    mask[1, Tk // 2:] = 0
    if kind == "causal":
        am = O.additive_causal_mask(mask)
    else:
        am = O.additive_key_mask(mask, tgt_len=Tq)
    amask = am.to(dev) if explicit else S.key_padding_mask(mask.to(dev), causal=(kind == "causal"))
    xg, kvg = x.to(dev).requires_grad_(True), kv.to(dev).requires_grad_(True)
    out = m(xg, kvg, amask) if kind == "cross" else m(xg, amask)
    g = torch.randn(out.shape)
    out.backward(g.to(dev))
    p = _ref_params(m)
    xr, kvr = x.clone().requires_grad_(True), kv.clone().requires_grad_(True)
    ref = O.attention({"a." + k: v for k, v in p.items()}, "a", xr, kvr if kind == "cross" else xr, am, H, kind,
                      O.Drop(0.3, seedlog.stream(0)))
    assert len(seedlog.draws) == 1  # one seed per call
    assert rel_err(out, ref) < PARITY_TOL
    (ref * g).sum().backward()
    assert rel_err(xg.grad, xr.grad) < PARITY_TOL
    if kind == "cross":
        assert rel_err(kvg.grad, kvr.grad) < PARITY_TOL
    _grads_close(m, p)
    # dropout actually applied: the eval-mode output differs
    with torch.no_grad():
        m.eval()
        ev = m(xg, kvg, amask) if kind == "cross" else m(xg, amask)
    assert rel_err(ev, out.detach()) > 1e-2


@pytest.mark.gpu
def test_sca_stack_attention_and_block_dropout(seedlog):
    """The SCA stack (L = 2) with attention_dropout 0.1 AND the blocks' dropout 0.2: every
    attention draws its seed before its block's own (the reference's call order)."""
    import scattennet_amd as S
    dev = _dev()
    fx = load("sca_L2")
    cfg = dict(fx["meta"]["cfg"], dropout=0.2, attention_dropout=0.1)
    m = S.SeparativeCoordinateAttention(cfg)
    m.load_state_dict(fx["param"])
    m = m.to(dev).train()
    xe = fx["in"]["x_embed"].to(dev).requires_grad_(True)
    ye = fx["in"]["y_embed"].to(dev).requires_grad_(True)
    out = m(xe, ye, fx["in"]["mask"].to(dev))
    out.backward(fx["gout"].to(dev))
    p = _ref_params(m)
    xr = fx["in"]["x_embed"].clone().requires_grad_(True)
    yr = fx["in"]["y_embed"].clone().requires_grad_(True)
    seeds = iter(seedlog.stream(0))  # one stream of seeds shared by both dropout kinds
    ref = O.sca(p, "", xr, yr, fx["in"]["mask"], cfg, drop=O.Drop(0.2, seeds), attn_drop=O.Drop(0.1, seeds))
    assert next(seeds, None) is None  # every seed the HIP path drew was used
    assert rel_err(out, ref) < PARITY_TOL
    (ref * fx["gout"]).sum().backward()
    assert rel_err(xe.grad, xr.grad) < PARITY_TOL and rel_err(ye.grad, yr.grad) < PARITY_TOL
    _grads_close(m, p)
