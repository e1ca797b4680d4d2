"""fp16 / bf16 modules (scattennet_amd/precision.py): `model.half()` / `.to(torch.bfloat16)` of the
drop-in modules run the fp32 HIP path on fp32 views of the reduced parameters and return the
module's dtype; gradients land on the reduced parameters in their dtype.

Checked against the SAME module in fp32 holding the rounded parameters: the outputs differ only
by the final rounding to the module's dtype (fp16: 2^-11, bf16: 2^-8 relative), the gradients by
the rounding of the incoming gradient and of the parameter gradients themselves.  The reference
computes such a model in fp16 arithmetic (model/keypoint_module.py:74-78 clamps its overflow);
its fp16 / bf16 results are not reproduced bit for bit, but they are pinned: fixtures captured
from the reference running in float16 and bfloat16 (tests/golden/gen_golden_half.py; the SCA
stack and both CoordinateAttention kinds) are matched within 4e-3 / 6e-3 (fp16: outputs /
gradients, of their scale; measured 5e-4 to 1.9e-3) and 3e-2 / 4e-2 (bf16; measured 1.8e-3 to
8.6e-3).  Not covered: a fully padded clip under a materialised fp16 mask,
where the reference's fp16 s + finfo(fp16).min quantises the scores to multiples of 32.
"""
import copy

import pytest
import torch

from scattennet_amd import workloads as W
from tests.golden_util import close, rel_err

pytestmark = pytest.mark.gpu

TOL = {torch.float16: 2e-3, torch.bfloat16: 1.6e-2}


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda:0")


def _check(low, ref, kp, mask, gout, dt, name):
    outs_l = low(kp.to(dt), mask)
    outs_r = ref(kp.to(dt).float(), mask)
    outs_l = outs_l if isinstance(outs_l, (list, tuple)) else [outs_l]
    outs_r = outs_r if isinstance(outs_r, (list, tuple)) else [outs_r]
    for o in outs_l:
        assert o.dtype == dt, (name, o.dtype)
    for g, (a, b) in enumerate(zip(outs_l, outs_r)):
        assert rel_err(a.float(), b) < TOL[dt], (name, "out", g, rel_err(a.float(), b))
    torch.autograd.backward(outs_l, [gout[g].to(dt) for g in range(len(outs_l))])
    torch.autograd.backward(outs_r, [gout[g].to(dt).float() for g in range(len(outs_r))])
    torch.cuda.synchronize()
    named_r = dict(ref.named_parameters())
    grads = {k: p.grad for k, p in low.named_parameters() if p.grad is not None}
    assert grads, name
    gscale = max(float(named_r[k].grad.abs().max()) for k in grads)
    for k, gl in grads.items():
        assert gl.dtype == dt, (name, k, gl.dtype)
        gr = named_r[k].grad
        assert close(gl.float(), gr, 4 * TOL[dt], gscale), (name, k, rel_err(gl.float(), gr))


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_sca_streams_reduced_precision(dt):
    dev = _dev()
    w = W.WORKLOADS["cfg1"]
    base = W.build_streams(w, dev, seed=3, init="random")
    low = copy.deepcopy(base).to(dt)
    ref = copy.deepcopy(low).float()  # fp32 module holding the rounded parameters
    kp, mask, gout = W.synthetic_batch(w, dev, seed=5, ragged=True)
    _check(low, ref, kp, mask, gout, dt, "streams")


def test_encoder_half():
    dev = _dev()
    w = dict(W.WORKLOADS["cfg3_t234"], B=2)
    base = W.build_encoder(w, dev, seed=2, init="random")
    low = copy.deepcopy(base).half()
    ref = copy.deepcopy(low).float()
    kp, mask, _ = W.synthetic_batch(w, dev, seed=4, ragged=True)
    g = torch.Generator().manual_seed(9)
    shapes = [o.shape for o in ref(kp.half().float(), mask)]
    gout = [torch.randn(s, generator=g).to(dev) for s in shapes]
    _check(low, ref, kp, mask, gout, torch.float16, "encoder")


def test_fp16_clamp_matches_reference_rule():
    """An fp16 CoordinateAttention output overflowing fp16 is clamped like the reference's."""
    dev = _dev()
    from scattennet_amd import CoordinateAttention
    cfg = W.model_cfg(64, 4, 1, maxpos=64)
    torch.manual_seed(0)
    blk = CoordinateAttention(cfg, "self_attn").to(dev)
    with torch.no_grad():  # a LayerNorm gain that takes the outputs past fp16's range
        blk.last_layer_norm.weight.fill_(3e4)
    blk = blk.half()
    x = torch.randn(2, 16, 64, device=dev).half()
    mask = torch.zeros(2, 1, 16, 16, device=dev).half()
    y = blk(x, mask)
    # the bound as the reference's torch.clamp leaves it in fp16 (64504 rounds to 64512)
    cv = float(torch.tensor(torch.finfo(torch.float16).max - 1000).half())
    y = y.detach()
    assert y.dtype == torch.float16
    assert torch.isfinite(y).all()
    assert float(y.float().abs().max()) == cv


# fp16 / bf16 fixtures from the REFERENCE computing in that dtype on the CPU (tests/golden/
# gen_golden_half.py): the drop-in modules compute in fp32 and round at the module boundary,
# the reference rounds every intermediate — they agree to a few units of the dtype's roundoff
# (fp16 4.9e-4, bf16 3.9e-3) of the tensors' scale, not to the fp32 1e-3 of the fp32 fixtures.
REF_TOL = {torch.float16: {"out": 4e-3, "grad": 6e-3, "noise": 1e-4},    # measured: 5e-4 - 1.9e-3
           torch.bfloat16: {"out": 3e-2, "grad": 4e-2, "noise": 2e-3}}
PREFIX = {torch.float16: "half", torch.bfloat16: "bf16"}


def _ref_case(dt, name, build, call, grad_inputs):
    from tests.golden_util import load
    dev = _dev()
    tol = REF_TOL[dt]
    fx = load(f"{PREFIX[dt]}_{name}", "manifest_half.json")
    m = build(fx["meta"]["cfg"])
    m.load_state_dict(fx["param"])
    m = m.to(dt).to(dev).eval()
    inp = {}
    for k, v in fx["in"].items():
        t = v.to(dev).to(dt) if v.is_floating_point() else v.to(dev)  # bf16 fixtures store fp32 (exact)
        inp[k] = t.requires_grad_(True) if k in grad_inputs else t
    out = call(m, inp, dt)
    assert out.dtype == dt
    errs = {"out": rel_err(out.float(), fx["out"].float())}
    (out * fx["gout"].to(dev)).sum().backward()
    for k in grad_inputs:
        errs["d" + k] = rel_err(inp[k].grad.float(), fx["grad_in"][k].float())
    gscale = max(float(g.float().abs().max()) for g in fx["grad_param"].values())
    named = dict(m.named_parameters())
    for k, g in fx["grad_param"].items():
        got = named[k].grad
        assert got is not None and got.dtype == dt, k
        errs["d" + k] = rel_err(got.float(), g.float())
        assert close(got.float().cpu(), g.float(), tol["grad"], gscale, tol["noise"]), (k, rel_err(got.float(), g.float()))
    print(PREFIX[dt], name, {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["out"] < tol["out"], errs
    for k in grad_inputs:
        assert errs["d" + k] < tol["grad"], errs


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_sca_stack_vs_reference_low_precision(dt):
    import scattennet_amd as S
    _ref_case(dt, "sca_L2", S.SeparativeCoordinateAttention,
              lambda m, i, dt: m(i["x_embed"], i["y_embed"], i["mask"]), ("x_embed", "y_embed"))


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
@pytest.mark.parametrize("kind", ["self_attn", "causal_attn"])
def test_coordinate_attention_vs_reference_low_precision(kind, dt):
    import scattennet_amd as S

    def call(m, i, dt):
        x = i["coord_embed"]
        if kind == "causal_attn":
            return m(x, S.create_causal_attention_mask(i["mask"], x.shape[:2], x))
        return m(x, S.create_attention_mask(i["mask"], dt))
    _ref_case(dt, "coordattn_" + kind, lambda cfg: S.CoordinateAttention(cfg, kind), call, ("coord_embed",))
