"""Pin the CPU oracle (oracle/sca_oracle.py) to the reference's own outputs.

The golden vectors were captured from the reference implementation (tests/golden/gen_golden.py);
this test proves the restatement reproduces them (outputs AND gradients) before the oracle
is trusted as the checker for the HIP path at larger sizes.  CPU only.
"""
import pytest
import torch

from oracle import sca_oracle as O
from tests.golden_util import close, load, manifest, rel_err

TOL = 2e-5  # fp32 CPU vs fp32 CPU: only summation-order differences


def _run(name, fn, grad_inputs, manifest_name="manifest.json", tol=(TOL, TOL, 1e-4)):
    fx = load(name, manifest_name)
    f32 = lambda v: v.float() if v.is_floating_point() else v  # noqa: E731  (fp16 fixtures: fp32 oracle)
    params = {k: f32(v).clone().requires_grad_(True) for k, v in fx["param"].items() if v.is_floating_point()}
    inputs = {k: (f32(v).clone().requires_grad_(True) if k in grad_inputs else v) for k, v in fx["in"].items()}
    out = fn(params, inputs, fx["meta"])
    assert rel_err(out, fx["out"].float()) < tol[0]
    (out * fx["gout"]).sum().backward()
    for k in grad_inputs:
        assert rel_err(inputs[k].grad, fx["grad_in"][k].float()) < tol[1], k
    gscale = max(float(g.float().abs().max()) for g in fx["grad_param"].values())
    for k, g in fx["grad_param"].items():
        got = params[k].grad
        assert got is not None, k
        assert close(got, g.float(), tol[1], gscale, tol[2]), (k, rel_err(got, g.float()))
    # parameters the reference leaves without gradient must stay without gradient here
    for k, p in params.items():
        if k not in fx["grad_param"]:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k


ATTN = [n for n in manifest()["fixtures"] if n.startswith("attn_")]


@pytest.mark.parametrize("name", ATTN)
def test_attention_ops(name):
    kind = name.split("_")[1]
    H = manifest()["fixtures"][name]["H"]

    def fn(p, i, meta):
        x = i["hidden_states"]
        if kind == "cross":
            return O.attention(p, "", x, i["key_value_states"], O.additive_key_mask(i["mask"]), H, "cross")
        m = O.additive_causal_mask(i["mask"]) if kind == "causal" else O.additive_key_mask(i["mask"])
        return O.attention(p, "", x, x, m, H, kind)

    # prefix "" -> keys like ".q_proj.weight"; strip the leading dot
    def fn2(p, i, meta):
        p2 = {"." + k: v for k, v in p.items()}
        return fn(p2, i, meta)

    gi = ("hidden_states", "key_value_states") if kind == "cross" else ("hidden_states",)
    _run(name, fn2, gi)


@pytest.mark.parametrize("kind", ["self_attn", "causal_attn"])
def test_coordinate_attention(kind):
    def fn(p, i, meta):
        m = O.additive_key_mask(i["mask"]) if kind == "self_attn" else O.additive_causal_mask(i["mask"])
        return O.coordinate_attention(p, "", i["coord_embed"], m, meta["cfg"]["attention_heads"], kind)

    _run("coordattn_" + kind, fn, ("coord_embed",))


def test_coordinates_merge():
    def fn(p, i, meta):
        return O.coordinates_merge(p, "", i["y_embed"], i["x_embed"], O.additive_key_mask(i["mask"]),
                                   meta["cfg"]["attention_heads"])

    _run("coordmerge", fn, ("y_embed", "x_embed"))


def test_sca_stack():
    _run("sca_L2", lambda p, i, m: O.sca(p, "", i["x_embed"], i["y_embed"], i["mask"], m["cfg"]),
         ("x_embed", "y_embed"))


def test_coordinate_mapping():
    _run("coordmap", lambda p, i, m: torch.cat(O.coordinate_mapping(p, "", i["x_coord"], i["y_coord"]), -1),
         ("x_coord", "y_coord"))


def test_keypoint_module():
    _run("keypoint_module", lambda p, i, m: O.keypoint_module(p, "", i["keypoints"], i["mask"], m["cfg"]),
         ("keypoints",))


@pytest.mark.parametrize("name", ["residual_64_64_128_128", "residual_64_64", "residual_64_64_T45"])
def test_residual_network(name):
    _run(name, lambda p, i, m: O.residual_network(p, "", i["x"], m["blocks"]), ("x",))


@pytest.mark.parametrize("name", ["fusion", "fusion_T45", "fusion_T13"])
def test_fusion(name):
    _run(name, lambda p, i, m: O.coordinates_fusion(p, "", i["left"], i["right"], i["body"]),
         ("left", "right", "body"))


def test_position_table_overflow_raises():
    p = {"t": torch.zeros(6, 4)}
    with pytest.raises(IndexError):
        O.position_embed(p, "t", torch.zeros(1, 5, 4))


def test_xstream_cfg1():
    """BASELINE config 1's x-coordinate stream (the CPU baseline's config-1 workload)."""
    _run("xstream_cfg1", lambda p, i, m: O.x_stream(p, "", i["keypoints"], i["mask"], m["cfg"]), ("keypoints",))


# the reference computing in float16 / bfloat16 (tests/golden/gen_golden_half.py) against the
# fp32 oracle on the same (reduced-precision-valued) parameters and inputs: the rounding of
# every intermediate only — the tolerances the GPU modules are held to (tests/test_gpu_precision.py)
LOW = {"half": (4e-3, 6e-3, 1e-4), "bf16": (3e-2, 4e-2, 2e-3)}  # (outputs, gradients, noise floor)


@pytest.mark.parametrize("pre", ["half", "bf16"])
def test_sca_stack_low_precision_fixture(pre):
    _run(f"{pre}_sca_L2", lambda p, i, m: O.sca(p, "", i["x_embed"], i["y_embed"], i["mask"], m["cfg"]),
         ("x_embed", "y_embed"), "manifest_half.json", LOW[pre])


@pytest.mark.parametrize("pre", ["half", "bf16"])
@pytest.mark.parametrize("kind", ["self_attn", "causal_attn"])
def test_coordinate_attention_low_precision_fixture(kind, pre):
    def fn(p, i, meta):
        m = O.additive_key_mask(i["mask"]) if kind == "self_attn" else O.additive_causal_mask(i["mask"])
        return O.coordinate_attention(p, "", i["coord_embed"], m, meta["cfg"]["attention_heads"], kind)

    _run(f"{pre}_coordattn_" + kind, fn, ("coord_embed",), "manifest_half.json", LOW[pre])
