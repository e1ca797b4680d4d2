"""Generate golden input/output/gradient vectors from the REFERENCE implementation.

Runs ONLY in the survey/build container, where `/root/reference` (tinh2044/SCAttenNet,
snapshot 2025-07-18) is importable.  The reference never travels to the GPU box: the
outputs of this script are committed as small `.npz` fixtures (data only — inputs,
parameters, outputs and gradients) plus `manifest.json`.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Every fixture is fp32, eval mode (dropout off), fixed seed, and uses ragged key-padding
masks with lengths {T, T-37 (or T-5 for short T), T/2, 1, 0} so that the full / ragged /
length-1 / fully-padded cases of `model/utils.py:3-28` are covered.
Loss for the backward pass: `(out * G).sum()` with `G ~ N(0,1)` drawn from seed 1.
"""
import json
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)

from model.attention import CrossAttention, SelfAttention, SelfCausalAttention  # noqa: E402
from model.fusion import CoordinatesFusion  # noqa: E402
from model.keypoint_module import (  # noqa: E402
    CoordinateAttention,
    CoordinatesMerge,
    KeypointModule,
    SeparativeCoordinateAttention,
)
from model.layers import CoordinateMapping  # noqa: E402
from model.residual import ResidualNetwork  # noqa: E402
from model.utils import create_attention_mask, create_causal_attention_mask  # noqa: E402


def lengths_for(B, T):
    base = [T, max(T - 37, 1) if T > 40 else max(T - 5, 1), T // 2, 1, 0]
    return base[:B]


def key_mask(B, T):
    m = torch.zeros(B, T, dtype=torch.long)
    for b, n in enumerate(lengths_for(B, T)):
        m[b, :n] = 1
    return m


def randomize_params(module, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            if isinstance(p, torch.nn.Parameter) and p.dim() == 2 and "embed" not in name:
                fan_in = p.shape[1]
                p.copy_(torch.randn(p.shape, generator=g) / np.sqrt(fan_in))
            elif "embed" in name:
                p.copy_(torch.randn(p.shape, generator=g))
            elif name.endswith("weight"):  # LayerNorm gamma
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=g))
            else:  # biases / LayerNorm beta
                p.copy_(0.1 * torch.randn(p.shape, generator=g))


def capture(name, module, inputs, call, meta, grad_inputs=()):
    """Run fwd+bwd through the reference `module` and store everything in one npz."""
    module.eval()
    for k in grad_inputs:
        inputs[k] = inputs[k].detach().clone().requires_grad_(True)
    out = call(module, inputs)
    g = torch.Generator().manual_seed(1)
    G = torch.randn(out.shape, generator=g)
    module.zero_grad(set_to_none=True)
    (out * G).sum().backward()
    arrs = {}
    for k, v in inputs.items():
        arrs["in." + k] = v.detach().numpy()
    for k, v in module.state_dict().items():
        arrs["param." + k] = v.detach().numpy()
    arrs["out"] = out.detach().numpy()
    arrs["gout"] = G.numpy()
    for k in grad_inputs:
        arrs["grad.in." + k] = inputs[k].grad.numpy()
    for k, p in module.named_parameters():
        if p.grad is not None:
            arrs["grad.param." + k] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
    meta = dict(meta)
    meta["out_shape"] = list(out.shape)
    return name, meta


def main():
    torch.set_num_threads(1)
    manifest = {"torch": torch.__version__, "reference": "tinh2044/SCAttenNet @ 2025-07-18",
                "loss": "(out*G).sum(), G~N(0,1) seed 1", "fixtures": {}}

    def add(res):
        manifest["fixtures"][res[0]] = res[1]

    # ---- A5/A6/A7: the three attention operators (model/attention.py) -----------------
    for (B, T, d, H) in [(5, 64, 64, 4), (5, 48, 128, 4)]:
        tag = f"B{B}_T{T}_d{d}_H{H}"
        mask = key_mask(B, T)
        for cls, kind in [(SelfAttention, "self"), (SelfCausalAttention, "causal"), (CrossAttention, "cross")]:
            torch.manual_seed(0)
            m = cls(d, H)
            randomize_params(m, 10)
            x = torch.randn(B, T, d)
            inp = {"hidden_states": x, "mask": mask}
            if kind == "cross":
                inp["key_value_states"] = torch.randn(B, T, d)
                call = lambda mod, i: mod(i["hidden_states"], i["key_value_states"],
                                          create_attention_mask(i["mask"], torch.float32))
                gi = ("hidden_states", "key_value_states")
            elif kind == "causal":
                call = lambda mod, i: mod(i["hidden_states"], create_causal_attention_mask(
                    i["mask"], i["hidden_states"].shape[:2], i["hidden_states"]))
                gi = ("hidden_states",)
            else:
                call = lambda mod, i: mod(i["hidden_states"], create_attention_mask(i["mask"], torch.float32))
                gi = ("hidden_states",)
            add(capture(f"attn_{kind}_{tag}", m, inp, call,
                        {"op": cls.__name__, "B": B, "T": T, "d": d, "H": H,
                         "lengths": lengths_for(B, T), "ref": "model/attention.py"}, gi))

    cfg64 = {"d_model": 64, "attention_heads": 4, "attention_dropout": 0.0, "dropout": 0.2,
             "ff_dim": 192, "attn_layers": 2, "max_position_embeddings": 64,
             "residual_blocks": [64, 64, 128, 128]}
    B, T = 5, 48
    mask = key_mask(B, T)

    # ---- A9: CoordinateAttention (self / causal), A10: CoordinatesMerge -----------------
    for kind in ["self_attn", "causal_attn"]:
        torch.manual_seed(0)
        m = CoordinateAttention(cfg64, kind)
        randomize_params(m, 11)
        inp = {"coord_embed": torch.randn(B, T, 64), "mask": mask}
        if kind == "self_attn":
            call = lambda mod, i: mod(i["coord_embed"], create_attention_mask(i["mask"], torch.float32))
        else:
            call = lambda mod, i: mod(i["coord_embed"], create_causal_attention_mask(
                i["mask"], i["coord_embed"].shape[:2], i["coord_embed"]))
        add(capture(f"coordattn_{kind}", m, inp, call,
                    {"op": "CoordinateAttention", "attn_type": kind, "cfg": cfg64, "B": B, "T": T,
                     "ref": "model/keypoint_module.py:34-80"}, ("coord_embed",)))
    torch.manual_seed(0)
    m = CoordinatesMerge(cfg64)
    randomize_params(m, 12)
    inp = {"y_embed": torch.randn(B, T, 64), "x_embed": torch.randn(B, T, 64), "mask": mask}
    add(capture("coordmerge", m, inp,
                lambda mod, i: mod(i["y_embed"], i["x_embed"],
                                   create_attention_mask(i["mask"], torch.float32)),
                {"op": "CoordinatesMerge", "cfg": cfg64, "B": B, "T": T,
                 "ref": "model/keypoint_module.py:83-115"}, ("y_embed", "x_embed")))

    # ---- A11: SeparativeCoordinateAttention stack (L=2) ---------------------------------
    torch.manual_seed(0)
    m = SeparativeCoordinateAttention(cfg64)
    randomize_params(m, 13)
    inp = {"x_embed": torch.randn(B, T, 64), "y_embed": torch.randn(B, T, 64), "mask": mask}
    add(capture("sca_L2", m, inp, lambda mod, i: mod(i["x_embed"], i["y_embed"], i["mask"]),
                {"op": "SeparativeCoordinateAttention", "cfg": cfg64, "B": B, "T": T,
                 "ref": "model/keypoint_module.py:118-198"}, ("x_embed", "y_embed")))

    # ---- A2: CoordinateMapping -----------------------------------------------------------
    torch.manual_seed(0)
    m = CoordinateMapping(21, 64)
    randomize_params(m, 14)
    inp = {"x_coord": torch.rand(B, T, 21), "y_coord": torch.rand(B, T, 21)}
    add(capture("coordmap", m, inp,
                lambda mod, i: torch.cat(mod(i["x_coord"], i["y_coord"]), dim=-1),
                {"op": "CoordinateMapping", "K": 21, "d": 64, "B": B, "T": T,
                 "ref": "model/layers.py:111-123", "note": "out = cat(x_embed, y_embed, -1)"},
                ("x_coord", "y_coord")))

    # ---- A1..A12: KeypointModule (mapping + SCA + residual) -------------------------------
    torch.manual_seed(0)
    joint_idx = list(range(3, 24))
    m = KeypointModule(joint_idx, T, dict(cfg64, attn_layers=1))
    randomize_params(m, 15)
    inp = {"keypoints": torch.rand(B, T, 21, 2), "mask": mask}
    add(capture("keypoint_module", m, inp, lambda mod, i: mod(i["keypoints"], i["mask"]),
                {"op": "KeypointModule", "cfg": dict(cfg64, attn_layers=1), "K": 21, "B": B, "T": T,
                 "ref": "model/keypoint_module.py:13-31"}, ("keypoints",)))

    # ---- A12: ResidualNetwork ------------------------------------------------------------
    for blocks in ([64, 64, 128, 128], [64, 64]):
        torch.manual_seed(0)
        m = ResidualNetwork(blocks)
        randomize_params(m, 16)
        inp = {"x": torch.randn(B, T, 64)}
        add(capture("residual_" + "_".join(map(str, blocks)), m, inp, lambda mod, i: mod(i["x"])[0],
                    {"op": "ResidualNetwork", "blocks": blocks, "B": B, "T": T,
                     "ref": "model/residual.py:48-118"}, ("x",)))

    # ---- A13: CoordinatesFusion ----------------------------------------------------------
    torch.manual_seed(0)
    m = CoordinatesFusion(32, 64, 0.2)
    randomize_params(m, 17)
    inp = {"left": torch.randn(2, 16, 32), "right": torch.randn(2, 16, 32), "body": torch.randn(2, 16, 32)}
    add(capture("fusion", m, inp, lambda mod, i: mod(i["left"], i["right"], i["body"]),
                {"op": "CoordinatesFusion", "in": 32, "out": 64, "B": 2, "T": 16,
                 "ref": "model/fusion.py:6-78"}, ("left", "right", "body")))

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(manifest["fixtures"]), "fixtures")


if __name__ == "__main__":
    main()
