"""fp16 / bf16 golden vectors from the REFERENCE: its SeparativeCoordinateAttention stack (L = 2)
and CoordinateAttention blocks run in float16 (and bfloat16) arithmetic on the CPU
(`module.half()` / `.to(torch.bfloat16)`, inputs of that dtype, the reference's own masks of
that dtype and its fp16 overflow clamp, model/keypoint_module.py:74-78), forward and backward.  Pins the drop-in modules' `.half()` behaviour (tests/test_gpu_precision.py), which
computes in fp32 on fp32 views and rounds to fp16 at the module boundary: the two differ by
the reference's fp16 rounding inside the block, hence a tolerance of a few fp16 ulps of the
output scale instead of the fp32 1e-3.

Runs ONLY in the build container (`/root/reference` importable); writes `half_*.npz` and
`bf16_*.npz` (data only) and their entries in `manifest_half.json`.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_half.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (puts /root/reference on sys.path)
from model.keypoint_module import CoordinateAttention, SeparativeCoordinateAttention  # noqa: E402
from model.utils import create_attention_mask, create_causal_attention_mask  # noqa: E402


def capture(name, module, inputs, call, meta, grad_inputs=()):
    """gen_golden.capture for reduced-precision modules: bfloat16 arrays are stored as float32
    (exact: bf16 values are fp32 values; numpy has no bf16), float16 as float16."""
    np_ = lambda t: (t.float() if t.dtype == torch.bfloat16 else t).detach().numpy()  # noqa: E731
    module.eval()
    for k in grad_inputs:
        inputs[k] = inputs[k].detach().clone().requires_grad_(True)
    out = call(module, inputs)
    Gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(1))
    module.zero_grad(set_to_none=True)
    (out * Gout).sum().backward()
    arrs = {"in." + k: np_(v) for k, v in inputs.items()}
    arrs.update({"param." + k: np_(v) for k, v in module.state_dict().items()})
    arrs["out"], arrs["gout"] = np_(out), Gout.numpy()
    arrs.update({"grad.in." + k: np_(inputs[k].grad) for k in grad_inputs})
    arrs.update({"grad.param." + k: np_(p.grad) for k, p in module.named_parameters() if p.grad is not None})
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
    return name, dict(meta, out_shape=list(out.shape), dtype=str(out.dtype))


def main():
    torch.set_num_threads(4)
    cfg = {"d_model": 64, "attention_heads": 4, "attention_dropout": 0.0, "dropout": 0.2, "ff_dim": 192,
           "attn_layers": 2, "max_position_embeddings": 64}
    B, T = 5, 48
    mask = G.key_mask(B, T)
    manifest = {"torch": torch.__version__, "reference": "tinh2044/SCAttenNet @ 2025-07-18", "dtype": "float16 (half_*) / bfloat16 (bf16_*)",
                "fixtures": {}}

    def add(res):
        manifest["fixtures"][res[0]] = res[1]

    for dt, pre in ((torch.float16, "half"), (torch.bfloat16, "bf16")):
        torch.manual_seed(0)
        m = SeparativeCoordinateAttention(cfg)
        G.randomize_params(m, 13)
        m = m.to(dt)
        inp = {"x_embed": torch.randn(B, T, 64).to(dt), "y_embed": torch.randn(B, T, 64).to(dt), "mask": mask}
        add(capture(f"{pre}_sca_L2", m, inp, lambda mod, i: mod(i["x_embed"], i["y_embed"], i["mask"]),
                      {"op": f"SeparativeCoordinateAttention ({dt})", "cfg": cfg, "B": B, "T": T,
                       "ref": "model/keypoint_module.py:118-198"}, ("x_embed", "y_embed")))
        # the blocks with the reference's materialised masks of the dtype, 4 clips (lengths 48,
        # 11, 24, 1): a fully padded clip is left out — there the reference's fp16
        # s + finfo(fp16).min rounds the scores to multiples of 32 (near-uniform weights picked
        # by rounding), which neither its fp32 semantics (exactly uniform) nor the
        # fp32-computing drop-in reproduce
        B4 = 4
        for seed, kind in ((10, "self_attn"), (11, "causal_attn")):
            torch.manual_seed(0)
            m = CoordinateAttention(cfg, kind)
            G.randomize_params(m, seed)
            m = m.to(dt)
            inp = {"coord_embed": torch.randn(B4, T, 64).to(dt), "mask": G.key_mask(B4, T)}
            if kind == "causal_attn":
                def call(mod, i):
                    x = i["coord_embed"]
                    return mod(x, create_causal_attention_mask(i["mask"], x.shape[:2], x))
            else:
                def call(mod, i, dt=dt):
                    return mod(i["coord_embed"], create_attention_mask(i["mask"], dt))
            add(capture(f"{pre}_coordattn_{kind}", m, inp, call,
                          {"op": f"CoordinateAttention ({dt})", "attn_type": kind, "cfg": cfg, "B": B4, "T": T,
                           "ref": "model/keypoint_module.py:34-80"}, ("coord_embed",)))
    with open(os.path.join(HERE, "manifest_half.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", sorted(manifest["fixtures"]))


if __name__ == "__main__":
    main()
