"""Loading helpers for the committed golden fixtures (tests/golden/*.npz)."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest(fname="manifest.json"):
    with open(os.path.join(GOLDEN, fname)) as f:
        return json.load(f)


def load(name, manifest_name="manifest.json"):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))  # allow_pickle=False (default)
    fx = {"in": {}, "param": {}, "grad_in": {}, "grad_param": {}}
    for k in z.files:
        v = torch.from_numpy(z[k].copy())
        if k.startswith("in."):
            fx["in"][k[3:]] = v
        elif k.startswith("param."):
            fx["param"][k[6:]] = v
        elif k.startswith("grad.in."):
            fx["grad_in"][k[8:]] = v
        elif k.startswith("grad.param."):
            fx["grad_param"][k[11:]] = v
        else:
            fx[k] = v
    fx["meta"] = manifest(manifest_name)["fixtures"][name]
    return fx


def rel_err(a, b):
    """max |a-b| / max(|b|, floor) — the 'relative fp32' metric used by every parity test."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    scale = b.abs().max().clamp_min(1e-6)
    return float((a - b).abs().max() / scale)


def close(a, b, tol, gscale=None, noise=1e-4):
    """Parity predicate.  `rel_err(a, b) < tol`, except for tensors that are analytically
    zero in the reference (e.g. the key-projection bias gradient: softmax is invariant to
    a per-row constant, so d/d(bk) is pure rounding noise): when |b| is below 1e-4 of the
    fixture's gradient scale `gscale`, both sides only have to be noise-level (< 1e-4 gscale;
    `noise`: that fraction for reduced-precision fixtures, whose rounding noise is larger)."""
    if gscale is not None:
        bmax = float(b.detach().abs().max()) if b.numel() else 0.0
        if bmax < noise * gscale:
            amax = float(a.detach().abs().max()) if a.numel() else 0.0
            return amax < noise * gscale
    return rel_err(a, b) < tol
