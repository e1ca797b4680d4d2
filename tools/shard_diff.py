"""Diagnostic: does the config-3 encoder compute a clip's forward identically at 8 and at 64
clips per launch?  Prints the max |difference| per stage (mapping + SCA + residual per
stream, then the fusion) between the full 64-clip batch and its first 8-clip shard.

    SCA_GEMM_LN_BM=32 python tools/shard_diff.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import keypoint_module as KM, workloads as W  # noqa: E402


def stages(enc, kp, mask):
    """Run the encoder recording the outputs of the grouped stages keypoint_streams_forward calls."""
    rec = {}
    saved = {}
    for name in ("coordinate_mapping_grouped", "sca_grouped", "residual_network_grouped"):
        fn = getattr(KM, name)
        saved[name] = fn

        def wrap(*a, _fn=fn, _name=name, **k):
            out = _fn(*a, **k)
            flat = out[0] if _name == "sca_grouped" else out
            if _name == "coordinate_mapping_grouped":
                flat = list(out[0]) + list(out[1])
            rec[_name] = [o.detach().clone() for o in flat]
            return out
        setattr(KM, name, wrap)
    try:
        with torch.no_grad():
            fuse, left, right, body = enc(kp, mask)
    finally:
        for name, fn in saved.items():
            setattr(KM, name, fn)
    rec.update(fuse=fuse, left=left, right=right, body=body)
    return rec


def main():
    dev = torch.device("cuda:0")
    w = dict(W.WORKLOADS["cfg3"], B=64)
    enc = W.build_encoder(w, dev, seed=8, init="random").eval()
    kp, mask, _ = W.synthetic_batch(w, dev, seed=12)
    full = stages(enc, kp, mask)
    part = stages(enc, kp[:8], mask[:8])
    torch.cuda.synchronize()
    for k in part:
        a, b = full[k], part[k]
        if isinstance(a, list):
            for i, (x, y) in enumerate(zip(a, b)):
                print(f"{k}[{i}]: max|diff| {float((x[:8] - y).abs().max()):.3e}  scale {float(y.abs().max()):.3e}")
        else:
            print(f"{k}: max|diff| {float((a[:8] - b).abs().max()):.3e}  scale {float(b.abs().max()):.3e}")


if __name__ == "__main__":
    main()


def calls(enc, kp, mask):
    """Outputs of every autograd Function of ops, in call order."""
    from scattennet_amd import ops
    rec = []
    saved = {}
    for cname in ("AttentionBlock", "LinearResidual", "FeedForwardResidual", "LayerNormAdd", "MaxPoolT",
                  "CoordinateMappingOp", "LinearGelu", "ClipMatmul", "SoftmaxRows"):
        cls = getattr(ops, cname)
        fwd = cls.forward
        saved[cname] = fwd

        def wrap(ctx, *a, _fwd=fwd, _n=cname):
            out = _fwd(ctx, *a)
            outs = out if isinstance(out, tuple) else (out,)
            rec.append((_n, [o.detach().clone() for o in outs if torch.is_tensor(o)]))
            return out
        cls.forward = staticmethod(wrap)
    try:
        with torch.no_grad():
            enc(kp, mask)
    finally:
        for cname, fwd in saved.items():
            getattr(ops, cname).forward = staticmethod(fwd)
    return rec


def first_divergence():
    dev = torch.device("cuda:0")
    w = dict(W.WORKLOADS["cfg3"], B=64)
    enc = W.build_encoder(w, dev, seed=8, init="random").eval()
    kp, mask, _ = W.synthetic_batch(w, dev, seed=12)
    full = calls(enc, kp, mask)
    part = calls(enc, kp[:8], mask[:8])
    for i, ((n1, o1), (n2, o2)) in enumerate(zip(full, part)):
        for j, (a, b) in enumerate(zip(o1, o2)):
            a8 = a.reshape(64, -1)[:8] if a.shape[0] == 64 or a.numel() % 64 == 0 else a
            b8 = b.reshape(8, -1)
            if a8.shape != b8.shape:
                continue
            d = float((a8 - b8).abs().max())
            if d != 0.0:
                print(f"call {i} {n1} output {j}: max|diff| {d:.3e}")
                return
    print("no divergence")


if __name__ == "__main__" and os.environ.get("SHARD_CALLS"):
    first_divergence()
