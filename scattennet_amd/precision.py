"""fp16 / bf16 modules: what `model.half()` / `model.to(torch.bfloat16)` gives a user of the
reference (model/keypoint_module.py:74-78, 109-113: the float16 clamp after each post-LN block).

The HIP kernels compute in fp32 (north_star's precision; the matrix cores' fp32 MFMA).  A module
whose parameters (or, with no parameters, whose floating inputs) are fp16 / bf16 runs its forward
on fp32 views of its parameters and inputs — `torch.func.functional_call` with `p.float()` for
every parameter, so autograd casts the gradients back to the parameters' dtype — and returns its
floating outputs in the module's dtype.  The blocks the reference clamps (CoordinateAttention,
CoordinatesMerge) apply the same clamp to their fp16 output: when any element is inf / NaN, the
whole tensor is clamped to +-(finfo(float16).max - 1000).

Storage is the module's dtype; arithmetic is fp32, so results match the fp32 path on the rounded
parameters up to the final rounding (tests/test_gpu_precision.py), and the reference's fp16
overflow cases (an intermediate block overflowing fp16) do not arise inside a block.
"""
import functools

import torch
from torch.func import functional_call

_LOW = (torch.float16, torch.bfloat16)


def _low_dtype(module, args, kwargs):
    """The module's reduced dtype, or None when it is an fp32 module."""
    for p in module.parameters():
        if p.is_floating_point():
            return p.dtype if p.dtype in _LOW else None
    for a in list(args) + list(kwargs.values()):
        if torch.is_tensor(a) and a.is_floating_point():
            return a.dtype if a.dtype in _LOW else None
    return None


def _cast(x, src, dst):
    """Floating tensors of a dtype in `src` -> `dst`, through tuples / lists / dicts."""
    if torch.is_tensor(x):
        return x.to(dst) if x.dtype in src else x
    if isinstance(x, (tuple, list)):
        return type(x)(_cast(v, src, dst) for v in x)
    if isinstance(x, dict):
        return {k: _cast(v, src, dst) for k, v in x.items()}
    return x


def fp16_clamp(t):
    """model/keypoint_module.py:74-78 on one tensor."""
    if torch.is_tensor(t) and t.dtype == torch.float16 and (torch.isinf(t).any() or torch.isnan(t).any()):
        cv = torch.finfo(torch.float16).max - 1000
        t = torch.clamp(t, min=-cv, max=cv)
    return t


def fp32_compute(clamp=False):
    """Decorator for an nn.Module forward: fp32 modules run it unchanged; fp16 / bf16 modules run
    it on fp32 parameter / input views and get their floating outputs back in their dtype."""
    def deco(fwd):
        @functools.wraps(fwd)
        def wrapper(self, *args, **kwargs):
            dt = _low_dtype(self, args, kwargs)
            if dt is None:
                return fwd(self, *args, **kwargs)
            state = {n: p.float() if p.is_floating_point() else p for n, p in self.named_parameters()}
            state.update({n: b.float() if b.is_floating_point() else b for n, b in self.named_buffers()})
            out = functional_call(self, state, _cast(tuple(args), _LOW, torch.float32),
                                  _cast(dict(kwargs), _LOW, torch.float32))
            out = _cast(out, (torch.float32,), dt)
            if clamp:
                out = fp16_clamp(out)
            return out
        return wrapper
    return deco
