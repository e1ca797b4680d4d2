"""torch.library registrations of the core C-ABI ops ("the ops are
registered with torch.library plus autograd.Function").

The drop-in modules call the grouped autograd Functions in `ops` directly (one launch for
all keypoint streams); these registrations expose the same kernels as first-class torch
operators — schema, fake (meta) implementation for tracing, and autograd — so the path can
be composed with torch.compile / export and other torch code:

  torch.ops.scatten.masked_attention(q, k, v, key_valid, num_heads, causal, causal_plus_one)
      -> (o, row max, log2 row sum)   softmax(q k^T + mask) v per head; q is expected
                                pre-scaled (attention.py:53-72 after the q projection);
                                key_valid is the (B, Tk) 1/0 key-padding vector
                                (model/utils.py:3-28)
  torch.ops.scatten.layer_norm(x, weight, bias, eps) -> (y, mean, rstd)   (nn.LayerNorm)
  torch.ops.scatten.normalize_keypoints(kp, lengths, part_off, part_idx) -> kp'
                                SLR_Dataset.normalize_keypoints (dataset.py:134-170)

Every op runs on the HIP library only (no CPU kernel is registered: a CPU tensor raises).
"""
from typing import Optional

import torch
from torch import Tensor

from . import _lib as L
from . import ops

_LIB = "scatten"


# --------------------------------------------------------------------------- attention
@torch.library.custom_op(f"{_LIB}::masked_attention", mutates_args=())
def masked_attention(q: Tensor, k: Tensor, v: Tensor, key_valid: Optional[Tensor], num_heads: int,
                     causal: bool = False, causal_plus_one: bool = False) -> tuple[Tensor, Tensor, Tensor]:
    """-> (o, row max, log2 row sum): the statistics (base 2, per (clip, head, query)) are what
    the backward needs, as aten's attention ops return their logsumexp."""
    L.require_device(q, k, v)
    o, sm, sl = ops._attn_fwd(1, num_heads, causal, causal_plus_one, key_valid, None,
                              [q.contiguous()], [k.contiguous()], [v.contiguous()])
    return o[0], sm[0], sl[0]


@masked_attention.register_fake
def _(q, k, v, key_valid, num_heads, causal=False, causal_plus_one=False):
    B, Tq, _ = q.shape
    return torch.empty_like(q), q.new_empty(B * num_heads * Tq), q.new_empty(B * num_heads * Tq)


def _attn_setup(ctx, inputs, output):
    q, k, v, key_valid, num_heads, causal, plus_one = inputs
    o, sm, sl = output
    ctx.save_for_backward(q, k, v, o, sm, sl, key_valid)
    ctx.meta = (num_heads, causal, plus_one)
    ctx.mark_non_differentiable(sm, sl)


def _attn_backward(ctx, do, _dsm, _dsl):
    q, k, v, o, sm, sl, key_valid = ctx.saved_tensors
    num_heads, causal, plus_one = ctx.meta
    dq, dk, dv = ops._attn_bwd(1, num_heads, causal, plus_one, key_valid, None, [q.contiguous()],
                               [k.contiguous()], [v.contiguous()], [o], [sm], [sl], [do.contiguous()])
    return dq[0], dk[0], dv[0], None, None, None, None


masked_attention.register_autograd(_attn_backward, setup_context=_attn_setup)


# --------------------------------------------------------------------------- LayerNorm
@torch.library.custom_op(f"{_LIB}::layer_norm", mutates_args=())
def layer_norm(x: Tensor, weight: Tensor, bias: Tensor, eps: float = 1e-5) -> tuple[Tensor, Tensor, Tensor]:
    """-> (y, mean, rstd) over the last dimension, as aten.native_layer_norm."""
    L.require_device(x)
    x = x.contiguous()
    N = x.shape[-1]
    rows = x.numel() // N
    y = torch.empty_like(x)
    mean, rstd = x.new_empty(rows), x.new_empty(rows)
    arr = (L.LnFwdProblem * 1)(L.LnFwdProblem(x.data_ptr(), None, weight.data_ptr(), bias.data_ptr(), None,
                                              y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), 0, 0, 0.0))
    L.check(L.lib().sca_layernorm_fwd(1, arr, rows, N, max(rows, 1), 0, float(eps), L.stream_handle()),
            "sca_layernorm_fwd")
    return y, mean, rstd


@layer_norm.register_fake
def _(x, weight, bias, eps=1e-5):
    rows = x.numel() // x.shape[-1]
    return torch.empty_like(x), x.new_empty(rows), x.new_empty(rows)


def _ln_setup(ctx, inputs, output):
    x, weight, bias, eps = inputs
    _, mean, rstd = output
    ctx.save_for_backward(x, weight, mean, rstd)
    ctx.mark_non_differentiable(mean, rstd)


def _ln_backward(ctx, dy, _dm, _dr):
    x, weight, mean, rstd = ctx.saved_tensors
    dx, dg, db, _ = ops._ln_bwd([dy.contiguous()], [x.contiguous()], [weight], [mean], [rstd])
    return dx[0], dg[0], db[0], None


layer_norm.register_autograd(_ln_backward, setup_context=_ln_setup)


# --------------------------------------------------------------------------- input contract
@torch.library.custom_op(f"{_LIB}::normalize_keypoints", mutates_args=())
def normalize_keypoints(kp: Tensor, lengths: Tensor, part_off: Tensor, part_idx: Tensor) -> Tensor:
    L.require_device(kp)
    kp = kp.contiguous()
    B, T, K_all, _ = kp.shape
    out = torch.empty_like(kp)
    lens = lengths.to(torch.int32).contiguous()
    po, pi = part_off.to(torch.int32).contiguous(), part_idx.to(torch.int32).contiguous()
    L.check(L.lib().sca_normalize_parts(kp.data_ptr(), out.data_ptr(), lens.data_ptr(), B, T, K_all, po.data_ptr(),
                                        pi.data_ptr(), po.numel() - 1, L.stream_handle()), "sca_normalize_parts")
    return out


@normalize_keypoints.register_fake
def _(kp, lengths, part_off, part_idx):
    return torch.empty_like(kp)
