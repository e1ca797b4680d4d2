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
    B, Tq, d = q.shape
    if d // num_heads > 128:  # the GEMM path keeps P (B, H, Tq, Tk) instead of the row statistics
        return torch.empty_like(q), q.new_empty(B * num_heads * Tq * k.shape[1]), q.new_empty(0)
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


# =========================================================================== drop-in blocks
# The drop-in modules' operators, one keypoint stream per call: the grouped
# autograd Functions of `ops` run unchanged at G = 1 in library mode (no cross-op hand-offs,
# no side streams), driven through a stand-in context.  Each forward operator returns its
# output(s) followed by the intermediates its backward needs (marked non-differentiable);
# each backward is an operator of its own, so the pair composes with torch.compile /
# torch.export (FakeTensor shapes from the register_fake functions).  The modules route
# through these operators while torch.compile traces them (`compiling()`), and through the
# grouped launches otherwise.  Dropout must be off (p = 0 or eval) on this path.
from typing import List


class _Ctx:
    """Stand-in autograd context: the Functions only stash attributes and saved tensors."""

    def save_for_backward(self, *ts):
        self.saved_tensors = ts


def compiling():
    return torch.compiler.is_compiling()


def _opt(t):
    return [] if t is None else [t]


# --------------------------------------------------------------------------- attention block
@torch.library.custom_op(f"{_LIB}::attention_block", mutates_args=())
def attention_block(xq: Tensor, xkv: Optional[Tensor], params: List[Tensor], ln_weight: Optional[Tensor],
                    ln_bias: Optional[Tensor], key_valid: Optional[Tensor], add_mask: Optional[Tensor], kind: str,
                    num_heads: int, scale: float, plus_one: bool, resid: bool, ln_eps: float) -> List[Tensor]:
    """ops.AttentionBlock for one stream (model/attention.py:46-182 + the post-LN block's
    residual / LayerNorm, keypoint_module.py:61-72, 97-107).  params = [Wq, bq, Wk, bk, Wv,
    bv, Wo, bo]; kind "self" / "causal" / "cross" (xkv); ln_eps < 0: no LayerNorm.
    -> [y, q, k, v, o, row max, log2 row sum] (+ [v_pre, mean, rstd] with the LayerNorm)."""
    L.require_device(xq)
    ln = ln_eps >= 0
    d = xq.shape[-1]
    fused = ln and ops.ln_fusable(d, d)  # else: the LayerNorm as its own launch, same outputs
    ctx = _Ctx()
    ts = [xq] + _opt(xkv if kind == "cross" else None) + list(params) + ([ln_weight, ln_bias] if fused else [])
    with ops.library_mode():
        (y,) = ops.AttentionBlock.forward(ctx, 1, kind, num_heads, scale, plus_one, key_valid, add_mask, resid, 0.0,
                                          ln_eps if fused else None, None, 0.0, *ts)
        sv = ctx.saved_tensors
        i = 2 + 1 + (1 if kind == "cross" else 0) + 8
        inter = list(sv[i:i + 6])
        if fused:
            inter += [sv[i + 6], sv[i + 8], sv[i + 9]]  # v_pre, mean, rstd (gamma is an input)
        elif ln:
            v_pre = y
            y, mean, rstd = _ln_plain_fwd(v_pre, ln_weight, ln_bias, ln_eps)
            inter += [v_pre, mean, rstd]
    return [y] + inter


def _ln_plain_fwd(x, weight, bias, eps):
    ctx = _Ctx()
    (y,) = ops.LayerNormAdd.forward(ctx, 1, eps, False, False, 0, 0.0, x, weight, bias)
    return y, ctx.saved_tensors[2], ctx.saved_tensors[3]


def _ln_plain_bwd(dy, x, weight, bias, mean, rstd):
    ctx = _Ctx()
    N = x.shape[-1]
    ctx.G, ctx.pos, ctx.has_post, ctx.act = 1, False, False, 0
    ctx.r_mod, ctx.r_off = max(x.numel() // N, 1), 0
    ctx.drop_p, ctx.seeds, ctx.bet, ctx.lnsaved = 0.0, [0], (bias,), None
    ctx.saved_tensors = (x, weight, mean, rstd)
    g = ops.LayerNormAdd.backward(ctx, dy.contiguous())
    return g[6], g[7], g[8]  # dx, dgamma, dbeta


@attention_block.register_fake
def _(xq, xkv, params, ln_weight, ln_bias, key_valid, add_mask, kind, num_heads, scale, plus_one, resid, ln_eps):
    B, T, d = xq.shape
    kvs = xkv if kind == "cross" else xq
    Tk = kvs.shape[1]
    out = [torch.empty_like(xq), torch.empty_like(xq), kvs.new_empty(B, Tk, d), kvs.new_empty(B, Tk, d),
           torch.empty_like(xq), xq.new_empty(B * num_heads * T), xq.new_empty(B * num_heads * T)]
    if ln_eps >= 0:
        out += [torch.empty_like(xq), xq.new_empty(B * T), xq.new_empty(B * T)]
    return out


@torch.library.custom_op(f"{_LIB}::attention_block_backward", mutates_args=())
def attention_block_backward(dy: Tensor, xq: Tensor, xkv: Optional[Tensor], params: List[Tensor],
                             ln_weight: Optional[Tensor], ln_bias: Optional[Tensor], key_valid: Optional[Tensor],
                             add_mask: Optional[Tensor], saved: List[Tensor], kind: str, num_heads: int, scale: float,
                             plus_one: bool, resid: bool, ln_eps: float) -> List[Tensor]:
    """-> [dxq, (dxkv,) dWq, dbq, dWk, dbk, dWv, dbv, dWo, dbo (, dgamma, dbeta)]."""
    ln = ln_eps >= 0
    d = xq.shape[-1]
    fused = ln and ops.ln_fusable(d, d)
    cross = kind == "cross"
    ctx = _Ctx()
    ctx.G, ctx.kind, ctx.H, ctx.scale, ctx.plus_one, ctx.has_resid = 1, kind, num_heads, scale, plus_one, resid
    ctx.attn_drop, ctx.drop_p, ctx.seeds, ctx.ln = None, 0.0, [None], fused
    ctx.bet = (ln_bias,) if fused else ()
    ctx.lnsaved = ctx.lnprev = None
    sv = [key_valid, add_mask, xq] + _opt(xkv if cross else None) + list(params) + list(saved[:6])
    if fused:
        sv += [saved[6], ln_weight, saved[7], saved[8]]
    ctx.saved_tensors = tuple(sv)
    with ops.library_mode():
        dln = []
        if ln and not fused:
            dy, dg, db = _ln_plain_bwd(dy, saved[6], ln_weight, ln_bias, saved[7], saved[8])
            dln = [dg, db]
        g = ops.AttentionBlock.backward(ctx, dy.contiguous())
    return [t for t in g[12:] if t is not None] + dln


@attention_block_backward.register_fake
def _(dy, xq, xkv, params, ln_weight, ln_bias, key_valid, add_mask, saved, kind, num_heads, scale, plus_one, resid,
      ln_eps):
    out = [torch.empty_like(xq)] + ([torch.empty_like(xkv)] if kind == "cross" else [])
    out += [torch.empty_like(p) for p in params]
    if ln_eps >= 0:
        out += [torch.empty_like(ln_weight), torch.empty_like(ln_bias)]
    return out


def _attention_block_setup(ctx, inputs, output):
    xq, xkv, params, ln_weight, ln_bias, key_valid, add_mask, kind, num_heads, scale, plus_one, resid, ln_eps = inputs
    ctx.save_for_backward(xq, xkv, ln_weight, ln_bias, key_valid, add_mask, *params, *output[1:])
    ctx.meta = (kind, num_heads, scale, plus_one, resid, ln_eps, len(params))
    ctx.mark_non_differentiable(*output[1:])


def _attention_block_bwd(ctx, grads):
    kind, num_heads, scale, plus_one, resid, ln_eps, npar = ctx.meta
    sv = ctx.saved_tensors
    xq, xkv, ln_weight, ln_bias, key_valid, add_mask = sv[:6]
    params, saved = list(sv[6:6 + npar]), list(sv[6 + npar:])
    dy = grads[0] if grads[0] is not None else torch.zeros_like(xq)
    g = attention_block_backward(dy, xq, xkv, params, ln_weight, ln_bias, key_valid, add_mask, saved, kind,
                                 num_heads, scale, plus_one, resid, ln_eps)
    cross = kind == "cross"
    dxq, i = g[0], 1
    dxkv = g[1] if cross else None
    i += 1 if cross else 0
    dparams = list(g[i:i + npar])
    dln_w, dln_b = (g[i + npar], g[i + npar + 1]) if ln_eps >= 0 else (None, None)
    return dxq, dxkv, dparams, dln_w, dln_b, None, None, None, None, None, None, None, None


attention_block.register_autograd(_attention_block_bwd, setup_context=_attention_block_setup)


# --------------------------------------------------------------------------- feed-forward block
@torch.library.custom_op(f"{_LIB}::feed_forward", mutates_args=())
def feed_forward(x: Tensor, params: List[Tensor], ln_weight: Optional[Tensor], ln_bias: Optional[Tensor],
                 resid: bool, ln_eps: float) -> List[Tensor]:
    """ops.FeedForwardResidual for one stream: y = fc2(GELU(fc1 x)) (+ x) (+ post-LN),
    layers.py:94-108 / keypoint_module.py:71-72.  params = [W1, b1, W2, b2].
    -> [y, z (fc1 pre-activation), GELU(z)] (+ [v_pre, mean, rstd])."""
    L.require_device(x)
    ln = ln_eps >= 0
    fused = ln and ops.ln_fusable(x.shape[-1], params[2].shape[1])
    ctx = _Ctx()
    with ops.library_mode():
        (y,) = ops.FeedForwardResidual.forward(ctx, 1, resid, 0.0, ln_eps if fused else None, None, x, *params,
                                               *([ln_weight, ln_bias] if fused else []))
        sv = ctx.saved_tensors  # x, W1, W2, z, act (, v_pre, gamma, mean, rstd)
        extra = [sv[5], sv[7], sv[8]] if fused else []
        if ln and not fused:
            v_pre = y
            y, mean, rstd = _ln_plain_fwd(v_pre, ln_weight, ln_bias, ln_eps)
            extra = [v_pre, mean, rstd]
    return [y, sv[3], sv[4]] + extra


@feed_forward.register_fake
def _(x, params, ln_weight, ln_bias, resid, ln_eps):
    M, F_ = x.numel() // x.shape[-1], params[0].shape[0]
    out = [torch.empty_like(x), x.new_empty(M, F_), x.new_empty(M, F_)]
    if ln_eps >= 0:
        out += [torch.empty_like(x), x.new_empty(M), x.new_empty(M)]
    return out


@torch.library.custom_op(f"{_LIB}::feed_forward_backward", mutates_args=())
def feed_forward_backward(dy: Tensor, x: Tensor, params: List[Tensor], ln_weight: Optional[Tensor],
                          ln_bias: Optional[Tensor], saved: List[Tensor], resid: bool, ln_eps: float) -> List[Tensor]:
    """-> [dx, dW1, db1, dW2, db2 (, dgamma, dbeta)]."""
    ln = ln_eps >= 0
    W1, b1, W2, b2 = params
    fused = ln and ops.ln_fusable(x.shape[-1], W2.shape[1])
    ctx = _Ctx()
    ctx.G, ctx.has_r, ctx.drop_p, ctx.s1, ctx.s2, ctx.ln = 1, resid, 0.0, [None], [None], fused
    ctx.b1, ctx.b2, ctx.bet = (b1,), (b2,), ((ln_bias,) if fused else ())
    ctx.lnsaved = ctx.lnprev = None
    sv = [x, W1, W2, saved[0], saved[1]] + ([saved[2], ln_weight, saved[3], saved[4]] if fused else [])
    ctx.saved_tensors = tuple(sv)
    with ops.library_mode():
        dln = []
        if ln and not fused:
            dy, dg, db = _ln_plain_bwd(dy, saved[2], ln_weight, ln_bias, saved[3], saved[4])
            dln = [dg, db]
        g = ops.FeedForwardResidual.backward(ctx, dy.contiguous())
    return [t for t in g[5:]] + dln


@feed_forward_backward.register_fake
def _(dy, x, params, ln_weight, ln_bias, saved, resid, ln_eps):
    out = [torch.empty_like(x)] + [torch.empty_like(p) for p in params]
    if ln_eps >= 0:
        out += [torch.empty_like(ln_weight), torch.empty_like(ln_bias)]
    return out


def _ffn_setup(ctx, inputs, output):
    x, params, ln_weight, ln_bias, resid, ln_eps = inputs
    ctx.save_for_backward(x, ln_weight, ln_bias, *params, *output[1:])
    ctx.meta = (resid, ln_eps)
    ctx.mark_non_differentiable(*output[1:])


def _ffn_bwd(ctx, grads):
    resid, ln_eps = ctx.meta
    sv = ctx.saved_tensors
    x, ln_weight, ln_bias = sv[:3]
    params, saved = list(sv[3:7]), list(sv[7:])
    dy = grads[0] if grads[0] is not None else torch.zeros_like(x)
    g = feed_forward_backward(dy, x, params, ln_weight, ln_bias, saved, resid, ln_eps)
    # Function order: dx, dW1, db1, dW2, db2 (, dgamma, dbeta) -> params order W1, b1, W2, b2
    dln = (g[5], g[6]) if ln_eps >= 0 else (None, None)
    return g[0], [g[1], g[2], g[3], g[4]], dln[0], dln[1], None, None


feed_forward.register_autograd(_ffn_bwd, setup_context=_ffn_setup)


# --------------------------------------------------------------------------- Linear (+ GELU) (+ residual)
@torch.library.custom_op(f"{_LIB}::linear", mutates_args=())
def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor], resid: Optional[Tensor], gelu: bool) -> List[Tensor]:
    """ops.LinearResidual / ops.LinearGelu for one stream: y = [GELU](x W^T + b) (+ r)
    (attention out-projections, residual.py's Linears, fusion.py:43-50, 71-77).
    -> [y] (+ [z], the pre-activation, with gelu)."""
    L.require_device(x)
    ctx = _Ctx()
    fn = ops.LinearGelu if gelu else ops.LinearResidual
    with ops.library_mode():
        (y,) = fn.forward(ctx, 1, resid is not None, x, weight, bias, *_opt(resid))
    return [y] + ([ctx.saved_tensors[2]] if gelu else [])


@linear.register_fake
def _(x, weight, bias, resid, gelu):
    y = x.new_empty(*x.shape[:-1], weight.shape[0])
    return [y] + ([x.new_empty(x.numel() // x.shape[-1], weight.shape[0])] if gelu else [])


@torch.library.custom_op(f"{_LIB}::linear_backward", mutates_args=())
def linear_backward(dy: Tensor, x: Tensor, weight: Tensor, bias: Optional[Tensor], z: Optional[Tensor],
                    has_resid: bool) -> List[Tensor]:
    """-> [dx, dW (, db) (, dresid)]."""
    ctx = _Ctx()
    ctx.G, ctx.has_r, ctx.b = 1, has_resid, (bias,)
    ctx.saved_tensors = (x, weight) + ((z,) if z is not None else ())
    fn = ops.LinearGelu if z is not None else ops.LinearResidual
    with ops.library_mode():
        g = fn.backward(ctx, dy.contiguous())
    return [t for t in g[2:] if t is not None]


@linear_backward.register_fake
def _(dy, x, weight, bias, z, has_resid):
    out = [torch.empty_like(x), torch.empty_like(weight)] + ([torch.empty_like(bias)] if bias is not None else [])
    return out + ([torch.empty_like(dy)] if has_resid else [])


def _linear_setup(ctx, inputs, output):
    x, weight, bias, resid, gelu = inputs
    ctx.save_for_backward(x, weight, bias, output[1] if gelu else None)
    ctx.has_resid = resid is not None
    if gelu:
        ctx.mark_non_differentiable(output[1])


def _linear_bwd(ctx, grads):
    x, weight, bias, z = ctx.saved_tensors
    dy = grads[0] if grads[0] is not None else x.new_zeros(*x.shape[:-1], weight.shape[0])
    g = linear_backward(dy, x, weight, bias, z, ctx.has_resid)
    db = g[2] if bias is not None else None
    dr = g[-1] if ctx.has_resid else None
    return g[0], g[1], db, dr, None


linear.register_autograd(_linear_bwd, setup_context=_linear_setup)


# --------------------------------------------------------------------------- LayerNorm (+ table / post / ReLU)
@torch.library.custom_op(f"{_LIB}::layer_norm_ex", mutates_args=())
def layer_norm_ex(x: Tensor, table: Optional[Tensor], post: Optional[Tensor], weight: Tensor, bias: Tensor,
                  eps: float, relu: bool) -> List[Tensor]:
    """ops.LayerNormAdd for one stream: y = act(LayerNorm(x + table[t + 2]) + post) — the
    embedding LayerNorm over the position table (keypoint_module.py:154-165) and the
    ResidualBlock tails (model/residual.py:32-38).  -> [y, mean, rstd]."""
    L.require_device(x)
    ctx = _Ctx()
    with ops.library_mode():
        (y,) = ops.LayerNormAdd.forward(ctx, 1, eps, table is not None, post is not None, 1 if relu else 0, 0.0, x,
                                        *_opt(table), *_opt(post), weight, bias)
    sv = ctx.saved_tensors  # x (, table), gamma, mean, rstd (, y)
    o = 2 if table is not None else 1
    return [y, sv[o + 1], sv[o + 2]]


@layer_norm_ex.register_fake
def _(x, table, post, weight, bias, eps, relu):
    rows = x.numel() // x.shape[-1]
    return [torch.empty_like(x), x.new_empty(rows), x.new_empty(rows)]


@torch.library.custom_op(f"{_LIB}::layer_norm_ex_backward", mutates_args=())
def layer_norm_ex_backward(dy: Tensor, x: Tensor, table: Optional[Tensor], has_post: bool, weight: Tensor,
                           bias: Tensor, mean: Tensor, rstd: Tensor, y: Tensor, relu: bool) -> List[Tensor]:
    """-> [dx (, dtable) (, dpost), dgamma, dbeta]."""
    ctx = _Ctx()
    pos = table is not None
    N = x.shape[-1]
    rows = x.numel() // N
    ctx.G, ctx.pos, ctx.has_post, ctx.act = 1, pos, has_post, 1 if relu else 0
    ctx.r_mod, ctx.r_off = (x.shape[1], 2) if pos else (max(rows, 1), 0)
    ctx.drop_p, ctx.seeds, ctx.bet, ctx.lnsaved = 0.0, [0], (bias,), None
    ctx.saved_tensors = (x,) + ((table,) if pos else ()) + (weight, mean, rstd) + ((y,) if relu else ())
    with ops.library_mode():
        g = ops.LayerNormAdd.backward(ctx, dy.contiguous())
    return list(g[6:])


@layer_norm_ex_backward.register_fake
def _(dy, x, table, has_post, weight, bias, mean, rstd, y, relu):
    return [torch.empty_like(x)] + ([torch.empty_like(table)] if table is not None else []) + \
        ([torch.empty_like(x)] if has_post else []) + [torch.empty_like(weight), torch.empty_like(bias)]


def _lnx_setup(ctx, inputs, output):
    x, table, post, weight, bias, eps, relu = inputs
    ctx.save_for_backward(x, table, weight, bias, output[0], output[1], output[2])
    ctx.meta = (post is not None, relu)
    ctx.mark_non_differentiable(output[1], output[2])


def _lnx_bwd(ctx, grads):
    x, table, weight, bias, y, mean, rstd = ctx.saved_tensors
    has_post, relu = ctx.meta
    dy = grads[0] if grads[0] is not None else torch.zeros_like(x)
    g = layer_norm_ex_backward(dy, x, table, has_post, weight, bias, mean, rstd, y, relu)
    i = 1
    dtab = g[i] if table is not None else None
    i += 1 if table is not None else 0
    dpost = g[i] if has_post else None
    i += 1 if has_post else 0
    return g[0], dtab, dpost, g[i], g[i + 1], None, None


layer_norm_ex.register_autograd(_lnx_bwd, setup_context=_lnx_setup)


# --------------------------------------------------------------------------- MaxPool1d(2, 2) over frames
@torch.library.custom_op(f"{_LIB}::maxpool_t", mutates_args=())
def maxpool_t(x: Tensor) -> Tensor:
    """(B, T, C) -> (B, T // 2, C): MaxPool1d(2, 2) over the frame axis (model/residual.py:40-43)."""
    L.require_device(x)
    ctx = _Ctx()
    with ops.library_mode():
        (y,) = ops.MaxPoolT.forward(ctx, 1, x)
    return y


@maxpool_t.register_fake
def _(x):
    B, T, C = x.shape
    return x.new_empty(B, T // 2, C)


@torch.library.custom_op(f"{_LIB}::maxpool_t_backward", mutates_args=())
def maxpool_t_backward(dy: Tensor, x: Tensor) -> Tensor:
    ctx = _Ctx()
    ctx.G, ctx.saved_tensors = 1, (x.contiguous(),)
    with ops.library_mode():
        return ops.MaxPoolT.backward(ctx, dy.contiguous())[1]


@maxpool_t_backward.register_fake
def _(dy, x):
    return torch.empty_like(x)


def _pool_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])


def _pool_bwd(ctx, dy):
    (x,) = ctx.saved_tensors
    return maxpool_t_backward(dy, x)


maxpool_t.register_autograd(_pool_bwd, setup_context=_pool_setup)


# --------------------------------------------------------------------------- coordinate mapping
@torch.library.custom_op(f"{_LIB}::coordinate_mapping", mutates_args=())
def coordinate_mapping(kp: Tensor, joint_idx: Tensor, wx: Tensor, bx: Optional[Tensor], wy: Tensor,
                       by: Optional[Tensor]) -> List[Tensor]:
    """ops.CoordinateMappingOp for one stream: the stream's joints of the (B, T, K_all, 2)
    keypoints, x / y de-interleaved, two Linear(K -> d) (layers.py:111-123,
    model/__init__.py:133-142).  joint_idx: int32 joint indices.  -> [x_embed, y_embed]."""
    L.require_device(kp)
    ctx = _Ctx()
    with ops.library_mode():
        xe, ye = ops.CoordinateMappingOp.forward(ctx, 1, kp, joint_idx, wx, bx, wy, by)
    return [xe, ye]


@coordinate_mapping.register_fake
def _(kp, joint_idx, wx, bx, wy, by):
    B, T = kp.shape[0], kp.shape[1]
    return [kp.new_empty(B, T, wx.shape[0]), kp.new_empty(B, T, wy.shape[0])]


@torch.library.custom_op(f"{_LIB}::coordinate_mapping_backward", mutates_args=())
def coordinate_mapping_backward(dxe: Tensor, dye: Tensor, kp: Tensor, joint_idx: Tensor, wx: Tensor,
                                bx: Optional[Tensor], wy: Tensor, by: Optional[Tensor]) -> List[Tensor]:
    """-> [dkp, dWx (, dbx), dWy (, dby)]."""
    ctx = _Ctx()
    ctx.G, ctx.kp_grad, ctx.bx, ctx.by = 1, True, (bx,), (by,)
    ctx.saved_tensors = (kp.contiguous(), joint_idx, wx, wy)
    with ops.library_mode():
        g = ops.CoordinateMappingOp.backward(ctx, dxe, dye)
    return [t for t in (g[1],) + g[3:] if t is not None]


@coordinate_mapping_backward.register_fake
def _(dxe, dye, kp, joint_idx, wx, bx, wy, by):
    return [torch.empty_like(kp), torch.empty_like(wx)] + ([torch.empty_like(bx)] if bx is not None else []) + \
        [torch.empty_like(wy)] + ([torch.empty_like(by)] if by is not None else [])


def _map_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _map_bwd(ctx, grads):
    kp, joint_idx, wx, bx, wy, by = ctx.saved_tensors
    dxe, dye = (g if g is not None else kp.new_zeros(kp.shape[0], kp.shape[1], w.shape[0])
                for g, w in zip(grads, (wx, wy)))
    g = coordinate_mapping_backward(dxe.contiguous(), dye.contiguous(), kp, joint_idx, wx, bx, wy, by)
    i = 2
    dbx = g[i] if bx is not None else None
    i += 1 if bx is not None else 0
    dwy = g[i]
    dby = g[i + 1] if by is not None else None
    return g[0], None, g[1], dbx, dwy, dby


coordinate_mapping.register_autograd(_map_bwd, setup_context=_map_setup)


# --------------------------------------------------------------------------- per-clip matmul, row softmax
@torch.library.custom_op(f"{_LIB}::clip_matmul", mutates_args=())
def clip_matmul(a: Tensor, b: Tensor, trans_b: bool) -> Tensor:
    """C[i] = A[i] B[i]^T (trans_b) or A[i] B[i] per clip (model/fusion.py:52-55)."""
    L.require_device(a, b)
    with ops.library_mode():
        return ops.ClipMatmul.forward(_Ctx(), trans_b, a, b)


@clip_matmul.register_fake
def _(a, b, trans_b):
    return a.new_empty(a.shape[0], a.shape[1], b.shape[1] if trans_b else b.shape[2])


@torch.library.custom_op(f"{_LIB}::clip_matmul_backward", mutates_args=())
def clip_matmul_backward(dc: Tensor, a: Tensor, b: Tensor, trans_b: bool) -> List[Tensor]:
    ctx = _Ctx()
    ctx.trans_b, ctx.saved_tensors = trans_b, (a.contiguous(), b.contiguous())
    with ops.library_mode():
        _, da, db = ops.ClipMatmul.backward(ctx, dc)
    return [da, db]


@clip_matmul_backward.register_fake
def _(dc, a, b, trans_b):
    return [torch.empty_like(a), torch.empty_like(b)]


def _cm_setup(ctx, inputs, output):
    a, b, trans_b = inputs
    ctx.save_for_backward(a, b)
    ctx.trans_b = trans_b


def _cm_bwd(ctx, dc):
    a, b = ctx.saved_tensors
    da, db = clip_matmul_backward(dc, a, b, ctx.trans_b)
    return da, db, None


clip_matmul.register_autograd(_cm_bwd, setup_context=_cm_setup)


@torch.library.custom_op(f"{_LIB}::softmax_rows", mutates_args=())
def softmax_rows(x: Tensor) -> Tensor:
    """softmax over the last dimension (model/fusion.py:53)."""
    L.require_device(x)
    with ops.library_mode():
        return ops.SoftmaxRows.forward(_Ctx(), x)


@softmax_rows.register_fake
def _(x):
    return torch.empty_like(x)


@torch.library.custom_op(f"{_LIB}::softmax_rows_backward", mutates_args=())
def softmax_rows_backward(dy: Tensor, y: Tensor) -> Tensor:
    ctx = _Ctx()
    ctx.saved_tensors = (y,)
    with ops.library_mode():
        return ops.SoftmaxRows.backward(ctx, dy)


@softmax_rows_backward.register_fake
def _(dy, y):
    return torch.empty_like(y)


def _sm_setup(ctx, inputs, output):
    ctx.save_for_backward(output)


def _sm_bwd(ctx, dy):
    (y,) = ctx.saved_tensors
    return softmax_rows_backward(dy, y)


softmax_rows.register_autograd(_sm_bwd, setup_context=_sm_setup)


# --------------------------------------------------------------------------- grouped front-ends
# Same signatures as the `ops` Functions' .apply: eager -> the grouped launch; while
# torch.compile traces -> the operators above, one stream at a time (dropout active: the
# grouped launch, run eagerly behind a graph break).
_eager = torch.compiler.disable


def _bias_list(bs):
    return [b for b in bs]


def attention_block_apply(G, kind, H, scale, plus_one, key_valid, add_mask, has_resid, drop_p, ln_eps, nxt, attn_p,
                          *ts):
    if not compiling():
        return ops.AttentionBlock.apply(G, kind, H, scale, plus_one, key_valid, add_mask, has_resid, drop_p, ln_eps,
                                        nxt, attn_p, *ts)
    if drop_p > 0 or attn_p > 0:
        return _eager(ops.AttentionBlock.apply)(G, kind, H, scale, plus_one, key_valid, add_mask, has_resid, drop_p,
                                                ln_eps, None, attn_p, *ts)
    cross = kind == "cross"
    ln = ln_eps is not None
    o = G * (2 if cross else 1)
    W, Wo, bo = ts[o:o + 6 * G], ts[o + 6 * G:o + 7 * G], ts[o + 7 * G:o + 8 * G]
    gam = ts[o + 8 * G:o + 9 * G] if ln else [None] * G
    bet = ts[o + 9 * G:o + 10 * G] if ln else [None] * G
    outs = []
    for g in range(G):
        xkv = ts[G + g] if cross else None
        params = list(W[6 * g:6 * g + 6]) + [Wo[g], bo[g]]
        outs.append(attention_block(ts[g], xkv, params, gam[g], bet[g], key_valid, add_mask, kind, H, float(scale),
                                    bool(plus_one), bool(has_resid), float(ln_eps) if ln else -1.0)[0])
    return tuple(outs)


def feed_forward_apply(G, has_r, drop_p, ln_eps, nxt, *ts):
    if not compiling():
        return ops.FeedForwardResidual.apply(G, has_r, drop_p, ln_eps, nxt, *ts)
    if drop_p > 0:
        return _eager(ops.FeedForwardResidual.apply)(G, has_r, drop_p, ln_eps, None, *ts)
    ln = ln_eps is not None
    outs = []
    for g in range(G):
        params = [ts[G + g], ts[2 * G + g], ts[3 * G + g], ts[4 * G + g]]
        gam, bet = (ts[5 * G + g], ts[6 * G + g]) if ln else (None, None)
        outs.append(feed_forward(ts[g], params, gam, bet, bool(has_r), float(ln_eps) if ln else -1.0)[0])
    return tuple(outs)


def linear_apply(G, has_r, *ts, gelu=False):
    if not compiling():
        return (ops.LinearGelu if gelu else ops.LinearResidual).apply(G, has_r, *ts)
    return tuple(linear(ts[g], ts[G + g], ts[2 * G + g], ts[3 * G + g] if has_r else None, gelu)[0]
                 for g in range(G))


def layer_norm_add_apply(G, eps, pos_table, has_post, act, drop_p, *ts):
    if not compiling():
        return ops.LayerNormAdd.apply(G, eps, pos_table, has_post, act, drop_p, *ts)
    if drop_p > 0:
        return _eager(ops.LayerNormAdd.apply)(G, eps, pos_table, has_post, act, drop_p, *ts)
    o = G
    tab = ts[o:o + G] if pos_table else [None] * G
    o += G if pos_table else 0
    post = ts[o:o + G] if has_post else [None] * G
    o += G if has_post else 0
    gam, bet = ts[o:o + G], ts[o + G:o + 2 * G]
    return tuple(layer_norm_ex(ts[g], tab[g], post[g], gam[g], bet[g], float(eps), bool(act))[0] for g in range(G))


def maxpool_t_apply(G, *xs):
    if not compiling():
        return ops.MaxPoolT.apply(G, *xs)
    return tuple(maxpool_t(x) for x in xs)


def coordinate_mapping_apply(G, kp, *ts):
    if not compiling():
        return ops.CoordinateMappingOp.apply(G, kp, *ts)
    outs = [coordinate_mapping(kp, ts[g], ts[G + g], ts[2 * G + g], ts[3 * G + g], ts[4 * G + g]) for g in range(G)]
    return tuple(o[0] for o in outs) + tuple(o[1] for o in outs)


def clip_matmul_apply(trans_b, a, b):
    if not compiling():
        return ops.ClipMatmul.apply(trans_b, a, b)
    return clip_matmul(a, b, bool(trans_b))


def softmax_rows_apply(x):
    if not compiling():
        return ops.SoftmaxRows.apply(x)
    return softmax_rows(x)
