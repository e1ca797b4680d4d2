"""Drop-in attention operators (model/attention.py of tinh2044/SCAttenNet), MI355X-native.

Same constructors, forward signatures, error behaviour and state_dict keys as the reference;
the forward/backward run the grouped HIP kernels of `ops.py` (no ATen math on the path).

`attention_mask` may be
  * a `KeyPaddingMask` (what this package's SCA passes): per-clip key validity, the kernel
    synthesises the additive mask of model/utils.py:3-28 in registers (fast path), or
  * the reference's materialised additive (B, 1, Tq, Tk) fp32 tensor (general path: the
    kernel adds it exactly as `attn_weights += attention_mask` does, attention.py:65/117/171).
"""
import torch
from torch import nn

from . import library, ops
from .precision import fp32_compute


class BaseAttention(nn.Module):
    """model/attention.py:8-26."""

    def __init__(self, d_model, num_heads, dropout=0.0, bias=True):
        super().__init__()
        self.d_model = d_model
        self.num_heads = num_heads
        self.dropout = dropout
        self.head_dim = d_model // num_heads
        if (self.head_dim * num_heads) != self.d_model:
            raise ValueError(
                f"d_model must be divisible by num_heads (got `d_model`: {self.d_model}"
                f" and `num_heads`: {num_heads})."
            )
        self.scaling = self.head_dim ** -0.5
        # same construction order as the reference (k, v, q, out), so that a given torch
        # seed produces the same initial weights
        self.k_proj = nn.Linear(d_model, d_model, bias=bias)
        self.v_proj = nn.Linear(d_model, d_model, bias=bias)
        self.q_proj = nn.Linear(d_model, d_model, bias=bias)
        self.out_proj = nn.Linear(d_model, d_model, bias=bias)

    def _reinit_projections(self, d_model, bias):
        # the subclasses re-create the four projections (attention.py:41-44/:91-95/:143-146);
        # replicated for RNG-identical initialisation
        self.q_proj = nn.Linear(d_model, d_model, bias=bias)
        self.k_proj = nn.Linear(d_model, d_model, bias=bias)
        self.v_proj = nn.Linear(d_model, d_model, bias=bias)
        self.out_proj = nn.Linear(d_model, d_model, bias=bias)

    def qkv_params(self):
        return [self.q_proj.weight, self.q_proj.bias, self.k_proj.weight, self.k_proj.bias,
                self.v_proj.weight, self.v_proj.bias]


def _resolve_mask(mask, causal, B, Tq, Tk, device, H=1):
    """-> (key_valid, add_mask, plus_one).

    The kernels read `add_mask` as a dense contiguous (B, Tq, Tk) fp32 buffer (one mask for
    every head) or (B, H, Tq, Tk) (one per head), and `key_valid` as (B, Tk).  The reference
    adds the mask with `attn_weights += attention_mask` (attention.py:65/117/171), so every
    mask broadcastable to (B, H, Tq, Tk) is legal there: (B,1,Tq,Tk), (B,H,Tq,Tk),
    (1,1,Tq,Tk), (B,1,1,Tk), (Tq,Tk), (Tk,), a scalar ...  Such masks are expanded here to
    (B, Tq, Tk) when dim 1 is 1, to (B, H, Tq, Tk) when it is H.  `None` raises TypeError
    as `attn_weights += None` does."""
    if mask is None:
        raise TypeError("unsupported operand type(s) for +=: 'Tensor' and 'NoneType'")
    if isinstance(mask, ops.KeyPaddingMask):
        kv = mask.key_valid
        if tuple(kv.shape) != (B, Tk):
            raise ValueError(f"key padding mask is {tuple(kv.shape)}, expected (B, Tk) = {(B, Tk)}")
        if kv.device != device:
            raise RuntimeError(f"key padding mask on {kv.device}, queries on {device}")
        return kv, None, bool(causal and mask.causal_plus_one)
    if torch.is_tensor(mask):
        m = mask
        if m.dim() > 4:
            raise ValueError(f"attention_mask of shape {tuple(m.shape)} does not broadcast to (B, H, Tq, Tk)")
        if m.device != device:
            if m.dim() != 0:  # as in the reference, only a 0-dim CPU tensor may meet a device tensor
                raise RuntimeError(f"attention_mask on {m.device}, queries on {device}")
            m = m.to(device)
        m = m.reshape((1,) * (4 - m.dim()) + tuple(m.shape))
        for have, want, name in ((m.shape[0], B, "B"), (m.shape[1], H, "H"), (m.shape[2], Tq, "Tq"),
                                 (m.shape[3], Tk, "Tk")):
            if have not in (1, want):
                raise ValueError(f"attention_mask of shape {tuple(mask.shape)} does not broadcast to "
                                 f"(B, H, Tq, Tk) = {(B, H, Tq, Tk)} ({name})")
        m = m.to(torch.float32)
        if m.shape[1] == 1 or H == 1:
            return None, m.expand(B, 1, Tq, Tk)[:, 0].contiguous(), False
        return None, m.expand(B, H, Tq, Tk).contiguous(), False
    raise TypeError(f"unsupported attention_mask type {type(mask)}")


def attention_grouped(attns, kind, hidden, kv, mask, resid=False, drop_p=0.0, ln=None, nxt=None):
    """Run G attention operators of the same shape in lock-step (one launch per stage).

    kind: "self" | "causal" | "cross".  Returns dropout(out_proj(attn), drop_p), plus the
    operator's own query input when `resid` (the post-LN residual of the enclosing block;
    residual and dropout ride in the out-projection epilogue).  `ln` (G nn.LayerNorms): the
    enclosing block's LayerNorm applied to that result — fused into the out-projection
    launch (sca_gemm_ln) when d_model = 256, a separate LayerNorm launch otherwise.  `nxt`
    (ops.NextProjections): the next op's projections, chained into that launch when fused."""
    G = len(attns)
    a0 = attns[0]
    # attention-probability dropout (attention.py:67-69 / 119-121 / 173-175): F.dropout(p,
    # training=self.training); the grouped modules must share p and mode
    ps = {float(a.dropout) if a.training else 0.0 for a in attns}
    if len(ps) != 1:
        raise ValueError("grouped attention modules must share dropout and training mode")
    attn_p = ps.pop()
    if not 0.0 <= attn_p < 1.0:
        raise ValueError(f"dropout probability has to be in [0, 1), but got {attn_p}")
    causal = kind == "causal"
    hq = hidden[0]
    if hq.dim() != 3:
        raise ValueError(f"hidden_states must be (B, T, d_model), got {tuple(hq.shape)}")
    Tk = kv[0].shape[1] if kind == "cross" else hq.shape[1]
    key_valid, add_mask, plus_one = _resolve_mask(mask, causal, hq.shape[0], hq.shape[1], Tk, hq.device,
                                                  a0.num_heads)
    params = []
    for a in attns:
        params += a.qkv_params()
    ts = list(hidden) + (list(kv) if kind == "cross" else []) + params + \
        [a.out_proj.weight for a in attns] + [a.out_proj.bias for a in attns]
    d = hidden[0].shape[-1]
    fuse = ln is not None and ops.ln_fusable(d, d)
    if fuse:
        ts += [n.weight for n in ln] + [n.bias for n in ln]
    out = list(library.attention_block_apply(G, kind, a0.num_heads, a0.scaling, plus_one, key_valid, add_mask,
                                        bool(resid), float(drop_p), float(ln[0].eps) if fuse else None,
                                        nxt if fuse else None, attn_p, *ts))
    if ln is not None and not fuse:
        from .layers import layernorm_grouped
        out = layernorm_grouped(ln, out)
    return out


class SelfAttention(BaseAttention):
    """model/attention.py:29-76 — unmasked-in-time self-attention over the x-coordinate stream."""

    def __init__(self, d_model, num_heads, dropout=0.0, bias=True):
        super().__init__(d_model, num_heads, dropout=0.0, bias=True)
        self.dropout = dropout
        if (self.head_dim * num_heads) != d_model:
            raise ValueError("d_model must be divisible by num_heads")
        self._reinit_projections(d_model, bias)

    @fp32_compute()
    def forward(self, hidden_states, attention_mask):
        return attention_grouped([self], "self", [hidden_states], None, attention_mask)[0]


class CrossAttention(BaseAttention):
    """model/attention.py:79-128 — q from hidden_states, k/v from key_value_states (v from kv/2)."""

    def __init__(self, d_model, num_heads, dropout=0.0, bias=True):
        super().__init__(d_model, num_heads, dropout=0.0, bias=True)
        self.dropout = dropout
        if (self.head_dim * num_heads) != d_model:
            raise ValueError("d_model must be divisible by num_heads")
        self._reinit_projections(d_model, bias)

    @fp32_compute()
    def forward(self, hidden_states, key_value_states, attention_mask):
        return attention_grouped([self], "cross", [hidden_states], [key_value_states], attention_mask)[0]


class SelfCausalAttention(BaseAttention):
    """model/attention.py:131-182 — causal self-attention over the y-coordinate stream."""

    def __init__(self, d_model, num_heads, dropout=0.0, bias=True):
        super().__init__(d_model, num_heads, dropout=0.0, bias=True)
        self.dropout = dropout
        if (self.head_dim * num_heads) != d_model:
            raise ValueError("d_model must be divisible by num_heads")
        self._reinit_projections(d_model, bias)

    @fp32_compute()
    def forward(self, hidden_states, attention_mask):
        return attention_grouped([self], "causal", [hidden_states], None, attention_mask)[0]
