"""Mask builders of model/utils.py (tinh2044/SCAttenNet), plus the compact form the HIP
kernels consume.

`create_attention_mask` / `create_causal_attention_mask` keep the reference signatures and
return the reference's materialised additive fp32 masks (for callers that want them, e.g.
model/encoder.py).  The SCA path itself never materialises B*T^2 mask bytes: it passes a
`KeyPaddingMask` (per-clip key validity) and the kernels synthesise the same scores.
"""
import torch

from .ops import KeyPaddingMask

__all__ = ["create_attention_mask", "create_causal_attention_mask", "KeyPaddingMask", "key_padding_mask"]


def create_attention_mask(mask, dtype, tgt_len=None):
    """model/utils.py:3-12: (B,S) 0/1 -> (B,1,T,S); 0 where kept, finfo(dtype).min where padded."""
    bsz, src_len = mask.size()
    tgt_len = tgt_len if tgt_len is not None else src_len
    keep = mask[:, None, None, :].expand(bsz, 1, tgt_len, src_len).to(dtype)
    inv = 1.0 - keep
    return inv.masked_fill(inv.to(torch.bool), torch.finfo(dtype).min)


def create_causal_attention_mask(attention_mask, input_shape, inputs_embeds):
    """model/utils.py:15-28: the key-padding mask plus tril(ones) (+1.0 on j <= i)."""
    batch_size, query_length = input_shape[0], input_shape[1]
    m = create_attention_mask(attention_mask, inputs_embeds.dtype, tgt_len=query_length)
    tri = torch.tril(torch.ones((query_length, query_length), device=inputs_embeds.device,
                                dtype=inputs_embeds.dtype))
    return m + tri[None, None]


def key_padding_mask(mask, causal=False):
    """Compact equivalent of create_attention_mask (causal=False) or
    create_causal_attention_mask (causal=True)."""
    return KeyPaddingMask(mask, causal_plus_one=causal)
