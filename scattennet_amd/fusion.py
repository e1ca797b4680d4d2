"""Drop-in CoordinatesFusion + InvertedResidual (model/fusion.py of tinh2044/SCAttenNet):
the cross-stream fusion of the left / right / body stream encodings (BASELINE config 3)."""
import torch.nn as nn

from . import library, ops
from .layers import drop_p, layernorm_grouped
from .precision import fp32_compute


def _lin(layers, xs, gelu=False, resid=None):
    G = len(xs)
    W = [l.weight for l in layers]
    b = [l.bias for l in layers]
    extra = list(resid) if resid is not None else []
    return list(library.linear_apply(G, resid is not None, *xs, *W, *b, *extra, gelu=gelu))


class CoordinatesFusion(nn.Module):
    """model/fusion.py:6-55.

    l, r, b = GELU(Linear_in->out(.)) (one grouped launch); A = softmax(r l^T) per clip —
    no 1/sqrt(d) scale and no mask, so padded frames take part, as in the reference;
    f = LayerNorm(out_proj(A b)); out = InvertedResidual(f)."""

    def __init__(self, in_feat, out_feat, drop_rate=0.0):
        super().__init__()
        self.left_se = nn.Linear(in_feat, out_feat)
        self.right_se = nn.Linear(in_feat, out_feat)
        self.body_se = nn.Linear(in_feat, out_feat)
        self.out_proj = nn.Linear(out_feat, out_feat)
        self.norm = nn.LayerNorm(out_feat)
        self.gelu = nn.GELU()
        self.inverted_res = InvertedResidual(out_feat, out_feat)
        self.drop_rate = drop_rate

    @fp32_compute()
    def forward(self, left_embed, right_embed, body_embed):
        p = drop_p([self], "drop_rate")
        lo, ro, bo = _lin([self.left_se, self.right_se, self.body_se], [left_embed, right_embed, body_embed],
                          gelu=True)
        attn = library.softmax_rows_apply(library.clip_matmul_apply(True, ro, lo))
        if p > 0:  # fusion.py:48
            attn = ops.dropout_grouped([attn], p)[0]
        fuse = library.clip_matmul_apply(False, attn, bo)
        fuse = _lin([self.out_proj], [fuse])
        fuse = layernorm_grouped([self.norm], fuse)[0]
        fuse = self.inverted_res(fuse)
        if p > 0:  # fusion.py:54
            fuse = ops.dropout_grouped([fuse], p)[0]
        return fuse


class InvertedResidual(nn.Module):
    """model/fusion.py:58-78: LN(GELU(L1 x) + x) -> GELU(L2 .) -> L3 (no outer residual)."""

    def __init__(self, in_dim, out_dim):
        super().__init__()
        self.linear_1 = nn.Linear(in_dim, in_dim)
        self.linear_2 = nn.Linear(in_dim, in_dim * 3)
        self.linear_3 = nn.Linear(in_dim * 3, out_dim)
        self.gelu = nn.GELU()
        self.bn1 = nn.LayerNorm(in_dim)

    @fp32_compute()
    def forward(self, x):
        out = _lin([self.linear_1], [x], gelu=True, resid=[x])
        out = layernorm_grouped([self.bn1], out)
        out = _lin([self.linear_2], out, gelu=True)
        return _lin([self.linear_3], out)[0]
