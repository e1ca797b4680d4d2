"""Drop-in layers of model/layers.py (tinh2044/SCAttenNet) used on the SCA hot path."""
import torch
from torch import nn

from . import library, ops
from .precision import fp32_compute


class LearningPositionEmbedding(nn.Embedding):
    """model/layers.py:15-30 — learned table of num_embeddings + 2 rows; frame t reads row
    t + 2.  On the SCA path the add is fused with the following LayerNorm
    (`pos_embed_layernorm_grouped`); `forward` alone keeps the reference contract."""

    def __init__(self, num_embeddings, embedding_dim):
        self.offset = 2
        super().__init__(num_embeddings + self.offset, embedding_dim)

    @fp32_compute()
    def forward(self, inputs_embeds):
        seq_len = inputs_embeds.shape[1]
        if seq_len + self.offset > self.weight.shape[0]:
            raise IndexError("index out of range in self")
        return inputs_embeds + self.weight[self.offset:self.offset + seq_len][None]


def pos_embed_layernorm_grouped(tables, norms, xs, drop_p=0.0):
    """G-way fused  dropout(LayerNorm(x + table[2:T+2]))  (keypoint_module.py:154-165)."""
    return list(library.layer_norm_add_apply(len(xs), norms[0].eps, True, False, 0, float(drop_p), *xs,
                                       *[e.weight for e in tables], *[n.weight for n in norms],
                                       *[n.bias for n in norms]))


def layernorm_grouped(norms, xs, post=None, relu=False):
    """G-way y = act(LayerNorm(x) + post)."""
    extra = list(post) if post is not None else []
    return list(library.layer_norm_add_apply(len(xs), norms[0].eps, False, post is not None, 1 if relu else 0, 0.0, *xs,
                                       *extra, *[n.weight for n in norms], *[n.bias for n in norms]))


def drop_p(mods, attr="dropout"):
    """The dropout probability a group of same-config modules applies now: their `attr` in
    training mode, 0 in eval mode (F.dropout(..., training=self.training))."""
    ps = {float(getattr(m, attr)) if m.training else 0.0 for m in mods}
    if len(ps) != 1:
        raise ValueError("grouped modules must share dropout and training mode")
    p = ps.pop()
    if not 0.0 <= p < 1.0:
        raise ValueError(f"dropout probability has to be in [0, 1), but got {p}")
    return p


def ffn_grouped(ffns, xs, residual=True, ln=None, nxt=None):
    """G-way FFN (layers.py:104-108); with `residual` the enclosing block's residual add is
    fused (y = FFN(x) + x, keypoint_module.py:71-72 / :108-109); `ln` (G nn.LayerNorms): the
    block's last LayerNorm, fused into the fc2 launch when d_model = 256; `nxt`
    (ops.NextProjections): the next op's projections, chained into that launch when fused."""
    G = len(xs)
    ts = [*xs, *[f.fc1.weight for f in ffns], *[f.fc1.bias for f in ffns], *[f.fc2.weight for f in ffns],
          *[f.fc2.bias for f in ffns]]
    fuse = ln is not None and ops.ln_fusable(xs[0].shape[-1], ffns[0].fc2.weight.shape[1])
    if fuse:
        ts += [n.weight for n in ln] + [n.bias for n in ln]
    out = list(library.feed_forward_apply(G, residual, drop_p(ffns), float(ln[0].eps) if fuse else None,
                                             nxt if fuse else None, *ts))
    if ln is not None and not fuse:
        out = layernorm_grouped(ln, out)
    return out


class FeedForward(nn.Module):
    """model/layers.py:94-108 — fc2(dropout(GELU(fc1 x))) then dropout."""

    def __init__(self, in_dim, out_dim, dropout):
        super().__init__()
        self.fc1 = nn.Linear(in_dim, out_dim)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(out_dim, in_dim)
        self.dropout = dropout

    @fp32_compute()
    def forward(self, x):
        return ffn_grouped([self], [x], residual=False)[0]


def fc1_request(ffns):
    """ops.NextProjections for the FFNs' fc1 (bias + GELU, keeping the pre-activation),
    computed in the launch that produces their input; None when not applicable (dropout
    inside the FFN, widths other than d_model = 256 / d_ff <= 768, SCA_CHAIN_NEXT=0)."""
    if not ops._CHAIN_NEXT or drop_p(ffns) > 0 or library.compiling():
        return None
    specs = [[(f.fc1.weight, f.fc1.bias, 1.0, True)] for f in ffns]
    return ops.NextProjections(specs) if ops.NextProjections.eligible(specs) else None


def coordinate_mapping_grouped(maps, keypoints, joint_idx):
    """G streams sliced out of ONE (B, T, K_all, 2) keypoint tensor (model/__init__.py:133-142)
    and mapped (layers.py:118-123) in one launch.  joint_idx: list of int32 device tensors."""
    G = len(maps)
    out = library.coordinate_mapping_apply(G, keypoints, *joint_idx, *[m.mapping_x.weight for m in maps],
                                        *[m.mapping_x.bias for m in maps], *[m.mapping_y.weight for m in maps],
                                        *[m.mapping_y.bias for m in maps])
    return list(out[:G]), list(out[G:])


class CoordinateMapping(nn.Module):
    """model/layers.py:111-123 — two independent Linear(K -> d) on the x and y coordinates."""

    def __init__(self, in_feat, out_feat):
        super().__init__()
        self.mapping_x = nn.Linear(in_feat, out_feat)
        self.mapping_y = nn.Linear(in_feat, out_feat)
        self._idx = None

    def joint_index(self, device):
        K = self.mapping_x.weight.shape[1]
        if self._idx is None or self._idx.device != device:
            self._idx = torch.arange(K, dtype=torch.int32, device=device)
        return self._idx

    @fp32_compute()
    def forward(self, x_coord, y_coord):
        # the kernel reads interleaved (.., K, 2) coordinates — what KeypointModule hands it
        # directly; a standalone call interleaves its two inputs first
        kp = torch.stack([x_coord, y_coord], dim=-1)
        xe, ye = coordinate_mapping_grouped([self], kp, [self.joint_index(kp.device)])
        return xe[0], ye[0]
