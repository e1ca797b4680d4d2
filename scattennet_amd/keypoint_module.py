"""Drop-in SCA blocks of model/keypoint_module.py (tinh2044/SCAttenNet), MI355X-native.

Each module keeps the reference constructor, forward signature and state_dict keys.  The
math lives in `*_grouped` functions that run G same-shaped modules (one per keypoint
stream) in lock-step, one HIP launch per stage for all streams; a module's own `forward` is
the G = 1 case.  `KeypointStreams` drives several KeypointModules that way.
"""
import torch
from torch import nn

from . import library, ops
from .attention import CrossAttention, SelfAttention, SelfCausalAttention, attention_grouped
from .layers import (CoordinateMapping, FeedForward, LearningPositionEmbedding, coordinate_mapping_grouped, drop_p,
                     fc1_request, ffn_grouped, pos_embed_layernorm_grouped)
from .residual import ResidualNetwork, residual_network_grouped
from .utils import key_padding_mask
from .precision import fp32_compute


# --------------------------------------------------------------------------- A9
class CoordinateAttention(nn.Module):
    """model/keypoint_module.py:34-80 — post-LN attention block; "causal_attn" has no MLP."""

    def __init__(self, cfg, attn_type="self_attn"):
        super().__init__()
        self.attn_type = attn_type
        if attn_type == "self_attn":
            self.attn = SelfAttention(d_model=cfg["d_model"], num_heads=cfg["attention_heads"],
                                      dropout=cfg["attention_dropout"])
            self.mlp = FeedForward(cfg["d_model"], cfg["ff_dim"], cfg["dropout"])
            self.last_layer_norm = nn.LayerNorm(cfg["d_model"])
        elif attn_type == "causal_attn":
            self.attn = SelfCausalAttention(d_model=cfg["d_model"], num_heads=cfg["attention_heads"],
                                            dropout=cfg["attention_dropout"])
            self.mlp = nn.Identity()
            self.last_layer_norm = nn.Identity()
        else:
            raise ValueError(f"Invalid attention type: {attn_type}")
        self.attn_layer_norm = nn.LayerNorm(cfg["d_model"])
        self.dropout = cfg["dropout"]
        self.activation_fn = nn.GELU()

    @fp32_compute(clamp=True)
    def forward(self, coord_embed, attention_mask=None):
        return coordinate_attention_grouped([self], [coord_embed], attention_mask)[0]


def coordinate_attention_grouped(blocks, xs, mask, nxt=None):
    """h = LN(x + Attn(x)); self type: h = LN(h + FFN(h))  (keypoint_module.py:61-80).
    The residual adds ride in the out-projection / fc2 epilogues; the FFN's fc1 is chained
    into the out-projection launch, and `nxt` (the next block's q / k / v, qkv_request) into
    the block's last launch."""
    kind = "self" if blocks[0].attn_type == "self_attn" else "causal"
    h = attention_grouped([b.attn for b in blocks], kind, xs, None, mask, resid=True, drop_p=drop_p(blocks),
                          ln=[b.attn_layer_norm for b in blocks],
                          nxt=fc1_request([b.mlp for b in blocks]) if kind == "self" else nxt)
    if kind == "self":
        h = ffn_grouped([b.mlp for b in blocks], h, residual=True, ln=[b.last_layer_norm for b in blocks], nxt=nxt)
    return h


def qkv_request(blocks):
    """ops.NextProjections for the q / k / v projections of self / causal attention blocks
    (q carries the 1/sqrt(head_dim) scale, as AttentionBlock computes it)."""
    if not ops._CHAIN_NEXT or library.compiling():
        return None
    specs = []
    for b in blocks:
        a = b.attn
        Wq, bq, Wk, bk, Wv, bv = a.qkv_params()
        specs.append([(Wq, bq, a.scaling, False), (Wk, bk, 1.0, False), (Wv, bv, 1.0, False)])
    return ops.NextProjections(specs) if ops.NextProjections.eligible(specs) else None


# --------------------------------------------------------------------------- A10
class CoordinatesMerge(nn.Module):
    """model/keypoint_module.py:83-115 — y <- CrossAttn(q=y, kv=x) then FFN, both post-LN."""

    def __init__(self, cfg):
        super().__init__()
        self.attn = CrossAttention(d_model=cfg["d_model"], num_heads=cfg["attention_heads"],
                                   dropout=cfg["attention_dropout"])
        self.mlp = FeedForward(cfg["d_model"], cfg["ff_dim"], cfg["dropout"])
        self.attn_layer_norm = nn.LayerNorm(cfg["d_model"])
        self.last_layer_norm = nn.LayerNorm(cfg["d_model"])
        self.dropout = cfg["dropout"]

    @fp32_compute(clamp=True)
    def forward(self, y_embed, x_embed, cross_attn_mask=None):
        return coordinates_merge_grouped([self], [y_embed], [x_embed], cross_attn_mask)[0]


def coordinates_merge_grouped(blocks, ys, xs, mask, nxt=None):
    h = attention_grouped([b.attn for b in blocks], "cross", ys, xs, mask, resid=True, drop_p=drop_p(blocks),
                          ln=[b.attn_layer_norm for b in blocks], nxt=fc1_request([b.mlp for b in blocks]))
    return ffn_grouped([b.mlp for b in blocks], h, residual=True, ln=[b.last_layer_norm for b in blocks], nxt=nxt)


# --------------------------------------------------------------------------- A11
class SeparativeCoordinateAttention(nn.Module):
    """model/keypoint_module.py:118-198."""

    def __init__(self, cfg=None):
        super().__init__()
        self.dropout = cfg["dropout"]
        self.self_attn_layers = nn.ModuleList(
            [CoordinateAttention(cfg, attn_type="self_attn") for _ in range(cfg["attn_layers"])])
        self.causal_attn_layers = nn.ModuleList(
            [CoordinateAttention(cfg, attn_type="causal_attn") for _ in range(cfg["attn_layers"])])
        self.coordinates_merge = nn.ModuleList([CoordinatesMerge(cfg) for _ in range(cfg["attn_layers"])])
        self.first_self_norm = nn.LayerNorm(cfg["d_model"])
        self.first_causal_norm = nn.LayerNorm(cfg["d_model"])
        self.self_pos_embed = LearningPositionEmbedding(cfg["max_position_embeddings"], cfg["d_model"])
        self.causal_pos_embed = LearningPositionEmbedding(cfg["max_position_embeddings"], cfg["d_model"])
        self.x_self = cfg.get("self_attn_x", True)

    @fp32_compute()
    def forward(self, x_embed, y_embed, attention_mask=None, return_attn_map=False):
        outs, s_maps = sca_grouped([self], [x_embed], [y_embed], attention_mask)
        if return_attn_map:
            return {"outputs": outs[0], "self_attn_map": s_maps[0], "causal_attn_map": outs[0]}
        return outs[0]


def sca_grouped(scas, xs, ys, attention_mask):
    """Returns (y-stream outputs, final x-stream maps) for G same-shaped SCA stacks.

    Data dependency (keypoint_module.py:176-187): every merge layer reads the FINAL x-stream
    map, so the L self layers run first, then L x (causal, merge)."""
    p = drop_p(scas)
    if attention_mask is None:
        raise AttributeError("'NoneType' object has no attribute 'size'")  # reference: mask.size()
    if len({bool(m.x_self) for m in scas}) > 1:
        # one grouped launch serves every stream: their self / causal inputs must agree
        raise ValueError("sca_grouped: the grouped SCA stacks mix self_attn_x=True and False")
    x_self = scas[0].x_self  # keypoint_module.py:154-159
    se, ce = (xs, ys) if x_self else (ys, xs)
    tabs = [m.self_pos_embed for m in scas] + [m.causal_pos_embed for m in scas]
    norms = [m.first_self_norm for m in scas] + [m.first_causal_norm for m in scas]
    G = len(scas)
    if p == 0:  # both streams' embedding LayerNorms in one launch
        both = pos_embed_layernorm_grouped(tabs, norms, list(se) + list(ce), p)
        se, ce = both[:G], both[G:]
    else:  # one call (one seed draw) per stream kind, in the reference's order
        se = pos_embed_layernorm_grouped(tabs[:G], norms[:G], se, p)
        ce = pos_embed_layernorm_grouped(tabs[G:], norms[G:], ce, p)
    self_mask = key_padding_mask(attention_mask)  # model/utils.py:3-12
    causal_mask = self_mask.causal_view()  # model/utils.py:15-28 (same key validity, +1 on j <= i)
    cross_mask = self_mask  # create_attention_mask(tgt_len=T) — same key padding
    L = len(scas[0].self_attn_layers)
    # one stream: a second stream for the self stack (concurrent with causal layer 0) was
    # -13 % at config 3 and -2.6 % at config 2 — the graph executor runs a forked branch's
    # queue list behind the main list, so the weight gradients queued behind it waited for the
    # whole backward
    s = _self_stack(scas, se, self_mask, L)
    c = ce
    s_for = None
    for i in range(L):
        c = coordinate_attention_grouped([m.causal_attn_layers[i] for m in scas], c, causal_mask)
        if i == 0:
            # every merge layer reads the final x-stream map: one fan-out, so that its L
            # incoming gradients are summed in one grouped launch after the last merge's backward
            s_for = ops.fan_out(s, L) if not library.compiling() else [s] * L
        nxt = qkv_request([m.causal_attn_layers[i + 1] for m in scas]) if i + 1 < L else None
        c = coordinates_merge_grouped([m.coordinates_merge[i] for m in scas], c, s_for[i], cross_mask, nxt=nxt)
    return c, s


def _self_stack(scas, s, mask, L):
    for i in range(L):
        nxt = qkv_request([m.self_attn_layers[i + 1] for m in scas]) if i + 1 < L else None
        s = coordinate_attention_grouped([m.self_attn_layers[i] for m in scas], s, mask, nxt=nxt)
    return s




# --------------------------------------------------------------------------- A1 + A2 + A11 + A12
class KeypointModule(nn.Module):
    """model/keypoint_module.py:13-31 — one anatomical stream: mapping -> SCA -> residual."""

    def __init__(self, joint_idx, num_frame, cfg=None):
        super().__init__()
        self.joint_idx = joint_idx
        self.num_frame = num_frame
        self.coordinate_mapping = CoordinateMapping(len(joint_idx), cfg["d_model"])
        self.sca = SeparativeCoordinateAttention(cfg)
        self.residual = ResidualNetwork(cfg["residual_blocks"])

    @fp32_compute()
    def forward(self, keypoints, attention_mask=None):
        # `keypoints` is the stream's own (B, T, K, 2) slice, as MSCA_Net passes it
        idx = self.coordinate_mapping.joint_index(keypoints.device)
        xe, ye = coordinate_mapping_grouped([self.coordinate_mapping], keypoints, [idx])
        out, _ = sca_grouped([self.sca], xe, ye, attention_mask)
        return residual_network_grouped([self.residual], out)[0]


class KeypointStreams(nn.Module):
    """Several KeypointModules run in lock-step over ONE (B, T, K_all, 2) keypoint tensor.

    The stream slicing of MSCA_Net.forward (model/__init__.py:133-142) is fused into the
    mapping kernel's gather, and every later stage runs all streams in one launch.  Streams
    must share d_model / heads / layers (they do: one cfg).  `with_residual=False` stops after
    the SCA stack (BASELINE config 2); True adds the ResidualNetwork (config 3)."""

    def __init__(self, modules, with_residual=True):
        super().__init__()
        self.streams = nn.ModuleList(modules)
        self.with_residual = with_residual
        self._idx = None

    def joint_indices(self, device):
        if self._idx is None or self._idx[0].device != device:
            self._idx = joint_index_tensors(self.streams, device)
        return self._idx

    @fp32_compute()
    def forward(self, keypoints, attention_mask):
        return keypoint_streams_forward(list(self.streams), self.joint_indices(keypoints.device), keypoints,
                                        attention_mask, self.with_residual)


def joint_index_tensors(mods, device):
    return [torch.tensor(list(m.joint_idx), dtype=torch.int32, device=device) for m in mods]


def keypoint_streams_forward(mods, joint_idx, keypoints, attention_mask, with_residual=True):
    """G KeypointModules in lock-step over one (B, T, K_all, 2) tensor (stream slicing fused)."""
    xe, ye = coordinate_mapping_grouped([m.coordinate_mapping for m in mods], keypoints, joint_idx)
    out, _ = sca_grouped([m.sca for m in mods], xe, ye, attention_mask)
    if with_residual:
        out = residual_network_grouped([m.residual for m in mods], out)
    return out
