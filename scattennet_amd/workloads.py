"""The BASELINE.json configurations as concrete synthetic workloads (shared by bench.py,
the scale tests and __graft_entry__.smoke).

Stream layouts: the reference builds body / left / right streams with
6 / 21 / 21 joints (configs/phoenix-2014t.yaml:227-277); BASELINE's K=79 "four-stream"
config adds a 31-joint face stream; K=133 is the COCO-WholeBody split 23 / 68 / 21 / 21.
"""
import math

import torch

CFG_BASE = {
    "attention_dropout": 0.0,
    "dropout": 0.0,  # primary throughput runs use p=0; the yaml has 0.2
    "self_attn_x": True,
}


def model_cfg(d_model, heads, layers=4, ff_mult=3, maxpos=256, residual_blocks=None):
    cfg = dict(CFG_BASE)
    cfg.update({"d_model": d_model, "attention_heads": heads, "ff_dim": ff_mult * d_model, "attn_layers": layers,
                "max_position_embeddings": maxpos,
                "residual_blocks": residual_blocks or [d_model, d_model, 2 * d_model, 2 * d_model]})
    return cfg


def split_groups(sizes):
    out, o = [], 0
    for s in sizes:
        out.append(list(range(o, o + s)))
        o += s
    return out


WORKLOADS = {
    # BASELINE config 1 (CPU-runnable reference case): x-stream only, 27 joints
    "cfg1": dict(B=2, T=64, K_all=27, groups=[27], d=64, H=4, L=4, residual=False, maxpos=64),
    # BASELINE config 2 — the metric's configuration: four SCA streams of K=79 joints
    "cfg2": dict(B=8, T=256, K_all=79, groups=[6, 21, 21, 31], d=256, H=16, L=4, residual=False, maxpos=256),
    # BASELINE config 3: the full encoder with the Phoenix-2014T yaml model section
    # (configs/phoenix-2014t.yaml:208-277): body/left/right = joints 11-16 / 33-53 / 54-74 of
    # the (B, T, 542, 2) MediaPipe tensor, residual [256,256,512,512], fusion 512 -> 1024
    "cfg3": dict(B=8, T=256, K_all=542, groups=[6, 21, 21], d=256, H=16, L=4, residual=True, maxpos=256,
                 fusion=True, joint_idx=[list(range(11, 17)), list(range(33, 54)), list(range(54, 75))],
                 residual_blocks=[256, 256, 512, 512], in_fusion=512, out_fusion=1024),
    # config 3 at a padded batch length that is not a multiple of 16 (the collator pads to the
    # longest clip, dataset.py:76-89): two pools leave 58 frames for the fusion (parity case)
    "cfg3_t234": dict(B=4, T=234, K_all=542, groups=[6, 21, 21], d=256, H=16, L=4, residual=True, maxpos=256,
                      fusion=True, joint_idx=[list(range(11, 17)), list(range(33, 54)), list(range(54, 75))],
                      residual_blocks=[256, 256, 512, 512], in_fusion=512, out_fusion=1024),
    # the Phoenix-2014 yaml model section (configs/phoenix-2014.yaml:211-220): residual
    # [256, 256] (one pool), fusion 256 -> 1024; odd T = 181 -> 90 frames (parity case)
    "cfg2014_t181": dict(B=4, T=181, K_all=542, groups=[6, 21, 21], d=256, H=16, L=4, residual=True, maxpos=256,
                         fusion=True, joint_idx=[list(range(11, 17)), list(range(33, 54)), list(range(54, 75))],
                         residual_blocks=[256, 256], in_fusion=256, out_fusion=1024),
    # BASELINE config 5: long sequence, 133 joints split COCO-WholeBody style
    "cfg5": dict(B=8, T=1024, K_all=133, groups=[23, 68, 21, 21], d=512, H=16, L=4, residual=False, maxpos=1024),
}


def pooled_frames(w):
    """Frames after the residual network: MaxPool1d(2, 2) (floor) on every even-indexed block
    (model/residual.py:22-23, 40-43)."""
    t = w["T"]
    for i in range(len(w.get("residual_blocks", [w["d"], w["d"], 2 * w["d"], 2 * w["d"]]))):
        if i % 2 == 0:
            t //= 2
    return t


def encoder_cfg(w):
    """The yaml-style model dict for a fusion workload (SCAEncoder / oracle)."""
    cfg = model_cfg(w["d"], w["H"], w["L"], maxpos=w["maxpos"], residual_blocks=w["residual_blocks"])
    cfg.update({"body_idx": w["joint_idx"][0], "left_idx": w["joint_idx"][1], "right_idx": w["joint_idx"][2],
                "in_fusion_dim": w["in_fusion"], "out_fusion_dim": w["out_fusion"], "num_frame": w["T"]})
    return cfg


def build_encoder(w, device, seed=0, init="reference"):
    from .encoder import SCAEncoder
    torch.manual_seed(seed)
    enc = SCAEncoder(encoder_cfg(w))
    if init == "reference":
        init_like_msca(enc)
    elif init == "random":
        randomize(enc, seed)
    # primary throughput runs use p = 0 everywhere, including the fusion's
    # hard-coded 0.2 (model/__init__.py:96)
    enc.coordinates_fusion.drop_rate = CFG_BASE["dropout"]
    return enc.to(device)


def build_streams(w, device, seed=0, init="reference"):
    """KeypointStreams for workload dict `w` (random-init weights of the real architecture)."""
    from .keypoint_module import KeypointModule, KeypointStreams
    torch.manual_seed(seed)
    cfg = model_cfg(w["d"], w["H"], w["L"], maxpos=w["maxpos"])
    cfg.update(w.get("cfg_over", {}))  # e.g. {"self_attn_x": False}
    mods = [KeypointModule(g, w["T"], cfg) for g in split_groups(w["groups"])]
    streams = KeypointStreams(mods, with_residual=w["residual"])
    if init == "reference":
        init_like_msca(streams)
    elif init == "random":
        randomize(streams, seed)
    return streams.to(device)


def init_like_msca(module):
    """MSCA_Net._init_weights (model/__init__.py:108-117): xavier Linear, zero bias, LN (1, 0)."""
    for m in module.modules():
        if isinstance(m, torch.nn.Linear):
            torch.nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                torch.nn.init.constant_(m.bias, 0)
        elif isinstance(m, torch.nn.LayerNorm):
            torch.nn.init.constant_(m.bias, 0)
            torch.nn.init.constant_(m.weight, 1.0)


def randomize(module, seed):
    """Every parameter non-trivial (random biases / LN affine) — for parity tests."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            if p.dim() == 2 and "embed" not in name:
                p.copy_(torch.randn(p.shape, generator=g) / math.sqrt(p.shape[1]))
            elif "embed" in name:
                p.copy_(torch.randn(p.shape, generator=g))
            elif name.endswith("weight"):
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(0.1 * torch.randn(p.shape, generator=g))


def synthetic_batch(w, device, seed=0, ragged=False):
    """keypoints ~ U[0,1) (the dataset normalises every part into [0,1], dataset.py:134-170),
    mask all ones (throughput) or ragged lengths (parity)."""
    g = torch.Generator().manual_seed(seed)
    B, T = w["B"], w["T"]
    kp = torch.rand(B, T, w["K_all"], 2, generator=g)
    mask = torch.ones(B, T, dtype=torch.long)
    if ragged:
        lens = [T, max(T - 37, 1), T // 2, 1, 0, max(T - 5, 1), T // 4, T][:B]
        for b, n in enumerate(lens):
            mask[b, n:] = 0
    if w.get("fusion"):
        gout = torch.randn(1, B, pooled_frames(w), w["out_fusion"], generator=torch.Generator().manual_seed(1))
    else:
        gout = torch.randn(len(w["groups"]), B, T, w["d"], generator=torch.Generator().manual_seed(1))
    return kp.to(device), mask.to(device), gout.to(device)


def flops_per_step(w):
    """Algorithmic fwd+bwd FLOPs of one step: per stream forward
    F = L (24 N d^2 + 8 B T^2 d + 4 B d T(T+1)/2 + 8 N d F) + 4 N K d, causal core counted on
    the lower triangle only; step = 3 F summed over streams."""
    B, T, d, L = w["B"], w["T"], w["d"], w["L"]
    N = B * T
    Fd = 3 * d
    total = 0.0
    for K in w["groups"]:
        f = L * (24 * N * d * d + 8 * B * T * T * d + 4 * B * d * T * (T + 1) / 2 + 8 * N * d * Fd) + 4 * N * K * d
        if w.get("residual"):
            blocks, rows, prev = w.get("residual_blocks", [d, d, 2 * d, 2 * d]), N, None
            for i, c in enumerate(blocks):
                cin = blocks[i - 1] if i > 0 else blocks[0]
                f += 2 * rows * cin * c + 2 * rows * c * c + (2 * rows * cin * c if cin != c else 0)
                if i % 2 == 0:
                    rows //= 2
        total += 3 * f
    if w.get("fusion"):
        t4 = pooled_frames(w)
        n4, ci, co = B * t4, w["in_fusion"], w["out_fusion"]
        f = 3 * 2 * n4 * ci * co + 2 * 2 * B * t4 * t4 * co + 2 * n4 * co * co * 2 + 2 * 2 * n4 * co * 3 * co
        total += 3 * f
    return total
