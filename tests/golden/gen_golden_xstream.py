"""Golden vectors for BASELINE config 1's x-coordinate stream, from the REFERENCE.

Runs ONLY in the build container, where `/root/reference` (tinh2044/SCAttenNet, snapshot
2025-07-18) is importable; writes `xstream_cfg1.npz` (data only) and its entry in
`manifest.json`.  The stream is assembled from the reference's own modules and call order:
CoordinateMapping (model/layers.py:111-123; x half), the SCA's self position embedding and
first LayerNorm (model/keypoint_module.py:155, 161) and its self layers with the key-padding
mask (:167, :176-178) — config 1 at L = 2 (B=2, T=64, K=27, d=64, H=4; ragged lengths).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_xstream.py
"""
import json
import os
import sys

import torch
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (puts /root/reference on sys.path)
from model.keypoint_module import CoordinateAttention  # noqa: E402
from model.layers import CoordinateMapping, LearningPositionEmbedding  # noqa: E402
from model.utils import create_attention_mask  # noqa: E402


class XStream(nn.Module):
    """The reference modules of one stream's x half, under KeypointModule's key names."""

    def __init__(self, K, cfg):
        super().__init__()
        self.coordinate_mapping = CoordinateMapping(K, cfg["d_model"])
        self.sca = nn.Module()
        self.sca.self_attn_layers = nn.ModuleList([CoordinateAttention(cfg, "self_attn")
                                                   for _ in range(cfg["attn_layers"])])
        self.sca.first_self_norm = nn.LayerNorm(cfg["d_model"])
        self.sca.self_pos_embed = LearningPositionEmbedding(cfg["max_position_embeddings"], cfg["d_model"])

    def forward(self, keypoints, mask):
        x_embed, _ = self.coordinate_mapping(keypoints[:, :, :, 0], keypoints[:, :, :, 1])
        s = self.sca.first_self_norm(self.sca.self_pos_embed(x_embed))
        m = create_attention_mask(mask, s.dtype)
        for layer in self.sca.self_attn_layers:
            s = layer(s, m)
        return s


def main():
    torch.set_num_threads(1)
    cfg = {"d_model": 64, "attention_heads": 4, "attention_dropout": 0.0, "dropout": 0.2, "ff_dim": 192,
           "attn_layers": 2, "max_position_embeddings": 64}
    B, T, K = 2, 64, 27
    torch.manual_seed(0)
    m = XStream(K, cfg)
    G.randomize_params(m, 21)
    mask = torch.ones(B, T, dtype=torch.long)
    mask[1, 40:] = 0
    inp = {"keypoints": torch.rand(B, T, K, 2), "mask": mask}
    name, meta = G.capture("xstream_cfg1", m, inp, lambda mod, i: mod(i["keypoints"], i["mask"]),
                           {"op": "x-stream (config 1)", "cfg": cfg, "K": K, "B": B, "T": T, "lengths": [T, 40],
                            "ref": "model/layers.py:111-123, model/keypoint_module.py:155-178"}, ("keypoints",))
    path = os.path.join(HERE, "manifest.json")
    man = json.load(open(path))
    man["fixtures"][name] = meta
    json.dump(man, open(path, "w"), indent=1)
    print("wrote", name)


if __name__ == "__main__":
    main()
