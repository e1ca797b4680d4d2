"""The stream-encoder part of MSCA_Net (model/__init__.py:72-154): body / left / right
KeypointModules over one keypoint tensor, then CoordinatesFusion.  Attribute names match
MSCA_Net (body_encoder, left_encoder, right_encoder, coordinates_fusion) so the matching
subset of a reference checkpoint loads into it.  BASELINE config 3 ("full encoder")."""
from torch import nn

from .fusion import CoordinatesFusion
from .keypoint_module import KeypointModule, joint_index_tensors, keypoint_streams_forward
from .precision import fp32_compute


class SCAEncoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.body_encoder = KeypointModule(cfg["body_idx"], num_frame=cfg.get("num_frame", 0), cfg=cfg)
        self.left_encoder = KeypointModule(cfg["left_idx"], num_frame=cfg.get("num_frame", 0), cfg=cfg)
        self.right_encoder = KeypointModule(cfg["right_idx"], num_frame=cfg.get("num_frame", 0), cfg=cfg)
        # model/__init__.py:96: the fusion drop rate is hard-coded to 0.2
        self.coordinates_fusion = CoordinatesFusion(cfg["in_fusion_dim"], cfg["out_fusion_dim"], 0.2)

    @fp32_compute()
    def forward(self, keypoints, mask):
        """keypoints (B, T, K_all, 2), mask (B, T) -> (fuse, left, right, body) embeddings.
        The three streams run in lock-step (one launch per stage), their joint slicing
        (model/__init__.py:133-142) fused into the mapping kernel's gather."""
        mods = [self.body_encoder, self.left_encoder, self.right_encoder]
        idx = getattr(self, "_idx", None)
        if idx is None or idx[0].device != keypoints.device:
            idx = self._idx = joint_index_tensors(mods, keypoints.device)
        body, left, right = keypoint_streams_forward(mods, idx, keypoints, mask, with_residual=True)
        fuse = self.coordinates_fusion(left, right, body)
        return fuse, left, right, body
