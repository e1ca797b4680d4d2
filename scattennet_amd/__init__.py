"""scattennet_amd — MI355X-native (gfx950 / CDNA4) implementation of the SCAttenNet
spatial-coordinate-attention hot path (tinh2044/SCAttenNet: model/attention.py,
model/keypoint_module.py, model/fusion.py and their helpers).

Drop-in modules keep the reference constructors, forward signatures and state_dict keys;
their math runs in hand-written HIP kernels (libscatten_hip.so, C ABI in include/scatten.h).
"""
from .encoder import SCAEncoder  # noqa: F401
from .fusion import CoordinatesFusion, InvertedResidual  # noqa: F401
from .attention import BaseAttention, CrossAttention, SelfAttention, SelfCausalAttention  # noqa: F401
from .keypoint_module import (CoordinateAttention, CoordinatesMerge, KeypointModule, KeypointStreams,  # noqa: F401
                              SeparativeCoordinateAttention)
from .layers import CoordinateMapping, FeedForward, LearningPositionEmbedding  # noqa: F401
from .residual import ResidualBlock, ResidualNetwork  # noqa: F401
from .data import JointParts, collate_keypoints, normalize_keypoints  # noqa: F401
from .alignment import AlignmentModule  # noqa: F401
from .heads import RecognitionHead, SeqKD, compute_loss, distillation_loss  # noqa: F401
from . import library  # noqa: F401  (torch.ops.scatten.*)
from .utils import KeyPaddingMask, create_attention_mask, create_causal_attention_mask, key_padding_mask  # noqa: F401

__version__ = "0.1.0"
