"""Input contract of the SCA path: the keypoint half of
SLR_Dataset (dataset.py:58-170) on the GPU.

`normalize_keypoints` is SLR_Dataset.normalize_keypoints (dataset.py:134-170: per frame,
per anatomical part, the part's bounding box grown by 5 % of its longer side, squared,
clamped to [0, 1], and the joints mapped into it) over a whole zero-padded batch in one
launch (`sca_normalize_parts`).  `collate_keypoints` is the keypoint fields of
SLR_Dataset.data_collator (dataset.py:58-125): zero padding to the longest clip, the (B, T)
int64 attention mask, valid_len_in = T_i // 4 and mask_head.  Frame selection, augmentation,
the pickle loader and the gloss tokenizer stay host-side data plumbing (out of scope).
"""
import torch

from . import _lib as L


class JointParts:
    """cfg["joint_parts"] (a list of joint-index lists) as device CSR arrays."""

    def __init__(self, parts, device):
        off = [0]
        for p in parts:
            off.append(off[-1] + len(p))
        self.parts = [list(map(int, p)) for p in parts]
        self.off = torch.tensor(off, dtype=torch.int32, device=device)
        self.idx = torch.tensor([j for p in self.parts for j in p], dtype=torch.int32, device=device)
        self.max_joint = max((j for p in self.parts for j in p), default=-1)


def normalize_keypoints(kp, lengths, joint_parts):
    """kp: (B, T, K_all, 2) fp32 on the GPU; lengths: (B,) valid frames per clip.
    Returns a new tensor: frames < length normalised part by part, frames >= length zero."""
    L.require_device(kp)
    if kp.dim() != 4 or kp.shape[-1] != 2:
        raise ValueError("keypoints must be (B, T, K_all, 2)")
    kp = kp.contiguous()
    B, T, K_all, _ = kp.shape
    parts = joint_parts if isinstance(joint_parts, JointParts) else JointParts(joint_parts, kp.device)
    if parts.max_joint >= K_all:
        raise IndexError("joint index out of range")  # numpy fancy indexing in the reference
    lens = torch.as_tensor(lengths, device=kp.device).to(torch.int32).contiguous()
    out = torch.empty_like(kp)
    L.check(L.lib().sca_normalize_parts(kp.data_ptr(), out.data_ptr(), lens.data_ptr(), B, T, K_all,
                                        parts.off.data_ptr(), parts.idx.data_ptr(), len(parts.parts),
                                        L.stream_handle()), "sca_normalize_parts")
    return out


def collate_keypoints(samples, joint_parts, normalize=True, device="cuda"):
    """samples: (T_i, K_all, 2) arrays / tensors (already frame-selected).  Returns the
    collator's keypoint fields on `device`: keypoints (B, T_max, K_all, 2) fp32, mask
    (B, T_max) int64, valid_len_in (B,) int64, mask_head (B, max(T_i // 4)) int64."""
    ts = [torch.as_tensor(s, dtype=torch.float32) for s in samples]
    lens = torch.tensor([t.shape[0] for t in ts], dtype=torch.int64)
    T = int(lens.max())
    batch = torch.zeros((len(ts), T) + tuple(ts[0].shape[1:]), dtype=torch.float32)
    for i, t in enumerate(ts):
        batch[i, :t.shape[0]] = t
    batch = batch.to(device, non_blocking=True)
    lens_d = lens.to(device)
    if normalize:
        batch = normalize_keypoints(batch, lens_d, joint_parts)
    ar = torch.arange(T, device=device)
    mask = (ar[None, :] < lens_d[:, None]).to(torch.int64)
    vl = lens_d // 4
    head = (torch.arange(int(vl.max()), device=device)[None, :] < vl[:, None]).to(torch.int64)
    return {"keypoints": batch, "mask": mask, "valid_len_in": vl, "mask_head": head}
