"""Input contract of the SCA path: the keypoint half of
SLR_Dataset (dataset.py:58-170) on the GPU.

`normalize_keypoints` is SLR_Dataset.normalize_keypoints (dataset.py:134-170: per frame,
per anatomical part, the part's bounding box grown by 5 % of its longer side, squared,
clamped to [0, 1], and the joints mapped into it) over a whole zero-padded batch in one
launch (`sca_normalize_parts`).  `collate_keypoints` is the keypoint fields of
SLR_Dataset.data_collator (dataset.py:58-125): zero padding to the longest clip, the (B, T)
int64 attention mask, valid_len_in = T_i // 4 and mask_head.

`prepare_batch` is the whole sample pipeline of the collator for a batch: per clip the
frame selection (dataset.py:185-215) and the augmentation draw (dataset.py:124-132,
172-183) are decided on the host with the reference's own RNG calls in the reference's
order — Python's `random` and numpy's global generator — so a seeded run selects the same
frames and draws the same rotation / flip; the gather of the selected frames, the
augmentation (rotation about (0, 0), augmentation.py:3-18, and x -> 1 - x, :20-25, composed
into one affine per clip), the per-part normalisation and the padding then run as ONE
launch over the batch (`sca_prepare_keypoints`).  `load_sample` is the on-disk sample format
(dataset.py:40-56).  The gloss tokenizer stays host-side (out of scope).
"""
import math
import pickle
import random

import numpy as np
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


# --------------------------------------------------------------------------- sample pipeline
def load_sample(path):
    """dataset.py:40-56: one pickled sample {"keypoints": (T, K_all, 4), "gloss", "name" | "id"}
    -> (keypoints[:, :, :-2], gloss with double spaces collapsed once and stripped, name).
    The file is the caller's own data (as in the reference loader)."""
    with open(path, "rb") as f:
        sample = pickle.load(f)
    kp = sample["keypoints"][:, :, :-2]
    gloss = sample["gloss"].replace("  ", " ").strip()
    name = sample["name"] if "name" in sample else sample.get("id", "")
    return kp, gloss, name


def select_frames(n_frames, train, max_len, min_rate=0.5, max_rate=1.5):
    """dataset.py:185-215 -> the selected frame indices (sorted, int64).  Evaluation: all
    frames, or the centred max_len window.  Training: a target length drawn with
    random.randint(lo, hi + 1) (inclusive bounds, as the reference calls it) from
    [min_rate n, max_rate n] capped at max_len, then a sorted random subset
    (np.random.permutation) or every frame plus random repeats (np.random.randint)."""
    if not train:
        if n_frames <= max_len:
            return np.arange(n_frames, dtype=np.int64)
        start = (n_frames - max_len) // 2
        return np.arange(start, start + max_len, dtype=np.int64)
    lo = min(int(min_rate * n_frames), max_len)
    hi = min(int(max_rate * n_frames), max_len)
    tgt = random.randint(lo, hi + 1)
    if tgt <= n_frames:
        return np.sort(np.random.permutation(np.arange(n_frames))[:tgt]).astype(np.int64)
    extra = np.random.randint(0, n_frames, tgt - n_frames)
    return np.sort(np.concatenate([np.arange(n_frames), extra])).astype(np.int64)


def augmentation_draw(train):
    """dataset.py:127-128 + 172-183: with probability 1/2 (training only) a rotation by
    U(-15, 15) degrees about (0, 0) and / or a flip x -> 1 - x (each with probability 1/2,
    redrawn until at least one applies), drawn as the reference draws them.
    -> the ops in order: [("rot", degrees)] and / or [("flip",)], or [] (none)."""
    if not (train and np.random.rand() < 0.5):
        return []
    while True:
        ops = []
        if np.random.uniform(0, 1) < 0.5:
            ops.append(("rot", float(np.random.uniform(-15, 15))))
        if np.random.uniform(0, 1) < 0.5:
            ops.append(("flip",))
        if ops:
            return ops


def augmentation_affine(ops):
    """The ops of augmentation_draw composed into one 2x3 affine [[a00, a01, tx], [a10, a11,
    ty]] (float64), or None for no ops."""
    if not ops:
        return None
    m = np.eye(2, 3)
    for op in ops:
        if op[0] == "rot":  # augmentation.py:3-18 about (0, 0): p' = R p
            r = math.radians(op[1])
            c, s_ = math.cos(r), math.sin(r)
            m = np.array([[c, -s_], [s_, c]]) @ m
        else:  # augmentation.py:20-25: x -> 1 - x
            m = np.array([[-m[0, 0], -m[0, 1], 1.0 - m[0, 2]], m[1]])
    return m


def prepare_batch(samples, cfg, split, joint_parts=None, device="cuda"):
    """SLR_Dataset.data_collator's keypoint fields for `samples` ((T_i, K_all, 2) arrays,
    as load_sample returns them): frame selection and augmentation draws on the host in
    the reference's order (per sample: select_frames, then the augmentation draw), the
    gather / augmentation / normalisation / padding in one launch.  cfg: the dataset
    section ("max_len", "normalize", "joint_parts").  Returns keypoints (B, T, K_all, 2)
    fp32, mask (B, T) int64, valid_len_in (B,) int64 and mask_head, like collate_keypoints,
    plus "frames" (the selected indices) and "augment" (per clip, augmentation_draw's ops)."""
    train = split == "train"
    min_rate, max_rate = (0.5, 1.5) if train else (1.0, 1.0)
    picks, ops, affs, raws = [], [], [], []
    if not samples:
        raise ValueError("prepare_batch: empty batch")
    for kp in samples:
        kp = np.asarray(kp)
        # the kernel reads 2 * K_all floats per frame: a (T, K, 4) array that skipped
        # load_sample's [:, :, :-2] trim, or clips of different K_all, would be read at the
        # wrong stride
        if kp.ndim != 3 or kp.shape[-1] != 2 or kp.shape[1] != np.shape(samples[0])[1]:
            raise ValueError(f"prepare_batch: every sample must be (T, K_all, 2) with one K_all; got {kp.shape}")
        picks.append(select_frames(kp.shape[0], train, cfg["max_len"], min_rate, max_rate))
        ops.append(augmentation_draw(train))
        affs.append(augmentation_affine(ops[-1]))
        raws.append(kp.astype(np.float32, copy=False))
    B = len(raws)
    K_all = raws[0].shape[1]
    lens = [len(p) for p in picks]
    T = max(lens)
    base = np.cumsum([0] + [r.shape[0] for r in raws[:-1]])
    src = np.zeros((B, T), dtype=np.int32)
    for b, (pk, o) in enumerate(zip(picks, base)):
        src[b, :len(pk)] = pk + o
    raw = torch.from_numpy(np.concatenate(raws, 0)).to(device, non_blocking=True)
    src_d = torch.from_numpy(src).to(device, non_blocking=True)
    aff = None
    if any(a is not None for a in affs):
        aff = torch.tensor(np.stack([a if a is not None else np.eye(2, 3) for a in affs]).reshape(B, 6),
                           dtype=torch.float32, device=device)
    lens_d = torch.tensor(lens, dtype=torch.int32, device=device)
    parts = None
    if cfg.get("normalize", True):
        jp = joint_parts if joint_parts is not None else cfg["joint_parts"]
        parts = jp if isinstance(jp, JointParts) else JointParts(jp, device)
        if parts.max_joint >= K_all:
            raise IndexError("joint index out of range")
    out = torch.empty((B, T, K_all, 2), dtype=torch.float32, device=device)
    L.check(L.lib().sca_prepare_keypoints(raw.data_ptr(), src_d.data_ptr(), aff.data_ptr() if aff is not None else None,
                                          lens_d.data_ptr(), out.data_ptr(), B, T, K_all,
                                          parts.off.data_ptr() if parts else None,
                                          parts.idx.data_ptr() if parts else None,
                                          len(parts.parts) if parts else 0, L.stream_handle()),
            "sca_prepare_keypoints")
    lens64 = lens_d.to(torch.int64)
    ar = torch.arange(T, device=device)
    mask = (ar[None, :] < lens64[:, None]).to(torch.int64)
    vl = lens64 // 4
    head = (torch.arange(int(max(lens) // 4), device=device)[None, :] < vl[:, None]).to(torch.int64)
    return {"keypoints": out, "mask": mask, "valid_len_in": vl, "mask_head": head, "frames": picks,
            "augment": ops}
