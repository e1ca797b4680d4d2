"""Input contract pinned to the REFERENCE: vectors produced by the
reference's own dataset.py (tests/golden/gen_golden_dataset.py -> dataset.npz) for
SLR_Dataset.normalize_part / normalize_keypoints (dataset.py:134-170), select_frames
(:185-217, seeded draw sequences) and the keypoint fields of data_collator (:58-122, through
preprocess_keypoints: selection, augmentation draw, normalisation, padding, masks).

CPU: the oracle restatement and the host-side draws of scattennet_amd.data against them.
GPU: the one-launch pipeline (sca_prepare_keypoints) and sca_normalize_parts against them
(fp32 on the device; the reference normalises rotated clips in float64: 1e-5 absolute on
[0, 1]-scale coordinates).
"""
import os
import random

import numpy as np
import pytest
import torch

from oracle import sca_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "dataset.npz"))


def _split(flat, off):
    return [flat[off[i]:off[i + 1]] for i in range(len(off) - 1)]


def _parts(prefix):
    idx, off = G[prefix + "_idx"], G[prefix + "_off"]
    return [idx[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]


PARTS_2014T = _parts("parts2014t")
PARTS79 = _parts("coll_parts")
SAMPLES = _split(G["coll_in"], G["coll_in_off"])
COLLATE = [("train", 5), ("train", 9), ("dev", 0)]


def test_normalize_part_matches_reference():
    for x, want in zip(_split(G["part_in"], G["part_off"]), _split(G["part_out"], G["part_off"])):
        got = O.normalize_part(x)
        assert got.dtype == np.float32
        np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-7)
    for x, want in zip(_split(G["part64_in"], G["part64_off"]), _split(G["part64_out"], G["part64_off"])):
        got = O.normalize_part(x)
        assert got.dtype == np.float64
        np.testing.assert_allclose(got, want, rtol=1e-13, atol=1e-14)


def test_normalize_keypoints_matches_reference():
    got = O.normalize_keypoints(G["norm_in"], PARTS_2014T)
    np.testing.assert_allclose(got, G["norm_out"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("split", ["train", "dev"])
def test_select_frames_matches_reference(split):
    from scattennet_amd import data as D
    train = split == "train"
    max_len = int(G["sel_max_len"])
    for seed in range(4):
        random.seed(seed)
        np.random.seed(seed)
        want = _split(G[f"sel_{split}_{seed}"], G[f"sel_{split}_{seed}_off"])
        for n, w in zip(G["sel_lens"].tolist(), want):
            got = D.select_frames(n, train, max_len, 0.5 if train else 1.0, 1.5 if train else 1.0)
            np.testing.assert_array_equal(got, w)


def _host_pipeline(split, seed):
    """The collator through the host draws of scattennet_amd.data and the oracle arithmetic."""
    from scattennet_amd import data as D
    train = split == "train"
    random.seed(seed)
    np.random.seed(seed)
    kps = []
    for s in SAMPLES:
        frames = D.select_frames(s.shape[0], train, 128, 0.5 if train else 1.0, 1.5 if train else 1.0)
        ops = D.augmentation_draw(train)
        kps.append(O.prepare_sample(s, frames, ops, PARTS79, True))
    return O.collate_keypoints(kps, PARTS79, normalize=False)


@pytest.mark.parametrize("split,seed", COLLATE)
def test_collator_matches_reference(split, seed):
    got = _host_pipeline(split, seed)
    tag = f"coll_{split}_{seed}"
    np.testing.assert_allclose(got["keypoints"], G[tag + "_keypoints"], rtol=0, atol=1e-6)
    for k in ("mask", "valid_len_in", "mask_head"):
        np.testing.assert_array_equal(got[k], G[f"{tag}_{k}"])


@pytest.mark.gpu
@pytest.mark.parametrize("split,seed", COLLATE)
def test_gpu_prepare_batch_matches_reference(split, seed):
    from scattennet_amd import data as D
    random.seed(seed)
    np.random.seed(seed)
    out = D.prepare_batch(SAMPLES, {"max_len": 128, "normalize": True, "joint_parts": PARTS79}, split)
    torch.cuda.synchronize()
    tag = f"coll_{split}_{seed}"
    np.testing.assert_allclose(out["keypoints"].cpu().numpy(), G[tag + "_keypoints"], rtol=0, atol=1e-5)
    for k in ("mask", "valid_len_in", "mask_head"):
        np.testing.assert_array_equal(out[k].cpu().numpy(), G[f"{tag}_{k}"])


@pytest.mark.gpu
def test_gpu_normalize_keypoints_matches_reference():
    from scattennet_amd import data as D
    kp = torch.tensor(G["norm_in"], device="cuda")[None]
    got = D.normalize_keypoints(kp, [kp.shape[1]], PARTS_2014T)
    torch.cuda.synchronize()
    np.testing.assert_allclose(got[0].cpu().numpy(), G["norm_out"], rtol=1e-5, atol=1e-6)
