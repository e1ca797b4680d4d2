"""The sample pipeline of SLR_Dataset.data_collator (SURVEY.md §8(f) rank 3 remainder):
the on-disk sample format (dataset.py:40-56), frame selection (:185-215), augmentation
(:124-132, 172-183; augmentation.py), normalisation and padding — scattennet_amd.data.

* augmentation: the oracle's rotate / flip are pinned to vectors produced by the
  reference's own augmentation.py (tests/golden/gen_golden_augment.py); the composed
  per-clip affine the kernel applies is checked against them;
* frame selection and the augmentation draw: pinned to the reference's own dataset.py in
  tests/test_dataset_golden.py (seeded select_frames sequences, whole collator batches);
  here also against a scalar restatement of the reference's RNG call sequence (same seeds
  -> same draws), and for the properties the reference asserts;
* the GPU launch (sca_prepare_keypoints): against the oracle pipeline (oracle.prepare_sample)
  with the same decisions, fp32 (the reference rotates in float64: rounding-level
  differences, bound 1e-5 absolute on [0, 1] coordinates).
"""
import os
import pickle
import random

import numpy as np
import pytest
import torch

from oracle import sca_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
PARTS = [list(range(0, 6)), list(range(6, 27)), list(range(27, 48)), list(range(48, 75))]


def _golden():
    return np.load(os.path.join(HERE, "golden", "augment.npz"))


def test_oracle_augmentation_matches_reference_vectors():
    g = _golden()
    for a, want in zip(g["angles"], g["rotated"]):
        np.testing.assert_allclose(O.rotate_keypoints(g["kp"], a), want, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(O.flip_keypoints(g["kp"]), g["flipped"])
    np.testing.assert_allclose(O.flip_keypoints(O.rotate_keypoints(g["kp"], 9.0)), g["rot_then_flip"],
                               rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("ops", [[("rot", -7.25)], [("flip",)], [("rot", 9.0), ("flip",)], []])
def test_composed_affine_matches_reference_vectors(ops):
    from scattennet_amd import data as D
    g = _golden()
    kp = g["kp"].astype(np.float64)
    want = kp
    for op in ops:
        want = O.rotate_keypoints(want, op[1]) if op[0] == "rot" else O.flip_keypoints(want)
    m = D.augmentation_affine(ops)
    if not ops:
        assert m is None
        return
    got = kp @ m[:, :2].T + m[:, 2]
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)
    if ops == [("rot", 9.0), ("flip",)]:
        np.testing.assert_allclose(got, g["rot_then_flip"], rtol=1e-12, atol=1e-12)


def _scalar_select(n, train, max_len, min_rate, max_rate):
    """dataset.py:185-215, restated statement by statement (same RNG calls, same order)."""
    if not train:
        idx = list(range(n))
        if n > max_len:
            f_s = (n - max_len) // 2
            f_e = n - max_len - f_s
            idx = idx[f_s:-f_e]
        return idx
    lo = min(int(min_rate * n), max_len)
    hi = min(int(max_rate * n), max_len)
    tgt = random.randint(lo, hi + 1)
    if tgt <= n:
        return sorted(np.random.permutation(np.arange(n))[:tgt].tolist())
    copy = np.random.randint(0, n, tgt - n)
    return sorted(np.concatenate([np.arange(n), copy]).tolist())


def _scalar_augment_ops():
    """dataset.py:127-128, 172-183: the draw sequence (ops, not the arithmetic)."""
    if not np.random.rand() < 0.5:
        return []
    while True:
        ops = []
        if np.random.uniform(0, 1) < 0.5:
            ops.append(("rot", float(np.random.uniform(-15, 15))))
        if np.random.uniform(0, 1) < 0.5:
            ops.append(("flip",))
        if ops:
            return ops


@pytest.mark.parametrize("train", [True, False])
def test_selection_and_draws_follow_the_reference_rng_sequence(train):
    from scattennet_amd import data as D
    lens = [3, 17, 64, 200, 401, 1]
    for seed in range(6):
        random.seed(seed)
        np.random.seed(seed)
        mine = []
        for n in lens:
            mine.append((D.select_frames(n, train, 256, 0.5 if train else 1.0, 1.5 if train else 1.0).tolist(),
                         D.augmentation_draw(train)))
        random.seed(seed)
        np.random.seed(seed)
        ref = []
        for n in lens:
            ref.append((_scalar_select(n, train, 256, 0.5 if train else 1.0, 1.5 if train else 1.0),
                        _scalar_augment_ops() if train else []))
        assert mine == ref
    for sel, _ in mine:
        assert sel == sorted(sel)


def test_selection_properties():
    from scattennet_amd import data as D
    assert D.select_frames(300, False, 256).tolist() == list(range(22, 278))  # centred window
    assert D.select_frames(100, False, 256).tolist() == list(range(100))
    random.seed(1)
    np.random.seed(1)
    for n in (1, 10, 255, 256, 900):
        idx = D.select_frames(n, True, 256)
        lo, hi = min(int(0.5 * n), 256), min(int(1.5 * n), 256)
        assert lo <= len(idx) <= hi + 1  # random.randint(lo, hi + 1), inclusive (0 frames possible at n = 1)
        assert len(idx) == 0 or (idx.min() >= 0 and idx.max() < n)


def test_prepare_batch_rejects_bad_sample_shapes():
    from scattennet_amd import data as D
    cfg = {"max_len": 16, "normalize": False, "joint_parts": PARTS}
    bad = [[np.zeros((5, 75, 4), np.float32)],  # load_sample's [:, :, :-2] trim skipped
           [np.zeros((5, 75, 2), np.float32), np.zeros((5, 74, 2), np.float32)],  # mixed K_all
           [np.zeros((75, 2), np.float32)], []]
    for samples in bad:
        with pytest.raises(ValueError):
            D.prepare_batch(samples, cfg, "dev", device="cpu")


def test_load_sample_format(tmp_path):
    from scattennet_amd import data as D
    kp = np.random.default_rng(0).uniform(size=(12, 75, 4)).astype(np.float32)
    for extra in ({"name": "clip_a"}, {"id": "clip_b"}, {}):
        path = tmp_path / f"s{len(extra)}.pkl"
        with open(path, "wb") as f:  # a file written here (the test's own data)
            pickle.dump(dict({"keypoints": kp, "gloss": "  A  B C  "}, **extra), f)
        k, gloss, name = D.load_sample(str(path))
        np.testing.assert_array_equal(k, kp[:, :, :2])
        assert gloss == "A B C"  # "  A  B C  ".replace("  ", " ").strip()
        assert name == extra.get("name", extra.get("id", ""))


@pytest.mark.gpu
@pytest.mark.parametrize("split,normalize", [("train", True), ("dev", True), ("train", False)])
def test_prepare_batch_vs_oracle(split, normalize):
    from scattennet_amd import data as D
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    rng = np.random.default_rng(3)
    samples = [rng.uniform(-0.05, 1.05, size=(n, 75, 2)).astype(np.float32) for n in (40, 300, 7, 128)]
    cfg = {"max_len": 256, "normalize": normalize, "joint_parts": PARTS}
    random.seed(11)
    np.random.seed(11)
    out = D.prepare_batch(samples, cfg, split)
    torch.cuda.synchronize()
    kp = out["keypoints"].cpu().numpy()
    lens = [len(f) for f in out["frames"]]
    assert kp.shape == (4, max(lens), 75, 2)
    if split == "train":
        assert any(out["augment"])  # this seed draws at least one augmentation
    for b, s in enumerate(samples):
        want = O.prepare_sample(s, out["frames"][b], out["augment"][b], PARTS, normalize)
        np.testing.assert_allclose(kp[b, :lens[b]], want, rtol=0, atol=1e-5)
        assert not kp[b, lens[b]:].any()  # collator padding
    assert out["mask"].sum(1).tolist() == lens
    assert out["valid_len_in"].tolist() == [n // 4 for n in lens]
