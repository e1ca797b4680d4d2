"""Input contract: SLR_Dataset.normalize_keypoints and the keypoint
fields of its collator (dataset.py:58-170).

The oracle restatement (oracle/sca_oracle.py:normalize_keypoints) is pinned to the
reference's own dataset.py in tests/test_dataset_golden.py; here it is also checked against
an independent scalar restatement written straight from dataset.py:141-170 and hand-computed
cases, and the HIP kernel (sca_normalize_parts) against the oracle on the GPU (overlapping
parts, several joint layouts).
"""
import numpy as np
import pytest
import torch

from oracle import sca_oracle as O

PARTS_2014T = [list(range(11, 17)), list(range(33, 54)), list(range(54, 75)), list(range(75, 542))]  # yaml


def _scalar_normalize_part(xs, ys):
    """dataset.py:141-170 with Python floats (the arithmetic of the reference on float64)."""
    min_x, min_y, max_x, max_y = min(xs), min(ys), max(xs), max(ys)
    w, h = max_x - min_x, max_y - min_y
    if w > h:
        dx = 0.05 * w
        dy = dx + ((w - h) / 2)
    else:
        dy = 0.05 * h
        dx = dy + ((h - w) / 2)
    s = [max(0, min(min_x - dx, 1)), max(0, min(min_y - dy, 1))]
    e = [max(0, min(max_x + dx, 1)), max(0, min(max_y + dy, 1))]
    if (e[0] - s[0]) != 0.0:
        xs = [(x - s[0]) / (e[0] - s[0]) for x in xs]
    if e[1] - s[1]:
        ys = [(y - s[1]) / (e[1] - s[1]) for y in ys]
    return xs, ys


def _frames(T, K, seed, lo=-0.2, hi=1.2):
    rng = np.random.default_rng(seed)
    kp = rng.uniform(lo, hi, size=(T, K, 2)).astype(np.float32)
    kp[0, 11:17] = 0.5  # degenerate part: zero extent -> unchanged
    if T > 1:
        kp[1, 33:54, 0] = 0.25  # zero width only
    return kp


def test_oracle_matches_scalar_restatement():
    kp = _frames(5, 542, 0)
    got = O.normalize_keypoints(kp, PARTS_2014T)
    for t in range(kp.shape[0]):
        for part in PARTS_2014T:
            xs, ys = _scalar_normalize_part([float(v) for v in kp[t, part, 0]], [float(v) for v in kp[t, part, 1]])
            np.testing.assert_allclose(got[t, part, 0], xs, rtol=2e-5, atol=2e-6)
            np.testing.assert_allclose(got[t, part, 1], ys, rtol=2e-5, atol=2e-6)
    untouched = [k for k in range(542) if not any(k in p for p in PARTS_2014T)]
    np.testing.assert_array_equal(got[:, untouched], kp[:, untouched])


def test_oracle_hand_case():
    # x in [0.2, 0.6] (w 0.4), y in [0.3, 0.4] (h 0.1): dx = 0.02, dy = 0.02 + 0.15 = 0.17
    # s = (0.18, 0.13), e = (0.62, 0.57) -> x' = (x - 0.18) / 0.44, y' = (y - 0.13) / 0.44
    kp = np.array([[[0.2, 0.3], [0.6, 0.4], [0.4, 0.35]]], dtype=np.float32)
    got = O.normalize_keypoints(kp, [[0, 1, 2]])
    np.testing.assert_allclose(got[0, :, 0], (kp[0, :, 0] - 0.18) / 0.44, rtol=1e-5)
    np.testing.assert_allclose(got[0, :, 1], (kp[0, :, 1] - 0.13) / 0.44, rtol=1e-5)


def test_oracle_collate_fields():
    s = [_frames(9, 80, 1), _frames(4, 80, 2), _frames(13, 80, 3)]
    parts = [list(range(10)), list(range(20, 41))]
    c = O.collate_keypoints(s, parts)
    assert c["keypoints"].shape == (3, 13, 80, 2)
    assert c["mask"].tolist()[1] == [1] * 4 + [0] * 9
    assert c["valid_len_in"].tolist() == [2, 1, 3]
    assert c["mask_head"].tolist() == [[1, 1, 0], [1, 0, 0], [1, 1, 1]]
    assert not c["keypoints"][1, 4:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("K,parts", [(542, PARTS_2014T), (79, [list(range(6)), list(range(6, 27)),
                                                               list(range(27, 48)), list(range(48, 79))]),
                                     (40, [[0, 3, 5, 7], [3, 9, 11], list(range(20, 40))])])  # overlapping parts
def test_gpu_normalize_matches_oracle(K, parts):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from scattennet_amd import data as D
    lens = [17, 5, 1, 12]
    samples = [_frames(n, K, 10 + i) for i, n in enumerate(lens)]
    ref = O.collate_keypoints(samples, parts)
    got = D.collate_keypoints(samples, parts, device="cuda")
    torch.cuda.synchronize()
    np.testing.assert_allclose(got["keypoints"].cpu().numpy(), ref["keypoints"], rtol=1e-5, atol=1e-6)
    for k in ("mask", "valid_len_in", "mask_head"):
        np.testing.assert_array_equal(got[k].cpu().numpy(), ref[k])
