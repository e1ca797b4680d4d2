"""Golden vectors for the sample pipeline's augmentation, from the REFERENCE.

Runs ONLY in the build container, where `/root/reference` is importable: the reference's
augmentation.py (numpy only: rotate_keypoints, flip_keypoints) is imported and applied to a
fixed keypoint array; writes `augment.npz` (data only) and its entry in `manifest.json`.
(dataset.py's selection / normalisation / collator vectors: gen_golden_dataset.py.)

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_augment.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")
from augmentation import flip_keypoints, rotate_keypoints  # noqa: E402


def main():
    rng = np.random.default_rng(7)
    kp = rng.uniform(-0.1, 1.1, size=(9, 75, 2)).astype(np.float32)  # (T, K, 2), as dataset.py:46 leaves it
    angles = np.array([-15.0, -7.25, 0.0, 3.5, 14.999], dtype=np.float64)
    rotated = np.stack([rotate_keypoints(kp, (0, 0), a) for a in angles])
    flipped = flip_keypoints(kp)
    rot_then_flip = flip_keypoints(rotate_keypoints(kp, (0, 0), 9.0))
    np.savez(os.path.join(HERE, "augment.npz"), kp=kp, angles=angles, rotated=rotated, flipped=flipped,
             rot_then_flip=rot_then_flip)
    mpath = os.path.join(HERE, "manifest.json")
    man = json.load(open(mpath))
    man["fixtures"]["augment"] = {"op": "augmentation.py rotate_keypoints (origin (0, 0)) / flip_keypoints",
                                  "source": "reference augmentation.py, imported", "angles": angles.tolist(),
                                  "dtypes": {"kp": "float32", "outputs": "float64 (numpy promotion)"}}
    json.dump(man, open(mpath, "w"), indent=1)


if __name__ == "__main__":
    main()
