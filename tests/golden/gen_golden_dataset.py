"""Golden vectors for the input contract, from the REFERENCE's own
dataset.py: SLR_Dataset.normalize_part / normalize_keypoints / select_frames and the
keypoint fields of data_collator (dataset.py:58-217).

Runs ONLY in the build container, where `/root/reference` is importable.  dataset.py's
`import utils as utils` (dataset.py:4) pulls in the reference's utils.py, which needs loguru
(absent in this image); dataset.py never uses the name (its only `utils.` is `torch.utils`
on line 5), so the import is satisfied by an EMPTY module object registered under that name
before `import dataset`.  Every function called below is the reference's own code, unchanged;
SLR_Dataset is instantiated with object.__new__ (its __init__ lists a data directory) and
given the attributes __init__ would set (dataset.py:13-35).  The collator's gloss tokenizer
(out of scope) is a stand-in that returns empty id lists; only the keypoint fields are kept.

Writes `dataset.npz` (inputs and outputs only) and its entry in `manifest.json`.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_dataset.py
"""
import json
import os
import random
import sys
import types

import numpy as np
import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

sys.path.insert(0, REF)
sys.modules.setdefault("utils", types.ModuleType("utils"))  # dataset.py:4, unused by dataset.py
import dataset as ref_dataset  # noqa: E402

# the bench / parity streams' part layout over 79 joints (BASELINE config 2) for the collator cases
PARTS79 = [list(range(0, 6)), list(range(6, 27)), list(range(27, 48)), list(range(48, 79))]


class _NoTokenizer:
    def batch_encode(self, glosses, return_length=True):
        return {"input_ids": [[] for _ in glosses], "length": [0 for _ in glosses]}


def make_dataset(split, joint_parts, max_len, normalize=True):
    ds = object.__new__(ref_dataset.SLR_Dataset)
    ds.cfg = {"max_len": max_len, "normalize": normalize, "joint_parts": joint_parts}
    ds.max_len = max_len
    ds.split = split
    ds.normalize = normalize
    ds.joint_parts = joint_parts
    ds.gloss_tokenizer = _NoTokenizer()
    ds.min_rate, ds.max_rate = (0.5, 1.5) if split == "train" else (1.0, 1.0)
    return ds


def ragged(arrs, dtype):
    off = np.cumsum([0] + [len(a) for a in arrs]).astype(np.int64)
    flat = np.concatenate([np.asarray(a, dtype=dtype).reshape(len(a), *np.shape(a)[1:]) for a in arrs])
    return flat, off


def main():
    cfg = yaml.safe_load(open(os.path.join(REF, "configs", "phoenix-2014t.yaml")))
    parts_t = cfg["data"]["joint_parts"] if "data" in cfg else cfg["dataset"]["joint_parts"]
    max_len_t = (cfg.get("data") or cfg["dataset"])["max_len"]
    out = {}
    man = {}

    # 1. normalize_part on single parts (dataset.py:141-170): random, degenerate (zero
    # extent, zero width, zero height), square extent (w == h), outside [0, 1] (clamping)
    ds = make_dataset("dev", parts_t, max_len_t)
    rng = np.random.default_rng(20)
    cases = []
    for n in (1, 2, 6, 21, 64):
        cases.append(rng.uniform(0.0, 1.0, (n, 2)).astype(np.float32))
        cases.append(rng.uniform(-0.3, 1.3, (n, 2)).astype(np.float32))
    cases.append(np.full((5, 2), 0.5, np.float32))
    z = rng.uniform(0, 1, (7, 2)).astype(np.float32)
    z[:, 0] = 0.25
    cases.append(z)
    z = rng.uniform(0, 1, (7, 2)).astype(np.float32)
    z[:, 1] = 0.75
    cases.append(z)
    cases.append(np.array([[0.1, 0.2], [0.5, 0.6], [0.3, 0.4]], np.float32))  # w == h
    cases.append(np.array([[0.0, 0.0], [1.0, 1.0]], np.float32))  # box clamps to [0, 1] on both axes
    cases.append(np.array([[2.0, -1.0], [3.0, -0.5]], np.float32))  # entirely outside: e - s == 0 on x
    f64 = [c.astype(np.float64) * 0.9 + 0.03 for c in cases[:6]]  # float64 parts (after augmentation)
    res = [ds.normalize_part(c.copy()) for c in cases]
    res64 = [ds.normalize_part(c.copy()) for c in f64]
    out["part_in"], out["part_off"] = ragged(cases, np.float32)
    out["part_out"], _ = ragged(res, np.float32)
    out["part64_in"], out["part64_off"] = ragged(f64, np.float64)
    out["part64_out"], _ = ragged(res64, np.float64)
    assert all(r.dtype == np.float32 for r in res) and all(r.dtype == np.float64 for r in res64)

    # 2. normalize_keypoints over whole frames with the 2014T yaml's joint parts (K_all = 542)
    kp = rng.uniform(-0.1, 1.1, (6, 542, 2)).astype(np.float32)
    kp[0, parts_t[0]] = 0.5  # degenerate part
    kp[1, parts_t[1], 0] = 0.25
    out["norm_in"] = kp.copy()
    out["norm_out"] = ds.normalize_keypoints(kp.copy())
    pflat = [j for p in parts_t for j in p]
    out["parts2014t_idx"] = np.array(pflat, np.int64)
    out["parts2014t_off"] = np.cumsum([0] + [len(p) for p in parts_t]).astype(np.int64)
    out["max_len_2014t"] = np.array(max_len_t)

    # 3. select_frames (dataset.py:185-217): seeded draw sequences, train and evaluation
    lens = [1, 2, 3, 17, 64, 127, 128, 129, 200, 255, 256, 257, 401]
    sel = {}
    for split in ("train", "dev"):
        dsx = make_dataset(split, parts_t, 128)
        for seed in range(4):
            random.seed(seed)
            np.random.seed(seed)
            idx = []
            for n in lens:
                frames = np.arange(n, dtype=np.int64)[:, None, None] * np.ones((1, 1, 2), np.int64)
                got = dsx.select_frames(frames)[:, 0, 0]
                idx.append(np.asarray(got, np.int64))
            sel[(split, seed)] = idx
            out[f"sel_{split}_{seed}"], out[f"sel_{split}_{seed}_off"] = ragged(idx, np.int64)
    out["sel_lens"] = np.array(lens, np.int64)
    out["sel_max_len"] = np.array(128)

    # 4. the collator's keypoint fields (dataset.py:58-122) through preprocess_keypoints
    # (selection, augmentation draw, normalisation), seeded, over 79 joints in the config-2
    # part layout; train (draws) and dev (centred windows), max_len 128
    clip_lens = [40, 200, 7, 128, 90]
    samples = [rng.uniform(-0.05, 1.05, (n, 79, 2)).astype(np.float32) for n in clip_lens]
    out["coll_in"], out["coll_in_off"] = ragged(samples, np.float32)
    out["coll_parts_idx"] = np.array([j for p in PARTS79 for j in p], np.int64)
    out["coll_parts_off"] = np.cumsum([0] + [len(p) for p in PARTS79]).astype(np.int64)
    for split, seed in (("train", 5), ("train", 9), ("dev", 0)):
        dsx = make_dataset(split, PARTS79, 128)
        random.seed(seed)
        np.random.seed(seed)
        batch = [(s.copy(), "G", f"clip{i}") for i, s in enumerate(samples)]
        c = dsx.data_collator(batch)
        tag = f"coll_{split}_{seed}"
        out[tag + "_keypoints"] = c["keypoints"].numpy()
        out[tag + "_mask"] = c["mask"].numpy()
        out[tag + "_valid_len_in"] = c["valid_len_in"].numpy()
        out[tag + "_mask_head"] = c["mask_head"].numpy()
        man[tag] = {"split": split, "seed": seed, "T": int(c["keypoints"].shape[1])}

    np.savez_compressed(os.path.join(HERE, "dataset.npz"), **out)
    mpath = os.path.join(HERE, "manifest.json")
    m = json.load(open(mpath))
    m["fixtures"]["dataset"] = {
        "op": "dataset.py SLR_Dataset.normalize_part / normalize_keypoints / select_frames / data_collator "
              "(keypoint fields)",
        "source": "reference dataset.py, imported (its unused `import utils` satisfied by an empty module)",
        "numpy": np.__version__, "torch": torch.__version__, "collate": man,
        "seeding": "random.seed(s); np.random.seed(s) before each select_frames sequence / collator call"}
    json.dump(m, open(mpath, "w"), indent=1)


if __name__ == "__main__":
    main()
