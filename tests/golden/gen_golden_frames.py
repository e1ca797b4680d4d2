"""Golden vectors at frame counts that are not multiples of 4 / 16, from the REFERENCE.

The collator pads a batch to its longest clip (dataset.py:76-89), so real batches reach the
encoder at any T; the residual network's MaxPool1d(2, 2) floors odd lengths and the fusion
then sees T/4 (2014T: two pools) or T/2 (2014: one pool) frames.  Fixtures:
  fusion_T45  CoordinatesFusion at T/4 = 45 (the reference's own fusion smoke uses
              (32, 45, 512), model/fusion.py:81-88; smaller widths here, same frame count)
  fusion_T13  CoordinatesFusion at an odd T/4 = 13, B = 3
  residual_64_64_T45  ResidualNetwork([64, 64]) at odd T = 45 (one pool: 22 frames)

Runs ONLY in the build container (imports /root/reference); adds to manifest.json.
Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_frames.py
"""
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import capture, randomize_params  # noqa: E402  (imports the reference's model package)
from model.fusion import CoordinatesFusion  # noqa: E402
from model.residual import ResidualNetwork  # noqa: E402


def main():
    torch.set_num_threads(1)
    mpath = os.path.join(HERE, "manifest.json")
    man = json.load(open(mpath))
    for B, T4, seed in ((2, 45, 18), (3, 13, 19)):
        torch.manual_seed(0)
        m = CoordinatesFusion(32, 64, 0.2)
        randomize_params(m, seed)
        g = torch.Generator().manual_seed(seed)
        inp = {k: torch.randn(B, T4, 32, generator=g) for k in ("left", "right", "body")}
        name, meta = capture(f"fusion_T{T4}", m, inp, lambda mod, i: mod(i["left"], i["right"], i["body"]),
                             {"op": "CoordinatesFusion", "in": 32, "out": 64, "B": B, "T": T4,
                              "ref": "model/fusion.py:6-78"}, ("left", "right", "body"))
        man["fixtures"][name] = meta
    torch.manual_seed(0)
    m = ResidualNetwork([64, 64])
    randomize_params(m, 20)
    inp = {"x": torch.randn(3, 45, 64, generator=torch.Generator().manual_seed(20))}
    name, meta = capture("residual_64_64_T45", m, inp, lambda mod, i: mod(i["x"])[0],
                         {"op": "ResidualNetwork", "blocks": [64, 64], "B": 3, "T": 45,
                          "ref": "model/residual.py:48-118"}, ("x",))
    man["fixtures"][name] = meta
    json.dump(man, open(mpath, "w"), indent=1)


if __name__ == "__main__":
    main()
