"""Speed equivalence of the CPU baseline's restatement (oracle/) and the reference itself
(BASELINE.md "Restatement vs reference"), timed in the BUILD container where
`/root/reference` is importable — the reference never runs on the GPU box, where bench.py's
cpu_baseline times the restatement.  Same weights and inputs for both; the outputs are
compared too.  Writes profiles/ref_vs_oracle.json.

    PYTHONDONTWRITEBYTECODE=1 python tools/ref_vs_oracle.py
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gen_golden_xstream as GX  # noqa: E402  (puts /root/reference on sys.path)
from model.keypoint_module import SeparativeCoordinateAttention  # noqa: E402
from model.layers import CoordinateMapping  # noqa: E402

from oracle import sca_oracle as O  # noqa: E402
from scattennet_amd import workloads as W  # noqa: E402


def median_time(fn, iters, warm=1):
    ts = []
    for i in range(warm + iters):
        t0 = time.perf_counter()
        fn()
        if i >= warm:
            ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


class RefStream(torch.nn.Module):
    def __init__(self, K, cfg):
        super().__init__()
        self.coordinate_mapping = CoordinateMapping(K, cfg["d_model"])
        self.sca = SeparativeCoordinateAttention(cfg)

    def forward(self, kp, mask):
        x, y = self.coordinate_mapping(kp[:, :, :, 0], kp[:, :, :, 1])
        return self.sca(x, y, mask)


def cfg1(threads):
    w = W.WORKLOADS["cfg1"]
    cfg = dict(W.model_cfg(w["d"], w["H"], w["L"], maxpos=w["maxpos"]), dropout=0.0)
    torch.manual_seed(0)
    ref = GX.XStream(w["K_all"], cfg).eval()
    W.init_like_msca(ref)
    p = {k: v.detach().clone().requires_grad_(True) for k, v in ref.state_dict().items()}
    kp, mask, _ = W.synthetic_batch(w, "cpu", seed=1)
    g = torch.randn(w["B"], w["T"], w["d"], generator=torch.Generator().manual_seed(1))

    def run_ref():
        ref.zero_grad(set_to_none=True)
        (ref(kp, mask) * g).sum().backward()

    def run_or():
        for v in p.values():
            v.grad = None
        (O.x_stream(p, "", kp, mask, cfg) * g).sum().backward()

    err = float((ref(kp, mask) - O.x_stream(p, "", kp, mask, cfg)).abs().max())
    torch.set_num_threads(threads)
    return {"reference_ms": 1e3 * median_time(run_ref, 9, 2), "oracle_ms": 1e3 * median_time(run_or, 9, 2),
            "max_abs_out_diff": err}


def cfg2(threads, B):
    w = dict(W.WORKLOADS["cfg2"], B=B)
    cfg = dict(W.model_cfg(w["d"], w["H"], w["L"], maxpos=w["maxpos"]), dropout=0.0)
    groups = W.split_groups(w["groups"])
    torch.manual_seed(0)
    refs = [RefStream(len(gi), cfg).eval() for gi in groups]
    for r in refs:
        W.init_like_msca(r)
    plist = [{k: v.detach().clone().requires_grad_(True) for k, v in r.state_dict().items()} for r in refs]
    kp, mask, gout = W.synthetic_batch(w, "cpu", seed=1)

    def run_ref():
        outs = [r(kp[:, :, gi, :], mask) for r, gi in zip(refs, groups)]
        torch.autograd.backward(outs, [gout[i] for i in range(len(outs))])
        for r in refs:
            r.zero_grad(set_to_none=True)

    def run_or():
        outs = O.multi_stream_sca(plist, kp, mask, groups, cfg)
        torch.autograd.backward(outs, [gout[i] for i in range(len(outs))])
        for p in plist:
            for v in p.values():
                v.grad = None

    with torch.no_grad():
        a = refs[0](kp[:, :, groups[0], :], mask)
        b = O.multi_stream_sca(plist[:1], kp, mask, groups[:1], cfg)[0]
    torch.set_num_threads(threads)
    return {"B": B, "reference_ms": 1e3 * median_time(run_ref, 3), "oracle_ms": 1e3 * median_time(run_or, 3),
            "max_abs_out_diff": float((a - b).abs().max())}


def main():
    threads = os.cpu_count() or 1
    res = {"host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(" :\t"),
           "threads": threads, "torch": torch.__version__}
    res["cfg1_threads"] = cfg1(threads)
    res["cfg1_1thread"] = cfg1(1)
    res["cfg2_threads"] = cfg2(threads, 8)
    res["cfg2_1thread_1clip"] = cfg2(1, 1)
    for k, v in res.items():
        if isinstance(v, dict):
            v["oracle_over_reference"] = round(v["oracle_ms"] / v["reference_ms"], 3)
    out = os.path.join(ROOT, "profiles", "ref_vs_oracle.json")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
