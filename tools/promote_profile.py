"""Promote a rocprofv3 measurement of one bench workload to the files bench.py reads:

    profiles/latest/<workload>_kstats.csv    rocprofv3 --kernel-trace --stats (tools/prof_bench.sh)
    profiles/latest/<workload>_traffic.json  per-launch HBM bytes (tools/pmc_traffic.sh)
    profiles/latest/<workload>_util.json     per-kernel MFMA busy / wave states (tools/pmc_sq.sh)
    profiles/latest/<workload>_meta.json     the library source digest all were measured on

bench.py reports the profile's average launch duration / traffic for its dominant kernel
only when the workload matches and the digest equals the current sources' (no stale
figures).  Run in the build container after the GPU call that wrote <prof_dir> / <pmc_dir>:

    python tools/promote_profile.py <workload> gpurun_out/<set>/prof gpurun_out/<set>/pmc [gpurun_out/<set>/sq]
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from scattennet_amd import _lib  # noqa: E402


def main():
    wl, prof, pmc = sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None
    sq = sys.argv[4] if len(sys.argv) > 4 else None
    out = os.path.join(ROOT, "profiles", "latest")
    os.makedirs(out, exist_ok=True)
    meta = {"workload": wl, "source_digest": _lib.source_digest(), "prof_dir": prof, "pmc_dir": pmc, "sq_dir": sq}
    for d in (prof, pmc, sq):
        p = os.path.join(d, "digest.txt") if d else ""
        if p and os.path.exists(p):  # the digest the GPU run computed on its own tree
            meta["measured_digest"] = open(p).read().strip()
            if meta["measured_digest"] != meta["source_digest"]:
                sys.exit(f"profile {d} was measured on sources {meta['measured_digest']}, "
                         f"the tree is at {meta['source_digest']}")
    stats = glob.glob(os.path.join(prof, "**", "*kernel_stats.csv"), recursive=True)
    if len(stats) != 1:
        sys.exit(f"expected one kernel_stats.csv under {prof}, found {stats}")
    shutil.copy(stats[0], os.path.join(out, f"{wl}_kstats.csv"))
    if pmc:
        shutil.copy(os.path.join(pmc, "traffic.json"), os.path.join(out, f"{wl}_traffic.json"))
    if sq:
        shutil.copy(os.path.join(sq, "util.json"), os.path.join(out, f"{wl}_util.json"))
    json.dump(meta, open(os.path.join(out, f"{wl}_meta.json"), "w"), indent=1)
    print("promoted", meta)


if __name__ == "__main__":
    main()
