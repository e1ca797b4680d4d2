"""Per-kernel HBM traffic per launch from tools/pmc_traffic.sh output:
bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 averaged over dispatches (MI355X_MICROARCH.md
§HBM: gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads; WRITE_SIZE exact).
Writes <dir>/traffic.json."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/*counter_collection.csv"):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    for (disp, cname), v in per.items():
        acc[names[disp].split("(")[0]][cname].append(v)
out = {}
for k, c in acc.items():
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fk = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        wk = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        out[k] = {"fetch_kib": fk, "write_kib": wk, "bytes_per_launch": (2 * fk + wk) * 1024,
                  "dispatches": len(c["FETCH_SIZE"])}
json.dump(out, open(f"{d}/traffic.json", "w"), indent=1)
for k, v in sorted(out.items(), key=lambda kv: -kv[1]["bytes_per_launch"])[:12]:
    print(f"{k:45s} {v['bytes_per_launch'] / 1e6:9.2f} MB/launch  ({v['dispatches']} dispatches)")
