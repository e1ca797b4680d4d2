"""Per-dispatch PMC summary of a rocprofv3 counter_collection.csv (grouped by kernel and dispatch)."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:48], r["Dispatch_Id"])
        agg.setdefault(key, {})
        agg[key][r["Counter_Name"]] = agg[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seen = collections.Counter()
    for (name, disp), c in agg.items():
        seen[name] += 1
        if seen[name] > int(__import__("os").environ.get("PMC_MAX", "2")):
            continue
        print(path.split("/")[-1], name, disp, " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
