"""Summarise a rocprofv3 kernel_stats.csv: per-kernel share of GPU time (per step)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total GPU time {tot / 1e6:.2f} ms  ({tot / 1e6 / steps:.3f} ms per step over {steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:60]
    t = float(r["TotalDurationNs"])
    print(f"{name:60s} calls={int(r['Calls']):6d} avg_us={float(r['AverageNs']) / 1e3:8.2f} "
          f"ms/step={t / 1e6 / steps:7.3f} {100 * t / tot:5.1f}%")
