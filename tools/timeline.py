"""Per-step concurrency of a rocprofv3 kernel trace (tools/prof_bench.sh output): steps are
delimited by a once-per-step marker kernel; prints wall, idle / 1 / 2+ concurrent time and
each kernel's exclusive ("alone") and shared time per step.

    python tools/timeline.py gpurun_out/<dir>/run_kernel_trace.csv [marker] [first_step]
"""
import collections
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "coord_map_fwd"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
first = int(sys.argv[3]) if len(sys.argv) > 3 else max(0, len(idx) - 9)
# only intervals that are one graph replay: a marker-to-marker interval that also holds the
# warm-up, the capture or the bench's instrumented eager step (host gaps of 0.1-0.7 s) is not
# a step — round 4's "22 ms/step idle" at config 5 was one such interval averaged in
span = [int(rows[idx[k + 1]]["Start_Timestamp"]) - int(rows[idx[k]]["Start_Timestamp"]) for k in range(len(idx) - 1)]
med = sorted(span[first:])[len(span[first:]) // 2] if span[first:] else 0
keep = [k for k in range(first, len(idx) - 1) if span[k] <= 1.25 * med]
dropped = len(idx) - 1 - first - len(keep)
excl, shared, tot, cnt = (collections.Counter() for _ in range(4))
hist = collections.Counter()
walls = []
for k in keep:
    reg = rows[idx[k]:idx[k + 1]]
    t0, t1 = int(reg[0]["Start_Timestamp"]), int(rows[idx[k + 1]]["Start_Timestamp"])
    walls.append(t1 - t0)
    iv = [(int(r["Start_Timestamp"]), min(int(r["End_Timestamp"]), t1),
           r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:44]) for r in reg]
    pts = sorted(set([a for a, _, _ in iv] + [b for _, b, _ in iv] + [t0, t1]))
    for a, b, n in iv:
        tot[n] += b - a
        cnt[n] += 1
    for x, y in zip(pts, pts[1:]):
        act = [n for a, b, n in iv if a <= x and b >= y]
        hist[min(len(act), 3)] += y - x
        if len(act) == 1:
            excl[act[0]] += y - x
        for n in act[1:] if len(act) > 1 else []:
            pass
        if len(act) > 1:
            for n in act:
                shared[n] += (y - x) / len(act)
ns = len(walls)
print(f"({dropped} non-replay interval(s) left out) ", end="")
print(f"{ns} steps, wall {sum(walls) / ns / 1e6:.3f} ms/step; idle {hist[0] / ns / 1e6:.3f}, one kernel "
      f"{hist[1] / ns / 1e6:.3f}, two {hist[2] / ns / 1e6:.3f}, 3+ {hist[3] / ns / 1e6:.3f}")
print(f"{'kernel':44s} {'calls':>5s} {'total':>7s} {'alone':>7s} {'shared/n':>8s}  (ms per step)")
for n, v in sorted(tot.items(), key=lambda x: -x[1])[:24]:
    print(f"{n:44s} {cnt[n] // ns:5d} {v / 1e6 / ns:7.3f} {excl[n] / 1e6 / ns:7.3f} {shared[n] / 1e6 / ns:8.3f}")
