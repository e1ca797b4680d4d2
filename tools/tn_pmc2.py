"""Per-kernel MFMA busy, wave-state shares and effective clock from one rocprofv3 run with
--kernel-trace and --pmc (SQ counters + GRBM_GUI_ACTIVE) — tools/tn_pmc.sh.

    python tools/tn_pmc2.py <dir>
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
dur = {}
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
per = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
agg = collections.defaultdict(list)
for disp, c in per.items():
    t = dur.get(disp)
    if not t or not c.get("GRBM_GUI_ACTIVE"):
        continue
    clk = c["GRBM_GUI_ACTIVE"] / 8 / t
    simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 1024
    wave = c.get("SQ_WAVE_CYCLES", 0) or 1
    agg[names[disp]].append((t * 1e6, clk / 1e9, c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles,
                             c.get("SQ_WAIT_ANY", 0) / wave, c.get("SQ_WAIT_INST_ANY", 0) / wave,
                             c.get("SQ_ACTIVE_INST_ANY", 0) / wave))
print(f"{'kernel':46s} {'n':>3s} {'us':>8s} {'GHz':>5s} {'mfma':>6s} {'wait':>6s} {'w_inst':>6s} {'active':>6s}")
for k, rows in sorted(agg.items(), key=lambda kv: -sum(r[0] for r in kv[1])):
    n = len(rows)
    m = [sum(r[i] for r in rows) / n for i in range(6)]
    print(f"{k[:46]:46s} {n:3d} {m[0]:8.1f} {m[1]:5.2f} {m[2]:6.3f} {m[3]:6.3f} {m[4]:6.3f} {m[5]:6.3f}")
