"""One step of a rocprofv3 kernel trace in start order (tools/prof_bench.sh output): start and
end offsets from the step's marker kernel, duration, and how many other kernels overlap it.

    python tools/step_listing.py gpurun_out/<dir>/run_kernel_trace.csv [marker] [step_from_end]
"""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "coord_map_fwd"
back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
reg = rows[idx[-1 - back]:idx[-back]]
t0 = int(reg[0]["Start_Timestamp"])
iv = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Queue_Id"],
       r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40])
      for r in reg]
for a, b, q, n in iv:
    ov = sum(1 for a2, b2, _, _ in iv if a2 < b and b2 > a) - 1
    print(f"{a / 1e3:8.1f} {b / 1e3:8.1f} {(b - a) / 1e3:7.1f}  ov{ov}  q{q}  {n}")
