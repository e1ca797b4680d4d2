#!/bin/bash
# Counters of the weight-gradient kernels alone (tools/tn_bench.py, few variants): where the
# waves of the TN GEMM spend their cycles.  Separate rocprofv3 passes per counter group.
export TMPDIR=/tmp
out=gpurun_out/${1:-tn_pmc}
mkdir -p $out
ARGS="tools/tn_bench.py --iters 3 --rounds 1 --tiles ${TILES:-21,33} --splits ${SPLITS:-1,3}"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o trace -- python3 $ARGS > $out/trace.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $out -o sq -- python3 $ARGS > $out/sq.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --output-format csv -d $out -o lds -- python3 $ARGS > $out/lds.log 2>&1 || exit $?
python3 - $out <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add((f, r["Dispatch_Id"]))
for k, c in acc.items():
    n = len(cnt[k])
    print(k, f"dispatch-passes={n}")
    for name in sorted(c):
        print(f"   {name:26s} {c[name]:16.0f}")
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        print(f"   wait_any {c['SQ_WAIT_ANY']/w:.3f}  wait_inst {c['SQ_WAIT_INST_ANY']/w:.3f}  active {c['SQ_ACTIVE_INST_ANY']/w:.3f}")
        print(f"   mfma busy / (gui/8 * 1024 SIMD) {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
PY
