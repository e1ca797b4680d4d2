#!/bin/bash
# MFMA utilisation and HBM traffic of every kernel of the bench step (north_star: "rocprof
# showing achieved HBM GB/s and MFMA utilisation against gfx950 peak").  Separate rocprofv3
# passes (counter limits per block, MI355X_MICROARCH.md), kernel-trace durations from a
# plain --stats pass; tools/util_summary.py joins them -> <out>/summary.txt.
#   bash tools/pmc_util.sh <name> [bench args...]
export TMPDIR=/tmp
name=${1:-pmc_util}; shift
out=gpurun_out/$name
mkdir -p $out
ARGS="bench.py --steps 3 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o trace -- python3 $ARGS > $out/trace.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $out -o sq -- python3 $ARGS > $out/sq.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out -o fetch -- python3 $ARGS > $out/fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out -o write -- python3 $ARGS > $out/write.log 2>&1 || exit $?
python3 tools/util_summary.py $out
