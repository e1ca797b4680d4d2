#!/bin/bash
# MFMA utilisation per kernel of a short bench run (north_star: "rocprof showing ... MFMA
# utilisation"): a kernel-trace --stats pass and one SQ counter pass (SQ_VALU_MFMA_BUSY_CYCLES,
# wave states, GRBM_GUI_ACTIVE; counter passes serialise dispatches, so these are the kernels
# alone), joined by tools/util_summary.py -> gpurun_out/$1/{summary.txt,util.json}.
#   BENCH_EXTRA="--workload cfg3" bash tools/pmc_sq.sh <name>
export TMPDIR=/tmp
out=gpurun_out/${1:-pmc_sq}
mkdir -p $out
python3 -c "from scattennet_amd import _lib; print(_lib.source_digest())" > $out/digest.txt
ARGS="bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_EXTRA}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o trace -- python3 $ARGS > $out/trace.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $out -o sq -- python3 $ARGS > $out/sq.log 2>&1 || exit $?
python3 tools/util_summary.py $out > /dev/null
head -12 $out/summary.txt
