#!/bin/bash
# Kernel trace + PMC counters of the attention microbenchmark (separate passes).
export TMPDIR=/tmp
out=gpurun_out/pmc_attn${TAG}
mkdir -p $out
ARGS="tools/attn_bench.py --iters 5 --no-check ${ATTN_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o kt -- python3 $ARGS > $out/kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES --output-format csv -d $out -o p1 -- python3 $ARGS > $out/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_SALU --output-format csv -d $out -o p2 -- python3 $ARGS > $out/p2.log 2>&1 || exit $?
ls $out
