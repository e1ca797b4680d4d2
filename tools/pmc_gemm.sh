#!/bin/bash
# PMC counters of the GEMM microbenchmark (separate --pmc passes; no trace domains mixed in).
export TMPDIR=/tmp
out=gpurun_out/pmc_gemm
mkdir -p $out
ARGS="tools/gemm_bench.py --iters 10 --rounds 1 --no-check --cases ${CASES:-qkv} --tiles ${TILES:-1}"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $out -o p1 -- python3 $ARGS > $out/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_WAVES --output-format csv -d $out -o p2 -- python3 $ARGS > $out/p2.log 2>&1 || exit $?
ls $out
