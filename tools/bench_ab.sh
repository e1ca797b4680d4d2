#!/bin/bash
# bench A/B of command-line variants, alternated ${REPS:-2}x, config 2 (or BENCH_EXTRA):
#   bash tools/bench_ab.sh "--x6 none" "--x6 gemm" "--x6 gemm,ln,lnb"
mkdir -p gpurun_out
for i in $(seq ${REPS:-2}); do
  for v in "$@"; do
    timeout -k 10 300 python bench.py --steps ${STEPS:-40} --no-cpu-baseline ${BENCH_EXTRA} $v > gpurun_out/bab.log 2>&1 || { tail -5 gpurun_out/bab.log; exit 1; }
    echo "[$v] $(grep -o '"value": [0-9.]*' gpurun_out/bab.log) $(grep -o '"ms_per_step_median": [0-9.]*' gpurun_out/bab.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/bab.log)"
  done
done
