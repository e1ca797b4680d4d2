#!/bin/bash
# bench A/B of attribute overrides (tools/bench_var.py), alternated ${REPS:-2}x, config 2 (or
# BENCH_EXTRA):   bash tools/bench_ab.sh "" "ops._FAN_OUT=False"
mkdir -p gpurun_out
for i in $(seq ${REPS:-2}); do
  for v in "$@"; do
    timeout -k 10 300 python tools/bench_var.py $v -- --steps ${STEPS:-40} --no-cpu-baseline ${BENCH_EXTRA} > gpurun_out/bab.log 2>&1 || { tail -5 gpurun_out/bab.log; exit 1; }
    echo "[$v] $(grep -o '"value": [0-9.]*' gpurun_out/bab.log) $(grep -o '"ms_per_step_median": [0-9.]*' gpurun_out/bab.log)"
  done
done
