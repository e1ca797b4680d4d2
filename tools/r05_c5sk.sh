#!/bin/bash
# config 5: the 128x128 weight-gradient kernel's split forced to 1 / 2 vs the per-CU time model
set -o pipefail
O=gpurun_out/c5sk; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/model_$i.log 2>&1 || exit $?
  echo "cfg5 model #$i $(grep -o '"value": [0-9.]*' $O/model_$i.log)"
  for v in 1 2; do
    timeout -k 10 300 python tools/bench_var.py "ops._tnb_split = lambda K, t: $v" -- --workload cfg5 --steps 10 --no-cpu-baseline > $O/sk${v}_$i.log 2>&1 || exit $?
    echo "cfg5 sk=$v #$i $(grep -o '"value": [0-9.]*' $O/sk${v}_$i.log)"
  done
done
