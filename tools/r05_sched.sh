#!/bin/bash
# schedule A/Bs with the round's last kernels: graph queues 2 (default) / 3, and the weight
# gradients on the main stream (no side stream, no fork markers)
set -o pipefail
O=gpurun_out/sched; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/base_$i.log 2>&1 || exit $?
  echo "base #$i $(grep -o '"value": [0-9.]*' $O/base_$i.log)"
  DEBUG_HIP_FORCE_GRAPH_QUEUES=3 timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/gq3_$i.log 2>&1 || exit $?
  echo "gq3 #$i $(grep -o '"value": [0-9.]*' $O/gq3_$i.log)"
  timeout -k 10 300 python tools/bench_var.py "ops._WGRAD_SIDE = False" -- --steps 20 --no-cpu-baseline > $O/noside_$i.log 2>&1 || exit $?
  echo "noside #$i $(grep -o '"value": [0-9.]*' $O/noside_$i.log)"
done
