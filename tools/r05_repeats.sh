#!/bin/bash
# run-to-run spread of the bench lines on one box (5 x config 2, 3 x config 3, 3 x config 5)
set -o pipefail
O=gpurun_out/rep; mkdir -p $O
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/c2_$i.log 2>&1 || exit $?
  echo "cfg2 #$i $(grep -o '"value": [0-9.]*' $O/c2_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c2_$i.log)"
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/c3_$i.log 2>&1 || exit $?
  echo "cfg3 #$i $(grep -o '"value": [0-9.]*' $O/c3_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c3_$i.log)"
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/c5_$i.log 2>&1 || exit $?
  echo "cfg5 #$i $(grep -o '"value": [0-9.]*' $O/c5_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c5_$i.log)"
done
