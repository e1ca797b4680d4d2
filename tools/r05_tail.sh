#!/bin/bash
set -o pipefail
O=gpurun_out/tail; mkdir -p $O
for i in 1 2; do
  for v in 1 0.6 0.4 0.2; do
    SCA_TAIL_FRAC=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/t${v}_$i.log 2>&1 || exit $?
    echo "cfg2 tail_frac=$v #$i $(grep -o '"value": [0-9.]*' $O/t${v}_$i.log)"
  done
done
for v in 1 0.4; do
  SCA_TAIL_FRAC=$v timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/c3_${v}.log 2>&1 || exit $?
  echo "cfg3 tail_frac=$v $(grep -o '"value": [0-9.]*' $O/c3_${v}.log)"
done
