#!/bin/bash
# config 3: every variant-46 weight gradient forced to split 1 / 3 vs the rule
set -o pipefail
O=gpurun_out/c3sk; mkdir -p $O
for i in 1 2; do
  for v in 0 1 3; do
    SCA_TNR_SK=$v timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/sk${v}_$i.log 2>&1 || exit $?
    echo "cfg3 sk=$v #$i $(grep -o '"value": [0-9.]*' $O/sk${v}_$i.log)"
  done
done
