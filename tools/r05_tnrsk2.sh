#!/bin/bash
# split-K of variant 46 forced to 2 / 4 for every weight gradient vs the rule (4 for the FFN shapes, 2 else)
set -o pipefail
O=gpurun_out/tnrsk2; mkdir -p $O
for i in 1 2; do
  for v in 0 2 4; do
    SCA_TNR_SK=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/sk${v}_$i.log 2>&1 || exit $?
    echo "cfg2 sk=$v #$i $(grep -o '"value": [0-9.]*' $O/sk${v}_$i.log)"
  done
done
for v in 0 2; do
  SCA_TNR_SK=$v timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/c3sk${v}.log 2>&1 || exit $?
  echo "cfg3 sk=$v $(grep -o '"value": [0-9.]*' $O/c3sk${v}.log)"
done
