#!/bin/bash
# the split rule with the FFN-size condition: config 3 / 2 against the forced settings
set -o pipefail
O=gpurun_out/tnrrule; mkdir -p $O
for i in 1 2; do
  for v in 0 4; do
    SCA_TNR_SK=$v timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/c3sk${v}_$i.log 2>&1 || exit $?
    echo "cfg3 sk=$v #$i $(grep -o '"value": [0-9.]*' $O/c3sk${v}_$i.log)"
  done
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/c2_$i.log 2>&1 || exit $?
  echo "cfg2 rule #$i $(grep -o '"value": [0-9.]*' $O/c2_$i.log)"
done
