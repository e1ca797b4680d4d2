#!/bin/bash
set -o pipefail
O=gpurun_out/lnprio; mkdir -p $O
for i in 1 2; do
  for v in 0 1; do
    SCA_LN_PRIO=$v timeout -k 10 300 python bench.py --workload cfg5 --steps 8 --no-cpu-baseline > $O/p${v}_$i.log 2>&1 || exit $?
    echo "cfg5 ln_prio=$v #$i $(grep -o '"value": [0-9.]*' $O/p${v}_$i.log)"
  done
done
