#!/bin/bash
# A/B: side-queue kick at the n-th weight-gradient section (SCA_KICK=n) with the last kernels
set -o pipefail
O=gpurun_out/kick; mkdir -p $O
for i in 1 2; do
  for v in 0 2 4; do
    SCA_KICK=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/k${v}_$i.log 2>&1 || exit $?
    echo "kick=$v #$i $(grep -o '"value": [0-9.]*' $O/k${v}_$i.log)"
  done
done
