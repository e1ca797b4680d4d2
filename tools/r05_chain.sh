#!/bin/bash
set -o pipefail
O=gpurun_out/chain; mkdir -p $O
for i in 1 2; do
  for wl in cfg2 cfg3; do
    for v in 1 0; do
      SCA_CHAIN=$v timeout -k 10 300 python bench.py --workload $wl --steps 20 --no-cpu-baseline > $O/${wl}_${v}_$i.log 2>&1 || exit $?
      echo "${wl} chain=$v #$i $(grep -o '"value": [0-9.]*' $O/${wl}_${v}_$i.log)"
    done
  done
done
