#!/bin/bash
set -o pipefail
O=gpurun_out/chmin; mkdir -p $O
for i in 1 2; do
  for v in 256 128 64; do
    SCA_CHAIN_MIN_TILES=$v timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/c${v}_$i.log 2>&1 || exit $?
    echo "cfg3 chain_min=$v #$i $(grep -o '"value": [0-9.]*' $O/c${v}_$i.log)"
  done
done
