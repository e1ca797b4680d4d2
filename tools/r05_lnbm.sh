#!/bin/bash
set -o pipefail
O=gpurun_out/lnbm; mkdir -p $O
for i in 1 2; do
  for v in 0 32; do
    SCA_GEMM_LN_BM=$v timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/bm${v}_$i.log 2>&1 || exit $?
    echo "cfg3 bm=$v #$i $(grep -o '"value": [0-9.]*' $O/bm${v}_$i.log)"
  done
done
