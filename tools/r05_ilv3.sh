#!/bin/bash
# cfg5 step with variants 43 / 44 as defaults: parity, then A/B against the LDS-DMA kernels
set -o pipefail
O=gpurun_out/ilv3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -q -k cfg5 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/scale.log 2>&1; rc=$?; tail -1 $O/scale.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in off def; do
    case $v in off) e="SCA_NTB=0 SCA_TNB_MIN_K=0";; def) e="SCA_NTB=1";; esac
    env $e timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/${v}_$i.log 2>&1 || exit $?
    echo "${v}_$i $(grep -o '"value": [0-9.]*' $O/${v}_$i.log)"
  done
done
