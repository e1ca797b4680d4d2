#!/bin/bash
set -o pipefail
O=gpurun_out/lnbm2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_ln.py tests/test_gpu_lnb.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for wl in cfg2 cfg3; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --no-cpu-baseline > $O/${wl}.log 2>&1 || exit $?
  echo "${wl} $(grep -o '"value": [0-9.]*' $O/${wl}.log)"
done
