#!/bin/bash
# variant 41 as the default for the big forward GEMMs: NT kernel tests + cfg5 parity, then the
# cfg5 bench with and without it (SCA_NTB=0), twice each
set -o pipefail
O=gpurun_out/ntb2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_ntb.py tests/test_gpu_gemm_tn.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -q -k cfg5 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/scale.log 2>&1; rc=$?; tail -2 $O/scale.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  SCA_NTB=0 timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/off_$i.log 2>&1 || exit $?
  echo "off_$i $(grep -o '"value": [0-9.]*' $O/off_$i.log)"
  timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/on_$i.log 2>&1 || exit $?
  echo "on_$i $(grep -o '"value": [0-9.]*' $O/on_$i.log)"
done
