#!/bin/bash
set -o pipefail
O=gpurun_out/w4; mkdir -p $O
SCA_LNW4=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_ln.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_dropout.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  SCA_LNW4=$v timeout -k 10 200 python -u tools/gemm_ln_bench.py > $O/ln_$v.log 2>&1 || exit $?
  echo "== w4=$v"; grep -v "^$\|amdgpu.ids" $O/ln_$v.log | tail -6
done
for i in 1 2; do
  for wl in cfg2 cfg3; do
    for v in 0 1; do
      SCA_LNW4=$v timeout -k 10 300 python bench.py --workload $wl --steps 20 --no-cpu-baseline > $O/${wl}_${v}_$i.log 2>&1 || exit $?
      echo "${wl} w4=$v #$i $(grep -o '"value": [0-9.]*' $O/${wl}_${v}_$i.log)"
    done
  done
done
