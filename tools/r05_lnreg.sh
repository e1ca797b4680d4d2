#!/bin/bash
# register-staged main loop in the LayerNorm-fused GEMMs: their tests + parity, then step A/B
set -o pipefail
O=gpurun_out/lnreg; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_ln.py tests/test_gpu_lnb.py tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for wl in cfg2 cfg3; do
    for v in 0 1; do
      SCA_LNREG=$v timeout -k 10 300 python bench.py --workload $wl --steps 20 --no-cpu-baseline > $O/${wl}_${v}_$i.log 2>&1 || exit $?
      echo "${wl} lnreg=$v #$i $(grep -o '"value": [0-9.]*' $O/${wl}_${v}_$i.log)"
    done
  done
done
