#!/bin/bash
# A/B: the LayerNorm affine reductions deferred to one launch at the end of the backward
# (SCA_AFFINE_DEFER=1, default) against one launch per layer (0); the tests that cover them first
set -o pipefail
O=gpurun_out/aff; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_gpu_lnb.py tests/test_gpu_gemm_ln.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    SCA_AFFINE_DEFER=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/c2_${v}_$i.log 2>&1 || exit $?
    echo "cfg2 defer=$v #$i $(grep -o '"value": [0-9.]*' $O/c2_${v}_$i.log)"
  done
done
for v in 1 0; do
  SCA_AFFINE_DEFER=$v timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/c3_${v}.log 2>&1 || exit $?
  echo "cfg3 defer=$v $(grep -o '"value": [0-9.]*' $O/c3_${v}.log)"
done
