#!/bin/bash
# the stand-alone LayerNorms' affine reductions deferred too (LayerNormAdd: config 5's d = 512
# post-LNs, the residual network's LayerNorms): GPU tests touching them, then config 5 / 3 / 2 A/B
set -o pipefail
O=gpurun_out/aff2; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dp.py tests/test_dropout.py tests/test_gpu_precision.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    SCA_AFFINE_DEFER=$v timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/c5_${v}_$i.log 2>&1 || exit $?
    echo "cfg5 defer=$v #$i $(grep -o '"value": [0-9.]*' $O/c5_${v}_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c5_${v}_$i.log)"
  done
done
for v in 1 0; do
  SCA_AFFINE_DEFER=$v timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/c3_${v}.log 2>&1 || exit $?
  echo "cfg3 defer=$v $(grep -o '"value": [0-9.]*' $O/c3_${v}.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c3_${v}.log)"
  SCA_AFFINE_DEFER=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/c2_${v}.log 2>&1 || exit $?
  echo "cfg2 defer=$v $(grep -o '"value": [0-9.]*' $O/c2_${v}.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c2_${v}.log)"
done
