#!/bin/bash
# the float4 many-row reduction (reduce_rows_vec_kernel): kernel-level tests, then config 5 / 2 A/B
set -o pipefail
O=gpurun_out/redvec; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_reduce.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    SCA_REDUCE_VEC=$v timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/c5_${v}_$i.log 2>&1 || exit $?
    echo "cfg5 vec=$v #$i $(grep -o '"value": [0-9.]*' $O/c5_${v}_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c5_${v}_$i.log)"
  done
done
for v in 1 0; do
  SCA_REDUCE_VEC=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/c2_${v}.log 2>&1 || exit $?
  echo "cfg2 vec=$v $(grep -o '"value": [0-9.]*' $O/c2_${v}.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c2_${v}.log)"
done
