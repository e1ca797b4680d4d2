#!/bin/bash
# residual block input fanned out (one grouped gradient sum) vs autograd's per-stream adds
set -o pipefail
O=gpurun_out/resfan; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_fanout.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in True False; do
    timeout -k 10 300 python tools/bench_var.py "import scattennet_amd.residual as R; R._FAN_OUT_X = $v" -- \
      --workload cfg3 --steps 20 --no-cpu-baseline > $O/c3_${v}_$i.log 2>&1 || exit $?
    echo "cfg3 fan=$v #$i $(grep -o '"value": [0-9.]*' $O/c3_${v}_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c3_${v}_$i.log)"
  done
done
