#!/bin/bash
set -o pipefail
O=gpurun_out/res; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention_shapes.py tests/test_gpu_parity.py tests/test_dropout.py tests/test_masks.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  SCA_ATTN_RES=$v timeout -k 10 120 python tools/attn_bench.py > $O/ab_$v.log 2>&1 || exit $?
  echo "res=$v"; grep "fwd\|err" $O/ab_$v.log
done
for i in 1 2; do
  for wl in cfg2 cfg3; do
    for v in 0 1; do
      SCA_ATTN_RES=$v timeout -k 10 300 python bench.py --workload $wl --steps 20 --no-cpu-baseline > $O/${wl}_${v}_$i.log 2>&1 || exit $?
      echo "${wl} res=$v #$i $(grep -o '"value": [0-9.]*' $O/${wl}_${v}_$i.log)"
    done
  done
done
