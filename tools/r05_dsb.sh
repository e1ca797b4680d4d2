#!/bin/bash
set -o pipefail
O=gpurun_out/dsb; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention_shapes.py tests/test_gpu_parity.py tests/test_dropout.py tests/test_masks.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python tools/attn_bench.py --lib tools/old_lib.so > $O/old_$i.log 2>&1 || exit $?
  timeout -k 10 120 python tools/attn_bench.py > $O/new_$i.log 2>&1 || exit $?
  echo "old"; grep "bwd" $O/old_$i.log; echo "new"; grep "bwd" $O/new_$i.log
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/cfg2_$i.log 2>&1 || exit $?
  echo "cfg2 #$i $(grep -o '"value": [0-9.]*' $O/cfg2_$i.log)"
done
