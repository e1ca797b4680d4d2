#!/bin/bash
set -o pipefail
O=gpurun_out/kqb; mkdir -p $O
SCA_KBLK_QB=64 timeout -k 10 600 python -u -m pytest tests/test_gpu_attention_shapes.py tests/test_gpu_scale.py tests/test_dropout.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 32 64; do
  SCA_KBLK_QB=$v timeout -k 10 200 python tools/attn_bench.py --T 1024 --hd 32 --H 16 --B 8 --G 4 --iters 10 > $O/ab_$v.log 2>&1 || exit $?
  echo "qb=$v"; grep "bwd\|err" $O/ab_$v.log
done
for i in 1 2; do
  for v in 32 64; do
    SCA_KBLK_QB=$v timeout -k 10 300 python bench.py --workload cfg5 --steps 8 --no-cpu-baseline > $O/cfg5_${v}_$i.log 2>&1 || exit $?
    echo "cfg5 qb=$v #$i $(grep -o '"value": [0-9.]*' $O/cfg5_${v}_$i.log)"
  done
done
