#!/bin/bash
# A/B: the hd-32 key-block backward with 128-key blocks and 4 waves (two workgroups per CU)
# against 256-key blocks and 8 waves; tools/lib_kb128.so is the 128 / 4 build
set -o pipefail
O=gpurun_out/kb128; mkdir -p $O
SCA_LIB_PATH=$PWD/tools/lib_kb128.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_attention_shapes.py tests/test_gpu_scale.py tests/test_dropout.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in base kb128; do
  if [ $v = base ]; then e="SCA_X=0"; else e="SCA_LIB_PATH=$PWD/tools/lib_kb128.so"; fi
  env $e timeout -k 10 200 python -u tools/attn_bench.py --T 1024 --hd 32 --B 8 --H 16 --G 4 > $O/attn_$v.log 2>&1 || { tail -5 $O/attn_$v.log; exit 1; }
  echo "== $v"; grep -v "amdgpu.ids" $O/attn_$v.log | tail -6
done
for i in 1 2; do
  for v in base kb128; do
    if [ $v = base ]; then e="SCA_X=0"; else e="SCA_LIB_PATH=$PWD/tools/lib_kb128.so"; fi
    env $e timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/c5_${v}_$i.log 2>&1 || exit $?
    echo "cfg5 $v #$i $(grep -o '"value": [0-9.]*' $O/c5_${v}_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c5_${v}_$i.log)"
  done
done
