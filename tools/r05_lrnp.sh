#!/bin/bash
set -o pipefail
O=gpurun_out/lrnp; mkdir -p $O
for v in base 2 6; do
  if [ $v = base ]; then e="SCA_X=0"; else e="SCA_LIB_PATH=$PWD/tools/lib_np$v.so"; fi
  env $e timeout -k 10 200 python -u tools/gemm_ln_bench.py > $O/ln_$v.log 2>&1 || exit $?
  env $e timeout -k 10 200 python -u tools/lnb_bench.py > $O/lnb_$v.log 2>&1 || exit $?
  echo "== npre=$v"; grep -v "^$\|amdgpu.ids" $O/ln_$v.log | sed -n 3,4p; grep -v "^$\|amdgpu.ids" $O/lnb_$v.log | grep gemm_lnb
done
for i in 1 2; do
  for v in base 2 6; do
    if [ $v = base ]; then e="SCA_X=0"; else e="SCA_LIB_PATH=$PWD/tools/lib_np$v.so"; fi
    env $e timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/cfg2_${v}_$i.log 2>&1 || exit $?
    echo "cfg2 npre=$v #$i $(grep -o '"value": [0-9.]*' $O/cfg2_${v}_$i.log)"
  done
done
