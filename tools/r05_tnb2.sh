#!/bin/bash
# A/B: variant 43 (128x128 TN, interleaved) compiled for two workgroups per CU (252 VGPRs, no
# AGPR spill) against one (264 registers) — tools/lib_tnb2.so is the two-per-CU build
set -o pipefail
O=gpurun_out/tnb2; mkdir -p $O
for v in base two; do
  if [ $v = base ]; then e="SCA_X=0"; else e="SCA_LIB_PATH=$PWD/tools/lib_tnb2.so"; fi
  env $e timeout -k 10 300 python -u tools/tn_library_compare.py --only cfg5 --tnb-tiles 43 --splits 1,2,3,4 \
    --ksplit-tiles 46 --ksplit-splits 2 > $O/cmp_$v.log 2>&1 || { tail -5 $O/cmp_$v.log; exit 1; }
  echo "== $v"; grep " us " $O/cmp_$v.log
done
for i in 1 2; do
  for v in base two; do
    if [ $v = base ]; then e="SCA_X=0"; else e="SCA_LIB_PATH=$PWD/tools/lib_tnb2.so"; fi
    env $e timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/c5_${v}_$i.log 2>&1 || exit $?
    echo "cfg5 $v #$i $(grep -o '"value": [0-9.]*' $O/c5_${v}_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c5_${v}_$i.log)"
  done
done
