#!/bin/bash
set -o pipefail
O=gpurun_out/lnr; mkdir -p $O
SCA_LIB_PATH=$PWD/tools/lib_lnr32.so timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -q -k cfg5 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base 16 32; do
    if [ $v = base ]; then e="SCA_X=0"; else e="SCA_LIB_PATH=$PWD/tools/lib_lnr$v.so"; fi
    env $e timeout -k 10 300 python bench.py --workload cfg5 --steps 8 --no-cpu-baseline > $O/${v}_$i.log 2>&1 || exit $?
    echo "cfg5 lnrows=$v #$i $(grep -o '"value": [0-9.]*' $O/${v}_$i.log)"
  done
done
