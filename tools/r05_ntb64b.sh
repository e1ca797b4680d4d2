#!/bin/bash
# variant 45 default: the whole GPU suite, then cfg2 / cfg3 / cfg5 step A/B (SCA_NTB=0: LDS-DMA kernels)
set -o pipefail
O=gpurun_out/ntb64b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for wl in cfg2 cfg3 cfg5; do
    st=20; [ $wl = cfg5 ] && st=8
    for v in 0 1; do
      SCA_NTB=$v timeout -k 10 300 python bench.py --workload $wl --steps $st --no-cpu-baseline > $O/${wl}_${v}_$i.log 2>&1 || exit $?
      echo "${wl} ntb=$v #$i $(grep -o '"value": [0-9.]*' $O/${wl}_${v}_$i.log)"
    done
  done
done
