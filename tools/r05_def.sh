#!/bin/bash
# new GEMM defaults (variants 43 / 44 / 45 / 46): the whole GPU suite, then step A/B per workload:
# old = SCA_NTB=0 SCA_TNR=0 (LDS-DMA kernels), new = defaults
set -o pipefail
O=gpurun_out/def1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for wl in cfg2 cfg3 cfg5; do
    st=20; [ $wl = cfg5 ] && st=8
    for v in old new; do
      case $v in old) e="SCA_NTB=0 SCA_TNR=0";; new) e="SCA_NTB=1";; esac
      env $e timeout -k 10 300 python bench.py --workload $wl --steps $st --no-cpu-baseline > $O/${wl}_${v}_$i.log 2>&1 || exit $?
      echo "${wl} $v #$i $(grep -o '"value": [0-9.]*' $O/${wl}_${v}_$i.log)"
    done
  done
done
