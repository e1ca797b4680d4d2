#!/bin/bash
# reduced-precision GPU tests, stand-alone LayerNorm bench, NT / NN / GEMM+LN against the
# library, and the config-5 A/B of the deferred LayerNorm affine reductions
set -o pipefail
O=gpurun_out/m2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_precision.py \
  > $O/prec.log 2>&1; rc=$?; tail -6 $O/prec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/ln_bench.py > $O/lnbench.log 2>&1; rc=$?; cat $O/lnbench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/nt_library_compare.py > $O/ntlib.log 2>&1; rc=$?; cat $O/ntlib.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    SCA_AFFINE_DEFER=$v timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/c5_${v}_$i.log 2>&1 || exit $?
    echo "cfg5 defer=$v #$i $(grep -o '"value": [0-9.]*' $O/c5_${v}_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c5_${v}_$i.log)"
  done
done
