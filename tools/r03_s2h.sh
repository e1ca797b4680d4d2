# 2-slice-stage ring in gemm_lnb_kernel only: parity, then A/B in step
set -o pipefail
out=gpurun_out/r03_s2h; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lnb.py tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -1 $out/tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=100 bash tools/ab_lib.sh 2>&1 | tee $out/ab.txt
