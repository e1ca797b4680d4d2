# round-3 session 2: parity of the GEMM + LayerNorm kernels, then A/B of the 2-slice-stage ring
set -o pipefail
out=gpurun_out/r03_s2; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_ln.py tests/test_gpu_lnb.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=100 bash tools/ab_lib.sh 2>&1 | tee $out/ab.txt
