set -o pipefail
out=gpurun_out/r03_t10; mkdir -p $out
timeout -k 10 120 python -u tools/gemm_ln_stamps.py > $out/stamps.txt 2>&1; rc=$?; cat $out/stamps.txt | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_ln.py tests/test_gpu_lnb.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_dp.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $out/gpu_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
STEPS=100 bash tools/ab_lib.sh 2>&1 | tee $out/ab.txt
