set -o pipefail
out=gpurun_out/r03_t9; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_ln.py tests/test_gpu_lnb.py tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $out/gpu_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
SCA_WGRAD_DEFER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_dp.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests_defer.log 2>&1; rc=$?; echo "pytest defer rc=$rc"; grep -E "FAILED|passed|failed" $out/gpu_tests_defer.log | tail -5
[ $rc -eq 0 ] || exit $rc
STEPS=100 REPS=3 bash tools/env_ab.sh "SCA_WGRAD_DEFER=1" 2>&1 | tee $out/ab.txt
SCA_WGRAD_DEFER=1 STEPS=10 bash tools/prof_bench.sh r03_t9/prof > /dev/null 2>&1
f=$(ls gpurun_out/r03_t9/prof/*kernel_trace.csv | head -1); python3 tools/timeline.py $f | head -8; python3 tools/step_listing.py $f > $out/step_listing.txt
