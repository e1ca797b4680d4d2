# GPU call: weight-gradient kernel sweep, then the GPU tests that failed before -> gpurun_out/$1/
set -o pipefail
out=gpurun_out/${1:-r03_tn}
mkdir -p $out
timeout -k 10 300 python -u tools/tn_bench.py --splits ${SPLITS:-1,2,3,4} > $out/tn_bench.log 2>&1; rc=$?; echo "tn_bench rc=$rc"; cat $out/tn_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_scale.py tests/test_gpu_gemm_ln.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" $out/gpu_tests.log | tail -12
exit $rc
