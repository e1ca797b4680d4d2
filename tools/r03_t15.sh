set -o pipefail
out=gpurun_out/r03_t15; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_library_ops.py tests/test_gpu_scale.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" $out/gpu_tests.log | tail -12
exit $rc
