# round-3 session 2: padded head sizes, wide LayerNorm / softmax rows
set -o pipefail
out=gpurun_out/r03_s2b; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide_rows.py tests/test_gpu_attention_shapes.py tests/test_gpu_library_ops.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" $out/tests.log | tail -25; exit $rc
