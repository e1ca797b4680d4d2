set -o pipefail
out=gpurun_out/r03_t11; mkdir -p $out
for lib in scattennet_amd/libscatten_hip.so scattennet_amd/libscatten_hip_prev.so scattennet_amd/libscatten_hip.so; do
  echo "== $lib"; timeout -k 10 120 python -u tools/attn_bench.py --lib $lib --iters 50 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention_shapes.py tests/test_dropout.py tests/test_masks.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $out/gpu_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
STEPS=100 bash tools/ab_lib.sh 2>&1 | tee $out/ab.txt
