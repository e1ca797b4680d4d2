# software-pipelined hd-16 attention forward: parity, isolated timing, A/B in step
set -o pipefail
out=gpurun_out/r03_s2f; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_attention_shapes.py tests/test_gpu_parity.py tests/test_masks.py tests/test_dropout.py tests/test_gpu_library_ops.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -1 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python tools/attn_bench.py > $out/new$i.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/attn_bench.py --no-check --lib scattennet_amd/libscatten_hip_prev.so > $out/prev$i.txt 2>&1 || exit 1
done
for f in $out/new1.txt $out/prev1.txt $out/new2.txt $out/prev2.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
STEPS=100 bash tools/ab_lib.sh 2>&1 | tee $out/ab.txt
