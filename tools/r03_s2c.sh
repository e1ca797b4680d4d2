# attention backward A/B (in isolation, then in step) + parity of the attention shapes
set -o pipefail
out=gpurun_out/r03_s2c; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention_shapes.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python tools/attn_bench.py --no-check > $out/new$i.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/attn_bench.py --no-check --lib scattennet_amd/libscatten_hip_prev.so > $out/prev$i.txt 2>&1 || exit 1
done
for f in $out/new1.txt $out/prev1.txt $out/new2.txt $out/prev2.txt; do echo "== $f"; cat $f; done
STEPS=100 bash tools/ab_lib.sh 2>&1 | tee $out/ab.txt
