set -o pipefail
out=gpurun_out/r03_t13; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_ln.py tests/test_gpu_lnb.py tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" $out/gpu_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for v in fused unfused fused; do
  if [ $v = unfused ]; then export SCA_FUSE_LN=0 SCA_FUSE_LNB=0; else unset SCA_FUSE_LN SCA_FUSE_LNB; fi
  timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --warmup 3 --no-cpu-baseline > $out/cfg5_$v.log 2>&1 || exit 1
  echo "cfg5 $v $(grep -o '"value": [0-9.]*' $out/cfg5_$v.log) $(grep -o '"ms_per_step_median": [0-9.]*' $out/cfg5_$v.log)"
done
unset SCA_FUSE_LN SCA_FUSE_LNB
STEPS=100 bash tools/ab_lib.sh 2>&1 | tee $out/ab.txt
