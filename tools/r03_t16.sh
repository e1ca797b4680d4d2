set -o pipefail
out=gpurun_out/r03_t16; mkdir -p $out
SCA_TNK_MANY=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_dp.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" $out/gpu_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
STEPS=100 REPS=3 bash tools/env_ab.sh "SCA_TNK_MANY=1" 2>&1 | tee $out/ab.txt
