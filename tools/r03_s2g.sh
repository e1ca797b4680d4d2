# early weight-gradient forks (SCA_WGRAD_EARLY): parity with the switch on, then A/B in step
set -o pipefail
out=gpurun_out/r03_s2g; mkdir -p $out
SCA_WGRAD_EARLY=all timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_dp.py tests/test_gpu_parity.py tests/test_dropout.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -1 $out/tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=100 REPS=3 bash tools/env_ab.sh "SCA_WGRAD_EARLY=ffn" "SCA_WGRAD_EARLY=all" 2>&1 | tee $out/ab.txt
