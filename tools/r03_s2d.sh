# A/B of the critical-chain wave priority (s_setprio) in step, config 2 and config 3
set -o pipefail
out=gpurun_out/r03_s2d; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lnb.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -1 $out/tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=100 bash tools/ab_lib.sh 2>&1 | tee $out/ab.txt
