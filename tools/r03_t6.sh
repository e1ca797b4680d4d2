set -o pipefail
out=gpurun_out/r03_t6; mkdir -p $out
timeout -k 10 120 ./tools/mfma_peak > $out/mfma_peak.log 2>&1; cat $out/mfma_peak.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; echo "pytest rc=$?"; grep -E "FAILED|passed|failed" $out/gpu_tests.log | tail
STEPS=100 REPS=2 bash tools/env_ab.sh "SCA_TN_TILE=31 SCA_TN_SPLITK=1" "SCA_TN_TILE=21 SCA_TN_SPLITK=2" "SCA_TN_TILE=31 SCA_TN_SPLITK=2" "SCA_TN_TILE=33 SCA_TN_SPLITK=1" 2>&1 | tee $out/ab.txt
