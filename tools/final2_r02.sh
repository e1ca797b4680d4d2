# GPU call: full GPU suite, embedding-LN hand-off A/B, then the closing measurement set
# -> gpurun_out/r02_close2/ (bench lines, rocprofv3 kernel trace, PMC traffic, MFMA/HBM table)
set -o pipefail
mkdir -p gpurun_out/r02_close2
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r02_close2/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r02_close2/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
STEPS=100 REPS=2 bash tools/env_ab.sh "SCA_EMB_LNB=0" || exit 1
bash tools/round_measure.sh r02_close2 || exit $?
bash tools/pmc_util.sh r02_close2/util || exit $?
echo done
