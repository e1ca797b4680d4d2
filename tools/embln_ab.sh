# GPU call: full GPU suite, then in-step A/B of the embedding-LN hand-off (SCA_EMB_LNB=0 = off)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
STEPS=100 REPS=3 bash tools/env_ab.sh "SCA_EMB_LNB=0"
