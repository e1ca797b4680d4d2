# GPU call: parity suite, gemm_ln microbench per SCA_GEMM_LN_ROT, in-step A/B of the toggles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 0 1 3; do
  echo "ROT=$r"; SCA_GEMM_LN_ROT=$r timeout -k 10 120 python tools/gemm_ln_bench.py || exit 1
done
REPS=2 bash tools/env_ab.sh "SCA_GEMM_LN_ROT=1" "SCA_GEMM_LN_ROT=3"
