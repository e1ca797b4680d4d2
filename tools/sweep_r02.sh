# GPU call: GEMM + LN parity tests, then an env-toggle A/B sweep on config 2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_ln.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
STEPS=100 REPS=2 bash tools/env_ab.sh "$@"
