# GPU call: full GPU suite, in-step A/B vs libscatten_hip_prev.so, then a rocprofv3 kernel
# trace of the default bench -> gpurun_out/r02_late/prof
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
STEPS=100 bash tools/ab_lib.sh || exit 1
STEPS=10 bash tools/prof_bench.sh r02_late/prof || exit $?
echo done
