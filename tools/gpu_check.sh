#!/bin/bash
# GPU-box driver: parity tests, then a short bench.  Stops at the first crash / timeout
# (exit codes other than 0 = pass and 1 = test failures).
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/gpu_tests.log
ok $rc || exit $rc
if [ -n "${SKIP_BENCH}" ]; then exit 0; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -20 gpurun_out/bench.log
exit $rc
