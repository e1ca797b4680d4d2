#!/bin/bash
# round 6: the GPU suite (or a -k subset), the default bench line, and the 2-rank gloo rehearsal
# of the data-parallel path with its all-reduce self-check.  Stops at the first crash / timeout.
set -o pipefail
out=gpurun_out/${1:-r06check}
mkdir -p $out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 420 --timeout-method thread \
  ${PYTEST_K:+-k "$PYTEST_K"} > $out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $out/gpu_tests.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
grep '"metric"' $out/bench.log | cut -c1-400
SCA_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --no-cpu-baseline > $out/bench_gpus2_gloo.log 2>&1 || { tail -20 $out/bench_gpus2_gloo.log; exit 1; }
grep -o '"grad_allreduce": {[^}]*}' $out/bench_gpus2_gloo.log
