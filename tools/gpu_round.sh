#!/bin/bash
# One GPU call of the build loop: [GEMM microbench] -> parity subset -> short bench line.
#   GB_TILES="20,21,60,62" GB_CASES="NT,NN" PYTEST_K="cfg2 or parity" BENCH_ARGS="--steps 20" bash tools/gpu_round.sh
mkdir -p gpurun_out
if [ -n "$GB_TILES" ]; then
  timeout -k 10 400 python tools/gemm_bench.py --tiles "$GB_TILES" ${GB_CASES:+--cases "$GB_CASES"} --iters 20 --rounds 2 > gpurun_out/gb.log 2>&1
  rc=$?; echo "gemm_bench rc=$rc"; cat gpurun_out/gb.log | grep -v amdgpu.ids
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; grep '"metric"' gpurun_out/bench.log | cut -c1-600; tail -3 gpurun_out/bench.log | grep -v '"metric"'
  exit $rc
fi
