#!/bin/bash
# Round-4 measurement set in two GPU calls (each step under its own time limit, first failure
# stops the call):
#   bash tools/r04_measure.sh tests   -> full GPU suite, smoke, the bench lines (cfg2 with the
#                                       CPU baseline, cfg3, cfg5, cfg2 with dropout 0.2)
#   bash tools/r04_measure.sh prof    -> rocprofv3 kernel trace + PMC traffic of cfg2/3/5
# Results under gpurun_out/r04/; tools/promote_profile.py copies the profiles to
# profiles/latest/ (run here afterwards) so that bench.py reports the profiler's figures.
set -o pipefail
out=gpurun_out/r04
mkdir -p $out
if [ "$1" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $out/gpu_tests.log 2>&1; rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
  tail -1 $out/smoke.txt
  timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit $?
  grep '"metric"' $out/bench_default.log > $out/bench_default.json
  for wl in cfg3 cfg5; do
    st=20; [ $wl = cfg5 ] && st=10
    timeout -k 10 400 python bench.py --workload $wl --steps $st --no-cpu-baseline > $out/bench_$wl.log 2>&1 || exit $?
    grep '"metric"' $out/bench_$wl.log > $out/bench_$wl.json
  done
  timeout -k 10 300 python bench.py --dropout 0.2 --steps 40 --no-cpu-baseline > $out/bench_dropout.log 2>&1 || exit $?
  grep '"metric"' $out/bench_dropout.log > $out/bench_dropout.json
  for f in $out/bench_*.json; do echo "$f $(grep -o '"value": [0-9.]*' $f)"; done
fi
if [ "$1" = prof ]; then
  for wl in ${WLS:-cfg2 cfg3 cfg5}; do
    st=10; [ $wl = cfg5 ] && st=4
    STEPS=$st BENCH_EXTRA="--workload $wl" bash tools/prof_bench.sh r04/prof_$wl || exit $?
    BENCH_EXTRA="--workload $wl" bash tools/pmc_traffic.sh r04/pmc_$wl || exit $?
  done
  echo prof done
fi
