#!/bin/bash
# Measurement set (each step under its own time limit; the first failure stops the call):
#   bash tools/measure.sh tests <set>  -> full GPU suite, smoke, the bench lines (cfg2 with the
#                                            CPU baseline, cfg3, cfg5, cfg2 with dropout 0.2)
#   bash tools/measure.sh prof <set>   -> per workload (WLS, default cfg2 cfg3 cfg5): rocprofv3
#                                            kernel trace + stats, PMC traffic, SQ utilisation
# Results under gpurun_out/<set>/; then, here: python tools/promote_profile.py <wl>
#   gpurun_out/<set>/prof_<wl> gpurun_out/<set>/pmc_<wl> gpurun_out/<set>/sq_<wl>
set -o pipefail
set_=${2:-m}
out=gpurun_out/$set_
mkdir -p $out
if [ "$1" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 420 --timeout-method thread \
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
    STEPS=$st BENCH_EXTRA="--workload $wl" bash tools/prof_bench.sh $set_/prof_$wl || exit $?
    BENCH_EXTRA="--workload $wl" bash tools/pmc_traffic.sh $set_/pmc_$wl || exit $?
    BENCH_EXTRA="--workload $wl" bash tools/pmc_sq.sh $set_/sq_$wl || exit $?
  done
  echo prof done
fi
if [ "$1" = dpprof ]; then
  # the data-parallel path at world size 1 (captured bucketed RCCL all-reduces), kernel trace:
  # one rank started directly (no launcher between rocprofv3 and the program)
  export TMPDIR=/tmp
  mkdir -p $out/dpprof
  RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29633 SCA_DP_FORCE=1 \
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/dpprof -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/dpprof/bench.log 2>&1 || exit $?
  grep '"metric"' $out/dpprof/bench.log | cut -c1-300
fi
