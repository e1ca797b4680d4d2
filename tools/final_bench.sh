# round-end bench lines: default (with the CPU baseline), config 3, config 5, train-mode dropout
set -o pipefail
out=gpurun_out/${1:-final}
mkdir -p $out
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit 1
grep '"metric"' $out/bench_default.log > $out/bench_default.json
for wl in cfg3 cfg5; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --no-cpu-baseline > $out/bench_$wl.log 2>&1 || exit 1
  grep '"metric"' $out/bench_$wl.log > $out/bench_$wl.json
done
timeout -k 10 300 python bench.py --dropout 0.2 --steps 50 --no-cpu-baseline > $out/bench_dropout.log 2>&1 || exit 1
grep '"metric"' $out/bench_dropout.log > $out/bench_dropout.json
for f in $out/*.json; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"ms_per_step_median": [0-9.]*' $f)"; done
grep -o '"cpu_baseline": {[^}]*}' $out/bench_default.json
