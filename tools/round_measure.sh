# Round-end measurement set: default bench (with CPU baseline), workload variants, rocprofv3
# kernel-trace profile and the PMC traffic pass of the default workload -> gpurun_out/$1/
set -o pipefail
out=gpurun_out/${1:-round}
mkdir -p $out
timeout -k 10 300 python bench.py > $out/bench_default.log 2>&1 || exit $?
grep '"metric"' $out/bench_default.log > $out/bench_default.json
for wl in cfg3 cfg5; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --no-cpu-baseline > $out/bench_$wl.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --dropout 0.2 --steps 50 --no-cpu-baseline > $out/bench_dropout.log 2>&1 || exit $?
STEPS=10 bash tools/prof_bench.sh ${1:-round}/prof || exit $?
bash tools/pmc_traffic.sh ${1:-round}/pmc || exit $?
echo done
