# config 5: bench line + rocprofv3 kernel stats -> gpurun_out/cfg5/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg5
timeout -k 10 400 python bench.py --workload cfg5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/cfg5/bench_cfg5.json 2> gpurun_out/cfg5/bench.err || exit 1
cut -c1-420 gpurun_out/cfg5/bench_cfg5.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg5 -o run -- python3 bench.py --workload cfg5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cfg5/prof_bench.log 2>&1 || exit 1
f=$(ls gpurun_out/cfg5/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/cfg5/run_kernel_stats.csv)
cut -c1-160 $f | head -16
