# rocprofv3 kernel trace of the config-5 attention microbench (fused key-block backward)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/kblk_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kblk_prof -o run -- python3 tools/attn_bench.py --T 1024 --hd 32 --H 16 --B 8 --G 4 --iters 5 --no-check > gpurun_out/kblk_prof/bench.log 2>&1 || exit 1
f=$(ls gpurun_out/kblk_prof/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/kblk_prof/run_kernel_stats.csv)
cut -c1-150 $f
