# hd-32 attention backward: fused key-block kernel vs the split kernels at config 5's shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/attn_bench.py --T 1024 --hd 32 --H 16 --B 8 --G 4 --iters 10 > gpurun_out/kblk.log 2>&1 || exit 1
timeout -k 10 120 python tools/attn_bench.py --T 1024 --hd 32 --H 16 --B 8 --G 4 --iters 10 --split > gpurun_out/split.log 2>&1 || exit 1
echo fused-kblk; grep -h "err\|us" gpurun_out/kblk.log | grep -v Warn; echo split; grep -h "us" gpurun_out/split.log
