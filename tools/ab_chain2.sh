# chained next-op projections, bench A/B over the variants (SCA_CHAIN_NEXT=1 / 0 / fc1 / qkv)
set -o pipefail
mkdir -p gpurun_out
for v in 1 0 fc1 qkv 1 0 fc1 qkv; do SCA_CHAIN_NEXT=$v timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline > gpurun_out/b_ch$v.log 2>&1 || exit 1; echo "CHAIN=$v $(grep -o '"value": [0-9.]*' gpurun_out/b_ch$v.log) $(grep -o '"ms_per_step_median": [0-9.]*' gpurun_out/b_ch$v.log)"; done
