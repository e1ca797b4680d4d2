# chained next-op projections: parity tests, then bench A/B (SCA_CHAIN_NEXT=1 / 0)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_ln.py tests/test_gpu_lnb.py tests/test_gpu_scale.py tests/test_gpu_dp.py > gpurun_out/t_chain.log 2>&1 || { tail -40 gpurun_out/t_chain.log; exit 1; }
tail -2 gpurun_out/t_chain.log
for v in 1 0 1 0; do SCA_CHAIN_NEXT=$v timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline > gpurun_out/b_ch$v.log 2>&1 || exit 1; echo "CHAIN=$v $(grep -o '"value": [0-9.]*' gpurun_out/b_ch$v.log)"; done
