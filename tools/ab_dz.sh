# dz chained into the consumer's gemm_lnb: parity tests, then bench A/B (SCA_CHAIN_DZ=1 / 0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lnb.py tests/test_gpu_gemm_ln.py tests/test_gpu_scale.py tests/test_gpu_parity.py > gpurun_out/t_dz.log 2>&1 || { tail -30 gpurun_out/t_dz.log; exit 1; }
tail -1 gpurun_out/t_dz.log
for v in 1 0 1 0 1 0; do SCA_CHAIN_DZ=$v timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline > gpurun_out/b_dz$v.log 2>&1 || exit 1; echo "DZ=$v $(grep -o '"value": [0-9.]*' gpurun_out/b_dz$v.log) $(grep -o '"ms_per_step_median": [0-9.]*' gpurun_out/b_dz$v.log)"; done
