# merge-chain key/value gradient accumulated in the GEMM epilogue: parity tests, bench A/B (SCA_KV_ACC)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm_ln.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_dp.py > gpurun_out/t_kv.log 2>&1 || { tail -30 gpurun_out/t_kv.log; exit 1; }
tail -1 gpurun_out/t_kv.log
for v in 1 0 1 0 1 0; do SCA_KV_ACC=$v timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline > gpurun_out/b_kv$v.log 2>&1 || exit 1; echo "KV=$v $(grep -o '"value": [0-9.]*' gpurun_out/b_kv$v.log) $(grep -o '"ms_per_step_median": [0-9.]*' gpurun_out/b_kv$v.log)"; done
