# GPU call: GEMM parity subset with the in-tree library, gemm_ln microbench new vs prev, in-step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm or lnb or scale or parity" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
echo new; timeout -k 10 120 python tools/gemm_ln_bench.py || exit 1
echo prev; SCA_LIB_PATH=scattennet_amd/libscatten_hip_prev.so timeout -k 10 120 python tools/gemm_ln_bench.py || exit 1
STEPS=100 bash tools/ab_lib.sh
