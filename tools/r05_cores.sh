#!/bin/bash
# A/B: co-residency build (tools/lib_cores.so: gemm_lnb loads its epilogue operands after the
# main loop -> 138 VGPRs; the register-staged weight-gradient kernel's LDS 48 -> 35 KB), so one
# gemm_lnb workgroup fits beside one weight-gradient workgroup; with and without split-K 1
set -o pipefail
O=gpurun_out/cores; mkdir -p $O
SCA_LIB_PATH=$PWD/tools/lib_cores.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_lnb.py tests/test_gpu_gemm_tn.py tests/test_gpu_scale.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in base cores cores_sk1; do
    case $v in base) e="SCA_X=0";; cores) e="SCA_LIB_PATH=$PWD/tools/lib_cores.so";; cores_sk1) e="SCA_LIB_PATH=$PWD/tools/lib_cores.so SCA_TNR_SK=1";; esac
    env $e timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/c2_${v}_$i.log 2>&1 || exit $?
    echo "cfg2 $v #$i $(grep -o '"value": [0-9.]*' $O/c2_${v}_$i.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c2_${v}_$i.log)"
  done
done
for v in base cores; do
  case $v in base) e="SCA_X=0";; cores) e="SCA_LIB_PATH=$PWD/tools/lib_cores.so";; esac
  env $e timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --no-cpu-baseline > $O/c3_${v}.log 2>&1 || exit $?
  echo "cfg3 $v $(grep -o '"value": [0-9.]*' $O/c3_${v}.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/c3_${v}.log)"
done
