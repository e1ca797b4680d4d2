#!/bin/bash
# GEMM + LayerNorm kernels: the LDS-DMA main loop (SCA_LNREG=0) against the register-staged one
set -o pipefail
O=gpurun_out/lneff; mkdir -p $O
for v in 0 1; do
  SCA_LNREG=$v timeout -k 10 200 python -u tools/gemm_ln_bench.py > $O/ln_$v.log 2>&1 || exit $?
  SCA_LNREG=$v timeout -k 10 200 python -u tools/lnb_bench.py > $O/lnb_$v.log 2>&1 || exit $?
  echo "== lnreg=$v"; grep -v "^$\|amdgpu.ids" $O/ln_$v.log | tail -8; grep -v "^$\|amdgpu.ids" $O/lnb_$v.log | tail -6
done
