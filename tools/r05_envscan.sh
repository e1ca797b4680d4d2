#!/bin/bash
# env-switch scan with the final kernels (config 3 / 5 / 2): NT/NN 128x128 threshold, the
# register-staged GEMM + LayerNorm loop, chaining
set -o pipefail
O=gpurun_out/envscan; mkdir -p $O
run() { # name workload steps env...
  local n=$1 wl=$2 st=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --workload $wl --steps $st --no-cpu-baseline > $O/${wl}_$n.log 2>&1 || exit $?
  echo "$wl $n $(grep -o '"value": [0-9.]*' $O/${wl}_$n.log)"
}
for i in 1 2; do
  run base$i cfg3 20 SCA_X=0
  run ntbk256_$i cfg3 20 SCA_NTB_MIN_K=256
  run chain0_$i cfg3 20 SCA_CHAIN=0
  run base$i cfg5 10 SCA_X=0
  run ntb0_$i cfg5 10 SCA_NTB=0
  run base$i cfg2 20 SCA_X=0
  run ntbk256_$i cfg2 20 SCA_NTB_MIN_K=256
done
