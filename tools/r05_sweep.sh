#!/bin/bash
set -o pipefail
O=gpurun_out/sweep; mkdir -p $O
for np in 2 4 6 8; do
  SCA_NPRE45=$np timeout -k 10 200 python -u tools/gemm_bench.py --cases "NT,NN" --tiles 45 --iters 20 --no-check > $O/np$np.log 2>&1 || exit $?
  echo "== NPRE $np"; tail -7 $O/np$np.log
done
for i in 1 2; do
  for v in 1 0; do
    SCA_LN_AFFINE_SIDE=$v timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/aff${v}_$i.log 2>&1 || exit $?
    echo "affine_side=$v #$i $(grep -o '"value": [0-9.]*' $O/aff${v}_$i.log)"
  done
done
for i in 1 2; do
  for v in 0 1; do
    SCA_FUSE_LN512=$v timeout -k 10 300 python bench.py --workload cfg5 --steps 8 --no-cpu-baseline > $O/ln512_${v}_$i.log 2>&1 || exit $?
    echo "cfg5 fuse_ln512=$v #$i $(grep -o '"value": [0-9.]*' $O/ln512_${v}_$i.log)"
  done
done
