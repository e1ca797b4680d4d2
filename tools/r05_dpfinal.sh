#!/bin/bash
# final DP check with this round's kernels: RCCL world 1 with captured bucketed all-reduces
# (launched like the driver: torch.distributed.run), then --gpus 2 over gloo sharing the card
set -o pipefail
O=gpurun_out/dpfinal; mkdir -p $O
env SCA_DP_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 1 --steps 20 --no-cpu-baseline > $O/dp_force.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' $O/dp_force.log
env SCA_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --no-cpu-baseline > $O/gpus2.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*' $O/gpus2.log
