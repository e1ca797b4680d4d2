#!/bin/bash
# The data-parallel path at RCCL world size 1 with the collectives forced on (captured bucketed
# all-reduces, as on an 8-GPU node) under two settings, alternated: DP_A / DP_B are env lists.
set -o pipefail
out=gpurun_out/${1:-dp_ab}
mkdir -p $out
for i in 1 2; do
  for v in A B; do
    envs=$([ $v = A ] && echo "${DP_A:-X=1}" || echo "${DP_B:-X=1}")
    env $envs SCA_DP_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $((29611 + i)) bench.py --steps 40 --no-cpu-baseline > $out/${v}_$i.log 2>&1 || { tail -20 $out/${v}_$i.log; exit 1; }
    echo "$v [$envs] $(grep -o '"value": [0-9.]*' $out/${v}_$i.log) $(grep -o '"check_max_abs": [0-9.e-]*' $out/${v}_$i.log)"
  done
done
