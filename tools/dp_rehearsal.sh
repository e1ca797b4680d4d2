#!/bin/bash
# Rehearse bench.py's data-parallel path on a one-GPU box: world size 1 over RCCL with the
# collectives forced on (SCA_DP_FORCE=1), so the bucketed all-reduces are issued from the
# backward and captured into the step's hipGraph exactly as on an 8-GPU node.
mkdir -p gpurun_out
SCA_DP_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port ${PORT:-29611} bench.py --steps ${STEPS:-20} --no-cpu-baseline \
  > gpurun_out/dp_rehearsal.log 2>&1
rc=$?; echo "dp rehearsal rc=$rc"; grep '"metric"' gpurun_out/dp_rehearsal.log | cut -c1-600 || tail -20 gpurun_out/dp_rehearsal.log
exit $rc
