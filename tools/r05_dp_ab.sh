#!/bin/bash
# A/B of the data-parallel path's graph schedule at RCCL world size 1 (SCA_DP_FORCE=1):
# the deferred RCCL fork (SCA_DP_DEFER) x the graph executor's queue count; plain bench beside.
set -o pipefail
O=gpurun_out/r05dpab
mkdir -p $O
dp() { local name=$1; shift; env RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29650 + RANDOM % 200)) \
       SCA_DP_FORCE=1 "$@" timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > $O/$name.log 2>&1 || { echo "[$name] failed"; tail -3 $O/$name.log; exit 1; }
       echo "[$name] $(grep -o '"value": [0-9.]*' $O/$name.log) $(grep -o '"ms_per_step_median": [0-9.]*' $O/$name.log)"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "captured" > $O/test.log 2>&1 || { tail -5 $O/test.log; exit 1; }
tail -1 $O/test.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > $O/plain_$i.log 2>&1 || exit 1
  echo "[plain] $(grep -o '"value": [0-9.]*' $O/plain_$i.log)"
  dp new_$i
  dp old_$i SCA_DP_DEFER=0 SCA_DP_GRAPH_QUEUES=2
  dp defer_q2_$i SCA_DP_GRAPH_QUEUES=2
  dp nodefer_q3_$i SCA_DP_DEFER=0
done
export TMPDIR=/tmp
mkdir -p $O/prof
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29633 SCA_DP_FORCE=1 \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof/bench.log 2>&1 || exit $?
echo prof done
