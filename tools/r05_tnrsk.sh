#!/bin/bash
# cfg2 step A/B: variant 46's split-K (model / 3), two weight-gradient side streams (graph queues 2 / 3)
set -o pipefail
O=gpurun_out/tnrsk; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log
for i in 1 2; do
  for v in base sk3 ws2q2 ws2q3; do
    case $v in base) e="SCA_TNR_SK=0";; sk3) e="SCA_TNR_SK=3";; ws2q2) e="SCA_WGRAD_STREAMS=2";;
      ws2q3) e="SCA_WGRAD_STREAMS=2 DEBUG_HIP_FORCE_GRAPH_QUEUES=3";; esac
    env $e timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/${v}_$i.log 2>&1 || exit $?
    echo "$v #$i $(grep -o '"value": [0-9.]*' $O/${v}_$i.log)"
  done
done
