# HIP graph executor knobs vs the default, bench at config 2 (alternating; never more graph
# queues than GPU_MAX_HW_QUEUES = 4: 8 segfaults in the runtime)
set -o pipefail
mkdir -p gpurun_out
run() { env "$@" timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline > gpurun_out/ge.log 2>&1 || return 1; echo "$* $(grep -o '"value": [0-9.]*' gpurun_out/ge.log) $(grep -o '"ms_per_step_median": [0-9.]*' gpurun_out/ge.log)"; }
for i in 1 2 3; do
  run X=default || exit 1
  run DEBUG_HIP_FORCE_GRAPH_QUEUES=2 || exit 1
  run DEBUG_HIP_FORCE_GRAPH_QUEUES=3 || exit 1
done
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
