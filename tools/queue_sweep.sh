# per-step kernel listing (with hardware queue ids) under the graph executor's queue counts
export TMPDIR=/tmp
for q in ${QUEUES:-3 4}; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q STEPS=6 bash tools/prof_bench.sh prof_q$q || exit 1
  python tools/step_listing.py gpurun_out/prof_q$q/run_kernel_trace.csv > gpurun_out/prof_q$q/listing.txt || exit 1
done
