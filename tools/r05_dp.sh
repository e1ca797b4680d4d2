#!/bin/bash
# Round 5, first GPU call: the data-parallel abort fix, the GPU suite, the bench lines.
#   watchdog_fixed probe -> GPU suite -> bench (cfg2) -> DP rehearsal (RCCL world 1, captured
#   bucketed all-reduces) -> bench --gpus 2 (two gloo ranks sharing the card) -> watchdog_race
#   probe LAST (expected to abort: it reproduces the round-4 SIGABRT on purpose).
set -o pipefail
O=gpurun_out/r05dp
mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "[$name] rc=$rc"; tail -n 4 "$O/$name.log" | cut -c1-400; return $rc; }
step probe_fixed 120 python -u tools/dp_capture_diag.py watchdog_fixed || exit 1
if [ -z "$SKIP_TESTS" ]; then
  step tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread -p no:cacheprovider || exit 1
fi
step bench 300 python -u bench.py || exit 1
step dp_force 300 env SCA_DP_FORCE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --steps 20 --no-cpu-baseline || exit 1
step gpus2 300 env SCA_DIST_BACKEND=gloo python -u bench.py --gpus 2 --steps 20 --no-cpu-baseline || exit 1
step probe_race 120 python -u tools/dp_capture_diag.py watchdog_race
echo "probe_race finished (134 = the reproduced abort)"
exit 0
