# bench A/B of env toggles against the default (alternating), config 2
#   [STEPS=K REPS=R BENCH_EXTRA="--workload cfg5"] bash tools/env_ab.sh "SCA_CHAIN_DZ=1" "SCA_KV_ACC=1" ...
set -o pipefail
mkdir -p gpurun_out
run() { env "$@" timeout -k 10 300 python bench.py --steps ${STEPS:-100} --no-cpu-baseline ${BENCH_EXTRA} > gpurun_out/eab.log 2>&1 || return 1; echo "$* $(grep -o '"value": [0-9.]*' gpurun_out/eab.log) $(grep -o '"ms_per_step_median": [0-9.]*' gpurun_out/eab.log)"; }
for i in $(seq ${REPS:-2}); do
  run X=default || exit 1
  for v in "$@"; do run $v || exit 1; done
done
