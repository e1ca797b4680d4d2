# round-3 profile set: cfg2 (bench default), cfg3, cfg5 — kernel trace + PMC traffic each
set -o pipefail
bash tools/r03_prof.sh r03_p_cfg2 || exit $?
BENCH_EXTRA="--workload cfg3" bash tools/r03_prof.sh r03_p_cfg3 || exit $?
BENCH_EXTRA="--workload cfg5" bash tools/r03_prof.sh r03_p_cfg5 || exit $?
