# round-3 closing set, part B: cfg3 / cfg5 kernel traces + PMC traffic, per-kernel MFMA-busy /
# HBM table of the default bench
set -o pipefail
BENCH_EXTRA="--workload cfg3" bash tools/r03_prof.sh ${1:-r03_closeB}_cfg3 > /dev/null || exit $?
BENCH_EXTRA="--workload cfg5" bash tools/r03_prof.sh ${1:-r03_closeB}_cfg5 > /dev/null || exit $?
bash tools/pmc_util.sh ${1:-r03_closeB}_util || exit $?
head -30 gpurun_out/${1:-r03_closeB}_util/summary.txt
