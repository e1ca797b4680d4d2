# GPU call: kernel trace of a default bench run + timeline + listing, PMC traffic -> gpurun_out/$1/
set -o pipefail
n=${1:-r03_prof}
STEPS=10 bash tools/prof_bench.sh $n/prof || exit $?
f=$(ls gpurun_out/$n/prof/*kernel_trace.csv | head -1)
python3 tools/timeline.py $f > gpurun_out/$n/timeline.txt && python3 tools/step_listing.py $f > gpurun_out/$n/step_listing.txt
head -25 gpurun_out/$n/timeline.txt
bash tools/pmc_traffic.sh $n/pmc || exit $?
