# round-3 closing set, part A: full GPU suite, smoke, bench lines (default with CPU baseline,
# cfg3, cfg5, dropout), kernel trace + PMC traffic of the default bench -> gpurun_out/$1/
set -o pipefail
n=${1:-r03_closeA}; out=gpurun_out/$n; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
tail -2 $out/smoke.txt
bash tools/round_measure.sh $n || exit $?
f=$(ls $out/prof/*kernel_trace.csv | head -1)
python3 tools/timeline.py $f > $out/timeline.txt && python3 tools/step_listing.py $f > $out/step_listing.txt
grep -h '"metric"' $out/bench_*.log | cut -c1-220
head -12 $out/timeline.txt
