# GPU call: the watchdog probe, the full GPU suite, a default bench line -> gpurun_out/$1/
set -o pipefail
out=gpurun_out/${1:-r03_check}
mkdir -p $out
timeout -k 10 120 python -u tools/watchdog_probe.py > $out/watchdog_probe.log 2>&1; echo "probe rc=$?"; cat $out/watchdog_probe.log | tail -4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_EXTRA} > $out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || exit $?
cut -c1-300 $out/bench.json
