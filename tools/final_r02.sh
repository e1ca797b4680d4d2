# Round-2 closing measurement set -> gpurun_out/r02_close/: full GPU suite, default bench (with
# the CPU baseline), cfg3 / cfg5 / dropout lines, rocprofv3 kernel trace of the default bench,
# per-kernel MFMA-busy / HBM table (separate SQ / FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
out=gpurun_out/r02_close
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/round_measure.sh r02_close || exit $?
bash tools/pmc_util.sh r02_close/util || exit $?
echo done
