#!/bin/bash
# HBM traffic per dispatch (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE (KiB) in two
# separate --pmc passes over a short bench run; tools/traffic_summary.py turns them into
# bytes per launch (FETCH_SIZE doubled: gfx950 tallies 128-B reads at 64 B).
export TMPDIR=/tmp
out=gpurun_out/${1:-pmc_traffic}
mkdir -p $out
python3 -c "from scattennet_amd import _lib; print(_lib.source_digest())" > $out/digest.txt
ARGS="bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_EXTRA}"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out -o fetch -- python3 $ARGS > $out/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out -o write -- python3 $ARGS > $out/write.log 2>&1 || exit $?
python3 tools/traffic_summary.py $out
