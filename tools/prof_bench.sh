#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run -> gpurun_out/$1/
export TMPDIR=/tmp
out=gpurun_out/${1:-prof}
mkdir -p $out
python3 -c "from scattennet_amd import _lib; print(_lib.source_digest())" > $out/digest.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline ${BENCH_EXTRA} > $out/bench.log 2>&1
rc=$?
grep '"metric"' $out/bench.log | cut -c1-400
exit $rc
