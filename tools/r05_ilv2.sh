#!/bin/bash
# variants 43 / 44 at the config-2 / config-3 shapes
set -o pipefail
O=gpurun_out/ilv2; mkdir -p $O
timeout -k 10 400 python -u tools/tn_library_compare.py --only "cfg2,cfg3" --splits 1,2,4,8 --tnb-tiles 43 > $O/tn.log 2>&1; rc=$?; grep "tnb\|ksplit" $O/tn.log | grep "us" ; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --cases "NT,NN" --tiles 20,21,44 --iters 20 > $O/bench.log 2>&1; rc=$?; tail -12 $O/bench.log; exit $rc
