#!/bin/bash
# interleaved phases (variants 43 / 44) against 40 / 41: kernel tests, TN compare at the cfg5 /
# cfg2 attention shapes, NT / NN bench at the cfg5 shapes
set -o pipefail
O=gpurun_out/ilv1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_ntb.py tests/test_gpu_gemm_tn.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/tn_library_compare.py --only "cfg5" --splits 1,2,4 --tnb-tiles 40,43 > $O/tn.log 2>&1; rc=$?; grep "tnb\|ksplit" $O/tn.log | grep "us" ; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --cfg5 --cases "NT5,NN5" --tiles 20,21,41,44 --iters 10 > $O/bench.log 2>&1; rc=$?; tail -7 $O/bench.log; exit $rc
