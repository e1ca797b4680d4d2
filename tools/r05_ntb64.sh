#!/bin/bash
set -o pipefail
O=gpurun_out/ntb64; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_ntb.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --cases "NT,NN" --tiles 20,21,44,45 --iters 20 > $O/bench.log 2>&1; rc=$?; tail -12 $O/bench.log; exit $rc
