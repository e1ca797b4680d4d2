#!/bin/bash
# gemm_ntb_kernel (variants 41 / 42): kernel tests, then the NT shapes of configs 5 and 2 against
# the LDS-DMA kernel (variant 20)
set -o pipefail
O=gpurun_out/ntb3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_ntb.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --cfg5 --cases "NT5,NN5" --tiles 20,21,41,42 --iters 10 > $O/bench.log 2>&1; rc=$?; tail -20 $O/bench.log; exit $rc
