#!/bin/bash
set -o pipefail
O=gpurun_out/tnr2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tn.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/tn_library_compare.py --only "cfg2,cfg3" --splits 0 --tnb-tiles 0 --ksplit-tiles 21,46 > $O/tn.log 2>&1; rc=$?; grep "ksplit" $O/tn.log | grep "us" ; exit $rc
