set -o pipefail
O=gpurun_out/tnb1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_tn.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/tn_library_compare.py --only "cfg2 attn,cfg5" --splits 1,2,4 > $O/cmp.log 2>&1; rc=$?; tail -70 $O/cmp.log; exit $rc
