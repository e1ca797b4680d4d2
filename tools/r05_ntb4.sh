#!/bin/bash
# 128x128 NT / NN kernel: bench at the cfg5 shapes (explicit variants), cfg5 step A/B
# (off / default min K 1024 / min K 512), a kernel trace of the default cfg5 step
set -o pipefail
O=gpurun_out/ntb4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_ntb.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --cfg5 --cases "NT5,NN5" --tiles 20,21,41,42 --iters 10 > $O/bench.log 2>&1; rc=$?; tail -8 $O/bench.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in off def k512; do
    case $v in off) e="SCA_NTB=0";; def) e="SCA_NTB=1";; k512) e="SCA_NTB_MIN_K=512";; esac
    env $e timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --no-cpu-baseline > $O/${v}_$i.log 2>&1 || exit $?
    echo "${v}_$i $(grep -o '"value": [0-9.]*' $O/${v}_$i.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload cfg5 --steps 4 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
python3 tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt 2>&1; head -14 $O/timeline.txt
