#!/bin/bash
# Round 5: the stream-K weight-gradient kernel — kernel-level parity, shape benchmark, bench A/B.
set -o pipefail
O=gpurun_out/r05tn
mkdir -p $O
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "[$name] rc=$rc"; tail -n ${TAILN:-4} "$O/$name.log" | cut -c1-300; return $rc; }
step tn_tests 300 python -u -m pytest tests/test_gpu_gemm_tn.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
TAILN=40 step tn_bench 300 python -u tools/tn_streamk_bench.py || exit 1
for i in 1 2; do
  step bench_sk_$i 200 python -u bench.py --no-cpu-baseline || exit 1
  grep -o '"value": [0-9.]*' $O/bench_sk_$i.log
  step bench_old_$i 200 env SCA_TN_STREAMK=0 python -u bench.py --no-cpu-baseline || exit 1
  grep -o '"value": [0-9.]*' $O/bench_old_$i.log
done
