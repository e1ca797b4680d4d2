set -o pipefail
out=gpurun_out/${1:-r03_tn}
mkdir -p $out
timeout -k 10 300 python -u tools/tn_bench.py --tiles 21,30,31,32,33,34,35 --splits 1,2,3,4 > $out/tn_bench.log 2>&1; rc=$?; echo "tn_bench rc=$rc"; grep attn $out/tn_bench.log
[ $rc -eq 0 ] || exit $rc
SHARD_CALLS=1 SCA_GEMM_LN_BM=32 timeout -k 10 200 python -u tools/shard_diff.py > $out/shard_diff.log 2>&1; rc=$?; echo "shard_diff rc=$rc"; tail -3 $out/shard_diff.log
exit $rc
