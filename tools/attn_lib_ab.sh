# attention microbenchmark of the in-tree library vs libscatten_hip_prev.so (ATTN_ARGS shapes),
# then the attention parity tests on the in-tree library
mkdir -p gpurun_out
for v in new prev; do
  lib=scattennet_amd/libscatten_hip.so; [ $v = prev ] && lib=scattennet_amd/libscatten_hip_prev.so
  timeout -k 10 120 python tools/attn_bench.py --lib $lib --no-check ${ATTN_ARGS} > gpurun_out/attn_$v.log 2>&1 || exit $?
  echo "== $v"; grep "us" gpurun_out/attn_$v.log
done
