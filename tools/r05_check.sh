#!/bin/bash
# New GPU tests of this round (large heads, DP capture with the deferred fork), the attention
# backward sub-block A/B (parity under both, then timings), then the DP A/B.
set -o pipefail
O=gpurun_out/r05chk
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention_shapes.py tests/test_gpu_dp.py -x -q --timeout 400 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SCA_ATTN_SBC=2 SCA_ATTN_SBN=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_attention_shapes.py tests/test_gpu_parity.py tests/test_dropout.py tests/test_masks.py \
  -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > $O/tests_sb2.log 2>&1; rc=$?; tail -2 $O/tests_sb2.log
[ $rc -eq 0 ] || exit $rc
for sb in 1 2 1 2; do
  SCA_ATTN_SBC=$sb SCA_ATTN_SBN=$sb timeout -k 10 120 python tools/attn_bench.py > $O/attn_sb$sb.log 2>&1 || exit $?
  echo "sb=$sb"; grep us $O/attn_sb$sb.log
done
bash tools/r05_dp_ab.sh
