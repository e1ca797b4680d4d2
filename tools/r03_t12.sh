set -o pipefail
for v in 8 4 8; do
  echo "== waves $v"; SCA_ATTN16_WAVES=$v timeout -k 10 120 python -u tools/attn_bench.py --iters 50 2>&1 | grep -E "causal" || exit 1
done
SCA_ATTN16_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_attention_shapes.py tests/test_dropout.py tests/test_masks.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread 2>&1 | tail -3
