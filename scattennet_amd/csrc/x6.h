// fp32 products on the bf16 matrix cores ("x6"): every fp32 operand x is split into three
// bf16 pieces x = hi + mid + lo (round-to-nearest at each step: |mid| <= 2^-8 |x|,
// |lo| <= 2^-16 |x|, the residual below 2^-24 |x|), and a product a*b is the sum of the six
// piece products whose magnitude reaches the fp32 rounding level:
//     hi*hi + hi*mid + mid*hi + mid*mid + hi*lo + lo*hi
// (the three dropped terms are <= 2^-24 |ab| together).  Each piece product is exact in fp32
// (8 x 8 significant bits) and the matrix core accumulates in fp32, so the result has fp32
// accuracy (measured against fp64: tests/test_gpu_x6.py) at 6 bf16 MFMAs per 16 k-steps of a
// 32x32 tile — 6 x 32 = 192 cycles against 8 x 64 = 512 for v_mfma_f32_32x32x2_f32.
#pragma once
#include "common.h"

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// two floats -> one packed bf16 pair (v_cvt_pk_bf16_f32, round to nearest even)
__device__ __forceinline__ unsigned x6_pk(float a, float b) {
  const bf16x2 h = __builtin_convertvector((f32x2){a, b}, bf16x2);
  return __builtin_bit_cast(unsigned, h);
}

// two floats -> their three packed bf16 pieces
__device__ __forceinline__ void x6_split2(float a, float b, unsigned& h, unsigned& m, unsigned& l) {
  h = x6_pk(a, b);
  a -= __uint_as_float(h << 16);
  b -= __uint_as_float(h & 0xffff0000u);
  m = x6_pk(a, b);
  a -= __uint_as_float(m << 16);
  b -= __uint_as_float(m & 0xffff0000u);
  l = x6_pk(a, b);
}

// four consecutive floats -> three 8-byte pieces (4 bf16 each)
__device__ __forceinline__ void x6_split4(f32x4 v, uint2& h, uint2& m, uint2& l) {
  x6_split2(v[0], v[1], h.x, m.x, l.x);
  x6_split2(v[2], v[3], h.y, m.y, l.y);
}

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// c += a * b over one 16-deep k-step of a 32x32 tile, a[p] / b[p] = piece p's fragment
// (the smallest products first)
__device__ __forceinline__ f32x16 x6_mma(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  c = mfma_bf16(a[2], b[0], c);
  c = mfma_bf16(a[0], b[2], c);
  c = mfma_bf16(a[1], b[1], c);
  c = mfma_bf16(a[1], b[0], c);
  c = mfma_bf16(a[0], b[1], c);
  c = mfma_bf16(a[0], b[0], c);
  return c;
}
