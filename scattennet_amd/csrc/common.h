// Shared device helpers for the SCA HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define SCA_FMIN (-3.40282346638528859812e+38f)  // torch.finfo(torch.float32).min
#define SCA_LOG2E 1.4426950408889634f

// erf for the GELU epilogues, branch-free: erfc(z) = t exp(-z^2 + P(t)), t = 1 / (1 + z / 2), with
// the 10-term Chebyshev fit of Numerical Recipes (fractional error of erfc < 1.2e-7; in fp32,
// |erf - erf_exact| <= 3.9e-7 over the whole line).  ocml's erff branches on |x| (both paths
// run in a wave holding small and large arguments) and cost the fused fc1 chains ~2 us per
// 32 x 256 pass.  SCA_ERF_OCML=1 (build flag) restores erff.
#ifndef SCA_ERF_OCML
#define SCA_ERF_OCML 0
#endif
__device__ __forceinline__ float erf_ep(float x) {
  if constexpr (SCA_ERF_OCML) {
    return erff(x);
  } else {
    const float z = fabsf(x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
    float p = 0.17087277f;
    p = fmaf(p, t, -0.82215223f);
    p = fmaf(p, t, 1.48851587f);
    p = fmaf(p, t, -1.13520398f);
    p = fmaf(p, t, 0.27886807f);
    p = fmaf(p, t, -0.18628806f);
    p = fmaf(p, t, 0.09678418f);
    p = fmaf(p, t, 0.37409196f);
    p = fmaf(p, t, 1.00002368f);
    p = fmaf(p, t, -1.26551223f);
    const float r = t * __expf(fmaf(-z, z, p));  // erfc(z)
    return copysignf(1.0f - r, x);
  }
}

__device__ __forceinline__ float gelu_erf(float x) {
  // nn.GELU() default (approximate='none'): x * 0.5 * (1 + erf(x / sqrt(2)))
  return x * 0.5f * (1.0f + erf_ep(x * 0.70710678118654752f));
}

__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erf_ep(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
// stores through the GLOBAL address space (global_store_*, counted in order by vmcnt): a
// generic pointer the compiler cannot resolve becomes a flat_store, which completes out of
// order with respect to vmcnt — unusable where a counted vmcnt lets stores stay in flight
typedef __attribute__((address_space(1))) f32x4 g_f32x4;
typedef __attribute__((address_space(1))) float g_float;
__device__ __forceinline__ void st4g(float* p, f32x4 v) { *(g_f32x4*)(p) = v; }
__device__ __forceinline__ void st1g(float* p, float v) { *(g_float*)(p) = v; }

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations (lgkmcnt(0))
// but not for its global stores / loads / LDS-DMA in flight — __syncthreads() waits for those
// too (vmcnt(0)), which would drain an epilogue's stores and the next phase's prefetched
// slices at every such barrier.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt, expcnt unconstrained
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Counter-based dropout mask (include/scatten.h, sca_dropout): element e of the tensor
// dropped by seed `seed` is kept iff mix(mix(e ^ key) + key) >= thr.
__host__ __device__ __forceinline__ uint32_t sca_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

extern "C" const unsigned long long* sca_drop_offset_ptr(void);

struct DropMask {
  uint32_t key, thr;
  float scale;
  // off: the registered device step counter (sca_dropout_offset) or NULL
  __device__ __forceinline__ void init(unsigned long long seed, float p, const unsigned long long* off) {
    if (off) seed += *off * 0x9E3779B97F4A7C15ull;
    key = sca_mix32((uint32_t)seed ^ sca_mix32((uint32_t)(seed >> 32) + 0x9e3779b9U));
    thr = (uint32_t)fminf(p * 4294967296.0f, 4294967040.0f);
    scale = 1.0f / (1.0f - p);
  }
  __device__ __forceinline__ float apply(uint32_t e, float v) const {
    return sca_mix32(sca_mix32(e ^ key) + key) >= thr ? v * scale : 0.0f;
  }
};
