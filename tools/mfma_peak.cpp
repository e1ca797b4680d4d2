// Diagnostic: the fp32 MFMA rate this chip sustains with operands in registers (random data),
// and the clock it holds meanwhile — the ceiling the GEMM kernels are measured against.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_peak.cpp -o tools/mfma_peak && ./tools/mfma_peak
// Variants: 32x32x2 with 1 / 4 independent accumulators per wave, 1 or 2 waves per SIMD
// (256 or 512 threads per workgroup, one workgroup per CU); 16x16x4 with 4 accumulators.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ void mfma32_loop(float* out, int iters, unsigned long long* clk) {
  float a = threadIdx.x * 1.0e-3f + 0.5f, b = blockIdx.x * 1.0e-3f + 0.25f;
  f32x16 acc[NACC];
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = (float)(r + i) * 1e-3f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16 / NACC; ++u)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

__global__ void mfma16_loop(float* out, int iters, unsigned long long* clk) {
  float a = threadIdx.x * 1.0e-3f + 0.5f, b = blockIdx.x * 1.0e-3f + 0.25f;
  f32x4 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 4; ++r) acc[i][r] = (float)(r + i) * 1e-3f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u)  // 32 MFMAs of 32 cycles = 16 of the 32x32x2 form
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 4; ++r) s += acc[i][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  const int nwg = 256, iters = 20000;
  float* out;
  unsigned long long* clk;
  hipMalloc(&out, nwg * 512 * sizeof(float));
  hipMalloc(&clk, nwg * 2 * sizeof(unsigned long long));
  unsigned long long hclk[512];
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct V { const char* name; int threads; int kind; };
  V vs[] = {{"32x32x2, 1 acc, 1 wave/SIMD", 256, 1}, {"32x32x2, 4 acc, 1 wave/SIMD", 256, 4},
            {"32x32x2, 1 acc, 2 waves/SIMD", 512, 1}, {"32x32x2, 4 acc, 2 waves/SIMD", 512, 4},
            {"16x16x4, 4 acc, 1 wave/SIMD", 256, 16}};
  for (int rep = 0; rep < 2; ++rep)
    for (const V& v : vs) {
      hipEventRecord(e0);
      if (v.kind == 1) hipLaunchKernelGGL(mfma32_loop<1>, dim3(nwg), dim3(v.threads), 0, 0, out, iters, clk);
      else if (v.kind == 4) hipLaunchKernelGGL(mfma32_loop<4>, dim3(nwg), dim3(v.threads), 0, 0, out, iters, clk);
      else hipLaunchKernelGGL(mfma16_loop, dim3(nwg), dim3(v.threads), 0, 0, out, iters, clk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(hclk, clk, sizeof(hclk), hipMemcpyDeviceToHost);
      double ghz = 0;
      for (int i = 0; i < nwg; ++i) ghz += (double)hclk[2 * i] / (double)hclk[2 * i + 1] * 0.1;  // memrealtime 100 MHz
      ghz /= nwg;
      const double flops = (double)nwg * (v.threads / 64) * iters * 16 * 32.0 * 32 * 2 * 2;
      printf("%-32s %8.3f ms  %7.1f TFLOP/s  in-kernel clock %.2f GHz\n", v.name, ms, flops / ms / 1e9, ghz);
    }
  return 0;
}
