// Timing probe of the GEMM + LayerNorm main loop (32 x 256 row tile per workgroup, 8 waves,
// each a 32x32 column block, K slices of 32): where does a slice's time go?
//   mode 0: the kernel's LDS-DMA ring (3 stages), DMA + fragments + MFMAs
//   mode 1: DMA only            mode 2: fragments + MFMAs only (no DMA)
//   mode 3: no LDS, no barrier: every wave loads its own A / B fragments straight into
//           registers (global_load_dwordx4), D slices ahead
//   mode 4: A through the LDS-DMA ring, B straight into registers
// Standalone: hipcc -O3 --offload-arch=gfx950 tools/lnloop_probe.hip -o /tmp/lnloop_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int BM = 32, BN = 256, BK = 32, NW = 8, PIECE = 1024;
constexpr int A_BYTES = BM * BK * 4, B_BYTES = BN * BK * 4, STAGE = A_BYTES + B_BYTES;

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ void dma(const float* src, char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ const float* src_of(const float* base, int ld, int row0, int pc, int lane) {
  const int r = 8 * pc + (lane >> 3);
  const int ks = (lane & 7) ^ swz(r);
  return base + (long)(row0 + r) * ld + 4 * ks;
}
__device__ __forceinline__ f32x4 frag(const char* img, int r0, int g, int lane) {
  const int r = r0 + (lane & 31), h = lane >> 5;
  return *(const f32x4*)(img + r * 128 + 16 * ((2 * g + h) ^ swz(r)));
}
// LDS read the compiler does not track (the caller waits with lgkm_wait<N> on the registers)
__device__ __forceinline__ f32x4 ds_read128(const char* p) {
  f32x4 v;
  const unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
  return v;
}
template <int N>
__device__ __forceinline__ void lgkm_wait(f32x4& x, f32x4& y) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(x), "+v"(y) : "n"(N));
}
__device__ __forceinline__ f32x4 frag_asm(const char* img, int r0, int g, int lane) {
  const int r = r0 + (lane & 31), h = lane >> 5;
  return ds_read128(img + r * 128 + 16 * ((2 * g + h) ^ swz(r)));
}
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ unsigned long long g_clk[4];
__device__ __forceinline__ void clk_stamp(int slot) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    g_clk[2 * slot] = __builtin_amdgcn_s_memtime();
    g_clk[2 * slot + 1] = __builtin_amdgcn_s_memrealtime();
  }
}
struct Args {
  const float* A;  // [P][M][K]
  const float* B;  // [P][256][K]
  float* C;        // [P][M][256]
  int M, K;
};

__device__ __forceinline__ void tile_of(const Args& a, int& p, int& m0) {
  const unsigned nwg = gridDim.x, orig = blockIdx.x;
  const unsigned xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles = a.M / BM;
  p = wgid / tiles;
  m0 = (wgid % tiles) * BM;
}

__device__ __forceinline__ void store_acc(const Args& a, int p, int m0, int wave, int lane, const f32x16& acc) {
  const int col = lane & 31, rowh = 4 * (lane >> 5);
  float* C = a.C + (long)p * a.M * BN;
#pragma unroll
  for (int r = 0; r < 16; ++r) C[(long)(m0 + (r & 3) + 8 * (r >> 2) + rowh) * BN + 32 * wave + col] = acc[r];
}

template <int MODE, int SG = 0>
__global__ __launch_bounds__(512) void ring_kernel(const Args a) {
  constexpr int S = 3;
  __shared__ __attribute__((aligned(1024))) char smem[S * STAGE];
  int p, m0;
  tile_of(a, p, m0);
  clk_stamp(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* A = a.A + (long)p * a.M * a.K;
  const float* B = a.B + (long)p * BN * a.K;
  const int total = a.K / BK;
  const bool has_a = wave < 4;
  const float* pa = src_of(A, a.K, m0, has_a ? wave : 0, lane);
  const float* pb[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) pb[c] = src_of(B, a.K, 0, 4 * wave + c, lane);
  auto issue = [&](int t, int stage) {
    if (MODE == 2) return;
    char* base = smem + stage * STAGE;
    const long kk = (long)t * BK;
    if (has_a) dma(pa + kk, base + wave * PIECE);
#pragma unroll
    for (int c = 0; c < 4; ++c) dma(pb[c] + kk, base + A_BYTES + (4 * wave + c) * PIECE);
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int i = 0; i < S - 1; ++i) issue(i, i);
  for (int t = 0; t < total; ++t) {
    if (MODE != 2) {
      if (t + S - 2 < total) {
        if (has_a) wait_vm<5>();
        else wait_vm<4>();
      } else {
        wait_vm<0>();
      }
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (SG < 4 && t + S - 1 < total) issue(t + S - 1, (t + S - 1) % S);
    if (MODE != 1) {
      const char* As = smem + (t % S) * STAGE;
      const char* Bs = As + A_BYTES;
      f32x4 fa[4], fb[4];
      if (SG >= 4) {  // DMA of slice t+S-1 issued under the MFMAs: after group 0 (4) / spread (5)
#define SB __builtin_amdgcn_sched_barrier(0)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          fa[g] = frag(As, 0, g, lane);
          fb[g] = frag(Bs, 32 * wave, g, lane);
        }
        SB;
        const bool more = t + S - 1 < total;
        char* base = smem + ((t + S - 1) % S) * STAGE;
        const long kk = (long)(t + S - 1) * BK;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = mfma32(fa[g][j], fb[g][j], acc);
          SB;
          if (MODE != 2 && more) {
            if (SG == 4 && g == 0) {
              if (has_a) dma(pa + kk, base + wave * PIECE);
#pragma unroll
              for (int c = 0; c < 4; ++c) dma(pb[c] + kk, base + A_BYTES + (4 * wave + c) * PIECE);
            } else if (SG == 5) {
              if (g == 0 && has_a) dma(pa + kk, base + wave * PIECE);
              dma(pb[g] + kk, base + A_BYTES + (4 * wave + g) * PIECE);
            }
          }
          SB;
        }
#undef SB
        continue;
      }
      if (SG == 3) {  // untracked reads, partial waits
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          fa[g] = frag_asm(As, 0, g, lane);
          fb[g] = frag_asm(Bs, 32 * wave, g, lane);
        }
#define SB __builtin_amdgcn_sched_barrier(0)
        SB; lgkm_wait<6>(fa[0], fb[0]); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[0][j], fb[0][j], acc);
        SB; lgkm_wait<4>(fa[1], fb[1]); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[1][j], fb[1][j], acc);
        SB; lgkm_wait<2>(fa[2], fb[2]); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[2][j], fb[2][j], acc);
        SB; lgkm_wait<0>(fa[3], fb[3]); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[3][j], fb[3][j], acc);
#undef SB
        continue;
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        fa[g] = frag(As, 0, g, lane);
        fb[g] = frag(Bs, 32 * wave, g, lane);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[g][j], fb[g][j], acc);
      if (SG == 1) {  // all 8 reads, then the 16 MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
      } else if (SG == 2) {  // 4 reads (g = 0, 1), 4 MFMAs, 2 reads, 4 MFMAs, 2 reads, 8 MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      }
    }
  }
  if (MODE == 1) {
    __syncthreads();
    acc[0] = ((const float*)smem)[threadIdx.x];
  }
  clk_stamp(1);
  store_acc(a, p, m0, wave, lane, acc);
}

// direct-to-register fragments, D slices in flight; MODE 3: A and B direct, MODE 4: A by
// LDS-DMA ring (S = D + 1 stages of 4 KiB), B direct
template <int MODE, int D>
__global__ __launch_bounds__(512) void direct_kernel(const Args a) {
  __shared__ __attribute__((aligned(1024))) char smem[MODE == 4 ? (D + 1) * A_BYTES : 16];
  int p, m0;
  tile_of(a, p, m0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const float* A = a.A + (long)p * a.M * a.K + (long)(m0 + r) * a.K + 4 * h;
  const float* B = a.B + (long)p * BN * a.K + (long)(32 * wave + r) * a.K + 4 * h;
  const int total = a.K / BK;
  f32x4 fa[D][4], fb[D][4];
  const float* pa = src_of(a.A + (long)p * a.M * a.K, a.K, m0, wave & 3, lane);
  auto issue = [&](int t, int slot) {
    const long kk = (long)t * BK;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (MODE == 3) fa[slot][g] = *(const f32x4*)(A + kk + 8 * g);
      fb[slot][g] = *(const f32x4*)(B + kk + 8 * g);
    }
    if (MODE == 4 && wave < 4) dma(pa + kk, smem + (t % (D + 1)) * A_BYTES + wave * PIECE);
  };
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
  for (int i = 0; i < D; ++i) issue(i, i);
  for (int t0 = 0; t0 < total; t0 += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int t = t0 + i;
      if (t < total) {
        if (MODE == 4) {
          // slice t's A pieces (this wave's, issued D slices ago) landed; then every wave's
          if (wave < 4) wait_vm<(D - 1) * 5>();
          __builtin_amdgcn_s_barrier();
          const char* As = smem + (t % (D + 1)) * A_BYTES;
#pragma unroll
          for (int g = 0; g < 4; ++g) fa[i][g] = frag(As, 0, g, lane);
        } else {
          wait_vm<(D - 1) * 8>();
        }
        f32x4 xa[4], xb[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          xa[g] = fa[i][g];
          xb[g] = fb[i][g];
        }
        if (t + D < total) issue(t + D, i);
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = mfma32(xa[g][j], xb[g][j], acc);
      }
    }
  }
  store_acc(a, p, m0, wave, lane, acc);
}

// mode 5: S-stage ring, fragments read one slice ahead into a second register set (the
// reads of slice t+1 issued right after barrier t, under slice t's MFMAs); mode 6: the
// same without DMA (compute only)
template <int MODE, int S>
__global__ __launch_bounds__(512) void pf_kernel(const Args a) {
  __shared__ __attribute__((aligned(1024))) char smem[S * STAGE];
  int p, m0;
  tile_of(a, p, m0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* A = a.A + (long)p * a.M * a.K;
  const float* B = a.B + (long)p * BN * a.K;
  const int total = a.K / BK;
  const bool has_a = wave < 4;
  const float* pa = src_of(A, a.K, m0, has_a ? wave : 0, lane);
  const float* pb[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) pb[c] = src_of(B, a.K, 0, 4 * wave + c, lane);
  auto issue = [&](int t, int stage) {
    if (MODE == 6) return;
    char* base = smem + stage * STAGE;
    const long kk = (long)t * BK;
    if (has_a) dma(pa + kk, base + wave * PIECE);
#pragma unroll
    for (int c = 0; c < 4; ++c) dma(pb[c] + kk, base + A_BYTES + (4 * wave + c) * PIECE);
  };
  auto wait_slice = [&](int t) {  // slice t landed for this wave (slices issued up to t + S - 2)
    if (MODE == 6) return;
    if (t + S - 3 < total - 1) {
      if (has_a) wait_vm<5 * (S - 3)>();
      else wait_vm<4 * (S - 3)>();
    } else {
      wait_vm<0>();
    }
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int i = 0; i < S - 1; ++i) issue(i, i);
  f32x4 fa[4], fb[4];
  wait_slice(0);
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    fa[g] = frag(smem, 0, g, lane);
    fb[g] = frag(smem + A_BYTES, 32 * wave, g, lane);
  }
  for (int t = 0; t < total; ++t) {
    f32x4 na[4], nb[4];
    if (t + 1 < total) {
      wait_slice(t + 1);
      __builtin_amdgcn_s_barrier();  // slice t+1 landed for all; stage (t-1)%S free
      __builtin_amdgcn_sched_barrier(0);
      if (t + S - 1 < total) issue(t + S - 1, (t + S - 1) % S);
      const char* As = smem + ((t + 1) % S) * STAGE;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        na[g] = frag(As, 0, g, lane);
        nb[g] = frag(As + A_BYTES, 32 * wave, g, lane);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma32(fa[g][j], fb[g][j], acc);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      fa[g] = na[g];
      fb[g] = nb[g];
    }
  }
  store_acc(a, p, m0, wave, lane, acc);
}

// mode 7: 2-stage ring of 64-k stages (two 32-k sub-slices, 72 KiB each): one barrier per
// 32 MFMAs per wave; SG3: untracked reads with partial waits per sub-slice
template <int MODE, int SG>
__global__ __launch_bounds__(512) void big_kernel(const Args a) {
  __shared__ __attribute__((aligned(1024))) char smem[4 * STAGE];
  int p, m0;
  tile_of(a, p, m0);
  clk_stamp(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* A = a.A + (long)p * a.M * a.K;
  const float* B = a.B + (long)p * BN * a.K;
  const int total = a.K / (2 * BK);
  const bool has_a = wave < 4;
  const float* pa = src_of(A, a.K, m0, has_a ? wave : 0, lane);
  const float* pb[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) pb[c] = src_of(B, a.K, 0, 4 * wave + c, lane);
  auto issue = [&](int t, int stage) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      char* base = smem + (2 * stage + u) * STAGE;
      const long kk = (long)(2 * t + u) * BK;
      if (has_a) dma(pa + kk, base + wave * PIECE);
#pragma unroll
      for (int c = 0; c < 4; ++c) dma(pb[c] + kk, base + A_BYTES + (4 * wave + c) * PIECE);
    }
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  issue(0, 0);
  for (int t = 0; t < total; ++t) {
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < total) issue(t + 1, (t + 1) & 1);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const char* As = smem + (2 * (t & 1) + u) * STAGE;
      const char* Bs = As + A_BYTES;
      f32x4 fa[4], fb[4];
      if (SG == 3) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          fa[g] = frag_asm(As, 0, g, lane);
          fb[g] = frag_asm(Bs, 32 * wave, g, lane);
        }
#define SB __builtin_amdgcn_sched_barrier(0)
        SB; lgkm_wait<6>(fa[0], fb[0]); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[0][j], fb[0][j], acc);
        SB; lgkm_wait<4>(fa[1], fb[1]); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[1][j], fb[1][j], acc);
        SB; lgkm_wait<2>(fa[2], fb[2]); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[2][j], fb[2][j], acc);
        SB; lgkm_wait<0>(fa[3], fb[3]); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[3][j], fb[3][j], acc);
#undef SB
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          fa[g] = frag(As, 0, g, lane);
          fb[g] = frag(Bs, 32 * wave, g, lane);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = mfma32(fa[g][j], fb[g][j], acc);
      }
    }
  }
  clk_stamp(1);
  store_acc(a, p, m0, wave, lane, acc);
}

// mode 8: barrier-free B stream — every wave DMAs its OWN 32 B rows (its column block) into
// a wave-private S-stage ring and waits on its own vmcnt only; the A operand of a 256-k chunk
// (32 rows x 256 k) goes through LDS once per chunk into registers (128 VGPRs); two barriers
// per chunk, none per slice.  SG: 3 = untracked B fragment reads with partial waits.
template <int S, int SG>
__global__ __launch_bounds__(512) void priv_kernel(const Args a) {
  constexpr int WB = 4096;  // one wave's B slice: 32 rows x 32 k
  __shared__ __attribute__((aligned(1024))) char smem[8 * S * WB + 8 * A_BYTES];
  int p, m0;
  tile_of(a, p, m0);
  clk_stamp(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* A = a.A + (long)p * a.M * a.K;
  const float* B = a.B + (long)p * BN * a.K;
  const int total = a.K / BK;
  char* ring = smem + wave * S * WB;
  char* Ach = smem + 8 * S * WB;  // 8 slices x 4 KiB
  // piece c of a slice = rows 8c .. 8c+7; the swizzle differs between even and odd pieces
  const float* pa[2] = {src_of(A, a.K, m0, 0, lane), src_of(A, a.K, m0, 1, lane)};
  const float* pb[2] = {src_of(B, a.K, 32 * wave, 0, lane), src_of(B, a.K, 32 * wave, 1, lane)};
  const long ld16 = 16L * a.K;
  auto issue_b = [&](int t) {
    char* base = ring + (t % S) * WB;
    const long kk = (long)t * BK;
#pragma unroll
    for (int c = 0; c < 4; ++c) dma(pb[c & 1] + (c >> 1) * ld16 + kk, base + c * PIECE);
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int i = 0; i < S - 1; ++i) if (i < total) issue_b(i);
  const int nch = total / 8;
  for (int ch = 0; ch < nch; ++ch) {
    __builtin_amdgcn_s_barrier();  // every wave has its A registers of chunk ch-1
    // A chunk: wave w fetches slice w of the chunk (4 pieces of 8 rows)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      dma(pa[c & 1] + (c >> 1) * ld16 + (long)(8 * ch + wave) * BK, Ach + wave * A_BYTES + c * PIECE);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    f32x4 fa[8][4];
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8)
#pragma unroll
      for (int g = 0; g < 4; ++g) fa[s8][g] = frag(Ach + s8 * A_BYTES, 0, g, lane);
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      const int t = 8 * ch + s8;
      if (s8 > 0) {
        if (t + S - 2 < total) wait_vm<4 * (S - 2)>();
        else wait_vm<0>();
      }
      if (t + S - 1 < total) issue_b(t + S - 1);
      const char* Bs = ring + (t % S) * WB;
      f32x4 fb[4];
      if (SG == 3) {
#pragma unroll
        for (int g = 0; g < 4; ++g) fb[g] = frag_asm(Bs, 0, g, lane);
        f32x4 dummy = fa[s8][0];
#define SB __builtin_amdgcn_sched_barrier(0)
        SB; lgkm_wait<3>(fb[0], dummy); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[s8][0][j], fb[0][j], acc);
        SB; lgkm_wait<2>(fb[1], dummy); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[s8][1][j], fb[1][j], acc);
        SB; lgkm_wait<1>(fb[2], dummy); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[s8][2][j], fb[2][j], acc);
        SB; lgkm_wait<0>(fb[3], dummy); SB;
        for (int j = 0; j < 4; ++j) acc = mfma32(fa[s8][3][j], fb[3][j], acc);
#undef SB
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) fb[g] = frag(Bs, 0, g, lane);
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = mfma32(fa[s8][g][j], fb[g][j], acc);
      }
    }
  }
  clk_stamp(1);
  store_acc(a, p, m0, wave, lane, acc);
}

// mode 9: ping-pong — waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave
// issues its 16 MFMAs (s_setprio 1) while the other reads its next fragments, issues its DMA
// pieces and retires the next slice; reads and vmcnt retired before each group's first
// barrier (RAW / WAR across the staggered groups)
template <int S, int PRIO>
__global__ __launch_bounds__(512) void pp_kernel(const Args a) {
  __shared__ __attribute__((aligned(1024))) char smem[S * STAGE];
  int p, m0;
  tile_of(a, p, m0);
  clk_stamp(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* A = a.A + (long)p * a.M * a.K;
  const float* B = a.B + (long)p * BN * a.K;
  const int total = a.K / BK;
  const bool has_a = wave < 4;
  const float* pa = src_of(A, a.K, m0, has_a ? wave : 0, lane);
  const float* pb[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) pb[c] = src_of(B, a.K, 0, 4 * wave + c, lane);
  auto issue = [&](int t) {
    char* base = smem + (t % S) * STAGE;
    const long kk = (long)t * BK;
    if (has_a) dma(pa + kk, base + wave * PIECE);
#pragma unroll
    for (int c = 0; c < 4; ++c) dma(pb[c] + kk, base + A_BYTES + (4 * wave + c) * PIECE);
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int i = 0; i < S - 1; ++i) if (i < total) issue(i);
  wait_vm<0>();  // prologue: the first S-1 slices (simple)
  __builtin_amdgcn_s_barrier();
  if (wave >= 4) __builtin_amdgcn_s_barrier();
  for (int t = 0; t < total; ++t) {
    const char* As = smem + (t % S) * STAGE;
    const char* Bs = As + A_BYTES;
    if (t + S - 1 < total) issue(t + S - 1);  // into slice t-1's stage: every read of it retired
    __builtin_amdgcn_sched_barrier(0);
    f32x4 fa[4], fb[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      fa[g] = frag(As, 0, g, lane);
      fb[g] = frag(Bs, 32 * wave, g, lane);
    }
    // retire slice t+1 (issued earlier) before this group's barrier
    if (t + S - 1 < total) {
      if (has_a) wait_vm<5 * (S - 2)>();
      else wait_vm<4 * (S - 2)>();
    } else if (t + 1 < total) {
      // slices t+1 .. total-1 in flight, the last issued at t' = total - S + 1 ... retire all
      wait_vm<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma32(fa[g][j], fb[g][j], acc);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (wave < 4) __builtin_amdgcn_s_barrier();
  clk_stamp(1);
  store_acc(a, p, m0, wave, lane, acc);
}

template <class F>
float time_it(F launch, int iters) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) launch();
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    best = ms * 1e3f / iters < best ? ms * 1e3f / iters : best;
  }
  return best;
}

int main(int argc, char** argv) {
  const int P = 4, M = 2048;
  const int K = argc > 1 ? atoi(argv[1]) : 768;
  std::vector<float> hA((size_t)P * M * K), hB((size_t)P * BN * K);
  srand(1);
  for (auto& x : hA) x = (rand() / (float)RAND_MAX) - 0.5f;
  for (auto& x : hB) x = (rand() / (float)RAND_MAX) - 0.5f;
  float *dA, *dB, *dC, *dR;
  CHK(hipMalloc(&dA, hA.size() * 4));
  CHK(hipMalloc(&dB, hB.size() * 4));
  CHK(hipMalloc(&dC, (size_t)P * M * BN * 4));
  CHK(hipMalloc(&dR, (size_t)P * M * BN * 4));
  CHK(hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
  Args a{dA, dB, dC, M, K};
  const int grid = P * M / BM;
  const double flops = 2.0 * P * M * BN * K;
  auto report = [&](const char* name, float us, bool check) {
    double err = 0;
    if (check) {
      std::vector<float> c((size_t)P * M * BN), ref((size_t)P * M * BN);
      CHK(hipMemcpy(c.data(), dC, c.size() * 4, hipMemcpyDeviceToHost));
      CHK(hipMemcpy(ref.data(), dR, ref.size() * 4, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < c.size(); ++i) err = fmax(err, fabs(c[i] - ref[i]));
    }
    unsigned long long c[4];
    CHK(hipMemcpyFromSymbol(c, HIP_SYMBOL(g_clk), sizeof(c)));
    const double ghz = (double)(c[2] - c[0]) / (double)(c[3] - c[1]) * 0.1;
    printf("%-44s %8.2f us  %6.1f TFLOP/s  %.3f of 157.3  maxdiff %.2e  clk %.2f GHz\n", name, us, flops / us * 1e-6,
           flops / us * 1e-6 / 157.3, err, ghz);
  };
  a.C = dR;
  report("mode 0: LDS-DMA ring (S=3), as gemm_ln", time_it([&] { ring_kernel<0><<<grid, 512>>>(a); }, 50), false);
  a.C = dC;
  report("mode 1: DMA only", time_it([&] { ring_kernel<1><<<grid, 512>>>(a); }, 50), false);
  report("mode 2: fragments + MFMA only", time_it([&] { ring_kernel<2><<<grid, 512>>>(a); }, 50), false);
  report("mode 3: direct registers, D=2", time_it([&] { direct_kernel<3, 2><<<grid, 512>>>(a); }, 50), true);
  report("mode 3: direct registers, D=3", time_it([&] { direct_kernel<3, 3><<<grid, 512>>>(a); }, 50), true);
  report("mode 3: direct registers, D=4", time_it([&] { direct_kernel<3, 4><<<grid, 512>>>(a); }, 50), true);
  report("mode 4: A ring + B direct, D=2", time_it([&] { direct_kernel<4, 2><<<grid, 512>>>(a); }, 50), true);
  report("mode 4: A ring + B direct, D=3", time_it([&] { direct_kernel<4, 3><<<grid, 512>>>(a); }, 50), true);
  report("mode 0, DMA after MFMA group 0 (SG4)", time_it([&] { ring_kernel<0, 4><<<grid, 512>>>(a); }, 50), true);
  report("mode 0, DMA spread over MFMA groups (SG5)", time_it([&] { ring_kernel<0, 5><<<grid, 512>>>(a); }, 50), true);
  report("mode 0 + all reads first (SG1)", time_it([&] { ring_kernel<0, 1><<<grid, 512>>>(a); }, 50), true);
  report("mode 0 + staged reads (SG2)", time_it([&] { ring_kernel<0, 2><<<grid, 512>>>(a); }, 50), true);
  report("mode 2 + all reads first (SG1)", time_it([&] { ring_kernel<2, 1><<<grid, 512>>>(a); }, 50), false);
  report("mode 2 + staged reads (SG2)", time_it([&] { ring_kernel<2, 2><<<grid, 512>>>(a); }, 50), false);
  report("mode 0 + untracked reads (SG3)", time_it([&] { ring_kernel<0, 3><<<grid, 512>>>(a); }, 50), true);
  report("mode 2 + untracked reads (SG3)", time_it([&] { ring_kernel<2, 3><<<grid, 512>>>(a); }, 50), false);
  report("mode 7: 64-k stages, S=2", time_it([&] { big_kernel<7, 0><<<grid, 512>>>(a); }, 50), true);
  report("mode 7: 64-k stages, S=2, SG3", time_it([&] { big_kernel<7, 3><<<grid, 512>>>(a); }, 50), true);
  report("mode 9: ping-pong, S=3", time_it([&] { pp_kernel<3, 0><<<grid, 512>>>(a); }, 50), true);
  report("mode 9: ping-pong, S=4", time_it([&] { pp_kernel<4, 0><<<grid, 512>>>(a); }, 50), true);
  report("mode 9: ping-pong, S=3, setprio", time_it([&] { pp_kernel<3, 1><<<grid, 512>>>(a); }, 50), true);
  report("mode 9: ping-pong, S=4, setprio", time_it([&] { pp_kernel<4, 1><<<grid, 512>>>(a); }, 50), true);
  report("mode 8: private B rings, S=3", time_it([&] { priv_kernel<3, 0><<<grid, 512>>>(a); }, 50), true);
  report("mode 8: private B rings, S=4", time_it([&] { priv_kernel<4, 0><<<grid, 512>>>(a); }, 50), true);
  report("mode 8: private B rings, S=3, SG3", time_it([&] { priv_kernel<3, 3><<<grid, 512>>>(a); }, 50), true);
  report("mode 8: private B rings, S=4, SG3", time_it([&] { priv_kernel<4, 3><<<grid, 512>>>(a); }, 50), true);
  report("mode 5: frag one slice ahead, S=4", time_it([&] { pf_kernel<5, 4><<<grid, 512>>>(a); }, 50), true);
  report("mode 5: frag one slice ahead, S=3", time_it([&] { pf_kernel<5, 3><<<grid, 512>>>(a); }, 50), true);
  report("mode 6: frag one slice ahead, no DMA", time_it([&] { pf_kernel<6, 4><<<grid, 512>>>(a); }, 50), false);
  CHK(hipFree(dA));
  CHK(hipFree(dB));
  CHK(hipFree(dC));
  CHK(hipFree(dR));
  return 0;
}
