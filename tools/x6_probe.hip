// Probe: fp32 GEMM on the bf16 matrix cores through a three-piece split of every operand
// (x = hi + mid + lo, three bf16 values, exact to 2^-24 relative) and the six products
// whose magnitude reaches the fp32 rounding level (hi*hi, hi*mid, mid*hi, mid*mid, hi*lo,
// lo*hi).  Measures the three GEMM layouts of the SCA step at config-2 shapes against the
// library's fp32-MFMA kernels (libscatten_hip.so, sca_gemm / sca_gemm_partial) and checks
// both against an fp64 host product.
//
//   hipcc -O3 --offload-arch=gfx950 tools/x6_probe.hip -Lscattennet_amd -lscatten_hip \
//         -Wl,-rpath,$PWD/scattennet_amd -o tools/x6_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <type_traits>
#include <vector>

#include "../include/scatten.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

struct Prob {
  const float* A;
  const float* B;
  const unsigned short* Bp;  // pre-split B planes [3][...][K] (NT only), plane stride bplane
  long bplane;
  float* C;
  int M, N, K, lda, ldb, ldc;
};
struct Args {
  Prob p[16];
  int splitk;
};

__device__ __forceinline__ unsigned pk(float a, float b) {
  bf16x2 h = __builtin_convertvector((f32x2){a, b}, bf16x2);
  return __builtin_bit_cast(unsigned, h);
}
// two floats -> three packed bf16 pairs, a = h + m + l to 2^-24
__device__ __forceinline__ void split2(float a, float b, unsigned& h, unsigned& m, unsigned& l) {
  h = pk(a, b);
  a -= __uint_as_float(h << 16);
  b -= __uint_as_float(h & 0xffff0000u);
  m = pk(a, b);
  a -= __uint_as_float(m << 16);
  b -= __uint_as_float(m & 0xffff0000u);
  l = pk(a, b);
}
__device__ __forceinline__ void split4(f32x4 v, uint2& h, uint2& m, uint2& l) {
  split2(v[0], v[1], h.x, m.x, l.x);
  split2(v[2], v[3], h.y, m.y, l.y);
}

// LDS image of one operand slice: [piece 3][ROWS][BK bf16 + 8 pad]
template <int ROWS, int BK>
struct Img {
  static constexpr int PITCH = BK * 2 + 16;            // bytes per row
  static constexpr int PIECE = ROWS * PITCH;           // bytes per piece
  static constexpr int BYTES = 3 * PIECE;
};

// stage one BK slice of an operand (ROWS x BK, rows r0.., k k0..) into registers
template <bool KC, int ROWS, int BK>
struct Stage {
  static constexpr int NV = KC ? ROWS * BK / 4 / 256 : 0;           // float4 per thread (KC)
  static constexpr int NB = KC ? 0 : ROWS * BK / 16;                 // 4x4 blocks (KM)
  static constexpr int NBT = KC ? 0 : (NB + 255) / 256;              // blocks per thread
  static constexpr int NREG = KC ? NV : 4 * NBT;
  f32x4 v[NREG > 0 ? NREG : 1];

  __device__ __forceinline__ void load(const float* base, int ld, int r0, int k0) {
    if (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int e = threadIdx.x + i * 256;
        const int row = e / (BK / 4), kq = e % (BK / 4);
        v[i] = *(const f32x4*)(base + (long)(r0 + row) * ld + k0 + 4 * kq);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NBT; ++i) {
        const int b = threadIdx.x + i * 256;
        if (b < NB) {
          const int kq = b % (BK / 4), rq = b / (BK / 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[4 * i + j] = *(const f32x4*)(base + (long)(k0 + 4 * kq + j) * ld + r0 + 4 * rq);
        }
      }
    }
  }
  __device__ __forceinline__ void store(char* img) {
    using I = Img<ROWS, BK>;
    if (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int e = threadIdx.x + i * 256;
        const int row = e / (BK / 4), kq = e % (BK / 4);
        uint2 h, m, l;
        split4(v[i], h, m, l);
        char* p = img + row * I::PITCH + kq * 8;
        *(uint2*)(p) = h;
        *(uint2*)(p + I::PIECE) = m;
        *(uint2*)(p + 2 * I::PIECE) = l;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NBT; ++i) {
        const int b = threadIdx.x + i * 256;
        if (b < NB) {
          const int kq = b % (BK / 4), rq = b / (BK / 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const f32x4 t = {v[4 * i + 0][r], v[4 * i + 1][r], v[4 * i + 2][r], v[4 * i + 3][r]};
            uint2 h, m, l;
            split4(t, h, m, l);
            char* p = img + (4 * rq + r) * I::PITCH + kq * 8;
            *(uint2*)(p) = h;
            *(uint2*)(p + I::PIECE) = m;
            *(uint2*)(p + 2 * I::PIECE) = l;
          }
        }
      }
    }
  }
};

// pre-split k-contiguous operand: three bf16 planes [3][rows][ld] (no VALU in the stage)
template <int ROWS, int BK>
struct StageP {
  static constexpr int NV = ROWS * BK / 4 / 256;
  uint2 v[3 * NV];
  __device__ __forceinline__ void load(const unsigned short* base, long plane, int ld, int r0, int k0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = threadIdx.x + i * 256;
      const int row = e / (BK / 4), kq = e % (BK / 4);
      const unsigned short* p = base + (long)(r0 + row) * ld + k0 + 4 * kq;
#pragma unroll
      for (int q = 0; q < 3; ++q) v[3 * i + q] = *(const uint2*)(p + q * plane);
    }
  }
  __device__ __forceinline__ void store(char* img) {
    using I = Img<ROWS, BK>;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = threadIdx.x + i * 256;
      const int row = e / (BK / 4), kq = e % (BK / 4);
      char* p = img + row * I::PITCH + kq * 8;
#pragma unroll
      for (int q = 0; q < 3; ++q) *(uint2*)(p + q * I::PIECE) = v[3 * i + q];
    }
  }
};

__device__ __forceinline__ bf16x8 frag(const char* p) { return *(const bf16x8*)p; }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// LAYOUT 0 NT (A[M,K], B[N,K]), 1 NN (A[M,K], B[K,N]), 2 TN (A[K,M], B[K,N])
template <int LAYOUT, int BM, int BN, int BK, bool PREB = false>
__global__ __launch_bounds__(256) void x6_kernel(const Args args) {
  constexpr bool AKC = LAYOUT != 2, BKC = LAYOUT == 0;
  static_assert(!PREB || LAYOUT == 0, "pre-split B: NT only");
  using IA = Img<BM, BK>;
  using IB = Img<BN, BK>;
  constexpr int STAGEB = IA::BYTES + IB::BYTES;
  constexpr int RM = BM / 64, RN = BN / 64;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGEB];

  const Prob& P = args.p[blockIdx.y];
  const int tn = (P.N + BN - 1) / BN;
  const int tiles_mn = ((P.M + BM - 1) / BM) * tn;
  const int kz = blockIdx.x / tiles_mn;
  const int t = blockIdx.x % tiles_mn;
  const int m0 = (t / tn) * BM, n0 = (t % tn) * BN;
  const int kchunk = P.K / args.splitk;
  const int kbeg = kz * kchunk;
  const int nk = kchunk / BK;
  float* C = P.C + (long)kz * P.M * P.N;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;

  Stage<AKC, BM, BK> sa;
  using SB = typename std::conditional<PREB, StageP<BN, BK>, Stage<BKC, BN, BK>>::type;
  SB sb;
  auto load_b = [&](int k0) {
    if constexpr (PREB) sb.load(P.Bp, P.bplane, P.ldb, n0, k0);
    else sb.load(P.B, P.ldb, n0, k0);
  };
  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x16){};

  sa.load(P.A, P.lda, m0, kbeg);
  load_b(kbeg);
  sa.store(smem);
  sb.store(smem + IA::BYTES);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const char* st = smem + (kt & 1) * STAGEB;
    if (kt + 1 < nk) {
      sa.load(P.A, P.lda, m0, kbeg + (kt + 1) * BK);
      load_b(kbeg + (kt + 1) * BK);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      bf16x8 a[RM][3], b[RN][3];
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          a[i][p] = frag(st + p * IA::PIECE + (wm * (BM / 2) + i * 32 + r) * IA::PITCH + kk * 32 + h * 16);
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          b[j][p] = frag(st + IA::BYTES + p * IB::PIECE + (wn * (BN / 2) + j * 32 + r) * IB::PITCH + kk * 32 + h * 16);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          f32x16 c = acc[i][j];
          c = mfma(a[i][2], b[j][0], c);
          c = mfma(a[i][0], b[j][2], c);
          c = mfma(a[i][1], b[j][1], c);
          c = mfma(a[i][1], b[j][0], c);
          c = mfma(a[i][0], b[j][1], c);
          c = mfma(a[i][0], b[j][0], c);
          acc[i][j] = c;
        }
    }
    if (kt + 1 < nk) {
      char* nx = smem + ((kt + 1) & 1) * STAGEB;
      sa.store(nx);
      sb.store(nx + IA::BYTES);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + wm * (BM / 2) + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
        const int n = n0 + wn * (BN / 2) + j * 32 + r;
        C[(long)m * P.ldc + n] = acc[i][j][q];
      }
}

// ---------------------------------------------------------------- host
struct Case {
  const char* name;
  int layout, nprob, M, N, K, splitk;
};

static void fill(std::vector<float>& v, unsigned seed) {
  unsigned s = seed * 2654435761u + 12345u;
  for (auto& x : v) {
    s = s * 1664525u + 1013904223u;
    x = ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
  }
}

template <int LAYOUT, int BM, int BN, int BK, bool PREB = false>
static float run_x6(const Args& a, int nprob, int maxM, int maxN, hipStream_t st, int iters) {
  const int tiles = ((maxM + BM - 1) / BM) * ((maxN + BN - 1) / BN) * a.splitk;
  dim3 grid(tiles, nprob);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((x6_kernel<LAYOUT, BM, BN, BK, PREB>), grid, dim3(256), 0, st, a);
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((x6_kernel<LAYOUT, BM, BN, BK, PREB>), grid, dim3(256), 0, st, a);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / iters;
}

int main(int argc, char** argv) {
  const int iters = 50;
  Case cases[] = {
      {"NT qkv 12x(2048,256,256)", 0, 12, 2048, 256, 256, 1},
      {"NT fc1 4x(2048,768,256)", 0, 4, 2048, 768, 256, 1},
      {"NT fc2 4x(2048,256,768)", 0, 4, 2048, 256, 768, 1},
      {"NN dX 12x(2048,256,256)", 1, 12, 2048, 256, 256, 1},
      {"NN dX fc1 4x(2048,256,768)", 1, 4, 2048, 256, 768, 1},
      {"TN dW 16x(256,256,2048) sk8", 2, 16, 256, 256, 2048, 8},
      {"TN dW fc 8x(768,256,2048) sk4", 2, 8, 768, 256, 2048, 4},
  };
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (const Case& cs : cases) {
    const int L = cs.layout;
    // element counts
    const long szA = (long)cs.M * cs.K, szB = (long)cs.N * cs.K, szC = (long)cs.M * cs.N * cs.splitk;
    std::vector<float> hA(szA * cs.nprob), hB(szB * cs.nprob);
    fill(hA, 1 + L);
    fill(hB, 7 + L);
    float *dA, *dB, *dC, *dC2, *ws;
    CK(hipMalloc(&dA, hA.size() * 4));
    CK(hipMalloc(&dB, hB.size() * 4));
    CK(hipMalloc(&dC, szC * cs.nprob * 4));
    CK(hipMalloc(&dC2, szC * cs.nprob * 4));
    CK(hipMalloc(&ws, szC * cs.nprob * 4 + 1024 * 1024 * 64));
    CK(hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
    // host RNE split of B into three bf16 planes (NT pre-split variants)
    std::vector<unsigned short> hBp(3 * hB.size());
    auto rne = [](float f) -> unsigned short {
      unsigned u;
      memcpy(&u, &f, 4);
      return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
    };
    auto bf = [](unsigned short h) -> float {
      unsigned u = (unsigned)h << 16;
      float f;
      memcpy(&f, &u, 4);
      return f;
    };
    for (size_t i = 0; i < hB.size(); ++i) {
      float x = hB[i];
      unsigned short h = rne(x);
      x -= bf(h);
      unsigned short m = rne(x);
      x -= bf(m);
      hBp[i] = h;
      hBp[hB.size() + i] = m;
      hBp[2 * hB.size() + i] = rne(x);
    }
    unsigned short* dBp;
    CK(hipMalloc(&dBp, hBp.size() * 2));
    CK(hipMemcpy(dBp, hBp.data(), hBp.size() * 2, hipMemcpyHostToDevice));
    Args a;
    memset(&a, 0, sizeof a);
    a.splitk = cs.splitk;
    std::vector<sca_gemm_problem> sp(cs.nprob);
    for (int i = 0; i < cs.nprob; ++i) {
      Prob& p = a.p[i];
      p.A = dA + szA * i;
      p.B = dB + szB * i;
      p.Bp = dBp + szB * i;
      p.bplane = (long)hB.size();
      p.C = dC + szC * i;
      p.M = cs.M;
      p.N = cs.N;
      p.K = cs.K;
      p.lda = L == 2 ? cs.M : cs.K;
      p.ldb = L == 0 ? cs.K : cs.N;
      p.ldc = cs.N;
      memset(&sp[i], 0, sizeof(sca_gemm_problem));
      sp[i].seg[0].A = p.A;
      sp[i].seg[0].B = p.B;
      sp[i].seg[0].lda = p.lda;
      sp[i].seg[0].ldb = p.ldb;
      sp[i].seg[0].K = p.K;
      sp[i].seg[0].alpha = 1.f;
      sp[i].nseg = 1;
      sp[i].M = p.M;
      sp[i].N = p.N;
      sp[i].C = dC2 + (long)cs.M * cs.N * i;
      sp[i].ldc = cs.N;
      sp[i].post_scale = 1.f;
    }
    const double gf = 2.0 * cs.M * cs.N * cs.K * cs.nprob * 1e-9;
    // library fp32 kernels
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 5; ++i) sca_gemm_partial(L, cs.nprob, sp.data(), cs.splitk, ws, st);
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) sca_gemm_partial(L, cs.nprob, sp.data(), cs.splitk, ws, st);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const float t_lib = ms * 1000.f / iters;
    printf("%-32s lib fp32 %7.1f us %6.1f TF\n", cs.name, t_lib, gf / t_lib * 1e-3 * 1e3);
    float tt[8] = {0};
    const char* tn[8] = {"128x128x16", "128x64x32", "64x128x32", "64x64x32", "128x128x32", "128x64x16",
                         "P128x128x16", "P128x64x32"};
    int nv = 6;
    switch (L) {
      case 0:
        tt[0] = run_x6<0, 128, 128, 16>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[1] = run_x6<0, 128, 64, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[2] = run_x6<0, 64, 128, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[3] = run_x6<0, 64, 64, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[4] = run_x6<0, 128, 128, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[5] = run_x6<0, 128, 64, 16>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[6] = run_x6<0, 128, 128, 16, true>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[7] = run_x6<0, 128, 64, 32, true>(a, cs.nprob, cs.M, cs.N, st, iters);
        nv = 8;
        break;
      case 1:
        tt[0] = run_x6<1, 128, 128, 16>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[1] = run_x6<1, 128, 64, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[2] = run_x6<1, 64, 128, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[3] = run_x6<1, 64, 64, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[4] = run_x6<1, 128, 128, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[5] = run_x6<1, 128, 64, 16>(a, cs.nprob, cs.M, cs.N, st, iters);
        break;
      default:
        tt[0] = run_x6<2, 128, 128, 16>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[1] = run_x6<2, 128, 64, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[2] = run_x6<2, 64, 128, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[3] = run_x6<2, 64, 64, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[4] = run_x6<2, 128, 128, 32>(a, cs.nprob, cs.M, cs.N, st, iters);
        tt[5] = run_x6<2, 128, 64, 16>(a, cs.nprob, cs.M, cs.N, st, iters);
        break;
    }
    for (int v = 0; v < nv; ++v) printf("    x6 %-11s %7.1f us %6.1f TF(fp32-eq)\n", tn[v], tt[v], gf / tt[v] * 1e3);
    CK(hipStreamSynchronize(st));
    CK(hipGetLastError());
    // accuracy (last x6 variant's output in dC, library's in dC2 / ws): problem 0, split 0
    // compared on 64 sampled rows of the (split 0) product against fp64
    std::vector<float> c1((long)cs.M * cs.N), c2((long)cs.M * cs.N);
    CK(hipMemcpy(c1.data(), dC, c1.size() * 4, hipMemcpyDeviceToHost));
    if (cs.splitk > 1) CK(hipMemcpy(c2.data(), ws, c2.size() * 4, hipMemcpyDeviceToHost));
    else CK(hipMemcpy(c2.data(), dC2, c2.size() * 4, hipMemcpyDeviceToHost));
    const int kc = cs.K / cs.splitk;
    double e_x6 = 0, e_lib = 0, e_x6n = 0, e_libn = 0;
    for (int mi = 0; mi < 64; ++mi) {
      const int m = (mi * 977) % cs.M;
      for (int n = 0; n < cs.N; ++n) {
        double s = 0, sa = 0;
        for (int k = 0; k < kc; ++k) {
          const double av = L == 2 ? hA[(long)k * cs.M + m] : hA[(long)m * cs.K + k];
          const double bv = L == 0 ? hB[(long)n * cs.K + k] : hB[(long)k * cs.N + n];
          s += av * bv;
          sa += fabs(av * bv);
        }
        const double d1 = fabs(c1[(long)m * cs.N + n] - s), d2 = fabs(c2[(long)m * cs.N + n] - s);
        e_x6 = fmax(e_x6, d1);
        e_lib = fmax(e_lib, d2);
        e_x6n = fmax(e_x6n, d1 / sa);
        e_libn = fmax(e_libn, d2 / sa);
      }
    }
    printf("    max|err| vs fp64: x6 %.3e (%.2e of sum|ab|)  lib fp32 %.3e (%.2e)\n", e_x6, e_x6n, e_lib, e_libn);
    CK(hipFree(dA));
    CK(hipFree(dB));
    CK(hipFree(dC));
    CK(hipFree(dC2));
    CK(hipFree(ws));
    CK(hipFree(dBp));
  }
  return 0;
}
