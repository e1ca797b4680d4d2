// Grouped fp32 GEMM on the gfx950 f32-input matrix cores (v_mfma_f32_32x32x2_f32).
//
// Replaces every nn.Linear forward / backward on the SCA hot path (see include/scatten.h
// for the reference call sites).  One launch runs up to SCA_GEMM_MAX_PROBLEMS independent
// problems (blockIdx.z) — e.g. the q/k/v projections of all keypoint streams at once — so
// that the small per-stream GEMMs (M = B*T = 2048, N,K = 256..768) fill the 256 CUs.
//
// Tile: BM x BN per 256-thread workgroup (4 waves, 2x2), each wave owns (BM/2) x (BN/2)
// built from 32x32 MFMA blocks.  K is staged through LDS in BK = 32 slices with a
// register prefetch of the next slice issued before the MFMAs of the current one.
//
// Operand images in LDS:
//   "k-contiguous" operand (A of NT/NN, B of NT): [rows][BK + 4]; a lane (r = l&31,
//     h = l>>5) reads one float4 = k {8g+4h .. 8g+4h+3} and feeds 4 MFMA k-steps, where
//     step s takes k = 8g + 4h + s (the MFMA's k index is a free permutation as long as A
//     and B agree).  Row stride 36 floats makes the ds_read_b128 conflict-free.
//   "row-contiguous" operand (B of NN, A and B of TN): [BK][rows + 4]; the same k map,
//     read as 4 ds_read_b32 (32 consecutive floats per half-wave: conflict-free).
//
// Numerics: exact f32 products, f32 accumulation (the MFMA is a k-ordered fmaf chain);
// summation order differs from ATen's, so results match the reference to ~1e-6 relative.
#include "common.h"
#include "../../include/scatten.h"

namespace {

constexpr int BK = 32;
constexpr int KC_STRIDE = BK + 4;  // k-contiguous image row stride (floats)

struct GemmArgs {
  sca_gemm_problem p[SCA_GEMM_MAX_PROBLEMS];
  int splitk;
  float* ws;
};

template <bool KCONTIG, int ROWS>
struct Operand {
  // LDS footprint in floats
  static constexpr int kLds = KCONTIG ? ROWS * KC_STRIDE : BK * (ROWS + 4);
  // float4 per thread for one BK slice of the tile
  static constexpr int kVec = ROWS * BK / 4 / 256;
};

// Load one BK-slice of an operand tile from global into registers (zero outside bounds).
// KCONTIG: global element (row, k) at base[row * ld + k];  else at base[k * ld + row].
template <bool KCONTIG, int ROWS>
__device__ __forceinline__ void load_tile(f32x4* reg, const float* base, int ld,
                                          int row0, int nrows, int k0, int kend, float alpha) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < Operand<KCONTIG, ROWS>::kVec; ++i) {
    const int e = t + i * 256;  // float4 index within the tile
    int row, k;
    if (KCONTIG) {
      row = e / (BK / 4);
      k = (e % (BK / 4)) * 4;
    } else {
      k = e / (ROWS / 4);
      row = (e % (ROWS / 4)) * 4;
    }
    const int gr = row0 + row, gk = k0 + k;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (KCONTIG) {
      if (gr < nrows && gk < kend) v = ld4(base + (long)gr * ld + gk);
    } else {
      if (gk < kend) {
        if (gr + 3 < nrows) {
          v = ld4(base + (long)gk * ld + gr);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (gr + j < nrows) v[j] = base[(long)gk * ld + gr + j];
        }
      }
    }
    reg[i] = v * alpha;
  }
}

template <bool KCONTIG, int ROWS>
__device__ __forceinline__ void store_tile(float* lds, const f32x4* reg) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < Operand<KCONTIG, ROWS>::kVec; ++i) {
    const int e = t + i * 256;
    if (KCONTIG) {
      const int row = e / (BK / 4), k = (e % (BK / 4)) * 4;
      st4(lds + row * KC_STRIDE + k, reg[i]);
    } else {
      const int k = e / (ROWS / 4), row = (e % (ROWS / 4)) * 4;
      st4(lds + k * (ROWS + 4) + row, reg[i]);
    }
  }
}

// Fragment for k-group g8 (8 k values), block row offset r0 within the tile.
template <bool KCONTIG, int ROWS>
__device__ __forceinline__ f32x4 read_frag(const float* lds, int r0, int g8, int lane) {
  const int r = r0 + (lane & 31);
  const int kb = g8 * 8 + (lane >> 5) * 4;
  if (KCONTIG) {
    return ld4(lds + r * KC_STRIDE + kb);
  } else {
    f32x4 v;
#pragma unroll
    for (int s = 0; s < 4; ++s) v[s] = lds[(kb + s) * (ROWS + 4) + r];
    return v;
  }
}

__device__ __forceinline__ float epilogue(const sca_gemm_problem& P, int m, int n, float v) {
  if (P.bias) v += P.bias[n];
  v *= P.post_scale;
  if (P.epi & SCA_EPI_GELU) {
    P.aux_out[(long)m * P.ldo + n] = v;
    v = gelu_erf(v);
  }
  if (P.epi & SCA_EPI_DGELU) v *= gelu_erf_grad(P.aux[(long)m * P.ldx + n]);
  if (P.resid) v += P.resid[(long)m * P.ldr + n];
  if (P.epi & SCA_EPI_ACCUM) v += P.C[(long)m * P.ldc + n];
  return v;
}

template <int LAYOUT, int BM, int BN>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmArgs args) {
  constexpr bool A_KC = (LAYOUT != SCA_GEMM_TN);
  constexpr bool B_KC = (LAYOUT == SCA_GEMM_NT);
  using OpA = Operand<A_KC, BM>;
  using OpB = Operand<B_KC, BN>;
  constexpr int RM = BM / 64, RN = BN / 64;  // 32x32 blocks per wave
  __shared__ __attribute__((aligned(16))) float smem[OpA::kLds + OpB::kLds];
  float* As = smem;
  float* Bs = smem + OpA::kLds;

  const int splitk = args.splitk;
  const int pid = blockIdx.z / splitk;
  const int ks = blockIdx.z % splitk;
  const sca_gemm_problem& P = args.p[pid];
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  if (m0 >= P.M || n0 >= P.N) return;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);

  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  f32x4 ra[OpA::kVec], rb[OpB::kVec];
  // fused bias gradient (TN): the first column tile sums its A slices (= alpha * dY rows)
  const bool do_bias = (LAYOUT == SCA_GEMM_TN) && P.bias_grad != nullptr && blockIdx.x == 0;
  float bsum = 0.f;

  for (int sidx = 0; sidx < P.nseg; ++sidx) {
    const sca_gemm_seg S = P.seg[sidx];
    int kbeg = 0, kend = S.K;
    if (splitk > 1) {
      const int chunk = ((S.K + splitk - 1) / splitk + BK - 1) / BK * BK;
      kbeg = ks * chunk;
      kend = min(S.K, kbeg + chunk);
    }
    if (kbeg >= kend) continue;
    load_tile<A_KC, BM>(ra, S.A, S.lda, m0, P.M, kbeg, kend, S.alpha);
    load_tile<B_KC, BN>(rb, S.B, S.ldb, n0, P.N, kbeg, kend, 1.0f);
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      __syncthreads();
      store_tile<A_KC, BM>(As, ra);
      store_tile<B_KC, BN>(Bs, rb);
      __syncthreads();
      if (k0 + BK < kend) {
        load_tile<A_KC, BM>(ra, S.A, S.lda, m0, P.M, k0 + BK, kend, S.alpha);
        load_tile<B_KC, BN>(rb, S.B, S.ldb, n0, P.N, k0 + BK, kend, 1.0f);
      }
      if (do_bias && threadIdx.x < BM) {
#pragma unroll 8
        for (int k = 0; k < BK; ++k) bsum += As[k * (BM + 4) + threadIdx.x];  // TN: A image is [BK][BM+4]
      }
#pragma unroll
      for (int g8 = 0; g8 < BK / 8; ++g8) {
        f32x4 fa[RM], fb[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) fa[i] = read_frag<A_KC, BM>(As, wm + i * 32, g8, lane);
#pragma unroll
        for (int j = 0; j < RN; ++j) fb[j] = read_frag<B_KC, BN>(Bs, wn + j * 32, g8, lane);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j) acc[i][j] = mfma32(fa[i][s], fb[j][s], acc[i][j]);
      }
    }
  }

  // C/D map of v_mfma_f32_32x32x2_f32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int col = lane & 31;
  const int rowh = 4 * (lane >> 5);
  if (do_bias && threadIdx.x < BM && m0 + (int)threadIdx.x < P.M) {
    if (splitk > 1)
      args.ws[(long)gridDim.z * P.M * P.N + (long)blockIdx.z * P.M + m0 + threadIdx.x] = bsum;
    else
      P.bias_grad[m0 + threadIdx.x] = bsum * P.bias_grad_scale;
  }
  if (splitk > 1) {
    float* slab = args.ws + (long)blockIdx.z * P.M * P.N;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + rowh;
          const int n = n0 + wn + j * 32 + col;
          if (m < P.M && n < P.N) slab[(long)m * P.N + n] = acc[i][j][r];
        }
    return;
  }
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + rowh;
        const int n = n0 + wn + j * 32 + col;
        if (m < P.M && n < P.N) P.C[(long)m * P.ldc + n] = epilogue(P, m, n, acc[i][j][r]);
      }
}

// Fixed-order split-K reduction + epilogue: C = epi(sum_s slab[s]); bias partials likewise.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmArgs args, int nprob) {
  const sca_gemm_problem& P = args.p[blockIdx.y];
  const long MN = (long)P.M * P.N;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= MN) {
    const long m = e - MN;
    if (P.bias_grad && m < P.M) {
      const float* bp = args.ws + (long)nprob * args.splitk * MN + (long)blockIdx.y * args.splitk * P.M + m;
      float v = 0.f;
      for (int s = 0; s < args.splitk; ++s) v += bp[(long)s * P.M];
      P.bias_grad[m] = v * P.bias_grad_scale;
    }
    return;
  }
  const int m = (int)(e / P.N), n = (int)(e % P.N);
  const float* slab = args.ws + (long)blockIdx.y * args.splitk * MN + e;
  float v = 0.f;
  for (int s = 0; s < args.splitk; ++s) v += slab[s * MN];
  P.C[(long)m * P.ldc + n] = epilogue(P, m, n, v);
}

template <int LAYOUT, int BM, int BN>
int launch(const GemmArgs& a, int nprob, int maxM, int maxN, hipStream_t st) {
  dim3 grid((maxN + BN - 1) / BN, (maxM + BM - 1) / BM, nprob * a.splitk);
  hipLaunchKernelGGL((gemm_kernel<LAYOUT, BM, BN>), grid, dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? SCA_OK : SCA_ERR_LAUNCH;
}

}  // namespace

extern "C" void sca_set_error(const char* msg);

extern "C" int sca_gemm(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
                        void* stream) {
  if (nprob <= 0) return SCA_OK;
  if (nprob > SCA_GEMM_MAX_PROBLEMS || layout < 0 || layout > 2 || splitk < 1) {
    sca_set_error("sca_gemm: bad nprob/layout/splitk");
    return SCA_ERR_ARG;
  }
  GemmArgs a;
  a.splitk = splitk;
  a.ws = workspace;
  int maxM = 0, maxN = 0;
  for (int i = 0; i < nprob; ++i) {
    const sca_gemm_problem& P = probs[i];
    if (P.nseg < 1 || P.nseg > SCA_GEMM_MAX_SEGS || P.M < 0 || P.N < 0 || !P.C) {
      sca_set_error("sca_gemm: bad problem");
      return SCA_ERR_ARG;
    }
    for (int s = 0; s < P.nseg; ++s) {
      const sca_gemm_seg& S = P.seg[s];
      const bool a_kc = layout != SCA_GEMM_TN, b_kc = layout == SCA_GEMM_NT;
      if ((S.K & 3) || !S.A || !S.B || (S.lda & 3) || (S.ldb & 3) ||
          (reinterpret_cast<uintptr_t>(S.A) & 15) || (reinterpret_cast<uintptr_t>(S.B) & 15)) {
        sca_set_error("sca_gemm: K, lda, ldb must be multiples of 4 and A/B 16-byte aligned");
        return SCA_ERR_ARG;
      }
      if ((a_kc && S.lda < S.K) || (!a_kc && S.lda < P.M) || (b_kc && S.ldb < S.K) || (!b_kc && S.ldb < P.N)) {
        sca_set_error("sca_gemm: leading dimension too small");
        return SCA_ERR_ARG;
      }
    }
    if ((P.epi & SCA_EPI_GELU) && !P.aux_out) { sca_set_error("sca_gemm: GELU needs aux_out"); return SCA_ERR_ARG; }
    if ((P.epi & SCA_EPI_DGELU) && !P.aux) { sca_set_error("sca_gemm: DGELU needs aux"); return SCA_ERR_ARG; }
    if (P.bias_grad && layout != SCA_GEMM_TN) { sca_set_error("sca_gemm: bias_grad only with TN"); return SCA_ERR_ARG; }
    if (splitk > 1 && (P.nseg != 1 || P.M != probs[0].M || P.N != probs[0].N)) {
      sca_set_error("sca_gemm: split-K needs one segment and equal M,N");
      return SCA_ERR_ARG;
    }
    a.p[i] = P;
    maxM = maxM > P.M ? maxM : P.M;
    maxN = maxN > P.N ? maxN : P.N;
  }
  if (splitk > 1 && !workspace) { sca_set_error("sca_gemm: split-K needs workspace"); return SCA_ERR_ARG; }
  if (maxM == 0 || maxN == 0) return SCA_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int rc;
  switch (layout) {
    case SCA_GEMM_NT: rc = launch<SCA_GEMM_NT, 64, 64>(a, nprob, maxM, maxN, st); break;
    case SCA_GEMM_NN: rc = launch<SCA_GEMM_NN, 64, 64>(a, nprob, maxM, maxN, st); break;
    default: rc = launch<SCA_GEMM_TN, 64, 64>(a, nprob, maxM, maxN, st); break;
  }
  if (rc != SCA_OK) { sca_set_error("sca_gemm: launch failed"); return rc; }
  if (splitk > 1) {
    const long MN = (long)maxM * maxN;
    dim3 grid((unsigned)((MN + maxM + 255) / 256), nprob);
    hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, st, a, nprob);
    if (hipGetLastError() != hipSuccess) { sca_set_error("sca_gemm: reduce launch failed"); return SCA_ERR_LAUNCH; }
  }
  return SCA_OK;
}
