#include <stdlib.h>

#include <type_traits>
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

constexpr int KPAD = 4;  // LDS row padding (floats)

struct GemmArgs {
  sca_gemm_problem p[SCA_GEMM_MAX_PROBLEMS];
  int splitk;
  float* ws;
  const unsigned long long* drop_off;           // dropout step counter (sca_dropout_offset)
  long slab_off[SCA_GEMM_MAX_PROBLEMS];         // split-K: problem's first partial slab in ws
  long bias_off[SCA_GEMM_MAX_PROBLEMS];         // split-K: problem's first bias partial row in ws
  unsigned* counters;                           // split-K combined in-launch (sca_gemm_splitk_fused)
  int nprob;                                    // problems in p[]
  // flat grid (gemm_tnk_kernel): workgroups of problem i are tile_beg[i] .. tile_beg[i + 1] - 1,
  // its own tiles x splits only — problems of different shapes share a launch without the
  // empty workgroups of a max-shape grid
  int flat;
  int tile_beg[SCA_GEMM_MAX_PROBLEMS + 1];
};

// Workgroup tile configuration.
template <int BM_, int BN_, int WM_, int WN_, int BK_, int STAGES_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = BK_, STAGES = STAGES_;
  static constexpr int NT = 64 * WM * WN;             // threads
  static constexpr int TM = BM / WM, TN = BN / WN;     // wave tile
  static constexpr int RM = TM / 32, RN = TN / 32;     // 32x32 MFMA blocks per wave
  static_assert(TM % 32 == 0 && TN % 32 == 0, "wave tile must be a multiple of 32");
};

template <bool KCONTIG, int ROWS, int BK, int NT>
struct Operand {
  static constexpr int kLds = KCONTIG ? ROWS * (BK + KPAD) : BK * (ROWS + KPAD);  // floats
  static constexpr int kVec = ROWS * BK / 4 / NT;  // float4 per thread per K-slice
  static_assert(kVec >= 1 && ROWS * BK / 4 == kVec * NT, "tile not divisible among threads");
};

// Load one BK-slice of an operand tile from global into registers (zero outside bounds).
// KCONTIG: global element (row, k) at base[row * ld + k];  else at base[k * ld + row].
// VEC = false: element-wise loads with every element bounds-checked — the any-shape path
// (K, ld not multiples of 4, operands not 16-byte aligned: CoordinatesFusion's per-clip
// (T/4 x T/4) attention at any frame count, model/fusion.py:52-55).
template <bool KCONTIG, int ROWS, int BK, int NT, bool VEC = true>
__device__ __forceinline__ void load_tile(f32x4* reg, const float* base, int ld, int row0, int nrows, int k0,
                                          int kend) {
#pragma unroll
  for (int i = 0; i < Operand<KCONTIG, ROWS, BK, NT>::kVec; ++i) {
    const int e = threadIdx.x + i * NT;  // float4 index within the tile
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
    if (!VEC) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (KCONTIG) {
          if (gr < nrows && gk + j < kend) v[j] = base[(long)gr * ld + gk + j];
        } else if (gk < kend && gr + j < nrows) {
          v[j] = base[(long)gk * ld + gr + j];
        }
      }
    } else if (KCONTIG) {
      if (gr < nrows && gk < kend) v = ld4(base + (long)gr * ld + gk);
    } else if (gk < kend) {
      if (gr + 3 < nrows) {
        v = ld4(base + (long)gk * ld + gr);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (gr + j < nrows) v[j] = base[(long)gk * ld + gr + j];
      }
    }
    reg[i] = v;
  }
}

// alpha is applied here, not at load time: a multiply right after the global load would
// make the wave wait for the prefetch before the MFMAs it is meant to overlap.
template <bool KCONTIG, int ROWS, int BK, int NT>
__device__ __forceinline__ void store_tile(float* lds, const f32x4* reg, float alpha) {
#pragma unroll
  for (int i = 0; i < Operand<KCONTIG, ROWS, BK, NT>::kVec; ++i) {
    const int e = threadIdx.x + i * NT;
    const f32x4 v = reg[i] * alpha;
    if (KCONTIG) {
      const int row = e / (BK / 4), k = (e % (BK / 4)) * 4;
      st4(lds + row * (BK + KPAD) + k, v);
    } else {
      const int k = e / (ROWS / 4), row = (e % (ROWS / 4)) * 4;
      st4(lds + k * (ROWS + KPAD) + row, v);
    }
  }
}

// Fragment for k-group g8 (8 k values), block row offset r0 within the tile.
template <bool KCONTIG, int ROWS, int BK>
__device__ __forceinline__ f32x4 read_frag(const float* lds, int r0, int g8, int lane) {
  const int r = r0 + (lane & 31);
  const int kb = g8 * 8 + (lane >> 5) * 4;
  if (KCONTIG) return ld4(lds + r * (BK + KPAD) + kb);
  f32x4 v;
#pragma unroll
  for (int s = 0; s < 4; ++s) v[s] = lds[(kb + s) * (ROWS + KPAD) + r];
  return v;
}

__device__ __forceinline__ float epilogue(const sca_gemm_problem& P, int m, int n, float v,
                                          const unsigned long long* drop_off) {
  if (P.bias) v += P.bias[n];
  v *= P.post_scale;
  if (P.epi & SCA_EPI_GELU) {
    P.aux_out[(long)m * P.ldo + n] = v;
    v = gelu_erf(v);
  }
  if (P.epi & SCA_EPI_DROPOUT) {
    DropMask dm;
    dm.init(P.drop_seed, P.drop_p, drop_off);
    v = dm.apply((uint32_t)m * (uint32_t)P.N + (uint32_t)n, v);
  }
  if (P.epi & SCA_EPI_DGELU) v *= gelu_erf_grad(P.aux[(long)m * P.ldx + n]);
  if (P.resid) v += P.resid[(long)m * P.ldr + n];
  if (P.epi & SCA_EPI_ACCUM) v += P.C[(long)m * P.ldc + n];
  return v;
}

// Non-split epilogue of one wave's (RM x RN) 32x32 blocks: all loads of a block first (one
// wait), then compute + store.  Order: v = (acc + bias) * post_scale; GELU (keeps the
// pre-activation) / GELU'; + (resid + C_old).
template <int RM, int RN>
__device__ __forceinline__ void epilogue_block(const sca_gemm_problem& P, const f32x16 (&acc)[RM][RN], int mb, int nb,
                                               int col, int rowh, const unsigned long long* drop_off) {
  DropMask dm;
  if (P.epi & SCA_EPI_DROPOUT) dm.init(P.drop_seed, P.drop_p, drop_off);
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = nb + j * 32 + col;
      const bool nok = n < P.N;
      const float bias = (P.bias && nok) ? P.bias[n] : 0.f;
      float ex[16], ax[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + i * 32 + (r & 3) + 8 * (r >> 2) + rowh;
        const bool ok = nok && m < P.M;
        float e = 0.f;
        if (ok && P.resid) e += P.resid[(long)m * P.ldr + n];
        if (ok && (P.epi & SCA_EPI_ACCUM)) e += P.C[(long)m * P.ldc + n];
        ex[r] = e;
        ax[r] = (ok && (P.epi & SCA_EPI_DGELU)) ? P.aux[(long)m * P.ldx + n] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + i * 32 + (r & 3) + 8 * (r >> 2) + rowh;
        if (!nok || m >= P.M) continue;
        float v = (acc[i][j][r] + bias) * P.post_scale;
        if (P.epi & SCA_EPI_GELU) {
          P.aux_out[(long)m * P.ldo + n] = v;
          v = gelu_erf(v);
        }
        if (P.epi & SCA_EPI_DROPOUT) v = dm.apply((uint32_t)m * (uint32_t)P.N + (uint32_t)n, v);
        if (P.epi & SCA_EPI_DGELU) v *= gelu_erf_grad(ax[r]);
        P.C[(long)m * P.ldc + n] = v + ex[r];
      }
    }
}

// Row-form epilogue of one wave's 32x32 accumulator (the LDS-DMA kernels): the tile is
// transposed through a wave-private LDS scratch (row stride 40 floats: the two half-waves'
// rows 4 apart land 128 B apart, conflict-free) so that each lane owns 4 float4 row pieces
// (rows lane/8 + 8i, columns 4*(lane%8)) and every epilogue load / store is 16 B per lane —
// a quarter of the store instructions of the per-element form (the epilogue tail of these
// short-K launches is store-issue-bound).  Requires N % 4 == 0 (glds_ok).
constexpr int EPI_LD = 40;

__device__ __forceinline__ void acc_to_rows(const f32x16& acc, float* scratch, int lane, f32x4 (&v)[4]) {
  const int col = lane & 31, rowh = 4 * (lane >> 5);
#pragma unroll
  for (int r = 0; r < 16; ++r) scratch[((r & 3) + 8 * (r >> 2) + rowh) * EPI_LD + col] = acc[r];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = ld4(scratch + ((lane >> 3) + 8 * i) * EPI_LD + 4 * (lane & 7));
}

// v = (acc + bias) * post_scale; GELU (keeps the pre-activation) / dropout / GELU'; + resid
// (+ C_old): exactly epilogue()'s order, on float4 row pieces
__device__ __forceinline__ void epilogue_rows(const sca_gemm_problem& P, const f32x4 (&v)[4], int mb, int nb, int lane,
                                              const unsigned long long* drop_off) {
  const int n = nb + 4 * (lane & 7);
  if (n >= P.N) return;
  DropMask dm;
  if (P.epi & SCA_EPI_DROPOUT) dm.init(P.drop_seed, P.drop_p, drop_off);
  const f32x4 bias = P.bias ? ld4(P.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mb + (lane >> 3) + 8 * i;
    if (m >= P.M) continue;
    f32x4 ex = {0.f, 0.f, 0.f, 0.f}, ax = ex;
    if (P.resid) ex += ld4(P.resid + (long)m * P.ldr + n);
    if (P.epi & SCA_EPI_ACCUM) ex += ld4(P.C + (long)m * P.ldc + n);
    if (P.epi & SCA_EPI_DGELU) ax = ld4(P.aux + (long)m * P.ldx + n);
    f32x4 o = (v[i] + bias) * P.post_scale;
    if (P.epi & SCA_EPI_GELU) {
      st4(P.aux_out + (long)m * P.ldo + n, o);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = gelu_erf(o[j]);
    }
    if (P.epi & SCA_EPI_DROPOUT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = dm.apply((uint32_t)m * (uint32_t)P.N + (uint32_t)(n + j), o[j]);
    }
    if (P.epi & SCA_EPI_DGELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] *= gelu_erf_grad(ax[j]);
    }
    st4(P.C + (long)m * P.ldc + n, o + ex);
  }
}

// split-K partial slab of the same tile, float4 rows
__device__ __forceinline__ void slab_rows(float* slab, const f32x4 (&v)[4], int M, int N, int mb, int nb, int lane) {
  const int n = nb + 4 * (lane & 7);
  if (n >= N) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mb + (lane >> 3) + 8 * i;
    if (m < M) st4(slab + (long)m * N + n, v[i]);
  }
}

template <int LAYOUT, class C, bool VEC = true>
__global__ __launch_bounds__(C::NT) void gemm_kernel(const GemmArgs args) {
  constexpr int BM = C::BM, BN = C::BN, BK = C::BK, NT = C::NT, RM = C::RM, RN = C::RN;
  constexpr bool A_KC = (LAYOUT != SCA_GEMM_TN);
  constexpr bool B_KC = (LAYOUT == SCA_GEMM_NT);
  using OpA = Operand<A_KC, BM, BK, NT>;
  using OpB = Operand<B_KC, BN, BK, NT>;
  constexpr int STAGE = OpA::kLds + OpB::kLds;
  __shared__ __attribute__((aligned(16))) float smem[C::STAGES * STAGE];

  // XCD-aware remap (cdna_hip_programming.md T1): hardware deals workgroups round-robin over
  // the 8 XCDs; give each XCD a contiguous range of logical tiles (n fastest, then m, then
  // problem / K-split) so tiles sharing an A row-block or a B column-block share one L2.
  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned nwg = gx * gy * gridDim.z;
  const unsigned orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int bx = wgid % gx, by = (wgid / gx) % gy, bz = wgid / (gx * gy);

  const int splitk = args.splitk;
  const int pid = bz / splitk;
  const int ks = bz % splitk;
  const sca_gemm_problem& P = args.p[pid];
  const int m0 = by * BM, n0 = bx * BN;
  if (m0 >= P.M || n0 >= P.N) return;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave / C::WN) * C::TM, wn = (wave % C::WN) * C::TN;

  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  f32x4 ra[OpA::kVec], rb[OpB::kVec];
  // fused bias gradient (TN): the first column tile sums its A slices (= alpha * dY rows)
  const bool do_bias = (LAYOUT == SCA_GEMM_TN) && P.bias_grad != nullptr && bx == 0;
  float bsum = 0.f;

  // flatten (segment, K-slice) into one sequence so the pipeline runs across segments
  int seg_kbeg[SCA_GEMM_MAX_SEGS], seg_kend[SCA_GEMM_MAX_SEGS], seg_n[SCA_GEMM_MAX_SEGS];
  int total = 0;
#pragma unroll
  for (int s = 0; s < SCA_GEMM_MAX_SEGS; ++s) {
    seg_kbeg[s] = seg_kend[s] = seg_n[s] = 0;
    if (s < P.nseg) {
      int kbeg = 0, kend = P.seg[s].K;
      if (splitk > 1) {
        const int chunk = ((P.seg[s].K + splitk - 1) / splitk + BK - 1) / BK * BK;
        kbeg = ks * chunk;
        kend = min(P.seg[s].K, kbeg + chunk);
      }
      seg_kbeg[s] = kbeg;
      seg_kend[s] = kend;
      seg_n[s] = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
      total += seg_n[s];
    }
  }
  float alpha_f = 1.f;  // alpha of the segment held in ra
  auto fetch = [&](int t) {
    int s = 0;
    while (s + 1 < P.nseg && t >= seg_n[s]) { t -= seg_n[s]; ++s; }
    const sca_gemm_seg& S = P.seg[s];
    const int k0 = seg_kbeg[s] + t * BK;
    load_tile<A_KC, BM, BK, NT, VEC>(ra, S.A, S.lda, m0, P.M, k0, seg_kend[s]);
    load_tile<B_KC, BN, BK, NT, VEC>(rb, S.B, S.ldb, n0, P.N, k0, seg_kend[s]);
    alpha_f = S.alpha;
  };
  auto compute = [&](const float* As, const float* Bs) {
    if (do_bias && threadIdx.x < BM) {
#pragma unroll 8
      for (int k = 0; k < BK; ++k) bsum += As[k * (BM + KPAD) + threadIdx.x];  // TN: A image is [BK][BM+4]
    }
#pragma unroll
    for (int g8 = 0; g8 < BK / 8; ++g8) {
      f32x4 fa[RM], fb[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) fa[i] = read_frag<A_KC, BM, BK>(As, wm + i * 32, g8, lane);
#pragma unroll
      for (int j = 0; j < RN; ++j) fb[j] = read_frag<B_KC, BN, BK>(Bs, wn + j * 32, g8, lane);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) acc[i][j] = mfma32(fa[i][s], fb[j][s], acc[i][j]);
    }
  };

  if (C::STAGES == 1) {
    if (total > 0) fetch(0);
    for (int t = 0; t < total; ++t) {
      __syncthreads();
      store_tile<A_KC, BM, BK, NT>(smem, ra, alpha_f);
      store_tile<B_KC, BN, BK, NT>(smem + OpA::kLds, rb, 1.0f);
      __syncthreads();
      if (t + 1 < total) fetch(t + 1);
      compute(smem, smem + OpA::kLds);
    }
  } else {
    if (total > 0) {
      fetch(0);
      store_tile<A_KC, BM, BK, NT>(smem, ra, alpha_f);
      store_tile<B_KC, BN, BK, NT>(smem + OpA::kLds, rb, 1.0f);
      __syncthreads();
    }
    for (int t = 0; t < total; ++t) {
      const float* As = smem + (t & 1) * STAGE;
      if (t + 1 < total) fetch(t + 1);  // global loads in flight during the MFMAs below
      compute(As, As + OpA::kLds);
      if (t + 1 < total) {
        float* An = smem + ((t + 1) & 1) * STAGE;
        store_tile<A_KC, BM, BK, NT>(An, ra, alpha_f);
        store_tile<B_KC, BN, BK, NT>(An + OpA::kLds, rb, 1.0f);
      }
      __syncthreads();
    }
  }

  // C/D map of v_mfma_f32_32x32x2_f32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int col = lane & 31;
  const int rowh = 4 * (lane >> 5);
  if (do_bias && threadIdx.x < BM && m0 + (int)threadIdx.x < P.M) {
    if (splitk > 1)
      args.ws[args.bias_off[pid] + (long)ks * P.M + m0 + threadIdx.x] = bsum;
    else
      P.bias_grad[m0 + threadIdx.x] = bsum * P.bias_grad_scale;
  }
  if (splitk > 1) {
    float* slab = args.ws + args.slab_off[pid] + (long)ks * P.M * P.N;
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
  epilogue_block<RM, RN>(P, acc, m0 + wm, n0 + wn, col, rowh, args.drop_off);
}
// ------------------------------------------------------------------------------ LDS-DMA kernel
// 64x64 tile, 4 waves (32x32 each), BK = 32, an S-stage LDS ring filled by
// global_load_lds_dwordx4 (no VGPR staging, no ds_write pass), one raw barrier per slice
// and a counted vmcnt that keeps S-2 slices in flight across it.
//   k-contiguous operand tile [64 rows][32 k] (128-B rows, 8 rows per 1-KiB DMA piece):
//     float4 slot s of row r lives at slot s ^ ((r >> 1) & 7) — the swizzle is applied on
//     the per-lane SOURCE address (the DMA image is lane-linear) and on the fragment read;
//     conflict-free for the 32x32x2 fragment pattern in all four ds_read_b128 lane groups.
//   k-major operand tile [32 k][64 cols] (256-B rows, 4 per piece), unswizzled: a fragment
//     is ds_read_b32 of 32 consecutive floats per half-wave (conflict-free).
// Requirements (else the register-staged kernel runs): every segment's K (per split-K
// chunk) a multiple of 32, M and N multiples of 4, one alpha for all segments of a
// problem (applied to the accumulator).  Rows / columns past M, N are clamped on load and
// never stored.
// Wave priority of the backward's critical-chain kernels (input gradients, GEMM + LayerNorm
// backward, attention backward): they share CUs with the weight-gradient launches of the side
// stream, and s_setprio makes the SIMD arbiter issue their instructions first when both are
// ready (the weight gradients keep priority 0 and fill the gaps)
#ifndef SCA_CRIT_PRIO
#define SCA_CRIT_PRIO 2
#endif
constexpr int GL_BM = 64, GL_BN = 64, GL_BK = 32;
constexpr int GL_PIECE = 1024;                  // bytes per DMA wave-instruction
constexpr int GL_OP_BYTES = GL_BM * GL_BK * 4;  // 8 KiB per operand per stage

__device__ __forceinline__ int gl_swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void gl_dma(const float* src, char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void gl_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Per-lane source of this wave's two DMA pieces of one operand tile for K-slice at k0.
// KC: element (row, k) at base[row*ld + k]; else at base[k*ld + row].
template <bool KC>
__device__ __forceinline__ const float* gl_src(const float* base, int ld, int row0, int nrows, int k0, int c,
                                               int wave, int lane) {
  if (KC) {
    const int r = 16 * wave + 8 * c + (lane >> 3);
    const int ks = (lane & 7) ^ gl_swz(r);
    return base + (long)min(row0 + r, nrows - 1) * ld + k0 + 4 * ks;
  } else {
    const int kr = 4 * (2 * wave + c) + (lane >> 4);
    return base + (long)(k0 + kr) * ld + min(row0 + 4 * (lane & 15), nrows - 4);
  }
}

template <bool KC>
__device__ __forceinline__ int gl_dst(int c, int wave) {
  return KC ? (16 * wave + 8 * c) * 128 : (2 * wave + c) * GL_PIECE;
}

// 32x32x2 fragment for k-group g (k = 8g + 4h + j, j = 0..3) of rows r0 .. r0+31
template <bool KC>
__device__ __forceinline__ f32x4 gl_frag(const char* img, int r0, int g, int lane) {
  const int r = r0 + (lane & 31), h = lane >> 5;
  if (KC) return *(const f32x4*)(img + r * 128 + 16 * ((2 * g + h) ^ gl_swz(r)));
  const float* f = (const float*)img;
  f32x4 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = f[(8 * g + 4 * h + j) * 64 + r];
  return v;
}

// ---- in-launch split-K combine (write-through slabs + arrival ticket, last arriver sums) ----
// MI355X_MICROARCH.md § inter-workgroup visibility / cdna_hip_programming.md §6 G16 R1: the slab
// bytes are stored write-through (sc1, buffer stores with aux = 16), every storing wave drains
// (vmcnt 0) before the workgroup's barrier, ONE lane takes a ticket (relaxed agent-scope
// atomic add on the tile's counter); the workgroup that draws splitk - 1 reads every slab with
// sc1 loads (no acquire fence needed for sc1-stored, sc1-loaded bytes), in slice order 0 ..
// splitk-1 whichever arrived last (deterministic), resets the counter to 0 and runs the
// epilogue.  Correct for any placement of a tile's slices over XCDs / CUs.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void slab_rows_sc1(float* slab_base, long slab_floats, const f32x4 (&v)[4], int M, int N,
                                              int mb, int nb, int lane, long off0) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slab_base, 0, (int)(slab_floats * 4), 0x00020000);
  const int n = nb + 4 * (lane & 7);
  if (n >= N) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mb + (lane >> 3) + 8 * i;
    if (m < M) {
      const f32x4 x = v[i];
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(&x), rs,
                                             (int)((off0 + (long)m * N + n) * 4), 0, 16);
    }
  }
}

__device__ __forceinline__ f32x4 ld4_sc1(__amdgpu_buffer_rsrc_t rs, long float_off) {
  const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(float_off * 4), 0, 16);
  return *reinterpret_cast<const f32x4*>(&r);
}

#ifdef SCA_GEMM_STAMPS
// Diagnostic build only (make stamps): per-workgroup s_memrealtime stamps (100 MHz) at
// entry, first slice landed, main loop done, epilogue done -> tools/gemm_stamps.py
constexpr int STAMP_MAX = 16384;
__device__ unsigned long long g_stamps[STAMP_MAX][5];
__device__ unsigned long long g_clk[STAMP_MAX][2];  // s_memtime (shader clock) at entry / loop done
#define SCA_STAMP(slot)                                                            \
  do {                                                                             \
    if (threadIdx.x == 0 && stamp_id < STAMP_MAX) {                                \
      g_stamps[stamp_id][slot] = __builtin_amdgcn_s_memrealtime();                 \
      if ((slot) == 0 || (slot) == 2) g_clk[stamp_id][(slot) / 2] = __builtin_amdgcn_s_memtime(); \
    }                                                                              \
  } while (0)
#else
#define SCA_STAMP(slot) \
  do {                  \
  } while (0)
#endif

template <int LAYOUT, int S>
__global__ __launch_bounds__(256) void gemm_glds_kernel(const GemmArgs args) {
  if constexpr (LAYOUT == SCA_GEMM_NN && SCA_CRIT_PRIO > 0) __builtin_amdgcn_s_setprio(SCA_CRIT_PRIO);
  constexpr bool A_KC = (LAYOUT != SCA_GEMM_TN);
  constexpr bool B_KC = (LAYOUT == SCA_GEMM_NT);
  constexpr int STAGE = 2 * GL_OP_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[S * STAGE];
#ifdef SCA_GEMM_STAMPS
  const unsigned stamp_id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  if (threadIdx.x == 0 && stamp_id < STAMP_MAX) g_stamps[stamp_id][4] = (unsigned long long)__smid();
#endif
  SCA_STAMP(0);

  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned nwg = gx * gy * gridDim.z;
  const unsigned orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int bx = wgid % gx, by = (wgid / gx) % gy, bz = wgid / (gx * gy);

  const int splitk = args.splitk;
  const int pid = bz / splitk;
  const int ks = bz % splitk;
  const sca_gemm_problem& P = args.p[pid];
  const int m0 = by * GL_BM, n0 = bx * GL_BN;
  if (m0 >= P.M || n0 >= P.N) return;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;

  // flattened (segment, K-slice) sequence; every chunk is a whole number of slices
  int seg_kbeg[SCA_GEMM_MAX_SEGS], seg_n[SCA_GEMM_MAX_SEGS];
  int total = 0;
#pragma unroll
  for (int s = 0; s < SCA_GEMM_MAX_SEGS; ++s) {
    seg_kbeg[s] = seg_n[s] = 0;
    if (s < P.nseg) {
      int kbeg = 0, kend = P.seg[s].K;
      if (splitk > 1) {
        const int chunk = ((P.seg[s].K + splitk - 1) / splitk + GL_BK - 1) / GL_BK * GL_BK;
        kbeg = ks * chunk;
        kend = min(P.seg[s].K, kbeg + chunk);
      }
      seg_kbeg[s] = kbeg;
      seg_n[s] = kend > kbeg ? (kend - kbeg) / GL_BK : 0;
      total += seg_n[s];
    }
  }
  // Issue-side state: this lane's DMA source pointers at the first slice of the segment being
  // issued, and the per-slice step; recomputed only when the issue crosses into the next
  // segment (slices are issued in order), so a slice costs two pointer adds.
  int iseg = -1, tseg0 = 0, tend = 0;
  const float* pa[2] = {nullptr, nullptr};
  const float* pb[2] = {nullptr, nullptr};
  long stepA = 0, stepB = 0;
  auto dma = [&](int t, int stage) {
    while (t >= tend) {
      ++iseg;
      tseg0 = tend;
      tend += seg_n[iseg];
      const sca_gemm_seg& G = P.seg[iseg];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        pa[c] = gl_src<A_KC>(G.A, G.lda, m0, P.M, seg_kbeg[iseg], c, wave, lane);
        pb[c] = gl_src<B_KC>(G.B, G.ldb, n0, P.N, seg_kbeg[iseg], c, wave, lane);
      }
      stepA = A_KC ? GL_BK : (long)GL_BK * G.lda;
      stepB = B_KC ? GL_BK : (long)GL_BK * G.ldb;
    }
    const long kk = t - tseg0;
    char* base = smem + stage * STAGE;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      gl_dma(pa[c] + kk * stepA, base + gl_dst<A_KC>(c, wave));
      gl_dma(pb[c] + kk * stepB, base + GL_OP_BYTES + gl_dst<B_KC>(c, wave));
    }
  };

  const bool do_bias = (LAYOUT == SCA_GEMM_TN) && P.bias_grad != nullptr && bx == 0;
  float bsum = 0.f;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < total) dma(i, i);
  for (int t = 0; t < total; ++t) {
    // slice t landed for this wave (4 DMA pieces per slice; S-2 younger slices may fly)
    if (t + S - 2 < total) gl_wait_vm<4 * (S - 2)>();
    else gl_wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // every wave's pieces of slice t landed; slice t-1 fully read
    __builtin_amdgcn_sched_barrier(0);
#ifdef SCA_GEMM_STAMPS
    if (t == 0) SCA_STAMP(1);
#endif
    if (t + S - 1 < total) dma(t + S - 1, (t + S - 1) % S);
    const char* As = smem + (t % S) * STAGE;
    const char* Bs = As + GL_OP_BYTES;
    f32x4 fa[4], fb[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      fa[g] = gl_frag<A_KC>(As, wm, g, lane);
      fb[g] = gl_frag<B_KC>(Bs, wn, g, lane);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma32(fa[g][j], fb[g][j], acc);
    // bias gradient (TN: colsum of dY = the A tile's row sums) from the A fragments already
    // in registers: waves 0 and 2 hold rows wm .. wm+31, a lane k = 8g + 4h + j of its row
    // (the two half-waves' partials are combined after the loop).  Earlier form: wave 0
    // re-read the whole A image from LDS every slice (4 LDS round trips + a serial add
    // chain), which made the bias tiles the launch's slowest workgroups.
    if (do_bias && (wave & 1) == 0) {
      f32x4 s4 = (fa[0] + fa[1]) + (fa[2] + fa[3]);
      bsum += (s4[0] + s4[1]) + (s4[2] + s4[3]);
    }
  }

  const float alpha = P.seg[0].alpha;
  const bool fused_k = splitk > 1 && args.counters != nullptr;  // in-launch split-K combine
  if (do_bias) bsum += __shfl_xor(bsum, 32, 64);  // the two k halves of a row
  const int brow = wm + lane;                     // this lane's bias row (waves 0, 2; lanes < 32)
  if (do_bias && (wave & 1) == 0 && lane < 32 && m0 + brow < P.M) {
    float* bp = args.ws + args.bias_off[pid] + (long)ks * P.M + m0 + brow;
    if (fused_k)
      __hip_atomic_store(bp, bsum * alpha, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1 store
    else if (splitk > 1)
      *bp = bsum * alpha;
    else
      P.bias_grad[m0 + brow] = bsum * alpha * P.bias_grad_scale;
  }
  if (alpha != 1.f) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] *= alpha;
  }
  SCA_STAMP(2);
  // the ring is free once every wave has passed its last slice: wave-private transposition
  // scratch for the row-form epilogue (4 x 5 KB)
  __syncthreads();
  f32x4 rows[4];
  acc_to_rows(acc, reinterpret_cast<float*>(smem) + wave * 32 * EPI_LD, lane, rows);
  if (fused_k) {
    const long MN = (long)P.M * P.N;
    float* slabs = args.ws + args.slab_off[pid];
    slab_rows_sc1(slabs, (long)splitk * MN, rows, P.M, P.N, m0 + wm, n0 + wn, lane, (long)ks * MN);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    unsigned* flag = reinterpret_cast<unsigned*>(smem + 20 * 1024);  // one LDS array (trap 4a)
    unsigned* cnt = args.counters + (long)pid * gx * gy + (long)by * gx + bx;
    if (threadIdx.x == 0)
      *flag = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(splitk - 1);
    __syncthreads();
    if (!*flag) return;
    if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // sc1-stored, sc1-loaded: no agent acquire
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slabs, 0, (int)(splitk * MN * 4), 0x00020000);
    const int n = n0 + wn + 4 * (lane & 7);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = min(m0 + wm + (lane >> 3) + 8 * i, P.M - 1);
      const long e = (long)m * P.N + min(n, P.N - 4);
      f32x4 t = ld4_sc1(rs, e);
      for (int s2 = 1; s2 < splitk; ++s2) t += ld4_sc1(rs, s2 * MN + e);
      rows[i] = t;
    }
    if (do_bias && threadIdx.x < GL_BM && m0 + (int)threadIdx.x < P.M) {
      float* bp = args.ws + args.bias_off[pid] + m0 + threadIdx.x;
      float t = 0.f;
      for (int s2 = 0; s2 < splitk; ++s2)
        t += __hip_atomic_load(bp + (long)s2 * P.M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      P.bias_grad[m0 + threadIdx.x] = t * P.bias_grad_scale;
    }
    epilogue_rows(P, rows, m0 + wm, n0 + wn, lane, args.drop_off);
    return;
  }
  if (splitk > 1) {
    slab_rows(args.ws + args.slab_off[pid] + (long)ks * P.M * P.N, rows, P.M, P.N, m0 + wm, n0 + wn, lane);
    return;
  }
  epilogue_rows(P, rows, m0 + wm, n0 + wn, lane, args.drop_off);
#ifdef SCA_GEMM_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  SCA_STAMP(3);
}

constexpr int TB_BM = 128, TB_BK = 64;
constexpr int TB_OP = TB_BK * TB_BM;  // floats per operand tile (32 KB)


// Instruction interleave for the register-staged kernels' two phases (sched_group_barrier masks:
// 0x008 MFMA, 0x020 VMEM read, 0x100 DS read, 0x200 DS write): the store phase as R rounds of
// {W DS writes, 1 buffer load, M MFMAs} and the read phase as R rounds of {D DS reads, M MFMAs}
// (hipBLASLt's MT128x128x64 fp32 kernel spreads them the same way: a burst of 16 loads or
// writes stalls the issuing wave on the memory queues while the MFMA pipe idles)
template <int I, int R, int W, int M>
__device__ __forceinline__ void ilv_store() {
  if constexpr (I < R) {
    __builtin_amdgcn_sched_group_barrier(0x200, W, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, M, 0);
    ilv_store<I + 1, R, W, M>();
  }
}
template <int I, int R, int D, int M>
__device__ __forceinline__ void ilv_read() {
  if constexpr (I < R) {
    __builtin_amdgcn_sched_group_barrier(0x100, D, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, M, 0);
    ilv_read<I + 1, R, D, M>();
  }
}

__device__ __forceinline__ f32x4 tb_load(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
  return *reinterpret_cast<const f32x4*>(&r);
}

// ------------------------------------------------------------------------------ TN, k-split waves
// Weight-gradient GEMM (TN: dW[M x N] = A^T B over K rows; A = dY [K][M], B = X [K][N], both
// k-major, the LDS-DMA ring of gemm_glds_kernel) with 16x16x4 MFMAs in an outer-product form:
// a lane's float4 of A (4 consecutive m at one k) and of B (4 consecutive n) feed 16 MFMAs,
// MFMA (i, j) taking A's component i and B's component j, i.e. the tile rows m = 4a + i and
// columns n = 4b + j (a, b = the lane's index within 16).  Every wave accumulates the FULL
// 64x64 tile over its quarter of each K slice — one ds_read_b128 per operand per 16 MFMAs,
// where the 32x32x2 form reads 4 ds_read_b32 per fragment — and the 4 waves' partial tiles
// are summed in fixed order through LDS.  A lane ends with tile rows 16g .. 16g+15 x columns
// 4c .. 4c+3 (g = lane >> 4, c = lane & 15).  Epilogue, split-K slabs and in-launch combine
// as gemm_glds_kernel (same 32x32 quadrant row layout after the reduction).
constexpr int TNK_PLD = 68;  // partial-tile row stride (floats): 16-B shift per row
// 2 partial tiles + 4 bias partial rows: the waves' tiles are summed in two rounds (waves 2, 3
// hand theirs to waves 0, 1, which then publish the pair sums), so the reduction fits in the
// 48-KB ring and three workgroups share a CU (the one-round form took 70 KB: two per CU)
constexpr int TNK_RED = 2 * 64 * TNK_PLD * 4 + 4 * 64 * 4;

// SUB: K slices per ring stage (one wait + barrier per SUB x 32 k rows).  REG: the operand
// stream of gemm_tnb_kernel instead of the LDS-DMA ring — 64 k rows per iteration (wave w
// takes rows 16w .. 16w+15), the next iteration's pieces register-staged (4 + 4 float4 per
// thread), loads / stores / fragment reads interleaved with the MFMAs; one segment, K % 64 == 0
template <int S, int SUB, bool REG = false>
__global__ __launch_bounds__(256) void gemm_tnk_kernel(const GemmArgs args) {
  constexpr int SLICE = 2 * GL_OP_BYTES;
  constexpr int STAGE = SUB * SLICE;
  constexpr int SMEM = S * STAGE > TNK_RED ? S * STAGE : TNK_RED;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned nwg = gx * gy * gridDim.z;
  const unsigned orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int splitk = args.splitk;
  int bx, by, pid, ks;
  long cnt_idx;  // the tile's split-K counter
  if (args.flat) {
    int p = 0;
    while (p + 1 < args.nprob && (int)wgid >= args.tile_beg[p + 1]) ++p;
    const int tn = (args.p[p].N + GL_BN - 1) / GL_BN, tm = (args.p[p].M + GL_BM - 1) / GL_BM;
    int local = (int)wgid - args.tile_beg[p];
    bx = local % tn;
    local /= tn;
    by = local % tm;
    ks = local / tm;
    pid = p;
    cnt_idx = args.tile_beg[p] / splitk + (long)by * tn + bx;
  } else {
    bx = wgid % gx;
    by = (wgid / gx) % gy;
    const int bz = wgid / (gx * gy);
    pid = bz / splitk;
    ks = bz % splitk;
    cnt_idx = (long)pid * gx * gy + (long)by * gx + bx;
  }
  const sca_gemm_problem& P = args.p[pid];
  const int m0 = by * GL_BM, n0 = bx * GL_BN;
  if (m0 >= P.M || n0 >= P.N) return;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;

  int seg_kbeg[SCA_GEMM_MAX_SEGS], seg_n[SCA_GEMM_MAX_SEGS];
  int total = 0;
#pragma unroll
  for (int s = 0; s < SCA_GEMM_MAX_SEGS; ++s) {
    seg_kbeg[s] = seg_n[s] = 0;
    if (s < P.nseg) {
      int kbeg = 0, kend = P.seg[s].K;
      if (splitk > 1) {
        const int chunk = ((P.seg[s].K + splitk - 1) / splitk + GL_BK - 1) / GL_BK * GL_BK;
        kbeg = ks * chunk;
        kend = min(P.seg[s].K, kbeg + chunk);
      }
      seg_kbeg[s] = kbeg;
      seg_n[s] = kend > kbeg ? (kend - kbeg) / GL_BK : 0;
      total += seg_n[s];
    }
  }
  int iseg = -1, tseg0 = 0, tend = 0;
  const float* pa[2] = {nullptr, nullptr};
  const float* pb[2] = {nullptr, nullptr};
  long stepA = 0, stepB = 0;
  auto dma = [&](int t, int stage) {
    while (t >= tend) {
      ++iseg;
      tseg0 = tend;
      tend += seg_n[iseg];
      const sca_gemm_seg& G = P.seg[iseg];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        pa[q] = gl_src<false>(G.A, G.lda, m0, P.M, seg_kbeg[iseg], q, wave, lane);
        pb[q] = gl_src<false>(G.B, G.ldb, n0, P.N, seg_kbeg[iseg], q, wave, lane);
      }
      stepA = (long)GL_BK * G.lda;
      stepB = (long)GL_BK * G.ldb;
    }
    const long kk = t - tseg0;
    char* base = smem + stage * STAGE + (t % SUB) * SLICE;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      gl_dma(pa[q] + kk * stepA, base + gl_dst<false>(q, wave));
      gl_dma(pb[q] + kk * stepB, base + GL_OP_BYTES + gl_dst<false>(q, wave));
    }
  };
  const int nst = (total + SUB - 1) / SUB;  // ring stages to walk
  auto dma_stage = [&](int u, int stage) {
#pragma unroll
    for (int q = 0; q < SUB; ++q)
      if (u * SUB + q < total) dma(u * SUB + q, stage);
  };

  const bool do_bias = P.bias_grad != nullptr && bx == 0;
  f32x4 bs4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (REG) {
    const sca_gemm_seg& G = P.seg[0];
    const int K = G.K;
    const int chunk = ((K + splitk - 1) / splitk + TB_BK - 1) / TB_BK * TB_BK;
    const int kbeg = min(K, ks * chunk), kend = min(K, kbeg + chunk);
    const int nit = (kend - kbeg) / TB_BK;
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G.A), 0, (int)(((long)(K - 1) * G.lda + P.M) * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rb =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G.B), 0, (int)(((long)(K - 1) * G.ldb + P.N) * 4), 0x00020000);
    // thread's pieces j < 4: k row (tid >> 4) + 16j of the iteration, columns 4 (tid & 15) .. +3
    const int tid = threadIdx.x, srow = tid >> 4, scol = 4 * (tid & 15);
    const int va = (int)(((long)(kbeg + srow) * G.lda + min(m0 + scol, P.M - 4)) * 4);
    const int vb = (int)(((long)(kbeg + srow) * G.ldb + min(n0 + scol, P.N - 4)) * 4);
    const int rowA = 16 * G.lda * 4, rowB = 16 * G.ldb * 4, itA = TB_BK * G.lda * 4, itB = TB_BK * G.ldb * 4;
    float* As = reinterpret_cast<float*>(smem);  // [64 k][64 m], then [64 k][64 n]
    float* Bs = As + TB_BK * GL_BM;
    f32x4 st[8];
    auto load = [&](int it) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        st[j] = tb_load(ra, va, it * itA + j * rowA);
        st[4 + j] = tb_load(rb, vb, it * itB + j * rowB);
      }
    };
    auto store = [&]() {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        st4(As + (srow + 16 * j) * GL_BM + scol, st[j]);
        st4(Bs + (srow + 16 * j) * GL_BN + scol, st[4 + j]);
      }
    };
    auto iter = [&](auto wr_c, auto ld_c, int it) {
      constexpr bool WR = decltype(wr_c)::value, LD = decltype(ld_c)::value;
      f32x4 a[4], b[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int k = 16 * wave + 4 * n + g;
        a[n] = ld4(As + k * GL_BM + 4 * c);
        b[n] = ld4(Bs + k * GL_BN + 4 * c);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[0][i], b[0][j], acc[i][j]);
      ilv_read<0, 2, 4, 8>();
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (WR) {
        store();
        if constexpr (LD) load(it + 2);
      }
#pragma unroll
      for (int n = 1; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[n][i], b[n][j], acc[i][j]);
      if constexpr (WR) ilv_store<0, 8, 1, 6>();
      if (do_bias) {
#pragma unroll
        for (int n = 0; n < 4; ++n) bs4 += a[n];
      }
      __syncthreads();
    };
    if (nit > 0) {
      load(0);
      store();
      if (nit > 1) load(1);
      __syncthreads();
    }
    int it = 0;
#pragma unroll 1
    for (; it + 2 < nit; ++it) iter(std::true_type{}, std::true_type{}, it);
    if (it + 1 < nit) iter(std::true_type{}, std::false_type{}, it++);
    if (it < nit) iter(std::false_type{}, std::false_type{}, it);
  } else {
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < nst) dma_stage(i, i);
  // stage u landed: the younger in-flight stages hold 4 SUB pieces each, except a partial
  // last stage (then wait for everything)
  const bool whole = total % SUB == 0;
  for (int u = 0; u < nst; ++u) {
    if (u + S - 2 < nst && (whole || u + S - 2 < nst - 1)) gl_wait_vm<4 * SUB * (S - 2)>();
    else gl_wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (u + S - 1 < nst) dma_stage(u + S - 1, (u + S - 1) % S);
#pragma unroll
    for (int q = 0; q < SUB; ++q) {
      if (u * SUB + q >= total) break;
      const float* As = reinterpret_cast<const float*>(smem + (u % S) * STAGE + q * SLICE);
      const float* Bs = As + GL_BM * GL_BK;
      f32x4 a[2], b[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = 4 * (2 * wave + h) + g;  // image row: this wave's k quarter of the slice
        a[h] = ld4(As + k * GL_BM + 4 * c);
        b[h] = ld4(Bs + k * GL_BN + 4 * c);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (do_bias) bs4 += a[h];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[h][i], b[h][j], acc[i][j]);
      }
    }
  }
  }  // REG

  // the 4 waves' partial tiles (and bias rows) through LDS, summed in a fixed order:
  // (wave 0 + wave 2) + (wave 1 + wave 3), in two rounds over two tile slots
  __syncthreads();  // the ring is free
  float* red = reinterpret_cast<float*>(smem);
  float* bred = red + 2 * 64 * TNK_PLD;
  if (do_bias) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bs4[q] += __shfl_xor(bs4[q], 16, 64);
      bs4[q] += __shfl_xor(bs4[q], 32, 64);
    }
    if (g == 0) st4(bred + wave * 64 + 4 * c, bs4);
  }
  float* slot = red + (wave & 1) * 64 * TNK_PLD;
  if (wave >= 2) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        st4(slot + (16 * g + 4 * r + i) * TNK_PLD + 4 * c, f32x4{acc[i][0][r], acc[i][1][r], acc[i][2][r], acc[i][3][r]});
  }
  __syncthreads();
  if (wave < 2) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 t = ld4(slot + (16 * g + 4 * r + i) * TNK_PLD + 4 * c);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j][r] += t[j];
      }
  }
  __syncthreads();  // the partner tiles are consumed
  if (wave < 2) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        st4(slot + (16 * g + 4 * r + i) * TNK_PLD + 4 * c, f32x4{acc[i][0][r], acc[i][1][r], acc[i][2][r], acc[i][3][r]});
  }
  __syncthreads();
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const float alpha = P.seg[0].alpha;
  f32x4 rows[4];
#pragma unroll
  for (int i4 = 0; i4 < 4; ++i4) {
    const int e = (wm + (lane >> 3) + 8 * i4) * TNK_PLD + wn + 4 * (lane & 7);
    rows[i4] = ld4(red + e) + ld4(red + 64 * TNK_PLD + e);
    if (alpha != 1.f) rows[i4] *= alpha;
  }
  const bool fused_k = splitk > 1 && args.counters != nullptr;
  if (do_bias && threadIdx.x < GL_BM && m0 + (int)threadIdx.x < P.M) {
    const int br = threadIdx.x;
    const float bsum = ((bred[br] + bred[64 + br]) + bred[128 + br]) + bred[192 + br];
    float* bp = args.ws + args.bias_off[pid] + (long)ks * P.M + m0 + br;
    if (fused_k)
      __hip_atomic_store(bp, bsum * alpha, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1 store
    else if (splitk > 1)
      *bp = bsum * alpha;
    else
      P.bias_grad[m0 + br] = bsum * alpha * P.bias_grad_scale;
  }
  if (fused_k) {
    const long MN = (long)P.M * P.N;
    float* slabs = args.ws + args.slab_off[pid];
    slab_rows_sc1(slabs, (long)splitk * MN, rows, P.M, P.N, m0 + wm, n0 + wn, lane, (long)ks * MN);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    unsigned* flag = reinterpret_cast<unsigned*>(smem);  // the partial tiles are consumed
    unsigned* cnt = args.counters + cnt_idx;
    if (threadIdx.x == 0)
      *flag = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(splitk - 1);
    __syncthreads();
    if (!*flag) return;
    if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slabs, 0, (int)(splitk * MN * 4), 0x00020000);
    const int n = n0 + wn + 4 * (lane & 7);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = min(m0 + wm + (lane >> 3) + 8 * i, P.M - 1);
      const long e = (long)m * P.N + min(n, P.N - 4);
      f32x4 tt = ld4_sc1(rs, e);
      for (int s2 = 1; s2 < splitk; ++s2) tt += ld4_sc1(rs, s2 * MN + e);
      rows[i] = tt;
    }
    if (do_bias && threadIdx.x < GL_BM && m0 + (int)threadIdx.x < P.M) {
      float* bp = args.ws + args.bias_off[pid] + m0 + threadIdx.x;
      float tt = 0.f;
      for (int s2 = 0; s2 < splitk; ++s2)
        tt += __hip_atomic_load(bp + (long)s2 * P.M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      P.bias_grad[m0 + threadIdx.x] = tt * P.bias_grad_scale;
    }
    epilogue_rows(P, rows, m0 + wm, n0 + wn, lane, args.drop_off);
    return;
  }
  if (splitk > 1) {
    slab_rows(args.ws + args.slab_off[pid] + (long)ks * P.M * P.N, rows, P.M, P.N, m0 + wm, n0 + wn, lane);
    return;
  }
  epilogue_rows(P, rows, m0 + wm, n0 + wn, lane, args.drop_off);
}

// ------------------------------------------------------------------------------ TN, 128x128 tiles
// Weight-gradient GEMM (dW[M x N] = A^T B, A = dY [K][M], B = X [K][N], both k-major) on
// 128x128 tiles, 4 waves of 64x64, 64 k rows per iteration, one workgroup per CU.  The operand
// stream is register-staged: each thread holds the NEXT iteration's 16 float4 pieces (issued
// one iteration ahead with bounds-checked buffer loads), and the single 64-KB LDS tile is read
// whole into registers at the top of an iteration (32 ds_read_b128 per lane: 16 k-steps x A, B),
// so the staged pieces can be written over it while the iteration's 256 MFMAs run from
// registers.  Per lane and k-step one float4 of A (4 consecutive m) and one of B (4 consecutive
// n) feed 16 MFMAs in the outer-product form of gemm_tnk_kernel; a lane ends with rows
// wm + 16g + 4r + i (g = lane >> 4; r, i < 4) x columns wn + 4c .. 4c+3 (c = lane & 15), stored
// as float4 row pieces straight from the accumulators.  Split-K: slabs + in-launch combine
// (gemm_glds_kernel's protocol) or the separate reduction.  Requires K % 64 == 0 per problem.
// epilogue_rows' per-piece body: one float4 of row m at columns n .. n+3
__device__ __forceinline__ void epilogue_piece(const sca_gemm_problem& P, f32x4 v, int m, int n,
                                               const DropMask& dm) {
  f32x4 ex = {0.f, 0.f, 0.f, 0.f}, ax = ex;
  if (P.resid) ex += ld4(P.resid + (long)m * P.ldr + n);
  if (P.epi & SCA_EPI_ACCUM) ex += ld4(P.C + (long)m * P.ldc + n);
  if (P.epi & SCA_EPI_DGELU) ax = ld4(P.aux + (long)m * P.ldx + n);
  const f32x4 bias = P.bias ? ld4(P.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 o = (v + bias) * P.post_scale;
  if (P.epi & SCA_EPI_GELU) {
    st4(P.aux_out + (long)m * P.ldo + n, o);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = gelu_erf(o[j]);
  }
  if (P.epi & SCA_EPI_DROPOUT) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = dm.apply((uint32_t)m * (uint32_t)P.N + (uint32_t)(n + j), o[j]);
  }
  if (P.epi & SCA_EPI_DGELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] *= gelu_erf_grad(ax[j]);
  }
  st4(P.C + (long)m * P.ldc + n, o + ex);
}


// INTER: the MFMAs of k-steps NPRE .. 15 pinned after the staged-piece stores (they cover the
// store / load phase at one workgroup per CU, those of 0 .. NPRE-1 the fragment reads); else
// the compiler's order (every MFMA between the fragment reads, ~216 registers: two workgroups
// per CU cover each other's phases)
template <bool INTER, int NPRE, bool ILV = false>
__global__ __launch_bounds__(256, 1) void gemm_tnb_kernel(const GemmArgs args) {
  __shared__ __attribute__((aligned(16))) float lds[2 * TB_OP];
  __shared__ unsigned flag;

  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned nwg = gx * gy * gridDim.z;
  const unsigned orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int bx = wgid % gx, by = (wgid / gx) % gy, bz = wgid / (gx * gy);

  const int splitk = args.splitk;
  const int pid = bz / splitk, ks = bz % splitk;
  const sca_gemm_problem& P = args.p[pid];
  const int m0 = by * TB_BM, n0 = bx * TB_BM;
  if (m0 >= P.M || n0 >= P.N) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const sca_gemm_seg& G = P.seg[0];
  const int K = G.K;
  const int chunk = ((K + splitk - 1) / splitk + TB_BK - 1) / TB_BK * TB_BK;
  const int kbeg = min(K, ks * chunk), kend = min(K, kbeg + chunk);
  const int nit = (kend - kbeg) / TB_BK;

  // bounds-checked operand resources: a read past the operand's last element returns 0
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G.A), 0, (int)(((long)(K - 1) * G.lda + P.M) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G.B), 0, (int)(((long)(K - 1) * G.ldb + P.N) * 4), 0x00020000);
  // thread's staged pieces j < 8: k row (tid >> 5) + 8j of the iteration, columns 4 (tid & 31) ..
  const int srow = tid >> 5, scol = 4 * (tid & 31);
  const int va = (int)(((long)(kbeg + srow) * G.lda + min(m0 + scol, P.M - 4)) * 4);
  const int vb = (int)(((long)(kbeg + srow) * G.ldb + min(n0 + scol, P.N - 4)) * 4);
  const int rowA = 8 * G.lda * 4, rowB = 8 * G.ldb * 4;       // bytes between a thread's pieces
  const int itA = TB_BK * G.lda * 4, itB = TB_BK * G.ldb * 4;  // bytes per iteration
  f32x4 st[16];
  auto load = [&](int it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      st[j] = tb_load(ra, va, it * itA + j * rowA);
      st[8 + j] = tb_load(rb, vb, it * itB + j * rowB);
    }
  };
  float* wbase = lds + srow * TB_BM + scol;
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      st4(wbase + j * 8 * TB_BM, st[j]);
      st4(wbase + TB_OP + j * 8 * TB_BM, st[8 + j]);
    }
  };

  const bool do_bias = P.bias_grad != nullptr && bx == 0 && wn == 0;
  f32x4 bs4 = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const float* ra_lds = lds + g * TB_BM + wm + 4 * c;
  const float* rb_lds = lds + TB_OP + g * TB_BM + wn + 4 * c;
  // one iteration: the whole LDS tile into registers, barrier, the staged pieces over it (and
  // the loads of two iterations ahead), the 256 MFMAs, barrier
  auto iter = [&](auto wr_c, auto ld_c, int it) {
    constexpr bool WR = decltype(wr_c)::value, LD = decltype(ld_c)::value;
    f32x4 a[16], b[16];
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      a[n] = ld4(ra_lds + n * 4 * TB_BM);
      b[n] = ld4(rb_lds + n * 4 * TB_BM);
    }
#pragma unroll
    for (int n = 0; n < NPRE; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[n][i], b[n][j], acc[i][j]);
    if constexpr (ILV) ilv_read<0, 8, 4, 2 * NPRE>();
    if constexpr (INTER) __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    if constexpr (INTER) __builtin_amdgcn_sched_barrier(0);
    if constexpr (WR) {
      store();
      if constexpr (LD) load(it + 2);
    }
#pragma unroll
    for (int n = NPRE; n < 16; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[n][i], b[n][j], acc[i][j]);
    if constexpr (ILV && WR) ilv_store<0, 16, 1, (16 - NPRE)>();
    if (do_bias) {
#pragma unroll
      for (int n = 0; n < 16; ++n) bs4 += a[n];
    }
    __syncthreads();
  };
  if (nit > 0) {
    load(0);
    store();
    if (nit > 1) load(1);
    __syncthreads();
  }
  int it = 0;
#pragma unroll 1
  for (; it + 2 < nit; ++it) iter(std::true_type{}, std::true_type{}, it);
  if (it + 1 < nit) iter(std::true_type{}, std::false_type{}, it++);
  if (it < nit) iter(std::false_type{}, std::false_type{}, it);

  const float alpha = G.alpha;
  const bool fused_k = splitk > 1 && args.counters != nullptr;
  // bias partial: rows wm + 4c + i summed over the 4 k-lane groups (waves with wn == 0)
  if (do_bias) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bs4[q] += __shfl_xor(bs4[q], 16, 64);
      bs4[q] += __shfl_xor(bs4[q], 32, 64);
    }
    if (g == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm + 4 * c + i;
        if (m >= P.M) continue;
        float* bp = args.ws + args.bias_off[pid] + (long)ks * P.M + m;
        if (fused_k)
          __hip_atomic_store(bp, bs4[i] * alpha, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1 store
        else if (splitk > 1)
          *bp = bs4[i] * alpha;
        else
          P.bias_grad[m] = bs4[i] * alpha * P.bias_grad_scale;
      }
    }
  }
  const int n = n0 + wn + 4 * c;
  const bool ncol = n < P.N;
  if (splitk > 1) {
    const long MN = (long)P.M * P.N;
    float* slabs = args.ws + args.slab_off[pid];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slabs, 0, (int)(splitk * MN * 4), 0x00020000);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm + 16 * g + 4 * r + i;
        if (m < P.M && ncol) {
          const f32x4 x = f32x4{acc[i][0][r], acc[i][1][r], acc[i][2][r], acc[i][3][r]} * alpha;
          const int off = (int)(((long)ks * MN + (long)m * P.N + n) * 4);
          if (fused_k) __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(&x), rs, off, 0, 16);
          else __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(&x), rs, off, 0, 0);
        }
      }
    if (!fused_k) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    unsigned* cnt = args.counters + (long)pid * gx * gy + (long)by * gx + bx;
    if (tid == 0)
      flag = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(splitk - 1);
    __syncthreads();
    if (!flag) return;
    if (tid == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // sc1-stored, sc1-loaded: no agent acquire
    if (P.bias_grad && bx == 0 && tid < TB_BM && m0 + tid < P.M) {
      float* bp = args.ws + args.bias_off[pid] + m0 + tid;
      float t = 0.f;
      for (int s2 = 0; s2 < splitk; ++s2)
        t += __hip_atomic_load(bp + (long)s2 * P.M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      P.bias_grad[m0 + tid] = t * P.bias_grad_scale;
    }
    if (!ncol) return;
    DropMask dm;
    if (P.epi & SCA_EPI_DROPOUT) dm.init(P.drop_seed, P.drop_p, args.drop_off);
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      const int m = m0 + wm + 16 * g + q;
      if (m >= P.M) continue;
      const long e = (long)m * P.N + n;
      f32x4 t = ld4_sc1(rs, e);
      for (int s2 = 1; s2 < splitk; ++s2) t += ld4_sc1(rs, s2 * MN + e);
      epilogue_piece(P, t, m, n, dm);
    }
    return;
  }
  if (!ncol) return;
  DropMask dm;
  if (P.epi & SCA_EPI_DROPOUT) dm.init(P.drop_seed, P.drop_p, args.drop_off);
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm + 16 * g + 4 * r + i;
      if (m < P.M)
        epilogue_piece(P, f32x4{acc[i][0][r], acc[i][1][r], acc[i][2][r], acc[i][3][r]} * alpha, m, n, dm);
    }
}

// ------------------------------------------------------------------------------ NT / NN, 128x128 tiles
// C[M x N] = sum over segments of A[M][K] B^T (NT: B [N][K]) or A B (NN: B [K][N]) (+ the
// epilogue) on 128x128 tiles, gemm_tnb_kernel's pipeline with A k-contiguous: the staged A
// pieces are float4 runs along k, stored to LDS as a [row][k] image with a 68-float row stride
// (rows 16 B apart in the bank space: the 16-lane ds_read_b128 groups below are conflict-free),
// and the fragments are the plain 16x16x4 ones — a lane's float4 at (row i, k 16kc + 4kg .. +3)
// is its A (or B) operand of four consecutive k-steps.  NT's B is staged like A; NN's B pieces
// (4 consecutive n at one k; a wave's 64 lanes cover 16 k x 4 pieces) are transposed into the
// same [n][k] image by four ds_write_b32 each (64 distinct banks per instruction).  Segments
// (dX = dQ Wq + dK Wk + dV Wv) are walked back to back.  The accumulators go through LDS
// (per-wave 64 x 68 image) into float4 row pieces for epilogue_piece.  No split-K; every
// segment's K % 64 == 0.
constexpr int NB_LD = TB_BK + 4;               // 68
constexpr int NB_OP = TB_BM * NB_LD;           // floats per operand image

template <bool INTER, int NPRE, bool B_KN, bool ILV = false, int TM = 128>
__global__ __launch_bounds__(256, 1) void gemm_ntb_kernel(const GemmArgs args) {
  constexpr int WT = TM / 2, NQ = WT / 16, NJ = TM / 16;  // wave tile, its 16-blocks, pieces / operand
  constexpr int OP = TM * NB_LD;                            // floats per operand image
  __shared__ __attribute__((aligned(16))) float lds[2 * OP];
  if constexpr (B_KN && SCA_CRIT_PRIO > 0) __builtin_amdgcn_s_setprio(SCA_CRIT_PRIO);  // as gemm_glds_kernel<NN>

  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned nwg = gx * gy * gridDim.z;
  const unsigned orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int bx = wgid % gx, by = (wgid / gx) % gy, pid = wgid / (gx * gy);
  const sca_gemm_problem& P = args.p[pid];
  const int m0 = by * TM, n0 = bx * TM;
  if (m0 >= P.M || n0 >= P.N) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kg = lane >> 4, li = lane & 15;
  const int wm = (wave >> 1) * WT, wn = (wave & 1) * WT;
  const int nseg = P.nseg;
  const int it0 = P.seg[0].K / TB_BK, it1 = nseg > 1 ? P.seg[1].K / TB_BK : 0;
  const int nit = it0 + it1 + (nseg > 2 ? P.seg[2].K / TB_BK : 0);

  // thread's staged pieces j < NJ: A (and NT's B) row (tid >> 4) + 16j, k 4 (tid & 15) .. +3 of
  // the iteration; NN's B: k 16 (b & 3) + (lane & 15), columns 4 (4 (b >> 2) + (lane >> 4)) ..
  // +3 with b = NJ wave + j.  Rows / columns past the end re-read the last ones (never stored).
  const int srow = tid >> 4, sk4 = 4 * (tid & 15);
  f32x4 st[2 * NJ];
  auto load = [&](int it) {
    int s = 0, lit = it;  // segment and its local iteration (wave-uniform)
    if (lit >= it0) {
      lit -= it0;
      s = 1;
      if (lit >= it1) {
        lit -= it1;
        s = 2;
      }
    }
    const sca_gemm_seg& G = P.seg[s];
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(G.A), 0, (int)(((long)(P.M - 1) * G.lda + G.K) * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(G.B), 0,
        (int)((B_KN ? (long)(G.K - 1) * G.ldb + P.N : (long)(P.N - 1) * G.ldb + G.K) * 4), 0x00020000);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      st[j] = tb_load(ra, (int)(((long)min(m0 + srow + 16 * j, P.M - 1) * G.lda + sk4) * 4), lit * TB_BK * 4);
      if constexpr (B_KN) {
        const int b = NJ * wave + j;
        const int k = 16 * (b & 3) + li, c4 = 4 * (4 * (b >> 2) + kg);
        st[NJ + j] = tb_load(rb, (int)(((long)k * G.ldb + min(n0 + c4, P.N - 4)) * 4), lit * TB_BK * G.ldb * 4);
      } else {
        st[NJ + j] = tb_load(rb, (int)(((long)min(n0 + srow + 16 * j, P.N - 1) * G.ldb + sk4) * 4), lit * TB_BK * 4);
      }
    }
  };
  float* wbase = lds + srow * NB_LD + sk4;
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      st4(wbase + j * 16 * NB_LD, st[j]);
      if constexpr (B_KN) {
        const int b = NJ * wave + j;
        const int k = 16 * (b & 3) + li, c4 = 4 * (4 * (b >> 2) + kg);
#pragma unroll
        for (int q = 0; q < 4; ++q) lds[OP + (c4 + q) * NB_LD + k] = st[NJ + j][q];
      } else {
        st4(wbase + OP + j * 16 * NB_LD, st[NJ + j]);
      }
    }
  };

  f32x4 acc[NQ][NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i)
#pragma unroll
    for (int j = 0; j < NQ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const float* ra_lds = lds + (wm + li) * NB_LD + 4 * kg;
  const float* rb_lds = lds + OP + (wn + li) * NB_LD + 4 * kg;
  auto iter = [&](auto wr_c, auto ld_c, int it) {
    constexpr bool WR = decltype(wr_c)::value, LD = decltype(ld_c)::value;
    f32x4 a[4][NQ], b[4][NQ];  // [kc][block]
#pragma unroll
    for (int kc = 0; kc < 4; ++kc)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        a[kc][q] = ld4(ra_lds + 16 * q * NB_LD + 16 * kc);
        b[kc][q] = ld4(rb_lds + 16 * q * NB_LD + 16 * kc);
      }
    auto steps = [&](int t0, int t1) {
#pragma unroll
      for (int t = t0; t < t1; ++t)
#pragma unroll
        for (int i = 0; i < NQ; ++i)
#pragma unroll
          for (int j = 0; j < NQ; ++j) acc[i][j] = mfma16(a[t >> 2][i][t & 3], b[t >> 2][j][t & 3], acc[i][j]);
    };
    steps(0, NPRE);
    if constexpr (ILV) ilv_read<0, 8, NQ, NPRE * NQ * NQ / 8>();
    if constexpr (INTER) __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    if constexpr (INTER) __builtin_amdgcn_sched_barrier(0);
    if constexpr (WR) {
      store();
      if constexpr (LD) load(it + 2);
    }
    steps(NPRE, 16);
    if constexpr (ILV && WR) ilv_store<0, 2 * NJ, B_KN ? 3 : 1, (16 - NPRE) * NQ * NQ / (2 * NJ)>();
    __syncthreads();
  };
  load(0);
  store();
  if (nit > 1) load(1);
  __syncthreads();
  int it = 0;
#pragma unroll 1
  for (; it + 2 < nit; ++it) iter(std::true_type{}, std::true_type{}, it);
  if (it + 1 < nit) iter(std::true_type{}, std::false_type{}, it++);
  if (it < nit) iter(std::false_type{}, std::false_type{}, it);

  // accumulators -> this wave's WT x 68 image -> float4 row pieces (LR lanes per row: rows
  // lane / LR + (64 / LR) q, columns 4 (lane % LR))
  constexpr int LR = WT / 4;
  float* img = lds + wave * WT * NB_LD;
  const float alpha = P.seg[0].alpha;
#pragma unroll
  for (int i = 0; i < NQ; ++i)
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) img[(16 * i + 4 * kg + r) * NB_LD + 16 * j + li] = acc[i][j][r] * alpha;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int n = n0 + wn + 4 * (lane % LR);
  if (n >= P.N) return;
  DropMask dm;
  if (P.epi & SCA_EPI_DROPOUT) dm.init(P.drop_seed, P.drop_p, args.drop_off);
#pragma unroll 4
  for (int q = 0; q < WT * LR / 64; ++q) {
    const int rho = lane / LR + (64 / LR) * q, m = m0 + wm + rho;
    if (m < P.M) epilogue_piece(P, ld4(img + rho * NB_LD + 4 * (lane % LR)), m, n, dm);
  }
}

// ------------------------------------------------------------------------------ row-tile main loop
// The main loop of the LayerNorm-fused GEMMs (32 full rows x 256 columns, 512 threads, wave w
// owning columns 32w .. 32w+31 as 2 x 2 16x16 blocks) in the register-staged, interleaved form
// of gemm_ntb_kernel: per 64-k iteration one A piece and eight B pieces per thread, the
// A [32][68] and B [256][68] (k-contiguous, NN's B transposed on the store) images read whole
// into registers, loads / stores issued between the MFMAs.  Segments back to back; every
// segment's K % 64 == 0.  acc[i][j]: rows 16i + 4(lane >> 4) + r, columns 32w + 16j + (lane & 15).
constexpr int LR_SMEM = (32 + 256) * 68 * 4;  // 78 KB
template <bool B_KN>
__device__ __forceinline__ void ln_rows_reg(const sca_gemm_problem& P, int m0, float* lds, f32x4 (&acc)[2][2]) {
  constexpr int LD = 68, NPRE = 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kg = lane >> 4, li = lane & 15;
  float* Ai = lds;
  float* Bi = lds + 32 * LD;
  const int nseg = P.nseg;
  const int it0 = P.seg[0].K / 64, it1 = nseg > 1 ? P.seg[1].K / 64 : 0;
  const int nit = it0 + it1 + (nseg > 2 ? P.seg[2].K / 64 : 0);
  const int arow = tid >> 4, ak4 = 4 * (tid & 15);
  f32x4 st[9];
  auto load = [&](int it) {
    int sg = 0, lit = it;
    if (lit >= it0) {
      lit -= it0;
      sg = 1;
      if (lit >= it1) {
        lit -= it1;
        sg = 2;
      }
    }
    const sca_gemm_seg& G = P.seg[sg];
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(G.A), 0, (int)(((long)(P.M - 1) * G.lda + G.K) * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(G.B), 0,
        (int)((B_KN ? (long)(G.K - 1) * G.ldb + P.N : (long)(P.N - 1) * G.ldb + G.K) * 4), 0x00020000);
    st[0] = tb_load(ra, (int)(((long)min(m0 + arow, P.M - 1) * G.lda + ak4) * 4), lit * 256);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (B_KN) {
        const int b = 8 * wave + j, k = 16 * (b & 3) + li, c4 = 4 * (4 * (b >> 2) + kg);
        st[1 + j] = tb_load(rb, (k * G.ldb + c4) * 4, lit * 64 * G.ldb * 4);
      } else {
        st[1 + j] = tb_load(rb, ((arow + 32 * j) * G.ldb + ak4) * 4, lit * 256);
      }
    }
  };
  auto store = [&]() {
    st4(Ai + arow * LD + ak4, st[0]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (B_KN) {
        const int b = 8 * wave + j, k = 16 * (b & 3) + li, c4 = 4 * (4 * (b >> 2) + kg);
#pragma unroll
        for (int q = 0; q < 4; ++q) Bi[(c4 + q) * LD + k] = st[1 + j][q];
      } else {
        st4(Bi + (arow + 32 * j) * LD + ak4, st[1 + j]);
      }
    }
  };
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* ra_lds = Ai + li * LD + 4 * kg;
  const float* rb_lds = Bi + (32 * wave + li) * LD + 4 * kg;
  auto iter = [&](auto wr_c, auto ld_c, int it) {
    constexpr bool WR = decltype(wr_c)::value, LDN = decltype(ld_c)::value;
    f32x4 a[4][2], b[4][2];
#pragma unroll
    for (int kc = 0; kc < 4; ++kc)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        a[kc][q] = ld4(ra_lds + 16 * q * LD + 16 * kc);
        b[kc][q] = ld4(rb_lds + 16 * q * LD + 16 * kc);
      }
    auto steps = [&](int t0, int t1) {
#pragma unroll
      for (int t = t0; t < t1; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(a[t >> 2][i][t & 3], b[t >> 2][j][t & 3], acc[i][j]);
    };
    steps(0, NPRE);
    ilv_read<0, 4, 4, NPRE>();
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (WR) {
      store();
      if constexpr (LDN) load(it + 2);
    }
    steps(NPRE, 16);
    if constexpr (WR) ilv_store<0, 9, B_KN ? 4 : 1, 5>();
    __syncthreads();
  };
  if (nit > 0) {
    load(0);
    store();
    if (nit > 1) load(1);
    __syncthreads();
  }
  int it = 0;
#pragma unroll 1
  for (; it + 2 < nit; ++it) iter(std::true_type{}, std::true_type{}, it);
  if (it + 1 < nit) iter(std::true_type{}, std::false_type{}, it++);
  if (it < nit) iter(std::false_type{}, std::false_type{}, it);
}

// the row-tile main loop's requirements: every segment's K % 64 == 0, 32-bit operand offsets
bool ln_reg_ok(const sca_gemm_problem& P, bool b_kn) {
  const long lim = (1L << 31) - 1;
  for (int s = 0; s < P.nseg; ++s) {
    const sca_gemm_seg& G = P.seg[s];
    if (G.K % 64 || G.K == 0) return false;
    if (((long)P.M * G.lda + G.K) * 4 > lim) return false;
    if ((b_kn ? (long)G.K * G.ldb + P.N : (long)P.N * G.ldb + G.K) * 4 > lim) return false;
  }
  return true;
}

// SCA_LNREG=0 keeps the LayerNorm-fused GEMMs on their LDS-DMA main loops (A/B), read once
bool ln_reg_default() {
  static const bool on = !(getenv("SCA_LNREG") && atoi(getenv("SCA_LNREG")) == 0);
  return on;
}
// SCA_LNB_R3=1: the chained input-gradient passes on a 3-stage B ring (147.5 KB of LDS; opt-in:
// -0.17 % in the config 2 step, 3 alternated reps — the passes are not bound by the slice
// latency, and the larger footprint keeps the side stream's kernels off those CUs)
bool lnb_r3_default() {
  static const bool on = getenv("SCA_LNB_R3") && atoi(getenv("SCA_LNB_R3")) == 1;
  return on;
}

// ------------------------------------------------------------------------------ GEMM + LayerNorm
// NT GEMM whose epilogue completes the post-LN block (keypoint_module.py:63-72, 99-109):
// v = resid + dropout((A B^T + bias) * post_scale), y = LayerNorm(v) * gamma + beta, for
// d_model = N = 256 — a workgroup owns 32 FULL rows (32x256 tile), so the row statistics
// never leave the workgroup and the separate LayerNorm launch (plus its re-read of v)
// disappears.  Main loop: the LDS-DMA ring of gemm_glds_kernel (3 stages of A [32][32] +
// B [256][32], XOR-swizzled 128-B rows); wave w computes columns 64w .. 64w+63 (two
// 32x32 accumulators).  Epilogue: the 32x256 tile goes through LDS, then each wave
// normalises 8 rows with float4 lanes and wave reductions (two-pass mean / variance as
// ln_fwd_kernel).  Writes v (the LayerNorm input, kept for its backward), y, mean, rstd.
constexpr int LG_BN = 256, GL_A32 = 32, GL_A16 = 16;
constexpr int LG_B_BYTES = LG_BN * GL_BK * 4;  // 32 KiB
constexpr int LG_VS = LG_BN + 8;               // row stride of the epilogue tile (bank spread)

// tile variants: 32 rows (3-stage ring, 32x32x2 MFMAs, 1 workgroup / CU) or 16 rows
// (2-stage ring, 16x16x4 MFMAs, 68 KB LDS: 2 workgroups / CU, twice the workgroups)
template <int BM>
struct LgCfg {
  static constexpr int S = BM == 32 ? 3 : 2;
  static constexpr int A_BYTES = BM * GL_BK * 4;
  static constexpr int STAGE = A_BYTES + LG_B_BYTES;
  static constexpr int A_PIECES = BM / 8;  // 1-KiB DMA pieces of the A tile
  // 32 rows: 8 waves (two per SIMD: one workgroup fills a CU's LDS), a 32x32 column block
  // each; 16 rows: 4 waves, 64 columns each
  static constexpr int NW = BM == 32 ? 8 : 4;
  static constexpr int BPW = 32 / NW;      // B pieces (8 rows of 32 k) per wave per slice
};

// chained passes (CH): LDS map after the main loop — [0, 64 KB) a 2-stage B ring (a pass's
// [256][32] k-slice, the main loop's swizzled image), then the y tile (rows of 256 + 4
// floats: the A operand of every pass), then 8 wave-private 5-KB transposition scratches
constexpr int LG_A2_LD = 260;
constexpr int LG_A2_OFF = 2 * LG_B_BYTES;
constexpr int LG_SCR_OFF = LG_A2_OFF + 32 * LG_A2_LD * 4;
constexpr int LG_CH_SMEM = LG_SCR_OFF + 8 * 32 * EPI_LD * 4;
// register-staged chained passes (REG): the pass's B image [256][68] first, then the y tile,
// then the scratches (140.5 KB)
constexpr int LR_A2_OFF = 256 * 68 * 4;
constexpr int LR_SCR_OFF = LR_A2_OFF + 32 * LG_A2_LD * 4;
constexpr int LR_CH_SMEM = LR_SCR_OFF + 8 * 32 * EPI_LD * 4;

struct GemmLnArgs {
  sca_gemm_problem p[SCA_GEMM_LN_MAX_PROBLEMS];
  sca_gemm_ln_problem ln[SCA_GEMM_LN_MAX_PROBLEMS];
  float eps;
  const unsigned long long* drop_off;
  int rot;  // chained passes in a per-row-tile rotated order (SCA_GEMM_LN_ROT, default 1)
};

// per-lane source of DMA piece `pc` (rows 8pc .. 8pc+7 of a k-contiguous [rows][32] tile)
__device__ __forceinline__ const float* lg_src(const float* base, int ld, int row0, int nrows, int pc, int lane) {
  const int r = 8 * pc + (lane >> 3);
  const int ks = (lane & 7) ^ gl_swz(r);
  return base + (long)min(row0 + r, nrows - 1) * ld + 4 * ks;
}

// float4 of the k-contiguous swizzled image: row r, 16-B slot `slot` (4 consecutive k)
__device__ __forceinline__ f32x4 lg_slot(const char* img, int r, int slot) {
  return *(const f32x4*)(img + r * 128 + 16 * (slot ^ gl_swz(r)));
}

// one chained pass's epilogue on float4 row pieces: (acc + bias) * post_scale, GELU (keeps
// the pre-activation) — epilogue_rows' order
__device__ __forceinline__ f32x4 chain_bias(const sca_gemm_chain_pass& Q, int nb, int lane) {
  return Q.bias ? ld4(Q.bias + nb + 4 * (lane & 7)) : f32x4{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ void chain_rows(const sca_gemm_chain_pass& Q, const f32x4 (&v)[4], int mb, int M, int nb,
                                           int lane, f32x4 bias) {
  const int n = nb + 4 * (lane & 7);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mb + (lane >> 3) + 8 * i;
    if (m >= M) continue;
    f32x4 o = (v[i] + bias) * Q.post_scale;
    if (Q.epi & SCA_EPI_GELU) {
      st4g(Q.aux_out + (long)m * Q.ldo + n, o);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = gelu_erf(o[j]);
    }
    st4g(Q.C + (long)m * Q.ldc + n, o);
  }
}

// NC = 2: d_model = 512 as two 256-column halves of one continuous slice sequence (the A
// tile is re-read from L2 once; two accumulators per wave), one 32 x 512 epilogue tile and
// LayerNorm over the full row; no chained passes.
template <int BM, bool CH, int NC, bool REG = false>
__global__ __launch_bounds__(LgCfg<BM>::NW * 64) void gemm_ln_kernel(const GemmLnArgs args) {
  using CF = LgCfg<BM>;
  constexpr int S = CF::S;
  constexpr int VS = NC * LG_BN + 8;  // row stride of the epilogue tile
  constexpr int NROW = NC * LG_BN;
  static_assert(!CH || (BM == 32 && LG_CH_SMEM >= S * CF::STAGE && 32 * LG_VS * 4 <= LG_A2_OFF), "LDS map");
  static_assert(NC == 1 || (NC == 2 && BM == 32 && !CH && 32 * VS * 4 <= S * CF::STAGE), "LDS map (NC = 2)");
  static_assert(!REG || (BM == 32 && NC == 1 && LR_SMEM <= S * CF::STAGE), "LDS map (REG)");
  static_assert(!(REG && CH) || (32 * LG_VS * 4 <= LR_A2_OFF && LR_CH_SMEM <= 160 * 1024), "LDS map (REG, chained)");
  constexpr int A2OFF = REG ? LR_A2_OFF : LG_A2_OFF, SCROFF = REG ? LR_SCR_OFF : LG_SCR_OFF;
  __shared__ __attribute__((aligned(1024))) char smem[CH ? (REG ? LR_CH_SMEM : LG_CH_SMEM) : S * CF::STAGE];
  const unsigned gx = gridDim.x;
  const unsigned nwg = gx * gridDim.z;
  const unsigned orig = blockIdx.x + gx * blockIdx.z;
  const unsigned xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int pid = wgid / gx, bx = wgid % gx;
  const sca_gemm_problem& P = args.p[pid];
  const sca_gemm_ln_problem& LN = args.ln[pid];
  const int m0 = bx * BM;
  if (m0 >= P.M) return;
#ifdef SCA_GEMM_STAMPS
  // diagnostic build: entry, main loop done, LayerNorm done, first chained pass done, end
  const unsigned stamp_id = wgid;
#define SCA_LN_STAMP(slot) \
  if (threadIdx.x == 0 && stamp_id < STAMP_MAX) g_stamps[stamp_id][slot] = __builtin_amdgcn_s_memrealtime()
#else
#define SCA_LN_STAMP(slot) \
  do {                     \
  } while (0)
#endif
  SCA_LN_STAMP(0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const sca_gemm_seg& G = P.seg[0];
  const int total = G.K / GL_BK;
  const int ttot = NC * total;  // slices of all column halves

  // DMA sources: A pieces spread over the first waves, B pieces 8*wave .. 8*wave+7 (the
  // swizzle of row r is (r >> 1) & 7: pieces 2u and 2u + 1 differ in it, pieces 16 rows
  // apart do not — one source pointer per parity, stepped by 16 rows)
  const bool has_a = wave < CF::A_PIECES;
  const float* pa = lg_src(G.A, G.lda, m0, P.M, has_a ? wave : 0, lane);
  constexpr int BPW = CF::BPW;
  const float* pb[2] = {lg_src(G.B, G.ldb, 0, P.N, BPW * wave, lane),
                        lg_src(G.B, G.ldb, 0, P.N, BPW * wave + 1, lane)};
  const long pstep = 16L * G.ldb;
  auto dma = [&](int t, int stage) {
    char* base = smem + stage * CF::STAGE;
    const int half = NC == 2 && t >= total ? 1 : 0;
    const long kk = (long)(t - half * total) * GL_BK;
    const long hoff = (long)half * LG_BN * G.ldb;  // B rows of the second column half
    if (has_a) gl_dma(pa + kk, base + wave * GL_PIECE);
#pragma unroll
    for (int c = 0; c < BPW; ++c)
      gl_dma(pb[c & 1] + (c >> 1) * pstep + hoff + kk, base + CF::A_BYTES + (BPW * wave + c) * GL_PIECE);
  };

  // the epilogue's residual rows are loaded before the main loop (their HBM reads overlap
  // it); no residual: a harmless read of gamma, unused — keeps the loads branch-free
  constexpr int RPW = BM / CF::NW;
  const int n = 4 * lane;
  f32x4 rin[RPW][NC];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int m = min(m0 + RPW * wave + i, P.M - 1);
#pragma unroll
    for (int c = 0; c < NC; ++c) rin[i][c] = ld4((P.resid ? P.resid + (long)m * P.ldr : LN.gamma) + LG_BN * c + n);
  }
  // ... and the LayerNorm's affine / the bias (complete by the end of the main loop, where a
  // wait says so to the waitcnt pass: loaded after it, they were waited for behind the
  // chained passes' first two slices — vmcnt(0) on 64 KB per workgroup, ~3 us)
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4 bias4[NC], gam[NC], bet[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    bias4[c] = P.bias ? ld4(P.bias + LG_BN * c + n) : zero;
    gam[c] = ld4(LN.gamma + LG_BN * c + n);
    bet[c] = ld4(LN.beta + LG_BN * c + n);
  }
  float* V = reinterpret_cast<float*>(smem);
  const float alpha = G.alpha;
  if constexpr (REG) {
    f32x4 acc[2][2];
    ln_rows_reg<false>(P, m0, V, acc);
    SCA_LN_STAMP(1);
    const int li = lane & 15, kg = lane >> 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) V[(16 * i + 4 * kg + r) * VS + 32 * wave + 16 * j + li] = acc[i][j][r] * alpha;
  } else if constexpr (BM == 32) {
    f32x16 acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
#pragma unroll
    for (int i = 0; i < S - 1; ++i)
      if (i < ttot) dma(i, i);
    auto slice = [&](int t, f32x16& ac) {
      if (t + S - 2 < ttot) {
        if (has_a) gl_wait_vm<(BPW + 1) * (S - 2)>();
        else gl_wait_vm<BPW * (S - 2)>();
      } else {
        gl_wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + S - 1 < ttot) dma(t + S - 1, (t + S - 1) % S);
      const char* As = smem + (t % S) * CF::STAGE;
      const char* Bs = As + CF::A_BYTES;
      f32x4 fa[4], fb[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        fa[g] = gl_frag<true>(As, 0, g, lane);
        fb[g] = gl_frag<true>(Bs, 32 * wave, g, lane);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) ac = mfma32(fa[g][j], fb[g][j], ac);
    };
    for (int t = 0; t < total; ++t) slice(t, acc[0]);
    if constexpr (NC == 2)
      for (int t = total; t < ttot; ++t) slice(t, acc[1]);
    // 32 x 256 NC tile -> LDS (the ring is free once every wave has passed its last slice)
    __syncthreads();
    SCA_LN_STAMP(1);
    const int col = lane & 31, rowh = 4 * (lane >> 5);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        V[((r & 3) + 8 * (r >> 2) + rowh) * VS + LG_BN * c + 32 * wave + col] = acc[c][r] * alpha;
  } else {
    // 16 rows: wave w owns columns 64w .. 64w+63 as four 16x16 accumulators; per 16-k group
    // c a lane reads 4 consecutive k of its A row and of each B row (one float4 each)
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int li = lane & 15, grp = lane >> 4;
    if (total > 0) dma(0, 0);
    for (int t = 0; t < total; ++t) {
      gl_wait_vm<0>();               // slice t landed for this wave
      __builtin_amdgcn_s_barrier();  // ... for every wave; slice t-1's stage no longer read
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < total) dma(t + 1, (t + 1) % S);
      const char* As = smem + (t % S) * CF::STAGE;
      const char* Bs = As + CF::A_BYTES;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const f32x4 af = lg_slot(As, li, 4 * c + grp);
        f32x4 bf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = lg_slot(Bs, 64 * wave + 16 * j + li, 4 * c + grp);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = mfma16(af[r], bf[j][r], acc[j]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) V[(4 * grp + r) * VS + 64 * wave + 16 * j + li] = acc[j][r] * alpha;
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): every load of this wave so far has landed

  // each wave normalises BM/NW rows at once: every row is 64 lanes x float4 (coalesced), and
  // the rows' reductions are interleaved (independent shuffle chains, one latency each)
  DropMask dm;
  const bool drop = (P.epi & SCA_EPI_DROPOUT) != 0;
  if (drop) dm.init(P.drop_seed, P.drop_p, args.drop_off);
  const float invN = 1.0f / NROW;
  f32x4 v[RPW][NC];
  float s[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int lr = RPW * wave + i, m = min(m0 + lr, P.M - 1);
    s[i] = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      f32x4 x = (ld4(&V[lr * VS + LG_BN * c + n]) + bias4[c]) * P.post_scale;
      if (drop) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          x[j] = dm.apply((uint32_t)m * (uint32_t)P.N + (uint32_t)(LG_BN * c + n + j), x[j]);
      }
      if (P.resid) x += rin[i][c];
      v[i][c] = x;
      s[i] += (x[0] + x[1]) + (x[2] + x[3]);
    }
  }
  // REG chained passes: iteration u = 64 k rows of pass pass_of(u >> 2); thread's pieces j < 8:
  // B rows (tid >> 4) + 32j, k 4 (tid & 15) .. +3 — the first one loaded under the LayerNorm
  const int nit2 = CH && REG ? 4 * LN.npass : 0;
  f32x4 st2[8];
  auto load2 = [&](int u) {
    int q = (u >> 2) + (args.rot && LN.npass > 0 ? bx % LN.npass : 0);
    q = q >= LN.npass ? q - LN.npass : q;
    const sca_gemm_chain_pass& Q = LN.pass[q];
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(Q.B), 0, (int)(((long)(LG_BN - 1) * Q.ldb + LG_BN) * 4), 0x00020000);
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      st2[j] = tb_load(rb, (((t >> 4) + 32 * j) * Q.ldb + 4 * (t & 15)) * 4, (u & 3) * 256);
  };
  auto store2 = [&]() {
    float* Bi = reinterpret_cast<float*>(smem);
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < 8; ++j) st4(Bi + ((t >> 4) + 32 * j) * 68 + 4 * (t & 15), st2[j]);
  };
  if constexpr (CH && REG) {
    if (nit2 > 0) load2(0);
  }
  // chained passes: a slice of B (row r of the [256][32] image at r * 128 B, pieces 4w .. 4w+3
  // by wave w) — the first two stream in under the LayerNorm math, into the V tile's region
  // once every wave has read its rows of it
  const int nsl = CH && !REG ? 8 * LN.npass : 0;
  // every workgroup streams the same weights in near lock-step; row tile bx runs the passes
  // from pass bx % npass on, so that neighbouring tiles stream different weight matrices at
  // a time (each pass's own K order is unchanged: bit-identical results; +0.5 % in step,
  // 2 alternations, 1602 -> 1609-1611 clips/s)
  const int prot = CH && args.rot && LN.npass > 0 ? bx % LN.npass : 0;
  auto pass_of = [&](int u) {
    int q = (u >> 3) + prot;
    return q >= LN.npass ? q - LN.npass : q;
  };
  auto dma2 = [&](int u, int stage) {
    const sca_gemm_chain_pass& Q = LN.pass[pass_of(u)];
    char* base = smem + stage * LG_B_BYTES;
    const long k0 = 32L * (u & 7);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      gl_dma(lg_src(Q.B, Q.ldb, 0, LG_BN, 4 * wave + c, lane) + k0, base + (4 * wave + c) * GL_PIECE);
  };
  if constexpr (CH) {
    __syncthreads();
    if constexpr (REG) {
      if (nit2 > 0) store2();
      if (nit2 > 1) load2(1);
    } else {
      if (nsl > 0) dma2(0, 0);
      if (nsl > 1) dma2(1, 1);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int i = 0; i < RPW; ++i) s[i] += __shfl_xor(s[i], o, 64);
  float q[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    q[i] = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const f32x4 dv = v[i][c] - s[i] * invN;
      q[i] += (dv[0] * dv[0] + dv[1] * dv[1]) + (dv[2] * dv[2] + dv[3] * dv[3]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int i = 0; i < RPW; ++i) q[i] += __shfl_xor(q[i], o, 64);
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int lr = RPW * wave + i, m = m0 + lr;
    const float mean = s[i] * invN;
    const float rstd = 1.0f / sqrtf(q[i] * invN + args.eps);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const f32x4 y = (v[i][c] - mean) * rstd * gam[c] + bet[c];
      if (CH) st4(reinterpret_cast<float*>(smem + A2OFF) + lr * LG_A2_LD + n, y);  // rows past M: finite
      if (m < P.M) {
        st4g(P.C + (long)m * P.ldc + LG_BN * c + n, v[i][c]);
        st4g(LN.y + (long)m * NROW + LG_BN * c + n, y);
      }
    }
    if (m < P.M) {
      if (lane == 0) {
        st1g(LN.mean + m, mean);
        st1g(LN.rstd + m, rstd);
      }
    }
  }
  if constexpr (CH && REG) {
    // chained NT GEMMs, register-staged: out_p[32 x 256] = y_tile B_p^T, A fragments from the
    // y image, B through the [256][68] image (ln_rows_reg's arrangement), 4 iterations a pass
    const float* A2 = reinterpret_cast<const float*>(smem + A2OFF);
    const float* Bi = reinterpret_cast<const float*>(smem);
    float* scratch = reinterpret_cast<float*>(smem + SCROFF) + wave * 32 * EPI_LD;
    const int li = lane & 15, kg = lane >> 4;
    const int prot2 = args.rot && LN.npass > 0 ? bx % LN.npass : 0;
    f32x4 acc2[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    lds_barrier();  // the y rows and pass 0's first B tile are in LDS
    SCA_LN_STAMP(2);
    f32x4 cbias = f32x4{0.f, 0.f, 0.f, 0.f};  // the current pass's bias, loaded at its start
    auto iter2 = [&](auto wr_c, auto ld_c, int u) {
      constexpr bool WR = decltype(wr_c)::value, LDN = decltype(ld_c)::value;
      if ((u & 3) == 0) {
        int pq0 = (u >> 2) + prot2;
        pq0 = pq0 >= LN.npass ? pq0 - LN.npass : pq0;
        cbias = chain_bias(LN.pass[pq0], 32 * wave, lane);
      }
      f32x4 a[4][2], b[4][2];
#pragma unroll
      for (int kc = 0; kc < 4; ++kc)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          a[kc][q] = ld4(A2 + (16 * q + li) * LG_A2_LD + 64 * (u & 3) + 16 * kc + 4 * kg);
          b[kc][q] = ld4(Bi + (32 * wave + 16 * q + li) * 68 + 16 * kc + 4 * kg);
        }
      auto steps = [&](int t0, int t1) {
#pragma unroll
        for (int t = t0; t < t1; ++t)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc2[i][j] = mfma16(a[t >> 2][i][t & 3], b[t >> 2][j][t & 3], acc2[i][j]);
      };
      steps(0, 4);
      ilv_read<0, 4, 4, 4>();
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();  // every wave has read the B image
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (WR) {
        store2();
        if constexpr (LDN) load2(u + 2);
      }
      steps(4, 16);
      if constexpr (WR) ilv_store<0, 8, 1, 6>();
      if ((u & 3) == 3) {  // the pass's 32 x 256 block: this wave's 32 x 32 through its scratch
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) scratch[(16 * i + 4 * kg + r) * EPI_LD + 16 * j + li] = acc2[i][j][r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        f32x4 rows[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) rows[q] = ld4(scratch + ((lane >> 3) + 8 * q) * EPI_LD + 4 * (lane & 7));
        int pq = (u >> 2) + prot2;
        pq = pq >= LN.npass ? pq - LN.npass : pq;
        chain_rows(LN.pass[pq], rows, m0, P.M, 32 * wave, lane, cbias);
        if (u == 3) SCA_LN_STAMP(3);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // scratch reads done before the next pass
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      __syncthreads();  // the next B tile is in LDS
    };
    int u = 0;
#pragma unroll 1
    for (; u + 2 < nit2; ++u) iter2(std::true_type{}, std::true_type{}, u);
    if (u + 1 < nit2) iter2(std::true_type{}, std::false_type{}, u++);
    if (u < nit2) iter2(std::false_type{}, std::false_type{}, u);
  }
  if constexpr (CH && !REG) {
    // chained NT GEMMs: out_p[32 x 256] = y_tile[32 x 256] B_p^T — A from the LDS image
    // (published by the barrier below), B through the 2-stage ring one slice ahead;
    // the passes are one continuous slice sequence (the next pass's first slice streams in
    // under the current pass's last one)
    const float* A2 = reinterpret_cast<const float*>(smem + LG_A2_OFF);
    float* scratch = reinterpret_cast<float*>(smem + LG_SCR_OFF) + wave * 32 * EPI_LD;
    const int col = lane & 31, h = lane >> 5;
    f32x16 acc2;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[r] = 0.f;
    lds_barrier();  // every wave's y rows written to the image (its global stores stay in flight)
    SCA_LN_STAMP(2);
    // the waits for a slice's DMA let this wave's epilogue stores stay in flight (vmcnt counts
    // stores too, in issue order): at u = 0 the 16 LayerNorm stores (v, y, mean, rstd of 4
    // rows) and slice 1's 4 pieces are younger than slice 0; after a pass's epilogue its 4
    // (8 with GELU) row-piece stores are younger than the next slice.  Exact for full tiles
    // (every row < M); a partial tile waits for everything.
    const bool full = m0 + BM <= P.M;
    for (int u = 0; u < nsl; ++u) {
      if (!full) {
        gl_wait_vm<0>();
      } else if (u == 0) {
        if (nsl > 1) gl_wait_vm<20>();
        else gl_wait_vm<16>();
      } else if ((u & 7) == 0) {
        if (LN.pass[pass_of(u - 1)].epi & SCA_EPI_GELU) gl_wait_vm<8>();
        else gl_wait_vm<4>();
      } else {
        gl_wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (u >= 1 && u + 1 < nsl) dma2(u + 1, (u + 1) & 1);  // into the stage slice u-1 left
      const int t = u & 7;
      const char* Bs = smem + (u & 1) * LG_B_BYTES;
      f32x4 fa[4], fb[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        fa[g] = ld4(A2 + col * LG_A2_LD + 32 * t + 8 * g + 4 * h);
        fb[g] = gl_frag<true>(Bs, 32 * wave, g, lane);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc2 = mfma32(fa[g][j], fb[g][j], acc2);
      if (t == 7) {
        f32x4 rows[4];
        acc_to_rows(acc2, scratch, lane, rows);
        chain_rows(LN.pass[pass_of(u)], rows, m0, P.M, 32 * wave, lane, chain_bias(LN.pass[pass_of(u)], 32 * wave, lane));
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[r] = 0.f;
        if (u == 7) SCA_LN_STAMP(3);
      }
    }
  }
#ifdef SCA_GEMM_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  SCA_LN_STAMP(4);
#undef SCA_LN_STAMP
}

// ------------------------------------------------------------------------------ GEMM + LayerNorm backward
// NN input-gradient GEMM whose epilogue runs the backward of the LayerNorm below it (the
// post-LN block boundary, keypoint_module.py:69-72 / 105-109, walked backwards): a workgroup
// owns 32 FULL rows (32 x 256), so C = dL/dy is complete in the workgroup and the row
// reductions of the LayerNorm backward never leave it; the separate ln_bwd launch and its
// re-read of dL/dy disappear.  Main loop: the LDS-DMA ring of gemm_ln_kernel with a k-major
// B image (one 1-KiB DMA piece per k-row, rows 1056 B apart so the two half-waves of a
// fragment read, 4 k-rows apart, land on different banks); segments (dq Wq + dk Wk + dv Wv)
// are one continuous slice sequence.  Epilogue: the tile goes through LDS; each wave takes 4
// rows (float4 lanes, interleaved shuffle reductions); dgamma / dbeta partials are summed
// over the 32 rows in fixed order (waves through LDS) into one partial row per block.
// 8 waves (512 threads, two per SIMD, each a 32x32 column block): with one workgroup per CU
// (113 KB of LDS) a second wave per SIMD hides the DMA waits and the barrier; 4 waves of
// 32x64 ran 45 us per 4 x (2048 x 256 x 768) launch.
constexpr int LB_BM = 32, LB_S = 3;
constexpr int LB_BROW = 1056;                        // bytes per k-row of the B image
constexpr int LB_A_BYTES = LB_BM * GL_BK * 4;        // 4 KiB
constexpr int LB_STAGE = LB_A_BYTES + GL_BK * LB_BROW;
// epilogue / chained-GEMM LDS map: [0, 2 B-rows stages) the V tile, then phase 2's B ring
// (2 stages); then phase 2's A image (the dx tile, rows of 256 + 4 floats); then the
// dgamma / dbeta wave partials
constexpr int LB_B2 = GL_BK * LB_BROW;                // one phase-2 B stage (33 KB)
constexpr int LB_A2_LD = 260;                         // floats per row of the dx tile image
constexpr int LB_A2_OFF = 2 * LB_B2;
constexpr int LB_RED_OFF = LB_A2_OFF + LB_BM * LB_A2_LD * 4;
constexpr int LB_SMEM = LB_RED_OFF + 2 * 8 * 256 * 4 > LB_S * LB_STAGE ? LB_RED_OFF + 2 * 8 * 256 * 4
                                                                         : LB_S * LB_STAGE;
// R3: a third phase-2 B stage after everything else (147.5 KB), so the chained passes' B
// slices stream two slices ahead
constexpr int LB_B3_OFF = LB_SMEM;
constexpr int LB_SMEM3 = LB_B3_OFF + LB_B2;

struct GemmLnbArgs {
  sca_gemm_problem p[SCA_GEMM_MAX_PROBLEMS];
  sca_gemm_lnb_problem ln[SCA_GEMM_MAX_PROBLEMS];
};

// NC = 2: d_model = 512 as two 256-column halves (one continuous slice sequence, two
// accumulators per wave), a 32 x 512 epilogue tile, no chained GEMM.
template <int NC, bool REG = false, bool R3 = false>
__global__ __launch_bounds__(512) void gemm_lnb_kernel(const GemmLnbArgs args) {
  if constexpr (SCA_CRIT_PRIO > 0) __builtin_amdgcn_s_setprio(SCA_CRIT_PRIO);
  static_assert(!R3 || (NC == 1 && LB_SMEM3 <= 160 * 1024), "LDS map (R3)");
  __shared__ __attribute__((aligned(1024))) char smem[R3 ? LB_SMEM3 : LB_SMEM];
  constexpr int VS = NC * LG_BN + 8, NROW = NC * LG_BN;
  constexpr int RED_OFF = NC == 1 ? LB_RED_OFF : LB_BM * VS * 4;  // dgamma / dbeta wave partials
  static_assert(LB_B2 >= LB_BM * LG_VS * 4 && LB_RED_OFF + 2 * 8 * LG_BN * 4 <= LB_SMEM, "LDS map");
  static_assert(NC == 1 || RED_OFF + 2 * 8 * NROW * 4 <= LB_SMEM, "LDS map (NC = 2)");
  static_assert(!REG || (NC == 1 && LR_SMEM <= LB_SMEM), "LDS map (REG)");
  const unsigned gx = gridDim.x;
  const unsigned nwg = gx * gridDim.z;
  const unsigned orig = blockIdx.x + gx * blockIdx.z;
  const unsigned xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const unsigned wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int pid = wgid / gx, bx = wgid % gx;
  const sca_gemm_problem& P = args.p[pid];
  const sca_gemm_lnb_problem& LN = args.ln[pid];
  const int m0 = bx * LB_BM;
  if (m0 >= P.M) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;  // 8 waves: 2 per SIMD
  const bool has_a = wave < 4;                                  // waves 0-3 also fetch an A piece

  int seg_n[SCA_GEMM_MAX_SEGS];
  int total = 0;
#pragma unroll
  for (int s = 0; s < SCA_GEMM_MAX_SEGS; ++s) {
    seg_n[s] = s < P.nseg ? P.seg[s].K / GL_BK : 0;
    total += seg_n[s];
  }
  const int ttot = NC * total;  // slices of all column halves
  // issue state: A piece `wave` (rows 8*wave ..) and B pieces = k-rows 4*wave .. 4*wave+3
  int iseg = -1, tseg0 = 0, tend = 0;
  const float* pa = nullptr;
  const float* pb = nullptr;
  long ldb = 0;
  auto dma = [&](int t, int stage) {
    const int half = NC == 2 && t >= total ? 1 : 0;
    if (NC == 2 && t == total) {  // second column half: the segments again
      iseg = -1;
      tend = 0;
    }
    t -= half * total;
    while (t >= tend) {
      ++iseg;
      tseg0 = tend;
      tend += seg_n[iseg];
      const sca_gemm_seg& G = P.seg[iseg];
      pa = lg_src(G.A, G.lda, m0, P.M, has_a ? wave : 0, lane);
      ldb = G.ldb;
      pb = G.B + (long)(4 * wave) * ldb + 4 * lane + LG_BN * half;
    }
    const long k0 = (long)(t - tseg0) * GL_BK;
    char* base = smem + stage * LB_STAGE;
    if (has_a) gl_dma(pa + k0, base + wave * GL_PIECE);
#pragma unroll
    for (int c = 0; c < 4; ++c) gl_dma(pb + (k0 + c) * ldb, base + LB_A_BYTES + (4 * wave + c) * LB_BROW);
  };

  // the epilogue's row operands (this wave's 4 rows of the LayerNorm input, its statistics
  // and the residual gradient) are loaded before the main loop: their HBM reads overlap it
  // instead of forming the HBM-bound tail of every workgroup at once
  constexpr int RPW = LB_BM / 8;
  const int n = 4 * lane;
  f32x4 xin[RPW][NC], rin[RPW][NC], gam[NC];
  float mu[RPW], rs[RPW];
#pragma unroll
  for (int c = 0; c < NC; ++c) gam[c] = ld4(LN.gamma + LG_BN * c + n);  // with the other epilogue operands
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int m = min(m0 + RPW * wave + i, P.M - 1);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int nc = LG_BN * c + n;
      xin[i][c] = ld4(LN.x + (long)m * NROW + nc);
      if (LN.tab) xin[i][c] += ld4(LN.tab + (long)(m % LN.tab_T + 2) * NROW + nc);  // v = x + P[t + 2]
      // (no residual: a harmless read of gamma, unused — keeps the loads branch-free)
      rin[i][c] = ld4((P.resid ? P.resid + (long)m * P.ldr : LN.gamma) + nc);
    }
    mu[i] = LN.mean[m];
    rs[i] = LN.rstd[m];
  }
  f32x16 acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  const int col = lane & 31, h = lane >> 5;
  f32x4 racc[2][2];
  if constexpr (REG) {
    ln_rows_reg<true>(P, m0, reinterpret_cast<float*>(smem), racc);
  } else {
#pragma unroll
  for (int i = 0; i < LB_S - 1; ++i)
    if (i < ttot) dma(i, i);
  auto slice = [&](int t, f32x16& ac) {
    if (t + LB_S - 2 < ttot) {
      if (has_a) gl_wait_vm<5 * (LB_S - 2)>();
      else gl_wait_vm<4 * (LB_S - 2)>();
    } else {
      gl_wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + LB_S - 1 < ttot) dma(t + LB_S - 1, (t + LB_S - 1) % LB_S);
    const char* As = smem + (t % LB_S) * LB_STAGE;
    const float* Bf = reinterpret_cast<const float*>(As + LB_A_BYTES);
    f32x4 fa[4], fb[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      fa[g] = gl_frag<true>(As, 0, g, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[g][j] = Bf[(8 * g + 4 * h + j) * (LB_BROW / 4) + 32 * wave + col];
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) ac = mfma32(fa[g][j], fb[g][j], ac);
  };
  for (int t = 0; t < total; ++t) slice(t, acc[0]);
  if constexpr (NC == 2)
    for (int t = total; t < ttot; ++t) slice(t, acc[1]);
  }
  // 32 x 256 NC tile -> LDS (the ring is free once every wave has passed its last slice)
  __syncthreads();
  float* V = reinterpret_cast<float*>(smem);
  const float alpha = P.seg[0].alpha;
  const int rowh = 4 * h;
  if constexpr (REG) {
    const int li = lane & 15, kg = lane >> 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) V[(16 * i + 4 * kg + r) * VS + 32 * wave + 16 * j + li] = racc[i][j][r] * alpha;
  } else {
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      V[((r & 3) + 8 * (r >> 2) + rowh) * VS + LG_BN * c + 32 * wave + col] = acc[c][r] * alpha;
  }
  __syncthreads();

  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the epilogue operands have landed (see gemm_ln_kernel)
  const float invN = 1.0f / NROW;
  f32x4 g[RPW][NC], xh[RPW][NC];
  float s1[RPW], s2[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    s1[i] = s2[i] = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      g[i][c] = ld4(&V[(RPW * wave + i) * VS + LG_BN * c + n]);
      if (P.resid) g[i][c] += rin[i][c];
      xh[i][c] = (xin[i][c] - mu[i]) * rs[i];
      const f32x4 gg = g[i][c] * gam[c];
      s1[i] += (gg[0] + gg[1]) + (gg[2] + gg[3]);
      const f32x4 ggx = gg * xh[i][c];
      s2[i] += (ggx[0] + ggx[1]) + (ggx[2] + ggx[3]);
    }
  }
  // chained GEMM (dout = dx Wo, npass 256-column blocks of Wo): its first two B slices
  // stream in under the LayerNorm math, into the V tile's region once every wave has read
  // its rows of it; the passes are one continuous slice sequence
  const bool chain = NC == 1 && LN.wo != nullptr;
  const int npass = chain ? max(LN.npass, 1) : 0;
  const long ldw = LN.ldw ? LN.ldw : (long)LG_BN * npass;
  const float* pw = LN.wo + (long)(4 * wave) * ldw + 4 * lane;  // B pieces: k-rows 4*wave .. +3
  auto stage_at = [&](int stage) { return smem + (R3 && stage == 2 ? LB_B3_OFF : stage * LB_B2); };
  auto dma2 = [&](int u, int stage) {
    const float* src = pw + (u >> 3) * LG_BN + (long)(32 * (u & 7)) * ldw;
#pragma unroll
    for (int c = 0; c < 4; ++c) gl_dma(src + c * ldw, stage_at(stage) + (4 * wave + c) * LB_BROW);
  };
  if (chain) {
    __syncthreads();
    dma2(0, 0);
    dma2(1, 1);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      s1[i] += __shfl_xor(s1[i], o, 64);
      s2[i] += __shfl_xor(s2[i], o, 64);
    }
  f32x4 pg[NC], pbsum[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) pg[c] = pbsum[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float* A2 = reinterpret_cast<float*>(smem + LB_A2_OFF);
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int lr = RPW * wave + i, m = m0 + lr;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const f32x4 d = (g[i][c] * gam[c] - s1[i] * invN - xh[i][c] * (s2[i] * invN)) * rs[i];
      if (chain) st4(A2 + lr * LB_A2_LD + n, d);  // rows past M: finite, their products never stored
      if (m < P.M) {
        st4g(P.C + (long)m * P.ldc + LG_BN * c + n, g[i][c]);
        st4g(LN.dx + (long)m * NROW + LG_BN * c + n, d);
        pg[c] += g[i][c] * xh[i][c];
        pbsum[c] += g[i][c];
      }
    }
  }
  // the 8 waves' partial rows, summed in fixed order: dgamma, then dbeta (a thread per
  // column, NC columns per thread)
  float* red = reinterpret_cast<float*>(smem + RED_OFF);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    st4(red + wave * NROW + LG_BN * c + n, pg[c]);
    st4(red + (8 + wave) * NROW + LG_BN * c + n, pbsum[c]);
  }
  lds_barrier();  // the partial rows are in LDS (the row stores above stay in flight)
  const long nblk = (P.M + LB_BM - 1) / LB_BM;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int e = threadIdx.x + 512 * c;  // (which, column) of 2 x NROW sums
    const int cc = e % NROW, which = e / NROW;
    const float* rr = red + which * 8 * NROW + cc;
    const float sum = (((rr[0] + rr[NROW]) + (rr[2 * NROW] + rr[3 * NROW])) +
                       ((rr[4 * NROW] + rr[5 * NROW]) + (rr[6 * NROW] + rr[7 * NROW])));
    st1g(LN.partial + (which * nblk + bx) * NROW + cc, sum);
  }
  if (!chain) return;

  // chained GEMM: dout[32 x 256 npass] = dx_tile[32 x 256] Wo[256 x 256 npass]; A from the
  // LDS image (written above, published by the barrier), B through a 2-stage ring, one
  // slice ahead.  Passes before the last store straight from the accumulator (element form:
  // the ring is busy with the next pass); the last one in row form after the loop.
  const bool dgelu = LN.aux != nullptr;
  f32x16 acc2;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc2[r] = 0.f;
  const int nsl = 8 * npass;
  // as in gemm_ln_kernel: this wave's epilogue stores stay in flight across the slice waits —
  // at u = 0 the 8 row stores (g, dx of 4 rows), the partial-row store and slice 1's 4 pieces
  // are younger than slice 0; after a pass's element-form stores (16) the next slice is older
  // than them.  Exact for full tiles; a partial tile waits for everything.
  const bool full = m0 + LB_BM <= P.M;
  // GELU' operands of a pass (the forward's pre-activations): loaded at the pass's second
  // slice, behind its third slice's DMA pieces, so their latency is not the pass's tail —
  // element form (16 per lane) for the passes before the last, row form (4 float4) for it
  const long n2 = (long)(npass - 1) * LG_BN + 32 * wave + 4 * (lane & 7);
  float axe[16];
  f32x4 axr[4];
  for (int u = 0; u < nsl; ++u) {
    const bool last_pass = (u >> 3) == npass - 1;
    if constexpr (R3) {
      // slice u was issued two slices back; younger: slice u+1's pieces (4), the GELU'
      // operands issued behind slice u's or slice u+1's pieces (16 / 4 in the last pass), and
      // the element-form stores of a pass that ended in between (16); the LayerNorm
      // epilogue's 9 stores are younger than slices 0 and 1
      const int t = u & 7;
      if (!full || u == nsl - 1) gl_wait_vm<0>();
      else if (u < 2) gl_wait_vm<13>();
      else if (t < 2) gl_wait_vm<20>();
      else if (t < 4 && dgelu && !last_pass) gl_wait_vm<20>();
      else if (t < 4 && dgelu) gl_wait_vm<8>();
      else gl_wait_vm<4>();
    } else if (!full) {
      gl_wait_vm<0>();
    } else if (dgelu && (u & 7) == 2) {
      if (last_pass) gl_wait_vm<4>();  // the operands stay in flight
      else gl_wait_vm<16>();
    } else if (u == 0) {
      if (nsl > 1) gl_wait_vm<13>();
      else gl_wait_vm<9>();
    } else if ((u & 7) == 0) {
      gl_wait_vm<16>();
    } else {
      gl_wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (R3) {
      if (u + 2 < nsl) dma2(u + 2, (u + 2) % 3);  // into the stage slice u-1 left
    } else {
      if (u >= 1 && u + 1 < nsl) dma2(u + 1, (u + 1) & 1);  // into the stage slice u-1 left
    }
    const int t = u & 7;
    if (dgelu && t == 1) {
      if (!last_pass) {
        const long cn = (u >> 3) * LG_BN + 32 * wave + col;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          axe[r] = LN.aux[(long)min(m0 + (r & 3) + 8 * (r >> 2) + 4 * h, P.M - 1) * ldw + cn];
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) axr[i] = ld4(LN.aux + (long)min(m0 + (lane >> 3) + 8 * i, P.M - 1) * ldw + n2);
      }
    }
    const float* Bf = reinterpret_cast<const float*>(stage_at(R3 ? u % 3 : u & 1));
    f32x4 fa[4], fb[4];
#pragma unroll
    for (int g2 = 0; g2 < 4; ++g2) {
      fa[g2] = ld4(A2 + col * LB_A2_LD + 32 * t + 8 * g2 + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[g2][j] = Bf[(8 * g2 + 4 * h + j) * (LB_BROW / 4) + 32 * wave + col];
    }
#pragma unroll
    for (int g2 = 0; g2 < 4; ++g2)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc2 = mfma32(fa[g2][j], fb[g2][j], acc2);
    if (t == 7 && u + 1 < nsl) {
      // lane: column 32 wave + col of the pass, rows (r & 3) + 8 (r >> 2) + 4h
      const long cn = (u >> 3) * LG_BN + 32 * wave + col;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m >= P.M) continue;
        float o = acc2[r];
        if (dgelu) o *= gelu_erf_grad(axe[r]);
        st1g(LN.dout + (long)m * ldw + cn, o);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) acc2[r] = 0.f;
    }
  }
  __syncthreads();  // ring free: wave-private transposition scratch (8 x 5 KB) for row stores
  f32x4 rows[4];
  acc_to_rows(acc2, reinterpret_cast<float*>(smem) + wave * 32 * EPI_LD, lane, rows);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + (lane >> 3) + 8 * i;
    if (m >= P.M) continue;
    f32x4 o = rows[i];
    if (dgelu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] *= gelu_erf_grad(axr[i][j]);
    }
    st4(LN.dout + (long)m * ldw + n2, o);
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
      const float* bp = args.ws + args.bias_off[blockIdx.y] + m;
      float v = 0.f;
      for (int s = 0; s < args.splitk; ++s) v += bp[(long)s * P.M];
      P.bias_grad[m] = v * P.bias_grad_scale;
    }
    return;
  }
  const int m = (int)(e / P.N), n = (int)(e % P.N);
  const float* slab = args.ws + args.slab_off[blockIdx.y] + e;
  float v = 0.f;
  for (int s = 0; s < args.splitk; ++s) v += slab[s * MN];
  P.C[(long)m * P.ldc + n] = epilogue(P, m, n, v, args.drop_off);
}

// The same, four consecutive elements per thread (N % 4 == 0): 16-B slab loads and C stores.
// blockIdx.x < nc4: C elements 4e .. 4e+3; beyond: the bias partials (one per thread).
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(const GemmArgs args, int nc4) {
  const sca_gemm_problem& P = args.p[blockIdx.y];
  const long MN = (long)P.M * P.N;
  if ((int)blockIdx.x >= nc4) {
    const long m = (long)(blockIdx.x - nc4) * 256 + threadIdx.x;
    if (P.bias_grad && m < P.M) {
      const float* bp = args.ws + args.bias_off[blockIdx.y] + m;
      float v = 0.f;
      for (int s = 0; s < args.splitk; ++s) v += bp[(long)s * P.M];
      P.bias_grad[m] = v * P.bias_grad_scale;
    }
    return;
  }
  const long e = 4 * ((long)blockIdx.x * 256 + threadIdx.x);
  if (e >= MN) return;
  const int m = (int)(e / P.N), n = (int)(e % P.N);
  const float* slab = args.ws + args.slab_off[blockIdx.y] + e;
  f32x4 v = ld4(slab);
  for (int s = 1; s < args.splitk; ++s) v += ld4(slab + s * MN);
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = epilogue(P, m, n + j, v[j], args.drop_off);
  st4(P.C + (long)m * P.ldc + n, o);
}

template <int LAYOUT, class C, bool VEC = true>
int launch(const GemmArgs& a, int nprob, int maxM, int maxN, hipStream_t st) {
  dim3 grid((maxN + C::BN - 1) / C::BN, (maxM + C::BM - 1) / C::BM, nprob * a.splitk);
  hipLaunchKernelGGL((gemm_kernel<LAYOUT, C, VEC>), grid, dim3(C::NT), 0, st, a);
  return hipGetLastError() == hipSuccess ? SCA_OK : SCA_ERR_LAUNCH;
}

// Kernel variants (index = sca_gemm_tile_override value; every one computes the full result):
//   1  register-staged 64x64, 4 waves (the any-shape fallback: element-wise loads)
//   5  register-staged 64x64, single-buffered (TN fallback when the LDS-DMA kernel cannot take
//      the shapes)
//   7  register-staged 128x64, 8 waves (NN fallback)
//   20 / 21 / 22  LDS-DMA 64x64 with a 3- / 2- / 4-stage ring (the heuristic's kernels)
//   36 / 37  TN only: the k-split outer-product weight-gradient kernel, 3- / 4-stage ring
//   38 / 39 / 40  TN only: 128x128 tiles, register-staged operand stream (gemm_tnb_kernel<INTER, NPRE>)
//   41 / 42  NT / NN: the same with A k-contiguous (gemm_ntb_kernel<INTER, NPRE, B k-major>)
//   43 / 44  TN / NT-NN: variants 40 / 41 with the phases' instructions interleaved (ILV)
//   45  NT / NN: variant 44 on 64x64 tiles (4 waves of 32x32: four times the workgroups)
//   46  TN: the k-split kernel (36) with the register-staged, interleaved operand stream
using T1 = Cfg<64, 64, 2, 2, 32, 2>;    // 4 waves, 32x32 each, double-buffered
using T5 = Cfg<64, 64, 2, 2, 32, 1>;    // single-buffered (more workgroups per CU)
using T7 = Cfg<128, 64, 4, 2, 32, 2>;   // 8 waves, 32x32
constexpr int kTnFirst = 36, kTnLast = 40;

bool valid_tile(int layout, int tile) {
  switch (tile) {
    case 0: case 1: case 5: case 7: case 20: case 21: case 22: return true;
    case 36: case 37: case 38: case 39: case 40: case 43: case 46: return layout == SCA_GEMM_TN;
    case 41: case 42: case 44: case 45: return layout != SCA_GEMM_TN;
    default: return false;
  }
}

// the LDS-DMA kernel's shape requirements (see gemm_glds_kernel)
bool glds_ok(const GemmArgs& a, int nprob) {
  for (int i = 0; i < nprob; ++i) {
    const sca_gemm_problem& P = a.p[i];
    if ((P.M & 3) || (P.N & 3)) return false;
    for (int s = 0; s < P.nseg; ++s)
      if ((P.seg[s].K % GL_BK) || P.seg[s].alpha != P.seg[0].alpha) return false;
  }
  return true;
}

template <int LAYOUT, int S>
int launch_glds(const GemmArgs& a, int nprob, int maxM, int maxN, hipStream_t st) {
  dim3 grid((maxN + GL_BN - 1) / GL_BN, (maxM + GL_BM - 1) / GL_BM, nprob * a.splitk);
  hipLaunchKernelGGL((gemm_glds_kernel<LAYOUT, S>), grid, dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? SCA_OK : SCA_ERR_LAUNCH;
}

// float4 operand loads need K (k-contiguous operands), lda, ldb multiples of 4 and A, B
// 16-byte aligned; otherwise the element-wise (any-shape) form of the register-staged kernel
bool vec_ok(const GemmArgs& a, int nprob, int layout) {
  const bool a_kc = layout != SCA_GEMM_TN, b_kc = layout == SCA_GEMM_NT;
  for (int i = 0; i < nprob; ++i)
    for (int s = 0; s < a.p[i].nseg; ++s) {
      const sca_gemm_seg& S = a.p[i].seg[s];
      if (((a_kc || b_kc) && (S.K & 3)) || (S.lda & 3) || (S.ldb & 3) ||
          (reinterpret_cast<uintptr_t>(S.A) & 15) || (reinterpret_cast<uintptr_t>(S.B) & 15))
        return false;
    }
  return true;
}

template <int S, int SUB, bool REG = false>
int launch_tnk(GemmArgs& a, int nprob, int maxM, int maxN, hipStream_t st) {
  dim3 grid((maxN + GL_BN - 1) / GL_BN, (maxM + GL_BM - 1) / GL_BM, nprob * a.splitk);
  bool same = true;
  for (int i = 1; i < nprob; ++i) same = same && a.p[i].M == a.p[0].M && a.p[i].N == a.p[0].N;
  if (!same) {  // problems of different shapes: a flat grid of every problem's own tiles x splits
    a.flat = 1;
    int t = 0;
    for (int i = 0; i < nprob; ++i) {
      a.tile_beg[i] = t;
      t += ((a.p[i].M + GL_BM - 1) / GL_BM) * ((a.p[i].N + GL_BN - 1) / GL_BN) * a.splitk;
    }
    a.tile_beg[nprob] = t;
    grid = dim3(t, 1, 1);
  }
  hipLaunchKernelGGL((gemm_tnk_kernel<S, SUB, REG>), grid, dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? SCA_OK : SCA_ERR_LAUNCH;
}

bool tn_ok(const GemmArgs& a, int nprob) {
  for (int i = 0; i < nprob; ++i)
    if (a.p[i].nseg != 1) return false;
  return glds_ok(a, nprob);
}

// gemm_tnb_kernel: K a multiple of its 64-row iteration, every byte offset of the operands,
// the slabs included, within the 32-bit range of its buffer resources
bool tnb_ok(const GemmArgs& a, int nprob) {
  if (!tn_ok(a, nprob)) return false;
  const long lim = (1L << 31) - 1;
  for (int i = 0; i < nprob; ++i) {
    const sca_gemm_problem& P = a.p[i];
    const sca_gemm_seg& G = P.seg[0];
    if (G.K % TB_BK || P.M < 4 || P.N < 4) return false;
    if (((long)G.K * G.lda + P.M) * 4 > lim || ((long)G.K * G.ldb + P.N) * 4 > lim) return false;
    if ((long)a.splitk * P.M * P.N * 4 > lim) return false;
  }
  return true;
}

// gemm_ntb_kernel: no split-K, every segment's K a positive multiple of 64 (equal alphas:
// glds_ok), 32-bit operand offsets
bool ntb_ok(const GemmArgs& a, int nprob, bool b_kn) {
  if (a.splitk != 1 || !glds_ok(a, nprob)) return false;
  const long lim = (1L << 31) - 1;
  for (int i = 0; i < nprob; ++i) {
    const sca_gemm_problem& P = a.p[i];
    for (int s = 0; s < P.nseg; ++s) {
      const sca_gemm_seg& G = P.seg[s];
      if (G.K % TB_BK || G.K == 0) return false;
      if (((long)P.M * G.lda + G.K) * 4 > lim) return false;
      if ((b_kn ? (long)G.K * G.ldb + P.N : (long)P.N * G.ldb + G.K) * 4 > lim) return false;
    }
  }
  return true;
}

template <bool INTER, int NPRE, bool B_KN, bool ILV = false, int TM = 128>
int launch_ntb(const GemmArgs& a, int nprob, int maxM, int maxN, hipStream_t st) {
  dim3 grid((maxN + TM - 1) / TM, (maxM + TM - 1) / TM, nprob);
  hipLaunchKernelGGL((gemm_ntb_kernel<INTER, NPRE, B_KN, ILV, TM>), grid, dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? SCA_OK : SCA_ERR_LAUNCH;
}

template <bool INTER, int NPRE, bool ILV = false>
int launch_tnb(const GemmArgs& a, int nprob, int maxM, int maxN, hipStream_t st) {
  dim3 grid((maxN + TB_BM - 1) / TB_BM, (maxM + TB_BM - 1) / TB_BM, nprob * a.splitk);
  hipLaunchKernelGGL((gemm_tnb_kernel<INTER, NPRE, ILV>), grid, dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? SCA_OK : SCA_ERR_LAUNCH;
}

// The kernel a launch of `tile` (a requested variant) runs after the eligibility fallbacks —
// launch_tile dispatches on it and sca_gemm_kernel_name reports it (profiling names).
enum KernelId {
  K_T1_ANY, K_NTB45, K_NTB44, K_NTB41, K_NTB42, K_TNK46, K_TNB43, K_TNB38, K_TNB39, K_TNB40, K_TNK36, K_TNK37,
  K_GLDS3, K_GLDS2, K_GLDS4, K_T5, K_T7, K_T1
};

KernelId resolve_kernel(int layout, int tile, const GemmArgs& a, int nprob) {
  if (!vec_ok(a, nprob, layout)) return K_T1_ANY;
  if (tile == 41 || tile == 42 || tile == 44 || tile == 45) {
    if (layout != SCA_GEMM_TN && ntb_ok(a, nprob, layout == SCA_GEMM_NN))
      return tile == 45 ? K_NTB45 : tile == 44 ? K_NTB44 : tile == 41 ? K_NTB41 : K_NTB42;
    tile = layout == SCA_GEMM_NT ? 20 : 21;
  }
  if (tile == 46) {
    if (layout == SCA_GEMM_TN && tnb_ok(a, nprob)) return K_TNK46;
    tile = 36;
  }
  if ((tile >= 38 && tile <= 40) || tile == 43) {
    if (layout == SCA_GEMM_TN && tnb_ok(a, nprob))
      return tile == 43 ? K_TNB43 : tile == 38 ? K_TNB38 : tile == 39 ? K_TNB39 : K_TNB40;
    tile = 36;
  }
  if (tile >= kTnFirst && tile <= kTnLast) {
    if (layout == SCA_GEMM_TN && tn_ok(a, nprob)) return tile == 36 ? K_TNK36 : K_TNK37;
    tile = 21;
  }
  if (tile >= 20 && !glds_ok(a, nprob)) tile = layout == SCA_GEMM_TN ? 5 : (layout == SCA_GEMM_NN ? 7 : 1);
  switch (tile) {
    case 20: return K_GLDS3;
    case 21: return K_GLDS2;
    case 22: return K_GLDS4;
    case 5: return K_T5;
    case 7: return K_T7;
    default: return K_T1;
  }
}

template <int LAYOUT>
int launch_tile(int tile, GemmArgs& a, int nprob, int maxM, int maxN, hipStream_t st) {
  constexpr bool KN = LAYOUT == SCA_GEMM_NN;
  switch (resolve_kernel(LAYOUT, tile, a, nprob)) {
    case K_T1_ANY: return launch<LAYOUT, T1, false>(a, nprob, maxM, maxN, st);
    case K_NTB45: return launch_ntb<true, 6, KN, true, 64>(a, nprob, maxM, maxN, st);
    case K_NTB44: return launch_ntb<true, 6, KN, true>(a, nprob, maxM, maxN, st);
    case K_NTB41: return launch_ntb<true, 6, KN>(a, nprob, maxM, maxN, st);
    case K_NTB42: return launch_ntb<false, 2, KN>(a, nprob, maxM, maxN, st);
    case K_TNK46: return launch_tnk<3, 1, true>(a, nprob, maxM, maxN, st);
    case K_TNB43: return launch_tnb<true, 6, true>(a, nprob, maxM, maxN, st);
    case K_TNB38: return launch_tnb<false, 2>(a, nprob, maxM, maxN, st);
    case K_TNB39: return launch_tnb<true, 4>(a, nprob, maxM, maxN, st);
    case K_TNB40: return launch_tnb<true, 6>(a, nprob, maxM, maxN, st);
    case K_TNK36: return launch_tnk<3, 1>(a, nprob, maxM, maxN, st);
    case K_TNK37: return launch_tnk<4, 1>(a, nprob, maxM, maxN, st);
    case K_GLDS3: return launch_glds<LAYOUT, 3>(a, nprob, maxM, maxN, st);
    case K_GLDS2: return launch_glds<LAYOUT, 2>(a, nprob, maxM, maxN, st);
    case K_GLDS4: return launch_glds<LAYOUT, 4>(a, nprob, maxM, maxN, st);
    case K_T5: return launch<LAYOUT, T5>(a, nprob, maxM, maxN, st);
    case K_T7: return launch<LAYOUT, T7>(a, nprob, maxM, maxN, st);
    default: return launch<LAYOUT, T1>(a, nprob, maxM, maxN, st);
  }
}

// rocprofv3-style short names of the resolved kernels (layout substituted where templated)
int kernel_name(int layout, KernelId k, char* buf, int len) {
  const char* kn = layout == SCA_GEMM_NN ? "true" : "false";
  switch (k) {
    case K_T1_ANY: return snprintf(buf, len, "gemm_kernel<%d, T1, false>", layout);
    case K_NTB45: return snprintf(buf, len, "gemm_ntb_kernel<true, 6, %s, true, 64>", kn);
    case K_NTB44: return snprintf(buf, len, "gemm_ntb_kernel<true, 6, %s, true, 128>", kn);
    case K_NTB41: return snprintf(buf, len, "gemm_ntb_kernel<true, 6, %s, false, 128>", kn);
    case K_NTB42: return snprintf(buf, len, "gemm_ntb_kernel<false, 2, %s, false, 128>", kn);
    case K_TNK46: return snprintf(buf, len, "gemm_tnk_kernel<3, 1, true>");
    case K_TNB43: return snprintf(buf, len, "gemm_tnb_kernel<true, 6, true>");
    case K_TNB38: return snprintf(buf, len, "gemm_tnb_kernel<false, 2, false>");
    case K_TNB39: return snprintf(buf, len, "gemm_tnb_kernel<true, 4, false>");
    case K_TNB40: return snprintf(buf, len, "gemm_tnb_kernel<true, 6, false>");
    case K_TNK36: return snprintf(buf, len, "gemm_tnk_kernel<3, 1, false>");
    case K_TNK37: return snprintf(buf, len, "gemm_tnk_kernel<4, 1, false>");
    case K_GLDS3: return snprintf(buf, len, "gemm_glds_kernel<%d, 3>", layout);
    case K_GLDS2: return snprintf(buf, len, "gemm_glds_kernel<%d, 2>", layout);
    case K_GLDS4: return snprintf(buf, len, "gemm_glds_kernel<%d, 4>", layout);
    case K_T5: return snprintf(buf, len, "gemm_kernel<%d, T5>", layout);
    case K_T7: return snprintf(buf, len, "gemm_kernel<%d, T7>", layout);
    default: return snprintf(buf, len, "gemm_kernel<%d, T1>", layout);
  }
}

int g_tile_override[3] = {0, 0, 0};

// SCA_NTB=0 keeps the NT / NN GEMMs on the LDS-DMA kernels (A/B switch), read once;
// SCA_NTB_MIN_K: the shortest reduction (summed over segments) routed to the 128x128 kernel
bool ntb_default() {
  static const bool on = !(getenv("SCA_NTB") && atoi(getenv("SCA_NTB")) == 0);
  return on;
}
int ntb_min_k() {
  static const int k = getenv("SCA_NTB_MIN_K") ? atoi(getenv("SCA_NTB_MIN_K")) : 512;
  return k;
}

// Tile heuristic (measured with tools/gemm_bench.py at the workload's shapes, see
// DESIGN.md): the 3-stage LDS-DMA 64x64 kernel wins every layout; ineligible shapes fall
// back to 64x64 / 4 waves (NT), 128x64 / 8 waves (NN), single-buffered 64x64 (TN).
int pick_tile(int layout, long tiles64, int splitk) {
  if (g_tile_override[layout]) return g_tile_override[layout];
  (void)splitk;
  (void)tiles64;
  // LDS-DMA kernel; launch_tile falls back per layout when a shape is not eligible.  The
  // input- and weight-gradient layouts use the 2-stage ring (32 KB: up to 5 workgroups / CU
  // beside the concurrent streams' kernels; bench.py A/B +0.9 %), the forward 3 stages.
  return layout == SCA_GEMM_NT ? 20 : 21;
}

}  // namespace

#ifdef SCA_GEMM_STAMPS
extern "C" int sca_gemm_stamps(unsigned long long* out, int n) {
  if (n > STAMP_MAX) n = STAMP_MAX;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 5 * n) == hipSuccess ? 0 : 3;
}
extern "C" int sca_gemm_clk(unsigned long long* out, int n) {
  if (n > STAMP_MAX) n = STAMP_MAX;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk), sizeof(unsigned long long) * 2 * n) == hipSuccess ? 0 : 3;
}
#endif

extern "C" void sca_set_error(const char* msg);

extern "C" int sca_gemm_tile_override(int layout, int tile) {
  if (layout < 0 || layout > 2 || !valid_tile(layout, tile)) {
    sca_set_error("sca_gemm_tile_override: unknown layout or kernel variant id");
    return SCA_ERR_ARG;
  }
  g_tile_override[layout] = tile;
  return SCA_OK;
}

extern "C" void sca_set_error(const char* msg);

namespace {
// the requested variant of a launch: the caller's, the process-wide override, or the heuristic
int choose_tile(int layout, const sca_gemm_problem* probs, int nprob, int splitk, int variant) {
  long tiles64 = 0;
  for (int i = 0; i < nprob; ++i) tiles64 += (long)((probs[i].M + 63) / 64) * ((probs[i].N + 63) / 64);
  int tile = variant ? variant : pick_tile(layout, tiles64, splitk);
  if (!variant && !g_tile_override[layout] && layout != SCA_GEMM_TN && splitk == 1 && tiles64 >= 2048 &&
      ntb_default()) {
    // big forward / input-gradient GEMMs (config 5: 8192-row operands, hundreds of 128x128
    // tiles): the register-staged 128x128 kernel when every problem's reduction is long
    // enough (tools/gemm_bench.py --cfg5); launch_tile hands ineligible shapes back to the
    // LDS-DMA kernel
    bool longk = true;
    for (int i = 0; i < nprob; ++i) {
      int k = 0;
      for (int s2 = 0; s2 < probs[i].nseg; ++s2) k += probs[i].seg[s2].K;
      longk = longk && k >= ntb_min_k();
    }
    if (longk) tile = 44;
  }
  if (!variant && !g_tile_override[layout] && layout != SCA_GEMM_TN && splitk == 1 && tile != 44 &&
      ntb_default())
    tile = 45;  // every other NT / NN GEMM: the 64x64 form (tools/gemm_bench.py: +5 to +13 % over the
                // LDS-DMA kernels at config 2's shapes); launch_tile hands ineligible shapes back
  return tile;
}

// do_main: the GEMM launch; do_reduce: the split-K slab reduction (splitk > 1 only)
int gemm_impl(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace, void* stream,
              bool do_main, bool do_reduce, unsigned* counters = nullptr, int variant = 0) {
  if (nprob <= 0) return SCA_OK;
  if (nprob > SCA_GEMM_MAX_PROBLEMS || layout < 0 || layout > 2 || splitk < 1) {
    sca_set_error("sca_gemm: bad nprob/layout/splitk");
    return SCA_ERR_ARG;
  }
  GemmArgs a;
  a.splitk = splitk;
  a.nprob = nprob;
  a.ws = workspace;
  a.drop_off = sca_drop_offset_ptr();
  a.counters = nullptr;
  a.flat = 0;
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
      // any K, lda, ldb and operand alignment: shapes the float4 loads cannot take run the
      // element-wise form of the register-staged kernel (vec_ok)
      if (!S.A || !S.B || S.K < 0 || (reinterpret_cast<uintptr_t>(S.A) & 3) || (reinterpret_cast<uintptr_t>(S.B) & 3)) {
        sca_set_error("sca_gemm: null or misaligned (not 4-byte) operand, or negative K");
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
    if ((P.epi & SCA_EPI_DROPOUT) && !(P.drop_p >= 0.f && P.drop_p < 1.f)) {
      sca_set_error("sca_gemm: drop_p must be in [0, 1)");
      return SCA_ERR_ARG;
    }
    if (splitk > 1 && P.nseg != 1) {
      sca_set_error("sca_gemm: split-K needs one segment per problem");
      return SCA_ERR_ARG;
    }
    a.p[i] = P;
    maxM = maxM > P.M ? maxM : P.M;
    maxN = maxN > P.N ? maxN : P.N;
  }
  if (splitk > 1 && !workspace) { sca_set_error("sca_gemm: split-K needs workspace"); return SCA_ERR_ARG; }
  if (splitk > 1) {  // workspace: every problem's splitk slabs, then every problem's bias partials
    long o = 0;
    for (int i = 0; i < nprob; ++i) {
      a.slab_off[i] = o;
      o += (long)splitk * probs[i].M * probs[i].N;
    }
    for (int i = 0; i < nprob; ++i) {
      a.bias_off[i] = o;
      o += (long)splitk * probs[i].M;
    }
  }
  if (maxM == 0 || maxN == 0) return SCA_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int rc;
  int tile = choose_tile(layout, probs, nprob, splitk, variant);
  // in-launch split-K combine: the 4-wave LDS-DMA kernel only (else the separate reduce runs)
  const bool tn_big =
      layout == SCA_GEMM_TN && ((tile >= kTnFirst && tile <= kTnLast) || tile == 43 || tile == 46) && tn_ok(a, nprob);
  if (counters && splitk > 1 && (tile == 20 || tile == 21 || tile == 22 || tn_big) && glds_ok(a, nprob) &&
      vec_ok(a, nprob, layout)) {
    a.counters = counters;
    do_reduce = false;
  }
  if (do_main) switch (layout) {
    case SCA_GEMM_NT: rc = launch_tile<SCA_GEMM_NT>(tile, a, nprob, maxM, maxN, st); break;
    case SCA_GEMM_NN: rc = launch_tile<SCA_GEMM_NN>(tile, a, nprob, maxM, maxN, st); break;
    default: rc = launch_tile<SCA_GEMM_TN>(tile, a, nprob, maxM, maxN, st); break;
  }
  else rc = SCA_OK;
  if (rc != SCA_OK) { sca_set_error("sca_gemm: launch failed"); return rc; }
  if (splitk > 1 && do_reduce) {
    const long MN = (long)maxM * maxN;
    bool vec = true;  // 16-B form: every N and ldc a multiple of 4, C 16-byte aligned
    for (int i = 0; i < nprob; ++i)
      vec = vec && !(probs[i].N & 3) && !(probs[i].ldc & 3) && !(reinterpret_cast<uintptr_t>(probs[i].C) & 15);
    if (vec) {
      const int nc4 = (int)((MN / 4 + 255) / 256);
      dim3 grid((unsigned)(nc4 + (maxM + 255) / 256), nprob);
      hipLaunchKernelGGL(splitk_reduce4_kernel, grid, dim3(256), 0, st, a, nc4);
    } else {
      dim3 grid((unsigned)((MN + maxM + 255) / 256), nprob);
      hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, st, a, nprob);
    }
    if (hipGetLastError() != hipSuccess) { sca_set_error("sca_gemm: reduce launch failed"); return SCA_ERR_LAUNCH; }
  }
  return SCA_OK;
}
}  // namespace

extern "C" int sca_gemm(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
                        void* stream) {
  return gemm_impl(layout, nprob, probs, splitk, workspace, stream, true, true);
}

extern "C" int sca_gemm_partial(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
                                void* stream) {
  return gemm_impl(layout, nprob, probs, splitk, workspace, stream, true, false);
}

extern "C" int sca_gemm_reduce(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
                               void* stream) {
  return gemm_impl(layout, nprob, probs, splitk, workspace, stream, false, true);
}

extern "C" int sca_gemm_kernel_name(int layout, int nprob, const sca_gemm_problem* probs, int splitk, int variant,
                                    char* buf, int len) {
  if (nprob < 1 || nprob > SCA_GEMM_MAX_PROBLEMS || layout < 0 || layout > 2 || splitk < 1 || !buf || len < 1 ||
      (variant && !valid_tile(layout, variant))) {
    sca_set_error("sca_gemm_kernel_name: bad arguments");
    return SCA_ERR_ARG;
  }
  GemmArgs a;
  a.splitk = splitk;
  a.nprob = nprob;
  for (int i = 0; i < nprob; ++i) a.p[i] = probs[i];
  kernel_name(layout, resolve_kernel(layout, choose_tile(layout, probs, nprob, splitk, variant), a, nprob), buf, len);
  return SCA_OK;
}

extern "C" long sca_gemm_splitk_counters(int nprob, int maxM, int maxN) {
  return (long)nprob * ((maxM + GL_BM - 1) / GL_BM) * ((maxN + GL_BN - 1) / GL_BN);
}

extern "C" int sca_gemm_splitk_fused(int layout, int nprob, const sca_gemm_problem* probs, int splitk,
                                     float* workspace, unsigned* counters, void* stream) {
  return gemm_impl(layout, nprob, probs, splitk, workspace, stream, true, true, counters);
}

extern "C" int sca_gemm_variant(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
                                unsigned* counters, int variant, void* stream) {
  if (layout < 0 || layout > 2 || !valid_tile(layout, variant)) {
    sca_set_error("sca_gemm_variant: unknown layout or kernel variant id");
    return SCA_ERR_ARG;
  }
  return gemm_impl(layout, nprob, probs, splitk, workspace, stream, true, true, counters, variant);
}

// 32-row tiles (8 waves) whenever they give a workgroup per CU, else 16-row tiles (2
// workgroups / CU): tools/gemm_ln_bench.py 4x(2048,256,K): K = 768 41.0 vs 44.6 us,
// K = 256 19.8 vs 20.8 us; 1x(2048,256,256): 15.2 vs 10.9 us.  Chained passes: always 32.
// A forced tile height (16 / 32; 0 = the rule above): SCA_GEMM_LN_BM, read once on the first
// launch, or sca_gemm_ln_force_rows (tests that compare launches of different row counts).
static int g_ln_bm_force = -1;

static int ln_bm_force() {
  if (g_ln_bm_force < 0) {
    const char* env = getenv("SCA_GEMM_LN_BM");
    const int v = env ? atoi(env) : 0;
    g_ln_bm_force = (v == 16 || v == 32) ? v : 0;
  }
  return g_ln_bm_force;
}

extern "C" int sca_gemm_ln_force_rows(int bm) {
  if (bm != 0 && bm != 16 && bm != 32) {
    sca_set_error("sca_gemm_ln_force_rows: bm must be 0, 16 or 32");
    return SCA_ERR_ARG;
  }
  g_ln_bm_force = bm;
  return SCA_OK;
}

extern "C" int sca_gemm_ln_rows(int nprob, int maxM, int chain) {
  const int bm_force = ln_bm_force();
  const long wg32 = (long)nprob * ((maxM + 31) / 32);
  if (chain) return 32;
  if (bm_force) return bm_force;
  // the register-staged 32-row loop beats the 16-row LDS-DMA tiles even below one workgroup
  // per CU (config 3: 1605 -> 1630 clips/s, profiles/r05_ntb/ln_rows_cfg3_ab.txt), but not
  // at a quarter of the CUs (1 x (2048, 256, 256): 13.7 vs 10.7 us, tools/gemm_ln_bench.py)
  if (ln_reg_default() && wg32 >= 128) return 32;
  return wg32 >= 256 ? 32 : 16;
}

extern "C" int sca_gemm_ln(int nprob, const sca_gemm_problem* probs, const sca_gemm_ln_problem* ln, float eps,
                           void* stream) {
  if (nprob <= 0) return SCA_OK;
  if (nprob > SCA_GEMM_LN_MAX_PROBLEMS || !probs || !ln || !(eps >= 0.f)) {
    sca_set_error("sca_gemm_ln: bad nprob / pointers / eps");
    return SCA_ERR_ARG;
  }
  GemmLnArgs a;
  bool chain = false;
  static const int rot_env = getenv("SCA_GEMM_LN_ROT") ? atoi(getenv("SCA_GEMM_LN_ROT")) : 1;
  a.rot = rot_env;
  a.eps = eps;
  a.drop_off = sca_drop_offset_ptr();
  int maxM = 0;
  const int N = probs[0].N;  // 256, or 512 (two column halves, no chained passes)
  for (int i = 0; i < nprob; ++i) {
    const sca_gemm_problem& P = probs[i];
    const sca_gemm_ln_problem& L = ln[i];
    const sca_gemm_seg& S = P.seg[0];
    const bool al16 = !((reinterpret_cast<uintptr_t>(S.A) | reinterpret_cast<uintptr_t>(S.B) |
                         reinterpret_cast<uintptr_t>(P.C) | reinterpret_cast<uintptr_t>(P.resid) |
                         reinterpret_cast<uintptr_t>(P.bias) | reinterpret_cast<uintptr_t>(L.y) |
                         reinterpret_cast<uintptr_t>(L.gamma) | reinterpret_cast<uintptr_t>(L.beta)) & 15);
    if (P.nseg != 1 || (N != LG_BN && N != 2 * LG_BN) || P.N != N || P.M < 0 || S.K < GL_BK || (S.K % GL_BK) ||
        !S.A || !S.B || !P.C || !L.gamma || !L.beta || !L.y || !L.mean || !L.rstd || !al16 || (S.lda & 3) ||
        (S.ldb & 3) || S.lda < S.K || S.ldb < S.K || (P.ldc & 3) || P.ldc < N || (P.resid && ((P.ldr & 3) || P.ldr < N)) ||
        (P.epi & ~SCA_EPI_DROPOUT) || ((P.epi & SCA_EPI_DROPOUT) && !(P.drop_p >= 0.f && P.drop_p < 1.f))) {
      sca_set_error("sca_gemm_ln: needs one segment, N == 256 or 512 (the same for every problem), K a positive "
                    "multiple of 32, 16-byte aligned operands with leading dimensions multiple of 4, and no "
                    "epilogue other than dropout");
      return SCA_ERR_ARG;
    }
    if (L.npass < 0 || L.npass > 3 || (N != LG_BN && L.npass != 0)) {
      sca_set_error("sca_gemm_ln: npass must be 0..3 (0 at N = 512)");
      return SCA_ERR_ARG;
    }
    for (int q = 0; q < L.npass; ++q) {
      const sca_gemm_chain_pass& Q = L.pass[q];
      const bool gelu = Q.epi == SCA_EPI_GELU;
      if (!Q.B || !Q.C || (Q.ldb & 3) || Q.ldb < LG_BN || (Q.ldc & 3) || Q.ldc < LG_BN ||
          (Q.epi != 0 && !gelu) || (gelu && (!Q.aux_out || (Q.ldo & 3) || Q.ldo < LG_BN)) ||
          ((reinterpret_cast<uintptr_t>(Q.B) | reinterpret_cast<uintptr_t>(Q.C) |
            reinterpret_cast<uintptr_t>(Q.bias) | reinterpret_cast<uintptr_t>(gelu ? Q.aux_out : nullptr)) & 15)) {
        sca_set_error("sca_gemm_ln: chained pass needs B [256, ldb >= 256] and C (ldc >= 256), 16-byte aligned, "
                      "leading dimensions multiple of 4, epi 0 or SCA_EPI_GELU (with aux_out)");
        return SCA_ERR_ARG;
      }
    }
    chain = chain || L.npass > 0;
    a.p[i] = P;
    a.ln[i] = L;
    maxM = maxM > P.M ? maxM : P.M;
  }
  if (maxM == 0) return SCA_OK;
  const int bm = sca_gemm_ln_rows(nprob, maxM, chain);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (N != LG_BN) {
    hipLaunchKernelGGL((gemm_ln_kernel<GL_A32, false, 2>), dim3((maxM + 31) / 32, 1, nprob), dim3(512), 0, st, a);
  } else if (chain) {
    bool reg = ln_reg_default();
    for (int i = 0; i < nprob; ++i) reg = reg && ln_reg_ok(probs[i], false);
    if (reg)
      hipLaunchKernelGGL((gemm_ln_kernel<GL_A32, true, 1, true>), dim3((maxM + 31) / 32, 1, nprob), dim3(512), 0, st, a);
    else
      hipLaunchKernelGGL((gemm_ln_kernel<GL_A32, true, 1>), dim3((maxM + 31) / 32, 1, nprob), dim3(512), 0, st, a);
  } else if (bm == 16) {
    hipLaunchKernelGGL((gemm_ln_kernel<GL_A16, false, 1>), dim3((maxM + 15) / 16, 1, nprob), dim3(256), 0, st, a);
  } else {
    bool reg = ln_reg_default();
    for (int i = 0; i < nprob; ++i) reg = reg && ln_reg_ok(probs[i], false);
    if (reg)
      hipLaunchKernelGGL((gemm_ln_kernel<GL_A32, false, 1, true>), dim3((maxM + 31) / 32, 1, nprob), dim3(512), 0, st, a);
    else
      hipLaunchKernelGGL((gemm_ln_kernel<GL_A32, false, 1>), dim3((maxM + 31) / 32, 1, nprob), dim3(512), 0, st, a);
  }
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_gemm_ln: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_gemm_lnb_blocks(int M) { return M > 0 ? (M + LB_BM - 1) / LB_BM : 0; }

extern "C" int sca_gemm_lnb(int nprob, const sca_gemm_problem* probs, const sca_gemm_lnb_problem* lnb,
                            void* stream) {
  if (nprob <= 0) return SCA_OK;
  if (nprob > SCA_GEMM_MAX_PROBLEMS || !probs || !lnb) {
    sca_set_error("sca_gemm_lnb: bad nprob / pointers");
    return SCA_ERR_ARG;
  }
  GemmLnbArgs a;
  int maxM = 0;
  const int N = probs[0].N;  // 256, or 512 (two column halves, no chained GEMM)
  for (int i = 0; i < nprob; ++i) {
    const sca_gemm_problem& P = probs[i];
    const sca_gemm_lnb_problem& L = lnb[i];
    bool ok = P.nseg >= 1 && P.nseg <= SCA_GEMM_MAX_SEGS && (N == LG_BN || N == 2 * LG_BN) && P.N == N &&
              P.M >= 0 && P.C && L.x && L.mean &&
              L.rstd && L.gamma && L.dx && L.partial && P.epi == 0 && !P.bias && !P.bias_grad &&
              P.post_scale == 1.f && (P.ldc & 3) == 0 && P.ldc >= N &&
              (!P.resid || ((P.ldr & 3) == 0 && P.ldr >= N)) && (N == LG_BN || !L.wo) &&
              (!L.tab || (L.tab_T >= 1 && !(reinterpret_cast<uintptr_t>(L.tab) & 15)));
    uintptr_t al = reinterpret_cast<uintptr_t>(P.C) | reinterpret_cast<uintptr_t>(P.resid) |
                   reinterpret_cast<uintptr_t>(L.x) | reinterpret_cast<uintptr_t>(L.gamma) |
                   reinterpret_cast<uintptr_t>(L.dx) | reinterpret_cast<uintptr_t>(L.wo) |
                   reinterpret_cast<uintptr_t>(L.dout) | reinterpret_cast<uintptr_t>(L.aux);
    ok = ok && ((L.wo == nullptr) == (L.dout == nullptr)) && (L.wo || !L.aux);
    if (L.wo) {
      const int np = L.npass ? L.npass : 1;
      const int ldw = L.ldw ? L.ldw : LG_BN * np;
      ok = ok && L.npass >= 0 && L.npass <= 3 && (ldw & 3) == 0 && ldw >= LG_BN * np;
    }
    for (int s = 0; ok && s < P.nseg; ++s) {
      const sca_gemm_seg& S = P.seg[s];
      ok = S.A && S.B && S.K >= GL_BK && S.K % GL_BK == 0 && (S.lda & 3) == 0 && S.lda >= S.K &&
           (S.ldb & 3) == 0 && S.ldb >= N && S.alpha == P.seg[0].alpha;
      al |= reinterpret_cast<uintptr_t>(S.A) | reinterpret_cast<uintptr_t>(S.B);
    }
    if (!ok || (al & 15)) {
      sca_set_error("sca_gemm_lnb: needs N == 256 or 512 (the same for every problem), 1-3 segments with K a "
                    "positive multiple of 32 and one alpha, k-major B, no epilogue other than resid, 16-byte aligned "
                    "operands with leading dimensions multiple of 4; chained (N == 256 only): wo and dout both or "
                    "neither, npass 0..3, ldw >= 256 npass");
      return SCA_ERR_ARG;
    }
    a.p[i] = P;
    a.ln[i] = L;
    maxM = maxM > P.M ? maxM : P.M;
  }
  if (maxM == 0) return SCA_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  bool reg = N == LG_BN && ln_reg_default();
  for (int i = 0; i < nprob; ++i) reg = reg && ln_reg_ok(probs[i], true);
  bool chained = false;
  for (int i = 0; i < nprob; ++i) chained = chained || a.ln[i].wo != nullptr;
  if (reg && chained && lnb_r3_default())
    hipLaunchKernelGGL((gemm_lnb_kernel<1, true, true>), dim3((maxM + LB_BM - 1) / LB_BM, 1, nprob), dim3(512), 0, st, a);
  else if (reg) hipLaunchKernelGGL((gemm_lnb_kernel<1, true>), dim3((maxM + LB_BM - 1) / LB_BM, 1, nprob), dim3(512), 0, st, a);
  else if (N == LG_BN) hipLaunchKernelGGL(gemm_lnb_kernel<1>, dim3((maxM + LB_BM - 1) / LB_BM, 1, nprob), dim3(512), 0, st, a);
  else hipLaunchKernelGGL(gemm_lnb_kernel<2>, dim3((maxM + LB_BM - 1) / LB_BM, 1, nprob), dim3(512), 0, st, a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_gemm_lnb: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}
