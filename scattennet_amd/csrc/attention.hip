// Fused masked attention (forward + backward) on the gfx950 f32 matrix cores
// (v_mfma_f32_16x16x4_f32), for the three SCAttenNet attention operators:
//   SelfAttention        model/attention.py:46-76   (key-padding mask)
//   SelfCausalAttention  model/attention.py:148-182 (tril -> -inf, then +causal mask)
//   CrossAttention       model/attention.py:97-128  (key-padding mask, Tq may != Tk)
//
// Layout in HBM: activations stay (B, T, H*hd) row-major exactly as the projections write
// them (no head transposes: head h is the column slice h*hd .. h*hd+hd-1).
//
// Base-2 domain: a score s becomes t = s*log2(e) + add_j with one fma, where add_j is per
// key (in LDS):
//   valid key            plus*log2(e)   plus = 1.0 for the causal mask (utils.py:24-27), else 0
//   padded key           finfo.min      (utils.py:3-12; s + finfo.min rounds to finfo.min)
//   key >= Tk            -inf           (not part of the row at all)
// and p = exp2(t - m) is one raw v_exp_f32.  With an explicit additive (B,1,Tq,Tk) mask
// (general path) the mask value is added in natural units first.  Causal keys above the
// diagonal (attention.py:165-169) only exist in the last (diagonal) key block of a query
// block: that block runs a separately compiled step, every other block is branch-free.
//
// LDS images are unpadded and XOR-swizzled so that every ds_read_b128 fragment read is
// conflict-free in the gfx950 lane groups (row images: swizzle on the float4 slot by the
// row; transposed images [hd][64]: slot ^ 2*(row & 7)).
//
// Forward: one workgroup = (problem g, clip b, head h, 64 queries); 4 waves x 16 queries.
// K/V stream through LDS in 64-key blocks (register-prefetched one block ahead, one barrier
// per block).  Scores are computed SWAPPED (S^T = K Q^T) so a lane owns one query column and
// 4 keys per 16x16 tile: the row max / row sum need two xor-shuffles, and the S^T
// accumulator registers are already the B operand of O^T += V^T P^T — P never leaves
// registers.  Online softmax.  Saves m (row max) and ll = log2(row sum) per row: a fully
// padded row (all finfo.min) then recomputes to exactly uniform weights in the backward.
//
// Backward: two kernels, no atomics (deterministic):
//   dq kernel   (query-block major): delta = rowsum(dO*O); S^T, dP^T recomputed;
//               dS = P (dP - delta); dQ^T += K^T dS^T.
//   dkdv kernel (key-block major):   S, dP recomputed with the key on the lane;
//               dV^T += dO^T P ; dK^T += Q^T dS.
#include <type_traits>

#include "common.h"
#include "../../include/scatten.h"

namespace {

constexpr int QB = 64;  // queries per workgroup (16 per wave)
constexpr int KB = 64;  // keys per LDS block
constexpr float L2E = SCA_LOG2E;

struct FwdArgs {
  sca_attn_fwd_problem p[SCA_ATTN_MAX_PROBLEMS];
  int B, H, Tq, Tk, ldq, ldk, ldv, ldo, causal, plus_one;
  const unsigned long long* drop_off;  // dropout step counter (sca_dropout_offset) or NULL
};

struct BwdArgs {
  sca_attn_bwd_problem p[SCA_ATTN_MAX_PROBLEMS];
  int B, H, Tq, Tk, ldq, ldk, ldv, ldo, causal, plus_one;
  const unsigned long long* drop_off;
};

// attention-probability dropout (DROP kernels): the sca_dropout mask of the problem's seed
// over the (B, H, Tq, Tk) probabilities, element ((b H + h) Tq + i) Tk + j (mod 2^32)
__device__ __forceinline__ uint32_t drop_row(int b, int H, int h, int Tq, int Tk, int i) {
  return ((uint32_t)(b * H + h) * (uint32_t)Tq + (uint32_t)i) * (uint32_t)Tk;
}

using DiagStep = std::true_type;
using FullStep = std::false_type;

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Natural-units masked score -> base-2 domain (general additive-mask path).  Values that
// overflow to -inf only come from finfo.min masks: they all map to finfo.min.
__device__ __forceinline__ float to_log2(float t) {
  const float t2 = t * L2E;
  return (t2 == -INFINITY && t != -INFINITY) ? SCA_FMIN : t2;
}

// The validity word is loaded separately (kv_load) so that the compare happens at
// LDS-commit time: a compare right after the load would make the wave wait for the whole
// K/V prefetch that was issued with it.
__device__ __forceinline__ float kv_load(const float* key_valid, int b, int j, int Tk) {
  return key_valid ? key_valid[(long)b * Tk + min(j, Tk - 1)] : 1.f;
}

// per-key additive term in the base-2 domain (see header comment)
// (clip, head) slice of a materialised additive mask: [B, Tq, Tk] (mask_heads 0 / 1) or
// [B, H, Tq, Tk] (mask_heads = H)
__device__ __forceinline__ long mask_clip(int mask_heads, int b, int H, int h) {
  return mask_heads > 1 ? (long)b * H + h : (long)b;
}

__device__ __forceinline__ float key_add(float kv, bool add_mask, int j, int Tk, float plus2) {
  if (j >= Tk) return -INFINITY;
  if (add_mask) return 0.f;
  return kv == 0.f ? SCA_FMIN : plus2;
}

// Row block of HD floats per row, 64 rows: each thread owns RV = HD/16 float4 of it.
template <int HD>
struct Blk {
  static constexpr int V4 = HD / 4;          // float4 per row
  static constexpr int RV = 64 * V4 / 256;   // float4 per thread
};

// float4-slot swizzle of row r in a [64][HD] row image (conflict-free fragment reads)
template <int HD>
__device__ __forceinline__ int row_swz(int r) {
  if constexpr (HD == 16) return (0x78 >> (2 * ((r >> 2) & 3))) & 3;  // [0, 2, 3, 1]
  else if constexpr (HD == 32) return ((r >> 1) & 1) | (((r >> 2) & 1) << 2);
  else return (r & 3) | ((r & 4) << 1);
}

template <int HD>
__device__ __forceinline__ f32x4 row_frag(const float* img, int row, int slot) {
  return ld4(img + row * HD + 4 * (slot ^ row_swz<HD>(row)));
}

// float4-slot swizzle of row d in a transposed [HD][64] image.  Bits 1-3 carry d >> 2 so
// that the ds_write_b32 transposes of store_cols (32-lane groups, banks mod 32) are
// conflict-free at hd 16 and bits 0/3 carry d & 3 so that the 16-lane ds_read_b128 groups of
// col_frag stay conflict-free (MI355X_MICROARCH.md §LDS lane groups; hd 32/64 keep 2-way
// store conflicts instead of the 8-way of a d & 7 swizzle)
__device__ __forceinline__ int col_swz(int d) {
  return (((d >> 2) << 1) | (d & 1) | ((d & 2) << 2)) & 15;
}

// transposed image [HD][64]: 4 consecutive keys/queries at float4 slot `slot` of row d
__device__ __forceinline__ f32x4 col_frag(const float* img, int d, int slot) {
  return ld4(img + d * 64 + 4 * (slot ^ col_swz(d)));
}

template <int HD>
__device__ __forceinline__ void blk_load(f32x4* r, const float* base, long ld, int r0, int nrows) {
#pragma unroll
  for (int i = 0; i < Blk<HD>::RV; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int row = e / Blk<HD>::V4, c = (e % Blk<HD>::V4) * 4;
    // rows past the end read the last row (never used: their scores are -inf / not stored)
    r[i] = ld4(base + (long)min(r0 + row, nrows - 1) * ld + c);
  }
}

template <int HD>
__device__ __forceinline__ void store_rows(float* img, const f32x4* r) {
#pragma unroll
  for (int i = 0; i < Blk<HD>::RV; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int row = e / Blk<HD>::V4, s = e % Blk<HD>::V4;
    st4(img + row * HD + 4 * (s ^ row_swz<HD>(row)), r[i]);
  }
}

template <int HD>
__device__ __forceinline__ void store_cols(float* img, const f32x4* r) {
#pragma unroll
  for (int i = 0; i < Blk<HD>::RV; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int row = e / Blk<HD>::V4, c = (e % Blk<HD>::V4) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = c + j;
      img[d * 64 + 4 * ((row >> 2) ^ col_swz(d)) + (row & 3)] = r[i][j];
    }
  }
}

// XCD-aware block order (cdna_hip_programming.md T1): the hardware deals workgroups round-robin
// over the 8 XCDs (private L2 each).  Renumber so that each XCD gets a contiguous range of
// (problem, clip, head, block) tiles: the blocks of one (clip, head) re-read the same K/V
// (or Q/dO) slice, and neighbouring heads share 128-B lines, so both now hit one L2.
struct TileId {
  int x, y, z;
};
__device__ __forceinline__ TileId xcd_tile() {
  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned nwg = gx * gy * gridDim.z;
  const unsigned orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const unsigned id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  return TileId{(int)(id % gx), (int)((id / gx) % gy), (int)(id / (gx * gy))};
}

// ------------------------------------------------------------------------------ forward
template <int HD, bool ADDMASK, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256, HD <= 64 ? 2 : 1) void attn_fwd_kernel(const FwdArgs a) {
  constexpr int NS = HD / 4;   // MFMA k-steps over the head dim
  constexpr int ND = HD / 16;  // 16-wide output d-blocks
  constexpr int RV = Blk<HD>::RV;
  constexpr int NB = HD <= 64 ? 2 : 1;  // LDS buffers per image (hd 128: single, see commit)
  __shared__ __attribute__((aligned(16))) float Ks[NB][KB * HD];
  __shared__ __attribute__((aligned(16))) float Vt[NB][HD * KB];
  __shared__ __attribute__((aligned(16))) float Ka[NB][KB];

  const TileId tid = xcd_tile();
  const sca_attn_fwd_problem& P = a.p[tid.z];
  const int b = tid.y / a.H, h = tid.y % a.H;
  const int nqb = (a.Tq + QB - 1) / QB;  // causal: block x is paired with block nqb-1-x
  const int jobs = (CAUSAL && nqb - 1 - tid.x != tid.x) ? 2 : 1;
#pragma unroll 1
  for (int job = 0; job < jobs; ++job) {
  const int xb = job ? nqb - 1 - tid.x : tid.x;
  const int q0 = xb * QB;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int qi = lane & 15, grp = lane >> 4;
  const int qrow = q0 + 16 * w + qi;
  const float plus2 = (CAUSAL && a.plus_one) ? L2E : 0.0f;
  DropMask dm;
  if (DROP) dm.init(P.drop_seed, P.drop_p, a.drop_off);
  const uint32_t erow = drop_row(b, a.H, h, a.Tq, a.Tk, qrow);

  // Q fragment: lane holds Q[qrow][NS*grp + s], s < NS (B operand of S^T = K Q^T)
  float qreg[NS];
  {
    const float* qp = P.q + ((long)b * a.Tq + min(qrow, a.Tq - 1)) * a.ldq + h * HD + NS * grp;
#pragma unroll
    for (int s = 0; s < NS; s += 4) {
      const f32x4 v = ld4(qp + s);
#pragma unroll
      for (int j = 0; j < 4; ++j) qreg[s + j] = v[j];
    }
  }
  const float* amrow = ADDMASK ? P.add_mask + (mask_clip(P.mask_heads, b, a.H, h) * a.Tq + min(qrow, a.Tq - 1)) * a.Tk
                               : nullptr;

  f32x4 o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  // causal: Tq == Tk and QB == KB, so the last key block is the diagonal one
  const int nblk = CAUSAL ? xb + 1 : (a.Tk + KB - 1) / KB;
  const float* kbase = P.k + (long)b * a.Tk * a.ldk + h * HD;
  const float* vbase = P.v + (long)b * a.Tk * a.ldv + h * HD;

  f32x4 rk[RV], rv[RV];
  float kvraw = 1.f;
  int kbn = 0;
  auto prefetch = [&](int kb) {
    blk_load<HD>(rk, kbase, a.ldk, kb, a.Tk);
    blk_load<HD>(rv, vbase, a.ldv, kb, a.Tk);
    kvraw = kv_load(P.key_valid, b, kb + (threadIdx.x & (KB - 1)), a.Tk);
    kbn = kb;
  };
  auto commit = [&](int buf) {
    store_rows<HD>(Ks[buf], rk);
    store_cols<HD>(Vt[buf], rv);
    if (threadIdx.x < KB) Ka[buf][threadIdx.x] = key_add(kvraw, ADDMASK, kbn + threadIdx.x, a.Tk, plus2);
  };
  prefetch(0);
  commit(0);
  __syncthreads();

  auto step = [&](auto diag_c, int blk) {
    constexpr bool DIAG = decltype(diag_c)::value;
    const int kb = blk * KB, buf = NB == 2 ? (blk & 1) : 0;
    const bool more = blk + 1 < nblk;
    float sv[4][4];
    // the four key tiles' S chains are interleaved k-step by k-step: independent
    // accumulators keep the MFMA pipe busy instead of waiting out each chain's latency
    f32x4 sacc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) sacc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; s += 4) {
      f32x4 kv[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (!(DIAG && t > w)) kv[t] = row_frag<HD>(Ks[buf], 16 * t + qi, (NS * grp + s) >> 2);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (!(DIAG && t > w)) sacc[t] = mfma16(kv[t][j], qreg[s + j], sacc[t]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (DIAG && t > w) {  // wave-uniform: the whole tile is above the diagonal
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[t][r] = -INFINITY;
        continue;
      }
      const f32x4 acc = sacc[t];
      const int kl = 16 * t + 4 * grp;
      const f32x4 ad = ld4(&Ka[buf][kl]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t2;
        if (ADDMASK) t2 = to_log2(acc[r] + (kb + kl + r < a.Tk ? amrow[kb + kl + r] : 0.f) + ad[r]);
        else t2 = fmaf(acc[r], L2E, ad[r]);
        if (DIAG && t == w && 4 * grp + r > qi) t2 = -INFINITY;
        sv[t][r] = t2;
      }
    }
    // online softmax (row = this lane's query; 16 values here, 64 across the 4 lanes)
    float mloc = sv[0][0];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) mloc = fmaxf(mloc, sv[t][r]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);  // finite after block 0 (key 0 is always in the row)
    const float alpha = fast_exp2(m_run - m_new);
    m_run = m_new;
    float ps[4] = {0.f, 0.f, 0.f, 0.f};  // 4 partial sums: short dependent add chains
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = fast_exp2(sv[t][r] - m_new);
        ps[r] += p;  // the row sum (softmax statistics) of the undropped probabilities
        sv[t][r] = DROP ? dm.apply(erow + (uint32_t)(kb + 16 * t + 4 * grp + r), p) : p;
      }
    const float psum = (ps[0] + ps[1]) + (ps[2] + ps[3]);
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int d = 0; d < ND; ++d) o[d] *= alpha;
    if (more) prefetch(kb + KB);  // in flight during the P.V MFMAs and the barrier
    // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (DIAG && t > w) continue;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const f32x4 vv = col_frag(Vt[buf], 16 * d + qi, 4 * t + grp);
#pragma unroll
        for (int r = 0; r < 4; ++r) o[d] = mfma16(vv[r], sv[t][r], o[d]);
      }
    }
    if constexpr (NB == 2) {
      if (more) commit(buf ^ 1);
      __syncthreads();
    } else {  // one buffer: every wave done reading it before the next block is stored
      __syncthreads();
      if (more) {
        commit(0);
        __syncthreads();
      }
    }
  };
  for (int blk = 0; blk + (CAUSAL ? 1 : 0) < nblk; ++blk) step(FullStep{}, blk);
  if (CAUSAL) step(DiagStep{}, nblk - 1);

  float l_tot = l_run + __shfl_xor(l_run, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if (qrow < a.Tq) {
    const float inv = 1.0f / l_tot;
    float* op = P.o + ((long)b * a.Tq + qrow) * a.ldo + h * HD + 4 * grp;
#pragma unroll
    for (int d = 0; d < ND; ++d) st4(op + 16 * d, o[d] * inv);
    if (grp == 0) {
      const long si = ((long)b * a.H + h) * a.Tq + qrow;
      P.stat_m[si] = m_run;
      P.stat_ll[si] = log2f(l_tot);
    }
  }
  }  // job
}

// ------------------------------------------------------------------------------ backward: dQ
template <int HD, bool ADDMASK, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const BwdArgs a) {
  constexpr int NS = HD / 4;
  constexpr int ND = HD / 16;
  constexpr int RV = Blk<HD>::RV;
  constexpr int NB = HD <= 64 ? 2 : 1;  // hd 128: one buffer per image (96 KB of LDS)
  __shared__ __attribute__((aligned(16))) float Ks[NB][KB * HD];
  __shared__ __attribute__((aligned(16))) float Vs[NB][KB * HD];
  __shared__ __attribute__((aligned(16))) float Kt[NB][HD * KB];
  __shared__ __attribute__((aligned(16))) float Ka[NB][KB];

  const TileId tid = xcd_tile();
  const sca_attn_bwd_problem& P = a.p[tid.z];
  const int b = tid.y / a.H, h = tid.y % a.H;
  const int nqb = (a.Tq + QB - 1) / QB;  // causal: block x is paired with block nqb-1-x
  const int jobs = (CAUSAL && nqb - 1 - tid.x != tid.x) ? 2 : 1;
#pragma unroll 1
  for (int job = 0; job < jobs; ++job) {
  const int xb = job ? nqb - 1 - tid.x : tid.x;
  const int q0 = xb * QB;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int qi = lane & 15, grp = lane >> 4;
  const int qrow = q0 + 16 * w + qi;
  const bool qok = qrow < a.Tq;
  const int qc = min(qrow, a.Tq - 1);
  const float plus2 = (CAUSAL && a.plus_one) ? L2E : 0.0f;

  float qreg[NS], doreg[NS];
  float dpart = 0.f;
  {
    const long roff = (long)b * a.Tq + qc;
    const float* qp = P.q + roff * a.ldq + h * HD + NS * grp;
    const float* dp = P.dout + roff * a.ldo + h * HD + NS * grp;
    const float* opp = P.o + roff * a.ldo + h * HD + NS * grp;
#pragma unroll
    for (int s = 0; s < NS; s += 4) {
      const f32x4 qv = ld4(qp + s), dv = ld4(dp + s), ov = ld4(opp + s);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        qreg[s + j] = qv[j];
        doreg[s + j] = dv[j];
        dpart += dv[j] * ov[j];
      }
    }
  }
  dpart += __shfl_xor(dpart, 16, 64);
  dpart += __shfl_xor(dpart, 32, 64);
  const float delta = dpart;
  const long si = ((long)b * a.H + h) * a.Tq + qc;
  const float mrow = P.stat_m[si], llrow = P.stat_ll[si];
  if (qok && grp == 0) P.delta[si] = delta;
  const float* amrow = ADDMASK ? P.add_mask + (mask_clip(P.mask_heads, b, a.H, h) * a.Tq + qc) * a.Tk : nullptr;
  DropMask dm;
  if (DROP) dm.init(P.drop_seed, P.drop_p, a.drop_off);
  const uint32_t erow = drop_row(b, a.H, h, a.Tq, a.Tk, qrow);

  f32x4 dq[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nblk = CAUSAL ? xb + 1 : (a.Tk + KB - 1) / KB;
  const float* kbase = P.k + (long)b * a.Tk * a.ldk + h * HD;
  const float* vbase = P.v + (long)b * a.Tk * a.ldv + h * HD;
  f32x4 rk[RV], rv[RV];
  float kvraw = 1.f;
  int kbn = 0;
  auto prefetch = [&](int kb) {
    blk_load<HD>(rk, kbase, a.ldk, kb, a.Tk);
    blk_load<HD>(rv, vbase, a.ldv, kb, a.Tk);
    kvraw = kv_load(P.key_valid, b, kb + (threadIdx.x & (KB - 1)), a.Tk);
    kbn = kb;
  };
  auto commit = [&](int buf) {
    store_rows<HD>(Ks[buf], rk);
    store_cols<HD>(Kt[buf], rk);
    store_rows<HD>(Vs[buf], rv);
    if (threadIdx.x < KB) Ka[buf][threadIdx.x] = key_add(kvraw, ADDMASK, kbn + threadIdx.x, a.Tk, plus2);
  };
  prefetch(0);
  commit(0);
  __syncthreads();

  auto step = [&](auto diag_c, int blk) {
    constexpr bool DIAG = decltype(diag_c)::value;
    const int kb = blk * KB, buf = NB == 2 ? (blk & 1) : 0;
    const bool more = blk + 1 < nblk;
    if (more) prefetch(kb + KB);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (DIAG && t > w) continue;
      f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = s_acc;
#pragma unroll
      for (int s = 0; s < NS; s += 4) {
        const f32x4 kv = row_frag<HD>(Ks[buf], 16 * t + qi, (NS * grp + s) >> 2);
        const f32x4 vv = row_frag<HD>(Vs[buf], 16 * t + qi, (NS * grp + s) >> 2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s_acc = mfma16(kv[j], qreg[s + j], s_acc);
          dp_acc = mfma16(vv[j], doreg[s + j], dp_acc);
        }
      }
      const int kl = 16 * t + 4 * grp;
      const f32x4 ad = ld4(&Ka[buf][kl]);
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t2;
        if (ADDMASK) t2 = to_log2(s_acc[r] + (kb + kl + r < a.Tk ? amrow[kb + kl + r] : 0.f) + ad[r]);
        else t2 = fmaf(s_acc[r], L2E, ad[r]);
        if (DIAG && t == w && 4 * grp + r > qi) t2 = -INFINITY;
        const float p = fast_exp2((t2 - mrow) - llrow);
        // dropout: dP = dP' * keep / (1 - p); delta = rowsum(dO * O) is unchanged
        const float dpk = DROP ? dm.apply(erow + (uint32_t)(kb + kl + r), dp_acc[r]) : dp_acc[r];
        ds[r] = p * (dpk - delta);
      }
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const f32x4 kt = col_frag(Kt[buf], 16 * d + qi, 4 * t + grp);
#pragma unroll
        for (int r = 0; r < 4; ++r) dq[d] = mfma16(kt[r], ds[r], dq[d]);
      }
    }
    if constexpr (NB == 2) {
      if (more) commit(buf ^ 1);
      __syncthreads();
    } else {  // one buffer: every wave done reading it before the next block is stored
      __syncthreads();
      if (more) {
        commit(0);
        __syncthreads();
      }
    }
  };
  for (int blk = 0; blk + (CAUSAL ? 1 : 0) < nblk; ++blk) step(FullStep{}, blk);
  if (CAUSAL) step(DiagStep{}, nblk - 1);

  if (qok) {
    float* dqp = P.dq + ((long)b * a.Tq + qrow) * a.ldq + h * HD + 4 * grp;
#pragma unroll
    for (int d = 0; d < ND; ++d) st4(dqp + 16 * d, dq[d] * P.dq_scale);
  }
  }  // job
}

// ------------------------------------------------------------------------------ backward: dK, dV
template <int HD, bool ADDMASK, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(const BwdArgs a) {
  constexpr int NS = HD / 4;
  constexpr int ND = HD / 16;
  constexpr int RV = Blk<HD>::RV;
  constexpr int NB = HD <= 64 ? 2 : 1;  // hd 128: one buffer per image (128 KB of LDS)
  __shared__ __attribute__((aligned(16))) float Qs[NB][QB * HD];
  __shared__ __attribute__((aligned(16))) float Ds[NB][QB * HD];
  __shared__ __attribute__((aligned(16))) float Qt[NB][HD * QB];
  __shared__ __attribute__((aligned(16))) float Dt[NB][HD * QB];
  __shared__ __attribute__((aligned(16))) float Sm[NB][QB], Sl[NB][QB], Sd[NB][QB];

  const TileId tid = xcd_tile();
  const sca_attn_bwd_problem& P = a.p[tid.z];
  const int b = tid.y / a.H, h = tid.y % a.H;
  const int nkb = (a.Tk + KB - 1) / KB;  // causal: key block x is paired with block nkb-1-x
  const int jobs = (CAUSAL && nkb - 1 - tid.x != tid.x) ? 2 : 1;
#pragma unroll 1
  for (int job = 0; job < jobs; ++job) {
  const int k0 = (job ? nkb - 1 - tid.x : tid.x) * KB;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int kj = lane & 15, grp = lane >> 4;
  const int krow = k0 + 16 * w + kj;
  const bool kok = krow < a.Tk;
  const float plus2 = (CAUSAL && a.plus_one) ? L2E : 0.0f;

  float kreg[NS], vreg[NS];
  {
    const int kc = min(krow, a.Tk - 1);
    const float* kp = P.k + ((long)b * a.Tk + kc) * a.ldk + h * HD + NS * grp;
    const float* vp = P.v + ((long)b * a.Tk + kc) * a.ldv + h * HD + NS * grp;
#pragma unroll
    for (int s = 0; s < NS; s += 4) {
      const f32x4 kv = ld4(kp + s), vv = ld4(vp + s);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        kreg[s + j] = kv[j];
        vreg[s + j] = vv[j];
      }
    }
  }
  const float kadd = key_add(kv_load(P.key_valid, b, krow, a.Tk), ADDMASK, krow, a.Tk, plus2);
  DropMask dm;
  if (DROP) dm.init(P.drop_seed, P.drop_p, a.drop_off);
  const uint32_t ekey = drop_row(b, a.H, h, a.Tq, a.Tk, 0) + (uint32_t)krow;

  f32x4 dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dk[d] = dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  // causal: the first query block is the diagonal one (QB == KB, Tq == Tk)
  const int qbeg = CAUSAL ? k0 : 0;
  const int nblk = (a.Tq - qbeg + QB - 1) / QB;
  const float* qbase = P.q + (long)b * a.Tq * a.ldq + h * HD;
  const float* dbase = P.dout + (long)b * a.Tq * a.ldo + h * HD;
  f32x4 rq[RV], rd[RV];
  float cm = 0.f, cl = 0.f, cd = 0.f;
  auto prefetch = [&](int qb) {
    blk_load<HD>(rq, qbase, a.ldq, qb, a.Tq);
    blk_load<HD>(rd, dbase, a.ldo, qb, a.Tq);
    if (threadIdx.x < QB) {
      const int q = qb + threadIdx.x;
      const long si = ((long)b * a.H + h) * a.Tq + min(q, a.Tq - 1);
      cm = P.stat_m[si];
      cl = P.stat_ll[si];
      cd = P.delta[si];
      if (q >= a.Tq) cm = INFINITY;  // rows past the end: p = exp2(-inf) = 0
    }
  };
  auto commit = [&](int buf) {
    store_rows<HD>(Qs[buf], rq);
    store_cols<HD>(Qt[buf], rq);
    store_rows<HD>(Ds[buf], rd);
    store_cols<HD>(Dt[buf], rd);
    if (threadIdx.x < QB) {
      Sm[buf][threadIdx.x] = cm;
      Sl[buf][threadIdx.x] = cl;
      Sd[buf][threadIdx.x] = cd;
    }
  };
  prefetch(qbeg);
  commit(0);
  __syncthreads();

  auto step = [&](auto diag_c, int blk) {
    constexpr bool DIAG = decltype(diag_c)::value;
    const int qb = qbeg + blk * QB, buf = NB == 2 ? (blk & 1) : 0;
    const bool more = blk + 1 < nblk;
    if (more) prefetch(qb + QB);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (DIAG && t < w) continue;  // wave-uniform: every query of the tile precedes every key
      f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = s_acc;
#pragma unroll
      for (int s = 0; s < NS; s += 4) {
        const f32x4 qv = row_frag<HD>(Qs[buf], 16 * t + kj, (NS * grp + s) >> 2);
        const f32x4 dv4 = row_frag<HD>(Ds[buf], 16 * t + kj, (NS * grp + s) >> 2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s_acc = mfma16(qv[j], kreg[s + j], s_acc);
          dp_acc = mfma16(dv4[j], vreg[s + j], dp_acc);
        }
      }
      // lane holds S[q = qb + 16t + 4grp + r][krow]
      const int ql = 16 * t + 4 * grp;
      const f32x4 sm = ld4(&Sm[buf][ql]), sl = ld4(&Sl[buf][ql]), sd = ld4(&Sd[buf][ql]);
      float p[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t2;
        if (ADDMASK) {
          const int q = min(qb + ql + r, a.Tq - 1);
          t2 = to_log2(s_acc[r] + (kok ? P.add_mask[(mask_clip(P.mask_heads, b, a.H, h) * a.Tq + q) * a.Tk + krow] : 0.f) +
                       kadd);
        } else {
          t2 = fmaf(s_acc[r], L2E, kadd);
        }
        if (DIAG && t == w && kj > 4 * grp + r) t2 = -INFINITY;
        p[r] = fast_exp2((t2 - sm[r]) - sl[r]);
        if (DROP) {  // dV uses the dropped probabilities; dP = dP' * keep / (1 - p)
          const uint32_t e = ekey + (uint32_t)(qb + ql + r) * (uint32_t)a.Tk;
          ds[r] = p[r] * (dm.apply(e, dp_acc[r]) - sd[r]);
          p[r] = dm.apply(e, p[r]);
        } else {
          ds[r] = p[r] * (dp_acc[r] - sd[r]);
        }
      }
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const f32x4 dt = col_frag(Dt[buf], 16 * d + kj, 4 * t + grp);
        const f32x4 qt = col_frag(Qt[buf], 16 * d + kj, 4 * t + grp);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dv[d] = mfma16(dt[r], p[r], dv[d]);
          dk[d] = mfma16(qt[r], ds[r], dk[d]);
        }
      }
    }
    if constexpr (NB == 2) {
      if (more) commit(buf ^ 1);
      __syncthreads();
    } else {  // one buffer: every wave done reading it before the next block is stored
      __syncthreads();
      if (more) {
        commit(0);
        __syncthreads();
      }
    }
  };
  int blk = 0;
  if (CAUSAL) step(DiagStep{}, blk++);
  for (; blk < nblk; ++blk) step(FullStep{}, blk);

  if (kok) {
    float* dkp = P.dk + ((long)b * a.Tk + krow) * a.ldk + h * HD + 4 * grp;
    float* dvp = P.dv + ((long)b * a.Tk + krow) * a.ldv + h * HD + 4 * grp;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      st4(dkp + 16 * d, dk[d]);
      st4(dvp + 16 * d, dv[d] * P.dv_scale);
    }
  }
  }  // job
}

// ------------------------------------------------------------------------------ backward: fused
// One workgroup = one (problem, clip, head) with every key and query of it (Tq, Tk <= 256,
// hd = 16, key-padding / causal masks): S, P, dP and dS are computed ONCE per score (the
// split kernels above recompute S and dP in both), dK / dV accumulate in registers, one
// launch, no atomics.
//   wave w owns the key tiles g = 4i + w (i < 4; 16 keys each, interleaved so that the
//   causal triangle gives every wave the same work): K / V rows and the K^T fragments of
//   them in registers;
//   per 64-query block (Q, dO, their transposes and the row stats staged in LDS; the next
//   block's loads are issued at the top and consumed — delta = rowsum(dO * O) included — only
//   when it is committed at the end, so their latency hides under the block's tiles), for
//   each (query tile t, own key tile g): S = Q K^T, dP = dO V^T (key on the lane),
//     P = exp2(S log2e + add - m - ll), dS = P (dP - delta), dV += dO^T P, dK += Q^T dS,
//     dS transposed through a wave-private LDS tile (padded rows: conflict-free), and
//     dQ_w += dS K over the wave's own keys;
//   the four waves' dQ partials are summed in fixed order through LDS (deterministic).
// One staging buffer (the next block is committed after the barrier that ends every wave's
// reads of the current one and before the barrier that opens the next): 38 KB of LDS, so
// the register file (186-226 VGPRs: two waves per SIMD) sets the occupancy, and co-running
// kernels keep LDS room on the CU.
constexpr int FB_TMAX = 256;
constexpr int FB_TS = 20;  // row stride of the 16x16 dS transposition tile (16 + 4 pad)
constexpr int FB_NB = 1, FB_OCC = 2;

template <bool CAUSAL, bool DROP>
#ifndef SCA_CRIT_PRIO
#define SCA_CRIT_PRIO 2
#endif
__global__ __launch_bounds__(256, FB_OCC) void attn_bwd_fused_kernel(const BwdArgs a) {
  if constexpr (SCA_CRIT_PRIO > 0) __builtin_amdgcn_s_setprio(SCA_CRIT_PRIO);  // gemm.hip: critical chain
  constexpr int HD = 16, NS = 4;
  __shared__ __attribute__((aligned(16))) float Qs[FB_NB][QB * HD];
  __shared__ __attribute__((aligned(16))) float Ds[FB_NB][QB * HD];
  __shared__ __attribute__((aligned(16))) float Qt[FB_NB][HD * QB];
  __shared__ __attribute__((aligned(16))) float Dt[FB_NB][HD * QB];
  __shared__ __attribute__((aligned(16))) float Sm[FB_NB][QB], Sl[FB_NB][QB], Sd[FB_NB][QB];
  __shared__ __attribute__((aligned(16))) float dSw[4][16 * FB_TS];
  __shared__ __attribute__((aligned(16))) float dQr[4][QB * HD];

  const TileId tid = xcd_tile();
  const sca_attn_bwd_problem& P = a.p[tid.z];
  const int b = tid.y / a.H, h = tid.y % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int kj = lane & 15, grp = lane >> 4;
  const float plus2 = (CAUSAL && a.plus_one) ? L2E : 0.0f;
  const int Tq = a.Tq, Tk = a.Tk;
  DropMask dm;
  if (DROP) dm.init(P.drop_seed, P.drop_p, a.drop_off);
  const uint32_t ebase = drop_row(b, a.H, h, Tq, Tk, 0);

  // own key tiles: K, V rows (B operands of S = Q K^T, dP = dO V^T) and K^T fragments
  // (A operand of dQ^T = K^T dS^T: lane (d = kj, grp) holds K[16g + 4grp + r][d]).  Wave w
  // owns tiles w, 15 - w, 7 - w, 8 + w: under the causal mask key tile g meets 16 - g query
  // tiles, so every wave gets 34 tile pairs (the interleaved g = 4i + w gave wave 0 40 and
  // wave 3 28, and the two workgroups of a CU put their waves 0 on the same SIMD)
  auto own = [&](int i) { return i == 0 ? w : i == 1 ? 15 - w : i == 2 ? 7 - w : 8 + w; };
  float kreg[4][NS], vreg[4][NS], kadd[4];
  f32x4 ktf[4];
  const float* kb = P.k + (long)b * Tk * a.ldk + h * HD;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int g = own(i);
    const int key = 16 * g + kj;
    const int kc = min(key, Tk - 1);
    const f32x4 kv = ld4(kb + (long)kc * a.ldk + NS * grp);
    const f32x4 vv = ld4(P.v + ((long)b * Tk + kc) * a.ldv + h * HD + NS * grp);
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      kreg[i][j] = kv[j];
      vreg[i][j] = vv[j];
      ktf[i][j] = kb[(long)min(16 * g + 4 * grp + j, Tk - 1) * a.ldk + kj];
    }
    kadd[i] = key_add(kv_load(P.key_valid, b, key, Tk), false, key, Tk, plus2);
  }
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dk[i] = dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nqb = (Tq + QB - 1) / QB;
  const float* qbase = P.q + (long)b * Tq * a.ldq + h * HD;
  const float* dbase = P.dout + (long)b * Tq * a.ldo + h * HD;
  const float* obase = P.o + (long)b * Tq * a.ldo + h * HD;
  // prefetch only issues the loads (in flight during the block's tiles); everything that
  // consumes them — delta = rowsum(dO * O), the past-the-end rows' stats — waits for commit
  f32x4 rq[1], rd[1], ro[1];
  float cm = 0.f, cl = 0.f;
  int qbn = 0;
  auto prefetch = [&](int q0) {
    blk_load<HD>(rq, qbase, a.ldq, q0, Tq);
    blk_load<HD>(rd, dbase, a.ldo, q0, Tq);
    blk_load<HD>(ro, obase, a.ldo, q0, Tq);
    if (threadIdx.x < QB) {
      const long si = ((long)b * a.H + h) * Tq + min(q0 + (int)threadIdx.x, Tq - 1);
      cm = P.stat_m[si];
      cl = P.stat_ll[si];
    }
    qbn = q0;
  };
  auto commit = [&](int buf) {
    // delta of row (threadIdx.x >> 2): 4 consecutive lanes hold its 16 dO*O products
    float cdel = rd[0][0] * ro[0][0] + rd[0][1] * ro[0][1] + rd[0][2] * ro[0][2] + rd[0][3] * ro[0][3];
    cdel += __shfl_xor(cdel, 1, 64);
    cdel += __shfl_xor(cdel, 2, 64);
    store_rows<HD>(Qs[buf], rq);
    store_cols<HD>(Qt[buf], rq);
    store_rows<HD>(Ds[buf], rd);
    store_cols<HD>(Dt[buf], rd);
    if (threadIdx.x < QB) {
      Sm[buf][threadIdx.x] = qbn + (int)threadIdx.x < Tq ? cm : INFINITY;  // past the end: p = 0
      Sl[buf][threadIdx.x] = cl;
    }
    if ((threadIdx.x & 3) == 0) {
      const int row = threadIdx.x >> 2;
      Sd[buf][row] = cdel;
      if (qbn + row < Tq) P.delta[((long)b * a.H + h) * Tq + qbn + row] = cdel;
    }
  };
  prefetch(0);
  commit(0);
  float* tw = dSw[w];

#pragma unroll 1
  for (int qb = 0; qb < nqb; ++qb) {
    const int buf = qb % FB_NB;
    __syncthreads();  // block qb staged; the previous block's dQ partials consumed
    if (qb + 1 < nqb) prefetch((qb + 1) * QB);  // in flight during this block
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f32x4 qv = row_frag<HD>(Qs[buf], 16 * t + kj, grp);
      const f32x4 dov = row_frag<HD>(Ds[buf], 16 * t + kj, grp);
      const f32x4 dtf = col_frag(Dt[buf], kj, 4 * t + grp);
      const f32x4 qtf = col_frag(Qt[buf], kj, 4 * t + grp);
      const int ql = 16 * t + 4 * grp;
      const f32x4 sm = ld4(&Sm[buf][ql]), sl = ld4(&Sl[buf][ql]), sd = ld4(&Sd[buf][ql]);
      f32x4 dq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int g = own(i);
        if (16 * g >= Tk) continue;                    // wave-uniform: no keys in this tile
        if (CAUSAL && g > 4 * qb + t) continue;        // every key after every query of the tile
        f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = s_acc;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s_acc = mfma16(qv[j], kreg[i][j], s_acc);
          dp_acc = mfma16(dov[j], vreg[i][j], dp_acc);
        }
        float p[4], ds[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float t2 = fmaf(s_acc[r], L2E, kadd[i]);
          if (CAUSAL && g == 4 * qb + t && kj > 4 * grp + r) t2 = -INFINITY;
          p[r] = fast_exp2((t2 - sm[r]) - sl[r]);
          if (DROP) {  // dV uses the dropped probabilities; dP = dP' * keep / (1 - p)
            const uint32_t e = ebase + (uint32_t)(qb * QB + ql + r) * (uint32_t)Tk + (uint32_t)(16 * g + kj);
            ds[r] = p[r] * (dm.apply(e, dp_acc[r]) - sd[r]);
            p[r] = dm.apply(e, p[r]);
          } else {
            ds[r] = p[r] * (dp_acc[r] - sd[r]);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dv[i] = mfma16(dtf[r], p[r], dv[i]);
          dk[i] = mfma16(qtf[r], ds[r], dk[i]);
        }
        // dS^T for dQ: lane (kj, grp) holds dS[q = 4grp + r][key kj]; the B operand wants
        // lane (q, grp') holding keys 4grp' .. 4grp' + 3 of row q
#pragma unroll
        for (int r = 0; r < 4; ++r) tw[(4 * grp + r) * FB_TS + kj] = ds[r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const f32x4 dsv = ld4(&tw[kj * FB_TS + 4 * grp]);
#pragma unroll
        for (int r = 0; r < 4; ++r) dq = mfma16(ktf[i][r], dsv[r], dq);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads done before the tile is rewritten
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      // partial dQ^T[d = 4grp + r][q = 16t + kj] over this wave's keys
      st4(&dQr[w][(16 * t + kj) * HD + 4 * grp], dq);
    }
    __syncthreads();  // all four partials of the block written
    const int qrow = qb * QB + 16 * w + kj;
    if (qrow < Tq) {
      const int e = (16 * w + kj) * HD + 4 * grp;
      const f32x4 s = ((ld4(&dQr[0][e]) + ld4(&dQr[1][e])) + ld4(&dQr[2][e])) + ld4(&dQr[3][e]);
      st4(P.dq + ((long)b * Tq + qrow) * a.ldq + h * HD + 4 * grp, s * P.dq_scale);
    }
    if (qb + 1 < nqb) commit((qb + 1) % FB_NB);
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int key = 16 * own(i) + kj;
    if (key < Tk) {
      st4(P.dk + ((long)b * Tk + key) * a.ldk + h * HD + 4 * grp, dk[i]);
      st4(P.dv + ((long)b * Tk + key) * a.ldv + h * HD + 4 * grp, dv[i] * P.dv_scale);
    }
  }
}

// ------------------------------------------------------------------------------ backward: fused, key blocks
// Fused backward for hd 32 at any length (config 5: T = 1024, d = 512): one workgroup =
// (problem, clip, head, 256-key block) — attn_bwd_fused_kernel's scheme (each wave owns
// 16-key tiles with K, V, K^T in registers; S, P, dP, dS once per score; dV, dK accumulated
// in registers; dS transposed through a wave-private LDS tile for dQ) with 8 waves of two
// key tiles each (g = 8i + w: at hd 32 four tiles per wave would not fit 256 registers),
// 32-query blocks, and dQ summed over the waves in fixed order and written as this key
// block's PARTIAL; attn_dq_reduce_kernel adds the key blocks' partials in order
// (deterministic, no atomics).  40 MFMAs per 16x16 score tile at hd 32 against the split
// kernels' 56.  Causal: a key block sees only the queries at or after its first key.
constexpr int KBLK = 256, QB2 = 32, KW = 8;

// transposed image [HD][32 queries]: 4 consecutive queries at float4 slot `slot` (0..7) of
// row d; rows 128 B apart, swizzled by (d >> 1) & 7 so that 16 rows d of one slot hit 16
// distinct 16-B bank groups
__device__ __forceinline__ f32x4 col_frag32(const float* img, int d, int slot) {
  return ld4(img + d * QB2 + 4 * (slot ^ ((d >> 1) & 7)));
}

template <bool CAUSAL, bool DROP>
__global__ __launch_bounds__(64 * KW, 1) void attn_bwd_kblk_kernel(const BwdArgs a) {
  constexpr int HD = 32, NS = 8, ND = 2, TPW = KBLK / 16 / KW;
  __shared__ __attribute__((aligned(16))) float Qs[2][QB2 * HD];
  __shared__ __attribute__((aligned(16))) float Ds[2][QB2 * HD];
  __shared__ __attribute__((aligned(16))) float Qt[2][HD * QB2];
  __shared__ __attribute__((aligned(16))) float Dt[2][HD * QB2];
  __shared__ __attribute__((aligned(16))) float Sm[2][QB2], Sl[2][QB2], Sd[2][QB2];
  __shared__ __attribute__((aligned(16))) float dSw[KW][KBLK / 16 / KW][16 * FB_TS];
  __shared__ __attribute__((aligned(16))) float dQr[KW][QB2 * HD];

  // Dispatch order = blockIdx order (no XCD remap): x = (problem, clip, head), y = key block,
  // so with the causal mask the heaviest workgroups (key block 0 sees every query) are
  // dispatched first and the light ones fill in behind them (longest-first list scheduling;
  // an interleaved order left the CUs that drew key block 0 running long after the rest).
  // Consecutive workgroups still cycle over the 8 XCDs.
  const int bh = blockIdx.x % (a.B * a.H), pz = blockIdx.x / (a.B * a.H);
  const TileId tid{(int)blockIdx.y, bh, pz};
  const sca_attn_bwd_problem& P = a.p[tid.z];
  const int b = tid.y / a.H, h = tid.y % a.H;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int kj = lane & 15, grp = lane >> 4;
  const float plus2 = (CAUSAL && a.plus_one) ? L2E : 0.0f;
  const int Tq = a.Tq, Tk = a.Tk;
  const int k0 = tid.x * KBLK;
  DropMask dm;
  if (DROP) dm.init(P.drop_seed, P.drop_p, a.drop_off);
  const uint32_t ebase = drop_row(b, a.H, h, Tq, Tk, 0);

  // own key tiles (local to the block) w and 15 - w: under the causal mask local tile l meets
  // 16 - l of the diagonal region's 16 query tiles, so every wave gets 17 there (w and 8 + w
  // gave wave 0 24 and wave 7 10; the last key block is all diagonal region).  K, V rows (lane
  // (kj, grp): d = 8 grp .. 8 grp + 7) and the K^T fragments of both 16-wide d blocks (lane
  // (d = 16 dd + kj, grp): K[16g + 4grp + r][d])
  static_assert(TPW == 2, "two key tiles per wave");
  auto own = [&](int i) { return i == 0 ? w : KBLK / 16 - 1 - w; };
  float kreg[TPW][NS], vreg[TPW][NS], kadd[TPW];
  f32x4 ktf[TPW][ND];
  const float* kb = P.k + (long)b * Tk * a.ldk + h * HD;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int key = k0 + 16 * own(i) + kj;
    const int kc = min(key, Tk - 1);
#pragma unroll
    for (int s = 0; s < NS; s += 4) {
      const f32x4 kv = ld4(kb + (long)kc * a.ldk + NS * grp + s);
      const f32x4 vv = ld4(P.v + ((long)b * Tk + kc) * a.ldv + h * HD + NS * grp + s);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        kreg[i][s + j] = kv[j];
        vreg[i][s + j] = vv[j];
      }
    }
#pragma unroll
    for (int dd = 0; dd < ND; ++dd)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        ktf[i][dd][j] = kb[(long)min(k0 + 16 * own(i) + 4 * grp + j, Tk - 1) * a.ldk + 16 * dd + kj];
    kadd[i] = key_add(kv_load(P.key_valid, b, key, Tk), false, key, Tk, plus2);
  }
  f32x4 dk[TPW][ND], dv[TPW][ND];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) dk[i][dd] = dv[i][dd] = f32x4{0.f, 0.f, 0.f, 0.f};

  // query blocks: causal from the block holding this key block's first key (k0 % 32 == 0)
  const int qbeg = CAUSAL ? k0 : 0;
  const int nqb = qbeg < Tq ? (Tq - qbeg + QB2 - 1) / QB2 : 0;
  const float* qbase = P.q + (long)b * Tq * a.ldq + h * HD;
  const float* dbase = P.dout + (long)b * Tq * a.ldo + h * HD;
  const float* obase = P.o + (long)b * Tq * a.ldo + h * HD;
  // staging (waves 0-3): thread e owns row e / 8, float4 column (e % 8) of the 32 x 32 block
  const bool stager = threadIdx.x < 256;
  const int srow = (threadIdx.x & 255) >> 3, sc = 4 * (threadIdx.x & 7);
  f32x4 rq, rd;
  float cm = 0.f, cl = 0.f, cdel = 0.f;
  int qbn = 0;
  auto prefetch = [&](int q0) {
    if (!stager) return;
    const int q = min(q0 + srow, Tq - 1);
    rq = ld4(qbase + (long)q * a.ldq + sc);
    rd = ld4(dbase + (long)q * a.ldo + sc);
    const f32x4 ro = ld4(obase + (long)q * a.ldo + sc);
    // delta of row srow: 8 consecutive lanes hold its 32 dO*O products
    float dp = rd[0] * ro[0] + rd[1] * ro[1] + rd[2] * ro[2] + rd[3] * ro[3];
    dp += __shfl_xor(dp, 1, 64);
    dp += __shfl_xor(dp, 2, 64);
    dp += __shfl_xor(dp, 4, 64);
    cdel = dp;
    if (threadIdx.x < QB2) {
      const int qq = q0 + threadIdx.x;
      const long si = ((long)b * a.H + h) * Tq + min(qq, Tq - 1);
      cm = P.stat_m[si];
      cl = P.stat_ll[si];
      if (qq >= Tq) cm = INFINITY;  // rows past the end: p = exp2(-inf) = 0
    }
    qbn = q0;
  };
  auto commit = [&](int buf) {
    if (!stager) return;
    st4(Qs[buf] + srow * HD + 4 * ((sc >> 2) ^ row_swz<HD>(srow)), rq);
    st4(Ds[buf] + srow * HD + 4 * ((sc >> 2) ^ row_swz<HD>(srow)), rd);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = sc + j;
      const int o = d * QB2 + 4 * ((srow >> 2) ^ ((d >> 1) & 7)) + (srow & 3);
      Qt[buf][o] = rq[j];
      Dt[buf][o] = rd[j];
    }
    if (threadIdx.x < QB2) {
      Sm[buf][threadIdx.x] = cm;
      Sl[buf][threadIdx.x] = cl;
    }
    if ((threadIdx.x & 7) == 0) {
      Sd[buf][srow] = cdel;
      if (k0 == 0 && qbn + srow < Tq) P.delta[((long)b * a.H + h) * Tq + qbn + srow] = cdel;
    }
  };
  if (nqb > 0) {
    prefetch(qbeg);
    commit(0);
  }
  float* part = P.dq_part + ((long)tid.x * a.B + b) * Tq * (a.H * HD) + h * HD;

  // one 16-query tile against the wave's key tiles; GEN: the general form (key tiles past Tk
  // skipped, causal tiles after the query tile skipped, the diagonal one masked) — the
  // blocks where every key tile is whole and (causal) before every query run the
  // branch-free form, whose two key tiles' MFMA chains interleave
  auto qtile = [&](auto gen_c, int buf, int q0, int t) {
    constexpr bool GEN = decltype(gen_c)::value;
    const int qt = (q0 >> 4) + t;  // global 16-query tile index
    f32x4 qv[2], dov[2], dtf[ND], qtf[ND];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      qv[s2] = row_frag<HD>(Qs[buf], 16 * t + kj, 2 * grp + s2);
      dov[s2] = row_frag<HD>(Ds[buf], 16 * t + kj, 2 * grp + s2);
    }
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
      dtf[dd] = col_frag32(Dt[buf], 16 * dd + kj, 4 * t + grp);
      qtf[dd] = col_frag32(Qt[buf], 16 * dd + kj, 4 * t + grp);
    }
    const int ql = 16 * t + 4 * grp;
    const f32x4 sm = ld4(&Sm[buf][ql]), sl = ld4(&Sl[buf][ql]), sd = ld4(&Sd[buf][ql]);
    f32x4 dq[ND];
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) dq[dd] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int g = (k0 >> 4) + own(i);  // global 16-key tile index
      if (GEN && 16 * g >= Tk) continue;      // wave-uniform: no keys in this tile
      if (GEN && CAUSAL && g > qt) continue;  // every key after every query of the tile
      f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = s_acc;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s_acc = mfma16(qv[s2][j], kreg[i][4 * s2 + j], s_acc);
          dp_acc = mfma16(dov[s2][j], vreg[i][4 * s2 + j], dp_acc);
        }
      float p[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t2 = fmaf(s_acc[r], L2E, kadd[i]);
        if (GEN && CAUSAL && g == qt && kj > 4 * grp + r) t2 = -INFINITY;
        p[r] = fast_exp2((t2 - sm[r]) - sl[r]);
        if (DROP) {  // dV uses the dropped probabilities; dP = dP' * keep / (1 - p)
          const uint32_t e = ebase + (uint32_t)(q0 + ql + r) * (uint32_t)Tk + (uint32_t)(16 * g + kj);
          ds[r] = p[r] * (dm.apply(e, dp_acc[r]) - sd[r]);
          p[r] = dm.apply(e, p[r]);
        } else {
          ds[r] = p[r] * (dp_acc[r] - sd[r]);
        }
      }
#pragma unroll
      for (int dd = 0; dd < ND; ++dd)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dv[i][dd] = mfma16(dtf[dd][r], p[r], dv[i][dd]);
          dk[i][dd] = mfma16(qtf[dd][r], ds[r], dk[i][dd]);
        }
      float* tw = dSw[w][i];
#pragma unroll
      for (int r = 0; r < 4; ++r) tw[(4 * grp + r) * FB_TS + kj] = ds[r];
    }
    // dS^T through the wave-private tiles (one per key tile): one wave barrier for both
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int g = (k0 >> 4) + own(i);
      if (GEN && 16 * g >= Tk) continue;
      if (GEN && CAUSAL && g > qt) continue;
      const f32x4 dsv = ld4(&dSw[w][i][kj * FB_TS + 4 * grp]);
#pragma unroll
      for (int dd = 0; dd < ND; ++dd)
#pragma unroll
        for (int r = 0; r < 4; ++r) dq[dd] = mfma16(ktf[i][dd][r], dsv[r], dq[dd]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads done before the tiles are rewritten
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // partial dQ^T[d = 16 dd + 4grp + r][q = 16t + kj] over this wave's keys
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) st4(&dQr[w][(16 * t + kj) * HD + 16 * dd + 4 * grp], dq[dd]);
  };

#pragma unroll 1
  for (int qb = 0; qb < nqb; ++qb) {
    const int buf = qb & 1;
    const int q0 = qbeg + qb * QB2;
    __syncthreads();  // block qb staged; the previous block's dQ partials consumed
    if (qb + 1 < nqb) prefetch(q0 + QB2);  // in flight during this block
    const bool full = k0 + KBLK <= Tk && (!CAUSAL || (q0 >> 4) >= (k0 >> 4) + KBLK / 16 - 1);
    if (full) {
#pragma unroll
      for (int t = 0; t < QB2 / 16; ++t) qtile(std::false_type{}, buf, q0, t);
    } else {
#pragma unroll
      for (int t = 0; t < QB2 / 16; ++t) qtile(std::true_type{}, buf, q0, t);
    }
    __syncthreads();  // all partials of the block written
    if (stager) {
      const int e = srow * HD + sc;
      f32x4 sum = ld4(&dQr[0][e]);
#pragma unroll
      for (int u = 1; u < KW; ++u) sum += ld4(&dQr[u][e]);
      if (q0 + srow < Tq) st4(part + (long)(q0 + srow) * (a.H * HD) + sc, sum);
    }
    if (qb + 1 < nqb) commit(buf ^ 1);
  }

#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int key = k0 + 16 * own(i) + kj;
    if (key < Tk) {
#pragma unroll
      for (int dd = 0; dd < ND; ++dd) {
        st4(P.dk + ((long)b * Tk + key) * a.ldk + h * HD + 16 * dd + 4 * grp, dk[i][dd]);
        st4(P.dv + ((long)b * Tk + key) * a.ldv + h * HD + 16 * dd + 4 * grp, dv[i][dd] * P.dv_scale);
      }
    }
  }
}

// dq = dq_scale * (sum over the key blocks' partials, in order); causal rows only have
// partials from the key blocks at or before them
__global__ __launch_bounds__(256) void attn_dq_reduce_kernel(const BwdArgs a) {
  const sca_attn_bwd_problem& P = a.p[blockIdx.z];
  const int d = a.H * 32, c4 = d / 4;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long rows = (long)a.B * a.Tq;
  if (e >= rows * c4) return;
  const long row = e / c4;
  const int c = (int)(e % c4) * 4;
  const int q = (int)(row % a.Tq);
  const int nkb = (a.Tk + KBLK - 1) / KBLK;
  const int n = a.causal ? min(nkb, q / KBLK + 1) : nkb;
  const long stride = rows * d;
  f32x4 s = ld4(P.dq_part + row * d + c);
  for (int kb = 1; kb < n; ++kb) s += ld4(P.dq_part + kb * stride + row * d + c);
  st4(P.dq + row * a.ldq + c, s * P.dq_scale);
}

template <typename Args>
int check_common(const Args& a, int hd, int nprob) {
  if (nprob < 1 || nprob > SCA_ATTN_MAX_PROBLEMS || a.B < 1 || a.H < 1 || a.Tq < 1 || a.Tk < 1) return 1;
  if (hd != 16 && hd != 32 && hd != 64 && hd != 128) return 2;
  if ((a.ldq & 3) || (a.ldk & 3) || (a.ldv & 3) || (a.ldo & 3)) return 3;
  if (a.ldq < a.H * hd || a.ldk < a.H * hd || a.ldv < a.H * hd || a.ldo < a.H * hd) return 3;
  if (a.causal && a.Tq != a.Tk) return 4;
  return 0;
}

template <int HD, bool AM, bool DR>
void launch_fwd(const FwdArgs& a, dim3 grid, hipStream_t st) {
  if (a.causal) hipLaunchKernelGGL((attn_fwd_kernel<HD, AM, true, DR>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((attn_fwd_kernel<HD, AM, false, DR>), grid, dim3(256), 0, st, a);
}

template <int HD, bool AM>
void launch_fwd(const FwdArgs& a, dim3 grid, hipStream_t st, bool drop) {
  if (drop) launch_fwd<HD, AM, true>(a, grid, st);
  else launch_fwd<HD, AM, false>(a, grid, st);
}

bool g_bwd_fused = true;

template <int HD, bool AM, bool DR>
void launch_bwd(const BwdArgs& a, dim3 gq, dim3 gk, hipStream_t st) {
  if (HD == 16 && !AM && g_bwd_fused && a.Tq <= FB_TMAX && a.Tk <= FB_TMAX) {
    const dim3 g(1, a.B * a.H, gq.z);
    if (a.causal) hipLaunchKernelGGL((attn_bwd_fused_kernel<true, DR>), g, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_bwd_fused_kernel<false, DR>), g, dim3(256), 0, st, a);
    return;
  }
  if (HD == 32 && !AM && g_bwd_fused && a.p[0].dq_part) {
    const dim3 g(a.B * a.H * gq.z, (a.Tk + KBLK - 1) / KBLK, 1);
    if (a.causal) hipLaunchKernelGGL((attn_bwd_kblk_kernel<true, DR>), g, dim3(64 * KW), 0, st, a);
    else hipLaunchKernelGGL((attn_bwd_kblk_kernel<false, DR>), g, dim3(64 * KW), 0, st, a);
    const long n4 = (long)a.B * a.Tq * a.H * 32 / 4;
    hipLaunchKernelGGL(attn_dq_reduce_kernel, dim3((unsigned)((n4 + 255) / 256), 1, gq.z), dim3(256), 0, st, a);
    return;
  }
  if (a.causal) {
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, AM, true, DR>), gq, dim3(256), 0, st, a);
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, AM, true, DR>), gk, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, AM, false, DR>), gq, dim3(256), 0, st, a);
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, AM, false, DR>), gk, dim3(256), 0, st, a);
  }
}

template <int HD, bool AM>
void launch_bwd(const BwdArgs& a, dim3 gq, dim3 gk, hipStream_t st, bool drop) {
  if (drop) launch_bwd<HD, AM, true>(a, gq, gk, st);
  else launch_bwd<HD, AM, false>(a, gq, gk, st);
}

}  // namespace

extern "C" void sca_set_error(const char* msg);

// floats of dq_part per problem the fused hd-32 backward needs (0: that path does not apply)
extern "C" long sca_attn_bwd_workspace(int B, int H, int Tq, int Tk, int hd) {
  if (hd != 32 || B < 1 || H < 1 || Tq < 1 || Tk < 1) return 0;
  return (long)((Tk + KBLK - 1) / KBLK) * B * Tq * H * hd;
}

extern "C" int sca_attn_bwd_fused(int enable) {
  g_bwd_fused = enable != 0;
  return SCA_OK;
}

extern "C" int sca_attn_fwd(int nprob, const sca_attn_fwd_problem* probs, int B, int H, int Tq, int Tk, int hd,
                            int ldq, int ldk, int ldv, int ldo, int causal, int plus_one, void* stream) {
  FwdArgs a;
  a.B = B; a.H = H; a.Tq = Tq; a.Tk = Tk; a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
  a.causal = causal; a.plus_one = plus_one;
  a.drop_off = sca_drop_offset_ptr();
  const int err = check_common(a, hd, nprob);
  if (err) {
    sca_set_error(err == 2 ? "sca_attn_fwd: head_dim must be 16, 32, 64 or 128"
                           : "sca_attn_fwd: bad shape / leading dimension / causal with Tq != Tk");
    return SCA_ERR_ARG;
  }
  bool am = false, drop = false;
  for (int i = 0; i < nprob; ++i) {
    a.p[i] = probs[i];
    if (!probs[i].q || !probs[i].k || !probs[i].v || !probs[i].o || !probs[i].stat_m || !probs[i].stat_ll) {
      sca_set_error("sca_attn_fwd: null pointer");
      return SCA_ERR_ARG;
    }
    if ((probs[i].add_mask != nullptr) != (probs[0].add_mask != nullptr)) {
      sca_set_error("sca_attn_fwd: all problems must agree on add_mask");
      return SCA_ERR_ARG;
    }
    am = probs[i].add_mask != nullptr;
    if (probs[i].mask_heads < 0 || (probs[i].mask_heads > 1 && probs[i].mask_heads != H)) {
      sca_set_error("sca_attn_fwd: mask_heads must be 0, 1 or H");
      return SCA_ERR_ARG;
    }
    if (!(probs[i].drop_p >= 0.f && probs[i].drop_p < 1.f)) {
      sca_set_error("sca_attn_fwd: drop_p must be in [0, 1)");
      return SCA_ERR_ARG;
    }
    drop = drop || probs[i].drop_p > 0.f;
  }
  const int nqb = (Tq + QB - 1) / QB;  // causal: two paired query blocks per workgroup
  dim3 grid(causal ? (nqb + 1) / 2 : nqb, B * H, nprob);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hd == 16) am ? launch_fwd<16, true>(a, grid, st, drop) : launch_fwd<16, false>(a, grid, st, drop);
  else if (hd == 32) am ? launch_fwd<32, true>(a, grid, st, drop) : launch_fwd<32, false>(a, grid, st, drop);
  else if (hd == 64) am ? launch_fwd<64, true>(a, grid, st, drop) : launch_fwd<64, false>(a, grid, st, drop);
  else am ? launch_fwd<128, true>(a, grid, st, drop) : launch_fwd<128, false>(a, grid, st, drop);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_attn_fwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_attn_bwd(int nprob, const sca_attn_bwd_problem* probs, int B, int H, int Tq, int Tk, int hd,
                            int ldq, int ldk, int ldv, int ldo, int causal, int plus_one, void* stream) {
  BwdArgs a;
  a.B = B; a.H = H; a.Tq = Tq; a.Tk = Tk; a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
  a.causal = causal; a.plus_one = plus_one;
  a.drop_off = sca_drop_offset_ptr();
  const int err = check_common(a, hd, nprob);
  if (err) {
    sca_set_error(err == 2 ? "sca_attn_bwd: head_dim must be 16, 32, 64 or 128"
                           : "sca_attn_bwd: bad shape / leading dimension / causal with Tq != Tk");
    return SCA_ERR_ARG;
  }
  bool am = false, drop = false;
  for (int i = 0; i < nprob; ++i) {
    const sca_attn_bwd_problem& p = probs[i];
    if (!p.q || !p.k || !p.v || !p.o || !p.dout || !p.stat_m || !p.stat_ll || !p.dq || !p.dk || !p.dv || !p.delta) {
      sca_set_error("sca_attn_bwd: null pointer");
      return SCA_ERR_ARG;
    }
    if ((p.add_mask != nullptr) != (probs[0].add_mask != nullptr)) {
      sca_set_error("sca_attn_bwd: all problems must agree on add_mask");
      return SCA_ERR_ARG;
    }
    am = p.add_mask != nullptr;
    if (p.mask_heads < 0 || (p.mask_heads > 1 && p.mask_heads != H)) {
      sca_set_error("sca_attn_bwd: mask_heads must be 0, 1 or H");
      return SCA_ERR_ARG;
    }
    if ((p.dq_part != nullptr) != (probs[0].dq_part != nullptr)) {
      sca_set_error("sca_attn_bwd: all problems must agree on dq_part");
      return SCA_ERR_ARG;
    }
    if (!(p.drop_p >= 0.f && p.drop_p < 1.f)) {
      sca_set_error("sca_attn_bwd: drop_p must be in [0, 1)");
      return SCA_ERR_ARG;
    }
    drop = drop || p.drop_p > 0.f;
    a.p[i] = p;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nqb = (Tq + QB - 1) / QB, nkb = (Tk + KB - 1) / KB;  // causal: paired blocks
  dim3 gq(causal ? (nqb + 1) / 2 : nqb, B * H, nprob), gk(causal ? (nkb + 1) / 2 : nkb, B * H, nprob);
  if (hd == 16) am ? launch_bwd<16, true>(a, gq, gk, st, drop) : launch_bwd<16, false>(a, gq, gk, st, drop);
  else if (hd == 32) am ? launch_bwd<32, true>(a, gq, gk, st, drop) : launch_bwd<32, false>(a, gq, gk, st, drop);
  else if (hd == 64) am ? launch_bwd<64, true>(a, gq, gk, st, drop) : launch_bwd<64, false>(a, gq, gk, st, drop);
  else am ? launch_bwd<128, true>(a, gq, gk, st, drop) : launch_bwd<128, false>(a, gq, gk, st, drop);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_attn_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}
