// Fused masked attention (forward + backward) on the gfx950 f32 matrix cores
// (v_mfma_f32_16x16x4_f32), for the three SCAttenNet attention operators:
//   SelfAttention        model/attention.py:46-76   (key-padding mask)
//   SelfCausalAttention  model/attention.py:148-182 (tril -> -inf, then +causal mask)
//   CrossAttention       model/attention.py:97-128  (key-padding mask, Tq may != Tk)
//
// Layout in HBM: activations stay (B, T, H*hd) row-major exactly as the projections write
// them (no head transposes: head h is the column slice h*hd .. h*hd+hd-1).
//
// Mask encoding (branch-free): every key j of a block gets a pair (mul_j, add_j) in LDS and
// the masked score is fma(s, mul_j, add_j):
//   valid key            (1, plus)      plus = 1.0 for the causal mask (utils.py:24-27), else 0
//   padded key           (0, finfo.min) (utils.py:3-12; s*0 + min == min, as s + min rounds)
//   key >= Tk            (0, -inf)      (not part of the row at all)
// With an explicit additive (B,1,Tq,Tk) mask (general path) every key is (1, 0) and the
// mask value is added.  Causal keys above the diagonal are set to -inf (attention.py:165-169)
// only in the diagonal blocks (wave-uniform branch).
//
// Forward: one workgroup = (problem g, clip b, head h, 64 queries); 4 waves x 16 queries.
// K/V stream through LDS in 64-key blocks (register-prefetched one block ahead, one barrier
// per block).  Scores are computed SWAPPED (S^T = K Q^T) so a lane owns one query column and
// 4 keys per 16x16 tile: the row max / row sum need two xor-shuffles, and the S^T
// accumulator registers are already the B operand of O^T += V^T P^T — P never leaves
// registers.  Online softmax.  Saves m (row max) and ll = log(row sum) per row: a fully
// padded row (all finfo.min) then recomputes to exactly uniform weights in the backward.
//
// Backward: two kernels, no atomics (deterministic):
//   dq kernel   (query-block major): delta = rowsum(dO*O); S^T, dP^T recomputed;
//               dS = P (dP - delta); dQ^T += K^T dS^T.
//   dkdv kernel (key-block major):   S, dP recomputed with the key on the lane;
//               dV^T += dO^T P ; dK^T += Q^T dS.
#include "common.h"
#include "../../include/scatten.h"

namespace {

constexpr int QB = 64;  // queries per workgroup (16 per wave)
constexpr int KB = 64;  // keys per LDS block
constexpr int TP = 4;   // LDS padding (floats)

struct FwdArgs {
  sca_attn_fwd_problem p[SCA_ATTN_MAX_PROBLEMS];
  int B, H, Tq, Tk, ldq, ldk, ldv, ldo, causal, plus_one;
};

struct BwdArgs {
  sca_attn_bwd_problem p[SCA_ATTN_MAX_PROBLEMS];
  int B, H, Tq, Tk, ldq, ldk, ldv, ldo, causal, plus_one;
};

// (mul, add) of key j (see header comment).  The validity word is loaded separately
// (kv_load) so that the compare happens at LDS-commit time: a compare right after the load
// would make the wave wait for the whole K/V prefetch that was issued with it.
__device__ __forceinline__ float kv_load(const float* key_valid, int b, int j, int Tk) {
  return key_valid ? key_valid[(long)b * Tk + min(j, Tk - 1)] : 1.f;
}

__device__ __forceinline__ void key_coef(float kv, bool add_mask, int j, int Tk, float plus, float& mul,
                                         float& add) {
  if (j >= Tk) {
    mul = 0.f;
    add = -INFINITY;
  } else if (add_mask) {
    mul = 1.f;
    add = 0.f;
  } else if (kv == 0.f) {
    mul = 0.f;
    add = SCA_FMIN;
  } else {
    mul = 1.f;
    add = plus;
  }
}

// Row block of HD floats per row, 64 rows: each thread owns RV = HD/16 float4 of it.
template <int HD>
struct Blk {
  static constexpr int V4 = HD / 4;          // float4 per row
  static constexpr int RV = 64 * V4 / 256;   // float4 per thread
};

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

// row image [64][HD+TP] and/or transposed image [HD][64+TP]
template <int HD>
__device__ __forceinline__ void blk_store(float* rowimg, float* colimg, const f32x4* r) {
#pragma unroll
  for (int i = 0; i < Blk<HD>::RV; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int row = e / Blk<HD>::V4, c = (e % Blk<HD>::V4) * 4;
    if (rowimg) st4(rowimg + row * (HD + TP) + c, r[i]);
    if (colimg) {
#pragma unroll
      for (int j = 0; j < 4; ++j) colimg[(c + j) * (64 + TP) + row] = r[i][j];
    }
  }
}

// ------------------------------------------------------------------------------ forward
template <int HD, bool ADDMASK>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const FwdArgs a) {
  constexpr int NS = HD / 4;   // MFMA k-steps over the head dim
  constexpr int ND = HD / 16;  // 16-wide output d-blocks
  constexpr int RV = Blk<HD>::RV;
  __shared__ __attribute__((aligned(16))) float Ks[2][KB * (HD + TP)];
  __shared__ __attribute__((aligned(16))) float Vt[2][HD * (KB + TP)];
  __shared__ __attribute__((aligned(16))) float Km[2][KB], Ka[2][KB];

  const sca_attn_fwd_problem& P = a.p[blockIdx.z];
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int q0 = blockIdx.x * QB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = lane & 15, grp = lane >> 4;
  const int qrow = q0 + 16 * w + qi;
  const float plus = (a.causal && a.plus_one) ? 1.0f : 0.0f;

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
  const float* amrow = ADDMASK ? P.add_mask + ((long)b * a.Tq + min(qrow, a.Tq - 1)) * a.Tk : nullptr;

  f32x4 o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  const int kend = a.causal ? min(a.Tk, q0 + QB) : a.Tk;
  const int nblk = (kend + KB - 1) / KB;
  const int wave_qmin = q0 + 16 * w, wave_qmax = wave_qmin + 15;
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
    blk_store<HD>(Ks[buf], nullptr, rk);
    blk_store<HD>(nullptr, Vt[buf], rv);
    if (threadIdx.x < KB) {
      float cm, ca;
      key_coef(kvraw, ADDMASK, kbn + threadIdx.x, a.Tk, plus, cm, ca);
      Km[buf][threadIdx.x] = cm;
      Ka[buf][threadIdx.x] = ca;
    }
  };
  prefetch(0);
  commit(0);
  __syncthreads();

  for (int blk = 0; blk < nblk; ++blk) {
    const int kb = blk * KB, buf = blk & 1;

    float sv[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bool live = !a.causal || (kb + 16 * t <= wave_qmax);
      if (!live) {
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[t][r] = -INFINITY;
        continue;
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* kr = Ks[buf] + (16 * t + qi) * (HD + TP) + NS * grp;
#pragma unroll
      for (int s = 0; s < NS; s += 4) {
        const f32x4 kv = ld4(kr + s);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = mfma16(kv[j], qreg[s + j], acc);
      }
      const int kl = 16 * t + 4 * grp;
      const f32x4 mm = ld4(&Km[buf][kl]), aa = ld4(&Ka[buf][kl]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = fmaf(acc[r], mm[r], aa[r]);
        if (ADDMASK && kb + kl + r < a.Tk) s += amrow[kb + kl + r];
        sv[t][r] = s;
      }
      if (a.causal && kb + 16 * t + 15 > wave_qmin) {  // diagonal sub-tile
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kb + kl + r > qrow) sv[t][r] = -INFINITY;
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
    const float alpha = exp2f((m_run - m_new) * SCA_LOG2E);
    m_run = m_new;
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2f((sv[t][r] - m_new) * SCA_LOG2E);
        sv[t][r] = p;
        psum += p;
      }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int d = 0; d < ND; ++d) o[d] *= alpha;
    if (blk + 1 < nblk) prefetch(kb + KB);  // in flight during the P.V MFMAs and the barrier
    // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (a.causal && kb + 16 * t > wave_qmax) continue;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const f32x4 vv = ld4(Vt[buf] + (16 * d + qi) * (KB + TP) + 16 * t + 4 * grp);
#pragma unroll
        for (int r = 0; r < 4; ++r) o[d] = mfma16(vv[r], sv[t][r], o[d]);
      }
    }
    if (blk + 1 < nblk) commit(buf ^ 1);
    __syncthreads();
  }
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
      P.stat_ll[si] = logf(l_tot);
    }
  }
}

// ------------------------------------------------------------------------------ backward: dQ
template <int HD, bool ADDMASK>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const BwdArgs a) {
  constexpr int NS = HD / 4;
  constexpr int ND = HD / 16;
  constexpr int RV = Blk<HD>::RV;
  __shared__ __attribute__((aligned(16))) float Ks[2][KB * (HD + TP)];
  __shared__ __attribute__((aligned(16))) float Vs[2][KB * (HD + TP)];
  __shared__ __attribute__((aligned(16))) float Kt[2][HD * (KB + TP)];
  __shared__ __attribute__((aligned(16))) float Km[2][KB], Ka[2][KB];

  const sca_attn_bwd_problem& P = a.p[blockIdx.z];
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int q0 = blockIdx.x * QB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = lane & 15, grp = lane >> 4;
  const int qrow = q0 + 16 * w + qi;
  const bool qok = qrow < a.Tq;
  const int qc = min(qrow, a.Tq - 1);
  const float plus = (a.causal && a.plus_one) ? 1.0f : 0.0f;

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
  const float* amrow = ADDMASK ? P.add_mask + ((long)b * a.Tq + qc) * a.Tk : nullptr;

  f32x4 dq[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kend = a.causal ? min(a.Tk, q0 + QB) : a.Tk;
  const int nblk = (kend + KB - 1) / KB;
  const int wave_qmin = q0 + 16 * w, wave_qmax = wave_qmin + 15;
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
    blk_store<HD>(Ks[buf], Kt[buf], rk);
    blk_store<HD>(Vs[buf], nullptr, rv);
    if (threadIdx.x < KB) {
      float cm, ca;
      key_coef(kvraw, ADDMASK, kbn + threadIdx.x, a.Tk, plus, cm, ca);
      Km[buf][threadIdx.x] = cm;
      Ka[buf][threadIdx.x] = ca;
    }
  };
  prefetch(0);
  commit(0);
  __syncthreads();

  for (int blk = 0; blk < nblk; ++blk) {
    const int kb = blk * KB, buf = blk & 1;
    if (blk + 1 < nblk) prefetch(kb + KB);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (a.causal && kb + 16 * t > wave_qmax) continue;
      f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = s_acc;
      const float* kr = Ks[buf] + (16 * t + qi) * (HD + TP) + NS * grp;
      const float* vr = Vs[buf] + (16 * t + qi) * (HD + TP) + NS * grp;
#pragma unroll
      for (int s = 0; s < NS; s += 4) {
        const f32x4 kv = ld4(kr + s), vv = ld4(vr + s);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s_acc = mfma16(kv[j], qreg[s + j], s_acc);
          dp_acc = mfma16(vv[j], doreg[s + j], dp_acc);
        }
      }
      const int kl = 16 * t + 4 * grp;
      const f32x4 mm = ld4(&Km[buf][kl]), aa = ld4(&Ka[buf][kl]);
      const bool diag = a.causal && kb + 16 * t + 15 > wave_qmin;
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = fmaf(s_acc[r], mm[r], aa[r]);
        if (ADDMASK && kb + kl + r < a.Tk) s += amrow[kb + kl + r];
        if (diag && kb + kl + r > qrow) s = -INFINITY;
        const float p = exp2f(((s - mrow) - llrow) * SCA_LOG2E);
        ds[r] = p * (dp_acc[r] - delta);
      }
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const f32x4 kt = ld4(Kt[buf] + (16 * d + qi) * (KB + TP) + 16 * t + 4 * grp);
#pragma unroll
        for (int r = 0; r < 4; ++r) dq[d] = mfma16(kt[r], ds[r], dq[d]);
      }
    }
    if (blk + 1 < nblk) commit(buf ^ 1);
    __syncthreads();
  }
  if (qok) {
    float* dqp = P.dq + ((long)b * a.Tq + qrow) * a.ldq + h * HD + 4 * grp;
#pragma unroll
    for (int d = 0; d < ND; ++d) st4(dqp + 16 * d, dq[d] * P.dq_scale);
  }
}

// ------------------------------------------------------------------------------ backward: dK, dV
template <int HD, bool ADDMASK>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(const BwdArgs a) {
  constexpr int NS = HD / 4;
  constexpr int ND = HD / 16;
  constexpr int RV = Blk<HD>::RV;
  __shared__ __attribute__((aligned(16))) float Qs[2][QB * (HD + TP)];
  __shared__ __attribute__((aligned(16))) float Ds[2][QB * (HD + TP)];
  __shared__ __attribute__((aligned(16))) float Qt[2][HD * (QB + TP)];
  __shared__ __attribute__((aligned(16))) float Dt[2][HD * (QB + TP)];
  __shared__ __attribute__((aligned(16))) float Sm[2][QB], Sl[2][QB], Sd[2][QB];

  const sca_attn_bwd_problem& P = a.p[blockIdx.z];
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int k0 = blockIdx.x * KB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kj = lane & 15, grp = lane >> 4;
  const int krow = k0 + 16 * w + kj;
  const bool kok = krow < a.Tk;
  const float plus = (a.causal && a.plus_one) ? 1.0f : 0.0f;

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
  float kmul, kadd;
  key_coef(kv_load(P.key_valid, b, krow, a.Tk), ADDMASK, krow, a.Tk, plus, kmul, kadd);

  f32x4 dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dk[d] = dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int qbeg = a.causal ? (k0 / QB) * QB : 0;
  const int nblk = (a.Tq - qbeg + QB - 1) / QB;
  const int wave_kmin = k0 + 16 * w, wave_kmax = wave_kmin + 15;
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
    }
  };
  auto commit = [&](int buf) {
    blk_store<HD>(Qs[buf], Qt[buf], rq);
    blk_store<HD>(Ds[buf], Dt[buf], rd);
    if (threadIdx.x < QB) {
      Sm[buf][threadIdx.x] = cm;
      Sl[buf][threadIdx.x] = cl;
      Sd[buf][threadIdx.x] = cd;
    }
  };
  prefetch(qbeg);
  commit(0);
  __syncthreads();

  for (int blk = 0; blk < nblk; ++blk) {
    const int qb = qbeg + blk * QB, buf = blk & 1;
    if (blk + 1 < nblk) prefetch(qb + QB);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (a.causal && qb + 16 * t + 15 < wave_kmin) continue;  // all queries before all keys
      f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = s_acc;
      const float* qr = Qs[buf] + (16 * t + kj) * (HD + TP) + NS * grp;
      const float* dr = Ds[buf] + (16 * t + kj) * (HD + TP) + NS * grp;
#pragma unroll
      for (int s = 0; s < NS; s += 4) {
        const f32x4 qv = ld4(qr + s), dv4 = ld4(dr + s);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s_acc = mfma16(qv[j], kreg[s + j], s_acc);
          dp_acc = mfma16(dv4[j], vreg[s + j], dp_acc);
        }
      }
      // lane holds S[q = qb + 16t + 4grp + r][krow]
      const int ql = 16 * t + 4 * grp;
      const f32x4 sm = ld4(&Sm[buf][ql]), sl = ld4(&Sl[buf][ql]), sd = ld4(&Sd[buf][ql]);
      const bool diag = a.causal && qb + 16 * t < wave_kmax;
      float p[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = qb + ql + r;
        float s = fmaf(s_acc[r], kmul, kadd);
        if (ADDMASK && q < a.Tq && krow < a.Tk) s += P.add_mask[((long)b * a.Tq + q) * a.Tk + krow];
        if (diag && krow > q) s = -INFINITY;
        if (q >= a.Tq) s = -INFINITY;
        p[r] = exp2f(((s - sm[r]) - sl[r]) * SCA_LOG2E);
        ds[r] = p[r] * (dp_acc[r] - sd[r]);
      }
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const f32x4 dt = ld4(Dt[buf] + (16 * d + kj) * (QB + TP) + 16 * t + 4 * grp);
        const f32x4 qt = ld4(Qt[buf] + (16 * d + kj) * (QB + TP) + 16 * t + 4 * grp);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dv[d] = mfma16(dt[r], p[r], dv[d]);
          dk[d] = mfma16(qt[r], ds[r], dk[d]);
        }
      }
    }
    if (blk + 1 < nblk) commit(buf ^ 1);
    __syncthreads();
  }
  if (kok) {
    float* dkp = P.dk + ((long)b * a.Tk + krow) * a.ldk + h * HD + 4 * grp;
    float* dvp = P.dv + ((long)b * a.Tk + krow) * a.ldv + h * HD + 4 * grp;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      st4(dkp + 16 * d, dk[d]);
      st4(dvp + 16 * d, dv[d] * P.dv_scale);
    }
  }
}

template <typename Args>
int check_common(const Args& a, int hd, int nprob) {
  if (nprob < 1 || nprob > SCA_ATTN_MAX_PROBLEMS || a.B < 1 || a.H < 1 || a.Tq < 1 || a.Tk < 1) return 1;
  if (hd != 16 && hd != 32 && hd != 64) return 2;
  if ((a.ldq & 3) || (a.ldk & 3) || (a.ldv & 3) || (a.ldo & 3)) return 3;
  if (a.ldq < a.H * hd || a.ldk < a.H * hd || a.ldv < a.H * hd || a.ldo < a.H * hd) return 3;
  if (a.causal && a.Tq != a.Tk) return 4;
  return 0;
}

template <int HD, bool AM>
void launch_fwd(const FwdArgs& a, dim3 grid, hipStream_t st) {
  hipLaunchKernelGGL((attn_fwd_kernel<HD, AM>), grid, dim3(256), 0, st, a);
}

template <int HD, bool AM>
void launch_bwd(const BwdArgs& a, dim3 gq, dim3 gk, hipStream_t st) {
  hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, AM>), gq, dim3(256), 0, st, a);
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, AM>), gk, dim3(256), 0, st, a);
}

}  // namespace

extern "C" void sca_set_error(const char* msg);

extern "C" int sca_attn_fwd(int nprob, const sca_attn_fwd_problem* probs, int B, int H, int Tq, int Tk, int hd,
                            int ldq, int ldk, int ldv, int ldo, int causal, int plus_one, void* stream) {
  FwdArgs a;
  a.B = B; a.H = H; a.Tq = Tq; a.Tk = Tk; a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
  a.causal = causal; a.plus_one = plus_one;
  const int err = check_common(a, hd, nprob);
  if (err) {
    sca_set_error(err == 2 ? "sca_attn_fwd: head_dim must be 16, 32 or 64"
                           : "sca_attn_fwd: bad shape / leading dimension / causal with Tq != Tk");
    return SCA_ERR_ARG;
  }
  bool am = false;
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
  }
  dim3 grid((Tq + QB - 1) / QB, B * H, nprob);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hd == 16) am ? launch_fwd<16, true>(a, grid, st) : launch_fwd<16, false>(a, grid, st);
  else if (hd == 32) am ? launch_fwd<32, true>(a, grid, st) : launch_fwd<32, false>(a, grid, st);
  else am ? launch_fwd<64, true>(a, grid, st) : launch_fwd<64, false>(a, grid, st);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_attn_fwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_attn_bwd(int nprob, const sca_attn_bwd_problem* probs, int B, int H, int Tq, int Tk, int hd,
                            int ldq, int ldk, int ldv, int ldo, int causal, int plus_one, void* stream) {
  BwdArgs a;
  a.B = B; a.H = H; a.Tq = Tq; a.Tk = Tk; a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
  a.causal = causal; a.plus_one = plus_one;
  const int err = check_common(a, hd, nprob);
  if (err) {
    sca_set_error(err == 2 ? "sca_attn_bwd: head_dim must be 16, 32 or 64"
                           : "sca_attn_bwd: bad shape / leading dimension / causal with Tq != Tk");
    return SCA_ERR_ARG;
  }
  bool am = false;
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
    a.p[i] = p;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 gq((Tq + QB - 1) / QB, B * H, nprob), gk((Tk + KB - 1) / KB, B * H, nprob);
  if (hd == 16) am ? launch_bwd<16, true>(a, gq, gk, st) : launch_bwd<16, false>(a, gq, gk, st);
  else if (hd == 32) am ? launch_bwd<32, true>(a, gq, gk, st) : launch_bwd<32, false>(a, gq, gk, st);
  else am ? launch_bwd<64, true>(a, gq, gk, st) : launch_bwd<64, false>(a, gq, gk, st);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_attn_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}
