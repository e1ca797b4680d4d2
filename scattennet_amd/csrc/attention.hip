// Fused masked attention (forward + backward) on the gfx950 f32 matrix cores
// (v_mfma_f32_16x16x4_f32), for the three SCAttenNet attention operators:
//   SelfAttention        model/attention.py:46-76   (key-padding mask)
//   SelfCausalAttention  model/attention.py:148-182 (tril -> -inf, then +causal mask)
//   CrossAttention       model/attention.py:97-128  (key-padding mask, Tq may != Tk)
//
// Layout in HBM: activations stay (B, T, H*hd) row-major exactly as the projections write
// them (no head transposes: head h is the column slice h*hd .. h*hd+hd-1).
//
// Forward: one workgroup = (problem g, clip b, head h, 64 queries); 4 waves x 16 queries.
// K/V stream through LDS in 64-key blocks.  Scores are computed SWAPPED (S^T = K Q^T) so a
// lane owns one query column and 4 keys per 16x16 tile: the row max / row sum need only two
// cross-lane xor-shuffles, and the S^T accumulator registers are already the B operand of
// the P.V MFMA (O^T += V^T P^T) — P never leaves registers.  Online softmax (running max m,
// running sum l).  Saves m and ll = log(l) per row: a fully padded row (all finfo.min)
// then recomputes to exactly uniform weights in the backward pass (m + log(l) would round
// back to finfo.min).
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

struct FwdArgs {
  sca_attn_fwd_problem p[SCA_ATTN_MAX_PROBLEMS];
  int B, H, Tq, Tk, ldq, ldk, ldv, ldo, causal, plus_one;
};

struct BwdArgs {
  sca_attn_bwd_problem p[SCA_ATTN_MAX_PROBLEMS];
  int B, H, Tq, Tk, ldq, ldk, ldv, ldo, causal, plus_one;
};

// Score transform shared by forward and both backward kernels (see scatten.h).
__device__ __forceinline__ float mask_score(float s, int qi, int kj, int Tq, int Tk, int causal, int plus_one,
                                            float valid, const float* add_mask_row) {
  if (kj >= Tk || qi >= Tq) return -INFINITY;
  if (causal && kj > qi) return -INFINITY;
  if (add_mask_row) return s + add_mask_row[kj];
  if (valid == 0.f) return SCA_FMIN;
  return (causal && plus_one) ? s + 1.0f : s;
}

// Cooperative load of a [64 x HD] row block (rows r0.., columns col0..) into LDS, row-major
// with stride HD+4 (rowimg) and/or transposed [HD][64+4] (colimg).  Rows >= nrows -> 0.
template <int HD>
__device__ __forceinline__ void load_block(float* rowimg, float* colimg, const float* base, long ld, int r0,
                                           int nrows) {
  constexpr int V4 = HD / 4;  // float4 per row
  for (int e = threadIdx.x; e < 64 * V4; e += 256) {
    const int r = e / V4, c = (e % V4) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (r0 + r < nrows) v = ld4(base + (long)(r0 + r) * ld + c);
    if (rowimg) st4(rowimg + r * (HD + 4) + c, v);
    if (colimg) {
#pragma unroll
      for (int j = 0; j < 4; ++j) colimg[(c + j) * (64 + 4) + r] = v[j];
    }
  }
}

// ------------------------------------------------------------------------------ forward
template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const FwdArgs a) {
  constexpr int NS = HD / 4;   // MFMA k-steps over the head dim
  constexpr int ND = HD / 16;  // 16-wide output d-blocks
  __shared__ __attribute__((aligned(16))) float Ks[KB * (HD + 4)];
  __shared__ __attribute__((aligned(16))) float Vt[HD * (KB + 4)];
  __shared__ float Mk[KB];

  const sca_attn_fwd_problem& P = a.p[blockIdx.z];
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int q0 = blockIdx.x * QB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = lane & 15, grp = lane >> 4;
  const int qrow = q0 + 16 * w + qi;

  // Q fragment: lane holds Q[qrow][NS*grp + s], s < NS (B operand of S^T = K Q^T)
  float qreg[NS];
  {
    const float* qp = P.q + ((long)b * a.Tq + qrow) * a.ldq + h * HD + NS * grp;
#pragma unroll
    for (int s = 0; s < NS; s += 4) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (qrow < a.Tq) v = ld4(qp + s);
#pragma unroll
      for (int j = 0; j < 4; ++j) qreg[s + j] = v[j];
    }
  }
  const float* amrow = (P.add_mask && qrow < a.Tq) ? P.add_mask + ((long)b * a.Tq + qrow) * a.Tk : nullptr;

  f32x4 o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  const int kend = a.causal ? min(a.Tk, q0 + QB) : a.Tk;
  const int wave_qmax = q0 + 16 * w + 15;
  for (int kb = 0; kb < kend; kb += KB) {
    __syncthreads();
    load_block<HD>(Ks, nullptr, P.k + (long)b * a.Tk * a.ldk + h * HD, a.ldk, kb, a.Tk);
    load_block<HD>(nullptr, Vt, P.v + (long)b * a.Tk * a.ldv + h * HD, a.ldv, kb, a.Tk);
    if (threadIdx.x < KB) {
      const int kj = kb + threadIdx.x;
      Mk[threadIdx.x] = (P.key_valid && kj < a.Tk) ? P.key_valid[(long)b * a.Tk + kj] : 1.f;
    }
    __syncthreads();

    float sv[4][4];
    bool live[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      live[t] = !a.causal || (kb + 16 * t <= wave_qmax);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (live[t]) {
        const float* kr = Ks + (16 * t + qi) * (HD + 4) + NS * grp;
#pragma unroll
        for (int s = 0; s < NS; s += 4) {
          const f32x4 kv = ld4(kr + s);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = mfma16(kv[j], qreg[s + j], acc);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kl = 16 * t + 4 * grp + r;
        sv[t][r] = live[t] ? mask_score(acc[r], qrow, kb + kl, a.Tq, a.Tk, a.causal, a.plus_one, Mk[kl], amrow)
                           : -INFINITY;
      }
    }
    // online softmax (row = this lane's query; 16 values here, 64 across the 4 lanes)
    float mloc = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) mloc = fmaxf(mloc, sv[t][r]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);
    const float alpha = (m_run == -INFINITY) ? 0.f : exp2f((m_run - m_new) * SCA_LOG2E);
    m_run = m_new;
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = (sv[t][r] == -INFINITY) ? 0.f : exp2f((sv[t][r] - m_new) * SCA_LOG2E);
        sv[t][r] = p;
        psum += p;
      }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int d = 0; d < ND; ++d) o[d] *= alpha;
    // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (!live[t]) continue;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const f32x4 vv = ld4(Vt + (16 * d + qi) * (KB + 4) + 16 * t + 4 * grp);
#pragma unroll
        for (int r = 0; r < 4; ++r) o[d] = mfma16(vv[r], sv[t][r], o[d]);
      }
    }
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
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const BwdArgs a) {
  constexpr int NS = HD / 4;
  constexpr int ND = HD / 16;
  __shared__ __attribute__((aligned(16))) float Ks[KB * (HD + 4)];
  __shared__ __attribute__((aligned(16))) float Vs[KB * (HD + 4)];
  __shared__ __attribute__((aligned(16))) float Kt[HD * (KB + 4)];
  __shared__ float Mk[KB];

  const sca_attn_bwd_problem& P = a.p[blockIdx.z];
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int q0 = blockIdx.x * QB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qi = lane & 15, grp = lane >> 4;
  const int qrow = q0 + 16 * w + qi;
  const bool qok = qrow < a.Tq;

  float qreg[NS], doreg[NS];
  float dpart = 0.f;
  {
    const long roff = ((long)b * a.Tq + qrow);
    const float* qp = P.q + roff * a.ldq + h * HD + NS * grp;
    const float* dp = P.dout + roff * a.ldo + h * HD + NS * grp;
    const float* opp = P.o + roff * a.ldo + h * HD + NS * grp;
#pragma unroll
    for (int s = 0; s < NS; s += 4) {
      f32x4 qv = {0.f, 0.f, 0.f, 0.f}, dv = qv, ov = qv;
      if (qok) {
        qv = ld4(qp + s);
        dv = ld4(dp + s);
        ov = ld4(opp + s);
      }
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
  const long si = ((long)b * a.H + h) * a.Tq + qrow;
  float mrow = 0.f, llrow = 0.f;
  if (qok) {
    mrow = P.stat_m[si];
    llrow = P.stat_ll[si];
    if (grp == 0) P.delta[si] = delta;
  }
  const float* amrow = (P.add_mask && qok) ? P.add_mask + ((long)b * a.Tq + qrow) * a.Tk : nullptr;

  f32x4 dq[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kend = a.causal ? min(a.Tk, q0 + QB) : a.Tk;
  const int wave_qmax = q0 + 16 * w + 15;
  for (int kb = 0; kb < kend; kb += KB) {
    __syncthreads();
    load_block<HD>(Ks, Kt, P.k + (long)b * a.Tk * a.ldk + h * HD, a.ldk, kb, a.Tk);
    load_block<HD>(Vs, nullptr, P.v + (long)b * a.Tk * a.ldv + h * HD, a.ldv, kb, a.Tk);
    if (threadIdx.x < KB) {
      const int kj = kb + threadIdx.x;
      Mk[threadIdx.x] = (P.key_valid && kj < a.Tk) ? P.key_valid[(long)b * a.Tk + kj] : 1.f;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (a.causal && kb + 16 * t > wave_qmax) continue;
      f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = s_acc;
      const float* kr = Ks + (16 * t + qi) * (HD + 4) + NS * grp;
      const float* vr = Vs + (16 * t + qi) * (HD + 4) + NS * grp;
#pragma unroll
      for (int s = 0; s < NS; s += 4) {
        const f32x4 kv = ld4(kr + s), vv = ld4(vr + s);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s_acc = mfma16(kv[j], qreg[s + j], s_acc);
          dp_acc = mfma16(vv[j], doreg[s + j], dp_acc);
        }
      }
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kl = 16 * t + 4 * grp + r;
        const float sm = mask_score(s_acc[r], qrow, kb + kl, a.Tq, a.Tk, a.causal, a.plus_one, Mk[kl], amrow);
        const float p = (sm == -INFINITY) ? 0.f : exp2f(((sm - mrow) - llrow) * SCA_LOG2E);
        ds[r] = p * (dp_acc[r] - delta);
      }
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const f32x4 kt = ld4(Kt + (16 * d + qi) * (KB + 4) + 16 * t + 4 * grp);
#pragma unroll
        for (int r = 0; r < 4; ++r) dq[d] = mfma16(kt[r], ds[r], dq[d]);
      }
    }
  }
  if (qok) {
    float* dqp = P.dq + ((long)b * a.Tq + qrow) * a.ldq + h * HD + 4 * grp;
#pragma unroll
    for (int d = 0; d < ND; ++d) st4(dqp + 16 * d, dq[d] * P.dq_scale);
  }
}

// ------------------------------------------------------------------------------ backward: dK, dV
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(const BwdArgs a) {
  constexpr int NS = HD / 4;
  constexpr int ND = HD / 16;
  __shared__ __attribute__((aligned(16))) float Qs[QB * (HD + 4)];
  __shared__ __attribute__((aligned(16))) float Ds[QB * (HD + 4)];
  __shared__ __attribute__((aligned(16))) float Qt[HD * (QB + 4)];
  __shared__ __attribute__((aligned(16))) float Dt[HD * (QB + 4)];
  __shared__ float Sm[QB], Sl[QB], Sd[QB];

  const sca_attn_bwd_problem& P = a.p[blockIdx.z];
  const int b = blockIdx.y / a.H, h = blockIdx.y % a.H;
  const int k0 = blockIdx.x * KB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kj = lane & 15, grp = lane >> 4;
  const int krow = k0 + 16 * w + kj;
  const bool kok = krow < a.Tk;

  float kreg[NS], vreg[NS];
  {
    const float* kp = P.k + ((long)b * a.Tk + krow) * a.ldk + h * HD + NS * grp;
    const float* vp = P.v + ((long)b * a.Tk + krow) * a.ldv + h * HD + NS * grp;
#pragma unroll
    for (int s = 0; s < NS; s += 4) {
      f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = kv;
      if (kok) {
        kv = ld4(kp + s);
        vv = ld4(vp + s);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        kreg[s + j] = kv[j];
        vreg[s + j] = vv[j];
      }
    }
  }
  const float kvalid = (P.key_valid && kok) ? P.key_valid[(long)b * a.Tk + krow] : 1.f;

  f32x4 dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) dk[d] = dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int qbeg = a.causal ? (k0 / QB) * QB : 0;
  const int wave_kmin = k0 + 16 * w;
  for (int qb = qbeg; qb < a.Tq; qb += QB) {
    __syncthreads();
    load_block<HD>(Qs, Qt, P.q + (long)b * a.Tq * a.ldq + h * HD, a.ldq, qb, a.Tq);
    load_block<HD>(Ds, Dt, P.dout + (long)b * a.Tq * a.ldo + h * HD, a.ldo, qb, a.Tq);
    if (threadIdx.x < QB) {
      const int q = qb + threadIdx.x;
      const long si = ((long)b * a.H + h) * a.Tq + q;
      const bool ok = q < a.Tq;
      Sm[threadIdx.x] = ok ? P.stat_m[si] : 0.f;
      Sl[threadIdx.x] = ok ? P.stat_ll[si] : 0.f;
      Sd[threadIdx.x] = ok ? P.delta[si] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (a.causal && qb + 16 * t + 15 < wave_kmin) continue;
      f32x4 s_acc = {0.f, 0.f, 0.f, 0.f}, dp_acc = s_acc;
      const float* qr = Qs + (16 * t + kj) * (HD + 4) + NS * grp;
      const float* dr = Ds + (16 * t + kj) * (HD + 4) + NS * grp;
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
      float p[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * t + 4 * grp + r;
        const int q = qb + ql;
        const float* amrow = (P.add_mask && q < a.Tq) ? P.add_mask + ((long)b * a.Tq + q) * a.Tk : nullptr;
        const float sm = mask_score(s_acc[r], q, krow, a.Tq, a.Tk, a.causal, a.plus_one, kvalid, amrow);
        p[r] = (sm == -INFINITY) ? 0.f : exp2f(((sm - Sm[ql]) - Sl[ql]) * SCA_LOG2E);
        ds[r] = p[r] * (dp_acc[r] - Sd[ql]);
      }
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const f32x4 dt = ld4(Dt + (16 * d + kj) * (QB + 4) + 16 * t + 4 * grp);
        const f32x4 qt = ld4(Qt + (16 * d + kj) * (QB + 4) + 16 * t + 4 * grp);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dv[d] = mfma16(dt[r], p[r], dv[d]);
          dk[d] = mfma16(qt[r], ds[r], dk[d]);
        }
      }
    }
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
  for (int i = 0; i < nprob; ++i) {
    a.p[i] = probs[i];
    if (!probs[i].q || !probs[i].k || !probs[i].v || !probs[i].o || !probs[i].stat_m || !probs[i].stat_ll) {
      sca_set_error("sca_attn_fwd: null pointer");
      return SCA_ERR_ARG;
    }
  }
  dim3 grid((Tq + QB - 1) / QB, B * H, nprob);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hd == 16) hipLaunchKernelGGL(attn_fwd_kernel<16>, grid, dim3(256), 0, st, a);
  else if (hd == 32) hipLaunchKernelGGL(attn_fwd_kernel<32>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, st, a);
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
  for (int i = 0; i < nprob; ++i) {
    const sca_attn_bwd_problem& p = probs[i];
    if (!p.q || !p.k || !p.v || !p.o || !p.dout || !p.stat_m || !p.stat_ll || !p.dq || !p.dk || !p.dv || !p.delta) {
      sca_set_error("sca_attn_bwd: null pointer");
      return SCA_ERR_ARG;
    }
    a.p[i] = p;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 gq((Tq + QB - 1) / QB, B * H, nprob), gk((Tk + KB - 1) / KB, B * H, nprob);
  if (hd == 16) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<16>, gq, dim3(256), 0, st, a);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<16>, gk, dim3(256), 0, st, a);
  } else if (hd == 32) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<32>, gq, dim3(256), 0, st, a);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<32>, gk, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<64>, gq, dim3(256), 0, st, a);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<64>, gk, dim3(256), 0, st, a);
  }
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_attn_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}
