// Recognition-head losses of MSCA_Net:
//   * CTC: MSCA_Net.compute_loss (model/__init__.py:241-290) = log_softmax -> clamp(-100, 0)
//     -> nn.CTCLoss(blank=0, reduction='none', zero_infinity=True) -> mean over finite
//     losses -> clamp(0, 100).  The log-space alpha/beta recursions and the gradient follow
//     torch's published CPU algorithm (aten/src/ATen/native/LossCTC.cpp, the third-party op
//     the reference calls; formulas restated in oracle/heads_oracle.py).
//   * SeqKD (loss.py:5-21) with the weight and clamp(-100, 100) of model/__init__.py:203-214.
//   * clamp(+-50) of RecognitionHead.forward (model/__init__.py:54-58) with its gradient gate.
// All of it is latency-bound (one sample's alpha row depends on the previous frame's); the
// HBM traffic is a few (B, T, C) passes.  Batch-major logits (B, T, C): the reference's
// permute(1, 0, 2) (:245) is a view and never materialised.
#include "common.h"
#include "../../include/scatten.h"

extern "C" void sca_set_error(const char* msg);

namespace {

constexpr int CTC_THREADS = 256;
constexpr int CTC_MAX_L = 2 * SCA_CTC_MAX_S + 1;
constexpr float NEG_INF = -__builtin_huge_valf();

__device__ __forceinline__ float lse3(float a, float b, float c) {
  float m = fmaxf(a, fmaxf(b, c));
  if (m == NEG_INF) m = 0.0f;
  return __logf(__expf(a - m) + __expf(b - m) + __expf(c - m)) + m;
}

// log_probs element = clamp(log_softmax(x), -100, 0) with torch's (x - max) - log(sum) order
__device__ __forceinline__ float ctc_lp_raw(float x, float m, float ls) { return (x - m) - ls; }
__device__ __forceinline__ float ctc_lp(float raw) { return fminf(fmaxf(raw, -100.0f), 0.0f); }

struct CtcDims {
  int B, T, C, S;
};

// workspace layout (floats): rowstat[B*T*2] | alpha[B*T*Lm] | beta[B*T*Lm] | nll[B] | scale[B]
struct CtcWs {
  float *rowstat, *alpha, *beta, *nll, *scale;
  __host__ __device__ CtcWs(float* ws, CtcDims d) {
    const long Lm = 2L * d.S + 1, BT = (long)d.B * d.T;
    rowstat = ws;
    alpha = rowstat + 2 * BT;
    beta = alpha + BT * Lm;
    nll = beta + BT * Lm;
    scale = nll + d.B;
  }
};

__device__ __forceinline__ void ctc_lengths(const int* in_len, const int* tgt_len, int b, CtcDims d, int& Tb,
                                            int& Sb) {
  // model/__init__.py:262-266: clamp both to >= 1, then input = max(input, target)
  Sb = max(tgt_len[b], 1);
  Tb = max(max(in_len[b], 1), Sb);
  Sb = min(Sb, d.S);  // host validates; the clamps only keep a bad call in bounds
  Tb = min(Tb, d.T);
}

__device__ __forceinline__ int ctc_label(const int* lab, int Sb, int s, int C) {
  if (!(s & 1)) return 0;
  const int c = lab[(s - 1) >> 1];
  (void)Sb;
  return min(max(c, 0), C - 1);
}

// one wave per (b, t) row: max and log-sum-exp of the logits row
__global__ __launch_bounds__(256) void ctc_rowstat_kernel(const float* __restrict__ x, float* __restrict__ rowstat,
                                                          long rows, int C) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + row * C;
  float m = NEG_INF;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, xr[c]);
  m = wave_max(m);
  float s = 0.0f;
  for (int c = lane; c < C; c += 64) s += __expf(xr[c] - m);
  s = wave_sum(s);
  if (lane == 0) {
    rowstat[2 * row] = m;
    rowstat[2 * row + 1] = __logf(s);
  }
}

// grid (B, 2): y = 0 runs the alpha (forward) recursion, y = 1 the beta (backward) one
__global__ __launch_bounds__(CTC_THREADS) void ctc_alpha_beta_kernel(const float* __restrict__ x,
                                                                     const int* __restrict__ labels,
                                                                     const int* __restrict__ in_len,
                                                                     const int* __restrict__ tgt_len, CtcDims d,
                                                                     float* ws) {
  __shared__ float buf[2][CTC_MAX_L];
  __shared__ int lab_s[CTC_MAX_L];
  CtcWs w(ws, d);
  const int b = blockIdx.x, tid = threadIdx.x;
  const bool beta_pass = blockIdx.y == 1;
  int Tb, Sb;
  ctc_lengths(in_len, tgt_len, b, d, Tb, Sb);
  const int L = 2 * Sb + 1;
  const long Lm = 2L * d.S + 1;
  const int* lab = labels + (long)b * d.S;
  for (int s = tid; s < L; s += CTC_THREADS) lab_s[s] = ctc_label(lab, Sb, s, d.C);
  __syncthreads();
  const float* xb = x + (long)b * d.T * d.C;
  const float* rs = w.rowstat + 2L * b * d.T;
  float* out = (beta_pass ? w.beta : w.alpha) + (long)b * d.T * Lm;
  auto lp_at = [&](int t, int s) {
    const float m = rs[2 * t], ls = rs[2 * t + 1];
    return ctc_lp(ctc_lp_raw(xb[(long)t * d.C + lab_s[s]], m, ls));
  };
  int cur = 0;
  // first frame (alpha: t = 0, beta: t = Tb - 1)
  const int t0 = beta_pass ? Tb - 1 : 0;
  for (int s = tid; s < L; s += CTC_THREADS) {
    float v = NEG_INF;
    if (!beta_pass && s < 2) v = lp_at(t0, s);
    if (beta_pass && s >= L - 2) v = lp_at(t0, s);
    buf[cur][s] = v;
    out[(long)t0 * Lm + s] = v;
  }
  __syncthreads();
  for (int step = 1; step < Tb; ++step) {
    const int t = beta_pass ? Tb - 1 - step : step;
    const float* prev = buf[cur];
    float* nxt = buf[cur ^ 1];
    for (int s = tid; s < L; s += CTC_THREADS) {
      const int l = lab_s[s];
      float a1 = prev[s], a2, a3;
      if (!beta_pass) {
        a2 = s > 0 ? prev[s - 1] : NEG_INF;
        a3 = (s > 1 && lab_s[s - 2] != l) ? prev[s - 2] : NEG_INF;
      } else {
        a2 = s < L - 1 ? prev[s + 1] : NEG_INF;
        a3 = (s < L - 2 && lab_s[s + 2] != l) ? prev[s + 2] : NEG_INF;
      }
      const float v = lse3(a1, a2, a3) + lp_at(t, s);
      nxt[s] = v;
      out[(long)t * Lm + s] = v;
    }
    cur ^= 1;
    __syncthreads();
  }
  if (!beta_pass && tid == 0) {
    // nll = -log(exp(alpha[Tb-1][L-1]) + exp(alpha[Tb-1][L-2])); zero_infinity
    const float l1 = buf[cur][L - 1], l2 = buf[cur][L - 2];
    float m = fmaxf(l1, l2);
    if (m == NEG_INF) m = 0.0f;
    w.nll[b] = -(__logf(__expf(l1 - m) + __expf(l2 - m)) + m);  // +inf kept: zero_infinity below
  }
}

// one workgroup: loss = clamp(mean(finite nll), 0, 100); per-sample d loss / d nll
__global__ __launch_bounds__(256) void ctc_finalize_kernel(CtcDims d, float* ws, float* nll_out, float* loss) {
  __shared__ float red_s[4], red_n[4];
  CtcWs w(ws, d);
  const int tid = threadIdx.x;
  float s = 0.0f, n = 0.0f;
  for (int b = tid; b < d.B; b += 256) {
    const float raw = w.nll[b];
    const float v = raw == __builtin_huge_valf() ? 0.0f : raw;  // zero_infinity=True
    if (isfinite(v)) { s += v; n += 1.0f; }
    if (nll_out) nll_out[b] = v;
  }
  s = wave_sum(s);
  n = wave_sum(n);
  if ((tid & 63) == 0) { red_s[tid >> 6] = s; red_n[tid >> 6] = n; }
  __syncthreads();
  const float S = red_s[0] + red_s[1] + red_s[2] + red_s[3];
  const float N = red_n[0] + red_n[1] + red_n[2] + red_n[3];
  // model/__init__.py:276-283: no finite loss -> 0 (no gradient); else clamp(mean, 0, 100)
  const float mean = N > 0.0f ? S / N : 0.0f;
  const float gate = (N > 0.0f && mean >= 0.0f && mean <= 100.0f) ? 1.0f / N : 0.0f;
  if (tid == 0) loss[0] = fminf(fmaxf(mean, 0.0f), 100.0f);
  // zero_infinity'd samples count in the mean with loss 0 but get no gradient
  for (int b = tid; b < d.B; b += 256) w.scale[b] = isfinite(w.nll[b]) ? gate : 0.0f;
}

// one workgroup per (b, t) row: d loss / d logits (through the CTC gradient, the log-prob
// clamp and log_softmax)
__global__ __launch_bounds__(CTC_THREADS) void ctc_grad_kernel(const float* __restrict__ x,
                                                               const int* __restrict__ labels,
                                                               const int* __restrict__ in_len,
                                                               const int* __restrict__ tgt_len, CtcDims d,
                                                               const float* ws, const float* __restrict__ dloss,
                                                               float* __restrict__ dx) {
  __shared__ float ab[CTC_MAX_L];
  __shared__ float g_s[SCA_CTC_MAX_C];
  __shared__ float red[4];
  CtcWs w(const_cast<float*>(ws), d);
  const int b = blockIdx.y, t = blockIdx.x, tid = threadIdx.x;
  const long row = (long)b * d.T + t;
  const float* xr = x + row * d.C;
  float* dr = dx + row * d.C;
  int Tb, Sb;
  ctc_lengths(in_len, tgt_len, b, d, Tb, Sb);
  const float gr = dloss[0] * w.scale[b];
  if (t >= Tb || gr == 0.0f) {  // frames past the input length, zero_infinity samples, gated loss
    for (int c = tid; c < d.C; c += CTC_THREADS) dr[c] = 0.0f;
    return;
  }
  const int L = 2 * Sb + 1;
  const long Lm = 2L * d.S + 1;
  const int* lab = labels + (long)b * d.S;
  const float* al = w.alpha + row * Lm;
  const float* be = w.beta + row * Lm;
  for (int s = tid; s < L; s += CTC_THREADS) ab[s] = al[s] + be[s];
  for (int c = tid; c < d.C; c += CTC_THREADS) g_s[c] = NEG_INF;
  __syncthreads();
  // lcab[c] = logsumexp over states s with l'(s) = c of alpha + beta
  if (tid < 64) {  // wave 0: the blank (every even state, plus odd states whose label is 0)
    float m = NEG_INF;
    for (int s = tid; s < L; s += 64)
      if (!(s & 1) || ctc_label(lab, Sb, s, d.C) == 0) m = fmaxf(m, ab[s]);
    m = wave_max(m);
    float acc = 0.0f;
    if (m != NEG_INF)
      for (int s = tid; s < L; s += 64)
        if (!(s & 1) || ctc_label(lab, Sb, s, d.C) == 0) acc += __expf(ab[s] - m);
    acc = wave_sum(acc);
    if (tid == 0) g_s[0] = m == NEG_INF ? NEG_INF : __logf(acc) + m;
  } else {  // other waves: one thread per distinct non-blank label (its first occurrence)
    for (int j = tid - 64; j < Sb; j += CTC_THREADS - 64) {
      const int c = ctc_label(lab, Sb, 2 * j + 1, d.C);
      bool first = c != 0;
      for (int k = 0; k < j && first; ++k) first = ctc_label(lab, Sb, 2 * k + 1, d.C) != c;
      if (!first) continue;
      float m = NEG_INF;
      for (int k = j; k < Sb; ++k)
        if (ctc_label(lab, Sb, 2 * k + 1, d.C) == c) m = fmaxf(m, ab[2 * k + 1]);
      float acc = 0.0f;
      if (m != NEG_INF)
        for (int k = j; k < Sb; ++k)
          if (ctc_label(lab, Sb, 2 * k + 1, d.C) == c) acc += __expf(ab[2 * k + 1] - m);
      g_s[c] = m == NEG_INF ? NEG_INF : __logf(acc) + m;
    }
  }
  __syncthreads();
  const float m = w.rowstat[2 * row], ls = w.rowstat[2 * row + 1];
  const float nll = w.nll[b];
  float part = 0.0f;
  for (int c = tid; c < d.C; c += CTC_THREADS) {
    const float raw = ctc_lp_raw(xr[c], m, ls);
    const float lp = ctc_lp(raw);
    // torch ctc_loss_backward: (exp(lp) - exp(lcab + nll - lp)) * grad_out
    float g = (__expf(lp) - __expf(g_s[c] + nll - lp)) * gr;
    if (!(raw >= -100.0f && raw <= 0.0f)) g = 0.0f;  // clamp(-100, 0) backward
    g_s[c] = g;
    part += g;
  }
  part = wave_sum(part);
  if ((tid & 63) == 0) red[tid >> 6] = part;
  __syncthreads();
  const float G = red[0] + red[1] + red[2] + red[3];
  for (int c = tid; c < d.C; c += CTC_THREADS) dr[c] = g_s[c] - __expf(ctc_lp_raw(xr[c], m, ls)) * G;
}

// ------------------------------------------------------------------------------------ SeqKD
struct KdArgs {
  const float *s, *q;
  int R, C, start;
  float inv_temp, weight_t2, lo, hi;
};

// ws layout: row_loss[R] | stats[4R] (student max, log-sum, teacher max, log-sum) | dscale[1]
__global__ __launch_bounds__(256) void kd_row_kernel(KdArgs a, float* ws) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.R) return;
  const float* sr = a.s + row * a.C;
  const float* qr = a.q + row * a.C;
  float ms = NEG_INF, mq = NEG_INF;
  for (int c = a.start + lane; c < a.C; c += 64) {
    ms = fmaxf(ms, sr[c] * a.inv_temp);
    mq = fmaxf(mq, qr[c] * a.inv_temp);
  }
  ms = wave_max(ms);
  mq = wave_max(mq);
  float ss = 0.0f, sq = 0.0f;
  for (int c = a.start + lane; c < a.C; c += 64) {
    ss += __expf(sr[c] * a.inv_temp - ms);
    sq += __expf(qr[c] * a.inv_temp - mq);
  }
  const float lss = __logf(wave_sum(ss));
  const float sq_all = wave_sum(sq);
  const float lsq = __logf(sq_all);
  // KLDivLoss (log_target=False): xlogy(p, p) - p * log_softmax(student)
  float acc = 0.0f;
  for (int c = a.start + lane; c < a.C; c += 64) {
    const float p = __expf(qr[c] * a.inv_temp - mq) / sq_all;  // F.softmax
    const float lsm = (sr[c] * a.inv_temp - ms) - lss;         // F.log_softmax
    acc += (p > 0.0f ? p * __logf(p) : 0.0f) - p * lsm;
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    ws[row] = acc;
    float* st = ws + a.R + 4 * row;
    st[0] = ms; st[1] = lss; st[2] = mq; st[3] = lsq;
  }
}

__global__ __launch_bounds__(256) void kd_finalize_kernel(KdArgs a, float* ws, float* loss) {
  __shared__ float red[4];
  const int tid = threadIdx.x;
  float s = 0.0f;
  for (int r = tid; r < a.R; r += 256) s += ws[r];
  s = wave_sum(s);
  if ((tid & 63) == 0) red[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    // batchmean over the R = B*T rows of the .view(-1, C') (loss.py:13-19), * T^2 * weight
    const float v = (red[0] + red[1] + red[2] + red[3]) / (float)a.R * a.weight_t2;
    loss[0] = fminf(fmaxf(v, a.lo), a.hi);
    ws[5L * a.R] = (v >= a.lo && v <= a.hi) ? a.weight_t2 / (float)a.R : 0.0f;
  }
}

__global__ __launch_bounds__(256) void kd_grad_kernel(KdArgs a, const float* ws, const float* dloss, float* ds,
                                                      float* dq) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.R) return;
  const float k = dloss[0] * ws[5L * a.R] * a.inv_temp;
  const float* st = ws + a.R + 4 * row;
  const float ms = st[0], lss = st[1], mq = st[2], lsq = st[3];
  const float* sr = a.s + row * a.C;
  const float* qr = a.q + row * a.C;
  float hbar = 0.0f;
  if (dq) {  // sum_c p_c (log p_c - log_softmax(student)_c) for the teacher's softmax backward
    for (int c = a.start + lane; c < a.C; c += 64) {
      const float lp = (qr[c] * a.inv_temp - mq) - lsq;
      hbar += __expf(lp) * (lp - ((sr[c] * a.inv_temp - ms) - lss));
    }
    hbar = wave_sum(hbar);
  }
  for (int c = lane; c < a.C; c += 64) {
    float gs = 0.0f, gq = 0.0f;
    if (c >= a.start) {
      const float lsm = (sr[c] * a.inv_temp - ms) - lss;
      const float lp = (qr[c] * a.inv_temp - mq) - lsq;
      const float p = __expf(lp);
      gs = k * (__expf(lsm) - p);
      gq = k * p * ((lp - lsm) - hbar);
    }
    if (ds) ds[row * a.C + c] = gs;
    if (dq) dq[row * a.C + c] = gq;
  }
}

__global__ __launch_bounds__(256) void clamp_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                    const float* __restrict__ dy, float* __restrict__ dx, long n,
                                                    float lo, float hi) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float v = x[i];
    if (dy) dx[i] = (v >= lo && v <= hi) ? dy[i] : 0.0f;  // torch clamp backward gate
    else y[i] = fminf(fmaxf(v, lo), hi);
  }
}


// ------------------------------------------------------------------------------------ LSTM
// AlignmentModule's bidirectional nn.LSTM (model/alignment_module.py:24-30), batch-major.
// The input projection, the per-step recurrent product h W_hh^T (+ b_hh + the projection
// row, as GEMM epilogue) and all weight / input gradients are sca_gemm launches; these
// two kernels are the pointwise cell of one time step, both directions in one launch
// (grid.y = direction; direction 1 walks t = T-1 .. 0).  Layouts, D = ndir:
//   gates (B, D*4H) this step's pre-activations, gate order i, f, g, o (torch's)
//   act   (B, T, D*4H) saved activations      c, y (B, T, D*H) cell / hidden states
//   hp    (B, T, D*H) the hidden state each step READS: h_{t-1} (dir 0) / h_{t+1} (dir 1),
//         zero where there is none (the caller zero-fills it once)
//   dh, dc (B, D*H) scratch of the backward walk;  dg (B, T, D*4H) gate pre-activation grads
struct LstmArgs {
  const float* gates;
  float *act, *c, *y, *hp;
  const float *dh, *dy;
  float *dc, *dg;
  int B, T, H, D, step;
};

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ __launch_bounds__(256) void lstm_cell_fwd_kernel(LstmArgs a) {
  const int dir = blockIdx.y;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= a.B * a.H) return;
  const int b = idx / a.H, j = idx - b * a.H, H = a.H, DH = a.D * H;
  const int t = dir ? a.T - 1 - a.step : a.step;
  const int tp = dir ? t + 1 : t - 1, tn = dir ? t - 1 : t + 1;
  const long row = (long)b * a.T + t;
  const float* g = a.gates + (long)b * 4 * DH + dir * 4 * H;
  const float gi = sigm(g[j]), gf = sigm(g[H + j]), gg = tanhf(g[2 * H + j]), go = sigm(g[3 * H + j]);
  const float cp = (tp >= 0 && tp < a.T) ? a.c[((long)b * a.T + tp) * DH + dir * H + j] : 0.0f;
  const float c = gf * cp + gi * gg;
  const float h = go * tanhf(c);
  a.c[row * DH + dir * H + j] = c;
  a.y[row * DH + dir * H + j] = h;
  if (tn >= 0 && tn < a.T) a.hp[((long)b * a.T + tn) * DH + dir * H + j] = h;
  float* ac = a.act + row * 4 * DH + dir * 4 * H;
  ac[j] = gi; ac[H + j] = gf; ac[2 * H + j] = gg; ac[3 * H + j] = go;
}

// backward step `step` walks t = T-1-step (dir 0) / t = step (dir 1); dh holds
// dY_t + dG_{t'} W_hh (GEMM with the dY row as residual) except at step 0, where it is dY_t
__global__ __launch_bounds__(256) void lstm_cell_bwd_kernel(LstmArgs a) {
  const int dir = blockIdx.y;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= a.B * a.H) return;
  const int b = idx / a.H, j = idx - b * a.H, H = a.H, DH = a.D * H;
  const int t = dir ? a.step : a.T - 1 - a.step;
  const int tp = dir ? t + 1 : t - 1;
  const long row = (long)b * a.T + t;
  const float dh = a.step == 0 ? a.dy[row * DH + dir * H + j] : a.dh[(long)b * DH + dir * H + j];
  const float dcn = a.step == 0 ? 0.0f : a.dc[(long)b * DH + dir * H + j];
  const float* ac = a.act + row * 4 * DH + dir * 4 * H;
  const float gi = ac[j], gf = ac[H + j], gg = ac[2 * H + j], go = ac[3 * H + j];
  const float tc = tanhf(a.c[row * DH + dir * H + j]);
  const float cp = (tp >= 0 && tp < a.T) ? a.c[((long)b * a.T + tp) * DH + dir * H + j] : 0.0f;
  const float dcc = dcn + dh * go * (1.0f - tc * tc);
  float* dg = a.dg + row * 4 * DH + dir * 4 * H;
  dg[j] = dcc * gg * gi * (1.0f - gi);
  dg[H + j] = dcc * cp * gf * (1.0f - gf);
  dg[2 * H + j] = dcc * gi * (1.0f - gg * gg);
  dg[3 * H + j] = dh * tc * go * (1.0f - go);
  a.dc[(long)b * DH + dir * H + j] = dcc * gf;
}

bool ctc_dims_ok(int B, int T, int C, int S) {
  return B >= 1 && T >= 1 && C >= 1 && C <= SCA_CTC_MAX_C && S >= 1 && S <= SCA_CTC_MAX_S;
}

}  // namespace

extern "C" long sca_ctc_workspace_floats(int B, int T, int S) {
  const long BT = (long)B * T;
  return 2 * BT + 2 * BT * (2L * S + 1) + 2L * B;
}

extern "C" int sca_ctc_loss_fwd(const float* logits, const int* labels, const int* in_len, const int* tgt_len, int B,
                                int T, int C, int S, float* nll, float* loss, float* ws, void* stream) {
  if (!ctc_dims_ok(B, T, C, S) || !logits || !labels || !in_len || !tgt_len || !loss || !ws) {
    sca_set_error("sca_ctc_loss_fwd: bad arguments (C <= 8192, 1 <= S <= 1023)");
    return SCA_ERR_ARG;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const CtcDims d{B, T, C, S};
  const long rows = (long)B * T;
  hipLaunchKernelGGL(ctc_rowstat_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, logits, ws, rows, C);
  hipLaunchKernelGGL(ctc_alpha_beta_kernel, dim3(B, 2), dim3(CTC_THREADS), 0, st, logits, labels, in_len, tgt_len,
                     d, ws);
  hipLaunchKernelGGL(ctc_finalize_kernel, dim3(1), dim3(256), 0, st, d, ws, nll, loss);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_ctc_loss_fwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_ctc_loss_bwd(const float* logits, const int* labels, const int* in_len, const int* tgt_len, int B,
                                int T, int C, int S, const float* dloss, const float* ws, float* dlogits,
                                void* stream) {
  if (!ctc_dims_ok(B, T, C, S) || !logits || !labels || !in_len || !tgt_len || !dloss || !ws || !dlogits) {
    sca_set_error("sca_ctc_loss_bwd: bad arguments (C <= 8192, 1 <= S <= 1023)");
    return SCA_ERR_ARG;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(ctc_grad_kernel, dim3(T, B), dim3(CTC_THREADS), 0, st, logits, labels, in_len, tgt_len,
                     CtcDims{B, T, C, S}, ws, dloss, dlogits);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_ctc_loss_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" long sca_seqkd_workspace_floats(int R) { return 5L * R + 1; }

extern "C" int sca_seqkd_fwd(const float* student, const float* teacher, int R, int C, int start, float temp,
                             float weight, float lo, float hi, float* loss, float* ws, void* stream) {
  if (R < 1 || C < 1 || start < 0 || start >= C || !(temp > 0.0f) || !student || !teacher || !loss || !ws) {
    sca_set_error("sca_seqkd_fwd: bad arguments");
    return SCA_ERR_ARG;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const KdArgs a{student, teacher, R, C, start, 1.0f / temp, weight * temp * temp, lo, hi};
  hipLaunchKernelGGL(kd_row_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, st, a, ws);
  hipLaunchKernelGGL(kd_finalize_kernel, dim3(1), dim3(256), 0, st, a, ws, loss);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_seqkd_fwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_seqkd_bwd(const float* student, const float* teacher, int R, int C, int start, float temp,
                             const float* dloss, const float* ws, float* dstudent, float* dteacher, void* stream) {
  if (R < 1 || C < 1 || start < 0 || start >= C || !(temp > 0.0f) || !student || !teacher || !dloss || !ws ||
      (!dstudent && !dteacher)) {
    sca_set_error("sca_seqkd_bwd: bad arguments");
    return SCA_ERR_ARG;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const KdArgs a{student, teacher, R, C, start, 1.0f / temp, 0.0f, 0.0f, 0.0f};
  hipLaunchKernelGGL(kd_grad_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, st, a, ws, dloss, dstudent,
                     dteacher);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_seqkd_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_clamp(const float* x, float* y, const float* dy, float* dx, long n, float lo, float hi,
                         void* stream) {
  if (n < 0 || !x || (dy ? !dx : !y)) {
    sca_set_error("sca_clamp: bad arguments");
    return SCA_ERR_ARG;
  }
  if (n == 0) return SCA_OK;
  const long blocks = (n + 255) / 256;
  hipLaunchKernelGGL(clamp_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, y, dy, dx, n, lo, hi);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_clamp: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_lstm_cell_fwd(const float* gates, float* act, float* c, float* y, float* hp, int B, int T, int H,
                                 int ndir, int step, void* stream) {
  if (B < 1 || T < 1 || H < 1 || ndir < 1 || ndir > 2 || step < 0 || step >= T || !gates || !act || !c || !y ||
      !hp) {
    sca_set_error("sca_lstm_cell_fwd: bad arguments");
    return SCA_ERR_ARG;
  }
  LstmArgs a{gates, act, c, y, hp, nullptr, nullptr, nullptr, nullptr, B, T, H, ndir, step};
  hipLaunchKernelGGL(lstm_cell_fwd_kernel, dim3((B * H + 255) / 256, ndir), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_lstm_cell_fwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_lstm_cell_bwd(const float* dh, const float* dy, const float* act, const float* c, float* dc,
                                 float* dg, int B, int T, int H, int ndir, int step, void* stream) {
  if (B < 1 || T < 1 || H < 1 || ndir < 1 || ndir > 2 || step < 0 || step >= T || !dy || !act || !c || !dc ||
      !dg || (step > 0 && !dh)) {
    sca_set_error("sca_lstm_cell_bwd: bad arguments");
    return SCA_ERR_ARG;
  }
  LstmArgs a{nullptr, const_cast<float*>(act), const_cast<float*>(c), nullptr, nullptr, dh, dy, dc, dg,
             B, T, H, ndir, step};
  hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3((B * H + 255) / 256, ndir), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_lstm_cell_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}
