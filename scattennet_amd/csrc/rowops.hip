// Row-wise HBM-bound kernels of the SCA hot path:
//   * residual-add + LayerNorm forward/backward (post-LN blocks, keypoint_module.py:67-72,
//     :101-111) and position-embedding-add + LayerNorm (layers.py:15-30 + :161-162)
//   * fixed-order row reductions (bias / LN-affine / position-table gradients)
//   * fused stream slicing + de-interleave + CoordinateMapping forward/backward
//     (model/__init__.py:133-142, keypoint_module.py:22-26, layers.py:111-123)
// One wave per row for the LayerNorms (a 256-wide fp32 row = one float4 per lane).
#include "common.h"
#include "../../include/scatten.h"

namespace {

// ------------------------------------------------------------------------------ LayerNorm
struct LnFwdArgs {
  sca_ln_fwd_problem p[SCA_LN_MAX_PROBLEMS];
  int rows, N, r_mod, r_off;
  float eps;
  const unsigned long long* drop_off;
};
struct LnBwdArgs {
  sca_ln_bwd_problem p[SCA_LN_MAX_PROBLEMS];
  int rows, N, r_mod, r_off, accumulate, nblk;
};

constexpr int LN_MAXV = 16;  // values per lane -> N <= 1024

__device__ __forceinline__ long rrow(int row, int r_mod, int r_off) { return (long)(row % r_mod) + r_off; }

// Row element access: NV > 0 -> N = 256*NV, lane owns float4 columns 4*lane + 256*j (16 B/lane
// loads); NV == 0 -> any N <= 1024, lane owns scalar columns lane + 64*j.
template <int NV>
struct RowMap {
  static constexpr int kVals = NV > 0 ? 4 * NV : LN_MAXV;
  __device__ static __forceinline__ int col(int lane, int i) {
    return NV > 0 ? 4 * lane + 256 * (i >> 2) + (i & 3) : lane + 64 * i;
  }
};

template <int NV>
__device__ __forceinline__ void load_row(float* v, const float* p, int lane, int N) {
  if (NV > 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const f32x4 t = ld4(p + 4 * lane + 256 * j);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * j + e] = t[e];
    }
  } else {
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      v[i] = c < N ? p[c] : 0.f;
    }
  }
}

template <int NV>
__device__ __forceinline__ void store_row(float* p, const float* v, int lane, int N) {
  if (NV > 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) st4(p + 4 * lane + 256 * j, f32x4{v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]});
  } else {
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < N) p[c] = v[i];
    }
  }
}

template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const LnFwdArgs a) {
  using RM = RowMap<NV>;
  constexpr int V = RM::kVals;
  const sca_ln_fwd_problem& P = a.p[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int N = a.N;
  float v[V], t[V];
  load_row<NV>(v, P.x + (long)row * N, lane, N);
  if (P.r) {
    load_row<NV>(t, P.r + rrow(row, a.r_mod, a.r_off) * N, lane, N);
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] += t[i];
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) s += v[i];
  const float mean = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const float d = (NV > 0 || RM::col(lane, i) < N) ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / N + a.eps);
  float g[V], b[V];
  load_row<NV>(g, P.gamma, lane, N);
  load_row<NV>(b, P.beta, lane, N);
  if (P.post) load_row<NV>(t, P.post + (long)row * N, lane, N);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    float o = (v[i] - mean) * rstd * g[i] + b[i];
    if (P.post) o += t[i];
    if (P.act == SCA_ACT_RELU) o = fmaxf(o, 0.f);
    v[i] = o;
  }
  if (P.drop_p > 0.f) {  // embedding dropout (keypoint_module.py:164-165)
    DropMask dm;
    dm.init(P.drop_seed, P.drop_p, a.drop_off);
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = dm.apply((uint32_t)row * (uint32_t)N + (uint32_t)RM::col(lane, i), v[i]);
  }
  store_row<NV>(P.y + (long)row * N, v, lane, N);
  if (lane == 0) {
    P.mean[row] = mean;
    P.rstd[row] = rstd;
  }
}

#ifndef SCA_LN_BWD_ROWS
#define SCA_LN_BWD_ROWS 8
#endif
constexpr int LN_BWD_ROWS = SCA_LN_BWD_ROWS;  // rows per workgroup (LN_BWD_ROWS / 4 per wave)

template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const LnBwdArgs a) {
  using RM = RowMap<NV>;
  constexpr int V = RM::kVals;
  constexpr int RW = LN_BWD_ROWS / 4;          // rows per wave
  constexpr int RED = NV > 0 ? 256 * NV : 1024;  // partial-row width held in LDS
  const sca_ln_bwd_problem& P = a.p[blockIdx.y];
  __shared__ float red[2][4][RED];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int N = a.N;
  float pg[V], pb[V], gam[V];
#pragma unroll
  for (int i = 0; i < V; ++i) pg[i] = pb[i] = 0.f;
  load_row<NV>(gam, P.gamma, lane, N);
  const int rbeg = blockIdx.x * LN_BWD_ROWS + w * RW;
  // phase 1: every load of the wave's rows in flight at once (the stores of phase 2 could
  // alias them, so the compiler would not hoist them on its own)
  float xv[RW][V], dy[RW][V], mean[RW], rstd[RW];
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) {
    const int row = min(rbeg + rr, a.rows - 1);
    mean[rr] = P.mean[row];
    rstd[rr] = P.rstd[row];
    load_row<NV>(xv[rr], P.x + (long)row * N, lane, N);
    load_row<NV>(dy[rr], P.dy + (long)row * N, lane, N);
    if (P.r) {
      float t[V];
      load_row<NV>(t, P.r + rrow(row, a.r_mod, a.r_off) * N, lane, N);
#pragma unroll
      for (int i = 0; i < V; ++i) xv[rr][i] += t[i];
    }
    if (P.act) {
      float t[V];
      load_row<NV>(t, P.y + (long)row * N, lane, N);
#pragma unroll
      for (int i = 0; i < V; ++i)
        if (!(t[i] > 0.f)) dy[rr][i] = 0.f;  // ReLU gate (threshold_backward: out > 0)
    }
  }
  // phase 2
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) {
    const int row = rbeg + rr;
    if (row >= a.rows) break;
    if (P.dpost) store_row<NV>(P.dpost + (long)row * N, dy[rr], lane, N);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const bool in = NV > 0 || RM::col(lane, i) < N;
      xv[rr][i] = in ? (xv[rr][i] - mean[rr]) * rstd[rr] : 0.f;  // x-hat
      const float g = dy[rr][i] * gam[i];
      sg += g;
      sgx += g * xv[rr][i];
      pg[i] += dy[rr][i] * xv[rr][i];
      pb[i] += dy[rr][i];
    }
    const float mg = wave_sum(sg) / N, mgx = wave_sum(sgx) / N;
    float* dxr = P.dx + (long)row * N;
    float t[V];
    if (a.accumulate) load_row<NV>(t, dxr, lane, N);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      float d = rstd[rr] * (dy[rr][i] * gam[i] - mg - xv[rr][i] * mgx);
      if (a.accumulate) d += t[i];
      t[i] = d;
    }
    store_row<NV>(dxr, t, lane, N);
  }
  // combine the 4 waves' partials in fixed order, one partial row per workgroup
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = RM::col(lane, i);
    if (c < N) {
      red[0][w][c] = pg[i];
      red[1][w][c] = pb[i];
    }
  }
  __syncthreads();
  float* part = P.partial;
  for (int c = threadIdx.x; c < N; c += 256) {
    const float gsum = ((red[0][0][c] + red[0][1][c]) + red[0][2][c]) + red[0][3][c];
    const float bsum = ((red[1][0][c] + red[1][1][c]) + red[1][2][c]) + red[1][3][c];
    part[(long)blockIdx.x * N + c] = gsum;
    part[((long)a.nblk + blockIdx.x) * N + c] = bsum;
  }
}

// ------------------------------------------------------------------------------ reductions
struct ReduceArgs {
  sca_reduce_problem p[SCA_REDUCE_MAX_PROBLEMS];
  int S, I, N, accumulate;
  long stride_s, stride_i;
};

// grid (ceil(N/64), I, nprob), 1024 threads: wave w sums s = w, w+16, ... with 8 loads in
// flight (the reduction is latency-bound: few workgroups, long strided columns); the 16 wave
// partials are combined in fixed order (deterministic).
constexpr int RED_WAVES = 16;
__global__ __launch_bounds__(1024) void reduce_rows_kernel(const ReduceArgs a) {
  const sca_reduce_problem& P = a.p[blockIdx.z];
  __shared__ float red[RED_WAVES][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const int i = blockIdx.y;
  float acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = 0.f;
  if (j < a.N) {
    const float* base = P.in + (long)i * a.stride_i + j;
    int s = w;
    for (; s + 7 * RED_WAVES < a.S; s += 8 * RED_WAVES) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += base[(long)(s + u * RED_WAVES) * a.stride_s];
    }
    for (; s < a.S; s += RED_WAVES) acc[0] += base[(long)s * a.stride_s];
  }
  red[w][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (w == 0 && j < a.N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < RED_WAVES; ++k) t += red[k][lane];
    t *= P.scale;
    float* o = P.out + (long)i * a.N + j;
    if (a.accumulate) t += *o;
    *o = t;
  }
}

// Few rows (S <= 16, e.g. the position-table gradient: the sum over the B clips of a
// (T, N) gradient): one thread per float4 column, the S rows summed in order — the same
// order, and so the same bits, as reduce_rows_kernel gives for S <= RED_WAVES (wave w holds
// row w alone; the wave partials are added in order); the 16-wave form left most waves
// idle and needed I x N/64 workgroups of 1024 threads.
__global__ __launch_bounds__(256) void reduce_rows_few_kernel(const ReduceArgs a) {
  const sca_reduce_problem& P = a.p[blockIdx.z];
  const int j = 4 * (blockIdx.x * 256 + threadIdx.x);
  if (j >= a.N) return;
  const float* base = P.in + (long)blockIdx.y * a.stride_i + j;
  f32x4 t = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < a.S; ++s) t += ld4(base + (long)s * a.stride_s);
  t *= P.scale;
  float* o = P.out + (long)blockIdx.y * a.N + j;
  if (a.accumulate) t += ld4(o);
  st4(o, t);
}

int launch_reduce(const ReduceArgs& a, int nprob, hipStream_t st) {
  const bool vec_ok = (a.N & 3) == 0 && (a.stride_s & 3) == 0 && (a.stride_i & 3) == 0;
  bool aligned = true;
  for (int i = 0; i < nprob; ++i)
    aligned = aligned && !((reinterpret_cast<uintptr_t>(a.p[i].in) | reinterpret_cast<uintptr_t>(a.p[i].out)) & 15);
  if (vec_ok && aligned && a.S <= RED_WAVES) {
    dim3 grid((a.N / 4 + 255) / 256, a.I, nprob);
    hipLaunchKernelGGL(reduce_rows_few_kernel, grid, dim3(256), 0, st, a);
  } else {
    dim3 grid((a.N + 63) / 64, a.I, nprob);
    hipLaunchKernelGGL(reduce_rows_kernel, grid, dim3(1024), 0, st, a);
  }
  return hipGetLastError() == hipSuccess ? SCA_OK : SCA_ERR_LAUNCH;
}

// ------------------------------------------------------------------------------ row softmax
struct SoftmaxArgs {
  sca_softmax_problem p[SCA_SOFTMAX_MAX_PROBLEMS];
  int rows, N;
};

template <int NV>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const SoftmaxArgs a) {
  using RM = RowMap<NV>;
  constexpr int V = RM::kVals;
  const sca_softmax_problem& P = a.p[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int N = a.N;
  float v[V];
  load_row<NV>(v, P.x + (long)row * N, lane, N);
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < V; ++i)
    if (NV > 0 || RM::col(lane, i) < N) m = fmaxf(m, v[i]);
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const bool in = NV > 0 || RM::col(lane, i) < N;
    v[i] = in ? __expf(v[i] - m) : 0.f;
    s += v[i];
  }
  const float inv = 1.0f / wave_sum(s);
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] *= inv;
  store_row<NV>(P.out + (long)row * N, v, lane, N);
}

template <int NV>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const SoftmaxArgs a) {
  using RM = RowMap<NV>;
  constexpr int V = RM::kVals;
  const sca_softmax_problem& P = a.p[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int N = a.N;
  float y[V], g[V];
  load_row<NV>(y, P.y + (long)row * N, lane, N);
  load_row<NV>(g, P.dy + (long)row * N, lane, N);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) s += y[i] * g[i];
  s = wave_sum(s);
#pragma unroll
  for (int i = 0; i < V; ++i) g[i] = y[i] * (g[i] - s);
  store_row<NV>(P.out + (long)row * N, g, lane, N);
}

// Wide rows (N > 1024, any N): one wave per row looping over the row in 64-column strides —
// the sum, the squared deviations and the output each re-read the row (L2-resident between
// the passes); same two-pass statistics as the register kernels above.
__global__ __launch_bounds__(256) void ln_fwd_wide_kernel(const LnFwdArgs a) {
  const sca_ln_fwd_problem& P = a.p[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int N = a.N;
  const float* x = P.x + (long)row * N;
  const float* r = P.r ? P.r + rrow(row, a.r_mod, a.r_off) * N : nullptr;
  float s = 0.f;
  for (int c = lane; c < N; c += 64) s += r ? x[c] + r[c] : x[c];
  const float mean = wave_sum(s) / N;
  float q = 0.f;
  for (int c = lane; c < N; c += 64) {
    const float d = (r ? x[c] + r[c] : x[c]) - mean;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / N + a.eps);
  DropMask dm;
  if (P.drop_p > 0.f) dm.init(P.drop_seed, P.drop_p, a.drop_off);
  const float* post = P.post ? P.post + (long)row * N : nullptr;
  float* y = P.y + (long)row * N;
  for (int c = lane; c < N; c += 64) {
    float o = ((r ? x[c] + r[c] : x[c]) - mean) * rstd * P.gamma[c] + P.beta[c];
    if (post) o += post[c];
    if (P.act == SCA_ACT_RELU) o = fmaxf(o, 0.f);
    if (P.drop_p > 0.f) o = dm.apply((uint32_t)row * (uint32_t)N + (uint32_t)c, o);
    y[c] = o;
  }
  if (lane == 0) {
    P.mean[row] = mean;
    P.rstd[row] = rstd;
  }
}

// Wide-row backward: a workgroup takes LN_BWD_ROWS rows; phase 1 (one wave per row) the two
// row sums of dy*gamma and dy*gamma*x-hat, phase 2 (thread per column, rows in order) dx and
// the workgroup's dgamma / dbeta partial row.
__global__ __launch_bounds__(256) void ln_bwd_wide_kernel(const LnBwdArgs a) {
  const sca_ln_bwd_problem& P = a.p[blockIdx.y];
  __shared__ float st[2][LN_BWD_ROWS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int N = a.N;
  const int rbeg = blockIdx.x * LN_BWD_ROWS;
  auto gated = [&](int row, int c) {  // dy with the ReLU gate (threshold_backward: out > 0)
    const float d = P.dy[(long)row * N + c];
    return P.act && !(P.y[(long)row * N + c] > 0.f) ? 0.f : d;
  };
  auto xin = [&](int row, int c) {
    const float v = P.x[(long)row * N + c];
    return P.r ? v + P.r[rrow(row, a.r_mod, a.r_off) * N + c] : v;
  };
  for (int rr = w; rr < LN_BWD_ROWS; rr += 4) {
    const int row = rbeg + rr;
    if (row >= a.rows) break;
    const float mean = P.mean[row], rstd = P.rstd[row];
    float sg = 0.f, sgx = 0.f;
    for (int c = lane; c < N; c += 64) {
      const float d = gated(row, c);
      if (P.dpost) P.dpost[(long)row * N + c] = d;
      const float g = d * P.gamma[c];
      sg += g;
      sgx += g * (xin(row, c) - mean) * rstd;
    }
    sg = wave_sum(sg);
    sgx = wave_sum(sgx);
    if (lane == 0) {
      st[0][rr] = sg / N;
      st[1][rr] = sgx / N;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += 256) {
    const float gam = P.gamma[c];
    float pg = 0.f, pb = 0.f;
    for (int rr = 0; rr < LN_BWD_ROWS; ++rr) {
      const int row = rbeg + rr;
      if (row >= a.rows) break;
      const float d = gated(row, c);
      const float xh = (xin(row, c) - P.mean[row]) * P.rstd[row];
      float dx = P.rstd[row] * (d * gam - st[0][rr] - xh * st[1][rr]);
      float* dxp = P.dx + (long)row * N + c;
      if (a.accumulate) dx += *dxp;
      *dxp = dx;
      pg += d * xh;
      pb += d;
    }
    P.partial[(long)blockIdx.x * N + c] = pg;
    P.partial[((long)a.nblk + blockIdx.x) * N + c] = pb;
  }
}

// Wide-row softmax (N > 1024): one wave per row, max / sum / output passes over the row.
__global__ __launch_bounds__(256) void softmax_fwd_wide_kernel(const SoftmaxArgs a) {
  const sca_softmax_problem& P = a.p[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int N = a.N;
  const float* x = P.x + (long)row * N;
  float m = -INFINITY;
  for (int c = lane; c < N; c += 64) m = fmaxf(m, x[c]);
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < N; c += 64) s += __expf(x[c] - m);
  const float inv = 1.0f / wave_sum(s);
  float* o = P.out + (long)row * N;
  for (int c = lane; c < N; c += 64) o[c] = __expf(x[c] - m) * inv;
}

__global__ __launch_bounds__(256) void softmax_bwd_wide_kernel(const SoftmaxArgs a) {
  const sca_softmax_problem& P = a.p[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int N = a.N;
  const float* y = P.y + (long)row * N;
  const float* g = P.dy + (long)row * N;
  float s = 0.f;
  for (int c = lane; c < N; c += 64) s += y[c] * g[c];
  s = wave_sum(s);
  float* o = P.out + (long)row * N;
  for (int c = lane; c < N; c += 64) o[c] = y[c] * (g[c] - s);
}

// ------------------------------------------------------------------------------ GELU backward
struct GeluArgs {
  sca_gelu_bwd_problem p[SCA_GELU_MAX_PROBLEMS];
  long n;
};

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const GeluArgs a) {
  const sca_gelu_bwd_problem& P = a.p[blockIdx.y];
  const long n4 = a.n / 4;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n4; e += (long)gridDim.x * 256) {
    const f32x4 dy = ld4(P.dy + 4 * e), z = ld4(P.z + 4 * e);
    f32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = dy[j] * gelu_erf_grad(z[j]);
    st4(P.dz + 4 * e, r);
  }
  for (long e = 4 * n4 + (long)blockIdx.x * 256 + threadIdx.x; e < a.n; e += (long)gridDim.x * 256)
    P.dz[e] = P.dy[e] * gelu_erf_grad(P.z[e]);
}

// ------------------------------------------------------------------------------ fixed-order tensor sum
struct SumArgs {
  sca_sum_problem p[SCA_SUM_MAX_PROBLEMS];
  long n;
};

__global__ __launch_bounds__(256) void sum_tensors_kernel(const SumArgs a) {
  const sca_sum_problem& P = a.p[blockIdx.y];
  const long n4 = a.n / 4;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n4; e += (long)gridDim.x * 256) {
    f32x4 s = ld4(P.in[0] + 4 * e);
    for (int j = 1; j < P.nin; ++j) s += ld4(P.in[j] + 4 * e);
    st4(P.out + 4 * e, s);
  }
  for (long e = 4 * n4 + (long)blockIdx.x * 256 + threadIdx.x; e < a.n; e += (long)gridDim.x * 256) {
    float s = P.in[0][e];
    for (int j = 1; j < P.nin; ++j) s += P.in[j][e];
    P.out[e] = s;
  }
}

// ------------------------------------------------------------------------------ MaxPool1d(2,2) over T
struct PoolArgs {
  sca_pool_problem p[SCA_POOL_MAX_PROBLEMS];
  int B, T, C;
};

__global__ __launch_bounds__(256) void maxpool_t_fwd_kernel(const PoolArgs a) {
  const sca_pool_problem& P = a.p[blockIdx.y];
  const int To = a.T / 2;
  const long n = (long)a.B * To * a.C;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % a.C);
    const long bt = e / a.C;
    const int t = (int)(bt % To), b = (int)(bt / To);
    const float* src = P.x + ((long)b * a.T + 2 * t) * a.C + c;
    const float x0 = src[0], x1 = src[a.C];
    P.y[e] = (x1 > x0) ? x1 : x0;
  }
}

__global__ __launch_bounds__(256) void maxpool_t_bwd_kernel(const PoolArgs a) {
  const sca_pool_problem& P = a.p[blockIdx.y];
  const int To = a.T / 2;
  const long n = (long)a.B * a.T * a.C;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % a.C);
    const long bt = e / a.C;
    const int t = (int)(bt % a.T), b = (int)(bt / a.T);
    float g = 0.f;
    const int to = t >> 1;
    if (to < To) {
      const float* src = P.x + ((long)b * a.T + 2 * to) * a.C + c;
      const float x0 = src[0], x1 = src[a.C];
      const bool second = x1 > x0;
      if ((t & 1) == (second ? 1 : 0)) g = P.dy[((long)b * To + to) * a.C + c];
    }
    P.dx[e] = g;
  }
}

// ------------------------------------------------------------------------------ coordinate mapping
struct MapArgs {
  sca_coord_map_problem p[SCA_MAP_MAX_PROBLEMS];
  int rows, K_all, N;
};
struct MapBwdArgs {
  sca_coord_map_bwd_problem p[SCA_MAP_MAX_PROBLEMS];
  int rows, K_all, N, nchunk;
};

constexpr int MAP_ROWS = 16;   // rows per workgroup (forward)
constexpr int MAP_KMAX = 136;  // max joints per stream (K=133 COCO-WholeBody face+body fits)
constexpr int MAP_CHUNK = 32;  // rows per partial (backward)

// Gather this workgroup's rows' joints into LDS: xs[r][k], ys[r][k].
__device__ __forceinline__ void gather_coords(float (*xs)[MAP_KMAX], float (*ys)[MAP_KMAX], const float* kp,
                                              const int* idx, int K, int K_all, int row0, int nrows, int rows) {
  for (int e = threadIdx.x; e < nrows * K; e += blockDim.x) {
    const int r = e / K, k = e % K;
    const int row = row0 + r;
    float x = 0.f, y = 0.f;
    if (row < rows) {
      const float* src = kp + ((long)row * K_all + idx[k]) * 2;
      x = src[0];
      y = src[1];
    }
    xs[r][k] = x;
    ys[r][k] = y;
  }
}

// The weights (N x K row-major, K = the stream's joint count: rows not float4-aligned) are
// staged through LDS in chunks of MAP_KC joints, transposed to [joint][column]: the chunk is
// read with consecutive lanes on consecutive joints of one weight row (64-B runs), where a
// thread reading its own row touched one cache line per lane per load; each thread then reads
// its column conflict-free.  Same k order per output: bit-identical to the direct form.
constexpr int MAP_KC = 16, MAP_WLD = 257;
__global__ __launch_bounds__(256) void coord_map_fwd_kernel(const MapArgs a) {
  const sca_coord_map_problem& P = a.p[blockIdx.y];
  __shared__ float xs[MAP_ROWS][MAP_KMAX], ys[MAP_ROWS][MAP_KMAX];
  __shared__ float wsx[MAP_KC][MAP_WLD], wsy[MAP_KC][MAP_WLD];
  const int row0 = blockIdx.x * MAP_ROWS;
  const int K = P.K;
  gather_coords(xs, ys, P.kp, P.idx, K, a.K_all, row0, MAP_ROWS, a.rows);
  for (int n0 = 0; n0 < a.N; n0 += 256) {
    const int n = n0 + threadIdx.x;
    float ax[MAP_ROWS], ay[MAP_ROWS];
#pragma unroll
    for (int r = 0; r < MAP_ROWS; ++r) ax[r] = ay[r] = 0.f;
    for (int k0 = 0; k0 < K; k0 += MAP_KC) {
      __syncthreads();  // the previous chunk consumed (first pass: the gather landed)
      // every load of the chunk issued before any is used: addresses past the weight are
      // clamped to its last element (always valid) and their values zeroed by a select
      constexpr int PER = 256 * MAP_KC / 256;
      float vx[PER], vy[PER];
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = threadIdx.x + 256 * i, nn = e / MAP_KC, kk = e % MAP_KC;
        const long off = min((long)(n0 + nn) * K + k0 + kk, (long)a.N * K - 1);
        vx[i] = P.wx[off];
        vy[i] = P.wy[off];
      }
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = threadIdx.x + 256 * i, nn = e / MAP_KC, kk = e % MAP_KC;
        const bool in = n0 + nn < a.N && k0 + kk < K;
        wsx[kk][nn] = in ? vx[i] : 0.f;
        wsy[kk][nn] = in ? vy[i] : 0.f;
      }
      __syncthreads();
      const int kc = min(MAP_KC, K - k0);
#pragma unroll
      for (int j = 0; j < MAP_KC; ++j) {
        if (j >= kc) break;  // wave-uniform
        const float wx = wsx[j][threadIdx.x], wy = wsy[j][threadIdx.x];
#pragma unroll
        for (int r = 0; r < MAP_ROWS; ++r) {
          ax[r] = fmaf(xs[r][k0 + j], wx, ax[r]);
          ay[r] = fmaf(ys[r][k0 + j], wy, ay[r]);
        }
      }
    }
    if (n >= a.N) continue;
    const float bx = P.bx ? P.bx[n] : 0.f, by = P.by ? P.by[n] : 0.f;
#pragma unroll
    for (int r = 0; r < MAP_ROWS; ++r) {
      const int row = row0 + r;
      if (row < a.rows) {
        P.xe[(long)row * a.N + n] = ax[r] + bx;
        P.ye[(long)row * a.N + n] = ay[r] + by;
      }
    }
  }
}

// Partial weight gradients: partial[c][chunk][k][n] = sum_{rows in chunk} d{x,y}e[row][n] * {x,y}[row][k]
// A thread owns one column n: the chunk's 2 x MAP_CHUNK gradient values are loaded into
// registers up front (one round of loads in flight, not one dependent load per row), then
// every joint's dot product runs out of registers and the LDS coordinates.
__global__ __launch_bounds__(256) void coord_map_bwd_w_kernel(const MapBwdArgs a) {
  const sca_coord_map_bwd_problem& P = a.p[blockIdx.y];
  __shared__ __attribute__((aligned(16))) float xs[MAP_CHUNK][MAP_KMAX], ys[MAP_CHUNK][MAP_KMAX];
  const int row0 = blockIdx.x * MAP_CHUNK;
  const int K = P.K;
  const int nr = min(MAP_CHUNK, a.rows - row0);
  gather_coords(xs, ys, P.kp, P.idx, K, a.K_all, row0, MAP_CHUNK, a.rows);
  constexpr int KC = 8;
  const int Kp = (K + KC - 1) / KC * KC;  // joints padded to whole float4 pairs (zeros)
  for (int e = threadIdx.x; e < MAP_CHUNK * (Kp - K); e += 256) {
    const int r = e / (Kp - K), k = K + e % (Kp - K);
    xs[r][k] = 0.f;
    ys[r][k] = 0.f;
  }
  __syncthreads();
  for (int n = threadIdx.x; n < a.N; n += 256) {
    float dx[MAP_CHUNK], dy[MAP_CHUNK];
#pragma unroll
    for (int r = 0; r < MAP_CHUNK; ++r) {
      const long off = (long)(row0 + min(r, nr - 1)) * a.N + n;
      dx[r] = r < nr ? P.dxe[off] : 0.f;
      dy[r] = r < nr ? P.dye[off] : 0.f;
    }
    // partial layout [chunk][k][n]: the lanes' stores (consecutive n) are coalesced
    float* px = P.partial + (long)blockIdx.x * a.N * K + n;
    float* py = P.partial + (long)(a.nchunk + blockIdx.x) * a.N * K + n;
    for (int kc = 0; kc < K; kc += KC) {
      float gx[KC], gy[KC];
#pragma unroll
      for (int j = 0; j < KC; ++j) gx[j] = gy[j] = 0.f;
#pragma unroll 8
      for (int r = 0; r < MAP_CHUNK; ++r) {  // rows >= nr carry zero gradients; joints >= K are never stored
        const f32x4 x0 = ld4(&xs[r][kc]), x1 = ld4(&xs[r][kc + 4]);  // broadcast float4 LDS reads
        const f32x4 y0 = ld4(&ys[r][kc]), y1 = ld4(&ys[r][kc + 4]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          gx[j] = fmaf(dx[r], x0[j], gx[j]);
          gx[j + 4] = fmaf(dx[r], x1[j], gx[j + 4]);
          gy[j] = fmaf(dy[r], y0[j], gy[j]);
          gy[j + 4] = fmaf(dy[r], y1[j], gy[j + 4]);
        }
      }
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        if (kc + j < K) {
          px[(long)(kc + j) * a.N] = gx[j];
          py[(long)(kc + j) * a.N] = gy[j];
        }
      }
    }
  }
}

// dW{x,y} = fixed-order sum of the chunk partials, every problem (per-problem K) in one launch
__global__ __launch_bounds__(256) void coord_map_reduce_kernel(const MapBwdArgs a) {
  const sca_coord_map_bwd_problem& P = a.p[blockIdx.z];
  const long NK = (long)a.N * P.K;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;  // partial index k * N + n (coalesced reads)
  if (e >= NK) return;
  const float* src = P.partial + (long)blockIdx.y * a.nchunk * NK + e;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  int c = 0;
  for (; c + 3 < a.nchunk; c += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] += src[(long)(c + u) * NK];
  }
  for (; c < a.nchunk; ++c) acc[0] += src[(long)c * NK];
  const long k = e / a.N, n = e % a.N;
  (blockIdx.y ? P.dwy : P.dwx)[n * P.K + k] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// Keypoint gradients (only when the keypoints require grad): one wave per row.
__global__ __launch_bounds__(256) void coord_map_bwd_kp_kernel(const MapBwdArgs a) {
  const sca_coord_map_bwd_problem& P = a.p[blockIdx.y];
  if (!P.dkp) return;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const float* dxr = P.dxe + (long)row * a.N;
  const float* dyr = P.dye + (long)row * a.N;
  for (int k = lane; k < P.K; k += 64) {
    float sx = 0.f, sy = 0.f;
    for (int n = 0; n < a.N; ++n) {
      sx = fmaf(dxr[n], P.wx[(long)n * P.K + k], sx);
      sy = fmaf(dyr[n], P.wy[(long)n * P.K + k], sy);
    }
    float* dst = P.dkp + ((long)row * a.K_all + P.idx[k]) * 2;
    atomicAdd(dst, sx);
    atomicAdd(dst + 1, sy);
  }
}

// ------------------------------------------------------------------------------ input contract
// SLR_Dataset.normalize_keypoints (dataset.py:134-170) on the padded batch: one wave per
// frame, the frame's joints staged in LDS, parts processed in order (a later part sees an
// earlier part's result, exactly as the reference's in-place loop), wave min / max
// reductions for the box.
constexpr int NORM_KMAX = 1024;

struct NormArgs {
  const float* in;
  float* out;
  const int* lengths;
  const int* part_off;
  const int* part_idx;
  int B, T, K_all, nparts;
  const int* src_row;   // prepare: row of `in` holding frame (b, t) (frame selection), or NULL: in is (B, T, ...)
  const float* affine;  // prepare: per clip [a00 a01 tx a10 a11 ty] (augmentation), or NULL
};

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ __launch_bounds__(256) void normalize_parts_kernel(const NormArgs a) {
  __shared__ __attribute__((aligned(16))) float fr[4][2 * NORM_KMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long frame = (long)blockIdx.x * 4 + w;
  if (frame >= (long)a.B * a.T) return;
  const int b = (int)(frame / a.T), t = (int)(frame % a.T);
  const int n2 = 2 * a.K_all;
  float* dst = a.out + frame * n2;
  if (t >= a.lengths[b]) {  // collator padding
    for (int e = lane; e < n2; e += 64) dst[e] = 0.f;
    return;
  }
  // frame selection (dataset.py:185-215): the selected source row; augmentation
  // (dataset.py:172-183, augmentation.py): x' = a00 x + a01 y + tx, y' = a10 x + a11 y + ty
  const float* src = a.in + (a.src_row ? (long)a.src_row[frame] : frame) * n2;
  float* F = fr[w];
  if (a.affine) {
    const float* m = a.affine + 6 * b;
    const float a00 = m[0], a01 = m[1], tx = m[2], a10 = m[3], a11 = m[4], ty = m[5];
    for (int k = lane; k < a.K_all; k += 64) {
      const float x = src[2 * k], y = src[2 * k + 1];
      F[2 * k] = fmaf(a00, x, fmaf(a01, y, tx));
      F[2 * k + 1] = fmaf(a10, x, fmaf(a11, y, ty));
    }
  } else {
    for (int e = lane; e < n2; e += 64) F[e] = src[e];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int p = 0; p < a.nparts; ++p) {
    const int j0 = a.part_off[p], j1 = a.part_off[p + 1];
    float mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
    for (int j = j0 + lane; j < j1; j += 64) {
      const int k = a.part_idx[j];
      mnx = fminf(mnx, F[2 * k]);
      mxx = fmaxf(mxx, F[2 * k]);
      mny = fminf(mny, F[2 * k + 1]);
      mxy = fmaxf(mxy, F[2 * k + 1]);
    }
    mnx = wave_min(mnx);
    mny = wave_min(mny);
    mxx = wave_max(mxx);
    mxy = wave_max(mxy);
    const float wd = mxx - mnx, ht = mxy - mny;
    float dx, dy;
    if (wd > ht) {
      dx = 0.05f * wd;
      dy = dx + (wd - ht) / 2.0f;
    } else {
      dy = 0.05f * ht;
      dx = dy + (ht - wd) / 2.0f;
    }
    const float s0 = fmaxf(0.f, fminf(mnx - dx, 1.f)), s1 = fmaxf(0.f, fminf(mny - dy, 1.f));
    const float e0 = fmaxf(0.f, fminf(mxx + dx, 1.f)), e1 = fmaxf(0.f, fminf(mxy + dy, 1.f));
    const float ex = e0 - s0, ey = e1 - s1;
    for (int j = j0 + lane; j < j1; j += 64) {
      const int k = a.part_idx[j];
      if (ex != 0.f) F[2 * k] = (F[2 * k] - s0) / ex;
      if (ey != 0.f) F[2 * k + 1] = (F[2 * k + 1] - s1) / ey;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the next part may share joints
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  for (int e = lane; e < n2; e += 64) dst[e] = F[e];
}

// ------------------------------------------------------------------------------ dropout
struct DropArgs {
  sca_dropout_problem p[SCA_DROPOUT_MAX_PROBLEMS];
  long n;
  float prob;
  const unsigned long long* drop_off;
};

__global__ __launch_bounds__(256) void dropout_kernel(const DropArgs a) {
  const sca_dropout_problem& P = a.p[blockIdx.y];
  DropMask dm;
  dm.init(P.seed, a.prob, a.drop_off);
  const long n4 = a.n >> 2;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    f32x4 v = ld4(P.x + 4 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = dm.apply((uint32_t)(4 * i + j), v[j]);
    st4(P.y + 4 * i, v);
  }
  for (long e = 4 * n4 + (long)blockIdx.x * 256 + threadIdx.x; e < a.n; e += (long)gridDim.x * 256)
    P.y[e] = dm.apply((uint32_t)e, P.x[e]);
}

// ------------------------------------------------------------------------------ key validity
// (model/utils.py:8-12, 19-23: 1.0 - mask.to(fp32) masks every non-zero, so only 1 keeps)
struct KeyValidArgs {
  const void* mask;
  float* out;
  long n;
  int dtype;
};

__device__ __forceinline__ float mask_value(const void* m, int dtype, long i) {
  switch (dtype) {
    case SCA_MASK_F64: return (float)static_cast<const double*>(m)[i];
    case SCA_MASK_I64: return (float)static_cast<const long long*>(m)[i];
    case SCA_MASK_I32: return (float)static_cast<const int*>(m)[i];
    case SCA_MASK_U8: return (float)static_cast<const unsigned char*>(m)[i];
    case SCA_MASK_F16: return (float)static_cast<const _Float16*>(m)[i];
    case SCA_MASK_BF16: return __uint_as_float((uint32_t)static_cast<const unsigned short*>(m)[i] << 16);
    case SCA_MASK_I8: return (float)static_cast<const signed char*>(m)[i];
    case SCA_MASK_I16: return (float)static_cast<const short*>(m)[i];
    default: return static_cast<const float*>(m)[i];
  }
}

__global__ __launch_bounds__(256) void key_valid_kernel(const KeyValidArgs a) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (long)gridDim.x * 256)
    a.out[i] = mask_value(a.mask, a.dtype, i) == 1.f ? 1.f : 0.f;
}

}  // namespace

// ------------------------------------------------------------------------------ C ABI
extern "C" void sca_set_error(const char* msg);

extern "C" int sca_layernorm_fwd(int nprob, const sca_ln_fwd_problem* probs, int rows, int N, int r_mod,
                                 int r_off, float eps, void* stream) {
  if (nprob < 1 || nprob > SCA_LN_MAX_PROBLEMS || N < 1 || rows < 0 || r_mod < 1) {
    sca_set_error("sca_layernorm_fwd: bad arguments");
    return SCA_ERR_ARG;
  }
  if (rows == 0) return SCA_OK;
  LnFwdArgs a;
  for (int i = 0; i < nprob; ++i) {
    a.p[i] = probs[i];
    if (!(probs[i].drop_p >= 0.f && probs[i].drop_p < 1.f) || (probs[i].drop_p > 0.f && probs[i].act != SCA_ACT_NONE)) {
      sca_set_error("sca_layernorm_fwd: drop_p must be in [0, 1) and needs act == SCA_ACT_NONE");
      return SCA_ERR_ARG;
    }
  }
  a.rows = rows; a.N = N; a.r_mod = r_mod; a.r_off = r_off; a.eps = eps;
  a.drop_off = sca_drop_offset_ptr();
  dim3 grid((rows + 3) / 4, nprob);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (N > 64 * LN_MAXV ? -1 : N % 256 == 0 ? N / 256 : 0) {
    case -1: hipLaunchKernelGGL(ln_fwd_wide_kernel, grid, dim3(256), 0, st, a); break;
    case 1: hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL(ln_fwd_kernel<2>, grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL(ln_fwd_kernel<3>, grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(ln_fwd_kernel<0>, grid, dim3(256), 0, st, a); break;
  }
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_layernorm_fwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_maxpool_t_fwd(int nprob, const sca_pool_problem* probs, int B, int T, int C, void* stream) {
  if (nprob < 1 || nprob > SCA_POOL_MAX_PROBLEMS || B < 0 || T < 0 || C < 1) {
    sca_set_error("sca_maxpool_t_fwd: bad arguments");
    return SCA_ERR_ARG;
  }
  PoolArgs a;
  for (int i = 0; i < nprob; ++i) a.p[i] = probs[i];
  a.B = B; a.T = T; a.C = C;
  const long n = (long)B * (T / 2) * C;
  if (n == 0) return SCA_OK;
  const int blocks = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(maxpool_t_fwd_kernel, dim3(blocks, nprob), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_maxpool_t_fwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_maxpool_t_bwd(int nprob, const sca_pool_problem* probs, int B, int T, int C, void* stream) {
  if (nprob < 1 || nprob > SCA_POOL_MAX_PROBLEMS || B < 0 || T < 0 || C < 1) {
    sca_set_error("sca_maxpool_t_bwd: bad arguments");
    return SCA_ERR_ARG;
  }
  PoolArgs a;
  for (int i = 0; i < nprob; ++i) a.p[i] = probs[i];
  a.B = B; a.T = T; a.C = C;
  const long n = (long)B * T * C;
  if (n == 0) return SCA_OK;
  const int blocks = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(maxpool_t_bwd_kernel, dim3(blocks, nprob), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_maxpool_t_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

template <bool BWD>
int launch_softmax(int nprob, const sca_softmax_problem* probs, int rows, int N, void* stream, const char* what) {
  if (nprob < 1 || nprob > SCA_SOFTMAX_MAX_PROBLEMS || rows < 0 || N < 1) {
    sca_set_error(what);
    return SCA_ERR_ARG;
  }
  if (rows == 0) return SCA_OK;
  SoftmaxArgs a;
  for (int i = 0; i < nprob; ++i) a.p[i] = probs[i];
  a.rows = rows;
  a.N = N;
  dim3 grid((rows + 3) / 4, nprob);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nv = N % 256 == 0 ? N / 256 : 0;
#define SCA_SM(NVV)                                                                   \
  if (BWD) hipLaunchKernelGGL(softmax_bwd_kernel<NVV>, grid, dim3(256), 0, st, a);   \
  else hipLaunchKernelGGL(softmax_fwd_kernel<NVV>, grid, dim3(256), 0, st, a);
  if (N > 64 * LN_MAXV) {
    if (BWD) hipLaunchKernelGGL(softmax_bwd_wide_kernel, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(softmax_fwd_wide_kernel, grid, dim3(256), 0, st, a);
  } else switch (nv) {
    case 1: SCA_SM(1) break;
    case 2: SCA_SM(2) break;
    case 3: SCA_SM(3) break;
    case 4: SCA_SM(4) break;
    default: SCA_SM(0) break;
  }
#undef SCA_SM
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_softmax_rows: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_softmax_rows_fwd(int nprob, const sca_softmax_problem* probs, int rows, int N, void* stream) {
  return launch_softmax<false>(nprob, probs, rows, N, stream, "sca_softmax_rows_fwd: bad arguments");
}

extern "C" int sca_softmax_rows_bwd(int nprob, const sca_softmax_problem* probs, int rows, int N, void* stream) {
  return launch_softmax<true>(nprob, probs, rows, N, stream, "sca_softmax_rows_bwd: bad arguments");
}

extern "C" int sca_gelu_bwd(int nprob, const sca_gelu_bwd_problem* probs, long n, void* stream) {
  if (nprob < 1 || nprob > SCA_GELU_MAX_PROBLEMS || n < 0) {
    sca_set_error("sca_gelu_bwd: bad arguments");
    return SCA_ERR_ARG;
  }
  if (n == 0) return SCA_OK;
  GeluArgs a;
  for (int i = 0; i < nprob; ++i) {
    a.p[i] = probs[i];
    if ((reinterpret_cast<uintptr_t>(probs[i].dy) | reinterpret_cast<uintptr_t>(probs[i].z) |
         reinterpret_cast<uintptr_t>(probs[i].dz)) & 15) {
      sca_set_error("sca_gelu_bwd: pointers must be 16-byte aligned");
      return SCA_ERR_ARG;
    }
  }
  a.n = n;
  const long blocks = (n / 4 + 255) / 256;
  dim3 grid((unsigned)(blocks < 2048 ? (blocks > 0 ? blocks : 1) : 2048), nprob);
  hipLaunchKernelGGL(gelu_bwd_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_gelu_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_sum_tensors(int nprob, const sca_sum_problem* probs, long n, void* stream) {
  if (nprob < 1 || nprob > SCA_SUM_MAX_PROBLEMS || n < 0 || !probs) {
    sca_set_error("sca_sum_tensors: bad arguments");
    return SCA_ERR_ARG;
  }
  SumArgs a;
  for (int i = 0; i < nprob; ++i) {
    const sca_sum_problem& P = probs[i];
    uintptr_t al = reinterpret_cast<uintptr_t>(P.out);
    bool ok = P.nin >= 1 && P.nin <= SCA_SUM_MAX_TERMS && P.out;
    for (int j = 0; ok && j < P.nin; ++j) {
      ok = P.in[j] != nullptr;
      al |= reinterpret_cast<uintptr_t>(P.in[j]);
    }
    if (!ok || (al & 15)) {
      sca_set_error("sca_sum_tensors: 1..8 non-null, 16-byte aligned inputs and an output per problem");
      return SCA_ERR_ARG;
    }
    a.p[i] = P;
  }
  if (n == 0) return SCA_OK;
  a.n = n;
  const long blocks = (n / 4 + 255) / 256;
  dim3 grid((unsigned)(blocks < 1024 ? (blocks > 0 ? blocks : 1) : 1024), nprob);
  hipLaunchKernelGGL(sum_tensors_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_sum_tensors: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_layernorm_bwd_blocks(int rows) { return (rows + LN_BWD_ROWS - 1) / LN_BWD_ROWS; }

extern "C" int sca_layernorm_bwd(int nprob, const sca_ln_bwd_problem* probs, int rows, int N, int r_mod,
                                 int r_off, int accumulate, void* stream) {
  if (nprob < 1 || nprob > SCA_LN_MAX_PROBLEMS || N < 1 || rows < 1 || r_mod < 1) {
    sca_set_error("sca_layernorm_bwd: bad arguments");
    return SCA_ERR_ARG;
  }
  LnBwdArgs a;
  for (int i = 0; i < nprob; ++i) a.p[i] = probs[i];
  a.rows = rows; a.N = N; a.r_mod = r_mod; a.r_off = r_off; a.accumulate = accumulate;
  a.nblk = sca_layernorm_bwd_blocks(rows);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (N > 64 * LN_MAXV ? -1 : N % 256 == 0 ? N / 256 : 0) {
    case -1: hipLaunchKernelGGL(ln_bwd_wide_kernel, dim3(a.nblk, nprob), dim3(256), 0, st, a); break;
    case 1: hipLaunchKernelGGL(ln_bwd_kernel<1>, dim3(a.nblk, nprob), dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL(ln_bwd_kernel<2>, dim3(a.nblk, nprob), dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL(ln_bwd_kernel<3>, dim3(a.nblk, nprob), dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL(ln_bwd_kernel<4>, dim3(a.nblk, nprob), dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(ln_bwd_kernel<0>, dim3(a.nblk, nprob), dim3(256), 0, st, a); break;
  }
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_layernorm_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  // dgamma / dbeta = fixed-order sums of the per-workgroup partial rows (problems with
  // dgamma == NULL leave them in `partial` for the caller's own sca_reduce_rows)
  ReduceArgs r;
  int np = 0;
  for (int i = 0; i < nprob; ++i) {
    if (!probs[i].dgamma) continue;
    r.p[np++] = sca_reduce_problem{probs[i].partial, probs[i].dgamma, 1.0f};
    r.p[np++] = sca_reduce_problem{probs[i].partial + (long)a.nblk * N, probs[i].dbeta, 1.0f};
  }
  r.S = a.nblk; r.I = 1; r.N = N; r.accumulate = 0; r.stride_s = N; r.stride_i = 0;
  if (np && launch_reduce(r, np, st) != SCA_OK) {
    sca_set_error("sca_layernorm_bwd: reduce launch failed");
    return SCA_ERR_LAUNCH;
  }
  return SCA_OK;
}

extern "C" int sca_reduce_rows(int nprob, const sca_reduce_problem* probs, int S, int I, int N, long stride_s,
                               long stride_i, int accumulate, void* stream) {
  if (nprob < 1 || nprob > SCA_REDUCE_MAX_PROBLEMS || S < 0 || I < 1 || N < 1) {
    sca_set_error("sca_reduce_rows: bad arguments");
    return SCA_ERR_ARG;
  }
  ReduceArgs r;
  for (int i = 0; i < nprob; ++i) r.p[i] = probs[i];
  r.S = S; r.I = I; r.N = N; r.accumulate = accumulate; r.stride_s = stride_s; r.stride_i = stride_i;
  if (launch_reduce(r, nprob, reinterpret_cast<hipStream_t>(stream)) != SCA_OK) {
    sca_set_error("sca_reduce_rows: launch failed");
    return SCA_ERR_LAUNCH;
  }
  return SCA_OK;
}

extern "C" int sca_coord_map_fwd(int nprob, const sca_coord_map_problem* probs, int rows, int K_all, int N,
                                 void* stream) {
  if (nprob < 1 || nprob > SCA_MAP_MAX_PROBLEMS || rows < 0 || N < 1) {
    sca_set_error("sca_coord_map_fwd: bad arguments");
    return SCA_ERR_ARG;
  }
  MapArgs a;
  for (int i = 0; i < nprob; ++i) {
    if (probs[i].K < 1 || probs[i].K > MAP_KMAX) { sca_set_error("sca_coord_map_fwd: K must be 1..136"); return SCA_ERR_ARG; }
    a.p[i] = probs[i];
  }
  if (rows == 0) return SCA_OK;
  a.rows = rows; a.K_all = K_all; a.N = N;
  dim3 grid((rows + MAP_ROWS - 1) / MAP_ROWS, nprob);
  hipLaunchKernelGGL(coord_map_fwd_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_coord_map_fwd: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_coord_map_bwd_chunks(int rows) { return (rows + MAP_CHUNK - 1) / MAP_CHUNK; }

extern "C" int sca_coord_map_bwd(int nprob, const sca_coord_map_bwd_problem* probs, int rows, int K_all, int N,
                                 void* stream) {
  if (nprob < 1 || nprob > SCA_MAP_MAX_PROBLEMS || rows < 1 || N < 1) {
    sca_set_error("sca_coord_map_bwd: bad arguments");
    return SCA_ERR_ARG;
  }
  MapBwdArgs a;
  for (int i = 0; i < nprob; ++i) {
    if (probs[i].K < 1 || probs[i].K > MAP_KMAX) { sca_set_error("sca_coord_map_bwd: K must be 1..136"); return SCA_ERR_ARG; }
    a.p[i] = probs[i];
  }
  a.rows = rows; a.K_all = K_all; a.N = N; a.nchunk = sca_coord_map_bwd_chunks(rows);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(coord_map_bwd_w_kernel, dim3(a.nchunk, nprob), dim3(256), 0, st, a);
  bool any_dkp = false;
  for (int i = 0; i < nprob; ++i) any_dkp |= probs[i].dkp != nullptr;
  if (any_dkp) hipLaunchKernelGGL(coord_map_bwd_kp_kernel, dim3((rows + 3) / 4, nprob), dim3(256), 0, st, a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_coord_map_bwd: launch failed"); return SCA_ERR_LAUNCH; }
  // dW = fixed-order sum over row chunks, all problems in one launch
  int maxK = 0;
  for (int i = 0; i < nprob; ++i) maxK = maxK > probs[i].K ? maxK : probs[i].K;
  hipLaunchKernelGGL(coord_map_reduce_kernel, dim3((unsigned)(((long)N * maxK + 255) / 256), 2, nprob), dim3(256), 0,
                     st, a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_coord_map_bwd: reduce launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_dropout(int nprob, const sca_dropout_problem* probs, long rows, int cols, float p, void* stream) {
  if (nprob < 1 || nprob > SCA_DROPOUT_MAX_PROBLEMS || rows < 0 || cols < 0 || !(p >= 0.f && p < 1.f)) {
    sca_set_error("sca_dropout: bad arguments (p must be in [0, 1))");
    return SCA_ERR_ARG;
  }
  DropArgs a;
  for (int i = 0; i < nprob; ++i) {
    if (!probs[i].x || !probs[i].y || (reinterpret_cast<uintptr_t>(probs[i].x) & 15) ||
        (reinterpret_cast<uintptr_t>(probs[i].y) & 15)) {
      sca_set_error("sca_dropout: x / y must be non-null and 16-byte aligned");
      return SCA_ERR_ARG;
    }
    a.p[i] = probs[i];
  }
  a.n = rows * (long)cols;
  a.prob = p;
  a.drop_off = sca_drop_offset_ptr();
  if (a.n == 0) return SCA_OK;
  const long want = (a.n / 4 + 255) / 256;
  const int blocks = (int)(want < 2048 ? (want > 0 ? want : 1) : 2048);
  hipLaunchKernelGGL(dropout_kernel, dim3(blocks, nprob), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_dropout: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_key_valid(const void* mask, int dtype, float* key_valid, long n, void* stream) {
  if (n < 0 || dtype < SCA_MASK_F32 || dtype > SCA_MASK_I16 || (n > 0 && (!mask || !key_valid))) {
    sca_set_error("sca_key_valid: bad arguments (dtype must be one of SCA_MASK_*)");
    return SCA_ERR_ARG;
  }
  if (n == 0) return SCA_OK;
  const long want = (n + 255) / 256;
  const int blocks = (int)(want < 1024 ? want : 1024);
  hipLaunchKernelGGL(key_valid_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     KeyValidArgs{mask, key_valid, n, dtype});
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_key_valid: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

// p[0 .. n) = 0: float4 stores over the 16-byte-aligned body, scalar stores at the ends
__global__ __launch_bounds__(256) void zero_kernel(float* p, long n, long head, long n4) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride)
    st4(p + head + 4 * i, f32x4{0.f, 0.f, 0.f, 0.f});
  const long tail = head + 4 * n4;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e < head) p[e] = 0.f;
  if (e < n - tail) p[tail + e] = 0.f;
}

extern "C" int sca_zero(float* p, long n, void* stream) {
  if (n < 0 || (n > 0 && !p) || (reinterpret_cast<uintptr_t>(p) & 3)) {
    sca_set_error("sca_zero: bad arguments (null or misaligned pointer, or n < 0)");
    return SCA_ERR_ARG;
  }
  if (n == 0) return SCA_OK;
  long head = (long)((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15) / 4;
  if (head > n) head = n;
  const long n4 = (n - head) / 4;
  const long want = (n4 + 255) / 256;
  const int blocks = (int)(want < 1 ? 1 : (want < 2048 ? want : 2048));
  hipLaunchKernelGGL(zero_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), p, n, head, n4);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_zero: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_normalize_parts(const float* kp_in, float* kp_out, const int* lengths, int B, int T, int K_all,
                                   const int* part_off, const int* part_idx, int nparts, void* stream) {
  if (B < 0 || T < 0 || K_all < 1 || K_all > NORM_KMAX || nparts < 0 || !kp_in || !kp_out || !lengths ||
      (nparts > 0 && (!part_off || !part_idx))) {
    sca_set_error("sca_normalize_parts: bad arguments (K_all must be 1..1024)");
    return SCA_ERR_ARG;
  }
  const long frames = (long)B * T;
  if (frames == 0) return SCA_OK;
  NormArgs a{kp_in, kp_out, lengths, part_off, part_idx, B, T, K_all, nparts, nullptr, nullptr};
  hipLaunchKernelGGL(normalize_parts_kernel, dim3((unsigned)((frames + 3) / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_normalize_parts: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}

extern "C" int sca_prepare_keypoints(const float* raw, const int* src_row, const float* affine, const int* lengths,
                                     float* kp_out, int B, int T, int K_all, const int* part_off, const int* part_idx,
                                     int nparts, void* stream) {
  if (B < 0 || T < 0 || K_all < 1 || K_all > NORM_KMAX || nparts < 0 || !raw || !src_row || !kp_out || !lengths ||
      (nparts > 0 && (!part_off || !part_idx)) || raw == kp_out) {
    sca_set_error("sca_prepare_keypoints: bad arguments (K_all must be 1..1024; raw must not alias kp_out)");
    return SCA_ERR_ARG;
  }
  const long frames = (long)B * T;
  if (frames == 0) return SCA_OK;
  NormArgs a{raw, kp_out, lengths, part_off, part_idx, B, T, K_all, nparts, src_row, affine};
  hipLaunchKernelGGL(normalize_parts_kernel, dim3((unsigned)((frames + 3) / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  if (hipGetLastError() != hipSuccess) { sca_set_error("sca_prepare_keypoints: launch failed"); return SCA_ERR_LAUNCH; }
  return SCA_OK;
}
