/*
 * scatten.h — C ABI of libscatten_hip.so, the MI355X (gfx950) implementation of the
 * SCAttenNet spatial-coordinate-attention hot path.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t (passed as
 * void*), never allocates, never synchronises, and is safe under hipGraph stream capture.
 * Each returns 0 on success or a nonzero SCA_ERR_* code (the Python layer maps it to an
 * exception; sca_last_error() gives the message).  All floating point is fp32.
 *
 * Reference interfaces replaced (tinh2044/SCAttenNet @ 2025-07-18; the reference is pure
 * PyTorch, so each entry point replaces an ATen op sequence, not a reference kernel):
 *   sca_gemm               nn.Linear forward/backward in model/attention.py:23-26,41-44,
 *                          49-51,74,101-103,126 ; model/layers.py:97-99,106-108 ;
 *                          model/fusion.py:31-34 ; model/residual.py:14-19
 *                          (q-scaling after bias :49, v-from-kv/2 :103, GELU :98 fused)
 *   sca_attn_fwd           attention.py:63-72 (SelfAttention), :115-124 (CrossAttention),
 *                          :165-178 (SelfCausalAttention) incl. model/utils.py:3-28 masks
 *   sca_attn_bwd           autograd of the same three op sequences
 *   sca_layernorm_fwd/bwd  nn.LayerNorm + the residual add in keypoint_module.py:67-72,
 *                          :101-111 and the position embedding add layers.py:15-30
 *   sca_reduce_rows        bias / LayerNorm-affine / position-table gradient reductions
 *   sca_coord_map_fwd/bwd  KeypointModule stream slicing + CoordinateMapping
 *                          (model/__init__.py:133-142, keypoint_module.py:22-26,
 *                          layers.py:111-123)
 *   sca_maxpool_t_fwd/bwd  ResidualBlock MaxPool1d(2,2) over frames (residual.py:40-43)
 *   sca_softmax_rows_*     CoordinatesFusion softmax (fusion.py:52-53)
 *   sca_gelu_bwd           GELU backward where no GEMM epilogue can absorb it
 *                          (fusion.py:43-50,74-77)
 *   sca_dropout            F.dropout in training mode (keypoint_module.py:64,100,164-165,
 *                          layers.py:105,107, fusion.py:48,54) with a counter-based mask;
 *                          also fused into the GEMM and LayerNorm epilogues
 *   sca_ctc_loss_fwd/bwd   MSCA_Net.compute_loss (model/__init__.py:241-290): log_softmax,
 *                          clamp(-100, 0), nn.CTCLoss(blank=0, reduction='none',
 *                          zero_infinity=True), finite mean, clamp(0, 100)
 *   sca_seqkd_fwd/bwd      SeqKD (loss.py:5-21) with the distillation weight and
 *                          clamp(-100, 100) of model/__init__.py:203-214
 *   sca_clamp              RecognitionHead logit clamp(+-50) (model/__init__.py:54-58)
 *   sca_lstm_cell_fwd/bwd  AlignmentModule's bidirectional nn.LSTM cell
 *                          (model/alignment_module.py:24-30, :68-69)
 */
#ifndef SCATTEN_H
#define SCATTEN_H

#ifdef __cplusplus
extern "C" {
#endif

#define SCA_OK 0
#define SCA_ERR_ARG 1      /* invalid shape / alignment / argument */
#define SCA_ERR_LAUNCH 2   /* hipLaunchKernel failed */

#define SCA_GEMM_MAX_PROBLEMS 16
#define SCA_GEMM_MAX_SEGS 3

/* GEMM layouts: C[M,N] = sum_seg alpha_s * op(A_s) op(B_s)                           */
#define SCA_GEMM_NT 0  /* A[M,K] row-major, B[N,K] row-major  (Linear forward)          */
#define SCA_GEMM_NN 1  /* A[M,K] row-major, B[K,N] row-major  (Linear dX = dY W)        */
#define SCA_GEMM_TN 2  /* A[K,M] row-major, B[K,N] row-major  (Linear dW = dY^T X)      */

/* Epilogue flags (applied in this order):
 *   v = acc ; v += bias[n] ; v *= post_scale ;
 *   GELU : aux_out[m,n] = v ; v = gelu_erf(v)
 *   DROPOUT: v *= keep(drop_seed, m*N + n) / (1 - drop_p)   (see sca_dropout)
 *   DGELU: v *= gelu_erf'(aux[m,n])
 *   v += resid[m,n] (if resid) ; ACCUM: v += C[m,n] ; C[m,n] = v
 * so the post-LN blocks' y = x + dropout(Linear(h)) (keypoint_module.py:64,100 and
 * layers.py:105,107) is one epilogue, and the backward of dropout(GELU(z)) is DROPOUT|DGELU
 * with the forward's seed.                                                             */
#define SCA_EPI_GELU 1
#define SCA_EPI_DGELU 2
#define SCA_EPI_ACCUM 4
#define SCA_EPI_DROPOUT 8

typedef struct {
  const float* A;
  const float* B;
  int lda, ldb;
  int K;       /* reduction length of this segment (any: K, lda, ldb not multiples of 4 or
                  operands not 16-byte aligned take the element-wise load form) */
  float alpha; /* scales A on load: alpha=0.5 reproduces v_proj(kv/2) exactly */
} sca_gemm_seg;

typedef struct {
  sca_gemm_seg seg[SCA_GEMM_MAX_SEGS];
  int nseg;
  int M, N;
  float* C;
  int ldc;
  int epi;
  const float* bias; /* [N] or NULL */
  float post_scale;
  const float* resid; /* [M, ldr] or NULL */
  int ldr;
  const float* aux; /* DGELU input [M, ldx] */
  int ldx;
  float* aux_out; /* GELU pre-activation output [M, ldo] */
  int ldo;
  /* TN layout only: bias_grad[m] = bias_grad_scale * sum_k alpha*A[k, m] (the Linear bias
   * gradient colsum(dY), fused into the weight-gradient GEMM), or NULL */
  float* bias_grad;
  float bias_grad_scale;
  unsigned long long drop_seed; /* DROPOUT: per-call seed (one mask per seed) */
  float drop_p;                 /* DROPOUT: drop probability in [0, 1) */
} sca_gemm_problem;

/* Grouped GEMM over `nprob` independent problems (e.g. q/k/v x streams).
 * splitk > 1 (single segment per problem; shapes may differ) writes fp32 partial slabs
 * into `workspace` (splitk * sum_p (M_p * N_p + M_p) floats) and reduces them in a second
 * launch in fixed order (deterministic).                                                  */
int sca_gemm(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
             void* stream);
/* The two launches of a split-K sca_gemm issued separately (same arguments): the GEMM
 * writing the slabs, then the fixed-order reduction + epilogue (lets a caller time them
 * apart, or put work between them).  sca_gemm_partial with splitk == 1 is sca_gemm.     */
int sca_gemm_partial(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
                     void* stream);
int sca_gemm_reduce(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
                    void* stream);
/* Split-K with the slab combine inside the GEMM launch (no second launch): every split writes
 * its partial slab write-through and takes a ticket on its output tile's counter; the last
 * arriver sums the slabs in slice order (deterministic) and runs the epilogue.
 * `counters`: sca_gemm_splitk_counters(nprob, max M, max N) unsigned ints, ZERO on entry and
 * left zero on exit (the last arriver resets its tile's counter), so one zeroed buffer serves
 * any number of launches that do not run concurrently on the same counters.  Falls back to
 * the two-launch form when the LDS-DMA kernel cannot take the shapes.                      */
long sca_gemm_splitk_counters(int nprob, int maxM, int maxN);
int sca_gemm_splitk_fused(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
                          unsigned* counters, void* stream);

/* NT GEMM + post-LN LayerNorm in one launch (d_model = 256): per problem
 *   C = resid + dropout((A B^T + bias) * post_scale)      (exactly sca_gemm's NT epilogue)
 *   y = (C - mean) * rstd * gamma + beta,  rstd = 1 / sqrt(var + eps)   (nn.LayerNorm)
 * over each full row of C; mean / rstd saved per row (as sca_layernorm_fwd).  Replaces the
 * out-projection / fc2 GEMM + LayerNorm pairs of keypoint_module.py:63-72, 99-109.
 * Requires nseg == 1, N == 256, K a positive multiple of 32, 16-byte aligned operands with
 * leading dimensions multiple of 4 (y has leading dimension 256), epi 0 or DROPOUT only;
 * else SCA_ERR_ARG (use sca_gemm + sca_layernorm_fwd).                                    */
/* Optional chained NT GEMMs on the LayerNorm output y (same launch, the 32-row tile): pass p
 * computes C_p = epi((y B_p^T + bias_p) * post_scale_p) for one 256-row block B_p of an
 * nn.Linear weight ([256, 256] k-contiguous, row stride ldb), epi 0 or SCA_EPI_GELU (then
 * aux_out receives the pre-activation) — the next op's projection (an FFN's fc1 = 3 passes,
 * an attention block's q / k / v = 3 passes) without re-reading y or a launch boundary.    */
typedef struct {
  const float* B;
  int ldb;
  const float* bias; /* [256] or NULL */
  float post_scale;
  int epi;
  float* C;
  int ldc;
  float* aux_out;
  int ldo;
} sca_gemm_chain_pass;

typedef struct {
  const float* gamma; /* [N] */
  const float* beta;  /* [N] */
  float* y;           /* [M, N] */
  float* mean;        /* [M] */
  float* rstd;        /* [M] */
  int npass;          /* 0..3 chained passes */
  sca_gemm_chain_pass pass[3];
} sca_gemm_ln_problem;
#define SCA_GEMM_LN_MAX_PROBLEMS 8

int sca_gemm_ln(int nprob, const sca_gemm_problem* probs, const sca_gemm_ln_problem* ln, float eps,
                void* stream);
/* Row-tile height (32 or 16) sca_gemm_ln launches for nprob problems of at most maxM rows,
 * chained passes or not — the rule the launcher applies (SCA_GEMM_LN_BM overrides without
 * chained passes); hosts use it to name the kernel variant in their profiles. */
int sca_gemm_ln_rows(int nprob, int maxM, int chain);
/* Force the unchained tile height: bm = 16 or 32, 0 = the rule above (process-global;
 * SCA_GEMM_LN_BM sets the initial value, read once). */
int sca_gemm_ln_force_rows(int bm);

/* NN input-gradient GEMM + the backward of the LayerNorm that produced its input, in one
 * launch (d_model = 256).  Per problem:
 *   C  = resid + sum_s alpha * A_s B_s           (sca_gemm NN, epilogue: resid only)
 *      = dL/dy, the gradient w.r.t. the output y of an nn.LayerNorm whose input was x
 *   dx = rstd * (C*gamma - mean_n(C*gamma) - xhat * mean_n(C*gamma*xhat)),
 *        xhat = (x - mean) * rstd                  (aten native_layer_norm_backward)
 *   partial[0][blk][n] = sum_{rows of blk} C * xhat,  partial[1][blk][n] = sum C
 *        (fixed-order dgamma / dbeta partials per 32-row block; blk = row / 32, reduce
 *        them with sca_reduce_rows over nblk = sca_gemm_lnb_blocks(M) rows)
 * Replaces the input-gradient GEMM of a post-LN block's first op (the attention block's
 * dX = dq Wq + dk Wk + dv Wv + dY, the FFN's dx = dz W1 + dY) followed by the separate
 * LayerNorm backward of the block below (keypoint_module.py:69-72, 105-109), and, with
 * `wo`, that block's out-projection input-gradient GEMM as well.
 * Requires N == 256, 1..3 segments with K a positive multiple of 32 and one alpha, B
 * k-major (B[k][n] at B + k*ldb + n), 16-byte aligned operands, leading dimensions
 * multiples of 4; else SCA_ERR_ARG.                                                       */
typedef struct {
  const float* x;     /* [M, 256] LayerNorm input saved by the forward */
  const float* mean;  /* [M] */
  const float* rstd;  /* [M] */
  const float* gamma; /* [256] */
  float* dx;          /* [M, 256] gradient w.r.t. x */
  float* partial;     /* [2, nblk, 256] dgamma / dbeta partials */
  /* optional chained GEMM (NULL = none): dout = dx Wo, Wo [256, 256 * npass] row-major
   * (an nn.Linear weight [out, in]: dout is the gradient of the Linear's INPUT when dx is the
   * gradient of its output), in the same launch — the out-projection input gradient of the
   * attention block that produced the LayerNorm input (attention.py:74 backwards, npass 1),
   * or the FFN's dz = (dx W2) * gelu'(aux) (layers.py:104-107 backwards, npass 3, aux = the
   * fc1 pre-activation)                                                                     */
  const float* wo;
  float* dout;        /* [M, 256 * npass] */
  const float* aux;   /* NULL, or [M, 256 * npass]: dout *= gelu'(aux) (exact-erf GELU) */
  int npass;          /* 1..3 (0 reads as 1) */
  int ldw;            /* row stride of wo, dout and aux (0 reads as 256 * npass) */
  /* optional position table (NULL = none): the LayerNorm input is x + tab[(row % tab_T) + 2]
   * — the embedding LayerNorm of keypoint_module.py:154-160 (x = the mapped coordinates,
   * tab = LearningPositionEmbedding.weight [>= tab_T + 2, 256], layers.py:15-30)          */
  const float* tab;
  int tab_T;
} sca_gemm_lnb_problem;

int sca_gemm_lnb(int nprob, const sca_gemm_problem* probs, const sca_gemm_lnb_problem* lnb, void* stream);
int sca_gemm_lnb_blocks(int M);

/* Tuning knob: force the kernel variant of one layout for every later sca_gemm* call
 * (0 = built-in heuristic; 1 / 5 / 7 register-staged 64x64 / single-buffered 64x64 /
 * 128x64 8 waves; 20 / 21 / 22 LDS-DMA 64x64 with a 3- / 2- / 4-stage ring; TN only: 36 / 37
 * the k-split weight-gradient kernel with a 3- / 4-stage ring, 46 the same with the
 * register-staged interleaved operand stream, 38 / 39 / 40 / 43 128x128 register-staged
 * (43: interleaved phases); NT / NN only: 41 / 42 / 44 128x128 and 45 64x64 register-staged
 * (44, 45: interleaved) — every variant computes the full result; a shape a variant cannot
 * take runs on the LDS-DMA kernels).  Any other id: SCA_ERR_ARG, nothing changed.
 * Process-global.                                                                          */
int sca_gemm_tile_override(int layout, int tile);
/* sca_gemm with the kernel variant chosen for this call only (ids as above, 0 = the override
 * or heuristic; an invalid id is SCA_ERR_ARG): split-K slabs combined in-launch when
 * `counters` is given and the variant can (sca_gemm_splitk_fused), else the two-launch form. */
int sca_gemm_variant(int layout, int nprob, const sca_gemm_problem* probs, int splitk, float* workspace,
                     unsigned* counters, int variant, void* stream);

/* The kernel a sca_gemm_variant launch of these problems would run (variant 0: the override or
 * the heuristic), as a short name ("gemm_tnk_kernel<3, 1, true>", ...) written into buf
 * (NUL-terminated, truncated to len).  Host-only: no GPU call; for profiling records.      */
int sca_gemm_kernel_name(int layout, int nprob, const sca_gemm_problem* probs, int splitk, int variant, char* buf,
                         int len);

/* Fused masked attention over (B, T, H*hd) row-major activations (head h at columns
 * h*hd .. h*hd+hd-1, row stride ld*).  Scores use q as given (the projection already
 * applied hd^-0.5).  Masking, per query row i and key j:
 *   causal && j > i                    -> -inf            (attention.py:165-169)
 *   add_mask != NULL                   -> s + add_mask[b, (h,) i, j]   (general (B,1|H,Tq,Tk))
 *   else key_valid != NULL && !valid_j -> finfo.min       (utils.py:3-12)
 *   else                               -> s + (causal && plus_one ? 1 : 0) (utils.py:24-27)
 * Softmax stats are saved per (g,b,h,i) in the base-2 domain the kernels compute in
 * (scores x log2(e)): m (row max) and ll (log2 of the row sum), kept apart so that fully
 * padded rows (all finfo.min) recompute to exactly uniform weights.  A materialised mask
 * value so negative that x log2(e) overflows is taken as finfo.min (it only arises from
 * finfo.min masks, whose sums with a score all round to finfo.min).                    */
typedef struct {
  const float* q;
  const float* k;
  const float* v;
  float* o;
  float* stat_m;  /* [B*H*Tq] */
  float* stat_ll; /* [B*H*Tq] */
  const float* key_valid; /* [B, Tk] 1.0/0.0, or NULL */
  const float* add_mask;  /* [B, Tq, Tk] additive, or NULL */
  /* attention-probability dropout (attention.py:67-69, 119-121, 173-175), drop_p = 0: none.
   * O = (P * keep / (1 - drop_p)) V with keep = the sca_dropout mask of drop_seed over the
   * (B, H, Tq, Tk) probabilities, element e = ((b H + h) Tq + i) Tk + j (mod 2^32); the
   * softmax statistics are those of P.  The backward must get the same seed and p.        */
  unsigned long long drop_seed;
  float drop_p;
  /* add_mask layout: 0 or 1 = [B, Tq, Tk] shared by every head; H = [B, H, Tq, Tk], one mask
   * per head (the reference adds any mask broadcastable to (B, H, Tq, Tk), attention.py:65) */
  int mask_heads;
} sca_attn_fwd_problem;

typedef struct {
  const float* q;
  const float* k;
  const float* v;
  const float* o;
  const float* dout;
  const float* stat_m;
  const float* stat_ll;
  const float* key_valid;
  const float* add_mask;
  float* dq;    /* written (not accumulated), scaled by dq_scale */
  float* dk;
  float* dv;
  float* delta; /* workspace [B*H*Tq] : rowsum(dO * O) */
  float dq_scale;
  float dv_scale;
  float* dq_part; /* workspace of sca_attn_bwd_workspace() floats, or NULL: with it (hd 32, no
                     add_mask) the backward is one fused launch over 256-key blocks + a
                     fixed-order dQ reduction; without it the split dq / dkdv kernels */
  unsigned long long drop_seed; /* the forward's attention-probability dropout */
  float drop_p;
  int mask_heads;               /* as sca_attn_fwd_problem */
} sca_attn_bwd_problem;

#define SCA_ATTN_MAX_PROBLEMS 8

int sca_attn_fwd(int nprob, const sca_attn_fwd_problem* probs, int B, int H, int Tq, int Tk, int hd,
                 int ldq, int ldk, int ldv, int ldo, int causal, int plus_one, void* stream);
/* dq_part floats per problem for the fused hd-32 backward (0 when that path does not apply) */
long sca_attn_bwd_workspace(int B, int H, int Tq, int Tk, int hd);
int sca_attn_bwd(int nprob, const sca_attn_bwd_problem* probs, int B, int H, int Tq, int Tk, int hd,
                 int ldq, int ldk, int ldv, int ldo, int causal, int plus_one, void* stream);
/* Backward kernel choice: enable = 1 (default) runs the single-launch fused kernel where it
 * applies (hd 16, Tq and Tk <= 256, no add_mask): S / P / dP / dS once per score, dK / dV in
 * registers, dQ from an LDS image of dS; enable = 0 always runs the split dq + dkdv pair.
 * Both are deterministic and write dq, dk, dv and delta.                               */
int sca_attn_bwd_fused(int enable);

/* y = act(LayerNorm(x + r) * gamma + beta + post) over rows of width N (eps given).
 * r row index = (row % r_mod) + r_off  (r_mod = rows for an ordinary residual; r_mod = T,
 * r_off = 2 for the LearningPositionEmbedding table); post (or NULL) is row-aligned with x;
 * act: 0 = identity, 1 = ReLU (ResidualBlock, model/residual.py:31-38).
 * drop_p > 0 (act must be identity): y = dropout(y) with the sca_dropout mask of
 * drop_seed — the embedding dropout after first_*_norm (keypoint_module.py:164-165); the
 * backward applies the same mask to dy (sca_dropout) before sca_layernorm_bwd.
 * Saves mean/rstd per row.  Any N (widths over 1024 take a row-looping kernel).         */
#define SCA_ACT_NONE 0
#define SCA_ACT_RELU 1
typedef struct {
  const float* x;
  const float* r; /* or NULL */
  const float* gamma;
  const float* beta;
  const float* post; /* or NULL */
  float* y;
  float* mean;
  float* rstd;
  int act;
  unsigned long long drop_seed;
  float drop_p;
} sca_ln_fwd_problem;

typedef struct {
  const float* dy;
  const float* x;
  const float* r;
  const float* gamma;
  const float* mean;
  const float* rstd;
  const float* y;  /* forward output, read when act == ReLU (gradient gate y > 0) */
  int act;
  float* dpost;  /* or NULL: receives the (gated) gradient of `post` */
  float* dx;     /* gradient of (x + r); ACCUM adds into dx */
  float* dgamma; /* [N] written; NULL: the affine partials stay in `partial` (rows 0..nblk-1
                  * sum to dgamma, rows nblk..2nblk-1 to dbeta) for a later sca_reduce_rows */
  float* dbeta;  /* [N] written (ignored when dgamma is NULL) */
  float* partial; /* workspace [2 * nblk * N], nblk from sca_layernorm_bwd_blocks() */
} sca_ln_bwd_problem;

#define SCA_LN_MAX_PROBLEMS 8
int sca_layernorm_fwd(int nprob, const sca_ln_fwd_problem* probs, int rows, int N, int r_mod, int r_off,
                      float eps, void* stream);
int sca_layernorm_bwd_blocks(int rows);
int sca_layernorm_bwd(int nprob, const sca_ln_bwd_problem* probs, int rows, int N, int r_mod, int r_off,
                      int accumulate, void* stream);

/* MaxPool1d(kernel 2, stride 2) over the frame axis of (B, T, C) -> (B, T/2, C)
 * (ResidualBlock downsample, model/residual.py:40-43).  Backward routes each gradient to
 * the first maximal element of its pair (ties -> the earlier frame), like ATen.          */
typedef struct {
  const float* x;
  float* y;  /* forward */
  const float* dy;
  float* dx; /* backward (fully written, odd trailing frame gets 0) */
} sca_pool_problem;
#define SCA_POOL_MAX_PROBLEMS 8
int sca_maxpool_t_fwd(int nprob, const sca_pool_problem* probs, int B, int T, int C, void* stream);
int sca_maxpool_t_bwd(int nprob, const sca_pool_problem* probs, int B, int T, int C, void* stream);

/* Row softmax over the last dim (any N) and its backward (CoordinatesFusion's
 * unscaled, unmasked attention weights, model/fusion.py:52-53):
 *   fwd: y = softmax(x)            bwd: dx = y * (dy - sum_j dy_j y_j)                  */
typedef struct {
  const float* x;  /* fwd input */
  const float* y;  /* fwd output / bwd input */
  const float* dy;
  float* out;      /* fwd: y ; bwd: dx */
} sca_softmax_problem;
#define SCA_SOFTMAX_MAX_PROBLEMS 8
int sca_softmax_rows_fwd(int nprob, const sca_softmax_problem* probs, int rows, int N, void* stream);
int sca_softmax_rows_bwd(int nprob, const sca_softmax_problem* probs, int rows, int N, void* stream);

/* Elementwise GELU backward: dz = dy * gelu_erf'(z) over n elements (the pre-activation z
 * is what the GEMM GELU epilogue stored).                                               */
typedef struct {
  const float* dy;
  const float* z;
  float* dz;
} sca_gelu_bwd_problem;
#define SCA_GELU_MAX_PROBLEMS 8
int sca_gelu_bwd(int nprob, const sca_gelu_bwd_problem* probs, long n, void* stream);

/* Fixed-order sum of up to SCA_SUM_MAX_TERMS same-shaped tensors, n elements each:
 * out = in[0] + in[1] + ... + in[nin-1] (left to right) — the gradient of a tensor read by
 * several ops (the final x-stream map read by every merge layer, keypoint_module.py:181-187)
 * in one launch per group instead of one autograd add per pair.  16-byte aligned.         */
#define SCA_SUM_MAX_TERMS 8
typedef struct {
  const float* in[SCA_SUM_MAX_TERMS];
  int nin;
  float* out;
} sca_sum_problem;
#define SCA_SUM_MAX_PROBLEMS 8
int sca_sum_tensors(int nprob, const sca_sum_problem* probs, long n, void* stream);

/* Dropout (F.dropout, training mode) over contiguous (rows, cols) tensors:
 *   y[e] = x[e] * keep(seed, e) / (1 - p),  e = row * cols + col
 * keep() is a counter-based hash RNG (no state, no sequence): with
 *   mix(x) = lowbias32 (x^=x>>16; x*=0x7feb352d; x^=x>>15; x*=0x846ca68b; x^=x>>16),
 *   key = mix(lo32(seed) ^ mix(hi32(seed) + 0x9e3779b9)),
 *   keep = mix(mix(e ^ key) + key) >= (uint32)(p * 2^32 in fp32)
 * so forward, backward and the CPU oracle regenerate the same mask from the seed alone
 * (masks differ from torch's Philox stream; the drop rate is the same).  The same mask
 * is applied by the GEMM DROPOUT epilogue and the LayerNorm forward.  In-place allowed.
 * Used for: the backward of every dropout site, and the fusion's attention-weight and
 * output dropout (model/fusion.py:48,54).                                               */
typedef struct {
  const float* x;
  float* y;
  unsigned long long seed;
} sca_dropout_problem;
#define SCA_DROPOUT_MAX_PROBLEMS 12
int sca_dropout(int nprob, const sca_dropout_problem* probs, long rows, int cols, float p, void* stream);

/* Key validity of the (B, T) attention mask the SCA stack receives, as the (B, T) fp32 1/0
 * vector the attention kernels read (key_valid):
 *   key_valid[i] = ((float)mask[i] == 1.0f) ? 1 : 0
 * — the reference's predicate: create_attention_mask / create_causal_attention_mask
 * (model/utils.py:8-12, 19-23) cast the mask to fp32 and mask every key where
 * 1.0 - mask != 0, so only the value 1 keeps a key (2, 0.5, -1, NaN all mask it).
 * dtype: the mask's element type (SCA_MASK_*); any alignment; n = 0 is a no-op.        */
#define SCA_MASK_F32 0
#define SCA_MASK_F64 1
#define SCA_MASK_I64 2
#define SCA_MASK_I32 3
#define SCA_MASK_U8 4   /* bool / uint8 */
#define SCA_MASK_F16 5
#define SCA_MASK_BF16 6
#define SCA_MASK_I8 7
#define SCA_MASK_I16 8
int sca_key_valid(const void* mask, int dtype, float* key_valid, long n, void* stream);

/* p[0 .. n) = 0 (fp32): the gradient buffers a backward only partly writes (the position
 * table's rows that no frame reads, model/layers.py LearningPositionEmbedding) — one launch
 * in the captured step instead of an ATen fill.                                          */
int sca_zero(float* p, long n, void* stream);

/* Registers a device-resident step counter (or NULL) read by every dropout mask at run
 * time: effective seed = seed + counter * 0x9E3779B97F4A7C15.  A hipGraph that captures
 * the counter's increment then draws fresh masks on every replay although the seeds in
 * its kernel arguments are frozen.  Process-global; applies to launches issued after. */
int sca_dropout_offset(const unsigned long long* counter);

/* out[i, j] (+)= scale * sum_{s < S} in[s * stride_s + i * stride_i + j],  i < I, j < N.
 * Column sums (bias gradients), slab reductions, position-table gradients.            */
typedef struct {
  const float* in;
  float* out;
  float scale;
} sca_reduce_problem;

#define SCA_REDUCE_MAX_PROBLEMS 64
int sca_reduce_rows(int nprob, const sca_reduce_problem* probs, int S, int I, int N, long stride_s,
                    long stride_i, int accumulate, void* stream);

/* Coordinate mapping of one stream (fused A1+A2): keypoints (B*T, K_all, 2) fp32,
 * joint index list idx[K] (int32, device) ->
 *   xe[row, n] = sum_k kp[row, idx[k], 0] * Wx[n, k] + bx[n]
 *   ye[row, n] = sum_k kp[row, idx[k], 1] * Wy[n, k] + by[n]                           */
typedef struct {
  const float* kp;
  const int* idx;
  int K;
  const float* wx;
  const float* bx;
  const float* wy;
  const float* by;
  float* xe;
  float* ye;
} sca_coord_map_problem;

typedef struct {
  const float* kp;
  const int* idx;
  int K;
  const float* wx;
  const float* wy;
  const float* dxe;
  const float* dye;
  float* dwx;     /* [N, K] written */
  float* dwy;     /* [N, K] written */
  float* dkp;     /* [rows, K_all, 2] accumulated into (must be zeroed by caller) or NULL */
  float* partial; /* workspace [2 * nchunk * N * K], nchunk = sca_coord_map_bwd_chunks(rows) */
} sca_coord_map_bwd_problem;

#define SCA_MAP_MAX_PROBLEMS 8
int sca_coord_map_fwd(int nprob, const sca_coord_map_problem* probs, int rows, int K_all, int N,
                      void* stream);
int sca_coord_map_bwd_chunks(int rows);
int sca_coord_map_bwd(int nprob, const sca_coord_map_bwd_problem* probs, int rows, int K_all, int N,
                      void* stream);

/* Input contract: SLR_Dataset.normalize_keypoints
 * (dataset.py:134-170) on a zero-padded batch.  kp_in / kp_out: (B, T, K_all, 2) fp32;
 * frame t of clip b with t < lengths[b] is normalised part by part, in order (part p owns
 * joints part_idx[part_off[p] .. part_off[p+1])): its bounding box grown by 5 % of the
 * longer side and squared, clamped to [0, 1], then x, y mapped into it (an axis whose
 * clamped extent is 0 is left as is).  Frames t >= lengths[b] are written as zeros (the
 * collator's padding, dataset.py:82-91).  K_all <= 1024; kp_out may alias kp_in.        */
/* The sample pipeline of SLR_Dataset.data_collator for a batch in one launch
 * (dataset.py:58-125 with preprocess_keypoints :124-132): for t < lengths[b], frame (b, t)
 * is raw row src_row[b T + t] (frame selection, dataset.py:185-215, decided on the host with
 * the reference's RNG calls), transformed by the clip's augmentation affine (affine + 6 b =
 * [a00 a01 tx a10 a11 ty]: rotation about (0, 0) and / or x -> 1 - x, augmentation.py:3-25;
 * NULL = none) and then normalised as sca_normalize_parts (nparts = 0: not normalised);
 * frames t >= lengths[b] are zeros.  raw: (R, K_all, 2) fp32, all clips' frames.          */
int sca_prepare_keypoints(const float* raw, const int* src_row, const float* affine, const int* lengths,
                          float* kp_out, int B, int T, int K_all, const int* part_off, const int* part_idx,
                          int nparts, void* stream);
int sca_normalize_parts(const float* kp_in, float* kp_out, const int* lengths, int B, int T, int K_all,
                        const int* part_off, const int* part_idx, int nparts, void* stream);

/* ---- recognition-head losses --------------------------------
 * CTC over batch-major logits (B, T, C) (the reference's permute(1, 0, 2) at
 * model/__init__.py:245 is a view; no copy), labels (B, S) int32 padded, in_len / tgt_len
 * (B) int32 device vectors.  Per sample: S_b = max(tgt_len, 1), T_b = max(in_len, 1, S_b)
 * (model/__init__.py:262-266); the caller validates T_b <= T, S_b <= S and labels in [0, C)
 * (out-of-range values are clamped in-kernel only to stay in bounds).  nll (B, optional):
 * per-sample losses after zero_infinity; loss (1): clamp(mean over finite nll, 0, 100), 0
 * when none is finite.  ws: sca_ctc_workspace_floats(B, T, S) floats, kept between the
 * forward and the backward (row log-sum-exp, alpha, beta, per-sample gradient scale).
 * bwd: dlogits = d loss / d logits given dloss (1 float, device).  C <= 8192, S <= 1023. */
#define SCA_CTC_MAX_C 8192
#define SCA_CTC_MAX_S 1023
long sca_ctc_workspace_floats(int B, int T, int S);
int sca_ctc_loss_fwd(const float* logits, const int* labels, const int* in_len, const int* tgt_len, int B, int T,
                     int C, int S, float* nll, float* loss, float* ws, void* stream);
int sca_ctc_loss_bwd(const float* logits, const int* labels, const int* in_len, const int* tgt_len, int B, int T,
                     int C, int S, const float* dloss, const float* ws, float* dlogits, void* stream);

/* SeqKD over R rows of C logits (student, teacher): columns [start, C) only (use_blank=False
 * -> start 1), temperature temp:
 *   loss = clamp(weight * temp^2 * (1/R) * sum_rows KL(softmax(q/temp) || log_softmax(s/temp)),
 *                lo, hi)
 * (KLDivLoss 'batchmean' over the .view(-1, C') rows).  ws: sca_seqkd_workspace_floats(R).
 * bwd writes d loss / d student (dstudent) and/or d loss / d teacher (dteacher; NULL when
 * the teacher is detached, as the reference does), zeros in columns < start.              */
long sca_seqkd_workspace_floats(int R);
int sca_seqkd_fwd(const float* student, const float* teacher, int R, int C, int start, float temp, float weight,
                  float lo, float hi, float* loss, float* ws, void* stream);
int sca_seqkd_bwd(const float* student, const float* teacher, int R, int C, int start, float temp,
                  const float* dloss, const float* ws, float* dstudent, float* dteacher, void* stream);

/* torch.clamp(x, lo, hi) over n elements (dy == NULL), or its backward dx = dy * [lo <= x <= hi] */
int sca_clamp(const float* x, float* y, const float* dy, float* dx, long n, float lo, float hi, void* stream);

/* One time step of a (bi)directional LSTM cell (AlignmentModule's nn.LSTM,
 * model/alignment_module.py:24-30), batch-major, both directions per launch (direction 1
 * walks t = T-1 .. 0); gate order i, f, g, o.  The projections around it are sca_gemm
 * launches.  D = ndir.  fwd: gates (B, D*4H) pre-activations of this step -> act
 * (B, T, D*4H), c / y (B, T, D*H), and hp (B, T, D*H) = the hidden state each step reads
 * (h_{t-1} for direction 0, h_{t+1} for direction 1; zero-filled by the caller).
 * bwd (step k walks t = T-1-k / t = k): dh (B, D*H) = dY_t + dG_{t'} W_hh (NULL at k = 0,
 * where dy (B, T, D*H) is read instead), dc (B, D*H) carried in place, dg (B, T, D*4H) the
 * gate pre-activation gradients.                                                          */
int sca_lstm_cell_fwd(const float* gates, float* act, float* c, float* y, float* hp, int B, int T, int H, int ndir,
                      int step, void* stream);
int sca_lstm_cell_bwd(const float* dh, const float* dy, const float* act, const float* c, float* dc, float* dg,
                      int B, int T, int H, int ndir, int step, void* stream);

const char* sca_last_error(void);
int sca_version(void);
/* sha256 (first 16 hex digits) of the library sources the binary was built from
 * (the .cpp, .h and .hip files of scattennet_amd/csrc in name order, then this header); the Python binding
 * refuses a library whose digest does not match the sources beside it. */
const char* sca_build_digest(void);

#ifdef __cplusplus
}
#endif
#endif /* SCATTEN_H */
