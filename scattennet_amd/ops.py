"""Grouped autograd ops of the SCA hot path, each forward/backward a launch of the HIP C ABI.

Every op works on a GROUP of G independent problems (the keypoint streams of one clip batch,
or G = 1 for a standalone module), so that one launch covers all streams: at the BASELINE
config-2 shape (B=8, T=256, d=256) a single stream's GEMM is only 2048 x 256 x 256.

Activations are contiguous (B, T, C) fp32 on the GPU, viewed as (M = B*T, C) row-major.
Parameters keep the nn.Linear / nn.LayerNorm layouts of the reference (W is [out, in]).
"""
import ctypes
import os

import torch
from torch.autograd import Function

from . import _lib as L
from ._lib import ptr

# --------------------------------------------------------------------------- launch profiling
class LaunchProfiler:
    """While active, every C-ABI call is bracketed by HIP events on the stream it launches
    on, with its algorithmic FLOPs; used by bench.py for the dominant kernel's roofline."""

    def __init__(self):
        self.records = []

    def __enter__(self):
        global _PROFILER
        _PROFILER = self
        return self

    def __exit__(self, *exc):
        global _PROFILER
        _PROFILER = None

    def stats(self):
        out = {}
        for key, flops, e0, e1 in self.records:
            st = out.setdefault(key, {"flops": 0.0, "seconds": 0.0, "launches": 0})
            st["flops"] += flops
            st["seconds"] += e0.elapsed_time(e1) / 1e3
            st["launches"] += 1
        return out

    def launches(self, *prefixes):
        """Launch count of the kernels whose names start with any of `prefixes`."""
        return sum(v["launches"] for k, v in self.stats().items() if k.startswith(prefixes))

    def dominant(self):
        st = self.stats()
        k = max(st, key=lambda n: st[n]["seconds"])
        return k, st[k]


_PROFILER = None


class _timed:
    def __init__(self, key, flops):
        self.key, self.flops = key, flops

    def __enter__(self):
        if _PROFILER is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if _PROFILER is not None:
            self.e1.record()
            _PROFILER.records.append((self.key, self.flops, self.e0, self.e1))


# name prefixes of every kernel that can run a layout's plain GEMM (tests count launches by them)
GEMM_KERNELS = {lay: (f"gemm_glds_kernel<{lay},", f"gemm_kernel<{lay}") for lay in range(3)}
# the register-staged kernels (_gemm_kernel_name): NT / NN by their B-layout flag, TN by family
GEMM_KERNELS[0] += ("gemm_ntb_kernel<true, 6, false", "gemm_ntb_kernel<false, 2, false")
GEMM_KERNELS[1] += ("gemm_ntb_kernel<true, 6, true", "gemm_ntb_kernel<false, 2, true")
GEMM_KERNELS[2] += ("gemm_tnk_kernel<", "gemm_tnb_kernel<")

# rocprof names of the default (LDS-DMA) kernel per layout (gemm_glds_kernel<LAYOUT, STAGES>:
# the ring depth pick_tile chooses, 3 stages forward, 2 for the gradient layouts)

# --------------------------------------------------------------------------- launch helpers
_NOSEG = L.GemmSeg(None, None, 0, 0, 0, 0.0)


def _seg(A, B, lda, ldb, K, alpha=1.0):
    return L.GemmSeg(A.data_ptr(), B.data_ptr(), lda, ldb, K, alpha)


def _prob(segs, C, M, N, ldc, bias=None, post_scale=1.0, resid=None, ldr=0, epi=0, aux=None, ldx=0,
          aux_out=None, ldo=0, bias_grad=None, bias_grad_scale=1.0, drop=None):
    """drop: None or (seed, p) -> the DROPOUT epilogue with that seed's mask."""
    s = list(segs) + [_NOSEG] * (3 - len(segs))
    seed, p = (0, 0.0) if drop is None else drop
    if drop is not None:
        epi |= L.EPI_DROPOUT
    return L.GemmProblem((L.GemmSeg * 3)(*s), len(segs), M, N, C.data_ptr(), ldc, epi, ptr(bias), post_scale,
                         ptr(resid), ldr, ptr(aux), ldx, ptr(aux_out), ldo, ptr(bias_grad), bias_grad_scale,
                         seed, p)


# --------------------------------------------------------------------------- dropout
_SEED_SOURCE = None  # tests install a deterministic, logging source (tests/test_dropout.py)


_COUNTER = None


def dropout_counter():
    """The device step counter every dropout mask reads (include/scatten.h,
    sca_dropout_offset): incrementing it inside a captured graph step (advance_dropout)
    gives every replay fresh masks.  One per process (one GPU per process)."""
    global _COUNTER
    if _COUNTER is None:
        _COUNTER = torch.zeros(1, dtype=torch.int64, device=torch.device("cuda", torch.cuda.current_device()))
        L.check(L.lib().sca_dropout_offset(ptr(_COUNTER)), "sca_dropout_offset")
    return _COUNTER


def advance_dropout():
    """Next training step's masks (capture-safe: a device-side increment)."""
    dropout_counter().add_(1)


def dropout_seeds(n):
    """n fresh 64-bit dropout seeds, one mask each.  Drawn from torch's CPU generator, so
    torch.manual_seed() makes a training run reproducible, as with F.dropout."""
    dropout_counter()
    if _SEED_SOURCE is not None:
        return [int(v) for v in _SEED_SOURCE(n)]
    return [int(v) for v in torch.randint(0, 2 ** 63 - 1, (n,), dtype=torch.int64)]


def dropout_apply(items, p):
    """items: [(x, y, seed)] same-shaped contiguous fp32 tensors; y = dropout_seed(x) (y may be x)."""
    if not items:
        return
    x0 = items[0][0]
    cols = x0.shape[-1] if x0.dim() else 1
    rows = x0.numel() // max(cols, 1)
    for c in range(0, len(items), L.DROPOUT_MAX_PROBLEMS):
        chunk = items[c:c + L.DROPOUT_MAX_PROBLEMS]
        arr = (L.DropoutProblem * len(chunk))(*[L.DropoutProblem(x.data_ptr(), y.data_ptr(), sd) for x, y, sd in chunk])
        L.check(L.lib().sca_dropout(len(chunk), arr, rows, cols, float(p), L.stream_handle()), "sca_dropout")


class Dropout(Function):
    """F.dropout(x, p, training=True) for G same-shaped tensors (one seed each); the backward
    regenerates each mask from its seed."""

    @staticmethod
    def forward(ctx, p, *xs):
        xs = _contig(xs)
        L.require_device(*xs)
        seeds = dropout_seeds(len(xs))
        ys = [torch.empty_like(x) for x in xs]
        dropout_apply([(x, y, sd) for x, y, sd in zip(xs, ys, seeds)], p)
        ctx.p, ctx.seeds = p, seeds
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        dys = _contig(dys)
        dxs = [torch.empty_like(d) for d in dys]
        dropout_apply([(d, o, sd) for d, o, sd in zip(dys, dxs, ctx.seeds)], ctx.p)
        return (None,) + tuple(dxs)


def dropout_grouped(xs, p):
    """G-way F.dropout in training mode (p > 0)."""
    return list(Dropout.apply(float(p), *xs))


# split-K slabs combined inside the GEMM launch by the last-arriving split (sca_gemm_splitk_fused)
_SPLITK_FUSED = True
_CNT = {}  # device index -> [ring, position]
_CNT_SIZE = 1 << 16


def _splitk_counters(n, device=None):
    """n zeroed tile counters from a persistent per-device ring (the kernel leaves them
    zero).  A slot is reused only after the whole ring (65,536 counters) has been handed out
    since; one config-2 step uses ~6k, so the launches that shared a slot have completed
    (every launch of a step is ordered before the next step's)."""
    dev = torch.cuda.current_device() if device is None else device
    if n > _CNT_SIZE:
        raise RuntimeError(f"split-K launch needs {n} tile counters, more than the ring's {_CNT_SIZE}")
    ent = _CNT.get(dev)
    if ent is None:
        ent = _CNT[dev] = [torch.zeros(_CNT_SIZE, dtype=torch.int32, device=torch.device("cuda", dev)), 0]
    ring, pos = ent
    n = -(-n // 64) * 64
    if pos + n > _CNT_SIZE:
        pos = 0
    ent[1] = pos + n
    return ring[pos:pos + n]




def _gemm_kernel_name(layout, chunk, tile, splitk=1):
    """The kernel a sca_gemm / sca_gemm_variant launch of `chunk` runs (for the profiler's
    records), as the library's own launcher resolves it (sca_gemm_kernel_name: the variant
    choice with the process-wide override and the environment switches as the library read
    them, then the eligibility fallbacks of launch_tile).  Host-only, no GPU call."""
    buf = ctypes.create_string_buffer(96)
    arr = (L.GemmProblem * len(chunk))(*chunk)
    L.check(L.lib().sca_gemm_kernel_name(layout, len(chunk), arr, splitk, tile, buf, 96), "sca_gemm_kernel_name")
    return buf.value.decode()


def gemm(layout, probs, splitk=1, ws=None, tile=0):
    """tile: a kernel variant for this call only (sca_gemm_variant ids; 0 = the heuristic),
    passed per call through the C ABI (no process-global override is touched)."""
    lib = L.lib()
    st = L.stream_handle()
    for i in range(0, len(probs), L.GEMM_MAX_PROBLEMS):
        chunk = probs[i:i + L.GEMM_MAX_PROBLEMS]
        arr = (L.GemmProblem * len(chunk))(*chunk)
        flops = sum(2.0 * p.M * p.N * p.seg[j].K for p in chunk for j in range(p.nseg)) if _PROFILER else 0.0
        kname = _gemm_kernel_name(layout, chunk, tile, splitk) if _PROFILER else ""
        if splitk > 1 and _SPLITK_FUSED and "sca_gemm_splitk_fused" not in L.MISSING:
            cnt = _splitk_counters(lib.sca_gemm_splitk_counters(len(chunk), max(p.M for p in chunk),
                                                                max(p.N for p in chunk)),
                                   ws.device.index if ws is not None else None)
            with _timed(kname, flops):
                L.check(lib.sca_gemm_variant(layout, len(chunk), arr, splitk, ptr(ws), ptr(cnt), tile, st),
                        "sca_gemm_variant")
            continue
        if tile:
            with _timed(kname, flops):
                L.check(lib.sca_gemm_variant(layout, len(chunk), arr, splitk, ptr(ws), None, tile, st),
                        "sca_gemm_variant")
            continue
        with _timed(kname, flops):
            L.check(lib.sca_gemm_partial(layout, len(chunk), arr, splitk, ptr(ws), st), "sca_gemm")
        if splitk > 1:  # the fixed-order slab reduction: its own launch (timed apart)
            with _timed("splitk_reduce4_kernel", 0.0):
                L.check(lib.sca_gemm_reduce(layout, len(chunk), arr, splitk, ptr(ws), st), "sca_gemm_reduce")


# the fused LayerNorms' dgamma / dbeta reductions ride in the weight-gradient side section
_LN_AFFINE_SIDE = os.environ.get("SCA_LN_AFFINE_SIDE", "1") != "0"  # A/B switch

# GEMM + post-LN LayerNorm in one launch (sca_gemm_ln) where the shape allows it
_FUSE_LN = True


# d_model 512 (two 256-column halves, no chained passes): parity-green, but slower than the
# plain 64x64-tile GEMMs + separate LayerNorm launches at config 5 (71.9 vs 70.6 ms/step:
# the 32-row x 256-column tiles at one workgroup per CU run the big-M GEMMs at ~0.43 of
# peak against the plain kernel's ~0.6, which outweighs the LayerNorm launches saved;
# DESIGN.md §9) — opt-in (tests switch it on)
_FUSE_LN512 = os.environ.get("SCA_FUSE_LN512", "0") == "1"  # opt-in (A/B)


def ln_width_ok(N):
    """LayerNorm widths the fused GEMM + LayerNorm launches take (forward and backward)."""
    return N == 256 or (N == 512 and _FUSE_LN512)


def ln_fusable(N, K):
    """d_model 256 (chained passes possible) or, opt-in, 512 (two column halves)."""
    return _FUSE_LN and ln_width_ok(N) and K >= 32 and K % 32 == 0


def gemm_ln_force_rows(bm):
    """Force the unchained GEMM + LayerNorm tile height (16 / 32; 0 = the launcher's rule)."""
    L.check(L.lib().sca_gemm_ln_force_rows(int(bm)), "sca_gemm_ln_force_rows")


def gemm_ln(probs, lns, eps):
    """probs: NT sca_gemm problems (C receives the LayerNorm input v); lns: GemmLnProblem."""
    lib = L.lib()
    st = L.stream_handle()
    for i in range(0, len(probs), L.GEMM_LN_MAX_PROBLEMS):
        chunk, lchunk = probs[i:i + L.GEMM_LN_MAX_PROBLEMS], lns[i:i + L.GEMM_LN_MAX_PROBLEMS]
        arr = (L.GemmProblem * len(chunk))(*chunk)
        larr = (L.GemmLnProblem * len(lchunk))(*lchunk)
        flops = sum(2.0 * p.M * p.N * (p.seg[0].K + 256 * ln.npass) for p, ln in zip(chunk, lchunk)) \
            if _PROFILER else 0.0
        # the variant sca_gemm_ln picks, for the kernel name rocprofv3 shows
        chain = any(ln.npass > 0 for ln in lchunk)
        nc = chunk[0].N // 256
        bm = 32 if nc > 1 else lib.sca_gemm_ln_rows(len(chunk), max(p.M for p in chunk), int(chain))
        reg = nc == 1 and bm == 32 and _ln_reg(chunk)
        with _timed(f"gemm_ln_kernel<{bm}, {'true' if chain else 'false'}, {nc}, {'true' if reg else 'false'}>",
                    flops):
            L.check(lib.sca_gemm_ln(len(chunk), arr, larr, float(eps), st), "sca_gemm_ln")


_FUSE_LNB = True


def _ln_reg(probs):
    """Whether sca_gemm_ln / sca_gemm_lnb run the register-staged main loop (gemm.hip ln_reg_ok:
    every segment's K % 64 == 0; SCA_LNREG=0 switches it off) — for the kernel names."""
    return os.environ.get("SCA_LNREG", "1") != "0" and \
        all(p.seg[j].K % 64 == 0 and p.seg[j].K > 0 for p in probs for j in range(p.nseg))


class LnSaved:
    """What a fused GEMM + post-LN LayerNorm forward (sca_gemm_ln) leaves on its output
    tensor (`y._sca_ln`) so that the op consuming y can run this LayerNorm's backward in
    its own input-gradient GEMM's epilogue (sca_gemm_lnb): the LN input v, its row mean /
    rstd and gamma.  `handoff` carries the result back to the producer's backward:
    (dL/dy as the consumer returned it, its version, dL/dv, dgamma/dbeta partials, nblk,
    dout).  `wo`: the producer's next backward GEMM on dL/dv, chained into the same launch
    (`dout`) when no dropout sits between: an attention block's out-projection weight (dO =
    dL/dv Wo) or an FFN's fc2 weight with `aux` = the fc1 pre-activation (dz = (dL/dv W2) *
    gelu'(aux))."""
    __slots__ = ("v", "mean", "rstd", "gamma", "handoff", "wo", "aux", "tab", "T")

    def __init__(self, v, mean, rstd, gamma, wo=None, aux=None, tab=None, T=0):
        self.v, self.mean, self.rstd, self.gamma, self.handoff, self.wo = v, mean, rstd, gamma, None, wo
        self.aux = aux
        self.tab, self.T = tab, T  # position-table mode: the LN input is v + tab[t + 2]


def ln_saved_of(ts):
    """Consumer forward: the LnSaved of each input (all G or None)."""
    if not _FUSE_LNB or _LIBRARY_MODE:
        return None
    out = [getattr(t, "_sca_ln", None) for t in ts]
    return out if all(o is not None for o in out) else None


_CHAIN_DO = True
# the embedding LayerNorm (position-table mode) handed to its consumer's sca_gemm_lnb
_EMB_LNB = True
# the FFN's dz chained into its consumer's sca_gemm_lnb launch: parity-green, but -1.7 % in
# step at config 2 (three 256-column passes at one workgroup per CU lose to the stand-alone
# NN GEMM that shares the CUs with the weight gradients) — off (tests switch it on)
_CHAIN_DZ = False


def _attach_ln_saved(ys, vs, means, rstds, gam, wo=None, aux=None):
    """wo[g]: [256, 256 npass] k-major (an nn.Linear weight [out = 256, in]); aux[g]: the
    DGELU pre-activation [M, 256 npass] or None."""
    ok = wo is not None and _CHAIN_DO and all(
        w.dim() == 2 and w.shape[0] == 256 and w.shape[1] % 256 == 0 and w.shape[1] <= 768 and w.is_contiguous()
        for w in wo)
    if _LIBRARY_MODE:
        return None
    objs = [LnSaved(vs[g], means[g], rstds[g], gam[g], wo[g] if ok else None,
                    aux[g] if (ok and aux is not None) else None)
            for g in range(len(ys))]
    for y, o in zip(ys, objs):
        y._sca_ln = o
    return objs


_CHAIN_NEXT = os.environ.get("SCA_CHAIN", "1") != "0"  # A/B switch


class NextProjections:
    """A request to compute the NEXT op's input projections inside a fused GEMM + LayerNorm
    launch (sca_gemm_ln's chained passes): y = LN(v) of the 32-row tile is still in LDS, so
    out_j = epi((y W_j^T + b_j) * s_j) costs no y re-read and no launch of its own.  Made by
    the caller that knows which op reads y next (keypoint_module: a block's FFN fc1, the next
    block's q / k / v); the producer op fills it (`passes`), the consumer op takes the
    results (`take`) only if it runs with exactly the requested, unmodified parameters on the
    unmodified y — otherwise it computes its projections itself.

    specs[g]: [(W [n, 256] contiguous, b or None, post_scale, gelu)], sum(n) <= 768, n % 256 == 0."""

    def __init__(self, specs):
        self.specs = specs
        self.vers = [[(W._version, None if b is None else b._version) for W, b, _, _ in s] for s in specs]
        self.outs = [None] * len(specs)
        self.ys = [None] * len(specs)

    @staticmethod
    def eligible(specs):
        for s in specs:
            if sum(W.shape[0] for W, _, _, _ in s) > 256 * 3:
                return False
            for W, b, _, _ in s:
                if (W.dim() != 2 or W.shape[1] != 256 or W.shape[0] % 256 or not W.is_contiguous() or
                        (b is not None and not b.is_contiguous())):
                    return False
        return True

    def passes(self, g, M, like):
        """Producer: the ChainPass list of stream g (outputs allocated here)."""
        ps, outs = [], []
        for W, b, scale, gelu in self.specs[g]:
            n = W.shape[0]
            C = like.new_empty(M, n)
            A = like.new_empty(M, n) if gelu else None
            for p in range(n // 256):
                ps.append(L.ChainPass(W[256 * p:].data_ptr(), W.stride(0),
                                      b[256 * p:].data_ptr() if b is not None else None, float(scale),
                                      L.EPI_GELU if gelu else 0, C[:, 256 * p:].data_ptr(), n,
                                      A[:, 256 * p:].data_ptr() if gelu else None, n if gelu else 0))
            outs.append((C, A))
        self.outs[g] = outs
        return ps

    def attach(self, ys):
        for g, y in enumerate(ys):
            if self.outs[g] is not None:
                y._sca_next = self
                self.ys[g] = (y._version, y.data_ptr())

    def take(self, g, y, params):
        """Consumer: [(C, aux)] for stream g if `params` [(W, b)] are the requested ones."""
        if self.outs[g] is None or self.ys[g] != (y._version, y.data_ptr()) or len(params) != len(self.specs[g]):
            return None
        for (W, b), (W0, b0, _, _), (wv, bv) in zip(params, self.specs[g], self.vers[g]):
            if W is not W0 or b is not b0 or W._version != wv or (b is not None and b._version != bv):
                return None
        out, self.outs[g] = self.outs[g], None  # one consumer
        return out


def _next_of(xs):
    return [getattr(x, "_sca_next", None) for x in xs]


# Chained passes only when the launch has a 32-row tile for every CU: the passes run at one
# workgroup per tile, so a launch of a few tiles would do them on a few CUs
# (tools/gemm_ln_bench.py, 1 x (2048, 256, 256) + fc1: 52.8 us chained vs 28.4 us as a
# separate 64x64-tile GEMM); the consumer then computes its projections itself
_CHAIN_MIN_TILES = 256


def _chain_lns(nxt, G, M, like, gam, bet, ys, means, rstds):
    """GemmLnProblems of a fused GEMM + LayerNorm launch, with `nxt`'s chained passes."""
    if nxt is not None and (G * ((M + 31) // 32) < _CHAIN_MIN_TILES or like.shape[-1] != 256):
        nxt = None  # (chained passes exist for d_model 256 only)
    lns = []
    for g in range(G):
        ps = nxt.passes(g, M, like) if nxt is not None else []
        arr = (L.ChainPass * 3)(*(ps + [L.ChainPass()] * (3 - len(ps))))
        lns.append(L.GemmLnProblem(gam[g].data_ptr(), bet[g].data_ptr(), ys[g].data_ptr(), means[g].data_ptr(),
                                   rstds[g].data_ptr(), len(ps), arr))
    return lns


_LNB_R3 = os.environ.get("SCA_LNB_R3", "0") == "1"  # the library's switch of the same name (names only)


def gemm_lnb(probs, lnp):
    """Consumer backward: the NN input-gradient GEMMs `probs` (C = dL/dy of the LayerNorms
    `lnp`, N = 256) with those LayerNorms' backward fused (sca_gemm_lnb); the LN-input
    gradients and dgamma/dbeta partials are handed to the producers' backward."""
    lib = L.lib()
    M = probs[0].M
    nblk = lib.sca_gemm_lnb_blocks(M)
    dv = [torch.empty_like(o.v) for o in lnp]
    part = [o.v.new_empty(2 * nblk * o.v.shape[-1]) for o in lnp]
    # the producers' next GEMM on dv (dO = dv Wo, or dz = (dv W2) gelu'(z)) in the same launch
    # (d_model 256 only)
    chain = (probs[0].N == 256 and all(o.wo is not None for o in lnp) and
             len({(o.wo.shape[1], o.aux is None) for o in lnp}) == 1)
    n2 = lnp[0].wo.shape[1] if chain else 0
    dout = [o.v.new_empty(*o.v.shape[:-1], n2) for o in lnp] if chain else [None] * len(lnp)
    arr = (L.GemmProblem * len(probs))(*probs)
    larr = (L.GemmLnbProblem * len(lnp))(*[L.GemmLnbProblem(o.v.data_ptr(), o.mean.data_ptr(), o.rstd.data_ptr(),
                                                           o.gamma.data_ptr(), dv[g].data_ptr(), part[g].data_ptr(),
                                                           ptr(o.wo) if chain else None, ptr(dout[g]),
                                                           ptr(o.aux) if chain else None, n2 // 256, n2,
                                                           ptr(o.tab), o.T)
                                            for g, o in enumerate(lnp)])
    flops = sum(2.0 * p.M * p.N * p.seg[j].K for p in probs for j in range(p.nseg)) if _PROFILER else 0.0
    if chain and _PROFILER:
        flops += sum(2.0 * p.M * 256 * n2 for p in probs)
    nc = probs[0].N // 256
    reg = nc == 1 and _ln_reg(probs)
    name = f"gemm_lnb_kernel<{nc}, {str(reg).lower()}, {str(bool(reg and chain and _LNB_R3)).lower()}>"
    with _timed(name, flops):
        L.check(lib.sca_gemm_lnb(len(probs), arr, larr, L.stream_handle()), "sca_gemm_lnb")
    return dv, part, nblk, dout


def hand_off(lnp, dxs, dv, part, nblk, dout):
    for g, o in enumerate(lnp):
        o.handoff = (dxs[g], dxs[g]._version, dv[g], part[g], nblk, dout[g])


def _take_handoff(lnsaved, dys):
    """Producer backward: the consumer's precomputed LayerNorm backward, valid only if the
    incoming gradients ARE the tensors the consumer returned, untouched (the consumer was
    the output's only one: with another, autograd's sum is a new tensor)."""
    if lnsaved is None:
        return None
    hs = [o.handoff for o in lnsaved]
    for o in lnsaved:
        o.handoff = None
    for h, d in zip(hs, dys):
        if h is None or d is None or d.data_ptr() != h[0].data_ptr() or d._version != h[1] or d.shape != h[0].shape:
            return None
    return hs


def _ln_bwd_or_handoff(dys, vs, gam, means, rstds, lnsaved, bet):
    """The fused post-LN LayerNorm's backward: taken over from the consumer's sca_gemm_lnb
    when it ran, else ln_bwd.  -> (dL/dv, dgamma, dbeta, deferred affine finish)."""
    hs = _take_handoff(lnsaved, dys)
    params = tuple(gam) + tuple(bet)
    if hs is None:
        dys = _contig(_zeros_for_none(dys, vs))
        return _ln_bwd(dys, vs, gam, means, rstds, defer_affine=_LN_AFFINE_SIDE, params=params) + (None,)
    G, N, nblk = len(gam), gam[0].shape[0], hs[0][4]
    dg = [param_grad_empty(t) for t in gam]
    db = [param_grad_empty(b) for b in bet]
    part = [h[3] for h in hs]

    # raw pointers, not the tensors: a closure holding dg / db would make autograd's
    # AccumulateGrad copy them (use count > 1) instead of taking them over
    pairs = _ptr_pairs([(part[g], dg[g]) for g in range(G)] + [(part[g], db[g], nblk * N) for g in range(G)])

    def reduce():
        reduce_rows_ptr(pairs, nblk, 1, N, N, 0)
    finish = (reduce, part, params, (pairs, nblk, N), list(dg) + list(db))
    if not _LN_AFFINE_SIDE:
        reduce()
        params_produced(params)
        finish = None
    dout = [h[5] for h in hs] if all(h[5] is not None for h in hs) else None
    return [h[2] for h in hs], dg, db, finish, dout


def _ln_fwd_outputs(xs):
    """(v, y, mean, rstd) buffers of a fused GEMM + LayerNorm over the rows of xs."""
    rows = xs[0].numel() // xs[0].shape[-1]
    return ([torch.empty_like(x) for x in xs], [torch.empty_like(x) for x in xs],
            [xs[0].new_empty(rows) for _ in xs], [xs[0].new_empty(rows) for _ in xs])


def _ln_bwd(dys, x, gam, means, rstds, defer_affine=False, params=None):
    """Plain LayerNorm backward (no residual table / post / activation): (dx, dgamma, dbeta,
    finish).  With `defer_affine` the dgamma / dbeta reduction is NOT launched here:
    `finish` = (launch function, its input tensors) is run by the caller later — inside the
    weight-gradient side-stream section (weight_grads(..., extra=finish)), so that the
    parameter-only reduction leaves the critical stream without a fork of its own."""
    G = len(x)
    N = x[0].shape[-1]
    rows = x[0].numel() // N
    nblk = L.lib().sca_layernorm_bwd_blocks(rows)
    bet = params[G:] if params is not None and len(params) == 2 * G else [None] * G
    dx = [torch.empty_like(t) for t in x]
    dg = [param_grad_empty(t) for t in gam]
    db = [param_grad_empty(bet[g]) if bet[g] is not None else torch.empty_like(gam[g]) for g in range(G)]
    part = [x[0].new_empty(2 * nblk * N) for _ in range(G)]
    for c in range(0, G, L.LN_MAX_PROBLEMS):
        gs = range(c, min(G, c + L.LN_MAX_PROBLEMS))
        arr = (L.LnBwdProblem * len(gs))(*[L.LnBwdProblem(dys[g].data_ptr(), x[g].data_ptr(), None,
                                                            gam[g].data_ptr(), means[g].data_ptr(),
                                                            rstds[g].data_ptr(), None, 0, None, dx[g].data_ptr(),
                                                            None if defer_affine else dg[g].data_ptr(),
                                                            None if defer_affine else db[g].data_ptr(),
                                                            part[g].data_ptr()) for g in gs])
        L.check(L.lib().sca_layernorm_bwd(len(gs), arr, rows, N, rows, 0, 0, L.stream_handle()),
                "sca_layernorm_bwd")
    finish = None
    if defer_affine:  # pointers only: see _ln_bwd_or_handoff
        pairs = _ptr_pairs([(part[g], dg[g]) for g in range(G)] + [(part[g], db[g], nblk * N) for g in range(G)])
        finish = (lambda: reduce_rows_ptr(pairs, nblk, 1, N, N, 0), part, params or (), (pairs, nblk, N),
                  list(dg) + list(db))
    else:
        params_produced(params or ())
    return dx, dg, db, finish


def _ptr_pairs(items):
    """[(input tensor, output tensor[, input float offset])] -> [(in ptr, out ptr, 1.0)]."""
    return [(a.data_ptr() + 4 * (it[2] if len(it) > 2 else 0), it[1].data_ptr(), 1.0) for it in items
            for a in (it[0],)]


def reduce_rows_ptr(pairs, S, I, N, stride_s, stride_i, accumulate=False):
    """reduce_rows over raw device pointers [(in, out, scale)] (no tensor references kept)."""
    lib = L.lib()
    st = L.stream_handle()
    for i in range(0, len(pairs), L.REDUCE_MAX_PROBLEMS):
        chunk = pairs[i:i + L.REDUCE_MAX_PROBLEMS]
        arr = (L.ReduceProblem * len(chunk))(*[L.ReduceProblem(a, o, s) for a, o, s in chunk])
        L.check(lib.sca_reduce_rows(len(chunk), arr, S, I, N, stride_s, stride_i, int(accumulate), st),
                "sca_reduce_rows")


def reduce_rows(pairs, S, I, N, stride_s, stride_i, accumulate=False):
    """pairs: list of (in_tensor, out_tensor_or_view, scale)."""
    lib = L.lib()
    st = L.stream_handle()
    for i in range(0, len(pairs), L.REDUCE_MAX_PROBLEMS):
        chunk = pairs[i:i + L.REDUCE_MAX_PROBLEMS]
        arr = (L.ReduceProblem * len(chunk))(*[L.ReduceProblem(a.data_ptr(), o.data_ptr(), s) for a, o, s in chunk])
        L.check(lib.sca_reduce_rows(len(chunk), arr, S, I, N, stride_s, stride_i, int(accumulate), st),
                "sca_reduce_rows")


_SPLITK_MAX = 8
_SPLITK_SLOTS = 768  # workgroup slots per round: 3 LDS-DMA 64x64 workgroups per CU


_TNK_TILES_PER_PROBLEM = 48
_TNR = os.environ.get("SCA_TNR", "1") != "0"  # A/B switch for variant 46
_TNR_SK = int(os.environ.get("SCA_TNR_SK", "0"))  # A/B: one split-K for every variant-46 launch
_TNR_MIXED = os.environ.get("SCA_TNR_MIXED", "0") != "0"  # A/B: mixed-shape variant-46 launches (-0.7 % in step)
_TNR_MIXED_SK = int(os.environ.get("SCA_TNR_MIXED_SK", "0"))  # A/B: split-K of mixed-shape launches


# the 128x128 register-staged weight-gradient kernel with interleaved phases (tile 43) for long
# reductions (config 5: K = 8192 rows); measured with tools/tn_library_compare.py (DESIGN.md
# §9R.1): 0.88 of peak with one workgroup per CU, 0.86 with two, against the k-split kernel's
# 0.74; at config 2 / 3's K <= 2048 it has too few tiles and loses
_TNB_MIN_K = int(os.environ.get("SCA_TNB_MIN_K", "4096"))  # A/B switch (0: never)
_TNB_RATE2, _TNB_RATE1, _TNB_EPI = 0.86, 0.88, 3.0


_TNB_MODEL = os.environ.get("SCA_TNB_MODEL", "0") != "0"  # A/B: the isolated-speed split model


def _tnb_split(K, tiles128):
    """Split-K for tile 43.  In the step: 1 — one long workgroup per output tile, the fewest
    workgroups holding CUs beside the critical chain (config 5: +0.5 % over the model below,
    whose FFN choice of split 4 is faster alone; profiles/r05_misc/tnb_split_cfg5_ab.txt).
    SCA_TNB_MODEL=1: the split whose estimated per-CU time is least — workgroups dealt over
    256 CUs, two at a time at _TNB_RATE2, a leftover one at _TNB_RATE1, plus an epilogue cost
    per workgroup (ties: the smaller split, fewer slabs)."""
    if not _TNB_MODEL:
        return 1
    best, best_sk = None, 1
    for sk in range(1, _SPLITK_MAX + 1):
        if sk > 1 and K // sk < 1024:
            break
        iters = -(-(-(-K // sk)) // 64)
        w = -(-tiles128 * sk // 256)
        cost = (w // 2) * 2 * iters / _TNB_RATE2 + (w % 2) * iters / _TNB_RATE1 + w * _TNB_EPI
        if best is None or cost < best - 1e-9:
            best, best_sk = cost, sk
    return best_sk


def _splitk_for(M_red, n_out_tiles):
    """Split the long reduction (rows of the batch) of weight-gradient GEMMs: the split that
    fills whole rounds of the LDS-DMA kernel's 3 workgroups per CU (768 slots) best, each
    split keeping >= 256 rows (+0.8 % over powers of two up to 1024 tiles; measured with
    tools/gemm_bench.py and in-step bench A/B)."""
    best, best_sk = -1.0, 1
    for sk in range(1, _SPLITK_MAX + 1):
        if sk > 1 and M_red // sk < 256:
            break
        n = n_out_tiles * sk
        if n < 512 and sk < _SPLITK_MAX and M_red // (sk + 1) >= 256:
            continue
        fill = n / (-(-n // _SPLITK_SLOTS) * _SPLITK_SLOTS)
        if fill > best + 1e-9:
            best, best_sk = fill, sk
    return best_sk


# ---- parameter-gradient sink -------------------------------------------------------------
# Every backward below allocates a parameter's gradient through `param_grad_empty` and, once
# the launches writing it are enqueued, reports it through `params_produced` (on the stream
# that wrote it).  With no sink installed that is torch.empty_like and a no-op.  The data-
# parallel reducer (dp.GradBuckets) installs itself as the sink: gradients are then written
# straight into slots of its flat all-reduce buckets, and a bucket's RCCL all-reduce is
# issued as soon as its last gradient has been enqueued — overlapped with the rest of the
# backward.
_GRAD_SINK = None


def set_grad_sink(sink):
    global _GRAD_SINK
    _GRAD_SINK = sink


# library mode (scattennet_amd.library's torch.library operators): the grouped Functions'
# bodies run for one stream, as pure functions of their operands — no cross-op hand-offs,
# no weight-gradient side stream, no gradient sink
_LIBRARY_MODE = False


class library_mode:
    def __enter__(self):
        global _LIBRARY_MODE, _GRAD_SINK
        self.prev = (_LIBRARY_MODE, _GRAD_SINK)
        _LIBRARY_MODE, _GRAD_SINK = True, None

    def __exit__(self, *exc):
        global _LIBRARY_MODE, _GRAD_SINK
        _LIBRARY_MODE, _GRAD_SINK = self.prev


def param_grad_empty(p):
    if _GRAD_SINK is not None:
        t = _GRAD_SINK.grad_buffer(p)
        if t is not None:
            return t
    return torch.empty_like(p)


def param_grad_zeros(p):
    if _GRAD_SINK is not None:
        t = _GRAD_SINK.grad_buffer(p)
        if t is not None:
            return t.zero_()
    return torch.zeros_like(p)


def params_produced(ps):
    if _GRAD_SINK is not None:
        _GRAD_SINK.produced([p for p in ps if p is not None and not isinstance(p, bool)])


# ---- weight-gradient side stream -------------------------------------------------------
# The weight/bias-gradient GEMMs of a layer do not feed the rest of the backward pass, so
# they go to a side HIP stream, forked from the point where their inputs are ready
# (wgrad_ready) and joined into the caller's stream by a callback queued on the autograd
# engine when backward() completes, so .grad is safe to read afterwards exactly as with a
# single stream (the same mechanism torch DDP uses).  Captured into the step's hipGraph as
# fork/join edges: the critical chain stays on one hardware queue and the weight gradients
# fill the other — in practice behind the chain's second half (the executor's queue lists,
# DESIGN.md §9).

_WGRAD_SIDE = True
_EARLY_FORK = True   # fork the weight gradients before the layer's input-gradient launch
_side_streams = {}
_join_pending = {}
# weight-gradient side streams per device, used round-robin by successive weight_grads calls
# (SCA_WGRAD_STREAMS, A/B: with 2 the tail of consecutive dW launches can overlap)
_WGRAD_STREAMS = max(1, int(os.environ.get("SCA_WGRAD_STREAMS", "1")))


def _side_stream(device):
    ent = _side_streams.get(device)
    if ent is None:
        ent = _side_streams[device] = [[torch.cuda.Stream(device=device) for _ in range(_WGRAD_STREAMS)], 0]
    streams, i = ent
    ent[1] = (i + 1) % len(streams)
    return streams[i]


class ForkLedger:
    """Host-side record of the stream forks and joins the hot path makes — weight-gradient side
    streams (weight_grads), RCCL's stream
    (dp.GradBuckets) — checked at the end of a graph capture: every stream forked during the
    capture must afterwards be joined DIRECTLY into the capture's origin stream.  (DESIGN §7,
    constraint (1): a forked stream joined into another forked stream that then joins the
    origin crashed hipGraph instantiation; a fork never joined fails capture outright.)"""

    def __init__(self, origin):
        self.origin = origin.cuda_stream
        self.seq = 0
        self.last_fork = {}   # child stream -> seq of its last fork
        self.last_join = {}   # child stream -> (seq, target) of its last join
        self.names = {}

    @staticmethod
    def _id(st):
        return st.cuda_stream if hasattr(st, "cuda_stream") else st

    def fork(self, child, parent, name=""):
        self.seq += 1
        c = self._id(child)
        if c != self.origin:
            self.last_fork[c] = self.seq
            self.names.setdefault(c, name)

    def join(self, into, child):
        self.seq += 1
        self.last_join[self._id(child)] = (self.seq, self._id(into))

    def problems(self):
        out = []
        for c, fs in self.last_fork.items():
            j = self.last_join.get(c)
            name = self.names.get(c) or hex(c)
            if j is None or j[0] < fs:
                out.append(f"stream {name} forked but not joined back")
            elif j[1] != self.origin:
                out.append(f"stream {name} joined into {hex(j[1])}, not into the capture origin")
        return out

    def check(self):
        bad = self.problems()
        if bad:
            raise RuntimeError("fork/join check at capture end: " + "; ".join(bad))


_LEDGER = None


def fork_ledger_begin(origin=None):
    """Start recording forks / joins (call inside the capture, on its origin stream)."""
    global _LEDGER
    _LEDGER = ForkLedger(origin if origin is not None else torch.cuda.current_stream())
    return _LEDGER


def fork_ledger_end():
    """Stop recording; raise if a fork was not joined back into the origin."""
    global _LEDGER
    led, _LEDGER = _LEDGER, None
    if led is not None:
        led.check()
    return led


def note_fork(child, parent, name=""):
    if _LEDGER is not None:
        _LEDGER.fork(child, parent, name)


def note_join(into, child):
    if _LEDGER is not None:
        _LEDGER.join(into, child)


def _queue_join(main, side):
    key = (main.cuda_stream, side.cuda_stream)
    task = torch._C._current_graph_task_id()  # one join per backward (keyed by the graph task, so
    if _join_pending.get(key) == task:         # a backward that raised leaves no stale entry)
        return
    _join_pending[key] = task

    def _join():
        _join_pending[key] = None
        if _held["entries"]:
            _flush_held(main, side)
        flush_deferred_affine()
        main.wait_stream(side)
        note_join(main, side)

    torch.autograd.Variable._execution_engine.queue_callback(_join)


def wgrad_ready():
    """Mark, on the current stream, the point where the inputs of a layer's weight gradients are
    ready — before the layer's last input-gradient launch.  weight_grads(..., ready=ev) forks
    its side stream from this point, so that in the captured graph the input-gradient launch is
    the first child of the producing node and the weight gradients the second: hipGraph keeps a
    node's first child on the parent's queue and starts a new queue list for the others, which
    keeps the critical chain on one hardware queue (forking after the input-gradient launch made
    the weight gradients its first child and moved the chain to the other queue at every layer,
    behind whatever that queue held)."""
    if not _EARLY_FORK or not _WGRAD_SIDE or _LIBRARY_MODE:
        return None
    ev = torch.cuda.Event()
    ev.record()
    return ev


# The LayerNorm affine reductions (dgamma / dbeta from the per-block partial rows) that ride in
# a weight-gradient side-stream section are not launched there but collected per side stream and
# launched together once the backward has been enqueued (flush_deferred_affine: from the side
# stream's join callback, or first thing in the data-parallel reducer's finish): one
# reduce_rows launch for all layers instead of one ~5-us launch between every layer's weight
# gradients.  SCA_AFFINE_DEFER=0: the per-layer launches (A/B).
_AFFINE_DEFER = os.environ.get("SCA_AFFINE_DEFER", "1") != "0"
_affine_pending = {}  # side stream handle -> (side stream, [(pairs, nblk, N, keep-alive tensors, params)])
_affine_task = None  # the autograd graph task the pending entries belong to


_flush_queued = [None]  # the autograd graph task whose final callbacks hold a flush
_side_written = {}  # id(parameter) -> graph task whose side stream wrote its gradient
_AFFINE_DEFER_MAX = 256 * 512  # partial-row floats per problem up to which a LayerNormAdd defers


def _plain_leaf(p):
    """A parameter whose gradient autograd hands over untouched until the backward ends: a leaf
    that requires grad, holds no .grad to add to and has no hooks (a tensor hook or a
    post-accumulate-grad hook would read the gradient as soon as it is returned — before a
    side-stream or deferred launch has written it)."""
    return (p.is_leaf and p.requires_grad and p.grad is None and not p._backward_hooks and
            getattr(p, "_post_accumulate_grad_hooks", None) is None)


def _affine_deferrable(params, needed=None):
    """Whether a LayerNorm's dgamma / dbeta reduction may be deferred to the end of the backward:
    autograd takes the (not yet written) gradient tensors over as .grad, which is safe only
    for plain leaf parameters (_plain_leaf) whose gradients the backward asked for."""
    return (_AFFINE_DEFER and not _LIBRARY_MODE and all(_plain_leaf(p) for p in params) and
            (needed is None or all(needed)))


def _keep(ts):
    """Storage references that keep gradient buffers allocated until a deferred launch has been
    enqueued, without raising the tensors' use count (autograd's AccumulateGrad copies a
    gradient tensor that anything else references instead of taking it over)."""
    return [t.untyped_storage() for t in ts if t is not None]


def _mark_unsettled(params):
    """Record that this backward returned these parameters' gradients before writing them (side
    stream or deferred reduction)."""
    task = torch._C._current_graph_task_id()
    if len(_side_written) > 4096:
        _side_written.clear()
    for p in params:
        _side_written[id(p)] = task


def _settle_reuse(params):
    """A parameter used twice in one backward whose first gradient is still pending (written on
    the side stream, or left to a deferred reduction): autograd adds the new gradient into the
    first one on the current stream, so the pending work is launched and joined here first.
    True when that happened (the caller then computes on the current stream)."""
    task = torch._C._current_graph_task_id()
    if not any(_side_written.get(id(p)) == task for p in params):
        return False
    flush_held()
    flush_deferred_affine()
    main = torch.cuda.current_stream()
    for streams, _ in _side_streams.values():
        for st in streams:
            main.wait_stream(st)
            note_join(main, st)
    return True


def _affine_finish(part, dg, db, nblk, N, params, defer):
    """dgamma / dbeta = fixed-order sums of the per-block partial rows: now, or (defer) collected
    on the current stream and launched with the other deferred reductions by
    flush_deferred_affine, which a final backward callback runs at the latest (the entry keeps
    the partials and the dgamma / dbeta buffers allocated until then: autograd may drop the
    gradients it did not ask for)."""
    G = len(part)
    pairs = _ptr_pairs([(part[g], dg[g]) for g in range(G)] + [(part[g], db[g], nblk * N) for g in range(G)])
    if not defer:
        reduce_rows_ptr(pairs, nblk, 1, N, N, 0)
        params_produced(params)
        return
    _affine_defer(torch.cuda.current_stream(), (pairs, nblk, N, list(part) + _keep(list(dg) + list(db)),
                                                list(params)))
    task = torch._C._current_graph_task_id()  # one flush callback per backward (a backward that
    if _flush_queued[0] != task:               # raised before its callbacks leaves no stale flag)
        _flush_queued[0] = task
        torch.autograd.Variable._execution_engine.queue_callback(flush_deferred_affine)


def _affine_defer(st, entry):
    """Collect one deferred reduction on stream st.  Entries left by a backward that raised
    before its final callbacks (their gradients are void) are dropped, never launched later."""
    global _affine_task
    task = torch._C._current_graph_task_id()
    if task != _affine_task:
        _affine_pending.clear()
        _affine_task = task
    _affine_pending.setdefault(st.cuda_stream, (st, []))[1].append(entry)


def flush_deferred_affine():
    """Launch every collected affine reduction on the side stream it was deferred on, grouped
    by (blocks, width), and report its parameters as produced.  Entries of another backward
    (one that raised before its final callbacks: its gradients are void) are dropped."""
    _flush_queued[0] = None
    if not _affine_pending:
        return
    if _affine_task != torch._C._current_graph_task_id():
        _affine_pending.clear()
        return
    pend = list(_affine_pending.values())
    _affine_pending.clear()
    for side, entries in pend:
        with torch.cuda.stream(side):
            groups = {}
            for pairs, nblk, N, _, params in entries:
                g = groups.setdefault((nblk, N), ([], []))
                g[0].extend(pairs)
                g[1].extend(params)
            for (nblk, N), (pairs, params) in groups.items():
                reduce_rows_ptr(pairs, nblk, 1, N, N, 0)
                params_produced(params)


def weight_grads(items, M=None, extra=None, ready=None, holdable=False):
    """dW_g = alpha_g * dY_g^T X_g  (TN layout, split-K) and db_g = bias_scale_g * colsum(dY_g),
    the bias gradient fused into the same GEMM (its first column tile sums the dY slices).

    items: list of (dY[M,out], X[M,in], alpha, W, bias[, bias_scale]) -> [(dW, db)]; W and
    bias are the parameters (bias None / False: no bias gradient; True: a bias gradient
    without its parameter at hand).  bias_scale defaults to alpha; it differs when alpha
    scales the INPUT X (v from kv/2: dWv = dV^T (kv/2) but dbv = colsum(dV))."""
    def run(defer=False, sk=0):
        out = _weight_grads(items, sk)
        params_produced([p for it in items for p in (it[3], it[4])])
        _run_extra(extra, defer)
        return out

    # a parameter that already holds a .grad gets the new gradient added by autograd as soon
    # as this returns (ordered on the current stream only), and so does a non-leaf parameter
    # view (precision.fp32_compute's p.float(): its cast backward reads the gradient at once):
    # compute on the current stream
    params = [it[3] for it in items] + [it[4] for it in items if torch.is_tensor(it[4])] + \
        list(extra[2] if extra is not None else ())
    if _settle_reuse(params) or not _WGRAD_SIDE or _LIBRARY_MODE or not all(_plain_leaf(p) for p in params):
        return run()
    dev = items[0][0].device
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    _mark_unsettled(params)
    if _WGRAD_HOLD_FRAC > 0:
        task = torch._C._current_graph_task_id()
        if _held["task"] != task:  # (held sections of a backward that raised are void)
            if _held["task"] is not None and _held["count"] > 0:
                _held["last_total"] = _held["count"]
            # only a backward that begins with the SCA blocks' sections holds (config 2); one that
            # begins elsewhere (config 3: fusion, residual network) forks every section
            _held.update(task=task, n=0, count=0, entries=[], hold=_hold_count() if holdable else 0)
    late_sk = 0
    if _WGRAD_HOLD_FRAC > 0 and holdable:
        _held["count"] += 1
        hold = _held["hold"]
        if _WGRAD_LATE_SK and hold > 0 and _held["count"] > _WGRAD_LATE_FROM * _held["last_total"]:
            late_sk = _WGRAD_LATE_SK
        if _held["n"] < hold:
            # held: the gradients are allocated and returned now, their launches issued together
            # with the following held sections' at the last one's fork (or at the join).  The
            # entry keeps the operands, raw-pointer problems and the gradients' STORAGES only:
            # a reference to a returned gradient tensor would make autograd copy it (unwritten)
            _held["n"] += 1
            out = _wgrad_alloc(items)
            ex = None if extra is None else (extra[0], extra[1], extra[2], extra[3] if len(extra) > 3 else None,
                                             _keep(extra[4]))
            _held["entries"].append((items, ex, _wgrad_specs(items, out),
                                     _keep([t for o in out for t in o])))
            if _held["n"] == hold:
                _flush_held(main, side, ready)
            _queue_join(main, side)
            return out
    if ready is not None:
        side.wait_event(ready)  # dY and X were ready at this point of the main stream
    else:
        side.wait_stream(main)  # dY and X are ready on the main stream
    note_fork(side, main, "weight-gradient side stream")
    _record_on(side, items, extra)
    with torch.cuda.stream(side):
        out = run(defer=_AFFINE_DEFER, sk=late_sk)
    _queue_join(main, side)
    return out


def _run_extra(extra, defer):
    """The LayerNorm affine reduction riding in a weight-gradient section: now, or deferred."""
    if extra is None:
        return
    if defer and len(extra) > 3:
        pairs, nblk, N = extra[3]
        _affine_defer(torch.cuda.current_stream(), (pairs, nblk, N, list(extra[1]) + _keep(extra[4]), list(extra[2])))
    else:
        extra[0]()
        params_produced(extra[2])


def _record_on(side, items, extra, outs=()):
    """Keep the section's operands (and gradient buffers written there) from being reused by
    the main stream before the side stream's launches have run."""
    for it in items:
        it[0].record_stream(side)
        it[1].record_stream(side)
    for t in (extra[1] if extra is not None else ()):
        t.record_stream(side)
    for t in (extra[4] if extra is not None else ()):  # dgamma / dbeta, written on the side stream
        t.record_stream(side)
    for dW, db in outs:
        dW.record_stream(side)
        if db is not None:
            db.record_stream(side)


# SCA_WGRAD_HOLD=n (A/B): the first n weight-gradient sections of a backward are not forked one
# by one: their launches are issued together (problems of equal shape across sections in one
# grouped launch) at the n-th section's fork — one fork marker instead of n, fuller launches
# SCA_WGRAD_HOLD=n (an integer: n sections) or a fraction f < 1 (the first f of the previous
# backward's sections; the first backward holds none)
_WGRAD_HOLD_FRAC = float(os.environ.get("SCA_WGRAD_HOLD", "0.5"))
_WGRAD_HOLD_MERGE = os.environ.get("SCA_WGRAD_HOLD_MERGE", "1") != "0"
# SCA_WGRAD_LATE_SK=k, SCA_WGRAD_LATE_FROM=f: in a backward that holds (one beginning with the
# SCA blocks), the sections after the first f of the previous backward's — the ones whose
# launches end up running alone after the main stream — at split-K k when their rule gave less
# (768 workgroups instead of 512 for 16 x (256, 256): the whole chip when nothing runs beside
# them).  Config 2: +0.31 % (f 0.5, 4 alternated reps), +0.19 % from the first non-held
# section; with the hold at 0.5: f 0.5 / 0.55 / 0.6 within 0.1 % of each other; config 3 (no
# hold, so not applied): -1.45 % if it were; 0 switches it off
_WGRAD_LATE_SK = int(os.environ.get("SCA_WGRAD_LATE_SK", "3"))
_WGRAD_LATE_FROM = float(os.environ.get("SCA_WGRAD_LATE_FROM", "0.55"))

_held = {"task": None, "n": 0, "count": 0, "entries": [], "hold": 0, "last_total": 0}


def _hold_count():
    if _WGRAD_HOLD_FRAC >= 1:
        return int(_WGRAD_HOLD_FRAC)
    return int(round(_WGRAD_HOLD_FRAC * _held["last_total"]))


def flush_held():
    """Issue any held weight-gradient sections now (the data-parallel reducer's finish: every
    gradient must have been produced before it reduces the last buckets)."""
    if _held["entries"]:
        dev = _held["entries"][0][0][0][0].device
        main = torch.cuda.current_stream(dev)
        _flush_held(main, _side_stream(dev))


def _flush_held(main, side, ready=None):
    """Launch the held weight-gradient sections on the side stream, forked at `ready` (else at
    the main stream's current point)."""
    ents = _held["entries"]
    _held["entries"] = []
    if not ents or _held["task"] != torch._C._current_graph_task_id():
        return
    if ready is not None:
        side.wait_event(ready)
    else:
        side.wait_stream(main)
    note_fork(side, main, "weight-gradient side stream (held sections)")
    for items, ex, _, stores in ents:
        _record_on(side, items, None)
        for t in (ex[1] if ex is not None else ()):
            t.record_stream(side)
        for st in stores + (list(ex[4]) if ex is not None else []):  # gradients written on the side stream
            torch.empty(0, device=items[0][0].device).set_(st).record_stream(side)
    with torch.cuda.stream(side):
        if _WGRAD_HOLD_MERGE:  # equal shapes across the held sections share launches
            _wgrad_launch([sp for _, _, specs, _ in ents for sp in specs])
        else:  # each section's own launches, issued back to back
            for _, _, specs, _ in ents:
                _wgrad_launch(specs)
        for items, ex, _, _ in ents:
            params_produced([p for it in items for p in (it[3], it[4])])
            if ex is None:
                continue
            if _AFFINE_DEFER and ex[3] is not None:
                pairs, nblk, N = ex[3]
                _affine_defer(torch.cuda.current_stream(), (pairs, nblk, N, list(ex[1]) + list(ex[4]), list(ex[2])))
            else:
                ex[0]()
                params_produced(ex[2])


def _weight_grads(items, sk=0):
    """Allocate the gradients and launch the grouped split-K TN GEMMs -> [(dW, db)]."""
    out = _wgrad_alloc(items)
    _wgrad_launch(_wgrad_specs(items, out), sk)
    return out


def _norm_items(items):
    return [it if len(it) == 6 else tuple(it) + (it[2],) for it in items]


def _wgrad_alloc(items):
    out = []
    for dY, X, alpha, W, bias, _ in _norm_items(items):
        dW = param_grad_empty(W)
        if torch.is_tensor(bias):
            db = param_grad_empty(bias)
        else:
            db = torch.empty(W.shape[0], device=W.device, dtype=W.dtype) if bias else None
        out.append((dW, db))
    return out


def _wgrad_specs(items, out):
    """One (shape key, problem) per item; the problem holds raw pointers only (no tensor
    references: a held section must not raise its gradients' use count)."""
    specs = []
    for (dY, X, alpha, W, _, bscale), (dW, db) in zip(_norm_items(items), out):
        n_out, n_in = W.shape
        Mr = dY.shape[0]
        specs.append(((n_out, n_in, Mr), _prob([_seg(dY, X, n_out, n_in, Mr, alpha)], dW, n_out, n_in, n_in,
                                              bias_grad=db, bias_grad_scale=bscale / alpha)))
    return specs


def _wgrad_launch(specs, sk_late=0):
    """Grouped launches of the weight-gradient problems: equal (out, in, rows) shapes share a
    launch (up to GEMM_MAX_PROBLEMS), the kernel variant and split-K chosen per launch."""
    if not specs:
        return
    by_shape = {}
    for key, prob in specs:
        n_out, n_in, Kr = key
        # the k-split kernel (variant 46) takes problems of different shapes in one flat grid:
        # they share a launch by reduction length alone (an FFN's fc1 and fc2 weight gradients)
        mixed = _TNR_MIXED and _TNR and Kr % 64 == 0 and Kr >= 128 and not (0 < _TNB_MIN_K <= Kr)
        by_shape.setdefault((0, 0, Kr) if mixed else key, []).append((key, prob))
    launches = []
    for (_, _, Kr), allkp in by_shape.items():
        for c in range(0, len(allkp), L.GEMM_MAX_PROBLEMS):
            subk = allkp[c:c + L.GEMM_MAX_PROBLEMS]
            sub = [pr for _, pr in subk]
            n_out, n_in = max(k[0] for k, _ in subk), max(k[1] for k, _ in subk)
            tiles = sum(((k[0] + 63) // 64) * ((k[1] + 63) // 64) for k, _ in subk)
            sk = _splitk_for(Kr, tiles)
            tile = 0
            if 0 < _TNB_MIN_K <= Kr and Kr % 64 == 0:
                tile = 43
                sk = _tnb_split(Kr, len(sub) * -(-n_out // 128) * -(-n_in // 128))
            elif _TNR and Kr % 64 == 0 and Kr >= 128:
                # the k-split kernel with the register-staged, interleaved operand stream (variant
                # 46): 6-20 % faster than both the LDS-DMA k-split (36) and the plain LDS-DMA
                # kernel at every config-2 / 3 shape (tools/tn_library_compare.py,
                # profiles/r05_tn/tnr_compare_*.log); split 2, or 4 when that makes exactly one
                # full round of three workgroups per CU with >= 512 rows per split and the
                # problems are FFN-sized (config 2's 4 x (768, 256): +0.6 % in step over 2); the
                # many small problems of config 3's attention (12 x (256, 256)) run better at 2
                # in step (+1.1 %, profiles/r05_misc/tnr_split_rule_ab.txt) though 4 is faster alone
                big = all(k[0] * k[1] >= 768 * 256 for k, _ in subk)
                tile, sk = 46, (4 if tiles * 4 == 768 and Kr >= 2048 and big else (2 if Kr >= 512 else 1))
                if _TNR_MIXED_SK and len({k for k, _ in subk}) > 1 and Kr // _TNR_MIXED_SK >= 256:
                    sk = _TNR_MIXED_SK
                if _TNR_SK and Kr // _TNR_SK >= 256:
                    sk = _TNR_SK
                if sk_late and sk < sk_late and Kr // sk_late >= 256:  # raise only
                    sk = sk_late
            elif (len(sub) >= 8 and tiles >= 256) or tiles >= _TNK_TILES_PER_PROBLEM * len(sub):
                # many-problem launches (an attention block's q/k/v/o of every stream) and big
                # weights (an FFN's 768 x 256): the k-split outer-product kernel at split-K 2
                # (tools/tn_bench.py: 16 x (256 x 256, K = 2048) 0.59-0.61 of peak vs 0.57 for
                # the 64x64 LDS-DMA kernel at split 3; the FFN launches at split 2 instead of 4
                # write half the partial slabs, same step time; profiles/r04_probe/ab_tnk_ffn.txt)
                tile, sk = 36, min(sk, 2)
            wsz = sum(sk * (k[0] * k[1] + k[0]) for k, _ in subk)
            ws = torch.empty(wsz, device=torch.device("cuda", torch.cuda.current_device()),
                             dtype=torch.float32) if sk > 1 else None
            launches.append((sub, sk, ws, tile))
    for p, k, w, tl in launches:
        gemm(L.GEMM_TN, p, splitk=k, ws=w, tile=tl)


def sum_tensors(groups):
    """groups: [(out, [in_0, in_1, ...])] same-shaped contiguous fp32 tensors: out = sum of the
    ins in list order (sca_sum_tensors, one launch per 8 groups)."""
    if not groups:
        return
    n = groups[0][0].numel()
    for out, ins in groups:  # the launch applies one n to every problem
        for t in [out] + list(ins):
            if t.numel() != n or not t.is_contiguous() or t.dtype != torch.float32 or not t.is_cuda:
                raise ValueError(f"sum_tensors: every tensor must be a contiguous fp32 GPU tensor of {n} elements; "
                                 f"got {tuple(t.shape)} {t.dtype} on {t.device}, contiguous={t.is_contiguous()}")
    for c in range(0, len(groups), L.SUM_MAX_PROBLEMS):
        chunk = groups[c:c + L.SUM_MAX_PROBLEMS]
        probs = []
        for out, ins in chunk:
            if len(ins) > L.SUM_MAX_TERMS:
                raise ValueError(f"sum_tensors: at most {L.SUM_MAX_TERMS} terms")
            arr = (ctypes.c_void_p * L.SUM_MAX_TERMS)(*[t.data_ptr() for t in ins])
            probs.append(L.SumProblem(arr, len(ins), out.data_ptr()))
        L.check(L.lib().sca_sum_tensors(len(probs), (L.SumProblem * len(probs))(*probs), n, L.stream_handle()),
                "sca_sum_tensors")


class FanOut(Function):
    """The same G tensors handed to n consumers: forward returns n aliases of each (views);
    backward sums each tensor's n incoming gradients in one grouped launch (sca_sum_tensors,
    fixed order) instead of autograd's n - 1 pairwise adds per tensor as they arrive — the
    final x-stream map read by every merge layer (keypoint_module.py:181-187)."""

    @staticmethod
    def forward(ctx, n, G, *xs):
        ctx.n, ctx.G = n, G
        ctx.set_materialize_grads(False)  # an alias that got no gradient arrives as None: skipped
        return tuple(x.view_as(x) for _ in range(n) for x in xs)

    @staticmethod
    def backward(ctx, *gs):
        n, G = ctx.n, ctx.G
        groups, outs = [], []
        for g in range(G):
            terms = [t.contiguous() for t in (gs[i * G + g] for i in range(n)) if t is not None]
            if not terms:
                outs.append(None)
            elif len(terms) == 1:
                outs.append(terms[0])
            else:
                o = torch.empty_like(terms[0])
                groups.append((o, terms))
                outs.append(o)
        sum_tensors(groups)
        return (None, None) + tuple(outs)


_FAN_OUT = True


def fan_out(xs, n):
    """n lists of aliases of the G tensors xs (FanOut); [xs] * n when n < 2 or not on the HIP path."""
    if not _FAN_OUT or n < 2 or _LIBRARY_MODE or not torch.is_grad_enabled() or not any(x.requires_grad for x in xs):
        return [list(xs)] * n
    out = FanOut.apply(n, len(xs), *xs)
    return [list(out[i * len(xs):(i + 1) * len(xs)]) for i in range(n)]


def _flat(x):
    return x.reshape(-1, x.shape[-1])


def _contig(ts):
    return [t if t is None or t.is_contiguous() else t.contiguous() for t in ts]


def _zeros_for_none(grads, refs):
    return [g if g is not None else torch.zeros_like(r) for g, r in zip(grads, refs)]


# --------------------------------------------------------------------------- attention
def _attn_bwd_kernel_name(hd, am, causal, drop, Tq, Tk, dq_part):
    """The launch's main backward kernel as rocprofv3 names it (attention.hip launch_bwd): the
    fused hd-16 kernel (T <= 256), the hd-32 key-block kernel (+ its dQ reduce), else the
    split dq + dkdv pair (timed together, named by the dq kernel)."""
    tf = lambda b: "true" if b else "false"  # noqa: E731
    if hd == 16 and not am and Tq <= 256 and Tk <= 256:
        return f"attn_bwd_fused_kernel<{tf(causal)}, {tf(drop)}>"
    if hd == 32 and not am and dq_part:
        return f"attn_bwd_kblk_kernel<{tf(causal)}, {tf(drop)}>"
    return f"attn_bwd_dq_kernel<{hd}, {tf(am)}, {tf(causal)}, {tf(drop)}>"


_MASK_DTYPES = {torch.float32: 0, torch.float64: 1, torch.int64: 2, torch.int32: 3, torch.bool: 4, torch.uint8: 4,
                torch.float16: 5, torch.bfloat16: 6, torch.int8: 7, torch.int16: 8}


def key_valid_vector(mask):
    """(B, T) mask of any integer / bool / float dtype -> (B, T) fp32 1/0 key validity with the
    reference's predicate (kept iff the fp32 value equals 1; sca_key_valid)."""
    code = _MASK_DTYPES.get(mask.dtype)
    if code is None:
        raise TypeError(f"attention mask dtype {mask.dtype} is not supported")
    if not mask.is_cuda or torch.compiler.is_compiling():
        # the same predicate as an expression torch.compile can trace (and for a mask built on
        # the CPU: the attention launches that read it refuse CPU tensors themselves)
        return (mask.to(torch.float32) == 1).to(torch.float32)
    m = mask.contiguous()
    out = torch.empty(mask.shape, dtype=torch.float32, device=mask.device)
    L.check(L.lib().sca_key_valid(m.data_ptr(), code, out.data_ptr(), m.numel(), L.stream_handle()), "sca_key_valid")
    return out


class KeyPaddingMask:
    """The SCA mask contract without the B*T^2 materialisation: per-clip key validity
    (B, Tk) as fp32 1/0 plus the causal flags.  Semantically identical to the additive masks
    of model/utils.py:3-28 (see include/scatten.h for the exact score transform)."""

    def __init__(self, mask, causal_plus_one=False):
        if mask.dim() != 2:
            raise ValueError("key padding mask must be (B, T)")
        self.mask = mask
        self.causal_plus_one = causal_plus_one
        # the reference keeps a key only where mask == 1 (model/utils.py:8-12: 1.0 - mask is
        # masked wherever non-zero), written as fp32 1/0 by one sca_key_valid launch
        self.key_valid = key_valid_vector(mask)

    def causal_view(self):
        """The causal variant (create_causal_attention_mask) sharing this key-validity vector."""
        m = KeyPaddingMask.__new__(KeyPaddingMask)
        m.mask, m.causal_plus_one, m.key_valid = self.mask, True, self.key_valid
        return m

    @property
    def shape(self):
        return self.mask.shape


def _mask_heads(add_mask):
    """add_mask (B, Tq, Tk) -> 1 (one mask for every head); (B, H, Tq, Tk) -> H."""
    return add_mask.shape[1] if add_mask is not None and add_mask.dim() == 4 else 1


_KERNEL_HD = (16, 32, 64, 128)  # head sizes the attention kernels are built for


def _padded_hd(hd):
    """Kernel head size for a module head size (<= 128): hd itself, or the next kernel size when the
    heads are zero-padded (exact: zero q / k columns add nothing to a score, zero v columns
    give zero output columns and the padded gradient columns are dropped).  Larger heads take
    the GEMM path (_attn_fwd_gemm) before this is asked."""
    for k in _KERNEL_HD:
        if hd <= k:
            return k
    raise ValueError(f"head_dim {hd} > {_KERNEL_HD[-1]} is not supported by the attention kernels")


def _pad_heads(ts, H, hd, hdp):
    """(B, T, H*hd) -> (B, T, H*hdp), each head's columns followed by hdp - hd zeros."""
    return [torch.nn.functional.pad(t.reshape(t.shape[0], t.shape[1], H, hd), (0, hdp - hd))
            .reshape(t.shape[0], t.shape[1], H * hdp) for t in ts]


def _unpad_heads(ts, H, hd, hdp):
    return [t.reshape(t.shape[0], t.shape[1], H, hdp)[..., :hd].reshape(t.shape[0], t.shape[1], H * hd)
            for t in ts]


# ---- head sizes over 128: scores through the grouped GEMM, softmax through the row kernel ----
# The reference accepts any d_model % num_heads == 0 (attention.py:16-20); the fused attention
# kernels are built for head sizes up to 128.  Larger heads run per (stream, clip, head) as
#   S = q k^T + M (NT GEMM, the additive mask M as its residual operand), P = softmax_rows(S),
#   o = P v (NN GEMM)
# with P kept (B, H, Tq, Tk) for the backward: dP = dO v^T (NT), dv = P^T dO (TN),
# dS = softmax_rows_bwd(P, dP), dq = dS k (NN), dk = dS^T q (TN).  M reproduces the kernels'
# masking exactly: causal j > i -> -inf; else the materialised additive mask, or finfo.min
# for an invalid key / +1 where causal && plus_one (include/scatten.h).

def _dense_mask(B, H, Tq, Tk, causal, plus_one, key_valid, add_mask, device):
    """(B, H or 1, Tq, Tk) additive mask with the attention kernels' semantics."""
    if add_mask is not None:
        m = add_mask if add_mask.dim() == 4 else add_mask[:, None]
        m = m.clone()
    else:
        base = torch.full((B, 1, Tq, Tk), 1.0 if (causal and plus_one) else 0.0, device=device)
        if key_valid is not None:
            base = torch.where(key_valid[:, None, None, :] == 0, torch.finfo(torch.float32).min, base)
        m = base
    if causal:
        above = torch.ones(Tq, Tk, dtype=torch.bool, device=device).triu(1)
        m = m.masked_fill(above, float("-inf"))
    return m.contiguous()


def _raw_prob(A, B, lda, ldb, K, C, M, N, ldc, alpha=1.0, resid=None, ldr=0):
    segs = (L.GemmSeg * 3)(L.GemmSeg(A, B, lda, ldb, K, alpha), _NOSEG, _NOSEG)
    return L.GemmProblem(segs, 1, M, N, C, ldc, 0, None, 1.0, resid, ldr, None, 0, None, 0, None, 1.0, 0, 0.0)


def _softmax_rows_launch(pairs, rows, N, bwd=False):
    """pairs: [(x or y, y or dy, out)] raw pointers, each `rows` rows of N."""
    fn = L.lib().sca_softmax_rows_bwd if bwd else L.lib().sca_softmax_rows_fwd
    for c in range(0, len(pairs), L.SOFTMAX_MAX_PROBLEMS):
        ch = pairs[c:c + L.SOFTMAX_MAX_PROBLEMS]
        probs = [L.SoftmaxProblem(None, a, b, o) if bwd else L.SoftmaxProblem(a, None, None, o) for a, b, o in ch]
        arr = (L.SoftmaxProblem * len(probs))(*probs)
        with _timed("softmax_bwd_kernel" if bwd else "softmax_fwd_kernel", 0.0):
            L.check(fn(len(probs), arr, rows, N, L.stream_handle()), "sca_softmax_rows_" + ("bwd" if bwd else "fwd"))


def _attn_fwd_gemm(G, H, causal, plus_one, key_valid, add_mask, q, k, v, drop):
    """drop: None or (p, seeds): o = dropout(P) v with the kernels' mask (sca_dropout over the
    (B, H, Tq, Tk) probabilities, element ((b H + h) Tq + i) Tk + j, attention.py:67-69); P
    itself (undropped) is kept for the backward."""
    B, Tq, d = q[0].shape
    Tk = k[0].shape[1]
    hd = d // H
    dev = q[0].device
    mask = _dense_mask(B, H, Tq, Tk, causal, plus_one, key_valid, add_mask, dev)
    mh = mask.shape[1]
    o = [torch.empty_like(t) for t in q]
    P = [torch.empty(B, H, Tq, Tk, device=dev) for _ in range(G)]
    probs, soft = [], []
    for g in range(G):
        for b in range(B):
            for h in range(H):
                S = P[g][b, h]
                mk = mask[b, h if mh > 1 else 0]
                probs.append(_raw_prob(q[g].data_ptr() + 4 * (b * Tq * d + h * hd),
                                       k[g].data_ptr() + 4 * (b * Tk * d + h * hd), d, d, hd,
                                       S.data_ptr(), Tq, Tk, Tk, resid=mk.data_ptr(), ldr=Tk))
                soft.append((S.data_ptr(), None, S.data_ptr()))
    gemm(L.GEMM_NT, probs)
    _softmax_rows_launch(soft, Tq, Tk)
    Pv = P
    if drop:
        Pv = [torch.empty_like(t) for t in P]
        dropout_apply([(P[g], Pv[g], drop[1][g]) for g in range(G)], drop[0])
    probs = [_raw_prob(Pv[g][b, h].data_ptr(), v[g].data_ptr() + 4 * (b * Tk * d + h * hd), Tk, d, Tk,
                       o[g].data_ptr() + 4 * (b * Tq * d + h * hd), Tq, hd, d)
             for g in range(G) for b in range(B) for h in range(H)]
    gemm(L.GEMM_NN, probs)
    # in place of the kernels' row statistics: P (flat) and an empty tensor
    return o, [p.view(-1) for p in P], [q[0].new_empty(0) for _ in range(G)]


def _attn_bwd_gemm(G, H, q, k, v, P, dout, dq_scale, dv_scale, drop=None):
    """With dropout (p, seeds): dP = dropout(dO v^T) (the same mask and 1/(1-p): the gradient of
    dropout(P)), dv = dropout(P)^T dO."""
    B, Tq, d = q[0].shape
    Tk = k[0].shape[1]
    hd = d // H
    P = [p.view(B, H, Tq, Tk) for p in P]
    dq = [torch.empty_like(t) for t in q]
    dk = [torch.empty_like(t) for t in k]
    dv = [torch.empty_like(t) for t in v]
    dS = [torch.empty_like(p) for p in P]
    idx = [(g, b, h) for g in range(G) for b in range(B) for h in range(H)]
    off = lambda b, h, T: 4 * (b * T * d + h * hd)  # noqa: E731
    # dP = dO v^T  (into dS), then dS = softmax_bwd(P, dP) in place
    gemm(L.GEMM_NT, [_raw_prob(dout[g].data_ptr() + off(b, h, Tq), v[g].data_ptr() + off(b, h, Tk), d, d, hd,
                               dS[g][b, h].data_ptr(), Tq, Tk, Tk) for g, b, h in idx])
    Pv = P
    if drop:
        dropout_apply([(dS[g], dS[g], drop[1][g]) for g in range(G)], drop[0])
        Pv = [torch.empty_like(t) for t in P]
        dropout_apply([(P[g], Pv[g], drop[1][g]) for g in range(G)], drop[0])
    _softmax_rows_launch([(P[g][b, h].data_ptr(), dS[g][b, h].data_ptr(), dS[g][b, h].data_ptr())
                          for g, b, h in idx], Tq, Tk, bwd=True)
    # dv = P^T dO, dk = dS^T q (TN over the Tq rows); dq = dS k (NN)
    gemm(L.GEMM_TN, [_raw_prob(Pv[g][b, h].data_ptr(), dout[g].data_ptr() + off(b, h, Tq), Tk, d, Tq,
                               dv[g].data_ptr() + off(b, h, Tk), Tk, hd, d, alpha=dv_scale) for g, b, h in idx])
    gemm(L.GEMM_TN, [_raw_prob(dS[g][b, h].data_ptr(), q[g].data_ptr() + off(b, h, Tq), Tk, d, Tq,
                               dk[g].data_ptr() + off(b, h, Tk), Tk, hd, d) for g, b, h in idx])
    gemm(L.GEMM_NN, [_raw_prob(dS[g][b, h].data_ptr(), k[g].data_ptr() + off(b, h, Tk), Tk, d, Tk,
                               dq[g].data_ptr() + off(b, h, Tq), Tq, hd, d, alpha=dq_scale) for g, b, h in idx])
    return dq, dk, dv


def _attn_fwd(G, H, causal, plus_one, key_valid, add_mask, q, k, v, drop=None):
    """drop: None or (p, seeds) — attention-probability dropout, one seed per problem.
    Head sizes other than 16 / 32 / 64 / 128 run zero-padded to the next kernel size; head
    sizes over 128 take the GEMM + row-softmax path (then `sm` is P, flat, and `sl` empty)."""
    B, Tq, d = q[0].shape
    Tk = k[0].shape[1]
    hd = d // H
    if hd > _KERNEL_HD[-1]:
        return _attn_fwd_gemm(G, H, causal, plus_one, key_valid, add_mask, q, k, v, drop)
    hdp = _padded_hd(hd)
    if hdp != hd:
        qp, kp, vp = (_pad_heads(ts, H, hd, hdp) for ts in (q, k, v))
        o, sm, sl = _attn_fwd(G, H, causal, plus_one, key_valid, add_mask, qp, kp, vp, drop)
        return _unpad_heads(o, H, hd, hdp), sm, sl
    o = [torch.empty_like(t) for t in q]
    sm = [q[0].new_empty(B * H * Tq) for _ in range(G)]
    sl = [q[0].new_empty(B * H * Tq) for _ in range(G)]
    for c in range(0, G, L.ATTN_MAX_PROBLEMS):
        gs = range(c, min(G, c + L.ATTN_MAX_PROBLEMS))
        arr = (L.AttnFwdProblem * len(gs))(*[
            L.AttnFwdProblem(q[g].data_ptr(), k[g].data_ptr(), v[g].data_ptr(), o[g].data_ptr(),
                             sm[g].data_ptr(), sl[g].data_ptr(), ptr(key_valid), ptr(add_mask),
                             drop[1][g] if drop else 0, drop[0] if drop else 0.0, _mask_heads(add_mask)) for g in gs])
        fl = len(gs) * 4.0 * B * H * hd * (Tq * (Tq + 1) / 2 if causal else Tq * Tk)
        tf = lambda b: "true" if b else "false"  # noqa: E731
        with _timed(f"attn_fwd_kernel<{hd}, {tf(add_mask is not None)}, {tf(causal)}, {tf(drop)}>", fl):
            L.check(L.lib().sca_attn_fwd(len(gs), arr, B, H, Tq, Tk, hd, d, d, d, d, int(causal), int(plus_one),
                                         L.stream_handle()), "sca_attn_fwd")
    return o, sm, sl


def _attn_bwd(G, H, causal, plus_one, key_valid, add_mask, q, k, v, o, sm, sl, dout, dq_scale=1.0, dv_scale=1.0,
              drop=None):
    B, Tq, d = q[0].shape
    Tk = k[0].shape[1]
    hd = d // H
    if hd > _KERNEL_HD[-1]:  # the GEMM path: sm is P
        return _attn_bwd_gemm(G, H, q, k, v, sm, dout, dq_scale, dv_scale, drop)
    hdp = _padded_hd(hd)
    if hdp != hd:
        qp, kp, vp, op, dop = (_pad_heads(ts, H, hd, hdp) for ts in (q, k, v, o, dout))
        grads = _attn_bwd(G, H, causal, plus_one, key_valid, add_mask, qp, kp, vp, op, sm, sl, dop, dq_scale,
                          dv_scale, drop)
        return tuple(_unpad_heads(g, H, hd, hdp) for g in grads)
    dq = [torch.empty_like(t) for t in q]
    dk = [torch.empty_like(t) for t in k]
    dv = [torch.empty_like(t) for t in v]
    delta = [q[0].new_empty(B * H * Tq) for _ in range(G)]
    # the fused hd-32 backward (256-key blocks) writes per-key-block dQ partials
    nws = L.lib().sca_attn_bwd_workspace(B, H, Tq, Tk, hd) if add_mask is None else 0
    part = [q[0].new_empty(nws) for _ in range(G)] if nws > 0 else [None] * G
    for c in range(0, G, L.ATTN_MAX_PROBLEMS):
        gs = range(c, min(G, c + L.ATTN_MAX_PROBLEMS))
        arr = (L.AttnBwdProblem * len(gs))(*[
            L.AttnBwdProblem(q[g].data_ptr(), k[g].data_ptr(), v[g].data_ptr(), o[g].data_ptr(),
                             dout[g].data_ptr(), sm[g].data_ptr(), sl[g].data_ptr(), ptr(key_valid),
                             ptr(add_mask), dq[g].data_ptr(), dk[g].data_ptr(), dv[g].data_ptr(),
                             delta[g].data_ptr(), dq_scale, dv_scale, ptr(part[g]),
                             drop[1][g] if drop else 0, drop[0] if drop else 0.0, _mask_heads(add_mask))
            for g in gs])
        fl = len(gs) * 8.0 * B * H * hd * (Tq * (Tq + 1) / 2 if causal else Tq * Tk)
        with _timed(_attn_bwd_kernel_name(hd, add_mask is not None, causal, drop is not None, Tq, Tk,
                                          part[0] is not None), fl):
            L.check(L.lib().sca_attn_bwd(len(gs), arr, B, H, Tq, Tk, hd, d, d, d, d, int(causal), int(plus_one),
                                         L.stream_handle()), "sca_attn_bwd")
    return dq, dk, dv


class AttentionBlock(Function):
    """One attention operator end to end, G streams per launch:

        q = (x_q Wq^T + bq) * scale ; k = x_kv Wk^T + bk ; v = (alpha_v x_kv) Wv^T + bv
        o = softmax(q k^T + mask) v      (per head; fused kernel, nothing T^2 in HBM)
        y = o Wo^T + bo (+ x_q)          (the enclosing post-LN block's residual, fused)

    kinds: "self" (attention.py:46-76), "causal" (:148-182), "cross" (:97-128, x_kv =
    key_value_states, alpha_v = 0.5 reproduces v_proj(kv / 2)).  The backward fuses the
    residual gradient into the dX GEMM epilogue and all of the block's weight/bias gradients
    into grouped split-K TN GEMMs."""

    @staticmethod
    def forward(ctx, G, kind, H, scale, plus_one, key_valid, add_mask, has_resid, drop_p, ln_eps, nxt, attn_p,
                *ts):
        cross = kind == "cross"
        ln = ln_eps is not None  # post-LN LayerNorm fused into the out-projection (sca_gemm_ln)
        if ln:
            gam, bet, ts = ts[-2 * G:-G], ts[-G:], ts[:-2 * G]
        causal = kind == "causal"
        lnprev = ln_saved_of(ts[:G])  # the query input came out of a fused GEMM + LayerNorm
        xq = _contig(ts[:G])
        o_ = G
        xkv = _contig(ts[o_:o_ + G]) if cross else xq
        o_ += G if cross else 0
        W = ts[o_:o_ + 6 * G]
        Wo, bo = ts[o_ + 6 * G:o_ + 7 * G], ts[o_ + 7 * G:o_ + 8 * G]
        L.require_device(*xq, *xkv)
        B, T, d = xq[0].shape
        Tk = xkv[0].shape[1]
        av = 0.5 if cross else 1.0
        q, k, v, probs = [], [], [], []
        pre = None
        if not cross:  # q / k / v computed by the producer of x (chained passes of its launch)
            pre = [n.take(g, ts[g], [(W[6 * g], W[6 * g + 1]), (W[6 * g + 2], W[6 * g + 3]),
                                     (W[6 * g + 4], W[6 * g + 5])]) if n is not None and ts[g] is xq[g] else None
                   for g, n in enumerate(_next_of(ts[:G]))]
            if any(p is None for p in pre):
                pre = None
        if pre is not None:
            q = [p[0][0].view(B, T, d) for p in pre]
            k = [p[1][0].view(B, T, d) for p in pre]
            v = [p[2][0].view(B, T, d) for p in pre]
        else:
            for g in range(G):
                Wq, bq, Wk, bk, Wv, bv = W[6 * g:6 * g + 6]
                xf, kf = _flat(xq[g]), _flat(xkv[g])
                q.append(xq[g].new_empty(B, T, d))
                k.append(xq[g].new_empty(B, Tk, d))
                v.append(xq[g].new_empty(B, Tk, d))
                probs.append(_prob([_seg(xf, Wq, d, d, d)], q[g], B * T, d, d, bias=bq, post_scale=scale))
                probs.append(_prob([_seg(kf, Wk, d, d, d)], k[g], B * Tk, d, d, bias=bk))
                probs.append(_prob([_seg(kf, Wv, d, d, d, av)], v[g], B * Tk, d, d, bias=bv))
            gemm(L.GEMM_NT, probs)
        # attention-probability dropout (attention.py:67-69): its seeds precede the block's own
        attn_drop = (attn_p, dropout_seeds(G)) if attn_p > 0 else None
        o, sm, sl = _attn_fwd(G, H, causal, plus_one, key_valid, add_mask, q, k, v, drop=attn_drop)
        # v = x + dropout(o Wo^T + bo)  (keypoint_module.py:63-65 / :99-101) in one epilogue,
        # and with `ln` the block's LayerNorm y = LN(v) in the same launch
        seeds = dropout_seeds(G) if drop_p > 0 else [None] * G
        if ln:
            vs, ys, means, rstds = _ln_fwd_outputs(xq)
        else:
            ys = vs = [torch.empty_like(x) for x in xq]
        probs = [_prob([_seg(_flat(o[g]), Wo[g], d, d, d)], vs[g], B * T, d, d, bias=bo[g],
                       resid=_flat(xq[g]) if has_resid else None, ldr=d,
                       drop=(seeds[g], drop_p) if drop_p > 0 else None) for g in range(G)]
        if ln:
            gemm_ln(probs, _chain_lns(nxt, G, B * T, xq[0], gam, bet, ys, means, rstds), ln_eps)
            if nxt is not None:
                nxt.attach(ys)
        else:
            gemm(L.GEMM_NT, probs)
        ctx.G, ctx.kind, ctx.H, ctx.scale, ctx.plus_one, ctx.has_resid = G, kind, H, scale, plus_one, has_resid
        ctx.attn_drop = attn_drop
        ctx.drop_p, ctx.seeds, ctx.ln = drop_p, seeds, ln
        ctx.bet = tuple(bet) if ln else ()  # parameters (leaves): identify their gradients' slots
        ctx.lnsaved = _attach_ln_saved(ys, vs, means, rstds, gam, Wo if drop_p == 0 else None) if ln else None
        ctx.lnprev = lnprev if (lnprev is not None and ln_width_ok(d) and has_resid) else None
        ctx.save_for_backward(key_valid, add_mask, *xq, *(xkv if cross else []), *W, *Wo, *bo, *q, *k, *v, *o,
                              *sm, *sl, *((*vs, *gam, *means, *rstds) if ln else ()))
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        G, kind, H, scale = ctx.G, ctx.kind, ctx.H, ctx.scale
        cross = kind == "cross"
        sv = ctx.saved_tensors
        key_valid, add_mask = sv[0], sv[1]
        i = 2
        xq = sv[i:i + G]
        i += G
        xkv = sv[i:i + G] if cross else xq
        i += G if cross else 0
        W = sv[i:i + 6 * G]
        i += 6 * G
        Wo, bo = sv[i:i + G], sv[i + G:i + 2 * G]
        i += 2 * G
        q, k, v, o, sm, sl = (sv[i + j * G:i + (j + 1) * G] for j in range(6))
        B, T, d = xq[0].shape
        Tk = xkv[0].shape[1]
        av = 0.5 if cross else 1.0
        dgam = dbet = ()
        ln_finish = None
        do = None
        if ctx.ln:  # through the fused LayerNorm first: dys becomes the gradient of v
            i += 6 * G
            vs, gam, means, rstds = (sv[i + j * G:i + (j + 1) * G] for j in range(4))
            dys, dgam, dbet, ln_finish, do = _ln_bwd_or_handoff(dys, vs, gam, means, rstds, ctx.lnsaved, ctx.bet)
            dgam, dbet = tuple(dgam), tuple(dbet)
        else:
            dys = _contig(_zeros_for_none(dys, xq))
        dyo = dys  # gradient of the out-projection output: the dropout mask applied to dY
        if ctx.drop_p > 0:
            dyo = [torch.empty_like(t) for t in dys]
            dropout_apply([(dys[g], dyo[g], ctx.seeds[g]) for g in range(G)], ctx.drop_p)
        # out-projection: dO = dY' Wo (unless the consumer's sca_gemm_lnb already chained it)
        if do is None:
            do = [torch.empty_like(t) for t in o]
            gemm(L.GEMM_NN, [_prob([_seg(_flat(dyo[g]), Wo[g], d, d, d)], do[g], B * T, d, d) for g in range(G)])
        # dq comes back pre-multiplied by the q scale and dv by alpha_v, so that every GEMM below
        # runs with unit segment scales: dX = dq' Wq + dk Wk + dv' Wv, dWq = dq'^T x, ...
        dq, dk, dv = _attn_bwd(G, H, kind == "causal", ctx.plus_one, key_valid, add_mask, q, k, v, o, sm, sl, do,
                               dq_scale=scale, dv_scale=av, drop=ctx.attn_drop)
        # input gradients (residual gradient fused as the epilogue's resid term); with `lnprev`
        # the query input's LayerNorm backward rides in the same launch (sca_gemm_lnb)
        dxq, dxkv, probs, kvprobs = [], [], [], []
        for g in range(G):
            Wq, _, Wk, _, Wv, _ = W[6 * g:6 * g + 6]
            dqf, dkf, dvf = _flat(dq[g]), _flat(dk[g]), _flat(dv[g])
            r = _flat(dys[g]) if ctx.has_resid else None
            gx = torch.empty_like(xq[g])
            if cross:
                gkv = torch.empty_like(xkv[g])
                probs.append(_prob([_seg(dqf, Wq, d, d, d)], gx, B * T, d, d, resid=r, ldr=d))
                kvprobs.append(_prob([_seg(dkf, Wk, d, d, d), _seg(dvf, Wv, d, d, d)], gkv, B * Tk, d, d))
                dxkv.append(gkv)
            else:
                probs.append(_prob([_seg(dqf, Wq, d, d, d), _seg(dkf, Wk, d, d, d), _seg(dvf, Wv, d, d, d)],
                                   gx, B * T, d, d, resid=r, ldr=d))
            dxq.append(gx)
        ready = wgrad_ready()
        if ctx.lnprev is not None:
            hand_off(ctx.lnprev, dxq, *gemm_lnb(probs, ctx.lnprev))
            ctx.lnprev = None
            gemm(L.GEMM_NN, kvprobs)
        else:
            gemm(L.GEMM_NN, probs + kvprobs)
        # weight / bias gradients (bias colsum fused in the TN GEMMs)
        items = []
        for g in range(G):
            Wq, bq, Wk, bk, Wv, bv = W[6 * g:6 * g + 6]
            xf, kf = _flat(xq[g]), _flat(xkv[g])
            items += [(_flat(dq[g]), xf, 1.0, Wq, bq), (_flat(dk[g]), kf, 1.0, Wk, bk),
                      (_flat(dv[g]), kf, 1.0, Wv, bv, 1.0 / av),
                      (_flat(dyo[g]), _flat(o[g]), 1.0, Wo[g], bo[g])]
        wg = weight_grads(items, extra=ln_finish, ready=ready, holdable=True)
        dW, dWo, dbo = [], [], []
        for g in range(G):
            for j in range(3):
                dW += list(wg[4 * g + j])
            dWo.append(wg[4 * g + 3][0])
            dbo.append(wg[4 * g + 3][1])
        return (None,) * 12 + tuple(dxq) + (tuple(dxkv) if cross else ()) + tuple(dW) + tuple(dWo) + \
            tuple(dbo) + dgam + dbet


# --------------------------------------------------------------------------- Linear (+ residual)
class LinearResidual(Function):
    """y = x W^T + b (+ r).  Out-projection of every attention op (attention.py:74) fused with
    the post-LN residual add of keypoint_module.py:69-70 / :105-106 when r is given."""

    @staticmethod
    def forward(ctx, G, has_r, *ts):
        x = _contig(ts[:G])
        W, b = ts[G:2 * G], ts[2 * G:3 * G]
        r = _contig(ts[3 * G:4 * G]) if has_r else [None] * G
        L.require_device(*x)
        probs, ys = [], []
        for g in range(G):
            n_out, n_in = W[g].shape
            lead = x[g].shape[:-1]
            M = x[g].numel() // n_in
            y = x[g].new_empty(*lead, n_out)
            probs.append(_prob([_seg(_flat(x[g]), W[g], n_in, n_in, n_in)], y, M, n_out, n_out, bias=b[g],
                               resid=r[g], ldr=n_out))
            ys.append(y)
        gemm(L.GEMM_NT, probs)
        ctx.G, ctx.has_r, ctx.b = G, has_r, tuple(b)  # biases: parameters (leaves) or None
        ctx.save_for_backward(*x, *W)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        G = ctx.G
        sv = ctx.saved_tensors
        x, W = sv[:G], sv[G:2 * G]
        dys = _contig(_zeros_for_none(dys, [x[g].new_empty(*x[g].shape[:-1], W[g].shape[0]) for g in range(G)]))
        probs, dxs = [], []
        for g in range(G):
            n_out, n_in = W[g].shape
            M = x[g].numel() // n_in
            dx = torch.empty_like(x[g])
            probs.append(_prob([_seg(_flat(dys[g]), W[g], n_out, n_in, n_out)], dx, M, n_in, n_in))
            dxs.append(dx)
        ready = wgrad_ready()
        gemm(L.GEMM_NN, probs)
        wg = weight_grads([(_flat(dys[g]), _flat(x[g]), 1.0, W[g], ctx.b[g]) for g in range(G)], ready=ready)
        return (None, None) + tuple(dxs) + tuple(w for w, _ in wg) + tuple(bb for _, bb in wg) + \
            (tuple(dys) if ctx.has_r else ())


# --------------------------------------------------------------------------- FFN (+ residual)
class FeedForwardResidual(Function):
    """y = fc2(GELU(fc1 x)) (+ x when has_r)  (layers.py:94-108 with the residual of keypoint_module.py:71-72,
    :108-109).  fc1's epilogue applies bias + exact-erf GELU and keeps the pre-activation; the
    backward's dX GEMM of fc2 applies GELU' in its epilogue."""

    @staticmethod
    def forward(ctx, G, has_r, drop_p, ln_eps, nxt, *ts):
        lnprev = ln_saved_of(ts[:G])  # the input came out of a fused GEMM + LayerNorm
        x = _contig(ts[:G])
        W1, b1, W2, b2 = ts[G:2 * G], ts[2 * G:3 * G], ts[3 * G:4 * G], ts[4 * G:5 * G]
        ln = ln_eps is not None  # the block's last LayerNorm fused into fc2 (sca_gemm_ln)
        if ln:
            gam, bet = ts[5 * G:6 * G], ts[6 * G:7 * G]
        L.require_device(*x)
        B, T, d = x[0].shape
        M = B * T
        F_ = W1[0].shape[0]
        # layers.py:104-107: dropout(GELU(fc1 x)) -> fc2 -> dropout (+ x), each dropout fused
        s1 = dropout_seeds(G) if drop_p > 0 else [None] * G
        s2 = dropout_seeds(G) if drop_p > 0 else [None] * G
        pre = None
        if drop_p == 0:  # fc1 computed by the producer of x (chained passes of its launch)
            pre = [n.take(g, ts[g], [(W1[g], b1[g])]) if n is not None and ts[g] is x[g] else None
                   for g, n in enumerate(_next_of(ts[:G]))]
            if any(p is None for p in pre):
                pre = None
        if pre is not None:
            acts = [p[0][0] for p in pre]
            zs = [p[0][1] for p in pre]
        else:
            zs = [x[0].new_empty(M, F_) for _ in range(G)]
            acts = [x[0].new_empty(M, F_) for _ in range(G)]
            gemm(L.GEMM_NT, [_prob([_seg(_flat(x[g]), W1[g], d, d, d)], acts[g], M, F_, F_, bias=b1[g],
                                   epi=L.EPI_GELU, aux_out=zs[g], ldo=F_,
                                   drop=(s1[g], drop_p) if drop_p > 0 else None) for g in range(G)])
        if ln:
            vs, ys, means, rstds = _ln_fwd_outputs(x)
        else:
            ys = vs = [torch.empty_like(x[g]) for g in range(G)]
        probs = [_prob([_seg(acts[g], W2[g], F_, F_, F_)], vs[g], M, d, d, bias=b2[g],
                       resid=_flat(x[g]) if has_r else None, ldr=d,
                       drop=(s2[g], drop_p) if drop_p > 0 else None) for g in range(G)]
        if ln:
            gemm_ln(probs, _chain_lns(nxt, G, M, x[0], gam, bet, ys, means, rstds), ln_eps)
            if nxt is not None:
                nxt.attach(ys)
        else:
            gemm(L.GEMM_NT, probs)
        ctx.G, ctx.has_r, ctx.drop_p, ctx.s1, ctx.s2, ctx.ln = G, has_r, drop_p, s1, s2, ln
        ctx.b1, ctx.b2, ctx.bet = tuple(b1), tuple(b2), (tuple(bet) if ln else ())  # parameters (leaves)
        # dz = (dL/dv W2) * gelu'(z) chained into the consumer's launch (no dropout in between)
        dz_chain = drop_p == 0 and _CHAIN_DZ
        ctx.lnsaved = _attach_ln_saved(ys, vs, means, rstds, gam, W2 if dz_chain else None,
                                       zs if dz_chain else None) if ln else None
        ctx.lnprev = lnprev if (lnprev is not None and ln_width_ok(d) and has_r and F_ % 32 == 0) else None
        ctx.save_for_backward(*x, *W1, *W2, *zs, *acts, *((*vs, *gam, *means, *rstds) if ln else ()))
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        G = ctx.G
        sv = ctx.saved_tensors
        x, W1, W2, zs, acts = (sv[i * G:(i + 1) * G] for i in range(5))
        dgam = dbet = ()
        ln_finish = dzc = None
        if ctx.ln:  # through the fused LayerNorm first: dys becomes the gradient of v
            vs, gam, means, rstds = (sv[(5 + i) * G:(6 + i) * G] for i in range(4))
            dys, dgam, dbet, ln_finish, dzc = _ln_bwd_or_handoff(dys, vs, gam, means, rstds, ctx.lnsaved, ctx.bet)
            dgam, dbet = tuple(dgam), tuple(dbet)
        else:
            dys = _contig(_zeros_for_none(dys, x))
        B, T, d = x[0].shape
        M = B * T
        F_ = W1[0].shape[0]
        p = ctx.drop_p
        dyo = dys  # gradient of fc2's output (second dropout's mask applied)
        if p > 0:
            dyo = [torch.empty_like(t) for t in dys]
            dropout_apply([(dys[g], dyo[g], ctx.s2[g]) for g in range(G)], p)
        # dz = mask1 * (dy' W2) * gelu'(z) — or already computed by the consumer's launch
        if dzc is not None and p == 0:
            dz = [t.reshape(M, F_) for t in dzc]
        else:
            dz = [x[0].new_empty(M, F_) for _ in range(G)]
            gemm(L.GEMM_NN, [_prob([_seg(_flat(dyo[g]), W2[g], d, F_, d)], dz[g], M, F_, F_, epi=L.EPI_DGELU,
                                   aux=zs[g], ldx=F_, drop=(ctx.s1[g], p) if p > 0 else None) for g in range(G)])
        # dx = dz W1 + dy   (residual); with `lnprev` the input's LayerNorm backward rides in
        # the same launch (sca_gemm_lnb)
        dx = [torch.empty_like(x[g]) for g in range(G)]
        ready = wgrad_ready()
        probs = [_prob([_seg(dz[g], W1[g], F_, d, F_)], dx[g], M, d, d,
                       resid=_flat(dys[g]) if ctx.has_r else None, ldr=d) for g in range(G)]
        if ctx.lnprev is not None:
            hand_off(ctx.lnprev, dx, *gemm_lnb(probs, ctx.lnprev))
            ctx.lnprev = None
        else:
            gemm(L.GEMM_NN, probs)
        items = [(_flat(dyo[g]), acts[g], 1.0, W2[g], ctx.b2[g] if ctx.b2[g] is not None else True)
                 for g in range(G)] + \
                [(dz[g], _flat(x[g]), 1.0, W1[g], ctx.b1[g] if ctx.b1[g] is not None else True) for g in range(G)]
        wg = weight_grads(items, extra=ln_finish, ready=ready, holdable=True)
        dW2 = [wg[g] for g in range(G)]
        dW1 = [wg[G + g] for g in range(G)]
        return (None,) * 5 + tuple(dx) + tuple(w for w, _ in dW1) + tuple(b for _, b in dW1) + \
            tuple(w for w, _ in dW2) + tuple(b for _, b in dW2) + dgam + dbet


# --------------------------------------------------------------------------- LayerNorm
class LayerNormAdd(Function):
    """y = act(LayerNorm(x + r) + post).

    r: None (plain LayerNorm) or the LearningPositionEmbedding table (layers.py:15-30), row
       (t % T) + 2 of which is added to frame t;
    post, act: the ResidualBlock tail relu(norm2(.) + residual) (model/residual.py:35-38),
       or ReLU alone (norm1 -> relu, :32-33)."""

    @staticmethod
    def forward(ctx, G, eps, pos_table, has_post, act, drop_p, *ts):
        x = _contig(ts[:G])
        o = G
        tab = ts[o:o + G] if pos_table else [None] * G
        o += G if pos_table else 0
        post = _contig(ts[o:o + G]) if has_post else [None] * G
        o += G if has_post else 0
        gam, bet = ts[o:o + G], ts[o + G:o + 2 * G]
        L.require_device(*x)
        N = x[0].shape[-1]
        rows = x[0].numel() // N
        if pos_table:
            T = x[0].shape[1]
            if T + 2 > tab[0].shape[0]:
                raise IndexError("index out of range in self")  # nn.Embedding past its table
            r_mod, r_off = T, 2
        else:
            r_mod, r_off = max(rows, 1), 0
        ys = [torch.empty_like(t) for t in x]
        means = [x[0].new_empty(rows) for _ in range(G)]
        rstds = [x[0].new_empty(rows) for _ in range(G)]
        seeds = dropout_seeds(G) if drop_p > 0 else [0] * G
        for c in range(0, G, L.LN_MAX_PROBLEMS):
            gs = range(c, min(G, c + L.LN_MAX_PROBLEMS))
            arr = (L.LnFwdProblem * len(gs))(*[L.LnFwdProblem(x[g].data_ptr(), ptr(tab[g]), gam[g].data_ptr(),
                                                                bet[g].data_ptr(), ptr(post[g]), ys[g].data_ptr(),
                                                                means[g].data_ptr(), rstds[g].data_ptr(), act,
                                                                seeds[g], float(drop_p))
                                                 for g in gs])
            L.check(L.lib().sca_layernorm_fwd(len(gs), arr, rows, N, r_mod, r_off, eps, L.stream_handle()),
                    "sca_layernorm_fwd")
        ctx.G, ctx.pos, ctx.has_post, ctx.act, ctx.r_mod, ctx.r_off = G, pos_table, has_post, act, r_mod, r_off
        ctx.drop_p, ctx.seeds = drop_p, seeds
        ctx.bet = tuple(bet)  # parameters (leaves): identify their gradients' slots
        # the embedding LayerNorm (position table, no tail, no dropout): its backward can ride
        # in the consuming attention block's input-gradient GEMM (sca_gemm_lnb, tab mode)
        ctx.lnsaved = None
        if (pos_table and not has_post and not act and drop_p == 0 and ln_width_ok(N) and _FUSE_LNB and _EMB_LNB and
                not _LIBRARY_MODE):
            ctx.lnsaved = [LnSaved(x[g], means[g], rstds[g], gam[g], tab=tab[g], T=T) for g in range(G)]
            for y, o in zip(ys, ctx.lnsaved):
                y._sca_ln = o
        ctx.save_for_backward(*x, *(tab if pos_table else []), *gam, *means, *rstds, *(ys if act else []))
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        G, pos, act = ctx.G, ctx.pos, ctx.act
        sv = list(ctx.saved_tensors)
        x = sv[:G]
        o = G
        tab = sv[o:o + G] if pos else [None] * G
        o += G if pos else 0
        gam, means, rstds = sv[o:o + G], sv[o + G:o + 2 * G], sv[o + 2 * G:o + 3 * G]
        ys = sv[o + 3 * G:o + 4 * G] if act else [None] * G
        dys = _contig(_zeros_for_none(dys, x))
        if ctx.drop_p > 0:  # gradient of the pre-dropout LayerNorm output
            dd = [torch.empty_like(t) for t in dys]
            dropout_apply([(dys[g], dd[g], ctx.seeds[g]) for g in range(G)], ctx.drop_p)
            dys = dd
        N = x[0].shape[-1]
        rows = x[0].numel() // N
        hs = _take_handoff(ctx.lnsaved, dys)  # the consumer's sca_gemm_lnb ran this backward
        ctx.lnsaved = None
        dpost = [torch.empty_like(t) for t in x] if ctx.has_post else [None] * G
        dg = [param_grad_empty(t) for t in gam]
        db = [param_grad_empty(t) for t in ctx.bet]
        params = list(gam) + list(ctx.bet)
        # deferred when the partial rows are few (config 2 / 3: +0.5-0.7 %); config 5's 1024 x 512
        # partials per problem reduce better beside the weight gradients where they fall (-0.4 %
        # deferred; profiles/r05_misc/affine_defer2_ab.txt)
        defer = (not _settle_reuse(params) and _affine_deferrable(params, (getattr(ctx, "needs_input_grad", None) or (True,))[-2 * G:]) and
                 L.lib().sca_layernorm_bwd_blocks(rows) * N <= _AFFINE_DEFER_MAX)
        if defer:
            _mark_unsettled(params)
        if hs is not None:  # dL/dv (= dL/dx) done; the dgamma / dbeta partials summed below
            dx, part, nblk = [h[2] for h in hs], [h[3] for h in hs], hs[0][4]
        else:
            nblk = L.lib().sca_layernorm_bwd_blocks(rows)
            dx = [torch.empty_like(t) for t in x]
            part = [x[0].new_empty(2 * nblk * N) for _ in range(G)]
            for c in range(0, G, L.LN_MAX_PROBLEMS):
                gs = range(c, min(G, c + L.LN_MAX_PROBLEMS))
                arr = (L.LnBwdProblem * len(gs))(*[L.LnBwdProblem(dys[g].data_ptr(), x[g].data_ptr(), ptr(tab[g]),
                                                                    gam[g].data_ptr(), means[g].data_ptr(),
                                                                    rstds[g].data_ptr(), ptr(ys[g]), act,
                                                                    ptr(dpost[g]), dx[g].data_ptr(),
                                                                    None if defer else dg[g].data_ptr(),
                                                                    None if defer else db[g].data_ptr(),
                                                                    part[g].data_ptr()) for g in gs])
                L.check(L.lib().sca_layernorm_bwd(len(gs), arr, rows, N, ctx.r_mod, ctx.r_off, 0,
                                                  L.stream_handle()), "sca_layernorm_bwd")
        if hs is not None or defer:
            _affine_finish(part, dg, db, nblk, N, params, defer)
        else:
            params_produced(params)
        dtab = []
        if pos:
            B, T = x[0].shape[0], x[0].shape[1]
            if _GRAD_SINK is None:  # one sca_zero launch for the G tables (rows no frame reads stay 0)
                flat = torch.empty((G,) + tuple(tab[0].shape), device=tab[0].device)
                L.check(L.lib().sca_zero(flat.data_ptr(), flat.numel(), L.stream_handle()), "sca_zero")
                dtab = list(flat.unbind(0))
            else:
                dtab = [param_grad_zeros(t) for t in tab]
            # d table[t + 2] = sum_b dv[b, t]
            reduce_rows([(dx[g], dtab[g][2:], 1.0) for g in range(G)], B, T, N, T * N, N)
            params_produced(tab)
        return (None,) * 6 + tuple(dx) + tuple(dtab) + (tuple(dpost) if ctx.has_post else ()) + \
            tuple(dg) + tuple(db)


class MaxPoolT(Function):
    """MaxPool1d(2, 2) over the frame axis of (B, T, C) (model/residual.py:40-43)."""

    @staticmethod
    def forward(ctx, G, *xs):
        xs = _contig(xs)
        L.require_device(*xs)
        B, T, C = xs[0].shape
        ys = [x.new_empty(B, T // 2, C) for x in xs]
        for c in range(0, G, L.POOL_MAX_PROBLEMS):
            gs = range(c, min(G, c + L.POOL_MAX_PROBLEMS))
            arr = (L.PoolProblem * len(gs))(*[L.PoolProblem(xs[g].data_ptr(), ys[g].data_ptr(), None, None)
                                               for g in gs])
            L.check(L.lib().sca_maxpool_t_fwd(len(gs), arr, B, T, C, L.stream_handle()), "sca_maxpool_t_fwd")
        ctx.G = G
        ctx.save_for_backward(*xs)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        G = ctx.G
        xs = ctx.saved_tensors
        B, T, C = xs[0].shape
        dys = _contig(_zeros_for_none(dys, [x.new_empty(B, T // 2, C) for x in xs]))
        dx = [torch.empty_like(x) for x in xs]
        for c in range(0, G, L.POOL_MAX_PROBLEMS):
            gs = range(c, min(G, c + L.POOL_MAX_PROBLEMS))
            arr = (L.PoolProblem * len(gs))(*[L.PoolProblem(xs[g].data_ptr(), None, dys[g].data_ptr(),
                                                             dx[g].data_ptr()) for g in gs])
            L.check(L.lib().sca_maxpool_t_bwd(len(gs), arr, B, T, C, L.stream_handle()), "sca_maxpool_t_bwd")
        return (None,) + tuple(dx)


# --------------------------------------------------------------------------- coordinate mapping
class CoordinateMappingOp(Function):
    """Fused A1 + A2: slice each stream's joints out of the (B, T, K_all, 2) keypoints,
    de-interleave x / y and apply the two Linear(K -> d) maps (layers.py:111-123)."""

    @staticmethod
    def forward(ctx, G, kp, *ts):
        idx = ts[:G]
        Wx, bx, Wy, by = ts[G:2 * G], ts[2 * G:3 * G], ts[3 * G:4 * G], ts[4 * G:5 * G]
        kpc = kp.contiguous()
        L.require_device(kpc)
        B, T, K_all, _ = kpc.shape
        rows = B * T
        N = Wx[0].shape[0]
        xe = [kpc.new_empty(B, T, N) for _ in range(G)]
        ye = [kpc.new_empty(B, T, N) for _ in range(G)]
        for c in range(0, G, L.MAP_MAX_PROBLEMS):
            gs = range(c, min(G, c + L.MAP_MAX_PROBLEMS))
            arr = (L.CoordMapProblem * len(gs))(*[
                L.CoordMapProblem(kpc.data_ptr(), idx[g].data_ptr(), idx[g].numel(), Wx[g].data_ptr(), ptr(bx[g]),
                                  Wy[g].data_ptr(), ptr(by[g]), xe[g].data_ptr(), ye[g].data_ptr()) for g in gs])
            L.check(L.lib().sca_coord_map_fwd(len(gs), arr, rows, K_all, N, L.stream_handle()), "sca_coord_map_fwd")
        ctx.G = G
        ctx.kp_grad = kp.requires_grad
        ctx.bx, ctx.by = tuple(bx), tuple(by)  # parameters (leaves) or None
        ctx.save_for_backward(kpc, *idx, *Wx, *Wy)
        return tuple(xe) + tuple(ye)

    @staticmethod
    def backward(ctx, *grads):
        G = ctx.G
        sv = ctx.saved_tensors
        kp = sv[0]
        idx, Wx, Wy = sv[1:1 + G], sv[1 + G:1 + 2 * G], sv[1 + 2 * G:1 + 3 * G]
        B, T, K_all, _ = kp.shape
        rows = B * T
        N = Wx[0].shape[0]
        refs = [kp.new_empty(B, T, N)] * (2 * G)
        grads = _contig(_zeros_for_none(grads, refs))
        dxe, dye = grads[:G], grads[G:]
        dwx = [param_grad_empty(w) for w in Wx]
        dwy = [param_grad_empty(w) for w in Wy]
        dkp = torch.zeros_like(kp) if ctx.kp_grad else None
        nchunk = L.lib().sca_coord_map_bwd_chunks(rows)
        part = [kp.new_empty(2 * nchunk * N * idx[g].numel()) for g in range(G)]
        for c in range(0, G, L.MAP_MAX_PROBLEMS):
            gs = range(c, min(G, c + L.MAP_MAX_PROBLEMS))
            arr = (L.CoordMapBwdProblem * len(gs))(*[
                L.CoordMapBwdProblem(kp.data_ptr(), idx[g].data_ptr(), idx[g].numel(), Wx[g].data_ptr(),
                                     Wy[g].data_ptr(), dxe[g].data_ptr(), dye[g].data_ptr(), dwx[g].data_ptr(),
                                     dwy[g].data_ptr(), ptr(dkp), part[g].data_ptr()) for g in gs])
            L.check(L.lib().sca_coord_map_bwd(len(gs), arr, rows, K_all, N, L.stream_handle()), "sca_coord_map_bwd")
        params_produced(list(Wx) + list(Wy))
        dbx = [param_grad_empty(b) if b is not None else None for b in ctx.bx]
        dby = [param_grad_empty(b) if b is not None else None for b in ctx.by]
        pairs = [(dxe[g], dbx[g], 1.0) for g in range(G) if dbx[g] is not None] + \
                [(dye[g], dby[g], 1.0) for g in range(G) if dby[g] is not None]
        if pairs:
            reduce_rows(pairs, rows, 1, N, N, 0)
            params_produced(list(ctx.bx) + list(ctx.by))
        return (None, dkp) + (None,) * G + tuple(dwx) + tuple(dbx) + tuple(dwy) + tuple(dby)


# --------------------------------------------------------------------------- Linear + GELU (+ residual)
def gelu_bwd(dys, zs):
    """dz = dy * gelu'(z) for lists of equally sized tensors."""
    outs = [torch.empty_like(z) for z in zs]
    for c in range(0, len(zs), L.GELU_MAX_PROBLEMS):
        gs = range(c, min(len(zs), c + L.GELU_MAX_PROBLEMS))
        arr = (L.GeluBwdProblem * len(gs))(*[L.GeluBwdProblem(dys[g].data_ptr(), zs[g].data_ptr(),
                                                              outs[g].data_ptr()) for g in gs])
        L.check(L.lib().sca_gelu_bwd(len(gs), arr, zs[0].numel(), L.stream_handle()), "sca_gelu_bwd")
    return outs


class LinearGelu(Function):
    """y = GELU_erf(x W^T + b) (+ r) — the Linear+GELU pairs of model/fusion.py:43-50 and
    InvertedResidual (:71-77).  The GEMM epilogue applies bias + GELU (and the residual) and
    keeps the pre-activation for the backward."""

    @staticmethod
    def forward(ctx, G, has_r, *ts):
        x = _contig(ts[:G])
        W, b = ts[G:2 * G], ts[2 * G:3 * G]
        r = _contig(ts[3 * G:4 * G]) if has_r else [None] * G
        L.require_device(*x)
        probs, ys, zs = [], [], []
        for g in range(G):
            n_out, n_in = W[g].shape
            M = x[g].numel() // n_in
            y = x[g].new_empty(*x[g].shape[:-1], n_out)
            z = x[g].new_empty(M, n_out)
            probs.append(_prob([_seg(_flat(x[g]), W[g], n_in, n_in, n_in)], y, M, n_out, n_out, bias=b[g],
                               resid=r[g], ldr=n_out, epi=L.EPI_GELU, aux_out=z, ldo=n_out))
            ys.append(y)
            zs.append(z)
        gemm(L.GEMM_NT, probs)
        ctx.G, ctx.has_r, ctx.b = G, has_r, tuple(b)  # biases: parameters (leaves) or None
        ctx.save_for_backward(*x, *W, *zs)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        G = ctx.G
        sv = ctx.saved_tensors
        x, W, zs = sv[:G], sv[G:2 * G], sv[2 * G:3 * G]
        dys = _contig(_zeros_for_none(dys, [x[g].new_empty(*x[g].shape[:-1], W[g].shape[0]) for g in range(G)]))
        dz = gelu_bwd([_flat(d) for d in dys], zs)
        probs, dxs = [], []
        for g in range(G):
            n_out, n_in = W[g].shape
            M = x[g].numel() // n_in
            dx = torch.empty_like(x[g])
            probs.append(_prob([_seg(dz[g], W[g], n_out, n_in, n_out)], dx, M, n_in, n_in))
            dxs.append(dx)
        ready = wgrad_ready()
        gemm(L.GEMM_NN, probs)
        wg = weight_grads([(dz[g], _flat(x[g]), 1.0, W[g], ctx.b[g]) for g in range(G)], ready=ready)
        return (None, None) + tuple(dxs) + tuple(w for w, _ in wg) + tuple(bb for _, bb in wg) + \
            (tuple(dys) if ctx.has_r else ())


# --------------------------------------------------------------------------- per-clip matmuls
def _clip_views(t):
    return [t[i] for i in range(t.shape[0])]


class ClipMatmul(Function):
    """C[b] = A[b] B[b]^T (trans_b) or A[b] B[b], one grouped GEMM problem per clip
    (CoordinatesFusion's r l^T and attn . body, model/fusion.py:52-55)."""

    @staticmethod
    def forward(ctx, trans_b, A, Bm):
        A, Bm = A.contiguous(), Bm.contiguous()
        L.require_device(A, Bm)
        nb, m, k = A.shape
        n = Bm.shape[1] if trans_b else Bm.shape[2]
        C = A.new_empty(nb, m, n)
        Av, Bv, Cv = _clip_views(A), _clip_views(Bm), _clip_views(C)
        if trans_b:
            probs = [_prob([_seg(Av[i], Bv[i], k, k, k)], Cv[i], m, n, n) for i in range(nb)]
            gemm(L.GEMM_NT, probs)
        else:
            probs = [_prob([_seg(Av[i], Bv[i], k, n, k)], Cv[i], m, n, n) for i in range(nb)]
            gemm(L.GEMM_NN, probs)
        ctx.trans_b = trans_b
        ctx.save_for_backward(A, Bm)
        return C

    @staticmethod
    def backward(ctx, dC):
        A, Bm = ctx.saved_tensors
        dC = dC.contiguous()
        nb, m, k = A.shape
        n = dC.shape[2]
        dA, dB = torch.empty_like(A), torch.empty_like(Bm)
        Av, Bv, dCv, dAv, dBv = (_clip_views(t) for t in (A, Bm, dC, dA, dB))
        if ctx.trans_b:  # C = A B^T:  dA = dC B (NN),  dB = dC^T A (TN)
            gemm(L.GEMM_NN, [_prob([_seg(dCv[i], Bv[i], n, k, n)], dAv[i], m, k, k) for i in range(nb)])
            gemm(L.GEMM_TN, [_prob([_seg(dCv[i], Av[i], n, k, m)], dBv[i], n, k, k) for i in range(nb)])
        else:  # C = A B:  dA = dC B^T (NT),  dB = A^T dC (TN)
            gemm(L.GEMM_NT, [_prob([_seg(dCv[i], Bv[i], n, n, n)], dAv[i], m, k, k) for i in range(nb)])
            gemm(L.GEMM_TN, [_prob([_seg(Av[i], dCv[i], k, n, m)], dBv[i], k, n, n) for i in range(nb)])
        return None, dA, dB


class SoftmaxRows(Function):
    """softmax over the last dim (model/fusion.py:53: no scale, no mask)."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        L.require_device(x)
        N = x.shape[-1]
        y = torch.empty_like(x)
        arr = (L.SoftmaxProblem * 1)(L.SoftmaxProblem(x.data_ptr(), None, None, y.data_ptr()))
        L.check(L.lib().sca_softmax_rows_fwd(1, arr, x.numel() // N, N, L.stream_handle()), "sca_softmax_rows_fwd")
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        N = y.shape[-1]
        dx = torch.empty_like(y)
        arr = (L.SoftmaxProblem * 1)(L.SoftmaxProblem(None, y.data_ptr(), dy.data_ptr(), dx.data_ptr()))
        L.check(L.lib().sca_softmax_rows_bwd(1, arr, y.numel() // N, N, L.stream_handle()), "sca_softmax_rows_bwd")
        return dx
