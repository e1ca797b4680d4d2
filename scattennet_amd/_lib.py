"""ctypes binding of libscatten_hip.so (the C ABI declared in include/scatten.h).

The product path has exactly one implementation: the HIP kernels in this library.  If the
library is missing, or a tensor is not on a ROCm device, every op raises — there is no CPU
fallback.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SCA_LIB_PATH") or os.path.join(_HERE, "libscatten_hip.so")  # override: A/B builds

c_int, c_float, c_long, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_long, ctypes.c_void_p
c_u64 = ctypes.c_uint64

GEMM_NT, GEMM_NN, GEMM_TN = 0, 1, 2
EPI_GELU, EPI_DGELU, EPI_ACCUM, EPI_DROPOUT = 1, 2, 4, 8
GEMM_LN_MAX_PROBLEMS = 8
GEMM_MAX_PROBLEMS = 16
ATTN_MAX_PROBLEMS = 8
LN_MAX_PROBLEMS = 8
REDUCE_MAX_PROBLEMS = 64
MAP_MAX_PROBLEMS = 8
POOL_MAX_PROBLEMS = 8
SOFTMAX_MAX_PROBLEMS = 8
GELU_MAX_PROBLEMS = 8
DROPOUT_MAX_PROBLEMS = 12
ACT_NONE, ACT_RELU = 0, 1


class GemmSeg(ctypes.Structure):
    _fields_ = [("A", c_void_p), ("B", c_void_p), ("lda", c_int), ("ldb", c_int), ("K", c_int), ("alpha", c_float)]


class GemmProblem(ctypes.Structure):
    _fields_ = [("seg", GemmSeg * 3), ("nseg", c_int), ("M", c_int), ("N", c_int), ("C", c_void_p), ("ldc", c_int),
                ("epi", c_int), ("bias", c_void_p), ("post_scale", c_float), ("resid", c_void_p), ("ldr", c_int),
                ("aux", c_void_p), ("ldx", c_int), ("aux_out", c_void_p), ("ldo", c_int), ("bias_grad", c_void_p),
                ("bias_grad_scale", c_float), ("drop_seed", c_u64), ("drop_p", c_float)]


class AttnFwdProblem(ctypes.Structure):
    _fields_ = [("q", c_void_p), ("k", c_void_p), ("v", c_void_p), ("o", c_void_p), ("stat_m", c_void_p),
                ("stat_ll", c_void_p), ("key_valid", c_void_p), ("add_mask", c_void_p), ("drop_seed", ctypes.c_uint64),
                ("drop_p", c_float), ("mask_heads", c_int)]


class AttnBwdProblem(ctypes.Structure):
    _fields_ = [("q", c_void_p), ("k", c_void_p), ("v", c_void_p), ("o", c_void_p), ("dout", c_void_p),
                ("stat_m", c_void_p), ("stat_ll", c_void_p), ("key_valid", c_void_p), ("add_mask", c_void_p),
                ("dq", c_void_p), ("dk", c_void_p), ("dv", c_void_p), ("delta", c_void_p), ("dq_scale", c_float),
                ("dv_scale", c_float), ("dq_part", c_void_p), ("drop_seed", ctypes.c_uint64), ("drop_p", c_float),
                ("mask_heads", c_int)]


class LnFwdProblem(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("r", c_void_p), ("gamma", c_void_p), ("beta", c_void_p), ("post", c_void_p),
                ("y", c_void_p), ("mean", c_void_p), ("rstd", c_void_p), ("act", c_int), ("drop_seed", c_u64),
                ("drop_p", c_float)]


class LnBwdProblem(ctypes.Structure):
    _fields_ = [("dy", c_void_p), ("x", c_void_p), ("r", c_void_p), ("gamma", c_void_p), ("mean", c_void_p),
                ("rstd", c_void_p), ("y", c_void_p), ("act", c_int), ("dpost", c_void_p), ("dx", c_void_p),
                ("dgamma", c_void_p), ("dbeta", c_void_p), ("partial", c_void_p)]


class ChainPass(ctypes.Structure):
    _fields_ = [("B", c_void_p), ("ldb", c_int), ("bias", c_void_p), ("post_scale", c_float), ("epi", c_int),
                ("C", c_void_p), ("ldc", c_int), ("aux_out", c_void_p), ("ldo", c_int)]


class GemmLnProblem(ctypes.Structure):
    _fields_ = [("gamma", c_void_p), ("beta", c_void_p), ("y", c_void_p), ("mean", c_void_p), ("rstd", c_void_p),
                ("npass", c_int), ("passes", ChainPass * 3)]


class GemmLnbProblem(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("mean", c_void_p), ("rstd", c_void_p), ("gamma", c_void_p), ("dx", c_void_p),
                ("partial", c_void_p), ("wo", c_void_p), ("dout", c_void_p), ("aux", c_void_p), ("npass", c_int),
                ("ldw", c_int), ("tab", c_void_p), ("tab_T", c_int)]


class PoolProblem(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("y", c_void_p), ("dy", c_void_p), ("dx", c_void_p)]


class SoftmaxProblem(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("y", c_void_p), ("dy", c_void_p), ("out", c_void_p)]


class GeluBwdProblem(ctypes.Structure):
    _fields_ = [("dy", c_void_p), ("z", c_void_p), ("dz", c_void_p)]


class DropoutProblem(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("y", c_void_p), ("seed", c_u64)]


SUM_MAX_TERMS, SUM_MAX_PROBLEMS = 8, 8


class SumProblem(ctypes.Structure):
    _fields_ = [("inp", c_void_p * SUM_MAX_TERMS), ("nin", c_int), ("out", c_void_p)]


class ReduceProblem(ctypes.Structure):
    _fields_ = [("inp", c_void_p), ("out", c_void_p), ("scale", c_float)]


class CoordMapProblem(ctypes.Structure):
    _fields_ = [("kp", c_void_p), ("idx", c_void_p), ("K", c_int), ("wx", c_void_p), ("bx", c_void_p),
                ("wy", c_void_p), ("by", c_void_p), ("xe", c_void_p), ("ye", c_void_p)]


class CoordMapBwdProblem(ctypes.Structure):
    _fields_ = [("kp", c_void_p), ("idx", c_void_p), ("K", c_int), ("wx", c_void_p), ("wy", c_void_p),
                ("dxe", c_void_p), ("dye", c_void_p), ("dwx", c_void_p), ("dwy", c_void_p), ("dkp", c_void_p),
                ("partial", c_void_p)]


EXPORTS = {
    "sca_gemm": ([c_int, c_int, c_void_p, c_int, c_void_p, c_void_p], c_int),
    "sca_gemm_partial": ([c_int, c_int, c_void_p, c_int, c_void_p, c_void_p], c_int),
    "sca_gemm_reduce": ([c_int, c_int, c_void_p, c_int, c_void_p, c_void_p], c_int),
    "sca_gemm_tile_override": ([c_int, c_int], c_int),
    "sca_gemm_splitk_counters": ([c_int, c_int, c_int], c_long),
    "sca_gemm_splitk_fused": ([c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p], c_int),
    "sca_gemm_variant": ([c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p], c_int),
    "sca_gemm_kernel_name": ([c_int, c_int, c_void_p, c_int, c_int, ctypes.c_char_p, c_int], c_int),
    "sca_gemm_ln": ([c_int, c_void_p, c_void_p, c_float, c_void_p], c_int),
    "sca_gemm_ln_rows": ([c_int, c_int, c_int], c_int),
    "sca_gemm_ln_force_rows": ([c_int], c_int),
    "sca_gemm_lnb": ([c_int, c_void_p, c_void_p, c_void_p], c_int),
    "sca_gemm_lnb_blocks": ([c_int], c_int),
    "sca_attn_fwd": ([c_int, c_void_p] + [c_int] * 11 + [c_void_p], c_int),
    "sca_attn_bwd": ([c_int, c_void_p] + [c_int] * 11 + [c_void_p], c_int),
    "sca_attn_bwd_workspace": ([c_int] * 5, ctypes.c_long),
    "sca_attn_bwd_fused": ([c_int], c_int),
    "sca_layernorm_fwd": ([c_int, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p], c_int),
    "sca_layernorm_bwd_blocks": ([c_int], c_int),
    "sca_layernorm_bwd": ([c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p], c_int),
    "sca_maxpool_t_fwd": ([c_int, c_void_p, c_int, c_int, c_int, c_void_p], c_int),
    "sca_maxpool_t_bwd": ([c_int, c_void_p, c_int, c_int, c_int, c_void_p], c_int),
    "sca_softmax_rows_fwd": ([c_int, c_void_p, c_int, c_int, c_void_p], c_int),
    "sca_softmax_rows_bwd": ([c_int, c_void_p, c_int, c_int, c_void_p], c_int),
    "sca_gelu_bwd": ([c_int, c_void_p, c_long, c_void_p], c_int),
    "sca_sum_tensors": ([c_int, c_void_p, c_long, c_void_p], c_int),
    "sca_dropout": ([c_int, c_void_p, c_long, c_int, c_float, c_void_p], c_int),
    "sca_dropout_offset": ([c_void_p], c_int),
    "sca_key_valid": ([c_void_p, c_int, c_void_p, c_long, c_void_p], c_int),
    "sca_zero": ([c_void_p, c_long, c_void_p], c_int),
    "sca_reduce_rows": ([c_int, c_void_p, c_int, c_int, c_int, c_long, c_long, c_int, c_void_p], c_int),
    "sca_coord_map_fwd": ([c_int, c_void_p, c_int, c_int, c_int, c_void_p], c_int),
    "sca_coord_map_bwd_chunks": ([c_int], c_int),
    "sca_coord_map_bwd": ([c_int, c_void_p, c_int, c_int, c_int, c_void_p], c_int),
    "sca_prepare_keypoints": ([c_void_p] * 5 + [c_int] * 3 + [c_void_p, c_void_p, c_int, c_void_p], c_int),
    "sca_normalize_parts": ([c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                             c_void_p], c_int),
    "sca_ctc_workspace_floats": ([c_int, c_int, c_int], c_long),
    "sca_ctc_loss_fwd": ([c_void_p] * 4 + [c_int] * 4 + [c_void_p] * 4, c_int),
    "sca_ctc_loss_bwd": ([c_void_p] * 4 + [c_int] * 4 + [c_void_p] * 4, c_int),
    "sca_seqkd_workspace_floats": ([c_int], c_long),
    "sca_seqkd_fwd": ([c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_void_p,
                       c_void_p, c_void_p], c_int),
    "sca_seqkd_bwd": ([c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_void_p], c_int),
    "sca_clamp": ([c_void_p] * 4 + [c_long, c_float, c_float, c_void_p], c_int),
    "sca_lstm_cell_fwd": ([c_void_p] * 5 + [c_int] * 5 + [c_void_p], c_int),
    "sca_lstm_cell_bwd": ([c_void_p] * 6 + [c_int] * 5 + [c_void_p], c_int),
    "sca_last_error": ([], ctypes.c_char_p),
    "sca_version": ([], c_int),
    "sca_build_digest": ([], ctypes.c_char_p),
}

_lib = None
MISSING = set()  # entry points an alternative build (SCA_LIB_PATH) does not export


def lib():
    """Load the HIP library (once).  Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"scattennet_amd: {LIB_PATH} is missing — run __graft_entry__.build() "
                               "(make -C scattennet_amd/csrc).  There is no fallback path.")
        L = ctypes.CDLL(LIB_PATH)
        alternative = os.environ.get("SCA_LIB_PATH") is not None
        if not alternative:  # the binary must be the build of the sources beside it
            built = L.sca_build_digest
            built.restype = ctypes.c_char_p
            built = built().decode()
            if built != library_digest():
                raise RuntimeError(f"scattennet_amd: {LIB_PATH} was built from other sources (library digest "
                                   f"{built}, sources {library_digest()}) — rebuild it (make -C scattennet_amd/csrc)")
        for name, (argt, rest) in EXPORTS.items():
            if alternative and not hasattr(L, name):  # an older A/B build: entry points it lacks
                MISSING.add(name)
                continue
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = rest
        _lib = L
    return _lib


class HipOpError(RuntimeError):
    pass


def check(rc, what):
    if rc != 0:
        msg = lib().sca_last_error().decode()
        if rc == 1:
            raise ValueError(f"{what}: {msg}")
        raise HipOpError(f"{what} failed ({rc}): {msg}")


def stream_handle():
    return c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return None if t is None else c_void_p(t.data_ptr())


def require_device(*tensors):
    for t in tensors:
        if t is not None and (not t.is_cuda or t.dtype != torch.float32):
            raise RuntimeError("scattennet_amd ops run only on ROCm (MI355X) fp32 tensors; got "
                               f"{t.device} {t.dtype}.  There is no CPU fallback.")


def library_digest():
    """sha256 (first 16 hex digits) of the HIP library's sources: csrc/*.cpp, *.h, *.hip in
    name order, then include/scatten.h — the same bytes the Makefile hashes into the binary
    (sca_build_digest)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(_HERE, "csrc", "*.hip")) + glob.glob(os.path.join(_HERE, "csrc", "*.h")) +
                   glob.glob(os.path.join(_HERE, "csrc", "*.cpp")), key=os.path.basename)
    for f in files + [os.path.join(os.path.dirname(_HERE), "include", "scatten.h")]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_digest():
    """The digest the loaded library was built with."""
    return lib().sca_build_digest().decode()


def source_digest():
    """sha256 (first 16 hex digits) of everything that decides which kernels a bench step
    runs and how: the HIP library's sources (csrc/*.hip, *.h, *.cpp, include/scatten.h), the
    Python dispatch that picks variants, tiles and split-K (scattennet_amd/*.py, bench.py) and
    the SCA_* environment settings in force (bench.py's own
    DEBUG_HIP_* default is part of its source).  Identifies the build a committed
    rocprofv3 profile was measured on (bench.py reports the profile's figures only for a
    matching digest)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    root = os.path.dirname(_HERE)
    files = sorted(glob.glob(os.path.join(_HERE, "csrc", "*.hip")) + glob.glob(os.path.join(_HERE, "csrc", "*.h")) +
                   glob.glob(os.path.join(_HERE, "csrc", "*.cpp")) + [os.path.join(root, "include", "scatten.h")] +
                   glob.glob(os.path.join(_HERE, "*.py")) + [os.path.join(root, "bench.py")])
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    env = sorted((k, v) for k, v in os.environ.items() if k.startswith("SCA_") and k != "SCA_LIB_PATH")
    h.update(repr(env).encode())
    return h.hexdigest()[:16]
