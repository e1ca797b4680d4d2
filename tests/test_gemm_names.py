"""The profiler's kernel attribution for GEMM launches (ops._gemm_kernel_name) follows the
launcher's eligibility rules in gemm.hip (launch_tile: vec_ok, glds_ok, tn_ok) — bench.py books
time and FLOPs to these names.  CPU only (problem structs with stand-in addresses)."""
import os

from scattennet_amd import _lib as L, ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _prob(M, N, K, lda, ldb, A=0x1000, B=0x2000, nseg=1, alpha2=1.0):
    segs = [L.GemmSeg(A, B, lda, ldb, K, 1.0)] + [L.GemmSeg(A, B, lda, ldb, K, alpha2)] * (nseg - 1)
    segs += [L.GemmSeg(None, None, 0, 0, 0, 0.0)] * (3 - nseg)
    p = L.GemmProblem()
    p.seg = (L.GemmSeg * 3)(*segs)
    p.nseg, p.M, p.N, p.C, p.ldc = nseg, M, N, 0x3000, N
    return p


def test_tn_ksplit_tile_when_eligible():
    assert ops._gemm_kernel_name(L.GEMM_TN, [_prob(256, 256, 2048, 256, 256)], 36) == "gemm_tnk_kernel<3, 1, false>"
    assert ops._gemm_kernel_name(L.GEMM_TN, [_prob(256, 256, 2048, 256, 256)], 37) == "gemm_tnk_kernel<4, 1, false>"


def test_tn_ksplit_falls_back_like_the_launcher():
    # K not a multiple of 32: no LDS-DMA kernel -> the single-buffered register-staged TN kernel
    assert ops._gemm_kernel_name(L.GEMM_TN, [_prob(64, 64, 200, 64, 64)], 36) == "gemm_kernel<2, T5>"
    # two segments: not the k-split kernel, the 2-stage LDS-DMA one
    assert ops._gemm_kernel_name(L.GEMM_TN, [_prob(64, 64, 256, 64, 64, nseg=2)], 36) == "gemm_glds_kernel<2, 2>"
    # misaligned operand: the element-wise register-staged kernel
    assert ops._gemm_kernel_name(L.GEMM_TN, [_prob(64, 64, 256, 64, 64, A=0x1004)], 36) == "gemm_kernel<2, T1, false>"


def test_heuristic_names(monkeypatch):
    # the register-staged 64x64 form by default (K % 64 == 0), 128x128 for 2048+ tiles and K >= 512
    assert ops._gemm_kernel_name(L.GEMM_NT, [_prob(2048, 256, 256, 256, 256)], 0) == \
        "gemm_ntb_kernel<true, 6, false, true, 64>"
    assert ops._gemm_kernel_name(L.GEMM_NN, [_prob(2048, 256, 768, 768, 256)], 0) == \
        "gemm_ntb_kernel<true, 6, true, true, 64>"
    assert ops._gemm_kernel_name(L.GEMM_NT, [_prob(8192, 512, 512, 512, 512)] * 4, 0) == \
        "gemm_ntb_kernel<true, 6, false, true, 128>"
    # K % 64 != 0: the LDS-DMA kernels
    assert ops._gemm_kernel_name(L.GEMM_NT, [_prob(2048, 256, 96, 96, 96)], 0) == "gemm_glds_kernel<0, 3>"
    assert ops._gemm_kernel_name(L.GEMM_NT, [_prob(64, 30, 30, 30, 30)], 0) == "gemm_kernel<0, T1, false>"


def test_names_follow_the_library_switches_and_override():
    """The names come from the library (sca_gemm_kernel_name): its SCA_NTB switch as read once
    at start-up (a fresh process here) and the process-wide tile override."""
    import os
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from tests.test_gemm_names import _prob; "
            "from scattennet_amd import _lib as L, ops; "
            "print(ops._gemm_kernel_name(L.GEMM_NT, [_prob(2048, 256, 256, 256, 256)], 0)); "
            "print(ops._gemm_kernel_name(L.GEMM_NN, [_prob(2048, 256, 768, 768, 256)], 0)); "
            "print(ops._gemm_kernel_name(L.GEMM_NN, [_prob(2046, 256, 768, 768, 256)], 0))") % ROOT
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SCA_NTB="0"), capture_output=True,
                         text=True, check=True).stdout.split("\n")
    assert out[:3] == ["gemm_glds_kernel<0, 3>", "gemm_glds_kernel<1, 2>", "gemm_kernel<1, T7>"], out
    lib = L.lib()
    assert lib.sca_gemm_tile_override(L.GEMM_TN, 37) == 0
    try:
        assert ops._gemm_kernel_name(L.GEMM_TN, [_prob(256, 256, 2048, 256, 256)], 0) == "gemm_tnk_kernel<4, 1, false>"
    finally:
        lib.sca_gemm_tile_override(L.GEMM_TN, 0)
