"""The C-ABI library loads and exports every entry point declared in include/*.h, and the
product path refuses to run anywhere but on the GPU (no silent CPU fallback).  CPU only."""
import ctypes
import glob
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(sca_\w+)\s*\(", src, flags=re.M))
    return sorted(names)


def test_header_declares_entry_points():
    names = _declared()
    assert "sca_gemm" in names and "sca_attn_fwd" in names and "sca_attn_bwd" in names
    assert len(names) >= 12


def test_library_exports_every_declared_symbol():
    from scattennet_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    # every declared symbol is bound with a signature by the Python layer
    assert set(_declared()) - {"sca_set_error"} <= set(_lib.EXPORTS), set(_declared()) - set(_lib.EXPORTS)


_STRUCTS = {  # C struct in include/scatten.h -> ctypes mirror in scattennet_amd/_lib.py
    "sca_gemm_seg": "GemmSeg", "sca_gemm_problem": "GemmProblem", "sca_attn_fwd_problem": "AttnFwdProblem",
    "sca_attn_bwd_problem": "AttnBwdProblem", "sca_ln_fwd_problem": "LnFwdProblem",
    "sca_ln_bwd_problem": "LnBwdProblem", "sca_pool_problem": "PoolProblem", "sca_softmax_problem": "SoftmaxProblem",
    "sca_gelu_bwd_problem": "GeluBwdProblem", "sca_reduce_problem": "ReduceProblem",
    "sca_coord_map_problem": "CoordMapProblem", "sca_coord_map_bwd_problem": "CoordMapBwdProblem",
    "sca_dropout_problem": "DropoutProblem", "sca_gemm_ln_problem": "GemmLnProblem",
    "sca_gemm_lnb_problem": "GemmLnbProblem", "sca_gemm_chain_pass": "ChainPass",
    "sca_sum_problem": "SumProblem",
}


def test_struct_layouts_match_header(tmp_path):
    """Every ctypes mirror has the C struct's size and field offsets (compiled with gcc from
    the header itself)."""
    import shutil
    import subprocess
    from scattennet_amd import _lib as L
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "scatten.h"', "int main(void) {"]
    for cs, py in _STRUCTS.items():
        lines.append(f'printf("{py} size %zu\\n", sizeof({cs}));')
        for f, _ in getattr(L, py)._fields_:
            cf = {"inp": "in", "passes": "pass"}.get(f, f)  # C field names that are Python keywords
            lines.append(f'printf("{py}.{f} %zu\\n", offsetof({cs}, {cf}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = dict(line.rsplit(" ", 1) for line in out if line)
    for cs, py in _STRUCTS.items():
        cls = getattr(L, py)
        assert int(got[f"{py} size"]) == ctypes.sizeof(cls), py
        for f, _ in cls._fields_:
            assert int(got[f"{py}.{f}"]) == getattr(cls, f).offset, (py, f)


def test_cpu_tensors_are_rejected():
    import scattennet_amd as S
    m = S.SelfAttention(32, 2)
    x = torch.randn(1, 8, 32)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(x, S.key_padding_mask(torch.ones(1, 8, dtype=torch.long)))


def test_constructor_errors_match_reference():
    import scattennet_amd as S
    with pytest.raises(ValueError):
        S.SelfAttention(30, 4)
    with pytest.raises(ValueError):
        S.CoordinateAttention({"d_model": 32, "attention_heads": 2, "attention_dropout": 0.0, "dropout": 0.0,
                               "ff_dim": 64}, "bogus")


def test_fusion_state_dict_keys_match_reference():
    import scattennet_amd as S
    from tests.golden_util import load
    fx = load("fusion")
    m = S.CoordinatesFusion(fx["meta"]["in"], fx["meta"]["out"], 0.2)
    assert set(m.state_dict().keys()) == set(fx["param"].keys())


def test_state_dict_keys_match_reference():
    """Key layout of one KeypointModule equals the reference's (golden fixture keys)."""
    import scattennet_amd as S
    from tests.golden_util import load
    fx = load("keypoint_module")
    m = S.KeypointModule(list(range(3, 24)), fx["meta"]["T"], fx["meta"]["cfg"])
    assert set(m.state_dict().keys()) == set(fx["param"].keys())
    m.load_state_dict(fx["param"])  # strict


def test_gemm_variant_ids_are_validated():
    """Only kernel variants that compute the full result can be selected through the C ABI
    (sca_gemm_tile_override / sca_gemm_variant): any other id is SCA_ERR_ARG and changes
    nothing.  Pure argument checks — no GPU call is made."""
    from scattennet_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    ERR, OK = 1, 0
    for layout, bad in [(2, 41), (2, 45), (2, 30), (2, 23), (0, 36), (1, 37), (0, 38), (1, 40), (2, 44), (0, 43), (2, 45), (0, 46), (0, 11), (0, 2), (0, 99), (3, 0), (-1, 0)]:
        assert lib.sca_gemm_tile_override(layout, bad) == ERR, (layout, bad)
        assert lib.sca_gemm_variant(layout, 0, None, 1, None, None, bad, None) == ERR, (layout, bad)
    for layout, good in [(0, 20), (1, 21), (2, 36), (2, 37), (2, 38), (2, 39), (2, 40), (2, 43), (0, 44), (1, 41), (0, 45), (1, 45), (2, 46), (2, 5), (1, 7), (0, 1), (2, 0)]:
        assert lib.sca_gemm_tile_override(layout, good) == OK, (layout, good)
        assert lib.sca_gemm_variant(layout, 0, None, 1, None, None, good, None) == OK, (layout, good)
    for layout in range(3):
        assert lib.sca_gemm_tile_override(layout, 0) == OK


def test_library_digest_matches_sources():
    """The loaded binary is the build of the sources beside it: the Makefile embeds the sha256
    of csrc + include/scatten.h (sca_build_digest) and _lib refuses a mismatch on load."""
    from scattennet_amd import _lib
    _lib.lib()
    assert _lib.build_digest() == _lib.library_digest()


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """A binary built from other sources does not load (no silent stale-kernel runs)."""
    import shutil

    from scattennet_amd import _lib
    fake_src = tmp_path / "scattennet_amd"
    shutil.copytree(os.path.join(ROOT, "scattennet_amd", "csrc"), fake_src / "csrc",
                    ignore=shutil.ignore_patterns("build"))
    os.makedirs(tmp_path / "include")
    shutil.copy(os.path.join(ROOT, "include", "scatten.h"), tmp_path / "include" / "scatten.h")
    with open(fake_src / "csrc" / "common.h", "a") as f:
        f.write("\n// edited after the build\n")
    monkeypatch.setattr(_lib, "_HERE", str(fake_src))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError, match="built from other sources"):
        _lib.lib()
