"""The C-ABI binding INTEGRATION.md shows a maintainer (§2) is run as written, on the CPU,
against a recording stand-in for the library: its ctypes struct must have the C struct's size
and field offsets (compiled with gcc from include/scatten.h), its argtypes must be the
package's own binding of the same entry points (scattennet_amd/_lib.py, itself checked
against the header by tests/test_capi.py), and the calls it makes must fill every field and
pass every argument.  No GPU call is made."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _snippet():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 2. C ABI level"):]
    m = re.search(r"```python\n(.*?)```", sec, flags=re.S)
    assert m, "no python block in INTEGRATION.md §2"
    return m.group(1)


class _Fn:
    def __init__(self, name, calls):
        self.name, self.calls = name, calls
        self.argtypes, self.restype = None, None

    def __call__(self, *args):
        self.calls.append((self.name, args, self.argtypes))
        return 0


class _FakeLib:
    """Records every call; the entry points it knows are the library's real exports."""

    def __init__(self, path):
        from scattennet_amd import _lib
        self.path, self.calls, self._fns = path, [], {}
        self._exports = set(_lib.EXPORTS)

    def __getattr__(self, name):
        if name.startswith("_") or name not in self._exports:
            raise AttributeError(name)
        if name not in self._fns:
            self._fns[name] = _Fn(name, self.calls)
        return self._fns[name]


class _FakeTensor:
    """Enough of a tensor for the snippet: shape, data_ptr, new_empty / empty_like."""
    _next = [0x1000]

    def __init__(self, *shape):
        self.shape = tuple(shape)
        self._ptr = _FakeTensor._next[0]
        _FakeTensor._next[0] += 0x1000

    def data_ptr(self):
        return self._ptr

    def numel(self):
        n = 1
        for s in self.shape:
            n *= s
        return n

    def new_empty(self, *shape):
        return _FakeTensor(*shape)


def _run_snippet(monkeypatch):
    ns = {}
    monkeypatch.setattr(ctypes, "CDLL", _FakeLib)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a: type("S", (), {"cuda_stream": 77})())
    monkeypatch.setattr(torch, "empty_like", lambda t: _FakeTensor(*t.shape))
    exec(compile(_snippet(), "INTEGRATION.md", "exec"), ns)
    return ns


def test_snippet_struct_matches_the_header(monkeypatch, tmp_path):
    ns = _run_snippet(monkeypatch)
    cls = ns["AttnFwdProblem"]
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "scatten.h"', "int main(void) {",
             'printf("size %zu\\n", sizeof(sca_attn_fwd_problem));']
    lines += [f'printf("{f} %zu\\n", offsetof(sca_attn_fwd_problem, {f}));' for f, _ in cls._fields_]
    lines.append("return 0; }")
    src = tmp_path / "snippet_layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "snippet_layout"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                         text=True).stdout.split("\n") if l)
    assert int(got["size"]) == ctypes.sizeof(cls)
    for f, _ in cls._fields_:
        assert int(got[f]) == getattr(cls, f).offset, f
    # every field of the C struct is declared (the header's struct has no fields beyond these)
    from scattennet_amd import _lib
    assert [f for f, _ in cls._fields_] == [f for f, _ in _lib.AttnFwdProblem._fields_]


def test_snippet_binds_and_calls_like_the_package(monkeypatch):
    from scattennet_amd import _lib
    ns = _run_snippet(monkeypatch)
    lib = ns["lib"]
    for name in ("sca_attn_fwd", "sca_key_valid"):
        fn = getattr(lib, name)
        assert fn.argtypes == _lib.EXPORTS[name][0], name
        assert fn.restype == _lib.EXPORTS[name][1], name
    B, T, H, d = 2, 16, 4, 64
    q, k, v = _FakeTensor(B, T, d), _FakeTensor(B, T, d), _FakeTensor(B, T, d)
    mask = _FakeTensor(B, T)
    ns["attention_core"](q, k, v, mask, H, causal=True)
    names = [c[0] for c in lib.calls]
    assert names == ["sca_key_valid", "sca_attn_fwd"], names
    for name, args, argtypes in lib.calls:
        assert len(args) == len(argtypes), (name, len(args), len(argtypes))
    _, args, _ = lib.calls[1]
    prob = args[1]._obj  # ctypes.byref(p)
    assert prob.drop_p == 0.0 and prob.drop_seed == 0 and prob.mask_heads == 1
    assert prob.key_valid is not None and prob.add_mask is None
    assert args[2:7] == (B, H, T, T, d // H)
    _, kargs, _ = lib.calls[0]
    assert kargs[1] == 2 and kargs[3] == B * T  # SCA_MASK_I64 over every mask element
    assert prob.key_valid == kargs[2]  # the kernel reads the vector sca_key_valid wrote


def test_mask_dtype_codes_match_the_header():
    from scattennet_amd.ops import _MASK_DTYPES
    src = open(os.path.join(ROOT, "include", "scatten.h")).read()
    codes = {n: int(v) for n, v in re.findall(r"#define SCA_MASK_(\w+) (\d+)", src)}
    want = {torch.float32: "F32", torch.float64: "F64", torch.int64: "I64", torch.int32: "I32", torch.bool: "U8",
            torch.uint8: "U8", torch.float16: "F16", torch.bfloat16: "BF16", torch.int8: "I8", torch.int16: "I16"}
    for dt, n in want.items():
        assert _MASK_DTYPES[dt] == codes[n], dt
    assert "SCA_MASK_I64" in _snippet() or "2 = SCA_MASK_I64" in _snippet()
