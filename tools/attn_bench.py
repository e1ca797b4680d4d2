"""Attention microbenchmark through the C ABI at the workload's shapes (graph-captured).

    python tools/attn_bench.py [--lib path.so] [--T 256] [--hd 16] [--G 4] [--iters 50]

Times sca_attn_fwd and sca_attn_bwd (non-causal and causal) and checks both against a
torch fp32 reference of the same math (masked softmax(q k^T) v and its autograd).
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from scattennet_amd import _lib as L  # noqa: E402


def reference(q, k, v, kvalid, H, causal):
    B, T, d = q.shape
    Tk = k.shape[1]
    hd = d // H
    qh = q.view(B, T, H, hd).transpose(1, 2)
    kh = k.view(B, Tk, H, hd).transpose(1, 2)
    vh = v.view(B, Tk, H, hd).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2)
    add = torch.where(kvalid[:, None, None, :] > 0, 0.0, torch.finfo(torch.float32).min)
    if causal:
        tri = torch.ones(T, T, device=q.device, dtype=torch.bool).tril()
        s = s.masked_fill(~tri, float("-inf")) + (add + tri.float())  # model/utils.py:15-28
    else:
        s = s + add
    p = torch.softmax(s, -1)
    return (p @ vh).transpose(1, 2).reshape(B, T, d)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--hd", type=int, default=16)
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--G", type=int, default=4)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--Tk", type=int, default=0, help="non-causal only: key length (default T)")
    ap.add_argument("--causal", default="0,1")
    ap.add_argument("--split", action="store_true", help="hd 32: the split dq / dkdv kernels (no workspace)")
    a = ap.parse_args()
    lib = ctypes.CDLL(a.lib) if a.lib else L.lib()
    if a.lib:
        for name, (argt, rest) in L.EXPORTS.items():
            fn = getattr(lib, name)
            fn.argtypes, fn.restype = argt, rest
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, T, H, hd, G = a.B, a.T, a.H, a.hd, a.G
    d = H * hd
    Tk = a.Tk or T
    mk = lambda n: [torch.randn(B, n, d, device=dev) for _ in range(G)]  # noqa: E731
    q, k, v, do = mk(T), mk(Tk), mk(Tk), mk(T)
    q = [t * hd ** -0.5 for t in q]
    kvalid = torch.ones(B, Tk, device=dev)
    kvalid[1, Tk // 2:] = 0
    kvalid[2, 1:] = 0
    kvalid[3, :] = 0
    o = [torch.empty_like(t) for t in q]
    sm = [torch.empty(B * H * T, device=dev) for _ in range(G)]
    sl = [torch.empty(B * H * T, device=dev) for _ in range(G)]
    dq = [torch.empty_like(t) for t in q]
    dk = [torch.empty_like(t) for t in k]
    dv = [torch.empty_like(t) for t in k]
    delta = [torch.empty(B * H * T, device=dev) for _ in range(G)]
    nws = lib.sca_attn_bwd_workspace(B, H, T, Tk, hd) if not a.split else 0  # fused hd-32 key-block path
    part = [torch.empty(nws, device=dev) if nws > 0 else None for _ in range(G)]
    P = lambda t: t.data_ptr()  # noqa: E731
    fwd = (L.AttnFwdProblem * G)(*[L.AttnFwdProblem(P(q[g]), P(k[g]), P(v[g]), P(o[g]), P(sm[g]), P(sl[g]),
                                                    P(kvalid), None) for g in range(G)])
    bwd = (L.AttnBwdProblem * G)(*[L.AttnBwdProblem(P(q[g]), P(k[g]), P(v[g]), P(o[g]), P(do[g]), P(sm[g]),
                                                    P(sl[g]), P(kvalid), None, P(dq[g]), P(dk[g]), P(dv[g]),
                                                    P(delta[g]), 1.0, 1.0,
                                                    P(part[g]) if part[g] is not None else None) for g in range(G)])

    for causal in [int(c) for c in a.causal.split(",")]:
        if causal and Tk != T:
            continue
        def run_fwd():
            L.check(lib.sca_attn_fwd(G, fwd, B, H, T, Tk, hd, d, d, d, d, causal, causal,
                                     torch.cuda.current_stream().cuda_stream), "fwd")

        def run_bwd():
            L.check(lib.sca_attn_bwd(G, bwd, B, H, T, Tk, hd, d, d, d, d, causal, causal,
                                     torch.cuda.current_stream().cuda_stream), "bwd")

        run_fwd()
        run_bwd()
        torch.cuda.synchronize()
        if not a.no_check:
            errs = []
            for g in range(G):
                qr, kr, vr = (t.detach().clone().requires_grad_(True) for t in (q[g], k[g], v[g]))
                ref = reference(qr, kr, vr, kvalid, H, causal)
                ref.backward(do[g])
                for got, want in ((o[g], ref), (dq[g], qr.grad), (dk[g], kr.grad), (dv[g], vr.grad)):
                    errs.append(float((got - want.detach()).abs().max() / want.abs().max().clamp_min(1e-30)))
            print(f"causal={causal} max rel err {max(errs):.2e}", "OK" if max(errs) < 1e-3 else "FAIL")
        fl_unit = G * 2.0 * B * H * hd * (T * (T + 1) / 2 if causal else T * Tk)
        for name, fn, units in (("fwd", run_fwd, 2), ("bwd", run_bwd, 4)):
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(a.iters):
                        fn()
            torch.cuda.current_stream().wait_stream(s)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            print(f"causal={causal} {name}: {us:8.2f} us  {fl_unit * units / us / 1e6:7.2f} TFLOP/s (algorithmic)")


if __name__ == "__main__":
    main()
