"""Diagnostic: gradients with deferred weight-gradient launches (SCA_WGRAD_DEFER) against the
default path, one small SCA stream; lists the parameters that differ and the pending-queue
bookkeeping.

    python tools/defer_debug.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scattennet_amd import ops, workloads as W  # noqa: E402


def grads(model, kp, mask, gout):
    for p in model.parameters():
        p.grad = None
    outs = model(kp, mask)
    torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])
    torch.cuda.synchronize()
    return {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}


def main():
    dev = torch.device("cuda:0")
    w = dict(W.WORKLOADS["cfg2"], B=2, T=64, L=2, groups=[6, 21])
    model = W.build_streams(w, dev, seed=3, init="random")
    kp, mask, gout = W.synthetic_batch(w, dev, seed=5, ragged=True)
    ref = grads(model, kp, mask, gout)
    ops._WGRAD_DEFER = True
    log = []
    orig_flush = ops.flush_weight_grads

    def flush(after_stream=None):
        log.append(("flush", after_stream, len(ops._PENDING_WGRAD)))
        return orig_flush(after_stream)
    ops.flush_weight_grads = flush
    got = grads(model, kp, mask, gout)
    ops.flush_weight_grads = orig_flush
    print("pending left:", len(ops._PENDING_WGRAD), "flush calls:", len(log), "with work:",
          sum(1 for _, _, n in log if n))
    for k in ref:
        d = float((ref[k] - got[k]).abs().max()) if k in got else float("nan")
        if not d <= 1e-6 * float(ref[k].abs().max()):
            print(f"DIFF {k}: max|d| {d:.3e} ref scale {float(ref[k].abs().max()):.3e} "
                  f"got zero: {bool((got[k] == 0).all()) if k in got else 'missing'}")
    print("done")


if __name__ == "__main__":
    main()
