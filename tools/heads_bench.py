"""Time the recognition heads + losses on one MI355X.

Workload: MSCA_Net's head at the 2014T yaml shapes — left/right/body features (B, T/4, 512),
fused features (B, T/4, 1024), vocabulary C, BiLSTM alignment head (1024 -> 2 x 512, 2
layers), two CTC losses (alignment + fuse_coord) and three SeqKD distillation terms
(model/__init__.py:119-236).  As in the reference's training step, the alignment head and its
CTC loss run forward only: `total_loss` sums the fuse_coord CTC loss and the three SeqKD terms
(model/__init__.py:207,236), so backward never reaches the BiLSTM.  Synthetic data; eval mode.
Prints one JSON line with ms per step and the per-part split.

Usage: python tools/heads_bench.py [--B 8] [--T 64] [--C 1124] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=64)
    ap.add_argument("--C", type=int, default=1124)
    ap.add_argument("--S", type=int, default=24)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    from scattennet_amd import heads
    torch.manual_seed(0)
    dev = torch.device("cuda")
    cfg = {"residual_blocks": [256, 256, 512, 512], "out_fusion_dim": 1024,
           "alignment_module": {"input_size": 1024, "hidden_size": 1024, "num_layers": 2, "dropout": 0.3,
                                "bidirectional": True}}
    head = heads.RecognitionHead(cfg, a.C).to(dev).eval()
    B, T = a.B, a.T
    feats = [torch.randn(B, T, 512, device=dev, requires_grad=True) for _ in range(3)]
    fuse = torch.randn(B, T, 1024, device=dev, requires_grad=True)
    labels = torch.randint(1, a.C, (B, a.S))
    tl = torch.randint(a.S // 2, a.S + 1, (B,))
    il = torch.full((B,), T)
    weights = {"left": 0.25, "right": 0.25, "body": 0.25}

    def step(parts=None):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        out = head(feats[0], feats[1], fuse, feats[2])
        ev[1].record()
        # alignment_loss is computed and reported by the reference but not added to total_loss
        heads.compute_loss(labels, tl, out["alignment_gloss_logits"], il)
        loss = heads.compute_loss(labels, tl, out["fuse_coord_gloss_logits"], il)
        for k, w in weights.items():
            loss = loss + heads.distillation_loss(out[k], out["fuse_coord_gloss_logits"], w)
        ev[2].record()
        loss.backward()
        ev[3].record()
        if parts is not None:
            parts.append(ev)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    parts = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(parts)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    fwd = sum(e[0].elapsed_time(e[1]) for e in parts) / a.steps
    loss_ms = sum(e[1].elapsed_time(e[2]) for e in parts) / a.steps
    bwd = sum(e[2].elapsed_time(e[3]) for e in parts) / a.steps
    print(json.dumps({"workload": "recognition heads + CTC x2 + SeqKD x3 fwd; bwd of total_loss (fuse CTC + SeqKD x3)", "B": B, "T": T, "C": a.C,
                      "ms_per_step": round(ms, 3), "head_fwd_ms": round(fwd, 3), "losses_fwd_ms": round(loss_ms, 3),
                      "bwd_ms": round(bwd, 3), "clips_per_s": round(B / ms * 1e3, 1)}))


if __name__ == "__main__":
    main()
