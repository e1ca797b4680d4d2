"""Generate golden vectors for the recognition-head losses from the REFERENCE implementation.

Runs ONLY in the build container, where `/root/reference` (tinh2044/SCAttenNet, snapshot
2025-07-18) is importable; the outputs (data only: inputs, losses, gradients) are committed
as `heads_*.npz`.  Calls the reference's own code:
  * `MSCA_Net.compute_loss` (model/__init__.py:241-290), unbound, on a stand-in `self` that
    holds the same `nn.CTCLoss(reduction='none', zero_infinity=True, blank=0)` the
    constructor builds (:100-102) — the method reads nothing else from `self`;
  * `SeqKD` (loss.py:5-21), then `weight * ...` and `clamp(-100, 100)` as
    model/__init__.py:203-214 does.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_heads.py
"""
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)

from loss import SeqKD  # noqa: E402
from model import MSCA_Net  # noqa: E402
from model.alignment_module import AlignmentModule  # noqa: E402


def ctc_case(name, logits, labels, in_len, tgt_len, manifest):
    stand_in = types.SimpleNamespace(loss_fn=torch.nn.CTCLoss(reduction="none", zero_infinity=True, blank=0))
    x = torch.tensor(logits, dtype=torch.float32, requires_grad=True)
    loss = MSCA_Net.compute_loss(stand_in, labels=torch.tensor(labels, dtype=torch.long),
                                 tgt_lengths=torch.tensor(tgt_len, dtype=torch.long), logits=x,
                                 input_lengths=torch.tensor(in_len, dtype=torch.long))
    if loss.grad_fn is not None:
        loss.backward()
        g = x.grad.numpy()
    else:
        g = np.zeros_like(logits)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), logits=logits.astype(np.float32),
                        labels=np.asarray(labels, np.int32), in_len=np.asarray(in_len, np.int32),
                        tgt_len=np.asarray(tgt_len, np.int32), loss=np.float32(loss.item()), dlogits=g)
    manifest[name] = {"op": "MSCA_Net.compute_loss", "ref": "model/__init__.py:241-290",
                      "shape": list(logits.shape), "loss": float(loss.item())}


def kd_case(name, student, teacher, weight, temp, use_blank, detach, manifest):
    s = torch.tensor(student, requires_grad=True)
    q = torch.tensor(teacher, requires_grad=not detach)
    kd = SeqKD(T=temp)
    loss = weight * kd(s, q.detach() if detach else q, use_blank=use_blank)
    loss = torch.clamp(loss, min=-100, max=100)
    loss.backward()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), student=student, teacher=teacher,
                        weight=np.float32(weight), temp=np.float32(temp), use_blank=np.int32(use_blank),
                        detach=np.int32(detach), loss=np.float32(loss.item()), dstudent=s.grad.numpy(),
                        dteacher=(np.zeros_like(teacher) if detach else q.grad.numpy()))
    manifest[name] = {"op": "SeqKD * weight, clamp(-100, 100)", "ref": "loss.py:5-21, model/__init__.py:203-214",
                      "shape": list(student.shape), "loss": float(loss.item())}


def align_case(name, B, T, In, Hd, cls, layers, manifest):
    """AlignmentModule (model/alignment_module.py) in eval mode: sequence-first input, loss
    (out * G).sum() with G ~ N(0, 1) seeded at 1; gradients w.r.t. input and every parameter."""
    torch.manual_seed(3)
    m = AlignmentModule(cls_num=cls, input_size=In, hidden_size=Hd, num_layers=layers, dropout=0.3,
                        bidirectional=True).eval()
    x = torch.randn(T, B, In, requires_grad=True)
    out = m(x)
    g = torch.randn(out.shape, generator=torch.Generator().manual_seed(1))
    (out * g).sum().backward()
    arrs = {"x": x.detach().numpy(), "out": out.detach().numpy(), "G": g.numpy(), "dx": x.grad.numpy()}
    for k, p in m.named_parameters():
        arrs["param." + k] = p.detach().numpy()
        arrs["grad." + k] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
    manifest[name] = {"op": "AlignmentModule (eval)", "ref": "model/alignment_module.py:5-69",
                      "B": B, "T": T, "input_size": In, "hidden_size": Hd, "cls_num": cls, "num_layers": layers}


def plant(logits, labels, in_len, tgt_len, boost):
    """Raise the logits along one valid alignment so that the losses stay below the clamp."""
    for b in range(logits.shape[0]):
        Sb = max(tgt_len[b], 1)
        Tb = max(in_len[b], 1, Sb)
        for t in range(Tb):
            logits[b, t, labels[b][min(t * Sb // Tb, Sb - 1)]] += boost
            logits[b, t, 0] += boost / 2
    return logits


def main():
    rng = np.random.default_rng(7)
    manifest = {"torch": torch.__version__, "reference": "tinh2044/SCAttenNet @ 2025-07-18", "fixtures": {}}
    fx = manifest["fixtures"]

    # ragged lengths, repeated labels, an impossible alignment (zero_infinity), target length 0
    # (clamped to 1), input length 0 (clamped to 1, then to the target length), saturated rows
    B, T, C, S = 6, 24, 40, 7
    logits = (rng.standard_normal((B, T, C)) * 3).astype(np.float32)
    logits[0, 3, :] = -50.0
    logits[0, 3, 5] = 50.0  # log-probs below -100 (clamped, no gradient)
    logits[2, :, 0] = 50.0  # head-clamped blank-heavy clip
    labels = rng.integers(1, C, size=(B, S))
    labels[1, :4] = [9, 9, 3, 9]
    labels[3, :3] = [7, 7, 7]
    in_len = [24, 20, 5, 3, 0, 17]
    tgt_len = [7, 4, 3, 3, 2, 0]
    logits[1:] = plant(logits[1:], labels[1:], in_len[1:], tgt_len[1:], 5.0)
    ctc_case("heads_ctc_ragged", logits, labels, in_len, tgt_len, fx)

    # loss above 100: the final clamp gates every gradient to zero
    B, T, C, S = 3, 16, 12, 5
    logits = np.full((B, T, C), -50.0, np.float32)
    logits[:, :, 0] = 50.0
    labels = rng.integers(1, C, size=(B, S))
    ctc_case("heads_ctc_gated", logits, labels, [16, 16, 12], [5, 4, 5], fx)

    # Phoenix-like head: T/4 = 64 frames, vocabulary 300, glosses up to 20
    B, T, C, S = 4, 64, 300, 20
    logits = (rng.standard_normal((B, T, C)) * 2).astype(np.float32)
    labels = rng.integers(1, C, size=(B, S))
    in_len, tgt_len = [64, 50, 33, 64], [20, 11, 16, 1]
    ctc_case("heads_ctc_vocab", plant(logits, labels, in_len, tgt_len, 9.0), labels, in_len, tgt_len, fx)

    # SeqKD as MSCA_Net uses it (teacher detached, use_blank=False, T=1, weight 0.5), plus
    # use_blank=True at temperature 2 with a live teacher (pins the teacher gradient)
    st = (rng.standard_normal((3, 20, 33)) * 3).astype(np.float32)
    te = (rng.standard_normal((3, 20, 33)) * 3).astype(np.float32)
    kd_case("heads_kd_distill", st, te, 0.5, 1.0, False, True, fx)
    kd_case("heads_kd_blank_t2", st, te, 1.0, 2.0, True, False, fx)
    kd_case("heads_kd_clamped", st * 40, te, 400.0, 1.0, False, True, fx)

    align_case("heads_align_B3_T12", 3, 12, 64, 64, 20, 2, fx)

    with open(os.path.join(HERE, "manifest_heads.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(fx), "fixtures")


if __name__ == "__main__":
    main()
