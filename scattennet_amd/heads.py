"""Recognition heads and losses of MSCA_Net on the HIP path.

* `RecognitionHead` — the four per-stream gloss classifiers of model/__init__.py:10-69
  (`left/right/body_gloss_classifier`, `fuse_coord_classifier`, same state_dict keys), each
  a `sca_gemm` Linear followed by the HIP clamp(+-50) of :54-58, and the BiLSTM
  `fuse_alignment_head` (scattennet_amd/alignment.py) when the cfg has `alignment_module`.
* `compute_loss` — MSCA_Net.compute_loss (model/__init__.py:241-290) as one HIP op chain
  (`sca_ctc_loss_fwd/bwd`): no host syncs — the reference's `.cpu()` of labels / lengths
  and its NaN / inf checks, which each stall the GPU, are gone.  Lengths given as CPU
  tensors (as the reference hands them to nn.CTCLoss) are validated on the host with the
  same RuntimeError torch raises; device tensors are trusted (in-kernel clamps only keep a
  bad call in bounds).
* `SeqKD` (loss.py:5-21) and `distillation_loss` (its use at model/__init__.py:203-214:
  `clamp(weight * SeqKD(...), -100, 100)`, fused) — `sca_seqkd_fwd/bwd`.
"""
import torch
from torch import nn
from torch.autograd import Function

from . import _lib as L
from . import ops
from .alignment import AlignmentModule
from .precision import fp32_compute


def _dev_i32(t, device):
    return torch.as_tensor(t).to(device=device, dtype=torch.int32, non_blocking=True).contiguous()


class ClampLogits(Function):
    """torch.clamp(z, lo, hi) with its gradient gate (model/__init__.py:54-58)."""

    @staticmethod
    def forward(ctx, z, lo, hi):
        z = z.contiguous()
        L.require_device(z)
        y = torch.empty_like(z)
        L.check(L.lib().sca_clamp(L.ptr(z), L.ptr(y), None, None, z.numel(), lo, hi, L.stream_handle()), "sca_clamp")
        ctx.save_for_backward(z)
        ctx.lo, ctx.hi = lo, hi
        return y

    @staticmethod
    def backward(ctx, dy):
        (z,) = ctx.saved_tensors
        dy = dy.contiguous()
        dz = torch.empty_like(z)
        L.check(L.lib().sca_clamp(L.ptr(z), None, L.ptr(dy), L.ptr(dz), z.numel(), ctx.lo, ctx.hi,
                                  L.stream_handle()), "sca_clamp")
        return dz, None, None


def clamp_logits(z, lo=-50.0, hi=50.0):
    return ClampLogits.apply(z, float(lo), float(hi))


class CTCLossOp(Function):
    """loss = MSCA_Net.compute_loss(labels, tgt_lengths, logits, input_lengths) on batch-major
    logits (B, T, C); labels (B, S), lengths (B,) int32 device tensors."""

    @staticmethod
    def forward(ctx, logits, labels, in_len, tgt_len):
        x = logits.contiguous()
        L.require_device(x)
        B, T, C = x.shape
        S = labels.shape[1]
        lib = L.lib()
        ws = x.new_empty(lib.sca_ctc_workspace_floats(B, T, S))
        loss = x.new_empty(())
        nll = x.new_empty(B)
        L.check(lib.sca_ctc_loss_fwd(L.ptr(x), L.ptr(labels), L.ptr(in_len), L.ptr(tgt_len), B, T, C, S, L.ptr(nll),
                                     L.ptr(loss), L.ptr(ws), L.stream_handle()), "sca_ctc_loss_fwd")
        ctx.save_for_backward(x, labels, in_len, tgt_len, ws)
        ctx.mark_non_differentiable(nll)
        return loss, nll

    @staticmethod
    def backward(ctx, dloss, _dnll):
        x, labels, in_len, tgt_len, ws = ctx.saved_tensors
        B, T, C = x.shape
        dloss = dloss.contiguous() if dloss is not None else x.new_zeros(())
        dx = torch.empty_like(x)
        L.check(L.lib().sca_ctc_loss_bwd(L.ptr(x), L.ptr(labels), L.ptr(in_len), L.ptr(tgt_len), B, T, C,
                                         labels.shape[1], L.ptr(dloss), L.ptr(ws), L.ptr(dx), L.stream_handle()),
                "sca_ctc_loss_bwd")
        return dx, None, None, None


def _host_lengths(t):
    """Lengths as a host tensor for validation, or None when that would need a device sync
    under hipGraph capture (the kernels' clamps then keep a bad call in bounds)."""
    t = torch.as_tensor(t)
    if t.device.type == "cpu":
        return t
    if torch.cuda.is_current_stream_capturing():
        return None
    return t.cpu()  # one sync, as the reference's own .cpu() of the lengths (model/__init__.py:265-269)


def _validate_ctc(labels, tgt_lengths, input_lengths, B, T, C):
    """torch.nn.CTCLoss's argument checks (as the reference's call raises them): labels (B, S)
    padded, one input / target length per clip, target lengths <= S, input lengths <= T,
    labels in [0, C)."""
    if labels.dim() != 2 or labels.shape[0] != B:
        raise RuntimeError(f"scattennet_amd compute_loss: labels must be (B, S) padded with B = {B}, "
                           f"got {tuple(labels.shape)}")
    for name, t in (("target_lengths", tgt_lengths), ("input_lengths", input_lengths)):
        if torch.as_tensor(t).numel() != B:
            raise RuntimeError(f"Expected {name} to have {B} entries (one per clip), got {torch.as_tensor(t).numel()}")
    tl, il = _host_lengths(tgt_lengths), _host_lengths(input_lengths)
    if tl is not None:
        S_eff = tl.clamp(min=1)
        if int(S_eff.max()) > labels.shape[1]:
            raise RuntimeError(f"Expected tensor to have size at least {int(S_eff.max())} at dimension 1, "
                               f"but got size {labels.shape[1]} for argument #2 'targets'")
        if il is not None:
            T_eff = torch.maximum(il.clamp(min=1), S_eff)
            if int(T_eff.max()) > T:
                raise RuntimeError(f"Expected input_lengths to have value at most {T}, but got value "
                                   f"{int(T_eff.max())}")
    if labels.device.type == "cpu" and labels.numel():
        lo, hi = int(labels.min()), int(labels.max())
        if lo < 0 or hi >= C:
            raise RuntimeError(f"target values must lie in [0, {C}); got [{lo}, {hi}]")


def _pad_concatenated(labels, tgt_lengths, B):
    """nn.CTCLoss's 1-D form: the targets of all clips concatenated, split by the target
    lengths as the reference passes them (clamped to >= 1, model/__init__.py:263) ->
    (B, max S) padded."""
    tl = _host_lengths(tgt_lengths)
    if tl is None:
        raise RuntimeError("compute_loss: 1-D (concatenated) labels need host-visible target lengths under "
                           "graph capture; pass (B, S) padded labels")
    tl = tl.reshape(-1).clamp(min=1).to(torch.int64)
    if tl.numel() != B:
        raise RuntimeError(f"Expected target_lengths to have {B} entries (one per clip), got {tl.numel()}")
    total = int(tl.sum())
    if labels.numel() < total:
        raise RuntimeError(f"concatenated targets hold {labels.numel()} labels, target_lengths sum to {total}")
    out = labels.new_zeros(B, int(tl.max()))
    o = 0
    for b in range(B):
        n = int(tl[b])
        out[b, :n] = labels[o:o + n]
        o += n
    return out


def compute_loss(labels, tgt_lengths, logits, input_lengths, return_per_sample=False):
    """MSCA_Net.compute_loss (model/__init__.py:241-290): logits (B, T, C) batch-major (the
    reference permutes to (T, B, C) itself).  labels: (B, S) padded, or 1-D concatenated as
    nn.CTCLoss also accepts.  Returns the clamped mean CTC loss (0-dim)."""
    B, T, C = logits.shape
    labels = torch.as_tensor(labels)
    if labels.dim() == 1:
        labels = _pad_concatenated(labels, tgt_lengths, B)
    _validate_ctc(labels, tgt_lengths, input_lengths, B, T, C)
    dev = logits.device
    loss, nll = CTCLossOp.apply(logits, _dev_i32(labels, dev), _dev_i32(input_lengths, dev),
                                _dev_i32(tgt_lengths, dev))
    return (loss, nll) if return_per_sample else loss


class SeqKDOp(Function):
    @staticmethod
    def forward(ctx, student, teacher, start, temp, weight, lo, hi):
        s, q = student.contiguous(), teacher.contiguous()
        L.require_device(s, q)
        if s.shape != q.shape:
            raise RuntimeError(f"SeqKD: student {tuple(s.shape)} and teacher {tuple(q.shape)} shapes differ")
        C = s.shape[-1]
        R = s.numel() // C
        lib = L.lib()
        ws = s.new_empty(lib.sca_seqkd_workspace_floats(R))
        loss = s.new_empty(())
        L.check(lib.sca_seqkd_fwd(L.ptr(s), L.ptr(q), R, C, start, temp, weight, lo, hi, L.ptr(loss), L.ptr(ws),
                                  L.stream_handle()), "sca_seqkd_fwd")
        ctx.save_for_backward(s, q, ws)
        ctx.args = (R, C, start, temp)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        s, q, ws = ctx.saved_tensors
        R, C, start, temp = ctx.args
        need_s, need_q = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        ds = torch.empty_like(s) if need_s else None
        dq = torch.empty_like(q) if need_q else None
        if need_s or need_q:
            L.check(L.lib().sca_seqkd_bwd(L.ptr(s), L.ptr(q), R, C, start, temp, L.ptr(dloss.contiguous()), L.ptr(ws),
                                          L.ptr(ds), L.ptr(dq), L.stream_handle()), "sca_seqkd_bwd")
        return ds, dq, None, None, None, None, None


class SeqKD(nn.Module):
    """loss.py:5-21 — KLDivLoss(batchmean)(log_softmax(pred[..., s:] / T), softmax(ref[..., s:] / T)) * T^2."""

    def __init__(self, T=1):
        super().__init__()
        self.T = T

    @fp32_compute()
    def forward(self, prediction_logits, ref_logits, use_blank=True):
        return SeqKDOp.apply(prediction_logits, ref_logits, 0 if use_blank else 1, float(self.T), 1.0,
                             float("-inf"), float("inf"))


def distillation_loss(student_logits, teacher_logits, weight, T=1.0):
    """model/__init__.py:203-214: clamp(weight * SeqKD(T)(student, teacher.detach(), use_blank=False), -100, 100)."""
    return SeqKDOp.apply(student_logits, teacher_logits.detach(), 1, float(T), float(weight), -100.0, 100.0)


class RecognitionHead(nn.Module):
    """model/__init__.py:10-69 (same state_dict keys); the alignment head is built when
    cfg["alignment_module"] is present, as the reference's yaml configs always have it."""

    def __init__(self, cfg, gloss_tokenizer):
        super().__init__()
        n = len(gloss_tokenizer) if not isinstance(gloss_tokenizer, int) else gloss_tokenizer
        self.left_gloss_classifier = nn.Linear(cfg["residual_blocks"][-1], n)
        self.right_gloss_classifier = nn.Linear(cfg["residual_blocks"][-1], n)
        self.body_gloss_classifier = nn.Linear(cfg["residual_blocks"][-1], n)
        self.fuse_coord_classifier = nn.Linear(cfg["out_fusion_dim"], n)
        self.fuse_alignment_head = (AlignmentModule(**cfg["alignment_module"], cls_num=n)
                                    if "alignment_module" in cfg else None)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.constant_(m.bias, 0)

    @fp32_compute()
    def forward(self, left_output, right_output, fuse_output, body_output):
        heads = [self.left_gloss_classifier, self.right_gloss_classifier, self.body_gloss_classifier]
        zs = list(ops.LinearResidual.apply(3, False, left_output, right_output, body_output,
                                           *[h.weight for h in heads], *[h.bias for h in heads]))
        zs += list(ops.LinearResidual.apply(1, False, fuse_output, self.fuse_coord_classifier.weight,
                                            self.fuse_coord_classifier.bias))
        left, right, body, fuse = [clamp_logits(z) for z in zs]
        out = {"left": left, "right": right, "body": body, "fuse_coord_gloss_logits": fuse}
        if self.fuse_alignment_head is not None:
            out["alignment_gloss_logits"] = clamp_logits(self.fuse_alignment_head(fuse_output.permute(1, 0, 2)))
        return out
