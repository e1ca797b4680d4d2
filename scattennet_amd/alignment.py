"""AlignmentModule (model/alignment_module.py) on the HIP path: a (bi)directional multi-layer
LSTM over the fused features followed by the gloss Linear, batch-major throughout.

Per layer (`LSTMLayer`), D = 2 directions:
  * input projection for all frames and both directions: one grouped NT `sca_gemm`
    (G = X W_ih^T + b_ih, (B, T, D*4H));
  * T recurrent steps, each ONE grouped NT `sca_gemm` for both directions
    (h W_hh^T + b_hh + the step's G row as residual epilogue, M = B) and one
    `sca_lstm_cell_fwd` (gates -> c, h; direction 1 walks the frames backwards);
  * backward: T steps of (grouped NN `sca_gemm` dG_t' W_hh + dY_t, `sca_lstm_cell_bwd`),
    then dX as one NN GEMM with a segment per direction, dW_ih / dW_hh (+ both biases, fused
    column sums) as grouped TN GEMMs over all B*T rows.
The recurrence is latency-bound by construction (2T dependent launches per layer); see
DESIGN.md §5.  Inter-layer dropout (nn.LSTM's `dropout`, training mode only) uses the
counter-based `sca_dropout` mask of the rest of the path.
Parameters live in an `nn.LSTM` so the state_dict keys are the reference's
(`rnn.weight_ih_l0`, `rnn.weight_hh_l0_reverse`, ...).
"""
import torch
from torch import nn
from torch.autograd import Function

from . import _lib as L
from . import ops
from .ops import _prob, _seg, gemm
from .precision import fp32_compute

# split-K of the per-step recurrent GEMMs (M = B rows only): forward K = H, backward K = 4H
# would otherwise run on N/64 workgroups per direction
_SPLITK_FWD = 8
_SPLITK_BWD = 16


def _stepper(template, a_step, r_step):
    """Per-step problem builder: a copy of `template` (the step-0 problem) with the A operand
    and residual pointers advanced by a_step / r_step bytes per step — the recurrent loop
    then costs a struct copy per launch instead of tensor slicing + _prob (host-bound)."""
    a0, r0 = template.seg[0].A, template.resid

    def at(k):
        p = L.GemmProblem.from_buffer_copy(template)
        p.seg[0].A = a0 + k * a_step
        p.resid = r0 + k * r_step
        return p
    return at


class LSTMLayer(Function):
    """One (bi)directional LSTM layer: x (B, T, In) -> y (B, T, D*H)."""

    @staticmethod
    def forward(ctx, D, x, *params):
        x = x.contiguous()
        L.require_device(x)
        B, T, In = x.shape
        w_ih, w_hh, b_ih, b_hh = params[0:D], params[D:2 * D], params[2 * D:3 * D], params[3 * D:4 * D]
        H = w_hh[0].shape[1]
        G = x.new_empty(B, T, D * 4 * H)  # projections, overwritten step by step with the activations
        xf = x.view(B * T, In)
        gemm(L.GEMM_NT, [_prob([_seg(xf, w_ih[d], In, In, In)], G[..., d * 4 * H:], B * T, 4 * H, D * 4 * H,
                               bias=b_ih[d]) for d in range(D)])
        hp = x.new_zeros(B, T, D * H)
        c = x.new_empty(B, T, D * H)
        y = x.new_empty(B, T, D * H)
        gt = x.new_empty(B, D * 4 * H)
        ws = x.new_empty(_SPLITK_FWD * D * (B * 4 * H + B)) if _SPLITK_FWD > 1 else None
        lib, st = L.lib(), L.stream_handle()
        steppers = []
        for d in range(D):
            t0, dt = (0, 1) if d == 0 else (T - 1, -1)
            tpl = _prob([_seg(hp[:, t0, d * H:], w_hh[d], T * D * H, H, H)], gt[:, d * 4 * H:], B, 4 * H, D * 4 * H,
                        bias=b_hh[d], resid=G[:, t0, d * 4 * H:], ldr=T * D * 4 * H)
            steppers.append(_stepper(tpl, 4 * dt * D * H, 4 * dt * D * 4 * H))
        for step in range(T):
            gemm(L.GEMM_NT, [f(step) for f in steppers], splitk=_SPLITK_FWD, ws=ws)
            L.check(lib.sca_lstm_cell_fwd(L.ptr(gt), L.ptr(G), L.ptr(c), L.ptr(y), L.ptr(hp), B, T, H, D, step, st),
                    "sca_lstm_cell_fwd")
        ctx.D = D
        ctx.save_for_backward(x, G, c, hp, *params)
        return y

    @staticmethod
    def backward(ctx, dy):
        D = ctx.D
        x, act, c, hp, *params = ctx.saved_tensors
        w_ih, w_hh, b_ih = params[0:D], params[D:2 * D], params[2 * D:3 * D]
        B, T, In = x.shape
        H = w_hh[0].shape[1]
        dy = dy.contiguous()
        dG = x.new_empty(B, T, D * 4 * H)
        dh = x.new_empty(B, D * H)
        dc = x.new_empty(B, D * H)
        ws = x.new_empty(_SPLITK_BWD * D * (B * H + B)) if _SPLITK_BWD > 1 else None
        lib, st = L.lib(), L.stream_handle()
        steppers = []
        for d in range(D):  # step 1: t = T-2 / 1, reading dG of the frame step 0 processed
            t1, dt = (T - 2, -1) if d == 0 else (1, 1)
            if T < 2:
                break
            tpl = _prob([_seg(dG[:, t1 - dt, d * 4 * H:], w_hh[d], T * D * 4 * H, H, 4 * H)], dh[:, d * H:], B, H,
                        D * H, resid=dy[:, t1, d * H:], ldr=T * D * H)
            steppers.append(_stepper(tpl, 4 * dt * D * 4 * H, 4 * dt * D * H))
        for step in range(T):
            if step > 0:
                gemm(L.GEMM_NN, [f(step - 1) for f in steppers], splitk=_SPLITK_BWD, ws=ws)
            L.check(lib.sca_lstm_cell_bwd(L.ptr(dh) if step > 0 else None, L.ptr(dy), L.ptr(act), L.ptr(c),
                                          L.ptr(dc), L.ptr(dG), B, T, H, D, step, st), "sca_lstm_cell_bwd")
        dGf = dG.view(B * T, D * 4 * H)
        dx = torch.empty_like(x)
        gemm(L.GEMM_NN, [_prob([_seg(dGf[:, d * 4 * H:], w_ih[d], D * 4 * H, In, 4 * H) for d in range(D)],
                               dx.view(B * T, In), B * T, In, In)])
        dw_ih = [torch.empty_like(w) for w in w_ih]
        dw_hh = [torch.empty_like(w) for w in w_hh]
        db_ih = [torch.empty_like(b) for b in b_ih]
        db_hh = [torch.empty_like(b) for b in b_ih]
        xf, hpf = x.view(B * T, In), hp.view(B * T, D * H)
        gemm(L.GEMM_TN, [_prob([_seg(dGf[:, d * 4 * H:], xf, D * 4 * H, In, B * T)], dw_ih[d], 4 * H, In, In,
                               bias_grad=db_ih[d]) for d in range(D)])
        gemm(L.GEMM_TN, [_prob([_seg(dGf[:, d * 4 * H:], hpf[:, d * H:], D * 4 * H, D * H, B * T)], dw_hh[d], 4 * H,
                               H, H, bias_grad=db_hh[d]) for d in range(D)])
        return (None, dx, *dw_ih, *dw_hh, *db_ih, *db_hh)


def lstm(rnn, x):
    """nn.LSTM(batch_first=False) semantics on batch-major x (B, T, In) -> (B, T, D*H)."""
    if rnn.proj_size or not rnn.bias:
        raise NotImplementedError("scattennet_amd LSTM: proj_size / bias=False are not used by the reference")
    D = 2 if rnn.bidirectional else 1
    for layer in range(rnn.num_layers):
        sfx = [f"_l{layer}", f"_l{layer}_reverse"][:D]
        ps = [getattr(rnn, f"{n}{s}") for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh") for s in sfx]
        x = LSTMLayer.apply(D, x, *ps)
        if layer < rnn.num_layers - 1 and rnn.training and rnn.dropout > 0:
            x = ops.dropout_grouped([x], float(rnn.dropout))[0]
    return x


class AlignmentModule(nn.Module):
    """model/alignment_module.py:5-69 — same constructor and state_dict keys; forward takes the
    reference's sequence-first (T, B, input_size) tensor and returns (B, T, cls_num) logits."""

    def __init__(self, cls_num, input_size, hidden_size, num_layers=2, dropout=0.3, bidirectional=True):
        super().__init__()
        self.hidden_size = hidden_size
        self.num_layers = num_layers
        self.input_size = input_size
        self.bidirectional = bidirectional
        self.num_directions = 2 if bidirectional else 1
        self.lstm_hidden_size = int(hidden_size / self.num_directions)
        self.dropout = dropout
        self.rnn = nn.LSTM(input_size=input_size, hidden_size=self.lstm_hidden_size, num_layers=num_layers,
                           dropout=dropout, bidirectional=bidirectional)
        self.gloss_layer = nn.Linear(hidden_size, cls_num)

    @fp32_compute()
    def forward(self, x):
        # the caller's (T, B, C) is the permute(1, 0, 2) view of a batch-major tensor
        # (model/__init__.py:52): permuting back is free
        y = lstm(self.rnn, x.permute(1, 0, 2).contiguous())
        return ops.LinearResidual.apply(1, False, y, self.gloss_layer.weight, self.gloss_layer.bias)[0]
