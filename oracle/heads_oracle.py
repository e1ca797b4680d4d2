"""CPU ORACLE for the recognition-head losses.

TEST INFRASTRUCTURE ONLY: imported by `tests/` as the checker, never by the product path
(`scattennet_amd`), which runs the HIP kernels of `scattennet_amd/csrc/heads.hip`.

A from-scratch numpy restatement (float64 accumulation, explicit loops over frames) of
  * MSCA_Net.compute_loss (model/__init__.py:241-290): log_softmax over classes,
    clamp(-100, 0), `nn.CTCLoss(blank=0, reduction='none', zero_infinity=True)` on
    (T, B, C) log-probs, mean over the finite per-sample losses, clamp(0, 100).
    The CTC op is torch's (third-party; the reference pins no version — fixtures record
    torch 2.10.0): its published algorithm is the log-space alpha recursion of Graves et
    al. 2006 over the blank-extended label sequence l' (blank at even states), the
    likelihood from the last two states, and the gradient w.r.t. the log-probs
    `exp(lp) - exp(lcab + nll - lp)` with lcab = logsumexp of alpha + beta over the states
    carrying the class (zero past the input length and for zero_infinity'd samples);
  * SeqKD (loss.py:5-21) times the distillation weight, clamp(-100, 100)
    (model/__init__.py:203-214).

Parity pin: `tests/test_heads.py` checks this restatement against golden vectors captured
from the reference itself (`tests/golden/heads_*.npz`, made by
`tests/golden/gen_golden_heads.py` with the reference importable in the build container).
"""
import numpy as np


def _log_softmax(x):
    m = x.max(axis=-1, keepdims=True)
    return (x - m) - np.log(np.exp(x - m).sum(axis=-1, keepdims=True))


def _lse(vals):
    vals = np.asarray(vals, dtype=np.float64)
    m = vals.max(axis=0)
    mm = np.where(np.isneginf(m), 0.0, m)
    with np.errstate(divide="ignore"):
        return np.log(np.exp(vals - mm).sum(axis=0)) + mm


def effective_lengths(in_len, tgt_len):
    """model/__init__.py:262-266: clamp(min=1) both, input = max(input, target)."""
    S = np.maximum(np.asarray(tgt_len, np.int64), 1)
    T = np.maximum(np.maximum(np.asarray(in_len, np.int64), 1), S)
    return T, S


def _ctc_one(lp, lab):
    """alpha, beta (Tb, L) and nll for one sample; lp (Tb, C) log-probs, lab (Sb,) labels."""
    Tb = lp.shape[0]
    ext = np.zeros(2 * len(lab) + 1, np.int64)
    ext[1::2] = lab
    L = len(ext)
    ninf = -np.inf
    skip = np.zeros(L, bool)  # s-2 -> s allowed (forward)
    skip[2:] = ext[2:] != ext[:-2]
    alpha = np.full((Tb, L), ninf)
    alpha[0, 0] = lp[0, ext[0]]
    if L > 1:
        alpha[0, 1] = lp[0, ext[1]]
    for t in range(1, Tb):
        a1 = alpha[t - 1]
        a2 = np.concatenate([[ninf], a1[:-1]])
        a3 = np.where(skip, np.concatenate([[ninf, ninf], a1[:-2]]), ninf)
        alpha[t] = _lse([a1, a2, a3]) + lp[t, ext]
    beta = np.full((Tb, L), ninf)
    beta[Tb - 1, L - 1] = lp[Tb - 1, ext[L - 1]]
    beta[Tb - 1, L - 2] = lp[Tb - 1, ext[L - 2]]
    skip_b = np.zeros(L, bool)  # s+2 -> s allowed (backward)
    skip_b[:-2] = ext[:-2] != ext[2:]
    for t in range(Tb - 2, -1, -1):
        b1 = beta[t + 1]
        b2 = np.concatenate([b1[1:], [ninf]])
        b3 = np.where(skip_b, np.concatenate([b1[2:], [ninf, ninf]]), ninf)
        beta[t] = _lse([b1, b2, b3]) + lp[t, ext]
    nll = -float(_lse([alpha[Tb - 1, L - 1], alpha[Tb - 1, L - 2]]))
    return alpha, beta, nll, ext


def ctc_compute_loss(logits, labels, in_len, tgt_len):
    """MSCA_Net.compute_loss on batch-major logits (B, T, C) -> (loss, nll (B,), dlogits).

    dlogits = d loss / d logits (float64), through the final clamp, the finite mean, the CTC
    gradient, the log-prob clamp(-100, 0) and log_softmax."""
    x = np.asarray(logits, np.float64)
    B, T, C = x.shape
    raw = _log_softmax(x)
    lp = np.clip(raw, -100.0, 0.0)
    Tb, Sb = effective_lengths(in_len, tgt_len)
    if (Tb > T).any():
        raise ValueError("input length exceeds the logits' frame count")
    nll = np.zeros(B)
    cache = []
    for b in range(B):
        al, be, n, ext = _ctc_one(lp[b, :Tb[b]], np.asarray(labels[b][:Sb[b]], np.int64))
        if np.isinf(n):  # zero_infinity=True
            n = 0.0
            cache.append(None)
        else:
            cache.append((al, be, ext))
        nll[b] = n
    finite = np.isfinite(nll)
    if finite.sum() == 0:
        return 0.0, nll, np.zeros_like(x)
    mean = nll[finite].mean()
    loss = min(max(mean, 0.0), 100.0)
    gate = 1.0 if 0.0 <= mean <= 100.0 else 0.0
    dlp = np.zeros_like(x)
    for b in range(B):
        if cache[b] is None or not finite[b]:
            continue
        al, be, ext = cache[b]
        gr = gate / finite.sum()
        ab = al + be  # (Tb, L)
        lcab = np.full((Tb[b], C), -np.inf)
        for c in np.unique(ext):
            lcab[:, c] = _lse(ab[:, ext == c].T)
        lpb = lp[b, :Tb[b]]
        dlp[b, :Tb[b]] = (np.exp(lpb) - np.exp(lcab + nll[b] - lpb)) * gr
    dlp = np.where((raw >= -100.0) & (raw <= 0.0), dlp, 0.0)  # clamp backward
    dx = dlp - np.exp(raw) * dlp.sum(axis=-1, keepdims=True)  # log_softmax backward
    return loss, nll, dx


def clamp_logits(z, lo=-50.0, hi=50.0):
    """RecognitionHead logit clamp (model/__init__.py:54-58) and its gradient gate."""
    z = np.asarray(z, np.float64)
    return np.clip(z, lo, hi), ((z >= lo) & (z <= hi)).astype(np.float64)


def seqkd(student, teacher, weight=1.0, temp=1.0, use_blank=False, lo=-np.inf, hi=np.inf):
    """clamp(weight * SeqKD(T)(student, teacher, use_blank), lo, hi) ->
    (loss, d loss / d student, d loss / d teacher)   (loss.py:11-21, model/__init__.py:203-214)."""
    s = np.asarray(student, np.float64)
    q = np.asarray(teacher, np.float64)
    st = 0 if use_blank else 1
    C = s.shape[-1]
    ss = s[..., st:].reshape(-1, C - st) / temp
    qq = q[..., st:].reshape(-1, C - st) / temp
    R = ss.shape[0]
    ls = _log_softmax(ss)
    lq = _log_softmax(qq)
    p = np.exp(lq)
    kl = (np.where(p > 0, p * lq, 0.0) - p * ls).sum() / R  # KLDivLoss(reduction='batchmean')
    v = weight * kl * temp * temp
    loss = min(max(v, lo), hi)
    k = (weight * temp * temp / R if lo <= v <= hi else 0.0) / temp
    ds = np.zeros_like(s)
    dq = np.zeros_like(q)
    h = lq - ls
    ds[..., st:] = (k * (np.exp(ls) - p)).reshape(*s.shape[:-1], C - st)
    dq[..., st:] = (k * p * (h - (p * h).sum(-1, keepdims=True))).reshape(*s.shape[:-1], C - st)
    return loss, ds, dq


def alignment_module(params, x, num_layers=2, bidirectional=True, G=None):
    """AlignmentModule forward (model/alignment_module.py:63-69) in eval mode as an explicit
    plain-torch CPU loop (torch fp32 autograd for the gradients): nn.LSTM's cell
    (i, f, g, o = chunks of x W_ih^T + b_ih + h W_hh^T + b_hh; c = sig(f) c + sig(i) tanh(g);
    h = sig(o) tanh(c)), direction 1 over reversed time, layers stacked on the concatenated
    directions, then the gloss Linear.  x: (T, B, In) sequence-first.  params: the module's
    state_dict names -> arrays.  Returns out (B, T, cls) and, with G, the gradients of
    (out * G).sum() w.r.t. x and every parameter."""
    import torch
    P = {k: torch.tensor(np.asarray(v), dtype=torch.float32, requires_grad=G is not None) for k, v in params.items()}
    xt = torch.tensor(np.asarray(x), dtype=torch.float32, requires_grad=G is not None)
    inp = xt
    D = 2 if bidirectional else 1
    for layer in range(num_layers):
        outs = []
        for d in range(D):
            s = f"_l{layer}" + ("_reverse" if d else "")
            w_ih, w_hh = P["rnn.weight_ih" + s], P["rnn.weight_hh" + s]
            b = P["rnn.bias_ih" + s] + P["rnn.bias_hh" + s]
            T, B = inp.shape[:2]
            H = w_hh.shape[1]
            h = inp.new_zeros(B, H)
            c = inp.new_zeros(B, H)
            hs = [None] * T
            for t in (range(T - 1, -1, -1) if d else range(T)):
                z = inp[t] @ w_ih.T + h @ w_hh.T + b
                i, f, g, o = z.split(H, dim=1)
                c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
                h = torch.sigmoid(o) * torch.tanh(c)
                hs[t] = h
            outs.append(torch.stack(hs))
        inp = torch.cat(outs, dim=-1)
    out = inp.permute(1, 0, 2) @ P["gloss_layer.weight"].T + P["gloss_layer.bias"]
    if G is None:
        return out.detach().numpy()
    (out * torch.tensor(np.asarray(G), dtype=torch.float32)).sum().backward()
    return out.detach().numpy(), xt.grad.numpy(), {k: v.grad.numpy() for k, v in P.items()}
