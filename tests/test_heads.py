"""Recognition-head losses: MSCA_Net.compute_loss (CTC) and SeqKD.

CPU: the numpy oracle (oracle/heads_oracle.py) against golden vectors captured from the
reference itself (tests/golden/heads_*.npz, tests/golden/gen_golden_heads.py) and against
torch's own CTC op at extra shapes.  GPU: the HIP path (scattennet_amd.heads ->
sca_ctc_loss_* / sca_seqkd_* / sca_clamp) against the same fixtures and the oracle.

Tolerances (fp32 kernels vs fp32 reference / float64 oracle): losses rel 1e-5 + abs 1e-4
(the CTC loss is a sum over up to 64 frames of log-sum-exps), gradients abs 2e-5.
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import heads_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CTC_FIX = sorted(glob.glob(os.path.join(GOLD, "heads_ctc_*.npz")))
KD_FIX = sorted(glob.glob(os.path.join(GOLD, "heads_kd_*.npz")))
LOSS_TOL = dict(rtol=1e-5, atol=1e-4)
GRAD_TOL = dict(rtol=1e-4, atol=2e-5)


def _load(p):
    return dict(np.load(p, allow_pickle=False))


def test_fixtures_present():
    assert len(CTC_FIX) == 3 and len(KD_FIX) == 3


@pytest.mark.parametrize("path", CTC_FIX, ids=os.path.basename)
def test_oracle_ctc_matches_reference(path):
    f = _load(path)
    loss, _, dx = O.ctc_compute_loss(f["logits"], f["labels"], f["in_len"], f["tgt_len"])
    np.testing.assert_allclose(loss, f["loss"], **LOSS_TOL)
    np.testing.assert_allclose(dx, f["dlogits"], **GRAD_TOL)


@pytest.mark.parametrize("path", KD_FIX, ids=os.path.basename)
def test_oracle_seqkd_matches_reference(path):
    f = _load(path)
    loss, ds, dq = O.seqkd(f["student"], f["teacher"], float(f["weight"]), float(f["temp"]), bool(f["use_blank"]),
                           -100.0, 100.0)
    np.testing.assert_allclose(loss, f["loss"], **LOSS_TOL)
    np.testing.assert_allclose(ds, f["dstudent"], **GRAD_TOL)
    if not f["detach"]:
        np.testing.assert_allclose(dq, f["dteacher"], **GRAD_TOL)


@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_ctc_matches_torch_ctc(seed):
    """Extra shapes: the per-sample nll against torch.nn.functional.ctc_loss directly."""
    rng = np.random.default_rng(seed)
    B, T, C, S = 5, 30, 17, 9
    x = rng.standard_normal((B, T, C)).astype(np.float32) * 2
    labels = rng.integers(1, C, size=(B, S))
    in_len = rng.integers(10, T + 1, size=B)
    tgt_len = rng.integers(1, S + 1, size=B)
    _, nll, _ = O.ctc_compute_loss(x, labels, in_len, tgt_len)
    lp = torch.log_softmax(torch.tensor(x), -1).clamp(-100, 0).permute(1, 0, 2)
    Te, Se = O.effective_lengths(in_len, tgt_len)
    ref = torch.nn.functional.ctc_loss(lp, torch.tensor(labels), torch.tensor(Te), torch.tensor(Se), blank=0,
                                       reduction="none", zero_infinity=True)
    np.testing.assert_allclose(nll, ref.numpy(), rtol=1e-5, atol=1e-4)


def test_cpu_tensors_refused():
    from scattennet_amd import heads
    with pytest.raises(RuntimeError):
        heads.clamp_logits(torch.zeros(4, 4))


def test_bad_lengths_raise_like_torch():
    from scattennet_amd import heads
    x = torch.zeros(2, 8, 5)
    with pytest.raises(RuntimeError, match="input_lengths"):
        heads._validate_ctc(torch.ones(2, 3, dtype=torch.long), torch.tensor([3, 2]), torch.tensor([9, 8]), 2, 8, 5)
    with pytest.raises(RuntimeError, match="targets"):
        heads._validate_ctc(torch.ones(2, 3, dtype=torch.long), torch.tensor([4, 2]), torch.tensor([8, 8]), 2, 8, 5)
    with pytest.raises(RuntimeError, match="target values"):
        heads._validate_ctc(torch.full((2, 3), 5, dtype=torch.long), torch.tensor([3, 2]), torch.tensor([8, 8]),
                            2, 8, x.shape[-1])


def test_batch_size_mismatches_raise():
    """labels / input_lengths / target_lengths must hold one entry per clip (the kernels index
    them by clip); the CPU-side checks run before any launch."""
    from scattennet_amd import heads
    x = torch.zeros(3, 8, 5)  # a CPU tensor: the checks must fire before the device check
    with pytest.raises(RuntimeError, match="labels must be"):
        heads.compute_loss(torch.ones(2, 3, dtype=torch.long), torch.tensor([3, 2, 1]), x, torch.tensor([8, 8, 8]))
    with pytest.raises(RuntimeError, match="target_lengths"):
        heads.compute_loss(torch.ones(3, 3, dtype=torch.long), torch.tensor([3, 2]), x, torch.tensor([8, 8, 8]))
    with pytest.raises(RuntimeError, match="input_lengths"):
        heads.compute_loss(torch.ones(3, 3, dtype=torch.long), torch.tensor([3, 2, 1]), x, torch.tensor([8, 8]))


def test_concatenated_targets_are_split_by_lengths():
    """nn.CTCLoss's 1-D target form: clip b's labels are the next tgt_len[b] entries (lengths
    clamped to >= 1 first, as the reference passes them)."""
    from scattennet_amd import heads
    flat = torch.tensor([4, 1, 2, 3, 3, 2])
    out = heads._pad_concatenated(flat, torch.tensor([2, 0, 3]), 3)
    assert out.tolist() == [[4, 1, 0], [2, 0, 0], [3, 3, 2]]
    with pytest.raises(RuntimeError, match="sum to"):
        heads._pad_concatenated(flat[:4], torch.tensor([2, 0, 3]), 3)


# ---------------------------------------------------------------------------- GPU parity
def _hip_ctc(f):
    from scattennet_amd import heads
    x = torch.tensor(f["logits"], device="cuda", requires_grad=True)
    loss, nll = heads.compute_loss(torch.tensor(f["labels"]), torch.tensor(f["tgt_len"]), x,
                                   torch.tensor(f["in_len"]), return_per_sample=True)
    loss.backward()
    torch.cuda.synchronize()
    return loss.item(), nll.cpu().numpy(), x.grad.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("path", CTC_FIX, ids=os.path.basename)
def test_hip_ctc_matches_reference(path):
    f = _load(path)
    loss, _, dx = _hip_ctc(f)
    np.testing.assert_allclose(loss, f["loss"], **LOSS_TOL)
    np.testing.assert_allclose(dx, f["dlogits"], **GRAD_TOL)


@pytest.mark.gpu
@pytest.mark.parametrize("concat", [False, True])
@pytest.mark.parametrize("B,T,C,S", [(8, 64, 1124, 24), (3, 200, 64, 90), (16, 1, 8, 1)])
def test_hip_ctc_matches_oracle(B, T, C, S, concat):
    rng = np.random.default_rng(B * 1000 + T)
    x = (rng.standard_normal((B, T, C)) * 2).astype(np.float32)
    labels = rng.integers(1, C, size=(B, S)).astype(np.int32)
    labels[0, :3] = labels[0, 0]  # repeats
    tgt_len = rng.integers(0, S + 1, size=B)
    in_len = np.maximum(rng.integers(0, T + 1, size=B), np.minimum(np.maximum(tgt_len, 1) * 2 + 1, T))
    for b in range(B):  # keep losses below the 100 clamp: plant one alignment
        Sb = max(int(tgt_len[b]), 1)
        Tb = max(int(in_len[b]), 1, Sb)
        for t in range(Tb):
            x[b, t, labels[b, min(t * Sb // Tb, Sb - 1)]] += 8.0
    f = {"logits": x, "labels": labels, "in_len": in_len.astype(np.int32), "tgt_len": tgt_len.astype(np.int32)}
    ref_loss, ref_nll, ref_dx = O.ctc_compute_loss(x, labels, in_len, tgt_len)
    if concat:  # the same targets in nn.CTCLoss's concatenated 1-D form
        f["labels"] = np.concatenate([labels[b, :max(int(tgt_len[b]), 1)] for b in range(B)])
    loss, nll, dx = _hip_ctc(f)
    np.testing.assert_allclose(nll, ref_nll, rtol=1e-5, atol=2e-4)
    np.testing.assert_allclose(loss, ref_loss, **LOSS_TOL)
    np.testing.assert_allclose(dx, ref_dx, **GRAD_TOL)


@pytest.mark.gpu
@pytest.mark.parametrize("path", KD_FIX, ids=os.path.basename)
def test_hip_seqkd_matches_reference(path):
    from scattennet_amd import heads
    f = _load(path)
    s = torch.tensor(f["student"], device="cuda", requires_grad=True)
    q = torch.tensor(f["teacher"], device="cuda", requires_grad=not bool(f["detach"]))
    w = float(f["weight"])
    if f["detach"] and not f["use_blank"] and float(f["temp"]) == 1.0:
        loss = heads.distillation_loss(s, q, w)
    else:
        loss = torch.clamp(w * heads.SeqKD(T=float(f["temp"]))(s, q, use_blank=bool(f["use_blank"])), -100, 100)
    loss.backward()
    np.testing.assert_allclose(loss.item(), f["loss"], **LOSS_TOL)
    np.testing.assert_allclose(s.grad.cpu().numpy(), f["dstudent"], **GRAD_TOL)
    if not f["detach"]:
        np.testing.assert_allclose(q.grad.cpu().numpy(), f["dteacher"], **GRAD_TOL)


@pytest.mark.gpu
def test_hip_recognition_head_and_losses_end_to_end():
    """Head classifiers + clamp + CTC + SeqKD fwd/bwd against the oracle."""
    from scattennet_amd import heads
    torch.manual_seed(0)
    cfg = {"residual_blocks": [256, 256, 512, 512], "out_fusion_dim": 1024}
    head = heads.RecognitionHead(cfg, 300).cuda()
    B, T = 4, 64
    feats = [torch.randn(B, T, 512, device="cuda", requires_grad=True) for _ in range(3)]
    fuse = torch.randn(B, T, 1024, device="cuda", requires_grad=True) * 20
    fuse.retain_grad()
    out = head(feats[0], feats[1], fuse, feats[2])
    W = head.fuse_coord_classifier
    z = (fuse.detach() @ W.weight.detach().T + W.bias.detach()).cpu().numpy()
    zc, gate = O.clamp_logits(z)
    np.testing.assert_allclose(out["fuse_coord_gloss_logits"].detach().cpu().numpy(), zc, rtol=1e-4, atol=1e-3)
    labels = torch.randint(1, 300, (B, 12))
    tl, il = torch.tensor([5, 4, 3, 1]), torch.tensor([12, 10, 6, 2])  # losses below the 100 clamp
    loss = heads.compute_loss(labels, tl, out["left"], il)
    loss = loss + heads.distillation_loss(out["body"], out["fuse_coord_gloss_logits"], 0.5)
    loss.backward()
    Wl = head.left_gloss_classifier
    zl = (feats[0].detach() @ Wl.weight.detach().T + Wl.bias.detach()).cpu().numpy()
    zlc, gate_l = O.clamp_logits(zl)
    ref_ctc, _, dctc = O.ctc_compute_loss(zlc.astype(np.float32), labels.numpy(), il.numpy(), tl.numpy())
    ref_kd, _, _ = O.seqkd(out["body"].detach().cpu().numpy(), zc, 0.5, 1.0, False, -100, 100)
    assert 0 < ref_ctc < 100
    np.testing.assert_allclose(loss.item(), ref_ctc + ref_kd, rtol=1e-4, atol=1e-3)
    # d loss / d left features = (dctc * gate) W_left; the SeqKD teacher (fuse) is detached
    dleft = (dctc * gate_l) @ Wl.weight.detach().cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(feats[0].grad.cpu().numpy(), dleft, rtol=1e-3, atol=1e-5)
    assert fuse.grad is None or float(fuse.grad.abs().max()) == 0.0


# ---------------------------------------------------------------------------- AlignmentModule
ALIGN_FIX = os.path.join(GOLD, "heads_align_B3_T12.npz")


def _align_params(f):
    return {k[6:]: f[k] for k in f if k.startswith("param.")}


def test_oracle_alignment_matches_reference():
    f = _load(ALIGN_FIX)
    out, dx, grads = O.alignment_module(_align_params(f), f["x"], 2, True, G=f["G"])
    np.testing.assert_allclose(out, f["out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(dx, f["dx"], rtol=1e-4, atol=1e-5)
    for k, g in grads.items():
        np.testing.assert_allclose(g, f["grad." + k], rtol=1e-4, atol=1e-5, err_msg=k)


def _hip_alignment(params, x, G, hidden, cls):
    from scattennet_amd.alignment import AlignmentModule
    m = AlignmentModule(cls, x.shape[-1], hidden, num_layers=2, dropout=0.3, bidirectional=True).cuda().eval()
    m.load_state_dict({k: torch.tensor(v) for k, v in params.items()})
    xt = torch.tensor(x, device="cuda", requires_grad=True)
    out = m(xt)
    (out * torch.tensor(G, device="cuda")).sum().backward()
    torch.cuda.synchronize()
    return out.detach().cpu().numpy(), xt.grad.cpu().numpy(), {k: p.grad.cpu().numpy() for k, p in
                                                                m.named_parameters()}


@pytest.mark.gpu
def test_hip_alignment_matches_reference():
    f = _load(ALIGN_FIX)
    out, dx, grads = _hip_alignment(_align_params(f), f["x"], f["G"], 64, 20)
    np.testing.assert_allclose(out, f["out"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(dx, f["dx"], rtol=1e-4, atol=2e-5)
    for k, g in grads.items():
        np.testing.assert_allclose(g, f["grad." + k], rtol=1e-4, atol=2e-5, err_msg=k)


@pytest.mark.gpu
def test_hip_alignment_phoenix_size_matches_oracle():
    """The yaml's head (input 1024, hidden 1024 = 2 x 512, 2 layers) at B = 4, T/4 = 64."""
    torch.manual_seed(0)
    from scattennet_amd.alignment import AlignmentModule
    ref = AlignmentModule(300, 1024, 1024)
    params = {k: v.numpy() for k, v in ref.state_dict().items()}
    rng = np.random.default_rng(5)
    x = rng.standard_normal((64, 4, 1024)).astype(np.float32)
    G = rng.standard_normal((4, 64, 300)).astype(np.float32)
    o_out, o_dx, o_grads = O.alignment_module(params, x, 2, True, G=G)
    out, dx, grads = _hip_alignment(params, x, G, 1024, 300)
    np.testing.assert_allclose(out, o_out, rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(dx, o_dx, rtol=1e-3, atol=1e-4)
    for k, g in grads.items():
        scale = float(np.abs(o_grads[k]).max())
        np.testing.assert_allclose(g, o_grads[k], rtol=1e-3, atol=1e-4 * max(scale, 1.0), err_msg=k)


def test_alignment_state_dict_keys_match_reference():
    """Drop-in boundary: the reference's AlignmentModule parameter names (from its fixture) load strictly."""
    from scattennet_amd.alignment import AlignmentModule
    f = _load(ALIGN_FIX)
    m = AlignmentModule(20, 64, 64, num_layers=2, dropout=0.3, bidirectional=True)
    m.load_state_dict({k: torch.tensor(v) for k, v in _align_params(f).items()}, strict=True)
    assert set(m.state_dict()) == set(_align_params(f))
