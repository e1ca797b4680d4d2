"""GPU parity at BASELINE sizes against the CPU oracle (oracle/sca_oracle.py, itself pinned
to the reference's golden vectors by tests/test_oracle_golden.py).

Config 2 (the metric's workload: B=8, T=256, K=79 as 6/21/21/31 joints, d=256, H=16, L=4)
and config 5 (T=1024, d=512, hd=32) with ragged key-padding masks (full, T-37, T/2, 1, 0, ...
lengths), forward AND every gradient, within the north-star 1e-3 relative fp32 bound.
"""
import pytest
import torch

from oracle import sca_oracle as O
from scattennet_amd import workloads as W
from tests.golden_util import close, rel_err

PARITY_TOL = 1e-3  # north_star: within 1e-3 relative fp32

pytestmark = pytest.mark.gpu


def _run(name, w, streams_used=None):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    torch.set_num_threads(min(16, torch.get_num_threads()))
    dev = torch.device("cuda:0")
    w = dict(w)
    if streams_used is not None:
        w["groups"] = w["groups"][:streams_used]
    model = W.build_streams(w, dev, seed=3, init="random")
    kp, mask, gout = W.synthetic_batch(w, dev, seed=5, ragged=True)
    outs = model(kp, mask)
    torch.autograd.backward(outs, [gout[g] for g in range(len(outs))])
    torch.cuda.synchronize()

    cfg = W.model_cfg(w["d"], w["H"], w["L"], maxpos=w["maxpos"])
    groups = W.split_groups(w["groups"])
    for g, mod in enumerate(model.streams):
        p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in mod.state_dict().items()}
        ref = O.multi_stream_sca([p], kp.cpu(), mask.cpu(), [groups[g]], cfg)[0]
        e = rel_err(outs[g], ref)
        assert e < PARITY_TOL, (name, g, "out", e)
        (ref * gout[g].cpu()).sum().backward()
        grads = {k: v.grad for k, v in p.items() if v.grad is not None}
        gscale = max(float(t.abs().max()) for t in grads.values())
        named = dict(mod.named_parameters())
        for k, gr in grads.items():
            got = named[k].grad
            assert got is not None, k
            assert close(got.cpu(), gr, PARITY_TOL, gscale), (name, g, k, rel_err(got.cpu(), gr))


def test_cfg2_four_streams_vs_oracle():
    _run("cfg2", W.WORKLOADS["cfg2"])


def test_cfg5_long_sequence_vs_oracle():
    # one stream of the T=1024, d=512 (hd=32) config: the causal y-stream tiles through LDS
    _run("cfg5", W.WORKLOADS["cfg5"], streams_used=1)


def _encoder_oracle(enc, cfg, kp, mask, gout):
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in enc.state_dict().items()}
    streams = {}
    for name, idx in (("body", cfg["body_idx"]), ("left", cfg["left_idx"]), ("right", cfg["right_idx"])):
        streams[name] = O.keypoint_module(p, f"{name}_encoder", kp[:, :, idx, :], mask, cfg)
    ref = O.coordinates_fusion(p, "coordinates_fusion", streams["left"], streams["right"], streams["body"])
    (ref * gout).sum().backward()
    return ref.detach(), {k: v.grad for k, v in p.items() if v.grad is not None}


def test_cfg3_full_encoder_vs_oracle():
    """BASELINE config 3: yaml model section, 3 streams + residual + fusion, ragged masks.

    The residual network's ReLU + MaxPool1d make a few gradients discontinuous at fp32
    resolution: at this seed right_encoder.residual.blocks.2 has max-pool pairs whose values
    differ by 4e-6 at magnitude 6 (7e-7 relative), below the fp32 forward error of ANY
    implementation, so which frame receives the gradient is a coin toss.  A gradient
    therefore passes at PARITY_TOL, or — only where the oracle itself is that ill-conditioned —
    within 2x the oracle's own spread when its inputs are perturbed at the fp32 level
    (3e-5 relative, two samples)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    torch.set_num_threads(min(16, torch.get_num_threads()))
    dev = torch.device("cuda:0")
    w = W.WORKLOADS["cfg3"]
    enc = W.build_encoder(w, dev, seed=4, init="random").eval()  # parity at eval (dropout off)
    kp, mask, gout = W.synthetic_batch(w, dev, seed=6, ragged=True)
    fuse = enc(kp, mask)[0]
    fuse.backward(gout[0])
    torch.cuda.synchronize()
    cfg = W.encoder_cfg(w)
    kpc, mc, gc = kp.cpu(), mask.cpu(), gout[0].cpu()
    ref, grads = _encoder_oracle(enc, cfg, kpc, mc, gc)
    assert rel_err(fuse, ref) < PARITY_TOL
    spread = {k: 0.0 for k in grads}
    gen = torch.Generator().manual_seed(11)
    for _ in range(2):
        kp_p = kpc * (1 + 3e-5 * torch.randn(kpc.shape, generator=gen))
        _, g_p = _encoder_oracle(enc, cfg, kp_p, mc, gc)
        for k in grads:
            spread[k] = max(spread[k], rel_err(g_p[k], grads[k]))
    gscale = max(float(t.abs().max()) for t in grads.values())
    named = dict(enc.named_parameters())
    relaxed = []
    for k, gr in grads.items():
        assert named[k].grad is not None, k
        got = named[k].grad.cpu()
        if close(got, gr, PARITY_TOL, gscale):
            continue
        e = rel_err(got, gr)
        assert spread[k] > PARITY_TOL and e < 2 * spread[k], (k, e, spread[k])
        relaxed.append(k)
    assert len(relaxed) < len(grads) // 4, relaxed
    for k, prm in named.items():  # parameters the reference never trains (long shortcuts)
        if k not in grads:
            assert prm.grad is None, k
