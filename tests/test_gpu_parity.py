"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors.

Every module is built with the reference's constructor arguments, loads the reference's
state_dict from the fixture (proving key-layout compatibility), runs forward + backward on
the MI355X with the same upstream gradient G, and must match the reference outputs and ALL
gradients within PARITY_TOL relative (BASELINE.json north_star: 1e-3 relative fp32).
"""
import pytest
import torch

from tests.golden_util import close, load, manifest, rel_err

PARITY_TOL = 1e-3  # north_star: outputs match the reference PyTorch forward within 1e-3 relative fp32

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda:0")


def _check(fx, module, out, inputs, grad_inputs, tol=PARITY_TOL):
    errs = {"out": rel_err(out, fx["out"])}
    assert errs["out"] < tol, errs
    (out * fx["gout"].to(out.device)).sum().backward()
    gscale = max(float(g.abs().max()) for g in fx["grad_param"].values())
    named = dict(module.named_parameters())
    for k in grad_inputs:
        e = rel_err(inputs[k].grad, fx["grad_in"][k])
        errs["d" + k] = e
        assert e < tol, (k, errs)
    for k, g in fx["grad_param"].items():
        got = named[k].grad
        assert got is not None, k
        assert close(got.cpu(), g, tol, gscale), (k, rel_err(got.cpu(), g))
    for k, p in named.items():
        if k not in fx["grad_param"]:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k
    return errs


def _inputs(fx, dev, grad_inputs):
    out = {}
    for k, v in fx["in"].items():
        t = v.to(dev)
        if k in grad_inputs:
            t.requires_grad_(True)
        out[k] = t
    return out


def _load(module, fx, dev):
    module.load_state_dict(fx["param"])
    return module.to(dev).eval()


ATTN = [n for n in manifest()["fixtures"] if n.startswith("attn_")]


@pytest.mark.parametrize("compact", [False, True], ids=["materialised_mask", "key_padding_mask"])
@pytest.mark.parametrize("name", ATTN)
def test_attention_ops(name, compact):
    import scattennet_amd as S
    dev = _dev()
    fx = load(name)
    meta = fx["meta"]
    kind = name.split("_")[1]
    cls = {"self": S.SelfAttention, "causal": S.SelfCausalAttention, "cross": S.CrossAttention}[kind]
    m = _load(cls(meta["d"], meta["H"]), fx, dev)
    gi = ("hidden_states", "key_value_states") if kind == "cross" else ("hidden_states",)
    i = _inputs(fx, dev, gi)
    x = i["hidden_states"]
    if compact:
        mask = S.key_padding_mask(i["mask"], causal=(kind == "causal"))
    elif kind == "causal":
        mask = S.create_causal_attention_mask(i["mask"], x.shape[:2], x)
    else:
        mask = S.create_attention_mask(i["mask"], torch.float32)
    out = m(x, i["key_value_states"], mask) if kind == "cross" else m(x, mask)
    _check(fx, m, out, i, gi)


@pytest.mark.parametrize("kind", ["self_attn", "causal_attn"])
def test_coordinate_attention(kind):
    import scattennet_amd as S
    dev = _dev()
    fx = load("coordattn_" + kind)
    m = _load(S.CoordinateAttention(fx["meta"]["cfg"], kind), fx, dev)
    i = _inputs(fx, dev, ("coord_embed",))
    mask = S.key_padding_mask(i["mask"], causal=(kind == "causal_attn"))
    _check(fx, m, m(i["coord_embed"], mask), i, ("coord_embed",))


def test_coordinates_merge():
    import scattennet_amd as S
    dev = _dev()
    fx = load("coordmerge")
    m = _load(S.CoordinatesMerge(fx["meta"]["cfg"]), fx, dev)
    i = _inputs(fx, dev, ("y_embed", "x_embed"))
    out = m(i["y_embed"], i["x_embed"], S.create_attention_mask(i["mask"], torch.float32))
    _check(fx, m, out, i, ("y_embed", "x_embed"))


def test_sca_stack():
    import scattennet_amd as S
    dev = _dev()
    fx = load("sca_L2")
    m = _load(S.SeparativeCoordinateAttention(fx["meta"]["cfg"]), fx, dev)
    i = _inputs(fx, dev, ("x_embed", "y_embed"))
    _check(fx, m, m(i["x_embed"], i["y_embed"], i["mask"]), i, ("x_embed", "y_embed"))


def test_coordinate_mapping():
    import scattennet_amd as S
    dev = _dev()
    fx = load("coordmap")
    m = _load(S.CoordinateMapping(21, 64), fx, dev)
    i = _inputs(fx, dev, ("x_coord", "y_coord"))
    out = torch.cat(m(i["x_coord"], i["y_coord"]), -1)
    _check(fx, m, out, i, ("x_coord", "y_coord"))


@pytest.mark.parametrize("name", ["residual_64_64_128_128", "residual_64_64", "residual_64_64_T45"])
def test_residual_network(name):
    import scattennet_amd as S
    dev = _dev()
    fx = load(name)
    m = _load(S.ResidualNetwork(fx["meta"]["blocks"]), fx, dev)
    i = _inputs(fx, dev, ("x",))
    _check(fx, m, m(i["x"])[0], i, ("x",))


def test_keypoint_module():
    import scattennet_amd as S
    dev = _dev()
    fx = load("keypoint_module")
    meta = fx["meta"]
    m = _load(S.KeypointModule(list(range(3, 24)), meta["T"], meta["cfg"]), fx, dev)
    i = _inputs(fx, dev, ("keypoints",))
    _check(fx, m, m(i["keypoints"], i["mask"]), i, ("keypoints",))


# T/4 = 16, and frame counts whose per-clip (T/4 x T/4) attention has rows that are not a
# multiple of 4 floats (the any-shape GEMM form): the reference's own smoke size 45, odd 13
@pytest.mark.parametrize("name", ["fusion", "fusion_T45", "fusion_T13"])
def test_coordinates_fusion(name):
    import scattennet_amd as S
    dev = _dev()
    fx = load(name)
    m = _load(S.CoordinatesFusion(fx["meta"]["in"], fx["meta"]["out"], 0.2), fx, dev)
    gi = ("left", "right", "body")
    i = _inputs(fx, dev, gi)
    _check(fx, m, m(i["left"], i["right"], i["body"]), i, gi)


def test_xstream_cfg1():
    """BASELINE config 1 (B=2 T=64 K=27 d=64 H=4, x-stream, L = 2 as captured) through the
    HIP drop-ins: CoordinateMapping's x half (model/layers.py:111-123), the self position
    embedding + first LayerNorm (keypoint_module.py:155, 161, one fused launch) and the self
    layers (:176-178) — against the reference's own vectors (gen_golden_xstream.py)."""
    import scattennet_amd as S
    from scattennet_amd.layers import coordinate_mapping_grouped, pos_embed_layernorm_grouped
    from torch import nn
    dev = _dev()
    fx = load("xstream_cfg1")
    cfg, K = fx["meta"]["cfg"], fx["meta"]["K"]

    class XStream(nn.Module):  # the fixture's module tree (KeypointModule key names)
        def __init__(self):
            super().__init__()
            self.coordinate_mapping = S.CoordinateMapping(K, cfg["d_model"])
            self.sca = nn.Module()
            self.sca.self_attn_layers = nn.ModuleList([S.CoordinateAttention(cfg, "self_attn")
                                                       for _ in range(cfg["attn_layers"])])
            self.sca.first_self_norm = nn.LayerNorm(cfg["d_model"])
            self.sca.self_pos_embed = S.LearningPositionEmbedding(cfg["max_position_embeddings"], cfg["d_model"])

        def forward(self, keypoints, mask):
            cm = self.coordinate_mapping
            xe, _ = coordinate_mapping_grouped([cm], keypoints, [cm.joint_index(keypoints.device)])
            s = pos_embed_layernorm_grouped([self.sca.self_pos_embed], [self.sca.first_self_norm], xe)[0]
            m = S.create_attention_mask(mask, s.dtype)
            for layer in self.sca.self_attn_layers:
                s = layer(s, m)
            return s

    m = _load(XStream(), fx, dev)
    i = _inputs(fx, dev, ("keypoints",))
    _check(fx, m, m(i["keypoints"], i["mask"]), i, ("keypoints",))
