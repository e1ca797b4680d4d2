"""torch.library coverage of the drop-in blocks (scattennet_amd/library.py).

CPU: every block operator has a fake (meta) implementation, and torch.compile captures a
whole drop-in SCA stack (x-stream self layers, y-stream causal layers, merges, embeddings)
as ONE graph (fullgraph=True: no graph break) whose forward is the scatten operators and
whose AOT backward is their *_backward operators — traced on FakeTensors, nothing executed.
GPU: tests/test_gpu_library_ops.py runs the compiled stack against the eager grouped path.
"""
import pytest
import torch

import scattennet_amd as S
from scattennet_amd import workloads as W


class _Captured(Exception):
    pass


def _trace(model, *args):
    """fullgraph dynamo + AOT autograd trace on FakeTensors; -> (forward ops, backward ops).
    The joint graph's partition records both graphs and stops before anything runs."""
    from torch._dynamo.backends.common import aot_autograd
    from torch._functorch.partitioners import default_partition
    graphs = {}

    def partition(joint, joint_inputs, **kw):
        fw, bw = default_partition(joint, joint_inputs, **kw)
        for name, gm in (("fw", fw), ("bw", bw)):
            graphs[name] = {str(n.target) for n in gm.graph.nodes if n.op == "call_function"}
        raise _Captured()

    def never(gm, example_inputs):
        raise AssertionError("compiler reached")

    backend = aot_autograd(fw_compiler=never, bw_compiler=never, partition_fn=partition)
    torch._dynamo.reset()
    fn = torch.compile(model, backend=backend, fullgraph=True)
    with pytest.raises(Exception) as ei:
        fn(*args)
    torch._dynamo.reset()
    return graphs, ei


def test_block_ops_have_fake_impls():
    from torch._subclasses.fake_tensor import FakeTensorMode
    ops = torch.ops.scatten
    with FakeTensorMode():
        B, T, d, H, F = 2, 12, 32, 4, 64
        x = torch.empty(B, T, d)
        p8 = [torch.empty(d, d), torch.empty(d)] * 4
        out = ops.attention_block(x, None, p8, torch.empty(d), torch.empty(d), torch.empty(B, T), None, "self", H,
                                  0.5, False, True, 1e-5)
        assert [tuple(t.shape) for t in out[:5]] == [(B, T, d)] * 5 and len(out) == 10
        kv = torch.empty(B, 7, d)
        out = ops.attention_block(x, kv, p8, None, None, torch.empty(B, 7), None, "cross", H, 0.5, False, True, -1.0)
        assert tuple(out[2].shape) == (B, 7, d) and len(out) == 7
        g = ops.attention_block_backward(x, x, kv, p8, None, None, None, None, out[1:], "cross", H, 0.5, False, True,
                                         -1.0)
        assert len(g) == 10 and tuple(g[1].shape) == (B, 7, d)
        out = ops.feed_forward(x, [torch.empty(F, d), torch.empty(F), torch.empty(d, F), torch.empty(d)],
                               torch.empty(d), torch.empty(d), True, 1e-5)
        assert tuple(out[1].shape) == (B * T, F) and len(out) == 6
        y, z = ops.linear(x, torch.empty(F, d), torch.empty(F), None, True)
        assert tuple(y.shape) == (B, T, F) and tuple(z.shape) == (B * T, F)
        y, m, r = ops.layer_norm_ex(x, torch.empty(T + 2, d), None, torch.empty(d), torch.empty(d), 1e-5, False)
        assert tuple(m.shape) == (B * T,)
        assert tuple(ops.maxpool_t(torch.empty(B, 9, d)).shape) == (B, 4, d)
        xe, ye = ops.coordinate_mapping(torch.empty(B, T, 40, 2), torch.empty(6, dtype=torch.int32),
                                        torch.empty(d, 6), torch.empty(d), torch.empty(d, 6), torch.empty(d))
        assert tuple(xe.shape) == (B, T, d) == tuple(ye.shape)
        assert tuple(ops.clip_matmul(torch.empty(B, 5, d), torch.empty(B, 6, d), True).shape) == (B, 5, 6)
        assert tuple(ops.softmax_rows(torch.empty(B, 5, 6)).shape) == (B, 5, 6)


def test_sca_stack_compiles_to_one_graph_of_scatten_ops():
    """SeparativeCoordinateAttention (L = 2, eval: dropout off) under torch.compile."""
    torch.manual_seed(0)
    d, H, T, B = 64, 4, 16, 2
    cfg = W.model_cfg(d, H, 2, maxpos=T)
    sca = S.SeparativeCoordinateAttention(cfg).eval()
    x = torch.randn(B, T, d, requires_grad=True)
    y = torch.randn(B, T, d, requires_grad=True)
    mask = torch.ones(B, T, dtype=torch.long)
    mask[1, 9:] = 0
    graphs, ei = _trace(lambda a, b: sca(a, b, mask), x, y)
    assert "bw" in graphs, ei.value  # a graph break or a failed trace ends before the partition
    fw, bw = graphs["fw"], graphs["bw"]
    for op in ("scatten.attention_block.default", "scatten.feed_forward.default", "scatten.layer_norm_ex.default"):
        assert op in fw, fw
    for op in ("scatten.attention_block_backward.default", "scatten.feed_forward_backward.default",
               "scatten.layer_norm_ex_backward.default"):
        assert op in bw, bw


def test_keypoint_module_with_residual_network_compiles():
    """KeypointModule (coordinate mapping -> SCA -> ResidualNetwork incl. MaxPool over
    frames) under torch.compile: one graph, the mapping / Linear / pool operators in it."""
    torch.manual_seed(1)
    d, H, T, B = 64, 4, 16, 2
    cfg = dict(W.model_cfg(d, H, 1, maxpos=T), residual_blocks=[d, d, 2 * d, 2 * d])
    mod = S.KeypointModule(list(range(5)), T, cfg).eval()
    kp = torch.rand(B, T, 5, 2)
    mask = torch.ones(B, T, dtype=torch.long)
    graphs, ei = _trace(lambda k: mod(k, mask), kp)
    assert "bw" in graphs, ei.value
    for op in ("scatten.coordinate_mapping.default", "scatten.linear.default", "scatten.maxpool_t.default"):
        assert op in graphs["fw"], graphs["fw"]
