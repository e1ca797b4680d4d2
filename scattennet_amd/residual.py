"""Drop-in ResidualNetwork (model/residual.py of tinh2044/SCAttenNet) — the Linear/LN/ReLU/
MaxPool1d "pool" stage after SCA in every KeypointModule.  HIP path: grouped GEMMs
(projection, linear1, linear2), LayerNorm with fused ReLU / residual+ReLU epilogues, and a
frame-axis max-pool kernel."""
import torch
import torch.nn as nn

from . import library, ops
from .layers import layernorm_grouped
from .precision import fp32_compute


class ResidualBlock(nn.Module):
    """model/residual.py:5-45."""

    def __init__(self, in_dim, out_dim, downsample=False):
        super().__init__()
        self.downsample = downsample
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.need_projection = in_dim != out_dim
        if self.need_projection:
            self.projection = nn.Linear(in_dim, out_dim)
        self.linear1 = nn.Linear(in_dim, out_dim)
        self.norm1 = nn.LayerNorm(out_dim)
        self.relu = nn.ReLU()
        self.linear2 = nn.Linear(out_dim, out_dim)
        self.norm2 = nn.LayerNorm(out_dim)
        if self.downsample:
            self.pool = nn.MaxPool1d(kernel_size=2, stride=2)

    @fp32_compute()
    def forward(self, x):
        return residual_block_grouped([self], [x])[0]


def _linear(layers, xs):
    G = len(xs)
    return list(library.linear_apply(G, False, *xs, *[l.weight for l in layers], *[l.bias for l in layers]))


_FAN_OUT_X = True  # A/B (tools/bench_var.py): the block input's two gradients summed by autograd


def residual_block_grouped(blocks, xs):
    """out = relu(norm2(linear2(relu(norm1(linear1 x)))) + proj?(x)); then MaxPool over T."""
    b0 = blocks[0]
    # x has two consumers (linear1 and the projection / the identity residual of norm2): one
    # fan-out, so that its two gradients are summed in one grouped launch for all streams
    # instead of one autograd add per stream
    x_lin, x_res = ops.fan_out(xs, 2) if _FAN_OUT_X and not library.compiling() else (xs, xs)
    r = _linear([b.projection for b in blocks], x_res) if b0.need_projection else x_res
    h = _linear([b.linear1 for b in blocks], x_lin)
    h = layernorm_grouped([b.norm1 for b in blocks], h, relu=True)
    h = _linear([b.linear2 for b in blocks], h)
    h = layernorm_grouped([b.norm2 for b in blocks], h, post=r, relu=True)
    if b0.downsample:
        h = list(library.maxpool_t_apply(len(h), *h))
    return h


class PermuteLayer(nn.Module):
    """model/residual.py:122-128."""

    def __init__(self, *dims):
        super().__init__()
        self.dims = dims

    @fp32_compute()
    def forward(self, x):
        return x.permute(*self.dims)


class ResidualNetwork(nn.Module):
    """model/residual.py:48-118.  Returns (x, outputs) like the reference."""

    def __init__(self, residual_blocks):
        super().__init__()
        self.residual_blocks = residual_blocks
        self.blocks = nn.ModuleList()
        self.shortcuts = nn.ModuleList()
        for i in range(len(residual_blocks)):
            in_dim = residual_blocks[i - 1] if i > 0 else residual_blocks[0]
            out_dim = residual_blocks[i]
            self.blocks.append(ResidualBlock(in_dim, out_dim, downsample=i % 2 == 0))
            if i > 0:
                need_projection = (residual_blocks[i - 2] != residual_blocks[i] if i > 1
                                   else residual_blocks[0] != residual_blocks[i])
                need_downsample = (i % 2 == 0) and ((i - 1) % 2 == 1)
                if need_projection or need_downsample:
                    sc = nn.Sequential()
                    if need_projection:
                        sc_in = residual_blocks[i - 2] if i > 1 else residual_blocks[0]
                        sc.add_module("projection", nn.Linear(sc_in, residual_blocks[i]))
                    if need_downsample:
                        sc.add_module("permute1", PermuteLayer(0, 2, 1))
                        sc.add_module("pool", nn.MaxPool1d(kernel_size=2, stride=2))
                        sc.add_module("permute2", PermuteLayer(0, 2, 1))
                    self.shortcuts.append(sc)
                else:
                    self.shortcuts.append(None)

    @fp32_compute()
    def forward(self, x):
        outs = residual_network_grouped([self], [x], return_all=True)
        return outs[0][-1], outs[0]


def _shortcut_matches(blocks, i, T_in_src, T_block):
    """Shape test of model/residual.py:110 evaluated analytically: the long shortcut output
    (outputs[i-2] or the input, optionally projected, pooled when need_downsample) vs the
    block output."""
    need_downsample = (i % 2 == 0) and ((i - 1) % 2 == 1)
    T_sc = T_in_src // 2 if need_downsample else T_in_src
    return T_sc == T_block  # channels always match (projection to blocks[i])


def residual_network_grouped(nets, xs, return_all=False):
    """G-way ResidualNetwork.  The long shortcuts (residual.py:63-90) are added only when
    their shape matches the block output (:110-113).  For every layout the reference ships
    ([256,256,512,512], [256,256]) they never match, so the reference computes them and
    throws them away (their parameters never receive a gradient); here their shape test is
    evaluated up front and they are not computed."""
    blocks = nets[0].residual_blocks
    T_hist = [xs[0].shape[1]]  # frames of shortcut_outputs[j]
    outs = []
    x = xs
    for i in range(len(blocks)):
        y = residual_block_grouped([n.blocks[i] for n in nets], x)
        if i > 0:
            src = i - 2 if i > 1 else 0
            if _shortcut_matches(blocks, i, T_hist[src], y[0].shape[1]):
                raise NotImplementedError("ResidualNetwork long shortcut with matching shape: not reachable for "
                                          "the reference configurations; not implemented")
        x = y
        outs.append(x)
        T_hist.append(x[0].shape[1])
    if return_all:
        return [[o[g] for o in outs] for g in range(len(nets))]
    return x
