"""sca_reduce_rows (the fixed-order row sums behind every bias / LayerNorm-affine / position-table
gradient) at kernel level against float64 sums: the few-row float4 form (S <= 16, N % 4 == 0)
and the 16-wave form (more rows, or N % 4 != 0), with a row stride, several column blocks (I), a
scale and accumulation; repeated launches are bit-identical (fixed order)."""
import pytest
import torch

from scattennet_amd import ops

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda:0")


@pytest.mark.parametrize("S,I,N", [(7, 1, 256), (16, 3, 64), (17, 1, 256), (1024, 1, 512), (300, 2, 100),
                                   (257, 1, 30), (2048, 1, 4), (64, 5, 1000)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_reduce_rows_vs_float64(S, I, N, accumulate):
    dev = _dev()
    g = torch.Generator().manual_seed(S * 131 + N)
    nprob = 3
    # rows of a (S, I, N) tensor with stride_s = I * N, stride_i = N
    ins = [torch.randn(S, I, N, generator=g).to(dev) for _ in range(nprob)]
    outs = [torch.randn(I, N, generator=g).to(dev) for _ in range(nprob)]
    base = [o.clone() for o in outs]
    scales = [1.0, 0.5, -2.0]
    ops.reduce_rows([(ins[p], outs[p], scales[p]) for p in range(nprob)], S, I, N, I * N, N, accumulate=accumulate)
    torch.cuda.synchronize()
    for p in range(nprob):
        ref = ins[p].double().sum(0) * scales[p]
        if accumulate:
            ref += base[p].double()
        err = float((outs[p].double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        assert err < 2e-6, (S, I, N, p, err)
    # deterministic: the same launch gives the same bits
    again = [torch.empty_like(o) for o in outs]
    for p in range(nprob):
        again[p].copy_(base[p])
    ops.reduce_rows([(ins[p], again[p], scales[p]) for p in range(nprob)], S, I, N, I * N, N, accumulate=accumulate)
    torch.cuda.synchronize()
    for p in range(nprob):
        assert torch.equal(again[p], outs[p]), (S, I, N, p)
