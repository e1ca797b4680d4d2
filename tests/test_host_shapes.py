"""Host-side shape logic of the attention drop-ins (CPU, no kernel calls): the kernel head size
chosen for a module head size and the zero-padded head layout (scattennet_amd/ops.py
_padded_hd / _pad_heads / _unpad_heads), which lets the (16, 32, 64, 128)-head kernels serve
every head size the reference's modules accept (model/attention.py:16-20)."""
import pytest
import torch

from scattennet_amd import ops


@pytest.mark.parametrize("hd,want", [(1, 16), (6, 16), (16, 16), (17, 32), (25, 32), (32, 32), (33, 64),
                                     (64, 64), (65, 128), (96, 128), (128, 128)])
def test_padded_head_size(hd, want):
    assert ops._padded_hd(hd) == want


def test_head_size_over_128_raises():
    with pytest.raises(ValueError):
        ops._padded_hd(129)


def test_pad_unpad_heads_round_trip():
    torch.manual_seed(0)
    B, T, H, hd, hdp = 2, 5, 3, 6, 16
    x = torch.randn(B, T, H * hd)
    (xp,) = ops._pad_heads([x], H, hd, hdp)
    assert xp.shape == (B, T, H * hdp)
    v = xp.view(B, T, H, hdp)
    assert torch.equal(v[..., :hd], x.view(B, T, H, hd))  # each head's columns first
    assert not v[..., hd:].any()                           # then zeros
    (back,) = ops._unpad_heads([xp], H, hd, hdp)
    assert torch.equal(back, x) and back.is_contiguous()


def test_padded_heads_leave_scores_and_outputs_exact():
    """Zero q / k columns add nothing to a score and zero v columns give zero output columns:
    the padded attention equals the unpadded one (the identity the GPU path relies on)."""
    torch.manual_seed(1)
    B, T, H, hd, hdp = 2, 7, 2, 5, 16

    def attn(q, k, v, d):
        qh, kh, vh = (t.view(B, T, H, d).transpose(1, 2) for t in (q, k, v))
        return (torch.softmax(qh @ kh.transpose(-1, -2), -1) @ vh).transpose(1, 2).reshape(B, T, H * d)
    q, k, v = (torch.randn(B, T, H * hd, dtype=torch.float64) for _ in range(3))
    qp, kp, vp = (ops._pad_heads([t], H, hd, hdp)[0] for t in (q, k, v))
    (o,) = ops._unpad_heads([attn(qp, kp, vp, hdp)], H, hd, hdp)
    torch.testing.assert_close(o, attn(q, k, v, hd), rtol=1e-12, atol=1e-12)
