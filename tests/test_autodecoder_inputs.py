"""The auto-decoder's bf16 input operand (ldm_sdf/autodecoder.py _ad_inputs):
the broadcast form used when every k-block lies in one shape equals the per-sample gathers,
in both layouts, padding rows and columns included.  CPU only (torch ops)."""
import pytest
import torch


@pytest.mark.parametrize("S,P,KT", [(4, 1024, 512), (3, 2048, 2048), (2, 256, 256)])
def test_broadcast_inputs_equal_gathers(S, P, KT):
    from ldm_sdf.autodecoder import _ad_inputs
    g = torch.Generator().manual_seed(S * P + KT)
    L, zw = 40, 64
    z = torch.randn(S, L, generator=g)
    xyz = torch.randn(S, P, 3, generator=g)
    N = S * P
    Np = -(-N // KT) * KT + KT                  # one all-padding block past the samples
    fast = _ad_inputs(z, xyz, S, P, Np, zw, KT)
    slow = _ad_inputs(z, xyz, S, P, Np, zw, KT, gather=True)
    for a, b in zip(fast, slow):
        assert torch.equal(a, b)
    Zx, ZxT = fast
    assert torch.equal(ZxT.permute(1, 0, 2).reshape(zw, Np), Zx.t())
    assert not Zx[N:].any() and not Zx[:, L + 3:].any()
