"""C19 (auto-decoder training) on the CPU: the oracle's objective pinned by known answers and
finite differences, and the product's host-side working layout (pure data movement)."""
import math

import pytest
import torch

from oracle import ref_cpu as R
from oracle import ref_autodecoder as A


def _tiny(seed=3):
    return R.make_decoder_params(L=4, H=16, n_hidden=8, skip=4, seed=seed)


def test_loss_zero_when_prediction_matches():
    p = _tiny()
    g = torch.Generator().manual_seed(0)
    z = torch.randn(2, 4, generator=g, dtype=torch.float64) * 0.3
    xyz = torch.rand(2, 5, 3, generator=g, dtype=torch.float64) * 2 - 1
    sdf = R.decoder_forward(p, z, xyz).detach()
    assert float(A.autodecoder_loss(p, z, xyz, sdf, reg_lambda=0.0)) == 0.0
    # targets far outside the clamp band on the same side as the prediction's clamp: only
    # the clamped parts differ
    big = torch.full_like(sdf, 5.0)
    pred_c = sdf.clamp(-0.1, 0.1)
    want = (pred_c - 0.1).abs().mean()
    assert abs(float(A.autodecoder_loss(p, z, xyz, big, reg_lambda=0.0)) - float(want)) < 1e-15


def test_code_regulariser_known_answer():
    """reg = lambda * min(1, epoch/100) * sum_samples |z| / N = lambda * w * mean_s |z_s|."""
    p = _tiny()
    z = torch.tensor([[3.0, 4.0, 0.0, 0.0], [0.0, 0.0, 0.0, 1.0]], dtype=torch.float64)
    xyz = torch.zeros(2, 3, 3, dtype=torch.float64)
    sdf = R.decoder_forward(p, z, xyz).detach()
    for epoch, w in ((100, 1.0), (50, 0.5), (250, 1.0)):
        got = float(A.autodecoder_loss(p, z, xyz, sdf, reg_lambda=0.01, epoch=epoch))
        assert abs(got - 0.01 * w * (5.0 + 1.0) / 2) < 1e-15


def test_oracle_gradients_match_finite_differences():
    """The float64 autograd the GPU parity tests compare against, against central differences
    (targets inside the clamp band, so the loss is smooth except on measure-zero kinks)."""
    p = _tiny(seed=11)
    g = torch.Generator().manual_seed(1)
    z = torch.randn(2, 4, generator=g, dtype=torch.float64) * 0.5
    xyz = torch.rand(2, 6, 3, generator=g, dtype=torch.float64) * 2 - 1
    sdf = (torch.rand(2, 6, generator=g, dtype=torch.float64) - 0.5) * 0.15
    loss, gr = A.autodecoder_grads(p, z, xyz, sdf, reg_lambda=0.05)
    eps = 1e-6

    def f(pp, zz):
        return float(A.autodecoder_loss(pp, zz, xyz, sdf, reg_lambda=0.05))

    for l in (0, 3, 4, 8):
        for (i, j) in ((0, 0), (1, 2)):
            W = p.weights[l]
            if i >= W.shape[0] or j >= W.shape[1]:
                continue
            hi, lo = p.to(torch.float64), p.to(torch.float64)
            hi.weights[l] = W.clone(); hi.weights[l][i, j] += eps
            lo.weights[l] = W.clone(); lo.weights[l][i, j] -= eps
            fd = (f(hi, z) - f(lo, z)) / (2 * eps)
            assert abs(fd - float(gr[f"W{l}"][i, j])) < 1e-6 * max(1.0, abs(fd)), (l, i, j)
    for (s, c) in ((0, 0), (1, 3)):
        zh, zl = z.clone(), z.clone()
        zh[s, c] += eps
        zl[s, c] -= eps
        fd = (f(p, zh) - f(p, zl)) / (2 * eps)
        assert abs(fd - float(gr["z"][s, c])) < 1e-6 * max(1.0, abs(fd))
    assert loss > 0


def test_work_layout_round_trip():
    """work_weights pads, master_grads cuts back: with the padded weights fed back in as
    'gradients' the masters come out unchanged, and every pad is zero."""
    from ldm_sdf.autodecoder import master_grads, work_weights
    L, H, skip = 256, 512, 4
    dims = R.decoder_layer_dims(L, H)
    g = torch.Generator().manual_seed(5)
    m = {}
    for l, (i, o) in enumerate(dims):
        m[f"W{l}"] = torch.randn(o, i, generator=g)
        m[f"b{l}"] = torch.randn(o, generator=g)
    w = work_weights(m, L, H, skip, torch.float32)
    assert tuple(w["W0"].shape) == (H, 264) and float(w["W0"][:, 259:].abs().sum()) == 0
    assert tuple(w["W3"].shape) == (256, H) and float(w["W3"][253:].abs().sum()) == 0
    assert float(w["b3p"][253:].abs().sum()) == 0
    assert float(w["W4h"][:, 253:].abs().sum()) == 0 and float(w["W4z"][:, 259:].abs().sum()) == 0
    gw = dict(w)
    for l in range(9):
        gw[f"b{l}"] = m[f"b{l}"]
    gw["b3"] = w["b3p"]
    out = {k: torch.empty_like(v) for k, v in m.items()}
    master_grads(gw, L, skip, 253, out)
    for k in m:
        assert torch.equal(out[k], m[k]), k
