"""C17 oracle pinning (CPU): the 1D-UNet oracle (oracle/ref_unet.py) against an independent
pure-Python loop restatement of DESIGN.md §9 on a small network, conv/upsample semantics
against hand sums, fp32 vs fp64 agreement, and the product's initialiser against the
oracle's (one seed = one network on both sides).  Parity vs the reference is unpinned (the
reference has no code, README.md:1)."""
import math

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from oracle import ref_unet as U


def _silu(v):
    return v / (1.0 + math.exp(-v))


def _conv_loop(x, w, b, stride=1, up2=False, silu=False):
    """x: list[C][L] floats, w: [Cout][Cin][K] (tensor), pad = (K-1)//2 -- textbook loops."""
    Cin, L = len(x), len(x[0])
    Cout, _, K = w.shape
    pad = (K - 1) // 2
    src = [[_silu(v) if silu else v for v in row] for row in x]
    if up2:
        src = [[row[p // 2] for p in range(2 * L)] for row in src]
        L = 2 * L
    Lout = (L + 2 * pad - K) // stride + 1
    out = []
    for co in range(Cout):
        row = []
        for l in range(Lout):
            s = float(b[co]) if b is not None else 0.0
            for ci in range(Cin):
                for k in range(K):
                    p = l * stride + k - pad
                    if 0 <= p < L:
                        s += float(w[co, ci, k]) * src[ci][p]
            row.append(s)
        out.append(row)
    return out


def _add(a, b):
    return [[u + v for u, v in zip(ra, rb)] for ra, rb in zip(a, b)]


def _unet_loop(up, x, t, emb):
    """DESIGN.md §9 for ONE sample, scalar loops (x: list[D])."""
    p = {k: v.double() for k, v in up.p.items()}
    e = torch.from_numpy(emb[t]).double()
    hid = [_silu(float(v)) for v in (p["Wt1"] @ e + p["bt1"])]
    temb = [float(v) for v in (p["Wt2"] @ torch.tensor(hid, dtype=torch.float64) + p["bt2"])]

    def res(i, xin):
        a = _conv_loop(xin, p[f"res{i}.w1"], p[f"res{i}.b1"], silu=True)
        pt = [sum(float(p[f"res{i}.p"][co, j]) * temb[j] for j in range(len(temb)))
              for co in range(len(a))]
        a = [[v + pt[co] for v in row] for co, row in enumerate(a)]
        y = _conv_loop(a, p[f"res{i}.w2"], p[f"res{i}.b2"], silu=True)
        if f"res{i}.ws" in p:
            return _add(y, _conv_loop(xin, p[f"res{i}.ws"], p[f"res{i}.bs"]))
        return _add(y, xin)

    h = _conv_loop([list(x)], p["conv_in.w"], p["conv_in.b"])
    s0 = res(0, h)
    h = _conv_loop(s0, p["down0.w"], p["down0.b"], stride=2)
    s1 = res(1, h)
    h = _conv_loop(s1, p["down1.w"], p["down1.b"], stride=2)
    h = res(3, res(2, h))
    h = _conv_loop(h, p["up1.w"], p["up1.b"], up2=True)
    h = res(4, h + s1)
    h = _conv_loop(h, p["up0.w"], p["up0.b"], up2=True)
    h = res(5, h + s0)
    return _conv_loop(h, p["conv_out.w"], p["conv_out.b"], silu=True)[0]


def test_unet_oracle_matches_scalar_loops():
    up = U.make_unet_params(D=16, C=(2, 3, 4), TE=8, HT=6, seed=5)
    emb = R.timestep_embedding_table(1000, 8)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 16, generator=g, dtype=torch.float64)
    t = torch.tensor([17, 803])
    got = U.unet_forward(up, x, t, torch.from_numpy(emb).double())
    for bi in range(2):
        want = _unet_loop(up, x[bi].tolist(), int(t[bi]), emb)
        np.testing.assert_allclose(got[bi].numpy(), np.array(want), rtol=1e-12, atol=1e-12)


def test_conv_semantics_hand_sums():
    """k=3 pad=1 cross-correlation, stride-2 taps and nearest-2x upsample on a 1-channel ramp."""
    x = torch.arange(1.0, 9.0, dtype=torch.float64)[None, None]          # 1..8
    w = torch.tensor([[[1.0, 10.0, 100.0]]], dtype=torch.float64)
    y = torch.nn.functional.conv1d(x, w, padding=1)[0, 0]
    assert y[0].item() == 0 * 1 + 1 * 10 + 2 * 100                       # left zero pad
    assert y[7].item() == 7 * 1 + 8 * 10 + 0 * 100                       # right zero pad
    y2 = torch.nn.functional.conv1d(x, w, stride=2, padding=1)[0, 0]
    assert y2.tolist() == [_conv_loop([x[0, 0].tolist()], w, None, stride=2)[0][i]
                           for i in range(4)]
    assert y2[1].item() == 2 * 1 + 3 * 10 + 4 * 100                       # taps 2l-1 .. 2l+1
    u = torch.nn.functional.interpolate(x, scale_factor=2, mode="nearest")[0, 0]
    assert u.tolist() == [1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8]


def test_unet_fp32_vs_fp64():
    up = U.make_unet_params(seed=2468)
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128))
    x = torch.randn(2, 1024, generator=torch.Generator().manual_seed(0), dtype=torch.float64)
    t = torch.tensor([999, 3])
    e64 = U.unet_forward(up, x, t, emb.double())
    e32 = U.unet_forward(up.map(lambda v: v.float()), x.float(), t, emb)
    assert float(e64.std()) > 0.05                     # O(1) output, meaningful tolerance
    assert float((e32.double() - e64).abs().max()) < 1e-4


def test_product_init_equals_oracle_init():
    from ldm_sdf import UNet1DDenoiser
    m = UNet1DDenoiser(seed=2468)
    up = U.make_unet_params(seed=2468, dtype=torch.float32)
    assert set(m.params) == set(up.p)
    for k, v in up.p.items():
        assert torch.equal(m.params[k], v), k


def test_unet_sample_loop_first_step():
    up = U.make_unet_params(D=64, C=(4, 8, 8), seed=9)
    tab = R.ddpm_tables()
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128)).double()
    g = torch.Generator().manual_seed(1)
    xT = torch.randn(3, 64, generator=g, dtype=torch.float64)
    noise = torch.randn(1000, 3, 64, generator=g, dtype=torch.float64)
    x1 = U.unet_sample_loop(up, tab, emb, xT, noise, steps=1)
    eps = U.unet_forward(up, xT, torch.full((3,), 999), emb)
    assert torch.equal(x1, R.ddpm_step(tab, xT, eps, noise[999], 999))


@pytest.mark.parametrize("D", [12, 30])
def test_unet_rejects_bad_length(D):
    from ldm_sdf import UNet1DDenoiser
    if D % 4:
        with pytest.raises(ValueError):
            UNet1DDenoiser(D=D)
    else:
        UNet1DDenoiser(D=D, C=(2, 2, 2), HT=8, TE=8)


def test_pack_conv_weight_layout():
    """ldm_conv1d's packed weight: [Cout16][K][Cw16], channel ci at perm16(ci), zero pad."""
    from ldm_sdf import ops
    g = torch.Generator().manual_seed(0)
    W = torch.randn(5, 20, 3, generator=g)
    P = ops.pack_conv_weight(W)
    assert P.shape == (16, 3, 32)
    perm = ops.perm16_index(32).tolist()
    assert sorted(perm) == list(range(32))
    for m in range(4):                 # lane group g reads channels 4m+g at 4g+m
        for gg in range(4):
            assert perm[4 * m + gg] == 4 * gg + m
    for co in range(5):
        for ci in range(20):
            for k in range(3):
                assert P[co, k, perm[ci]] == W[co, ci, k]
    assert int((P != 0).sum()) == W.numel()                   # everything else is zero


def test_conv_args_validation_on_host():
    """conv1d_args builds/validates the C struct without touching a GPU."""
    from ldm_sdf import LdmError, ops
    X = torch.randn(2, 20, 64)
    Wp = ops.pack_conv_weight(torch.randn(8, 40, 3))
    Y = torch.empty(2, 8, 64)
    a = ops.conv1d_args([ops.ConvSegment(X, Wp, silu=True), ops.ConvSegment(X, Wp, c_off=16)],
                        Y)
    assert a.n_seg == 2 and a.seg[1].W - a.seg[0].W == 16 * 4
    assert a.seg[0].ldw == 3 * 48 and a.seg[0].kstride == 48
    with pytest.raises(LdmError):      # channel offset not a multiple of 16
        ops.conv1d_args([ops.ConvSegment(X, Wp, c_off=8)], Y)
    with pytest.raises(LdmError):      # output length mismatch
        ops.conv1d_args([ops.ConvSegment(X, Wp)], torch.empty(2, 8, 63))
    with pytest.raises(LdmError):      # unpacked weight
        ops.conv1d_args([ops.ConvSegment(X, torch.randn(8, 20, 3))], Y)
