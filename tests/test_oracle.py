"""T0: pin the CPU oracle with known answers.

The reference ships no tests or fixtures (README.md:1 only), so the oracle is pinned by
closed-form cases and independent exact arithmetic rather than by reference vectors.
"""
import math
from decimal import Decimal, getcontext
from fractions import Fraction

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R


# ---------------------------------------------------------------------------- A1 grid
@pytest.mark.parametrize("N", [2, 3, 32, 33, 128, 256, 512])
def test_grid_corners_and_order(N):
    xyz = R.grid_coords_np(N, 0, min(N, 3))
    vs = np.float32(2.0 / (N - 1))
    # index (0,0,0) -> (-1,-1,-1); x fastest
    assert tuple(xyz[0]) == (-1.0, -1.0, -1.0)
    assert xyz[N - 1, 0] == np.float32(np.float32((N - 1) * vs) - 1)
    assert xyz[N, 1] == np.float32(vs - 1)           # j = 1 after one x row
    # last x is within 1 ulp of +1 (fl32 of (N-1)*fl32(2/(N-1)) may not be exactly 2)
    assert abs(float(xyz[N - 1, 0]) - 1.0) <= 2 * np.finfo(np.float32).eps


def test_grid_two_roundings_not_fma():
    """x = fl32(fl32(i*vs) + origin) differs from a single-rounding FMA on some i."""
    N = 256
    vs = np.float32(2.0 / (N - 1))
    i = np.arange(N, dtype=np.float32)
    two = ((i * vs).astype(np.float32) + np.float32(-1)).astype(np.float32)
    fma = (i.astype(np.float64) * np.float64(vs) - 1.0).astype(np.float32)
    assert (two != fma).sum() > 0
    assert np.array_equal(R.grid_coords_np(N, 0, 1)[:N, 0], two)


def test_grid_slab_is_slice_of_full():
    N = 17
    full = R.grid_coords_np(N)
    for k0, k1 in [(0, 5), (5, 11), (11, 17)]:
        assert np.array_equal(R.grid_coords_np(N, k0, k1), full[k0 * N * N:k1 * N * N])


# ---------------------------------------------------------------------------- A2/A3 decoder
def test_decoder_dims_deepsdf():
    dims = R.decoder_layer_dims(256, 512)
    assert dims[0] == (259, 512)
    assert dims[3] == (512, 253)
    assert dims[4] == (512, 512)           # 253 + 256 + 3
    assert dims[8] == (512, 1)
    assert len(dims) == 9
    wd = R.decoder_layer_dims(1024, 512, widen_skip=True)
    assert wd[3] == (512, 512) and wd[4] == (512 + 1027, 512)


def test_zero_weights_give_tanh_of_last_bias():
    p = R.make_decoder_params(L=16, H=64, seed=0)
    for w in p.weights:
        w.zero_()
    p.biases[-1].fill_(0.3)
    z = torch.randn(2, 16, dtype=torch.float64)
    xyz = torch.rand(5, 3, dtype=torch.float64)
    out = R.decoder_forward(p, z, xyz)
    assert torch.allclose(out, torch.full_like(out, math.tanh(0.3)), atol=0, rtol=0)


def test_analytic_l1_network():
    """Closed-form network: sdf = tanh(c (|x|+|y|+|z|) - r)."""
    L, H = 4, 64
    p = R.make_decoder_params(L=L, H=H, seed=0)
    for w, b in zip(p.weights, p.biases):
        w.zero_()
        b.zero_()
    W0 = p.weights[0]
    for a in range(3):     # h0 rows 2a, 2a+1 = relu(+x_a), relu(-x_a)
        W0[2 * a, L + a] = 1.0
        W0[2 * a + 1, L + a] = -1.0
    for l in range(1, 8):  # pass the 6 channels through (layer 3 out width is H-(L+3))
        for c in range(6):
            p.weights[l][c, c] = 1.0
    c, r = 0.7, 0.25
    p.weights[8][0, :6] = c
    p.biases[8][0] = -r
    xyz = torch.rand(100, 3, dtype=torch.float64) * 2 - 1
    z = torch.randn(1, L, dtype=torch.float64)
    want = torch.tanh(c * xyz.abs().sum(1) - r)[None]
    assert torch.allclose(R.decoder_forward(p, z, xyz), want, atol=1e-15)
    beta = R.latent_fold(p, z)
    assert torch.allclose(R.decoder_forward_folded(p, beta, xyz), want, atol=1e-15)


@pytest.mark.parametrize("L,H,widen", [(256, 512, False), (32, 128, False), (1024, 512, True)])
def test_fold_equals_concat(L, H, widen):
    p = R.make_decoder_params(L=L, H=H, widen_skip=widen, seed=3)
    z = torch.randn(3, L, dtype=torch.float64) * 0.1
    xyz = torch.rand(64, 3, dtype=torch.float64) * 2 - 1
    a = R.decoder_forward(p, z, xyz)
    b = R.decoder_forward_folded(p, R.latent_fold(p, z), xyz)
    assert torch.allclose(a, b, atol=1e-12)


def test_he_init_output_scale():
    """He-init keeps outputs O(0.01-0.1) so tolerances are meaningful."""
    p = R.make_decoder_params(seed=1234)
    z = torch.randn(1, 256, dtype=torch.float64) * 0.1
    out = R.decoder_forward(p, z, R.grid_coords(16).double())
    assert 0.005 < float(out.std()) < 0.5


# ---------------------------------------------------------------------------- A4 schedule
def test_schedule_constants_exact():
    tab = R.ddpm_tables(1000)
    assert tab.betas[0] == 1e-4 and abs(tab.betas[-1] - 0.02) < 1e-18
    assert tab.alphas_cumprod[0] == 1 - 1e-4
    assert np.all(np.diff(tab.alphas_cumprod) < 0)
    # independent exact product: abar_T with rational betas (linspace is exact in Q)
    getcontext().prec = 50
    prod = Decimal(1)
    for t in range(1000):
        beta = Fraction(1, 10000) + (Fraction(2, 100) - Fraction(1, 10000)) * Fraction(t, 999)
        prod *= Decimal(1) - Decimal(beta.numerator) / Decimal(beta.denominator)
    assert abs(float(prod) - tab.alphas_cumprod[-1]) / float(prod) < 1e-12
    # published ballpark: sqrt(abar_T) ~ 6.4e-3 for the DDPM linear schedule
    assert 6.0e-3 < tab.sqrt_ab[-1] < 6.6e-3
    # c2 * sqrt(1-abar) == beta ; c1^2 * alpha == 1
    assert np.allclose(tab.c2 * tab.sqrt_1mab, tab.betas, rtol=1e-14)
    assert np.allclose(tab.c1 ** 2 * tab.alphas, 1.0, rtol=1e-14)


# ---------------------------------------------------------------------------- A5 embedding
def test_timestep_embedding_known_values():
    e = R.timestep_embedding_table(1000, 128)
    assert e.shape == (1000, 128) and e.dtype == np.float32
    assert np.all(e[0, :64] == 0) and np.all(e[0, 64:] == 1)
    # k = 0 frequency is 1: e[t,0] = sin(t)
    assert abs(e[7, 0] - math.sin(7)) < 1e-7
    # k = 63 frequency is 1e-4
    assert abs(e[999, 63] - math.sin(999 * 1e-4)) < 1e-7


# ---------------------------------------------------------------------------- A8/A9/A10
def test_step_order_and_t0():
    tab = R.ddpm_tables()
    x = torch.randn(4, 8)
    eps = torch.randn(4, 8)
    z = torch.randn(4, 8)
    y0 = R.ddpm_step(tab, x, eps, z, 0)
    c1, c2 = np.float32(tab.c1[0]), np.float32(tab.c2[0])
    want = (np.float32(c1) * (x.numpy() - np.float32(c2) * eps.numpy())).astype(np.float32)
    assert np.array_equal(y0.numpy(), want)          # z ignored at t = 0
    y5 = R.ddpm_step(tab, x, eps, z, 5)
    assert not torch.equal(y5, R.ddpm_step(tab, x, eps, torch.zeros_like(z), 5))


def test_q_sample_endpoints():
    tab = R.ddpm_tables()
    x0 = torch.randn(3, 5, dtype=torch.float64)
    eps = torch.randn(3, 5, dtype=torch.float64)
    t = torch.tensor([0, 500, 999])
    xt = R.q_sample(tab, x0, eps, t)
    assert torch.allclose(xt[0], x0[0] * float(np.float32(tab.sqrt_ab[0])) +
                          eps[0] * float(np.float32(tab.sqrt_1mab[0])))
    # at t = T-1 the signal is almost gone
    assert float((xt[2] - eps[2]).abs().max()) < 0.02 * float(x0[2].abs().max()) + 1e-3


def test_train_grads_match_finite_difference():
    p = R.make_denoiser_params(D=8, H=16, n_blocks=2, TE=8, seed=1)
    tab = R.ddpm_tables(50)
    emb = torch.from_numpy(R.timestep_embedding_table(50, 8)).double()
    x0 = torch.randn(5, 8, dtype=torch.float64)
    eps = torch.randn(5, 8, dtype=torch.float64)
    t = torch.tensor([0, 3, 10, 25, 49])
    loss, grads = R.train_step_grads(p, tab, emb, x0, eps, t)
    h = 1e-6
    w = p.Wblk[1]
    i, j = 3, 20
    w[i, j] += h
    xt = R.q_sample(tab, x0, eps, t)
    lp = R.eps_mse_loss(R.denoiser_forward(p, xt, t, emb), eps)
    w[i, j] -= 2 * h
    lm = R.eps_mse_loss(R.denoiser_forward(p, xt, t, emb), eps)
    w[i, j] += h
    fd = (lp - lm) / (2 * h)
    assert abs(float(fd) - float(grads["Wblk1"][i, j])) < 1e-6
