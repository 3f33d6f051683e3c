"""C17 parity on the MI355X: ldm_conv1d (every tap geometry, segment / bias / residual / DDPM
epilogue combination) vs an fp64 torch conv of the same operands, and the 1D-UNet forward and
10-step sampling trajectory vs the fp64 oracle (oracle/ref_unet.py, tests/golden/unet_10.npz).

Tolerances (written here, measured on the box):
  conv1d fp32 weights: max abs <= 1e-5 (fp32 accumulate of <= 4*128*3 products of O(1) values)
  conv1d bf16 weights: vs fp64 conv with the SAME bf16-rounded weights, <= 1e-5
  UNet fp32 forward / 10-step trajectory vs fp64 oracle: <= 1e-4
  UNet bf16 forward vs fp64 oracle with bf16-rounded weights: <= 1e-4; vs unrounded: <= 0.1
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ldm_sdf
    ldm_sdf.load_library()
    return torch.device("cuda", 0)


def _ref_seg(X, W, c_off, stride, mode, silu):
    Cs = X.shape[1]
    w = W[:, c_off:c_off + Cs].double()
    x = X.double()
    if silu:
        x = x * torch.sigmoid(x)
    if mode == 1:
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    return F.conv1d(x, w, stride=stride, padding=(W.shape[2] - 1) // 2 if W.shape[2] != 4 else 1)


CASES = [
    # name, B, [(Cin, L_in, ksize, stride, mode, silu)], Cout, cbias, residual
    ("k3s1", 3, [(16, 100, 3, 1, 0, False)], 32, False, False),
    ("k3s1_silu_cb_res", 2, [(40, 130, 3, 1, 0, True)], 40, True, True),
    ("k3s2", 2, [(33, 257, 3, 2, 0, False)], 70, False, False),
    ("up2", 2, [(64, 37, 3, 1, 1, False)], 20, False, False),
    ("concat", 2, [(32, 64, 3, 1, 0, True), (20, 64, 3, 1, 0, True)], 24, True, False),
    ("big_b_tile64", 40, [(64, 256, 3, 1, 0, True)], 64, True, True),
    ("k3_plus_1x1", 2, [(32, 64, 3, 1, 0, True), (16, 64, 1, 1, 0, False),
                        (16, 64, 1, 1, 0, False)], 32, False, False),
    ("k4s2", 2, [(8, 130, 4, 2, 0, False)], 5, False, False),
    ("cin1_cout1", 5, [(1, 1024, 3, 1, 0, False)], 1, False, False),
    # direct staging (ldm_conv1d's launch kernel: power-of-two channel blocks, L_in % 4 == 0,
    # the cases above with other sizes take the generic staging)
    ("up2_direct", 2, [(64, 64, 3, 1, 1, True)], 32, True, False),
    ("k3s2_direct", 2, [(32, 128, 3, 2, 0, True)], 48, False, True),
    ("k4s2_direct", 3, [(16, 128, 4, 2, 0, False)], 16, False, False),
    ("concat_up2_direct", 2, [(64, 32, 3, 1, 1, True), (32, 32, 3, 1, 1, True)], 24, True, False),
    ("four_seg_generic", 2, [(32, 64, 3, 1, 0, True), (16, 64, 3, 1, 0, True),
                            (16, 64, 1, 1, 0, False), (64, 64, 1, 1, 0, False)], 32, True, True),
    ("c128_tile32_direct", 16, [(128, 128, 3, 1, 0, True)], 128, True, True),
]


@pytest.mark.parametrize("wdt", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_conv1d_vs_torch(dev, case, wdt):
    from ldm_sdf import ops
    name, B, segs, Cout, use_cb, use_r = case
    g = torch.Generator().manual_seed(sum(map(ord, name)))
    tdt = {"fp32": torch.float32, "bf16": torch.bfloat16}[wdt]
    Xs, Ws, specs = [], {}, []
    ref = None
    c_off = {}
    for (Cin, L_in, K, st, mode, silu) in segs:
        X = torch.randn(B, Cin, L_in, generator=g)
        Xs.append(X)
    # one weight per kernel size, segments of equal ksize are column blocks of it
    for K in sorted({s[2] for s in segs}):
        Ctot = sum(s[0] for s in segs if s[2] == K)
        Ws[K] = (torch.randn(Cout, Ctot, K, generator=g) / np.sqrt(Ctot * K)).to(tdt)
        c_off[K] = 0
    bias = torch.randn(Cout, generator=g)
    for X, (Cin, L_in, K, st, mode, silu) in zip(Xs, segs):
        specs.append((X, Ws[K], c_off[K], st, mode, silu))
        r = _ref_seg(X, Ws[K].float(), c_off[K], st, mode, silu)
        ref = r if ref is None else ref + r
        c_off[K] += Cin
    ref = ref + bias.double()[None, :, None]
    L_out = ref.shape[2]
    cb = torch.randn(B, Cout, generator=g) if use_cb else None
    if cb is not None:
        ref = ref + cb.double()[:, :, None]
    R = torch.randn(B, Cout, L_out, generator=g) if use_r else None
    if R is not None:
        ref = ref + R.double()
    Y = torch.empty(B, Cout, L_out, device=dev)
    segs_dev = [ops.ConvSegment(X.to(dev), ops.pack_conv_weight(W.to(dev)), c_off=co, stride=st, mode=mode, silu=silu,
                                pad=1)
                for (X, W, co, st, mode, silu) in specs]
    for s in segs_dev:
        if s.ksize == 1:
            s.pad = 0
    ops.conv1d(segs_dev, Y, bias=bias.to(dev), cbias=None if cb is None else cb.to(dev),
               scb=Cout, R=None if R is None else R.to(dev))
    err = float((Y.cpu().double() - ref).abs().max())
    assert err <= 1e-5, f"{name} {wdt}: {err}"


def test_conv1d_ddpm_epilogue(dev):
    from ldm_sdf import DDPMSchedule, ops
    from oracle import ref_cpu as R
    sch = DDPMSchedule()
    sd = sch.device(dev)["desc"]
    tab = R.ddpm_tables()
    g = torch.Generator().manual_seed(5)
    B, C, L = 3, 16, 256
    X = torch.randn(B, C, L, generator=g)
    W = torch.randn(1, C, 3, generator=g) / 7
    b = torch.randn(1, generator=g)
    x = torch.randn(B, L, generator=g)
    z = torch.randn(B, L, generator=g)
    for t in (0, 1, 640, 999):
        out = torch.empty(B, L, device=dev)
        ops.conv1d([ops.ConvSegment(X.to(dev), ops.pack_conv_weight(W.to(dev)), silu=True)],
                   out.view(B, 1, L),
                   bias=b.to(dev), epi=1, xlat=x.to(dev), z=z.to(dev), sched=sd, t=t)
        eps = _ref_seg(X, W, 0, 1, 0, True)[:, 0] + b.double()
        want = R.ddpm_step(tab, x.double(), eps, z.double(), t)
        assert float((out.cpu().double() - want).abs().max()) < 1e-5, t


def test_conv1d_rejects_bad_args(dev):
    from ldm_sdf import LdmError, ops
    X = torch.randn(1, 4, 10, device=dev)
    W = ops.pack_conv_weight(torch.randn(2, 4, 5, device=dev))      # ksize 5 unsupported
    with pytest.raises(LdmError):
        ops.conv1d([ops.ConvSegment(X, W)], torch.empty(1, 2, 10, device=dev))
    W3 = ops.pack_conv_weight(torch.randn(2, 4, 3, device=dev))
    with pytest.raises(LdmError):                 # wrong output length
        ops.conv1d([ops.ConvSegment(X, W3)], torch.empty(1, 2, 9, device=dev))
    with pytest.raises(LdmError):                 # unpacked [Cout, Cin, K] weight
        ops.conv1d([ops.ConvSegment(X, torch.randn(2, 4, 3, device=dev))],
                   torch.empty(1, 2, 10, device=dev))


def _unet(dtype=torch.float64, rounded=False):
    from oracle import ref_unet as U
    up = U.make_unet_params(seed=2468)
    if rounded:   # the bf16 product path's weights, exactly
        up = up.map(lambda v: v)
        for k in list(up.p):
            if not k.startswith("b") and not k.endswith((".b", ".b1", ".b2", ".bs")):
                up.p[k] = up.p[k].float().bfloat16().double()
    return up


def test_unet_forward_vs_golden(dev):
    import ldm_sdf
    from oracle import ref_cpu as R
    from oracle import ref_unet as U
    gd = dict(np.load(os.path.join(GOLD, "unet_10.npz")))
    m = ldm_sdf.UNet1DDenoiser(seed=2468)
    x = torch.from_numpy(gd["x_T"]).to(dev)
    for i, t in enumerate(gd["t_mixed"].tolist()):
        got = m.forward_uniform_t(x, int(t), dtype="fp32").cpu().double()
        err = float((got[i] - torch.from_numpy(gd["eps_mixed"][i])).abs().max())
        assert err <= 1e-4, (t, err)
    # bf16 weights: vs the oracle on the same rounded weights (tight) and unrounded (loose)
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128)).double()
    xt = torch.from_numpy(gd["x_T"]).double()
    want_r = U.unet_forward(_unet(rounded=True), xt, torch.full((2,), 999), emb)
    got = m.forward_uniform_t(x, 999, dtype="bf16").cpu().double()
    e_r = float((got - want_r).abs().max())
    e_u = float((got[0] - torch.from_numpy(gd["eps_mixed"][0])).abs().max())
    print(f"bf16 unet: vs rounded-weight oracle {e_r:.2e}, vs fp64 oracle {e_u:.2e}")
    assert e_r <= 1e-4 and e_u <= 0.1


@pytest.mark.parametrize("path", ["eager", "graph"])
@pytest.mark.parametrize("n", [2, 1])       # n = 1: the skip concats as one buffer (unet.py)
def test_unet_sampling_10_vs_golden(dev, path, n):
    import ldm_sdf
    gd = dict(np.load(os.path.join(GOLD, "unet_10.npz")))
    steps = int(gd["steps"])
    m = ldm_sdf.UNet1DDenoiser(seed=2468)
    sch = ldm_sdf.DDPMSchedule()
    noise = torch.zeros(1000, 2, 1024)
    noise[1000 - steps:] = torch.from_numpy(gd["noise_tail"])
    x = ldm_sdf.sample(m, sch, n, steps=steps, dtype="fp32",
                       x_T=torch.from_numpy(gd["x_T"])[:n], noise=noise[:, :n].contiguous(),
                       device=dev, use_graph=path == "graph").cpu().double()
    err = float((x - torch.from_numpy(gd["traj"][-1])[:n]).abs().max())
    assert err <= 1e-4, err


def test_unet_sampler_graph_equals_eager_bf16(dev):
    import ldm_sdf
    m = ldm_sdf.UNet1DDenoiser(seed=2468)
    sch = ldm_sdf.DDPMSchedule()
    g = torch.Generator(device=dev).manual_seed(0)
    xT = torch.randn(4, 1024, device=dev, generator=g)
    noise = torch.randn(1000, 4, 1024, device=dev, generator=g)
    a = ldm_sdf.Sampler(m, sch, 4, steps=25, dtype="bf16", device=dev, use_graph=False,
                        persistent=False)
    b = ldm_sdf.Sampler(m, sch, 4, steps=25, dtype="bf16", device=dev, use_graph=True,
                        persistent=False)
    ra = a.run(xT, noise).clone()
    rb = b.run(xT, noise).clone()
    assert torch.equal(ra, rb)
    assert bool(torch.isfinite(ra).all())


def test_unet_has_no_persistent_loop(dev):
    """The round-3 one-launch loop was retired in round 4 (0.53x the graph after the direct conv
    staging): asking for a persistent UNet sampler fails loudly."""
    import ldm_sdf
    m = ldm_sdf.UNet1DDenoiser(seed=2468)
    with pytest.raises(RuntimeError, match="no persistent"):
        ldm_sdf.Sampler(m, ldm_sdf.DDPMSchedule(), 1, steps=5, dtype="bf16", device=dev,
                        persistent=True)
