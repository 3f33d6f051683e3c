"""The BASELINE.json configs at their own sizes, on the MI355X, against the oracle.

* config 2 -- the bf16 DDPM training step at batch 1000 on 1k latents (`BASELINE.json:8`);
* config 3 -- 1000-step bf16 sampling of 8 latents -> decode of a 128^3 grid in the dtype
  dtype="auto" picks for the latents' scale (`BASELINE.json:9`): the bench's config 3 (a
  bounded denoiser, sampled latents at RMS ~0.45) decodes in FP16 -- that path is
  test_gpu_ddpm.py::test_config3_bounded_sample8_then_decode128_unscaled; the test here
  samples with the untrained denoiser (latents ~1e8, "auto" -> fp32) and decodes the codes
  rescaled to RMS 0.1, where "auto" picks bf16;
* config 5 -- fp16 decode of a 512^3 grid with the widen-skip decoder, L = 1024
  (`BASELINE.json:11`; the UNet sampling half is pinned in test_gpu_unet.py).

* config 4 -- the bench's own decode inputs at their own size: 64 shapes x 256^3, bf16
  (`BASELINE.json:10`; its 8-GPU z-slab reassembly is covered by the gloo tests,
  test_dist_gloo.py / test_bench_gloo.py);
Full volumes are checked on random point subsets (the fp64 oracle on 134 M points would take
hours); tolerances are SURVEY.md §8(c)'s.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = {"fp32": 2e-6, "fp16": 2e-3, "bf16": 1e-2}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ldm_sdf
    ldm_sdf.load_library()
    return torch.device("cuda", 0)


def _denoiser():
    from ldm_sdf import MLPDenoiser
    from oracle import ref_cpu as R
    p = R.make_denoiser_params(seed=4321)
    params = {n: getattr(p, n) for n in ("Wt1", "bt1", "Wt2", "bt2", "Win", "bin", "Wout", "bout")}
    for k in range(p.n_blocks):
        params[f"Wblk{k}"], params[f"bblk{k}"] = p.Wblk[k], p.bblk[k]
    return MLPDenoiser(params=params), p


def test_config2_train_step_bf16_batch1000(dev):
    """Config 2's step: 1000 latents, batch 1000, bf16 weights + matrix-core GEMMs, vs the fp64
    oracle's autograd on the same (x0, t, eps): loss within 1e-3 relative, every gradient
    (whole tensor) at cosine >= 0.999 and norm within 2 %."""
    import ldm_sdf
    from oracle import ref_cpu as R
    model, p = _denoiser()
    model.to_device(dev)
    g = torch.Generator().manual_seed(2024)
    x0 = torch.randn(1000, 256, generator=g) * 0.5
    t = torch.randint(0, 1000, (1000,), generator=g, dtype=torch.int32)
    eps = torch.randn(1000, 256, generator=g)
    loss, grads = ldm_sdf.train_step(model, ldm_sdf.DDPMSchedule(), x0.to(dev), t.to(dev),
                                     eps.to(dev), dtype="bf16")
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128)).double()
    torch.set_num_threads(min(16, torch.get_num_threads()))
    want_loss, want = R.train_step_grads(p, R.ddpm_tables(), emb, x0.double(), eps.double(),
                                         t.long())
    assert abs(float(loss) - float(want_loss)) / float(want_loss) < 1e-3
    for k, v in grads.items():
        got = v.cpu().double().flatten()
        w = want[k].flatten()
        cos = float(got @ w / (got.norm() * w.norm() + 1e-30))
        rel = abs(float(got.norm()) - float(w.norm())) / float(w.norm())
        print(f"config2 grad {k}: cos {cos:.6f} norm rel {rel:.2e}")
        assert cos >= 0.999, (k, cos)
        assert rel <= 2e-2, (k, rel)


def test_config3_sample8_then_decode128(dev):
    """Config 3 end to end with the untrained synthetic denoiser: sample(8) (1000 bf16 steps,
    the default persistent loop) -> decode(128^3) of the rescaled codes, which dtype="auto"
    decodes in bf16 (the bench's config 3, on bounded latents, decodes in fp16: see the end of
    this docstring).  The latents are checked against the
    fp64 oracle on the bf16-rounded weights (relative 2e-5, see test_gpu_ddpm.py).  That
    denoiser drives the latents to ~1e8, where every SDF saturates at +-1, so dtype="auto"
    refuses the 16-bit kernels there (fp32, api.FP16_MAX_LATENT_RMS) and the volume is checked
    for the sampled codes brought to the decoder's operating range (each rescaled to RMS 0.1,
    the synthetic-latent scale of SURVEY.md §8(d)) on 600 random points per shape against the
    fp64 oracle decoder.  The fp16 "auto" path on latents AS SAMPLED (bounded regime, not
    saturated) is test_gpu_ddpm.py::test_config3_bounded_sample8_then_decode128_unscaled."""
    import ldm_sdf
    from oracle import ref_cpu as R
    from tests.test_gpu_ddpm import _bf16_rounded_params, _oracle_sample
    model, p = _denoiser()
    gen = torch.Generator().manual_seed(33)
    xT = torch.randn(8, 256, generator=gen)
    noise = torch.randn(1000, 8, 256, generator=gen)
    lat = ldm_sdf.sample(model, ldm_sdf.DDPMSchedule(), 8, dtype="bf16", x_T=xT, noise=noise,
                         device=dev)
    want_lat = _oracle_sample(_bf16_rounded_params(p), xT, noise, 1000)
    rel = float((lat.cpu().double() - want_lat).abs().max()) / float(want_lat.abs().max())
    assert rel <= 2e-5, rel
    pd = R.make_decoder_params(seed=1234)
    dec = ldm_sdf.SDFDecoder(256, weights=pd.weights, biases=pd.biases)
    N = 128
    grid = torch.from_numpy(R.grid_coords_np(N)).double()
    assert ldm_sdf.resolve_decode_dtype("auto", lat) == "fp32"
    scaled = lat / lat.pow(2).mean(dim=1, keepdim=True).sqrt() * 0.1
    assert ldm_sdf.resolve_decode_dtype("auto", scaled) == "bf16"
    for z in (scaled,):
        vol = ldm_sdf.decode(dec, z, N)
        assert vol.shape == (8, N, N, N) and bool(torch.isfinite(vol).all())
        idx = torch.randint(0, N ** 3, (8, 600), generator=gen)
        got = vol.reshape(8, -1)[torch.arange(8)[:, None], idx.to(dev)].cpu().double()
        zc = z.cpu().double()
        for b in range(8):
            want = R.decoder_forward(pd, zc[b:b + 1], grid[idx[b]])[0]
            err = float((got[b] - want).abs().max())
            assert err <= TOL["bf16"], (b, err)


def _grid_xyz(idx: np.ndarray, N: int) -> torch.Tensor:
    """A1's coordinates of flat grid indices (z slowest), without building the whole grid."""
    from oracle import ref_cpu as R
    line = (np.arange(N, dtype=np.float32) * R.grid_voxel_size(N)).astype(np.float32) \
        + np.float32(-1.0)
    return torch.from_numpy(np.stack([line[idx % N], line[(idx // N) % N], line[idx // (N * N)]],
                                     axis=1).astype(np.float32)).double()


def test_config4_decode_b64_256_bench_inputs(dev):
    """Config 4 at its own size with the bench's exact inputs (bench.py main: decoder
    SDFDecoder(256, seed=1234), latents = randn(64, 256, device generator seed 0) * 0.1, bf16,
    256^3): 256 random points per shape plus every shape's 8 corners against the fp64 oracle at
    the bf16 bound; and one shape decoded alone is bitwise the same shape inside the batch."""
    import ldm_sdf
    from oracle import ref_cpu as R
    B, N = 64, 256
    dec = ldm_sdf.SDFDecoder(256, seed=1234)
    p = R.make_decoder_params(seed=1234)
    for l in range(9):       # the bench's decoder IS the oracle's seed-1234 decoder
        assert torch.equal(dec.weights[l], p.weights[l].float()), l
    gen = torch.Generator(device=dev).manual_seed(0)
    lat = torch.randn(B, 256, device=dev, generator=gen) * 0.1
    vol = ldm_sdf.decode(dec, lat, N, dtype="bf16")
    assert vol.shape == (B, N, N, N)
    g = torch.Generator().manual_seed(404)
    corners = torch.tensor([k * N * N + j * N + i for k in (0, N - 1) for j in (0, N - 1)
                            for i in (0, N - 1)])
    idx = torch.cat([torch.randint(0, N ** 3, (B, 256), generator=g),
                     corners[None].expand(B, -1)], dim=1)
    got = vol.reshape(B, -1)[torch.arange(B, device=dev)[:, None], idx.to(dev)].cpu().double()
    zc = lat.cpu().double()
    torch.set_num_threads(min(16, torch.get_num_threads()))
    worst = worst_lo = 0.0
    for b in range(B):
        xyz = _grid_xyz(idx[b].numpy(), N)
        want = R.decoder_forward(p, zc[b:b + 1], xyz)[0]
        err = float((got[b] - want).abs().max())
        worst = max(worst, err)
        assert err <= TOL["bf16"], (b, err)
        # and the bf16 precision contract itself (oracle decoder_forward_lowp), far tighter
        d_lo = (got[b] - R.decoder_forward_lowp(p, zc[b:b + 1], xyz)[0]).abs()
        e_lo = float(d_lo.max())
        worst_lo = max(worst_lo, e_lo)
        assert float(d_lo.median()) <= 2e-5, b    # fp32 summation order
        assert e_lo <= 3e-3, (b, e_lo)            # + rare 16-bit rounding-tie flips
    print(f"config4 64 x 256^3 bf16: max abs err {worst:.3e} vs fp64, {worst_lo:.3e} vs the "
          f"bf16-contract oracle, over {idx.numel()} points")
    assert bool(torch.isfinite(vol[:, 0]).all()) and bool(torch.isfinite(vol[:, -1]).all())
    one = ldm_sdf.decode(dec, lat[37:38], N, dtype="bf16")
    assert torch.equal(one[0], vol[37])


def test_config5_decode_512_fp16_widen_skip(dev):
    """Config 5's decode: 1 latent (L = 1024, widen-skip decoder), fp16 matrix cores, the full
    512^3 grid (134 M queries, the size the bench runs), 2000 random points vs the fp64 oracle
    at the fp16 tolerance, plus the grid's 8 corners and a full z-slice's finiteness."""
    import ldm_sdf
    from oracle import ref_cpu as R
    p = R.make_decoder_params(L=1024, widen_skip=True, seed=1235)
    dec = ldm_sdf.SDFDecoder(1024, weights=p.weights, biases=p.biases)
    assert dec.widen_skip and dec.skip_width == 512
    g = torch.Generator().manual_seed(55)
    z = torch.randn(1, 1024, generator=g) * 0.1
    N = 512
    vol = ldm_sdf.decode(dec, z.to(dev), N, dtype="fp16")
    assert vol.shape == (1, N, N, N)
    assert bool(torch.isfinite(vol[0, 0]).all()) and bool(torch.isfinite(vol[0, -1]).all())
    idx = torch.randint(0, N ** 3, (2000,), generator=g)
    corners = torch.tensor([k * N * N + j * N + i for k in (0, N - 1) for j in (0, N - 1)
                            for i in (0, N - 1)])
    idx = torch.cat([idx, corners])
    got = vol.reshape(-1)[idx.to(dev)].cpu().double()
    want = R.decoder_forward(p, z.double(), _grid_xyz(idx.numpy(), N))[0]
    err = float((got - want).abs().max())
    print(f"config5 512^3 fp16: max abs err {err:.3e} on {idx.numel()} points")
    assert err <= TOL["fp16"], err
