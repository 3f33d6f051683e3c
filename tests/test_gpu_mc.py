"""C18 parity on the MI355X: ldm_mc_* (classify / scan / emit) equals the CPU oracle
(oracle/ref_mc.py) BIT FOR BIT -- vertex positions (fp32), vertex order, face triples and face
order -- on analytic SDFs, white noise, ragged sizes (N not a multiple of the 4096-point scan
chunk), empty volumes, a non-zero level, and end to end on a decoded DeepSDF volume."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ldm_sdf
    ldm_sdf.load_library()
    return torch.device("cuda", 0)


def _grid(N):
    from oracle import ref_mc as M
    c = M._coords(N)
    return np.meshgrid(c, c, c, indexing="ij")


def _check(dev, vol, level=0.0, bbox=(-1.0, 1.0)):
    import ldm_sdf
    from oracle import ref_mc as M
    v, f = ldm_sdf.marching_cubes(torch.from_numpy(vol).to(dev), level, bbox)
    vo, fo = M.marching_cubes(vol, level, bbox)
    v, f = v.cpu().numpy(), f.cpu().numpy()
    assert v.shape == vo.shape and f.shape == fo.shape
    assert np.array_equal(v.view(np.uint32), vo.view(np.uint32)), "vertex bits differ"
    assert np.array_equal(f, fo), "faces differ"
    return v, f


@pytest.mark.parametrize("N", [2, 3, 17, 64, 129])
def test_sphere_bit_exact(dev, N):
    z, y, x = _grid(N)
    _check(dev, (np.sqrt(x * x + y * y + z * z) - 0.55).astype(np.float32))


@pytest.mark.parametrize("seed,N", [(0, 33), (1, 48), (2, 65)])
def test_noise_bit_exact(dev, seed, N):
    vol = np.random.default_rng(seed).standard_normal((N, N, N)).astype(np.float32)
    _check(dev, vol)
    _check(dev, vol, level=0.37, bbox=(-0.5, 1.5))


def test_torus_and_empty(dev):
    z, y, x = _grid(80)
    tor = (np.sqrt((np.sqrt(x * x + y * y) - 0.5) ** 2 + z * z) - 0.2).astype(np.float32)
    _check(dev, tor)
    v, f = _check(dev, np.ones((40, 40, 40), np.float32))
    assert len(v) == 0 and len(f) == 0


def test_golden(dev):
    g = dict(np.load(os.path.join(GOLD, "mc_24.npz")))
    import ldm_sdf
    v, f = ldm_sdf.marching_cubes(torch.from_numpy(g["vol"]).to(dev))
    assert np.array_equal(v.cpu().numpy(), g["verts"]) and np.array_equal(f.cpu().numpy(), g["faces"])


def test_decode_then_mesh_256(dev):
    """Config-4 consumer: decode one shape at 256^3 (bf16) and mesh it on the GPU; the mesh
    equals the oracle's mesh of the same volume, and is a closed surface when the volume's
    border is outside."""
    import ldm_sdf
    dec = ldm_sdf.SDFDecoder(256, seed=1234)
    z = torch.randn(1, 256, device=dev, generator=torch.Generator(device=dev).manual_seed(0)) * 0.1
    vol = ldm_sdf.decode(dec, z, 256, dtype="bf16")[0]
    vol_np = vol.cpu().numpy()
    v, f = _check(dev, vol_np)
    assert len(f) > 0


def test_batch_meshing(dev):
    import ldm_sdf
    z, y, x = _grid(32)
    vols = np.stack([(np.sqrt(x * x + y * y + z * z) - r).astype(np.float32) for r in (0.3, 0.6)])
    out = ldm_sdf.marching_cubes_batch(torch.from_numpy(vols).to(dev))
    assert [b for b, _, _ in out] == [0, 1]
    from oracle import ref_mc as M
    for b, v, f in out:
        vo, fo = M.marching_cubes(vols[b])
        assert np.array_equal(v.cpu().numpy(), vo) and np.array_equal(f.cpu().numpy(), fo)
