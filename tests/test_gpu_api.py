"""Small API pieces on the MI355X: the library's latent-RMS reduction behind dtype="auto"
(``ldm_latent_rms_max``, csrc/decoder.hip) against torch, and the "auto" choice it drives."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ldm_sdf
    ldm_sdf.load_library()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("B,L", [(1, 256), (8, 256), (64, 256), (3, 1024), (1000, 7)])
def test_latent_rms_max_matches_torch(dev, B, L):
    from ldm_sdf import ops
    g = torch.Generator().manual_seed(B * 31 + L)
    z = (torch.randn(B, L, generator=g) * torch.rand(B, 1, generator=g) * 2).to(dev)
    want = float(z.double().pow(2).mean(dim=1).sqrt().max())
    got = ops.latent_rms_max(z)
    assert abs(got - want) <= 1e-6 * want, (got, want)


def test_auto_dtype_on_device(dev):
    import ldm_sdf
    from ldm_sdf import api
    api.clear_auto_cache()
    z = torch.ones(4, 256, device=dev)
    for scale, want in ((0.1, "bf16"), (0.5, "fp16"), (2.0, "fp32")):
        assert ldm_sdf.resolve_decode_dtype("auto", z * scale) == want
