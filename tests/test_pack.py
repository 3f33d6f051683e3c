"""Host packing (C4) checked on the CPU: the fragment-level emulation of the MFMA kernel
(tests/mfma_emulator.py) fed with ldm_sdf.pack output must reproduce the oracle."""
import numpy as np
import pytest
import torch

from ldm_sdf import pack
from oracle import ref_cpu as R
from tests.mfma_emulator import emulate_split


def test_perm_is_accumulator_row_order():
    # element j of lane half h of k-step 2i+s is accumulator row 16s + 8(j>>2) + 4h + (j&3)
    for h in range(2):
        for j in range(8):
            assert pack.PERM[8 * h + j] == 8 * (j >> 2) + 4 * h + (j & 3)
    assert sorted(pack.PERM.tolist()) == list(range(16))


def test_w_last_permutation_roundtrip():
    w = torch.arange(512, dtype=torch.float32)
    wl = pack.permute_w_last_split(w)
    assert sorted(wl.tolist()) == list(range(512))


def test_fp32_blob_size():
    p = R.make_decoder_params()
    blob = pack.pack_f32_blob(pack.canonical_pieces(p.weights, p.biases, 256))
    # W1..W7 (5 of 512x512, W3 512x253, W4 253x512) + b1,b2,b3(253),b4(zeros),b5,b6,b7
    n = 5 * 512 * 512 + 2 * 512 * 253 + 6 * 512 + 253
    assert blob.numel() == n


@pytest.mark.parametrize("dtype,tol", [("bf16", 1e-2), ("fp16", 2e-3)])
def test_emulated_kernel_matches_oracle(dtype, tol):
    """The split kernel's dataflow replayed from the packed blob against the fp64 decoder at
    SURVEY §8(c)'s bounds (bf16 1e-2, fp16 2e-3) at the synthetic latent scale."""
    p = R.make_decoder_params(seed=1234)
    g = torch.Generator().manual_seed(0)
    z = torch.randn(2, 256, generator=g, dtype=torch.float64) * 0.1
    xyz = (torch.rand(2, 128, 3, generator=g, dtype=torch.float64) * 2 - 1).float()
    want = R.decoder_forward(p, z, xyz.double()).numpy()
    beta = R.latent_fold(p, z).float().numpy()
    packed = pack.pack_decoder(p.weights, p.biases, 256, dtype, layout="split")
    err = np.abs(emulate_split(packed, beta, xyz.numpy(), dtype) - want).max()
    assert err < tol, err
    # and it is not trivially close: outputs vary
    assert want.std() > 0.005


def test_emulated_widen_skip_fp16():
    p = R.make_decoder_params(L=1024, widen_skip=True, seed=5)
    g = torch.Generator().manual_seed(1)
    z = torch.randn(1, 1024, generator=g, dtype=torch.float64) * 0.1
    xyz = (torch.rand(1, 128, 3, generator=g, dtype=torch.float64) * 2 - 1).float()
    want = R.decoder_forward(p, z, xyz.double()).numpy()
    beta = R.latent_fold(p, z).float().numpy()
    packed = pack.pack_decoder(p.weights, p.biases, 1024, "fp16", layout="split")
    assert np.abs(emulate_split(packed, beta, xyz.numpy(), "fp16") - want).max() < 2e-3


@pytest.mark.parametrize("dtype,scale", [("bf16", 0.1), ("bf16", 0.5), ("fp16", 0.5)])
def test_lowp_oracle_matches_emulated_kernel(dtype, scale):
    """oracle decoder_forward_lowp (the 16-bit precision contract in fp64) against the
    fragment-level kernel emulation (fp64 accumulation too): they agree far inside the 16-bit
    rounding error itself, including at large latents where that error reaches 1e-2 -- which
    is what lets the GPU tests pin the 16-bit kernels tightly at any latent scale."""
    p = R.make_decoder_params(seed=1234)
    g = torch.Generator().manual_seed(3)
    z = torch.randn(2, 256, generator=g, dtype=torch.float64) * scale
    xyz = (torch.rand(2, 128, 3, generator=g, dtype=torch.float64) * 2 - 1).float()
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    lowp = R.decoder_forward_lowp(p, z, xyz.double(), dt).numpy()
    beta = R.latent_fold(p, z).float().numpy()
    packed = pack.pack_decoder(p.weights, p.biases, 256, dtype, layout="split")
    emu = emulate_split(packed, beta, xyz.numpy(), dtype)
    full = R.decoder_forward(p, z, xyz.double()).numpy()
    d = np.abs(emu - lowp)
    err, med = d.max(), np.median(d)
    rnd = np.abs(full - lowp).max()
    print(f"{dtype} z*{scale}: |emu - lowp| max {err:.2e} median {med:.2e}, "
          f"rounding error itself {rnd:.2e}")
    # identical arithmetic up to summation order: most points agree to ~1e-8; a point whose
    # pre-activation sits at a 16-bit rounding tie may round the other way (one ulp of one
    # activation: <= ~5e-4 seen at z*0.5)
    assert med < 1e-6, med
    assert err < 1e-3, err


def test_removed_layouts_raise():
    p = R.make_decoder_params(seed=1234)
    for lay in ("pass8", "quarter"):
        with pytest.raises(ValueError):
            pack.pack_decoder(p.weights, p.biases, 256, "bf16", layout=lay)


@pytest.mark.parametrize("dtype,sw", [("bf16", 253), ("fp16", 253), ("fp16", 512)])
def test_split_layout_emulation_matches_lowp_oracle(dtype, sw):
    """The split layout (csrc/decoder_fs.hip) replayed on the CPU from the packed blob: same
    numbers as the 16-bit precision-contract oracle (fp64 sums), for DeepSDF (skip 253) and the
    widen-skip decoder (L = 1024); the stream length matches the kernel's constant."""
    from tests.mfma_emulator import emulate_split
    L = 256 if sw == 253 else 1024
    p = R.make_decoder_params(L=L, widen_skip=(sw == 512), seed=1234)
    g = torch.Generator().manual_seed(5)
    z = torch.randn(2, L, generator=g, dtype=torch.float64) * 0.1
    xyz = (torch.rand(2, 128, 3, generator=g, dtype=torch.float64) * 2 - 1).float()
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dtype]
    packed = pack.pack_decoder(p.weights, p.biases, L, dtype, layout="split")
    assert packed["n_stages"] == (384 if sw == 253 else 448)
    beta = R.latent_fold(p, z).float().numpy()
    emu = emulate_split(packed, beta, xyz.numpy(), dtype)
    lowp = R.decoder_forward_lowp(p, z, xyz.double(), dt).numpy()
    d = np.abs(emu - lowp)
    assert np.median(d) < 1e-6 and d.max() < 1e-3, (np.median(d), d.max())
