"""C20 DeepSDF data/checkpoint formats on the CPU: .npz SDF samples (NaN removal, half/half
draws), the split-JSON layout, and model / latent-code checkpoint round trips through the
safe loaders.  Fixtures are synthetic files written here (the reference ships none)."""
import json
import os

import numpy as np
import pytest
import torch

from ldm_sdf import data, SDFDecoder


def _write_npz(path, n_pos, n_neg, seed, nan_rows=0):
    r = np.random.default_rng(seed)
    pos = np.concatenate([r.uniform(-1, 1, (n_pos, 3)), r.uniform(0, 0.1, (n_pos, 1))], 1)
    neg = np.concatenate([r.uniform(-1, 1, (n_neg, 3)), -r.uniform(0, 0.1, (n_neg, 1))], 1)
    pos[:nan_rows, 3] = np.nan
    os.makedirs(os.path.dirname(path), exist_ok=True)
    np.savez(path, pos=pos.astype(np.float32), neg=neg.astype(np.float32))
    return pos, neg


def test_load_drops_nan_rows(tmp_path):
    p = str(tmp_path / "a.npz")
    pos, neg = _write_npz(p, 50, 40, 0, nan_rows=7)
    tp, tn = data.load_sdf_samples(p)
    assert tp.shape == (43, 4) and tn.shape == (40, 4)
    assert torch.equal(tp, torch.from_numpy(pos[7:].astype(np.float32)))
    assert not torch.isnan(tp).any()


def test_load_rejects_bad_files(tmp_path):
    p = str(tmp_path / "b.npz")
    np.savez(p, pos=np.zeros((3, 3), np.float32), neg=np.zeros((3, 4), np.float32))
    with pytest.raises(ValueError):
        data.load_sdf_samples(p)
    q = str(tmp_path / "c.npz")
    np.savez(q, samples=np.zeros((3, 4), np.float32))
    with pytest.raises(ValueError):
        data.load_sdf_samples(q)


def test_unpack_half_and_half():
    pos = torch.cat([torch.rand(10, 3), torch.full((10, 1), 0.05)], 1)
    neg = torch.cat([torch.rand(6, 3), torch.full((6, 1), -0.05)], 1)
    g = torch.Generator().manual_seed(0)
    s = data.unpack_sdf_samples(pos, neg, 9, g)
    assert s.shape == (9, 4)
    assert (s[:4, 3] > 0).all() and (s[4:, 3] < 0).all()       # 4 positives, then 5 negatives
    for row in s[:4]:
        assert any(torch.equal(row, q) for q in pos)


def test_split_layout_and_draw(tmp_path):
    split = {"ShapeNetV2": {"02691156": ["i0", "i1"], "03001627": ["i2"]}}
    for k, (c, i) in enumerate([("02691156", "i0"), ("02691156", "i1"), ("03001627", "i2")]):
        _write_npz(str(tmp_path / "SdfSamples" / "ShapeNetV2" / c / (i + ".npz")), 20, 30, k)
    (tmp_path / "split.json").write_text(json.dumps(split))
    ds = data.SdfSampleSet.from_split(str(tmp_path), json.loads((tmp_path / "split.json").read_text()))
    assert len(ds) == 3 and ds.paths[2].endswith(os.path.join("03001627", "i2.npz"))
    xyz, sdf = ds.draw(16, generator=torch.Generator().manual_seed(1))
    assert xyz.shape == (3, 16, 3) and sdf.shape == (3, 16)
    assert (sdf[:, :8] >= 0).all() and (sdf[:, 8:] <= 0).all()


def test_model_checkpoint_round_trip(tmp_path):
    dec = SDFDecoder(seed=3)
    p = str(tmp_path / "ModelParameters" / "latest.pth")
    data.save_model(p, dec, epoch=17)
    back, ep = data.load_model(p, latent_dim=256)
    assert ep == 17
    for a, b in zip(dec.weights + dec.biases, back.weights + back.biases):
        assert torch.equal(a, b)
    # DataParallel-style prefixes and weight-norm pairs (DeepSDF's saved form)
    sd = {}
    for l, (w, b) in enumerate(zip(dec.weights, dec.biases)):
        g = w.norm(dim=1, keepdim=True)
        sd[f"module.lin{l}.weight_g"], sd[f"module.lin{l}.weight_v"] = g, w * 2.0
        sd[f"module.lin{l}.bias"] = b
    q = str(tmp_path / "wn.pth")
    torch.save({"epoch": 2, "model_state_dict": sd}, q)
    wn, _ = data.load_model(q, latent_dim=256)
    for a, b in zip(dec.weights, wn.weights):
        assert torch.allclose(a, b, atol=1e-6)


def test_latent_checkpoint_round_trip(tmp_path):
    lat = torch.randn(5, 256)
    p = str(tmp_path / "LatentCodes" / "100.pth")
    data.save_latent_codes(p, lat, epoch=100)
    back, ep = data.load_latent_codes(p)
    assert ep == 100 and torch.equal(back, lat)
    q = str(tmp_path / "old.pth")                    # older DeepSDF layout [n, 1, L]
    torch.save({"epoch": 3, "latent_codes": lat[:, None, :]}, q)
    back2, _ = data.load_latent_codes(q)
    assert torch.equal(back2, lat)
