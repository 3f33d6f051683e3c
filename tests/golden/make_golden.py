"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference (/root/reference) ships no code and no fixtures, so these vectors are the
oracle's own outputs (fp64 unless noted) on fixed seeds: they pin the GPU path to the oracle
on the GPU box, and ``tests/test_golden.py`` re-derives them on the CPU so that the oracle
and the fixtures cannot drift apart silently.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import ref_cpu as R  # noqa: E402
from oracle import ref_unet as U  # noqa: E402
from oracle import ref_mc as MC  # noqa: E402

DEC_SEED, LAT_SEED, PTS_SEED = 1234, 0, 7
DEN_SEED, SAMPLE_SEED = 4321, 11
UNET_SEED = 2468


def decoder_case():
    p = R.make_decoder_params(seed=DEC_SEED)
    z = (torch.randn(2, 256, generator=torch.Generator().manual_seed(LAT_SEED),
                     dtype=torch.float64) * 0.1)
    N = 32
    grid = R.grid_coords_np(N)
    sdf_grid = R.decoder_forward(p, z, torch.from_numpy(grid).double()).numpy()
    g = torch.Generator().manual_seed(PTS_SEED)
    pts = (torch.rand(2, 1000, 3, generator=g, dtype=torch.float64) * 2.2 - 1.1).float()
    sdf_pts = R.decoder_forward(p, z, pts.double()).numpy()
    return dict(z=z.float().numpy(), N=np.int32(N), grid=grid, sdf_grid=sdf_grid.astype(np.float64),
                pts=pts.numpy(), sdf_pts=sdf_pts)


def widen_case():
    p = R.make_decoder_params(L=1024, widen_skip=True, seed=DEC_SEED + 1)
    z = (torch.randn(1, 1024, generator=torch.Generator().manual_seed(LAT_SEED + 1),
                     dtype=torch.float64) * 0.1)
    g = torch.Generator().manual_seed(PTS_SEED + 1)
    pts = (torch.rand(1, 777, 3, generator=g, dtype=torch.float64) * 2 - 1).float()
    return dict(z=z.float().numpy(), pts=pts.numpy(),
                sdf_pts=R.decoder_forward(p, z, pts.double()).numpy())


def sampling_case(steps=20, B=4):
    p = R.make_denoiser_params(seed=DEN_SEED)
    tab = R.ddpm_tables(1000)
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128)).double()
    g = torch.Generator().manual_seed(SAMPLE_SEED)
    x_T = torch.randn(B, 256, generator=g, dtype=torch.float32)
    noise = torch.zeros(1000, B, 256, dtype=torch.float32)
    noise[1000 - steps:] = torch.randn(steps, B, 256, generator=g, dtype=torch.float32)
    x, traj = R.sample_loop(p, tab, emb, x_T.double(), noise.double(), steps=steps,
                            return_traj=True)
    eps0 = R.denoiser_forward(p, x_T.double(), torch.full((B,), 999), emb)
    return dict(x_T=x_T.numpy(), noise_tail=noise[1000 - steps:].numpy(),
                traj=torch.stack(traj).numpy(), eps_t999=eps0.numpy(), steps=np.int32(steps))


def train_case(B=64):
    p = R.make_denoiser_params(seed=DEN_SEED)
    tab = R.ddpm_tables(1000)
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128)).double()
    g = torch.Generator().manual_seed(SAMPLE_SEED + 1)
    x0 = torch.randn(B, 256, generator=g, dtype=torch.float32) * 0.5
    eps = torch.randn(B, 256, generator=g, dtype=torch.float32)
    t = torch.randint(0, 1000, (B,), generator=g)
    loss, grads = R.train_step_grads(p, tab, emb, x0.double(), eps.double(), t)
    out = dict(x0=x0.numpy(), eps=eps.numpy(), t=t.numpy().astype(np.int32),
               loss=np.float64(loss))
    for k, v in grads.items():
        out["g_" + k] = (v if k.startswith("b") else v[:8]).numpy()   # bias grads, W[:8]
        out["gnorm_" + k] = np.float64(v.norm())
    return out


def unet_case(steps=10, B=2):
    """C17: 1D-UNet (D=1024, C=(32,64,128)) eps at mixed t and a 10-step trajectory (fp64)."""
    up = U.make_unet_params(seed=UNET_SEED)
    tab = R.ddpm_tables(1000)
    emb = torch.from_numpy(R.timestep_embedding_table(1000, 128)).double()
    g = torch.Generator().manual_seed(SAMPLE_SEED + 2)
    x_T = torch.randn(B, 1024, generator=g, dtype=torch.float32)
    noise = torch.zeros(1000, B, 1024, dtype=torch.float32)
    noise[1000 - steps:] = torch.randn(steps, B, 1024, generator=g, dtype=torch.float32)
    t_mixed = torch.tensor([999, 5][:B])
    eps_mixed = U.unet_forward(up, x_T.double(), t_mixed, emb)
    x = x_T.double()
    traj = [x]
    for t in range(999, 999 - steps, -1):
        eps = U.unet_forward(up, x, torch.full((B,), t), emb)
        x = R.ddpm_step(tab, x, eps, noise[t].double(), t)
        traj.append(x)
    return dict(x_T=x_T.numpy(), noise_tail=noise[1000 - steps:].numpy(),
                traj=torch.stack(traj).numpy(), t_mixed=t_mixed.numpy().astype(np.int32),
                eps_mixed=eps_mixed.numpy(), steps=np.int32(steps))


def mc_case(N=24):
    """C18: marching cubes of a sphere-plus-noise volume (every ambiguous case occurs)."""
    rng = np.random.default_rng(5)
    c = MC._coords(N)
    z, y, x = np.meshgrid(c, c, c, indexing="ij")
    vol = (np.sqrt(x * x + y * y + z * z) - 0.6 + 0.15 * rng.standard_normal((N, N, N)))
    vol = vol.astype(np.float32)
    verts, faces = MC.marching_cubes(vol)
    return dict(vol=vol, verts=verts, faces=faces)


CASES = {"decoder_small": decoder_case, "decoder_widen": widen_case,
         "sampling_20": sampling_case, "train_step": train_case, "unet_10": unet_case,
         "mc_24": mc_case}


def main():
    only = sys.argv[1:]
    for name, fn in CASES.items():
        if only and name not in only:
            continue
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **fn())
        print(f"wrote {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
