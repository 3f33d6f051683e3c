"""Sweep of the auto-decoder's weight-gradient tile (autodecoder.WGRAD_TILE; 64 x 16384 samples,
bf16): the tiles in AB_TILES, alternating in one process, AD_STEPS steps per timing after one
warm-up step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import autodecoder  # noqa: E402

S, P, steps = 64, 16384, int(os.environ.get("AD_STEPS", "3"))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(7)
radii = 0.3 + 0.5 * torch.rand(S, device=dev, generator=g)
d = torch.randn(S, P, 3, device=dev, generator=g)
d = d / d.norm(dim=2, keepdim=True)
xyz = d * (radii[:, None] + 0.05 * torch.randn(S, P, device=dev, generator=g))[..., None]
sdf = xyz.norm(dim=2) - radii[:, None]
tiles = [int(t) for t in os.environ.get("AB_TILES", "3,6,14,16,17,23,26").split(",")]
base = autodecoder.WGRAD_TILE


dec = ldm_sdf.SDFDecoder(seed=1234)
dec.weights[8] = dec.weights[8] * 0.01
st = ldm_sdf.train_autodecoder(dec, xyz, sdf, steps=1, shapes_per_batch=S, samples_per_shape=P,
                               dtype="bf16", generator=g)
for rep in range(3):
    for t in tiles:
        name = f"wgrad tile {t}"
        autodecoder.WGRAD_TILE = t
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = ldm_sdf.train_autodecoder(dec, xyz, sdf, steps=steps, shapes_per_batch=S,
                                       samples_per_shape=P, dtype="bf16", generator=g, state=st)
        torch.cuda.synchronize()
        print(f"{name:26s} {(time.perf_counter() - t0) / steps * 1e3:.2f} ms/step", flush=True)
autodecoder.WGRAD_TILE = base
