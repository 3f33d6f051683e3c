"""Minimal config-2 training workload for profilers: DDPM training of the MLP denoiser on 1000
synthetic latents, batch 1000, bf16 (matrix-core GEMMs)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402

steps = int(os.environ.get("TRAIN_STEPS", "20"))
dtype = os.environ.get("TRAIN_DTYPE", "bf16")
dev = torch.device("cuda", 0)
den = ldm_sdf.MLPDenoiser(seed=4321)
sch = ldm_sdf.DDPMSchedule()
lat = torch.randn(1000, 256, device=dev) * 0.5
st = ldm_sdf.train(den, sch, lat, steps=3, batch=1000, dtype=dtype)
torch.cuda.synchronize()
t0 = time.perf_counter()
st = ldm_sdf.train(den, sch, lat, steps=steps, batch=1000, dtype=dtype, state=st)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print(f"train {dtype}: {1 / dt:.1f} steps/s ({dt * 1e3:.3f} ms/step), loss {st.losses[-1]:.4f}")
