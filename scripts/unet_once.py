"""Minimal UNet sampling workload for profilers: graph-captured reverse steps of B latents."""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402

B = int(os.environ.get("UNET_B", "1"))
STEPS = int(os.environ.get("UNET_STEPS", "1000"))
dtype = os.environ.get("UNET_DTYPE", "bf16")
dev = torch.device("cuda", 0)
m = ldm_sdf.UNet1DDenoiser(seed=2468)
sch = ldm_sdf.DDPMSchedule()
s = ldm_sdf.Sampler(m, sch, B, steps=STEPS, dtype=dtype, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
xT = torch.randn(B, 1024, device=dev, generator=g)
noise = torch.randn(1000, B, 1024, device=dev, generator=g)
out = s.run(xT, noise)
h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:16]
for _ in range(int(os.environ.get("UNET_REPS", "1"))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.run(xT, noise)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"lib {os.path.basename(os.environ.get('LDM_SDF_LIB', 'libldm_sdf.so'))} B={B} "
          f"steps={STEPS} {dtype}: {STEPS / dt:.1f} steps/s ({dt / STEPS * 1e6:.1f} us/step) "
          f"out {h}", flush=True)
