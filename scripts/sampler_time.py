"""DDPM sampler timing at B = 8 in two styles: stamp_sampler.py's (one warm run, status checked by
Sampler.run) and bench.py's (3 reps, check=False + the loop status read per rep); with
LDM_SDF_LIB pointing at another build of libldm_sdf.so this compares builds.
Usage: [LDM_SDF_LIB=...] python scripts/sampler_time.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402

dev = torch.device("cuda", 0)
den = ldm_sdf.MLPDenoiser(seed=4321)
sch = ldm_sdf.DDPMSchedule()
smp = ldm_sdf.Sampler(den, sch, 8, dtype="bf16", device=dev)
xT = torch.randn(8, 256, device=dev)
noise = torch.randn(1000, 8, 256, device=dev)
smp.run(xT, noise)
for _ in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    smp.run(xT, noise)
    torch.cuda.synchronize()
    one = 1000 / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(3):
        smp.run(xT, noise, check=False)
        smp.loop.status()
    torch.cuda.synchronize()
    three = 3000 / (time.perf_counter() - t0)
    print(f"lib {os.environ.get('LDM_SDF_LIB', 'product')}: one run {one:.0f} steps/s, "
          f"3 reps + status {three:.0f} steps/s, form {ldm_sdf.ops.sample_loop_last_form()}",
          flush=True)
