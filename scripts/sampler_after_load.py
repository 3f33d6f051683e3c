"""DDPM sampler steps/s (B = 8, bench.py's ddpm leg: 3 reps of 1000 steps, status read per rep)
on a fresh GPU, then right after the config-4 decode (B = 64 x 256^3, bench.py's first leg),
then again after a 2 s idle: does the heavy MFMA leg before it lower the latency-bound
sampler's rate (clock / power state)?  Prints the SCLK that rocm-smi-free torch reports nothing
about, so only the rates.  Usage: python scripts/sampler_after_load.py"""
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


def rate(reps=3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        smp.run(xT, noise, check=False)
        smp.loop.status()
    torch.cuda.synchronize()
    return 1000 * reps / (time.perf_counter() - t0)


print(f"fresh: {rate():.0f} steps/s", flush=True)
print(f"fresh again: {rate():.0f} steps/s", flush=True)
dec = ldm_sdf.SDFDecoder(256, seed=1234)
lat = torch.randn(64, 256, device=dev) * 0.1
for _ in range(4):                       # ~ bench.py's decode leg (warmup + 3 steps)
    ldm_sdf.decode(dec, lat, 256, dtype="bf16")
torch.cuda.synchronize()
print(f"after decode B=64 256^3 x4: {rate():.0f} steps/s", flush=True)
print(f"  and again: {rate():.0f} steps/s", flush=True)
time.sleep(2.0)
print(f"after 2 s idle: {rate():.0f} steps/s", flush=True)
