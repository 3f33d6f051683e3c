"""Config-5 sampler A/B: the one-launch UNet loop (ldm_unet_loop) vs the hipGraph of 18-launch
steps, same inputs, interleaved reps; checks the results are bit-identical.
Usage: python scripts/unet_loop_ab.py [B ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402

dev = torch.device("cuda", 0)
m = ldm_sdf.UNet1DDenoiser(D=1024, seed=2468)
sch = ldm_sdf.DDPMSchedule()
for n in [int(v) for v in sys.argv[1:]] or [1, 8]:
    g = torch.Generator(device=dev).manual_seed(0)
    xT = torch.randn(n, 1024, device=dev, generator=g)
    noise = torch.randn(1000, n, 1024, device=dev, generator=g)
    smp = {"loop": ldm_sdf.Sampler(m, sch, n, dtype="bf16", device=dev, persistent=True),
           "graph": ldm_sdf.Sampler(m, sch, n, dtype="bf16", device=dev, persistent=False)}
    res = {k: s.run(xT, noise).clone() for k, s in smp.items()}
    times = {k: [] for k in smp}
    for _ in range(3):
        for k, s in smp.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s.run(xT, noise, check=False)
            torch.cuda.synchronize()
            times[k].append(time.perf_counter() - t0)
    st = smp["loop"].loop.status()
    print(f"B={n}: " + "  ".join(f"{k} {1000 / min(v):.0f} steps/s ({min(v) * 1e3:.2f} ms)"
                                 for k, v in times.items()) +
          f"  loop status {st}  bit-identical {torch.equal(res['loop'], res['graph'])}",
          flush=True)
