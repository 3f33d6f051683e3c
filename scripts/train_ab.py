"""Same-process A/B of train() switches at config 2 (graph replay vs eager one-call steps):
interleaved rounds, median steps/s per variant."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402

dev = torch.device("cuda", 0)
lat = torch.randn(1000, 256, device=dev) * 0.5
sch = ldm_sdf.DDPMSchedule()
variants = {"graph": dict(graph=True), "eager": dict(graph=False)}
states, models = {}, {}
for k, kw in variants.items():
    models[k] = ldm_sdf.MLPDenoiser(seed=4321)
    states[k] = ldm_sdf.train(models[k], sch, lat, steps=3, batch=1000, **kw)
res = {k: [] for k in variants}
for r in range(4):
    for k, kw in variants.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        states[k] = ldm_sdf.train(models[k], sch, lat, steps=128, batch=1000, state=states[k], **kw)
        torch.cuda.synchronize()
        res[k].append(128 / (time.perf_counter() - t0))
for k in variants:
    print(f"{k}: median {statistics.median(res[k]):.1f} steps/s  all {[round(x) for x in res[k]]}")
