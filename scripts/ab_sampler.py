"""Same-process A/B of the sampling GEMV kernels (LDM_SMALL_LINEAR=1|2): 1000-step hipGraph
replays, interleaved rounds; also checks the variants agree."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
den, sch = ldm_sdf.MLPDenoiser(seed=4321), ldm_sdf.DDPMSchedule()
g = torch.Generator(device=dev).manual_seed(0)
xT = torch.randn(B, 256, device=dev, generator=g)
noise = torch.randn(1000, B, 256, device=dev, generator=g)
samplers = {}
for v in os.environ.get("AB_SMALL", "1,2,3").split(","):
    os.environ["LDM_SMALL_LINEAR"] = v
    samplers[v] = ldm_sdf.Sampler(den, sch, B, dtype="bf16", device=dev)
    samplers[v].run(xT, noise)          # capture under this variant
torch.cuda.synchronize()
outs = {v: s.result.clone() for v, s in samplers.items()}
ref = outs[list(outs)[0]]
for v, o in outs.items():
    print(f"max |v{list(outs)[0]} - v{v}| =", float((o - ref).abs().max()))
times = {v: [] for v in samplers}
for _ in range(5):
    for v, s in samplers.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.run(xT, noise)
        torch.cuda.synchronize()
        times[v].append(time.perf_counter() - t0)
for v in samplers:
    m = statistics.median(times[v])
    print(f"v{v}: {m*1e3:.2f} ms / 1000 steps -> {1000/m:.0f} steps/s (B={B})")
