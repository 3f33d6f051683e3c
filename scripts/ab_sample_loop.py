"""A/B of the DDPM sampling paths at B=8, 1000 steps (bf16): graph-replayed per-step launches
vs the persistent one-launch loop: XCD replicas, chip-wide with the XCD-hierarchical barrier, flat.
Each variant is checked bit-identical to the graph path.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402

import ldm_sdf  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
den = ldm_sdf.MLPDenoiser(seed=4321)
sch = ldm_sdf.DDPMSchedule()
g = torch.Generator(device=dev).manual_seed(0)
xT = torch.randn(B, 256, device=dev, generator=g)
noise = torch.randn(1000, B, 256, device=dev, generator=g)


def timeit(s, reps=5):
    s.run(xT, noise, check=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        s.run(xT, noise, check=False)
    torch.cuda.synchronize()
    return 1000 * reps / (time.perf_counter() - t)


res = {"batch": B}
sg = ldm_sdf.Sampler(den, sch, B, dtype="bf16", device=dev, persistent=False)
ref = sg.run(xT, noise).clone()
res["graph_steps_per_s"] = timeit(sg)
for mode in os.environ.get("MODES", "replica,xcd,flat").split(","):
    # "replica": tagged-granule hand-offs (default); "replica0": the same loop on XCD barriers
    os.environ["LDM_SAMPLE_LOOP_BARRIER"] = mode.rstrip("0")
    os.environ["LDM_SAMPLE_LOOP_TAGGED"] = "0" if mode.endswith("0") else "1"
    sp = ldm_sdf.Sampler(den, sch, B, dtype="bf16", device=dev, persistent=True)
    out = sp.run(xT, noise).clone()
    res[f"loop_{mode}_status"] = sp.loop.status()
    res[f"loop_{mode}_identical"] = bool(torch.equal(out, ref))
    res[f"loop_{mode}_steps_per_s"] = timeit(sp)
print(json.dumps(res))
