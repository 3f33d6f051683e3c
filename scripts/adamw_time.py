"""ldm_adamw_multi alone over config 2's parameter set (the MLP denoiser's 16 tensors, 10.1 M
fp32 parameters, bf16 + transposed bf16 copies of every matrix, as train() updates them): HIP
event time per launch (median of 200) and the algorithmic bytes per second (p, g, m, v read;
p, m, v written; the bf16 copies written).  Usage: python scripts/adamw_time.py
(LDM_SDF_LIB selects the library)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import ops  # noqa: E402

dev = torch.device("cuda", 0)
m = ldm_sdf.MLPDenoiser(seed=4321)
g = torch.Generator(device=dev).manual_seed(3)
ents, nbytes = [], 0
for n, p in m.params.items():
    p = p.to(dev)
    gr = torch.randn(p.shape, device=dev, generator=g)
    mm, vv = torch.zeros_like(p), torch.zeros_like(p)
    lo = lot = None
    nbytes += p.numel() * 28
    if p.dim() == 2:
        lo = torch.empty_like(p, dtype=torch.bfloat16)
        lot = torch.empty(p.shape[1], p.shape[0], device=dev, dtype=torch.bfloat16)
        nbytes += p.numel() * 4
    ents.append((p, gr, mm, vv, lo, lot))
table = ops.adamw_table(ents)
for s in range(1, 11):
    ops.adamw_multi(table, lr=1e-4, weight_decay=0.01, step=s, device=dev)
torch.cuda.synchronize()
ts = []
for s in range(11, 211):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    ops.adamw_multi(table, lr=1e-4, weight_decay=0.01, step=s, device=dev)
    b.record()
    ts.append((a, b))
torch.cuda.synchronize()
us = statistics.median(a.elapsed_time(b) * 1e3 for a, b in ts)
print(f"lib {os.path.basename(os.environ.get('LDM_SDF_LIB', 'libldm_sdf.so'))}: adamw_multi "
      f"{us:.1f} us, {nbytes / 1e6:.1f} MB, {nbytes / us / 1e6:.2f} TB/s")
