"""Per-phase times of the XCD-replica sampling loop (csrc/sample_loop.hip
sample_replica_kernel), from its stamps (on in the product build since round 5, SL_STAMP = 1):
every wave sums the s_memrealtime ticks (100 MHz) of each phase of every layer it runs -- own
granules landed, the workgroup's staging barrier, row dot products, reduce-scatter, epilogue +
publish.  Usage: python scripts/stamp_sampler.py [B]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import _capi as capi  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
lib = capi.load()
fn = lib.ldm_dev_sample_stamps
fn.restype = C.c_int
fn.argtypes = [C.c_void_p]
den = ldm_sdf.MLPDenoiser(seed=4321)
sch = ldm_sdf.DDPMSchedule()
smp = ldm_sdf.Sampler(den, sch, B, dtype="bf16", device=dev)
xT = torch.randn(B, 256, device=dev)
noise = torch.randn(1000, B, 256, device=dev)
smp.run(xT, noise)
torch.cuda.synchronize()
t0 = time.perf_counter()
smp.run(xT, noise)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"B={B}: {1000 / dt:.0f} steps/s ({dt * 1e3:.2f} ms / 1000 steps), form "
      f"{ldm_sdf.ops.sample_loop_last_form()}")
st = np.zeros((256, 8, 8), dtype=np.uint64)
assert fn(st.ctypes.data) == 0
a = st[:, :, :6].astype(np.float64)
layers = a[:, :, 5]
live = layers > 0
names = ["own granules landed", "staging barrier", "row dots", "reduce-scatter",
         "epilogue + publish"]
tot = 0.0
for k, nm in enumerate(names):
    per = a[:, :, k][live] / layers[live] * 10.0          # ns per layer (100 MHz ticks)
    tot += per.mean()
    print(f"  {nm:22s} mean {per.mean():7.1f} ns/layer  min {per.min():7.1f}  max {per.max():7.1f}")
print(f"  {'sum':22s} mean {tot:7.1f} ns/layer; waves {int(live.sum())}, layers/wave "
      f"{int(layers[live].mean())}; step {dt / 1000 * 1e9 / 6:.0f} ns/layer wall")
