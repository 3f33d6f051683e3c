"""Marching cubes of the bench's volume (config 4 shape 0: decoder seed 1234, latents seed 0 x
0.1, 256^3 bf16 decode), REPS times, for rocprofv3 --kernel-trace --stats: per-kernel times of
the C18 passes (csrc/mc.hip).  Usage: python scripts/mc_once.py [reps] [N]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda", 0)
dec = ldm_sdf.SDFDecoder(256, seed=1234)
gen = torch.Generator(device=dev).manual_seed(0)
z = torch.randn(64, 256, device=dev, generator=gen)[:1] * 0.1
vol = ldm_sdf.decode(dec, z, N, dtype="bf16")[0]
from ldm_sdf import _capi as capi  # noqa: E402
ws = torch.empty(capi.load().ldm_mc_workspace_bytes(N), device=dev, dtype=torch.uint8)
v, f = ldm_sdf.marching_cubes(vol, ws=ws)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    v, f = ldm_sdf.marching_cubes(vol, ws=ws)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
import hashlib  # noqa: E402
h = hashlib.sha1(v.cpu().numpy().tobytes() + f.cpu().numpy().tobytes()).hexdigest()[:16]
print(f"lib {os.path.basename(os.environ.get('LDM_SDF_LIB', 'libldm_sdf.so'))} N={N}: "
      f"{v.shape[0]} vertices, {f.shape[0]} faces, {dt * 1e3:.3f} ms per mesh (wall, incl. "
      f"the count read-back), mesh {h}")
