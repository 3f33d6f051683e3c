"""Run the split16 decoder's LDS-dump diagnostic build (-DFS16_DUMP=k) on a 32^3 grid decode
and save the dumped activation positions (workgroup 0, first tile) for CPU comparison."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402

k = sys.argv[1]
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(3)
z = torch.randn(1, 256, generator=g) * 0.1
dec = ldm_sdf.SDFDecoder(256, seed=1234)
dec.DEFAULT_LAYOUT = "split16"
out = ldm_sdf.decode(dec, z.to(dev), 32, dtype="bf16")
torch.cuda.synchronize()
raw = out.reshape(-1).view(torch.int32).cpu().numpy()
np.savez(os.path.join(ROOT, "gpurun_out", "r03f", f"dump{k}.npz"), raw=raw, z=z.numpy())
print("dumped", k, flush=True)
