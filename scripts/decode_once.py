"""Minimal decoder workload for profilers: warm-up + R launches of B x N^3 (bf16)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import ops  # noqa: E402

B = int(os.environ.get("DEC_B", "2"))
N = int(os.environ.get("DEC_N", "256"))
R = int(os.environ.get("DEC_R", "3"))
dtype = os.environ.get("DEC_DTYPE", "bf16")
dev = torch.device("cuda", 0)
dec = ldm_sdf.SDFDecoder(256, seed=1234)
pk = dec.device_pack(dtype, dev, layout=os.environ.get("DEC_LAYOUT") or None)
z = torch.randn(B, 256, device=dev) * 0.1
beta = ops.decoder_fold(pk["desc"], z)
out = torch.empty(B, N, N, N, device=dev)
for _ in range(R + 1):
    ops.decoder_grid_fwd(pk["desc"], beta, N, 0, N, out=out)
torch.cuda.synchronize()
print("ok", float(out.abs().mean()))
