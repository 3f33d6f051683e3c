"""One library's config-4-style decode (B shapes x N^3, bf16 split kernel), HIP event time per
decode (median of R after 2 warm-ups), TF/s and fraction of the dense bf16 peak, plus an output
checksum so that builds can be compared bit for bit.  Cross-library A/Bs run it once per
library, alternating (scripts/rounds/r06.sh dlib).  Usage: python scripts/decode_time.py [B] [N] [R]
(LDM_SDF_LIB selects the library)."""
import hashlib
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
R = int(sys.argv[3]) if len(sys.argv) > 3 else 5
FLOPS = 3146752
dev = torch.device("cuda", 0)
dec = ldm_sdf.SDFDecoder(256, seed=1234)
pk = dec.device_pack("bf16", dev)
g = torch.Generator(device=dev).manual_seed(0)
z = torch.randn(B, 256, device=dev, generator=g) * 0.1
beta = ops.decoder_fold(pk["desc"], z)
out = torch.empty(B, N, N, N, device=dev)
ts = []
for r in range(R + 2):
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    ops.decoder_grid_fwd(pk["desc"], beta, N, 0, N, out=out)
    e1.record()
    torch.cuda.synchronize()
    if r >= 2:
        ts.append(e0.elapsed_time(e1))
ms = statistics.median(ts)
tf = FLOPS * B * N ** 3 / (ms * 1e-3) / 1e12
h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:16]
print(f"lib {os.path.basename(os.environ.get('LDM_SDF_LIB', 'libldm_sdf.so'))}: B={B} N={N} "
      f"median {ms:.2f} ms  {tf:.1f} TF/s  frac {tf / 2516.6:.4f}  min {min(ts):.2f}  out {h}")
