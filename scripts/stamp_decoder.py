"""Per-quarter cycle breakdown of the quarter decoder kernel (diagnostic build with -DQSTAMP=1:
build with  make -C <csrc> BUILD=build_stamp OUT=../ldm_sdf/libldm_stamp.so HIPFLAGS="... -DQSTAMP=1"
and run with  LDM_SDF_LIB=.../libldm_stamp.so python scripts/stamp_decoder.py).
Wave 0 of each workgroup stamps s_memtime around every quarter of its second tile; the stamps
overwrite the start of the output.  Prints median cycles over workgroups per segment."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import ops  # noqa: E402

B, N = 16, 256
dev = torch.device("cuda", 0)
dec = ldm_sdf.SDFDecoder(256, seed=1234)
pk = dec.device_pack("bf16", dev, layout="quarter")
z = torch.randn(B, 256, device=dev) * 0.1
beta = ops.decoder_fold(pk["desc"], z)
out = torch.empty(B, N, N, N, device=dev)
for _ in range(2):
    ops.decoder_grid_fwd(pk["desc"], beta, N, 0, N, out=out)
torch.cuda.synchronize()
grid = torch.cuda.get_device_properties(0).multi_processor_count
st = out.reshape(-1)[: grid * 192].view(torch.int64).reshape(grid, 96).cpu().numpy()
nq = 26
t = st[:, : 3 + 3 * nq]
d = np.diff(t, axis=1)
med = np.median(d, axis=0)
total = np.median(t[:, 2 + 3 * nq] - t[:, 0])
print(f"tile total (median over {grid} WGs): {total:.0f} cycles; ideal MFMA "
      f"{3192 * 32} -> {3192 * 32 / total:.1%}")
print(f"layer 0: {med[0]:.0f}")
names = ["prologue(4 steps+epi)", "k-loop rest", "aux step + next start"]
agg = {}
for qi in range(nq):
    row = [med[1 + 3 * qi + k] for k in range(3)]
    if qi < 4: lay = 1
    elif qi < 8: lay = 2
    elif qi < 10: lay = 3
    elif qi < 14: lay = 4
    else: lay = 5 + (qi - 14) // 4
    print(f"q{qi:2d} (layer {lay}): " + "  ".join(f"{n} {v:6.0f}" for n, v in zip(names, row)))
    for n, v in zip(names, row):
        agg[n] = agg.get(n, 0) + v
print("sum:", {k: int(v) for k, v in agg.items()})
