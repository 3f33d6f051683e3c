"""Per-segment cycle breakdown of the split decoder kernel (diagnostic build -DFS_STAMP=1:
  make -C <csrc> BUILD=build_stamp OUT=../ldm_sdf/libldm_stamp.so \
       HIPFLAGS="<usual flags> -DFS_STAMP=1"
and run with  LDM_SDF_LIB=<...>/libldm_stamp.so python scripts/stamp_split.py).  Wave 0 of each
workgroup stamps s_memtime at part / layer boundaries of its second tile; the stamps overwrite
the start of the output.  Prints the median cycles over workgroups per segment (skip 253)."""
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
pk = dec.device_pack("bf16", dev, layout="split")
z = torch.randn(B, 256, device=dev) * 0.1
beta = ops.decoder_fold(pk["desc"], z)
out = torch.empty(B, N, N, N, device=dev)
for _ in range(2):
    ops.decoder_grid_fwd(pk["desc"], beta, N, 0, N, out=out)
torch.cuda.synchronize()
grid = torch.cuda.get_device_properties(0).multi_processor_count
st = out.reshape(-1)[: grid * 256].view(torch.int64).reshape(grid, 128).cpu().numpy()
labels = []


def part(name, kind):
    """stamps of one run_part (csrc/decoder_fs.hip): after its aux step (plus the first read,
    after a barrier for bar0 parts), after steps 0-15, at its end.  BAR = the in-stream barrier
    inside step 15, END = the one inside the part's last step."""
    if kind == "aux":
        return [f"{name} aux"]
    segs = {"E0mid": ("E 0-15 + BAR", "steps 16-31"),
            "E16": ("steps 0-15 + BAR", "E 16-31 + END"),
            "plain16": ("steps 0-15", "(none)"),
            "E0end16": ("E 0-15 + END", "(none)"),
            "FIN1": ("E(prev L7p1) 0-15 + BAR + store", "steps 16-31"),
            "FIN0": ("E 0-15", "steps 16-31 + END")}[kind]
    return [f"{name} aux"] + [f"{name} {x}" for x in segs]


labels += part("L0p0", "aux") + ["L0 serial A"] + part("L0p1", "aux") + ["L0 serial B"]
labels += part("L1p0", "FIN1") + part("L1p1", "E16")
labels += part("L2p0", "E0mid") + part("L2p1", "E16")
labels += part("L3p0", "E0mid") + ["L3 bar + serial write"]
labels += part("L4p0", "plain16") + part("L4p1", "E0end16")
for l in (5, 6):
    labels += part(f"L{l}p0", "E0mid") + part(f"L{l}p1", "E16")
labels += part("L7p0", "E0mid") + part("L7p1", "FIN0")
n = len(labels) + 1
t = st[:, :n]
d = np.diff(t, axis=1)
med = np.median(d, axis=0)
total = np.median(t[:, n - 1] - t[:, 0])
print(f"tile total (median over {grid} WGs): {total:.0f} cycles; ideal MFMA (3192 x 32) "
      f"{3192 * 32} -> {3192 * 32 / total:.1%}")
agg = {}
for lab, v in zip(labels, med):
    print(f"  {lab:28s} {v:8.0f}")
    key = lab.split(" ", 1)[1] if lab[0] == "L" and lab[2] == "p" else lab
    agg[key] = agg.get(key, 0) + v
print("by kind:")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
    print(f"  {k:24s} {v:8.0f}  {v / total:.1%}")
