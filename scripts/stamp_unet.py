"""Per-phase time breakdown of the UNet loop (ldm_unet_loop) from its diagnostic build:
  cp -rp build build_stamp && rm build_stamp/unet.o && \\
  make -C <csrc> BUILD=build_stamp OUT=../ldm_sdf/libldm_stamp.so \\
       HIPFLAGS="<usual flags> -DUNET_STAMP=1"
then  LDM_SDF_LIB=<...>/libldm_stamp.so python scripts/stamp_unet.py [B].
Thread 0 of XCD 0's tile-0 workgroup stamps s_memrealtime (100 MHz) in every phase of the
second step: start, staged, MFMA done, epilogue done, drained, prefetch done (then the wait)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
dev = torch.device("cuda", 0)
m = ldm_sdf.UNet1DDenoiser(D=1024, seed=2468)
sd = ldm_sdf.DDPMSchedule().device(dev)
loop = m.make_loop(B, "bf16", dev, sd["desc"])
x2 = torch.randn(2, B, 1024, device=dev)
noise = torch.randn(1000, B, 1024, device=dev)
for _ in range(3):
    loop(x2, noise, 999, 4)
torch.cuda.synchronize()
assert loop.status() == 0
nph = 18
raw = loop.ws.view(torch.uint8)[-4096:].view(torch.int64)[: nph * 6].cpu().numpy()
st = raw.reshape(nph, 6).astype(np.int64)
names = ["stage", "mfma", "epilogue", "drain", "prefetch", "wait"]
tot = np.zeros(6)
print("phase  " + "  ".join(f"{n:>9s}" for n in names) + "   (us)")
for p in range(nph):
    nxt = st[p + 1, 0] if p + 1 < nph else None
    d = [st[p, k + 1] - st[p, k] for k in range(5)] + [(nxt - st[p, 5]) if nxt else 0]
    tot += d
    print(f"{p:5d}  " + "  ".join(f"{v / 100:9.2f}" for v in d))
print("total  " + "  ".join(f"{v / 100:9.2f}" for v in tot) +
      f"   step (17 phases + last's tail) {(st[-1, 5] - st[0, 0]) / 100:.1f} us")
