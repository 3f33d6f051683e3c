"""Per-phase times of the 18 ldm_conv1d launches of one UNet reverse step (graph path, B = 1),
from the diagnostic build's stamps (-DUNET_STAMP=1): workgroup (0, 0, 0) of each launch stamps
s_memrealtime (100 MHz) at entry, after staging (barrier), after the MFMA loop (barrier), after
the partial-tile reduction (barrier) and after its stores drained; inside the staging, after
segment 0's weights, after segment 0's window and after the last segment (thread 0's view;
the rest up to the barrier is waiting for the other waves); inside the contraction, after its
first operand reads and after its MFMA loop; in the epilogue, after the stores are issued.
Stamps are held in registers and written at the kernel's end (no atomic in the timed path).
  build:  make -C <csrc> BUILD=build_stamp OUT=../ldm_sdf/libldm_stamp.so \\
            HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -DUNET_STAMP=1"
  run:    LDM_SDF_LIB=<...>/libldm_stamp.so python scripts/stamp_conv.py [B]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import _capi as capi  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
dev = torch.device("cuda", 0)
m = ldm_sdf.UNet1DDenoiser(seed=2468)
s = ldm_sdf.Sampler(m, ldm_sdf.DDPMSchedule(), B, steps=20, dtype="bf16", device=dev,
                    persistent=False)
xT = torch.randn(B, 1024, device=dev)
noise = torch.randn(1000, B, 1024, device=dev)
for _ in range(3):
    s.run(xT, noise)
torch.cuda.synchronize()
lib = capi.load()
lib.ldm_dev_conv_stamps.argtypes = [C.c_void_p, C.c_void_p]
buf = np.zeros((256, 16), dtype=np.uint64)
n = C.c_uint(0)
assert lib.ldm_dev_conv_stamps(buf.ctypes.data, C.byref(n)) == 0
n = n.value
slots = [(n - 18 * 2 + i) % 256 for i in range(18 * 2)]     # the last two steps
st = buf[slots].astype(np.int64)
names = ["conv_in", "r0.c1", "r0.c2", "down0", "r1.c1", "r1.c2", "down1", "r2.c1", "r2.c2",
         "r3.c1", "r3.c2", "up1", "r4.c1", "r4.c2", "up0", "r5.c1", "r5.c2", "conv_out"]
print(f"B={B}: per-launch phases of workgroup (0,0,0), us (s_memrealtime, 10 ns)")
print(f"{'conv':>9} {'stage':>7} {'mfma':>7} {'reduce':>7} {'epi+st':>7} {'total':>7} {'->next':>7}"
      f" | stage = {'w0':>6} {'x0':>6} {'segs+':>6} {'bar':>6} | mfma = {'pro':>6} {'loop':>6}"
      f" {'bar':>6} | epi {'issue':>6} {'drain':>6}")
tot = np.zeros(15)
for i in range(18):
    r = st[18 + i]
    nxt = st[18 + i + 1][0] if i + 1 < 18 else r[7]
    d = [(r[1] - r[0]) / 100, (r[2] - r[1]) / 100, (r[6] - r[2]) / 100, (r[7] - r[6]) / 100,
         (r[7] - r[0]) / 100, (nxt - r[7]) / 100,
         (r[3] - r[0]) / 100, (r[4] - r[3]) / 100, (r[5] - r[4]) / 100, (r[1] - r[5]) / 100,
         (r[8] - r[1]) / 100, (r[9] - r[8]) / 100, (r[2] - r[9]) / 100,
         (r[10] - r[6]) / 100, (r[7] - r[10]) / 100]
    tot += d
    print(f"{names[i]:>9} " + " ".join(f"{x:7.2f}" for x in d[:6]) + " | " +
          " ".join(f"{x:6.2f}" for x in d[6:10]) + " | " + " ".join(f"{x:6.2f}" for x in d[10:13])
          + " | " + " ".join(f"{x:6.2f}" for x in d[13:]))
print(f"{'sum':>9} " + " ".join(f"{x:7.2f}" for x in tot[:6]) + " | " +
      " ".join(f"{x:6.2f}" for x in tot[6:10]) + " | " + " ".join(f"{x:6.2f}" for x in tot[10:13])
      + " | " + " ".join(f"{x:6.2f}" for x in tot[13:]))
print(f"step span (entry of conv_in -> stores of conv_out): {(st[35][7] - st[18][0]) / 100:.1f} us")
if st[18:36, 11].any():
    print("direct staging split (us): entry->geo | ->loads issued | ->data landed | ->stores done")
    for i in range(18):
        r = st[18 + i]
        print(f"{names[i]:>9} {(r[13] - r[0]) / 100:7.2f} {(r[11] - r[13]) / 100:7.2f} "
              f"{(r[12] - r[11]) / 100:7.2f} {(r[3] - r[12]) / 100:7.2f}")
