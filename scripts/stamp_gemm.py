"""Per-phase times of the ldm_gemm_bf16 launches of one config-2 training step (batch 1000,
bf16), from the diagnostic build's stamps (-DGEMM_STAMP=1): workgroup 0 of every non-persistent
LDS-DMA launch stamps s_memrealtime (100 MHz) at entry, after its prologue stages are issued,
when the first stage has landed, after the k-loop, after the epilogue's stores are issued and
after they drained (csrc/gemm_bf16.hip GStamp).
  build:  make -C <csrc> BUILD=build_stamp OUT=../ldm_sdf/libldm_stamp.so \\
            HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics \\
                      -DUNET_STAMP=1 -DGEMM_STAMP=1 -DLDM_DEV_KNOBS"
  run:    LDM_SDF_LIB=<...>/libldm_stamp.so python scripts/stamp_gemm.py"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import _capi as capi  # noqa: E402

dev = torch.device("cuda", 0)
den = ldm_sdf.MLPDenoiser(seed=4321)
sch = ldm_sdf.DDPMSchedule()
lat = torch.randn(1000, 256, device=dev) * 0.5
st = ldm_sdf.train(den, sch, lat, steps=3, batch=1000, dtype="bf16")
torch.cuda.synchronize()
lib = capi.load()
lib.ldm_dev_gemm_stamps.argtypes = [C.c_void_p, C.c_void_p]
buf = np.zeros((256, 8), dtype=np.uint64)
n0 = C.c_uint(0)
assert lib.ldm_dev_gemm_stamps(buf.ctypes.data, C.byref(n0)) == 0
st = ldm_sdf.train(den, sch, lat, steps=1, batch=1000, dtype="bf16", state=st)
torch.cuda.synchronize()
n1 = C.c_uint(0)
assert lib.ldm_dev_gemm_stamps(buf.ctypes.data, C.byref(n1)) == 0
k = n1.value - n0.value
print(f"one training step: {k} stamped GEMM launches; workgroup 0, us (s_memrealtime, 10 ns)")
print(f"{'#':>3} {'grid':>5} {'tiles':>5} {'issue':>7} {'first':>7} {'kloop':>7} {'epi':>7} "
      f"{'drain':>7} {'total':>7} {'->next':>7}")
rows = [buf[(n0.value + i) % 256].astype(np.int64) for i in range(k)]
tot = np.zeros(7)
for i, r in enumerate(rows):
    nxt = (rows[i + 1][0] - r[5]) / 100 if i + 1 < k else 0.0
    d = [(r[1] - r[0]) / 100, (r[2] - r[1]) / 100, (r[3] - r[2]) / 100, (r[4] - r[3]) / 100,
         (r[5] - r[4]) / 100, (r[5] - r[0]) / 100, nxt]
    tot += d
    print(f"{i:>3} {r[6]:>5} {r[7]:>5} " + " ".join(f"{x:7.2f}" for x in d))
print(f"{'sum':>15} " + " ".join(f"{x:7.2f}" for x in tot))
