"""Timeline of one launch of the one-launch training step (csrc/train_dag.hip) at config 2, from
the diagnostic build's stamps (-DDAG_TRACE=1): per job the workgroup, the dequeue, the moment its
inputs were ready and its completion (s_memrealtime, 100 MHz).  Prints per node its window inside
the launch, the mean compute time of its jobs and their mean wait for inputs, and the launch's
totals: busy / waiting / scheduler shares of the workgroup-time.
  build:  make -C <csrc> BUILD=build_stamp OUT=../ldm_sdf/libldm_diag.so \\
            HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics \\
                      -DSL_STAMP=1 -DDAG_TRACE=1"
  run:    LDM_SDF_LIB=<...>/libldm_diag.so python scripts/trace_dag.py [M] [flags] [out.npz]"""
import ctypes as C
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import _capi as capi, api, ops  # noqa: E402
from ldm_sdf import dist as ldist  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
FLAGS = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
OUT = sys.argv[3] if len(sys.argv) > 3 else None
dev = torch.device("cuda", 0)
lib = capi.load()
den = ldm_sdf.MLPDenoiser(seed=4321)
den.to_device(dev)
sch = ldm_sdf.DDPMSchedule()
st = api.TrainState()
st.masters = {n: den.params[n] for n in den.names()}
st.adam = {n: (torch.zeros_like(v), torch.zeros_like(v)) for n, v in st.masters.items()}
grads = ldist.flat_buffers({n: tuple(v.shape) for n, v in st.masters.items()}, dev)[1]
table = api._adam_table(den, st, grads, "bf16", dev)
pack = den.device_pack("bf16", dev, with_tables=False)
sd = sch.device(dev)["desc"]
ws = den.train_workspace(M, dev)
gs = den.grads_struct(grads)
buf = C.create_string_buffer(1 << 20)
assert lib.ldm_denoiser_train_dag_describe(C.byref(pack["desc"]), C.byref(sd), M, ws.data_ptr(),
                                           C.byref(gs), table, len(table), buf, len(buf)) == 0
nodes = {}
for line in buf.value.decode().splitlines():
    m = re.match(r"(\d+) (\w+) (\d+)x(\d+) nk (\d+) kgp (\d+)", line)
    if m:
        nodes[int(m[1])] = (m[2], int(m[3]) * int(m[4]), int(m[5]))
ops.train_step_config("dag")
fl = lib.ldm_dev_train_dag_flags
fl.restype, fl.argtypes = C.c_int, [C.c_uint]
fl(FLAGS)
lat = torch.randn(M, 256, device=dev) * 0.5
t = torch.randint(0, 1000, (M,), device=dev, dtype=torch.int32)
eps = torch.randn(M, 256, device=dev)
loss = torch.zeros(1, device=dev)


def step():
    ops.denoiser_train_step_adamw(pack["desc"], sd, lat, eps, t, ws, gs, loss, table, lr=1e-4,
                                  weight_decay=0.0, step=1)


for _ in range(20):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    step()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 50
step()
torch.cuda.synchronize()
assert ops.train_step_last_form() == "dag"
ent = np.zeros((16384, 4), dtype=np.uint64)
wgs = np.zeros((4096, 2), dtype=np.uint64)
tr = lib.ldm_dev_train_dag_trace
tr.restype, tr.argtypes = C.c_int, [C.c_void_p, C.c_void_p]
assert tr(ent.ctypes.data, wgs.ctypes.data) == 0
grid = int((wgs[:, 0] > 0).sum())
wgs = wgs[:grid].astype(np.int64)
n_ent = sum(v[1] for v in nodes.values())
e = ent[:n_ent]
e = e[e[:, 3] > 0]
code = (e[:, 0] >> np.uint64(32)).astype(np.int64)
node = code >> 16
wg = (e[:, 0] & np.uint64(0xffff)).astype(np.int64)
xcc = ((e[:, 0] >> np.uint64(16)) & np.uint64(15)).astype(np.int64)
T0 = wgs[:, 0].min()
deq, rdy, done = [(e[:, k].astype(np.int64) - T0) / 100.0 for k in (1, 2, 3)]      # us
span = (wgs[:, 1].max() - T0) / 100.0
print(f"M={M} flags {hex(FLAGS)}: step wall {wall * 1e6:.1f} us (50 steps), traced launch span "
      f"{span:.1f} us, grid {grid}, jobs traced {len(e)} of {n_ent}; workgroup starts spread "
      f"{(wgs[:, 0].max() - T0) / 100:.1f} us, exits {(wgs[:, 1].min() - T0) / 100:.1f}.."
      f"{span:.1f} us")
# the queue mapping assumes workgroup b runs on XCD b % 8 (round-robin dispatch)
wx = {}
for w_, x_ in zip(wg.tolist(), xcc.tolist()):
    wx[w_] = x_
bad = sum(1 for w_, x_ in wx.items() if x_ != w_ % 8)
print(f"XCC_ID of {len(wx)} workgroups: {bad} differ from blockIdx % 8; per XCD "
      f"{np.bincount(np.array(list(wx.values()), dtype=np.int64), minlength=8).tolist()}")
print(" node type  jobs  nk    first_deq  first_rdy  last_done   compute_us  wait_us   "
      "(means per job)")
for i in sorted(nodes):
    s = node == i
    if not s.any():
        continue
    typ, jobs, nk = nodes[i]
    print(f"  {i:3d} {typ:4s} {jobs:5d} {nk:3d}  {deq[s].min():9.1f}  {rdy[s].min():9.1f}  "
          f"{done[s].max():9.1f}   {(done[s] - rdy[s]).mean():9.2f}  {(rdy[s] - deq[s]).mean():8.2f}")
busy = (done - rdy).sum()
wait = (rdy - deq).sum()
tot = grid * span
# scheduler gap: from a workgroup's previous completion (or start) to its next dequeue
order = np.lexsort((deq, wg))
gap = 0.0
prev_wg, prev_t = -1, 0.0
starts = {w: (wgs[w, 0] - T0) / 100.0 for w in range(grid)}
for k in order:
    w = wg[k]
    pt = prev_t if w == prev_wg else starts[w]
    gap += deq[k] - pt
    prev_wg, prev_t = w, done[k]
print(f"workgroup-time {tot:.0f} us: busy {100 * busy / tot:.1f}%  waiting for inputs "
      f"{100 * wait / tot:.1f}%  between jobs {100 * gap / tot:.1f}%  rest (drain / exit) "
      f"{100 * (tot - busy - wait - gap) / tot:.1f}%")
for typ in ("gemm", "prep", "sum", "adam"):
    s = np.array([nodes[int(n)][0] == typ for n in node])
    if s.any():
        print(f"  {typ}: {s.sum()} jobs, busy {(done[s] - rdy[s]).sum():.0f} us "
              f"({100 * (done[s] - rdy[s]).sum() / tot:.1f}%), mean {(done[s] - rdy[s]).mean():.2f} us")
if OUT:
    np.savez(OUT, node=node, job=code & 0xffff, wg=wg, deq=deq, rdy=rdy, done=done,
             wg_start=(wgs[:, 0] - T0) / 100.0, wg_end=(wgs[:, 1] - T0) / 100.0)
