"""Diagnostics of the one-launch training step (csrc/train_dag.hip): prints the job table the
host builds (ldm_denoiser_train_dag_describe), runs ONE step with a short dependency-wait limit
(so a stuck wait ends the launch instead of hanging it), and prints the status word, the queue
heads and, per node, its counters against their targets (the kernel leaves them in place when a
wait gave up).  Usage: timeout 60 python scripts/dag_diag.py [spin_limit_us] [M] [flags]
(flags: ldm_dev_train_dag_flags -- bit t skips node type t's compute, bit 4 the fences)"""
import ctypes as C
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import _capi as capi, api, ops  # noqa: E402
from ldm_sdf import dist as ldist  # noqa: E402

SPIN = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
M = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
FLAGS = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0
dev = torch.device("cuda", 0)
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
rc = capi.load().ldm_denoiser_train_dag_describe(C.byref(pack["desc"]), C.byref(sd), M,
                                                 ws.data_ptr(), C.byref(gs), table, len(table),
                                                 buf, len(buf))
desc = buf.value.decode()
print("describe rc", rc)
print(desc if FLAGS == 0x1F else desc.splitlines()[0], flush=True)
nodes = []
for line in desc.splitlines():
    m = re.match(r"(\d+) (\w+) (\d+)x(\d+) nk (\d+) kgp (\d+) band (-?\d+) all (\d+)", line)
    if m:
        nodes.append(dict(i=int(m[1]), type=m[2], tm=int(m[3]), tn=int(m[4]), band=int(m[7]),
                          all=int(m[8])))
ops.train_step_config("dag", spin_limit=SPIN)
_fl = capi.load().ldm_dev_train_dag_flags
_fl.restype, _fl.argtypes = C.c_int, [C.c_uint]
_fl(FLAGS)
print("flags", hex(FLAGS), "spin_us", SPIN, flush=True)
lat = torch.randn(M, 256, device=dev) * 0.5
t = torch.randint(0, 1000, (M,), device=dev, dtype=torch.int32)
eps = torch.randn(M, 256, device=dev)
loss = torch.zeros(1, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
ops.denoiser_train_step_adamw(pack["desc"], sd, lat, eps, t, ws, gs, loss, table, lr=1e-4,
                              weight_decay=0.0, step=1)
torch.cuda.synchronize()
print(f"step: {1e3 * (time.perf_counter() - t0):.2f} ms, form {ops.train_step_last_form()}, "
      f"loss {float(loss):.5f}")
C0 = 26                                  # train_dag.h kSyncCtr0 (heads 0-23, exit 24, status 25)
nsync = (C0 + 512) * 128
w = ws[-nsync:].view(torch.int32).cpu().view(-1, 32)[:, 0]
print("heads", w[:24].tolist(), "exit", int(w[24]), "status", int(w[25]))
for nd in nodes:
    allv = int(w[C0 + nd["all"]])
    bands = w[C0 + nd["band"]:C0 + nd["band"] + nd["tm"]].tolist() if nd["band"] >= 0 else []
    tot = nd["tm"] * nd["tn"]
    flag = "" if allv == tot else "   <-- incomplete"
    print(f"node {nd['i']:2d} {nd['type']:4s} all {allv}/{tot} bands {bands}{flag}")
print("status (read + cleared):", ops.train_status(pack["desc"], M, ws))
