"""Same-process A/B of the training-step forms at config 2 (batch 1000 on 1000 latents, bf16):
"dag" (the one-launch persistent step, csrc/train_dag.hip) vs "launches" (one launch per GEMM
group + AdamW); interleaved rounds, median steps/s per form.  Usage:
python scripts/train_form_ab.py [rounds] [steps]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import ops  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
S = int(sys.argv[2]) if len(sys.argv) > 2 else 128
dev = torch.device("cuda", 0)
lat = torch.randn(1000, 256, device=dev) * 0.5
sch = ldm_sdf.DDPMSchedule()
forms = os.environ.get("AB_FORMS", "dag,launches").split(",")
if os.environ.get("DAG_FLAGS"):            # ldm_dev_train_dag_flags, e.g. 0x100: claim scheduler
    import ctypes as C
    from ldm_sdf import _capi as capi
    fl = capi.load().ldm_dev_train_dag_flags
    fl.restype, fl.argtypes = C.c_int, [C.c_uint]
    fl(int(os.environ["DAG_FLAGS"], 0))
states, models, gens = {}, {}, {}
for f in forms:     # same weights, same t / eps draws per form: the params must end bit-identical
    ops.train_step_config(f)
    models[f] = ldm_sdf.MLPDenoiser(seed=4321)
    gens[f] = torch.Generator(device=dev).manual_seed(7)
    states[f] = ldm_sdf.train(models[f], sch, lat, steps=3, batch=1000, generator=gens[f])
res = {f: [] for f in forms}
for r in range(R):
    for f in forms:
        ops.train_step_config(f)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        states[f] = ldm_sdf.train(models[f], sch, lat, steps=S, batch=1000, state=states[f],
                                  generator=gens[f])
        torch.cuda.synchronize()
        res[f].append(S / (time.perf_counter() - t0))
        assert ops.train_step_last_form() == f
for f in forms:
    print(f"{f}: median {statistics.median(res[f]):.1f} steps/s  all {[round(x) for x in res[f]]}")
same = all(torch.equal(models[forms[0]].params[n], models[f].params[n])
           for f in forms[1:] for n in models[forms[0]].params)
print("params bit-identical across forms:", same)
