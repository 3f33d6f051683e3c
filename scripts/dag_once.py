"""Minimal one-launch training-step workload for profilers: config 2 (batch 1000) through the
DAG form (csrc/train_dag.hip), TRAIN_STEPS steps (default 20) after 3 warm-up steps."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import ops  # noqa: E402

S = int(os.environ.get("TRAIN_STEPS", "20"))
dev = torch.device("cuda", 0)
ops.train_step_config("dag")
den = ldm_sdf.MLPDenoiser(seed=4321)
lat = torch.randn(1000, 256, device=dev) * 0.5
sch = ldm_sdf.DDPMSchedule()
st = ldm_sdf.train(den, sch, lat, steps=3, batch=1000)
st = ldm_sdf.train(den, sch, lat, steps=S, batch=1000, state=st)
torch.cuda.synchronize()
assert ops.train_step_last_form() == "dag"
print("dag steps", S, "loss", st.losses[-1])
