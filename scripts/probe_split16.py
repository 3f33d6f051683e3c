"""Capture split16 decoder outputs on structured networks (for CPU hypothesis tests)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from oracle import ref_cpu as R  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(3)
z = torch.randn(1, 256, generator=g) * 0.1
pts = torch.rand(1, 128, 3, generator=g) * 2 - 1


def eye_like(w):
    e = torch.zeros_like(w)
    n = min(w.shape)
    e[range(n), range(n)] = 1.0
    return e


out = {"z": z.numpy(), "pts": pts.numpy()}
for name, L in (("full", 8), ("id1", 1), ("id4", 4), ("id6", 6)):
    p = R.make_decoder_params(seed=1234)
    for l in range(L, 8):
        p.weights[l].copy_(eye_like(p.weights[l]))
    dec = ldm_sdf.SDFDecoder(256, weights=p.weights, biases=p.biases)
    dec.DEFAULT_LAYOUT = "split16"
    out[name] = ldm_sdf.decode_points(dec, z.to(dev), pts.to(dev), dtype="bf16").cpu().numpy()
# constant layer-0 output (xyz columns of layers 0 and 4 zeroed), identity after
p = R.make_decoder_params(seed=1234)
for l in range(1, 8):
    p.weights[l].copy_(eye_like(p.weights[l]))
p.weights[0][:, 256:] = 0
p.weights[4][:, 253 + 256:] = 0
dec = ldm_sdf.SDFDecoder(256, weights=p.weights, biases=p.biases)
dec.DEFAULT_LAYOUT = "split16"
r1 = ldm_sdf.decode_points(dec, z.to(dev), pts.to(dev), dtype="bf16").cpu().numpy()
r2 = ldm_sdf.decode_points(dec, z.to(dev), pts.to(dev), dtype="bf16").cpu().numpy()
want = R.decoder_forward_lowp(p, z.double(), pts.double(), torch.bfloat16).numpy()
print("const-h0: run-to-run max diff", float(np.abs(r1 - r2).max()), " spread over points",
      float(r1.max() - r1.min()), " gpu", r1[0, :4], " want", want[0, :4], flush=True)
out["const"] = r1
np.savez(os.path.join(ROOT, "gpurun_out", "r03f", "split16_probe.npz"), **out)
print("saved", flush=True)
