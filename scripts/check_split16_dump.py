"""CPU check of the split16 LDS dumps (scripts/dump_split16.py, -DFS16_DUMP=3..6 builds): decode
the dumped B-fragment positions of workgroup 0s first tile (32^3 grid, decoder seed 1234) and
compare them with the 16-bit-contract layer outputs computed here (DESIGN.md §4 split16
bring-up).  Reads gpurun_out/r03f/dump{3..6}.npz."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
OUT = os.path.join(ROOT, "gpurun_out")
import numpy as np, torch
from oracle import ref_cpu as R

def bf(x): return torch.as_tensor(x, dtype=torch.float32).to(torch.bfloat16).to(torch.float64).numpy()
def hilo(t): h = bf(t); return h + bf(t - h)
def dump_vals(raw):
    u16 = raw.view(np.uint16).reshape(16, 8, 64, 8)
    return (u16.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
def feat(P, l, e, one_part_late=False):
    off = 16*(e>>2) + 4*(l>>4) + (e&3)
    if one_part_late and P >= 8:
        wq = P - 8; return 64*(wq>>1) + 32*(wq&1) + off
    return 128*((P&7)>>1) + 64*(P>>3) + 32*(P&1) + off
def check(vals, Ps, H, one_part_late=False, name=""):
    errs = []
    for P in Ps:
        for n in range(8):
            for l in range(64):
                for e in range(8):
                    f = feat(P, l, e, one_part_late)
                    errs.append(abs(vals[P, n, l, e] - H[f, 16*n + (l & 15)]))
    errs = np.array(errs)
    print(f"{name}: max {errs.max():.3e}  mean {errs.mean():.3e}  n>1e-2: {(errs > 1e-2).sum()} / {len(errs)}")

p = R.make_decoder_params(seed=1234)
d = {k: dict(np.load(os.path.join(OUT, "r03f", f"dump{k}.npz"))) for k in (3, 4, 5, 6)}
z = torch.from_numpy(d[3]["z"]).double()
xyz = R.grid_coords(32, 0, 32).numpy()[:128].astype(np.float64)
beta = R.latent_fold(p, z).numpy()[0]
x3 = hilo(xyz)
h = {}
h[0] = np.maximum(bf(x3 @ bf(p.weights[0][:, 256:259].numpy()).T + hilo(beta[0])), 0).T   # [512, 128]
for l in (1, 2, 3):
    W = bf(p.weights[l].numpy()); b = p.biases[l].numpy().astype(np.float32).astype(np.float64)
    h[l] = np.maximum(bf(W @ h[l-1] + b[:, None]), 0)
h3p = np.zeros((256, 128)); h3p[:253] = h[3]
W4 = p.weights[4].numpy()
a4 = bf(W4[:, :253]) @ h[3] + (x3 @ bf(W4[:, 253+256:]).T).T + hilo(beta[1])[:, None]
h[4] = np.maximum(bf(a4), 0)
v = {k: dump_vals(d[k]["raw"]) for k in d}
check(v[3], range(0, 8), h[1], name="dump3 pos0-7 = h1 u0")
check(v[3], range(8, 16), h[1], name="dump3 pos8-15 = h1 u1")
check(v[4], range(0, 8), h[2], name="dump4 pos0-7 = h2 u0")
check(v[4], range(8, 16), h[1], name="dump4 pos8-15 = h1 u1")
check(v[5], range(0, 8), h[2], name="dump5 pos0-7 = h2 u0")
check(v[5], range(8, 16), h3p, one_part_late=True, name="dump5 pos8-15 = h3")
check(v[6], range(0, 8), h[4], name="dump6 pos0-7 = h4 u0")
check(v[6], range(8, 16), h3p, one_part_late=True, name="dump6 pos8-15 = h3")
