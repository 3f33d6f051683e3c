"""Same-process A/B of decoder schedule variants (cdna guide §5.4 rule 24): interleaved
rounds, median + min per variant.  Usage: python scripts/ab_decoder.py [B] [N] [rounds]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
import ldm_sdf  # noqa: E402
from ldm_sdf import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
N = int(sys.argv[2]) if len(sys.argv) > 2 else 256
R = int(sys.argv[3]) if len(sys.argv) > 3 else 5
# variants: "s" = split layout (default kernel), "s<V>" (V = 1..3) = split with kernel variant
# FV = V (LDM_FS_V, needs the `make DEV=1` library: csrc/decoder_fs.hip)
VARIANTS = os.environ.get("AB_VARIANTS", "s,s2").split(",")
LAYOUT = {v: "split" for v in VARIANTS}
FLOPS = 3146752
dev = torch.device("cuda", 0)
dec = ldm_sdf.SDFDecoder(256, seed=1234)
for dtype in os.environ.get("AB_DTYPES", "bf16").split(","):
    pks = {v: dec.device_pack(dtype, dev, layout=LAYOUT[v]) for v in VARIANTS}
    z = torch.randn(B, 256, device=dev) * 0.1
    beta = ops.decoder_fold(pks[VARIANTS[0]]["desc"], z)
    out = torch.empty(B, N, N, N, device=dev)
    ref = None
    times = {v: [] for v in VARIANTS}
    for r in range(R + 1):
        for v in VARIANTS:
            if v.startswith("s") and v != "s16":
                os.environ["LDM_FS_V"] = v[1:] or "0"
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            ops.decoder_grid_fwd(pks[v]["desc"], beta, N, 0, N, out=out)
            e1.record()
            torch.cuda.synchronize()
            if r > 0:
                times[v].append(e0.elapsed_time(e1))
            if ref is None:
                ref = out.clone()
            elif not torch.equal(out, ref):
                print(f"  note: variant {v} differs from {VARIANTS[0]} by "
                      f"{float((out - ref).abs().max()):.3e} (accumulation order)")
    for v in VARIANTS:
        med = statistics.median(times[v])
        q = B * N ** 3
        print(f"{dtype} {v}: median {med:.2f} ms  min {min(times[v]):.2f} ms  "
              f"{q / med * 1e3:.3e} q/s  {q * FLOPS / med / 1e9:.1f} TF/s")
