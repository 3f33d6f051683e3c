"""Matrix-core ldm_linear (compute=BF16) error per layout, against the fp64 product of the
bf16-rounded operands.  Run twice (LDM_LINEAR_VEC=0 / 1) to A/B the vector-load tiles."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "latent-diffusion-models-for-shape-sdfs_amd")]
import torch  # noqa: E402
from ldm_sdf import ops, _capi as capi  # noqa: E402

dev = torch.device("cuda", 0)
BF = capi.COMPUTE_BF16


def bf(t):
    return t.float().bfloat16().double()


print("LDM_LINEAR_VEC =", os.environ.get("LDM_LINEAR_VEC", "(unset)"))
g = torch.Generator().manual_seed(5)
for Bn, M, K in [(64, 64, 64), (64, 64, 128), (128, 128, 256), (1000, 1024, 1024)]:
    for wdt in (torch.float32, torch.bfloat16):
        X = torch.randn(Bn, K, generator=g).to(dev)
        W = torch.randn(M, K, generator=g).to(dev).to(wdt)
        G = torch.randn(Bn, M, generator=g).to(dev)
        Y = torch.full((Bn, M), float("nan"), device=dev)
        ops.linear(X, W, Y, compute=BF)
        e_fwd = (Y.double() - bf(X) @ bf(W).T).abs().max().item()
        dW = torch.full((M, K), float("nan"), device=dev)
        ops.linear(G.T, X.T, dW, compute=BF)
        e_dw = (dW.double() - bf(G).T @ bf(X)).abs().max().item()
        dX = torch.full((Bn, K), float("nan"), device=dev)
        ops.linear(G, W.T, dX, compute=BF)
        e_dx = (dX.double() - bf(G) @ bf(W)).abs().max().item()
        print(f"{Bn:5d} {M:5d} {K:5d} {str(wdt):15s} fwd {e_fwd:.3e} dW {e_dw:.3e} dX {e_dx:.3e}",
              flush=True)
