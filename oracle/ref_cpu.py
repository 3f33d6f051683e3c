"""CPU oracle for the latent-diffusion-over-SDF hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  It is the checker (and the timed CPU baseline), never the product:
the product path in ``ldm_sdf`` runs HIP kernels through ``libldm_sdf.so`` and raises if
that library is missing.

PARITY STATUS: the reference repository (``/root/reference``) is an empty stub -- its only
file is ``README.md:1`` (a title line).  There is no reference code to import, compile or
run, and no reference fixture or golden vector.  Parity is therefore **unpinned by the
reference**.  This restatement follows SURVEY.md §8(a) rows A1-A11 line by line, which in
turn restate the published algorithms:

* DeepSDF auto-decoder MLP (Park et al., CVPR 2019): 8x512 hidden layers, latent re-injected
  at layer 4 (``latent_in=[4]``), ReLU, final tanh, input order ``[z || xyz]``.
* DDPM (Ho et al., NeurIPS 2020), Alg. 1 (training) and Alg. 2 (sampling), linear beta
  schedule 1e-4 -> 0.02, T = 1000, sigma_t^2 = beta_t ("fixedlarge").
* DDPM sinusoidal timestep embedding (``get_timestep_embedding`` convention).

Instead of reference fixtures, the oracle is pinned by known-answer tests
(``tests/test_oracle.py``): closed-form networks with analytic SDFs, exact grid corners,
schedule constants recomputed independently in exact rational / 50-digit decimal
arithmetic, and the latent-fold == concat identity.

Every function works in float64 (checker) or float32 (timed baseline) via ``dtype``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

__all__ = [
    "grid_coords", "grid_coords_np", "DecoderParams", "make_decoder_params", "latent_fold",
    "decoder_forward", "decoder_forward_folded", "decode_grid", "DDPMTables", "ddpm_tables",
    "timestep_embedding_table", "DenoiserParams", "make_denoiser_params", "denoiser_forward",
    "ddpm_step", "q_sample", "eps_mse_loss", "sample_loop", "train_step_grads",
]


# ----------------------------------------------------------------------------------------
# A1  grid_coords  
# ----------------------------------------------------------------------------------------
def grid_voxel_size(N: int, bbox: Tuple[float, float] = (-1.0, 1.0)) -> np.float32:
    """Voxel size, rounded to fp32 on the host first: ``fl32((hi-lo)/(N-1))`` (A1)."""
    lo, hi = bbox
    return np.float32((hi - lo) / (N - 1)) if N > 1 else np.float32(0.0)


def grid_coords_np(N: int, k0: int = 0, k1: Optional[int] = None,
                   bbox: Tuple[float, float] = (-1.0, 1.0)) -> np.ndarray:
    """Dense grid coordinates, float32 ``[ (k1-k0)*N*N, 3 ]`` (A1).

    Flat index ``p`` over the slab: z slowest, x fastest (``i = p % N``, ``j = (p // N) % N``,
    ``k = k0 + p // N^2``).  ``x = fl32(fl32(i * vs) + origin)`` -- two roundings, no FMA.
    DeepSDF's own ``create_mesh`` enumerates x slowest; here it is the documented transpose
    (SURVEY.md §8(a) A1).
    """
    if k1 is None:
        k1 = N
    vs = grid_voxel_size(N, bbox)
    origin = np.float32(bbox[0])
    idx = np.arange(N, dtype=np.float32)
    line = (idx * vs).astype(np.float32) + origin          # fp32 mul, then fp32 add
    line = line.astype(np.float32)
    k = np.arange(k0, k1)
    zz, yy, xx = np.meshgrid(line[k], line, line, indexing="ij")
    return np.stack([xx.ravel(), yy.ravel(), zz.ravel()], axis=1).astype(np.float32)


def grid_coords(N: int, k0: int = 0, k1: Optional[int] = None,
                bbox: Tuple[float, float] = (-1.0, 1.0)) -> torch.Tensor:
    return torch.from_numpy(grid_coords_np(N, k0, k1, bbox))


# ----------------------------------------------------------------------------------------
# A2/A3  DeepSDF decoder
# ----------------------------------------------------------------------------------------
@dataclass
class DecoderParams:
    """Canonical (unfolded, weight-norm already folded) DeepSDF decoder weights.

    ``weights[l]`` is ``[out_l, in_l]`` (torch ``nn.Linear`` convention), ``biases[l]`` is
    ``[out_l]``.  Layer 0 input is ``[z || xyz]`` (L+3); layer ``skip`` input is
    ``[h || z || xyz]``; the last layer maps H -> 1 followed by tanh.
    """
    latent_dim: int
    hidden: int
    n_hidden: int          # number of hidden layers (8 in DeepSDF) -> n_hidden+1 linears
    skip: int              # layer index that re-injects [z||xyz] (4 in DeepSDF)
    widen_skip: bool
    weights: List[torch.Tensor] = field(default_factory=list)
    biases: List[torch.Tensor] = field(default_factory=list)

    @property
    def n_linear(self) -> int:
        return self.n_hidden + 1

    def layer_dims(self) -> List[Tuple[int, int]]:
        return decoder_layer_dims(self.latent_dim, self.hidden, self.n_hidden, self.skip,
                                  self.widen_skip)

    def to(self, dtype) -> "DecoderParams":
        return DecoderParams(self.latent_dim, self.hidden, self.n_hidden, self.skip,
                             self.widen_skip, [w.to(dtype) for w in self.weights],
                             [b.to(dtype) for b in self.biases])


def decoder_layer_dims(L: int, H: int, n_hidden: int = 8, skip: int = 4,
                       widen_skip: bool = False) -> List[Tuple[int, int]]:
    """(in, out) per linear.  DeepSDF: layer skip-1 outputs ``H - (L+3)`` so that the
    re-injected input restores width H; ``widen_skip`` (config 5, L >= H) keeps H and widens
    layer ``skip``'s input to ``H + L + 3`` instead (SURVEY.md §7 'Config 5 geometry')."""
    dims = []
    d_in = L + 3
    for l in range(n_hidden):
        if l + 1 == skip:
            out = H if widen_skip else H - (L + 3)
            if out <= 0:
                raise ValueError(f"latent {L} too wide for hidden {H}; use widen_skip=True")
        else:
            out = H
        inp = d_in if l != skip else d_in + L + 3
        dims.append((inp, out))
        d_in = out
    dims.append((d_in, 1))
    return dims


def make_decoder_params(L: int = 256, H: int = 512, n_hidden: int = 8, skip: int = 4,
                        widen_skip: bool = False, seed: int = 1234,
                        dtype=torch.float64) -> DecoderParams:
    """He-normal weights N(0, 2/fan_in), biases N(0, 0.01^2): keeps the
    activations O(1) so the fp tolerances are meaningful."""
    g = torch.Generator().manual_seed(seed)
    ws, bs = [], []
    for (i, o) in decoder_layer_dims(L, H, n_hidden, skip, widen_skip):
        ws.append(torch.randn(o, i, generator=g, dtype=torch.float64) * math.sqrt(2.0 / i))
        bs.append(torch.randn(o, generator=g, dtype=torch.float64) * 0.01)
    return DecoderParams(L, H, n_hidden, skip, widen_skip,
                         [w.to(dtype) for w in ws], [b.to(dtype) for b in bs])


def decoder_forward(p: DecoderParams, z: torch.Tensor, xyz: torch.Tensor) -> torch.Tensor:
    """Canonical concat formulation (DeepSDF ``Decoder.forward`` in eval mode).

    z: [B, L] or [L]; xyz: [P, 3] shared or [B, P, 3].  Returns [B, P].
    """
    if z.dim() == 1:
        z = z[None]
    B = z.shape[0]
    if xyz.dim() == 2:
        xyz = xyz[None].expand(B, -1, -1)
    P = xyz.shape[1]
    inp = torch.cat([z[:, None, :].expand(B, P, z.shape[1]), xyz.to(z.dtype)], dim=2)
    inp = inp.reshape(B * P, -1)
    x = inp
    for l in range(p.n_linear):
        if l == p.skip:
            x = torch.cat([x, inp], dim=1)
        x = x @ p.weights[l].T + p.biases[l]
        if l < p.n_linear - 1:
            x = torch.relu(x)
    return torch.tanh(x).reshape(B, P)


def latent_fold(p: DecoderParams, z: torch.Tensor) -> torch.Tensor:
    """A2: per-shape biases ``beta[b,0] = W0[:, :L] z + b0`` and
    ``beta[b,1] = W_skip[:, h:h+L] z + b_skip`` (column order ``[h || z || xyz]``).
    Returns ``[B, 2, H]``."""
    if z.dim() == 1:
        z = z[None]
    L = p.latent_dim
    W0, b0 = p.weights[0], p.biases[0]
    Ws, bsk = p.weights[p.skip], p.biases[p.skip]
    hin = Ws.shape[1] - (L + 3)
    beta0 = z @ W0[:, :L].T + b0
    beta4 = z @ Ws[:, hin:hin + L].T + bsk
    return torch.stack([beta0, beta4], dim=1)


def decoder_forward_folded(p: DecoderParams, beta: torch.Tensor,
                           xyz: torch.Tensor) -> torch.Tensor:
    """A3 with the latent folded into per-shape biases (what the HIP kernels compute).

    beta: [B, 2, H]; xyz: [P, 3] shared or [B, P, 3].  Returns [B, P].
    """
    B = beta.shape[0]
    L = p.latent_dim
    if xyz.dim() == 2:
        xyz = xyz[None].expand(B, -1, -1)
    out = []
    Ws = p.weights[p.skip]
    hin = Ws.shape[1] - (L + 3)
    for b in range(B):
        x3 = xyz[b].to(beta.dtype)
        h = torch.relu(x3 @ p.weights[0][:, L:L + 3].T + beta[b, 0])
        for l in range(1, p.n_linear):
            if l == p.skip:
                h = h @ Ws[:, :hin].T + x3 @ Ws[:, hin + L:].T + beta[b, 1]
            else:
                h = h @ p.weights[l].T + p.biases[l]
            if l < p.n_linear - 1:
                h = torch.relu(h)
        out.append(torch.tanh(h[:, 0]))
    return torch.stack(out, 0)


def decoder_forward_lowp(p: DecoderParams, z: torch.Tensor, xyz: torch.Tensor,
                         dt: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """A3 at the perf kernels' 16-bit precision contract (SURVEY.md §8(a) A3 "bf16/fp16 in,
    fp32 acc"), evaluated in fp64: every weight matrix rounded to ``dt`` (RNE); every hidden
    activation that feeds a matrix product rounded to ``dt`` after its layer (ReLU commutes
    with the rounding); xyz and the folded biases beta (and the layer biases) enter as a ``dt``
    hi + lo pair (~16 significant bits, DESIGN.md §3 'aux k-step'); the last hidden layer stays
    unrounded (the 512 -> 1 layer is an fp32 dot with fp32 weights).  What is left between
    this and the device is fp32 accumulation order only, so it pins the bf16/fp16 kernels far
    tighter than the fp64 decoder can when the latents are large (their rounding error grows
    with the activations' scale).  z: [B, L]; xyz: [P, 3] shared or [B, P, 3] -> [B, P]."""
    def rd(t):
        return t.to(torch.float32).to(dt).to(torch.float64)

    def hilo(t):
        hi = rd(t)
        return hi + rd(t.to(torch.float64) - hi)

    if z.dim() == 1:
        z = z[None]
    B = z.shape[0]
    L = p.latent_dim
    if xyz.dim() == 2:
        xyz = xyz[None].expand(B, -1, -1)
    beta = hilo(latent_fold(p, z.to(torch.float64)))
    Ws = p.weights[p.skip]
    hin = Ws.shape[1] - (L + 3)
    out = []
    for b in range(B):
        x3 = hilo(xyz[b].to(torch.float64))
        h = torch.relu(x3 @ rd(p.weights[0][:, L:L + 3]).T + beta[b, 0])
        for l in range(1, p.n_linear):
            if l == p.skip:
                a = rd(h) @ rd(Ws[:, :hin]).T + x3 @ rd(Ws[:, hin + L:]).T + beta[b, 1]
            elif l == p.n_linear - 1:
                a = h @ p.weights[l].to(torch.float32).to(torch.float64).T \
                    + p.biases[l].to(torch.float32).to(torch.float64)
            else:
                a = rd(h) @ rd(p.weights[l]).T + hilo(p.biases[l])
            h = torch.relu(a) if l < p.n_linear - 1 else a
        out.append(torch.tanh(h[:, 0]))
    return torch.stack(out, 0)


def decode_grid(p: DecoderParams, z: torch.Tensor, N: int, k0: int = 0,
                k1: Optional[int] = None, chunk: int = 262144,
                bbox: Tuple[float, float] = (-1.0, 1.0)) -> torch.Tensor:
    """CPU decode of a (slab of a) dense grid, chunked (SURVEY.md §8(d) CPU baseline).
    Returns ``[B, k1-k0, N, N]`` in ``p``'s dtype."""
    if k1 is None:
        k1 = N
    if z.dim() == 1:
        z = z[None]
    xyz = grid_coords(N, k0, k1, bbox)
    beta = latent_fold(p, z.to(p.weights[0].dtype))
    outs = []
    with torch.inference_mode():
        for s in range(0, xyz.shape[0], chunk):
            outs.append(decoder_forward_folded(p, beta, xyz[s:s + chunk]))
    return torch.cat(outs, dim=1).reshape(z.shape[0], k1 - k0, N, N)


# ----------------------------------------------------------------------------------------
# A4  DDPM schedule, A5 timestep embedding
# ----------------------------------------------------------------------------------------
@dataclass
class DDPMTables:
    T: int
    betas: np.ndarray           # fp64 [T]
    alphas: np.ndarray
    alphas_cumprod: np.ndarray
    sqrt_ab: np.ndarray         # sqrt(abar)
    sqrt_1mab: np.ndarray       # sqrt(1 - abar)
    c1: np.ndarray              # 1/sqrt(alpha)
    c2: np.ndarray              # beta / sqrt(1 - abar)
    sigma: np.ndarray           # sqrt(beta)         ("fixedlarge")
    sigma_small: np.ndarray     # sqrt(beta_tilde)   ("fixedsmall", optional)

    def f32(self, name: str) -> np.ndarray:
        return getattr(self, name).astype(np.float32)


def ddpm_tables(T: int = 1000, beta_start: float = 1e-4, beta_end: float = 0.02) -> DDPMTables:
    """A4: linear schedule in fp64 on the host (DDPM §4), stored fp32 on device."""
    betas = np.linspace(beta_start, beta_end, T, dtype=np.float64)
    alphas = 1.0 - betas
    ab = np.cumprod(alphas)
    ab_prev = np.concatenate([[1.0], ab[:-1]])
    beta_tilde = betas * (1.0 - ab_prev) / (1.0 - ab)
    return DDPMTables(T, betas, alphas, ab, np.sqrt(ab), np.sqrt(1.0 - ab),
                      1.0 / np.sqrt(alphas), betas / np.sqrt(1.0 - ab), np.sqrt(betas),
                      np.sqrt(beta_tilde))


def timestep_embedding_table(T: int, dim: int = 128) -> np.ndarray:
    """A5: DDPM sinusoidal embedding for every t in [0, T): ``f_k = exp(-ln(1e4) k/(dim/2-1))``,
    ``e(t) = [sin(t f), cos(t f)]``.  fp64 -> fp32 table ``[T, dim]``."""
    half = dim // 2
    freqs = np.exp(-math.log(10000.0) * np.arange(half, dtype=np.float64) / (half - 1))
    ang = np.arange(T, dtype=np.float64)[:, None] * freqs[None, :]
    return np.concatenate([np.sin(ang), np.cos(ang)], axis=1).astype(np.float32)


# ----------------------------------------------------------------------------------------
# A6/A7  MLP denoiser
# ----------------------------------------------------------------------------------------
@dataclass
class DenoiserParams:
    """MLP denoiser (SURVEY.md §8 defaults D=256, H=1024, 4 blocks, TE=128, T=1000).

    ``e = table[t]``; ``u = SiLU(Wt1 e + bt1)``; ``temb = Wt2 u + bt2`` ([B,H]);
    ``h = Win x + bin``; per block ``a = Wblk[k] [h || temb] + bblk[k]``,
    ``h <- h + SiLU(a)``; ``eps = Wout h + bout``.  ``Wblk[k] = [W_k | U_k]`` is ``[H, 2H]`` so
    that ``U_k temb`` (A5's projected embedding) is part of the same contraction.
    """
    D: int
    H: int
    n_blocks: int
    TE: int
    Wt1: torch.Tensor
    bt1: torch.Tensor
    Wt2: torch.Tensor
    bt2: torch.Tensor
    Win: torch.Tensor
    bin: torch.Tensor
    Wblk: List[torch.Tensor]
    bblk: List[torch.Tensor]
    Wout: torch.Tensor
    bout: torch.Tensor

    def tensors(self) -> List[torch.Tensor]:
        return [self.Wt1, self.bt1, self.Wt2, self.bt2, self.Win, self.bin,
                *self.Wblk, *self.bblk, self.Wout, self.bout]

    def map(self, fn) -> "DenoiserParams":
        return DenoiserParams(self.D, self.H, self.n_blocks, self.TE, fn(self.Wt1),
                              fn(self.bt1), fn(self.Wt2), fn(self.bt2), fn(self.Win),
                              fn(self.bin), [fn(w) for w in self.Wblk],
                              [fn(b) for b in self.bblk], fn(self.Wout), fn(self.bout))


def make_denoiser_params(D: int = 256, H: int = 1024, n_blocks: int = 4, TE: int = 128,
                         seed: int = 4321, dtype=torch.float64) -> DenoiserParams:
    """Weights N(0, 1/fan_in) (block weights scaled by 1/sqrt(2 n_blocks) to keep the
    residual stream O(1)); biases N(0, 0.01^2)."""
    g = torch.Generator().manual_seed(seed)

    def lin(o, i, scale=1.0):
        w = torch.randn(o, i, generator=g, dtype=torch.float64) * (scale / math.sqrt(i))
        b = torch.randn(o, generator=g, dtype=torch.float64) * 0.01
        return w.to(dtype), b.to(dtype)

    Wt1, bt1 = lin(H, TE)
    Wt2, bt2 = lin(H, H)
    Win, bin_ = lin(H, D)
    Wblk, bblk = [], []
    for _ in range(n_blocks):
        w, b = lin(H, 2 * H, 1.0 / math.sqrt(2 * n_blocks) * math.sqrt(2.0))
        Wblk.append(w)
        bblk.append(b)
    Wout, bout = lin(D, H)
    return DenoiserParams(D, H, n_blocks, TE, Wt1, bt1, Wt2, bt2, Win, bin_, Wblk, bblk,
                          Wout, bout)


def silu(x: torch.Tensor) -> torch.Tensor:
    return x * torch.sigmoid(x)


def denoiser_forward(p: DenoiserParams, x: torch.Tensor, t: torch.Tensor,
                     emb_table: torch.Tensor) -> torch.Tensor:
    """A6 full network: eps_hat = net(x_t, t).  x: [B, D]; t: int [B]."""
    e = emb_table[t.long()].to(x.dtype)
    temb = silu(e @ p.Wt1.T + p.bt1) @ p.Wt2.T + p.bt2
    h = x @ p.Win.T + p.bin
    for k in range(p.n_blocks):
        a = torch.cat([h, temb], dim=1) @ p.Wblk[k].T + p.bblk[k]
        h = h + silu(a)
    return h @ p.Wout.T + p.bout


# ----------------------------------------------------------------------------------------
# A8  reverse step, A9 q_sample + loss, A10 sampling loop
# ----------------------------------------------------------------------------------------
def ddpm_step(tab: DDPMTables, x: torch.Tensor, eps: torch.Tensor, z: torch.Tensor,
              t: int, dtype=None) -> torch.Tensor:
    """A8: ``x' = c1[t] * (x - c2[t] * eps) + sigma[t] * z`` (z ignored at t = 0).  The op
    order is fixed; tables are the fp32-rounded values the device uses."""
    dt = dtype or x.dtype
    c1 = torch.tensor(tab.f32("c1")[t], dtype=dt)
    c2 = torch.tensor(tab.f32("c2")[t], dtype=dt)
    sg = torch.tensor(tab.f32("sigma")[t], dtype=dt)
    y = c1 * (x - c2 * eps)
    if t > 0:
        y = y + sg * z
    return y


def q_sample(tab: DDPMTables, x0: torch.Tensor, eps: torch.Tensor,
             t: torch.Tensor) -> torch.Tensor:
    """A9 forward noising ``x_t = sqrt(abar_t) x0 + sqrt(1 - abar_t) eps``."""
    a = torch.from_numpy(tab.f32("sqrt_ab")).to(x0.dtype)[t.long()][:, None]
    b = torch.from_numpy(tab.f32("sqrt_1mab")).to(x0.dtype)[t.long()][:, None]
    return a * x0 + b * eps


def eps_mse_loss(eps_hat: torch.Tensor, eps: torch.Tensor) -> torch.Tensor:
    """A9 loss ``mean((eps - eps_hat)^2)`` over B x D."""
    return ((eps - eps_hat) ** 2).mean()


def sample_loop(p: DenoiserParams, tab: DDPMTables, emb_table: torch.Tensor,
                x_T: torch.Tensor, noise: torch.Tensor, steps: Optional[int] = None,
                return_traj: bool = False):
    """A10 (DDPM Alg. 2): for t = T-1 .. T-steps: eps = net(x, t); x = step(x, eps, z_t, t).

    ``noise[t]`` is the z injected at step t (``[T, B, D]``), supplied by the caller so the
    GPU run can consume exactly the same numbers.
    """
    T = tab.T
    steps = T if steps is None else steps
    x = x_T
    traj = [x]
    with torch.inference_mode():
        for t in range(T - 1, T - 1 - steps, -1):
            tt = torch.full((x.shape[0],), t, dtype=torch.int64)
            eps = denoiser_forward(p, x, tt, emb_table)
            x = ddpm_step(tab, x, eps, noise[t], t)
            if return_traj:
                traj.append(x)
    return (x, traj) if return_traj else x


def train_step_grads(p: DenoiserParams, tab: DDPMTables, emb_table: torch.Tensor,
                     x0: torch.Tensor, eps: torch.Tensor, t: torch.Tensor):
    """A9 + A7 through autograd: returns (loss, {name: grad}) for one DDPM training step
    (DDPM Alg. 1 without the optimizer)."""
    params = p.map(lambda w: w.detach().clone().requires_grad_(True))
    with torch.enable_grad():
        xt = q_sample(tab, x0, eps, t)
        eps_hat = denoiser_forward(params, xt, t, emb_table)
        loss = eps_mse_loss(eps_hat, eps)
        loss.backward()
    names = ["Wt1", "bt1", "Wt2", "bt2", "Win", "bin", "Wout", "bout"]
    grads = {n: getattr(params, n).grad.detach() for n in names}
    for k in range(p.n_blocks):
        grads[f"Wblk{k}"] = params.Wblk[k].grad.detach()
        grads[f"bblk{k}"] = params.bblk[k].grad.detach()
    return loss.detach(), grads
