"""CPU oracle for the 1D-UNet latent denoiser.  TEST
INFRASTRUCTURE ONLY -- imported by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg, never by the product (``ldm_sdf`` runs ``ldm_conv1d`` in HIP).

PARITY STATUS: unpinned by the reference.  ``/root/reference`` holds only ``README.md:1`` (a
title line), so there is no reference UNet.  The architecture is build-defined in DESIGN.md
§9 from BASELINE.json configs[4] ("1D-UNet denoiser on 1024-d latents") and the DDPM
residual-block design (Ho et al. 2020, their ``ResnetBlock``: SiLU -> conv -> + temb
projection -> SiLU -> conv, 1x1 shortcut when widths differ), in one dimension and without
GroupNorm/dropout.  It is pinned by known-answer tests (``tests/test_unet_oracle.py``):
conv taps against hand-computed sums, identity networks, and fp32 vs fp64 agreement.

Layout: activations ``[B, C, L]`` (channels, then positions), a latent ``x [B, D]`` is
``[B, 1, D]``.  Network (channels ``C = (c0, c1, c2)``, ``D`` divisible by 4):

    temb = Wt2 SiLU(Wt1 e(t) + bt1) + bt2                         e = A5 sinusoid, [B, HT]
    h0 = conv3(x; conv_in)                                       [B, c0, D]
    r0 = Res_0(h0)            (c0 -> c0)                          skip s0
    d0 = conv3/stride2(r0)    (c0 -> c1)                          [B, c1, D/2]
    r1 = Res_1(d0)            (c1 -> c1)                          skip s1
    d1 = conv3/stride2(r1)    (c1 -> c2)                          [B, c2, D/4]
    m  = Res_3(Res_2(d1))     (c2 -> c2)
    u1 = conv3(up2(m))        (c2 -> c1)   up2 = nearest x2        [B, c1, D/2]
    r2 = Res_4([u1 || s1])    (2 c1 -> c1)
    u0 = conv3(up2(r2))       (c1 -> c0)                          [B, c0, D]
    r3 = Res_5([u0 || s0])    (2 c0 -> c0)
    eps = conv3(SiLU(r3); conv_out)   (c0 -> 1)                   [B, D]

    Res(x): a = conv3(SiLU(x); W1) + b1 + (P temb)[:, :, None]
            y = conv3(SiLU(a); W2) + b2 + (conv1(x; Ws) + bs  if cin != cout  else  x)

``conv3`` = kernel 3, padding 1 (zeros), cross-correlation as ``torch.nn.functional.conv1d``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

__all__ = ["UNetParams", "make_unet_params", "unet_res_specs", "unet_forward",
           "unet_sample_loop"]


def unet_res_specs(C: Tuple[int, int, int]) -> List[Tuple[int, int]]:
    """(cin, cout) of the six residual blocks, in execution order."""
    c0, c1, c2 = C
    return [(c0, c0), (c1, c1), (c2, c2), (c2, c2), (2 * c1, c1), (2 * c0, c0)]


@dataclass
class UNetParams:
    D: int
    C: Tuple[int, int, int]
    TE: int
    HT: int
    p: Dict[str, torch.Tensor] = field(default_factory=dict)

    def map(self, fn) -> "UNetParams":
        return UNetParams(self.D, self.C, self.TE, self.HT, {k: fn(v) for k, v in self.p.items()})


def make_unet_params(D: int = 1024, C: Tuple[int, int, int] = (32, 64, 128), TE: int = 128,
                     HT: int = 512, seed: int = 2468, dtype=torch.float64) -> UNetParams:
    """Weights ``N(0, gain/fan_in)``; each block's second conv is scaled by ``1/sqrt(12)``
    (6 residual blocks, as the MLP denoiser's ``1/sqrt(2 n_blocks)``) so the residual stream
    stays O(1); biases ``N(0, 0.01^2)``.  The same generator order as
    ``ldm_sdf.UNet1DDenoiser`` (so a seed names one network on both sides)."""
    g = torch.Generator().manual_seed(seed)
    p: Dict[str, torch.Tensor] = {}

    def w(name, shape, fan_in, gain=1.0):
        p[name] = (torch.randn(*shape, generator=g, dtype=torch.float64)
                   * math.sqrt(gain / fan_in)).to(dtype)

    def b(name, n):
        p[name] = (torch.randn(n, generator=g, dtype=torch.float64) * 0.01).to(dtype)

    c0, c1, c2 = C
    w("Wt1", (HT, TE), TE); b("bt1", HT)
    w("Wt2", (HT, HT), HT); b("bt2", HT)
    w("conv_in.w", (c0, 1, 3), 3, 2.0); b("conv_in.b", c0)
    for i, (ci, co) in enumerate(unet_res_specs(C)):
        w(f"res{i}.w1", (co, ci, 3), 3 * ci, 2.0); b(f"res{i}.b1", co)
        w(f"res{i}.p", (co, HT), HT)
        w(f"res{i}.w2", (co, co, 3), 3 * co, 2.0 / 12.0); b(f"res{i}.b2", co)
        if ci != co:
            w(f"res{i}.ws", (co, ci, 1), ci); b(f"res{i}.bs", co)
    w("down0.w", (c1, c0, 3), 3 * c0); b("down0.b", c1)
    w("down1.w", (c2, c1, 3), 3 * c1); b("down1.b", c2)
    w("up1.w", (c1, c2, 3), 3 * c2); b("up1.b", c1)
    w("up0.w", (c0, c1, 3), 3 * c1); b("up0.b", c0)
    w("conv_out.w", (1, c0, 3), 3 * c0); b("conv_out.b", 1)
    return UNetParams(D, tuple(C), TE, HT, p)


def silu(x: torch.Tensor) -> torch.Tensor:
    return x * torch.sigmoid(x)


def time_mlp(up: UNetParams, t: torch.Tensor, emb_table: torch.Tensor) -> torch.Tensor:
    p = up.p
    e = emb_table[t.long()].to(p["Wt1"].dtype)
    return silu(e @ p["Wt1"].T + p["bt1"]) @ p["Wt2"].T + p["bt2"]


def _res(p: Dict[str, torch.Tensor], i: int, x: torch.Tensor, temb: torch.Tensor):
    a = F.conv1d(silu(x), p[f"res{i}.w1"], p[f"res{i}.b1"], padding=1)
    a = a + (temb @ p[f"res{i}.p"].T)[:, :, None]
    y = F.conv1d(silu(a), p[f"res{i}.w2"], p[f"res{i}.b2"], padding=1)
    if f"res{i}.ws" in p:
        return y + F.conv1d(x, p[f"res{i}.ws"], p[f"res{i}.bs"])
    return y + x


def unet_forward(up: UNetParams, x: torch.Tensor, t: torch.Tensor,
                 emb_table: torch.Tensor) -> torch.Tensor:
    """eps_hat = UNet(x_t, t): ``x [B, D]``, ``t`` int ``[B]`` -> ``[B, D]``."""
    p = up.p
    temb = time_mlp(up, t, emb_table)
    h = F.conv1d(x[:, None, :], p["conv_in.w"], p["conv_in.b"], padding=1)
    s0 = _res(p, 0, h, temb)
    h = F.conv1d(s0, p["down0.w"], p["down0.b"], stride=2, padding=1)
    s1 = _res(p, 1, h, temb)
    h = F.conv1d(s1, p["down1.w"], p["down1.b"], stride=2, padding=1)
    h = _res(p, 3, _res(p, 2, h, temb), temb)
    h = F.conv1d(F.interpolate(h, scale_factor=2, mode="nearest"), p["up1.w"], p["up1.b"],
                 padding=1)
    h = _res(p, 4, torch.cat([h, s1], dim=1), temb)
    h = F.conv1d(F.interpolate(h, scale_factor=2, mode="nearest"), p["up0.w"], p["up0.b"],
                 padding=1)
    h = _res(p, 5, torch.cat([h, s0], dim=1), temb)
    return F.conv1d(silu(h), p["conv_out.w"], p["conv_out.b"], padding=1)[:, 0, :]


def unet_sample_loop(up: UNetParams, tab, emb_table: torch.Tensor, x_T: torch.Tensor,
                     noise: torch.Tensor, steps=None) -> torch.Tensor:
    """A10 with the UNet as the denoiser (DDPM Alg. 2); ``tab`` is ``ref_cpu.ddpm_tables()``."""
    from .ref_cpu import ddpm_step
    T = tab.T
    steps = T if steps is None else steps
    x = x_T
    with torch.inference_mode():
        for t in range(T - 1, T - 1 - steps, -1):
            tt = torch.full((x.shape[0],), t, dtype=torch.int64)
            x = ddpm_step(tab, x, unet_forward(up, x, tt, emb_table), noise[t], t)
    return x
