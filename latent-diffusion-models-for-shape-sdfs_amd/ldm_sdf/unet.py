"""C17: 1D-UNet eps-denoiser over a latent code seen as a 1-channel signal (config 5:
1024-d latents).  Architecture: DESIGN.md §9 (the same network as ``oracle/ref_unet.py``).

Every conv runs in ``ldm_conv1d`` (``csrc/unet.hip``); a reverse step is 18 launches:

    conv_in | Res_0 (2) | down0 | Res_1 (2) | down1 | Res_2 (2) | Res_3 (2) | up1 |
    Res_4 (2, concat as two segments) | up0 | Res_5 (2) | conv_out + DDPM step (A8)

The timestep-embedding MLP and each block's projection are tabulated for all t once per
weight version (``E_i[t] = P_i temb(t) + b1_i``, fp32 ``[T, Cout_i]``), so a sampling step
reads one table row per block as a per-channel bias (A5's table trick, as for the MLP).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch

from . import _capi as capi
from . import ops
from .models import timestep_embedding_table


def unet_res_specs(C: Tuple[int, int, int]) -> List[Tuple[int, int]]:
    """(cin, cout) of the six residual blocks in execution order."""
    c0, c1, c2 = C
    return [(c0, c0), (c1, c1), (c2, c2), (c2, c2), (2 * c1, c1), (2 * c0, c0)]


class UNet1DDenoiser:
    """eps-prediction 1D-UNet (D divisible by 4; channels ``C = (c0, c1, c2)``).

    ``params`` are fp32 master tensors named as in ``oracle/ref_unet.py``; the initialiser
    draws them in the same order from the same generator, so one seed is one network on
    both sides.
    """

    def __init__(self, D: int = 1024, C: Tuple[int, int, int] = (32, 64, 128), TE: int = 128,
                 HT: int = 512, T: int = 1000, seed: int = 2468,
                 params: Optional[Dict[str, torch.Tensor]] = None):
        if D % 4:
            raise ValueError("UNet1D needs D divisible by 4 (two stride-2 levels)")
        self.D, self.C, self.TE, self.HT, self.T = D, tuple(C), TE, HT, T
        if params is None:
            params = self._init(seed)
        self.params = {k: v.detach().to("cpu", torch.float32).contiguous()
                       for k, v in params.items()}
        self.emb_table = torch.from_numpy(timestep_embedding_table(T, TE))
        self._dev: Dict[Tuple[str, torch.device], Dict[str, object]] = {}

    def _init(self, seed: int) -> Dict[str, torch.Tensor]:
        g = torch.Generator().manual_seed(seed)
        p: Dict[str, torch.Tensor] = {}

        def w(name, shape, fan_in, gain=1.0):
            p[name] = torch.randn(*shape, generator=g, dtype=torch.float64) * math.sqrt(gain / fan_in)

        def b(name, n):
            p[name] = torch.randn(n, generator=g, dtype=torch.float64) * 0.01

        c0, c1, c2 = self.C
        HT, TE = self.HT, self.TE
        w("Wt1", (HT, TE), TE); b("bt1", HT)
        w("Wt2", (HT, HT), HT); b("bt2", HT)
        w("conv_in.w", (c0, 1, 3), 3, 2.0); b("conv_in.b", c0)
        for i, (ci, co) in enumerate(unet_res_specs(self.C)):
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
        return p

    def n_params(self) -> int:
        return sum(v.numel() for v in self.params.values())

    def conv_list(self) -> List[Tuple[str, int, int, int, int, int, bool]]:
        """The 18 convs of one forward, in launch order: (name, cin (all segments, the 1x1
        shortcut's included as k=1 taps below), cout, k, L_in, L_out, identity residual)."""
        c0, c1, c2 = self.C
        D = self.D
        out = [("conv_in", 1, c0, 3, D, D, False)]
        lv = {0: (c0, D), 1: (c1, D // 2), 2: (c2, D // 4), 3: (c2, D // 4), 4: (c1, D // 2),
              5: (c0, D)}

        def res(i):
            ci, co = unet_res_specs(self.C)[i]
            L = lv[i][1]
            out.append((f"res{i}.w1", ci, co, 3, L, L, False))
            out.append((f"res{i}.w2", co, co, 3, L, L, ci == co))
            if ci != co:
                out.append((f"res{i}.ws", ci, co, 1, L, L, False))
        res(0)
        out.append(("down0", c0, c1, 3, D, D // 2, False))
        res(1)
        out.append(("down1", c1, c2, 3, D // 2, D // 4, False))
        res(2)
        res(3)
        out.append(("up1", c2, c1, 3, D // 4, D // 2, False))
        res(4)
        out.append(("up0", c1, c0, 3, D // 2, D, False))
        res(5)
        out.append(("conv_out", c0, 1, 3, D, D, False))
        return out

    def step_cost(self, n: int, weight_bytes: int = 2) -> Dict[str, float]:
        """Algorithmic work of one reverse step at batch ``n`` (bench.py config5.unet_roofline):
        FLOPs = 2 n Cout L_out Cin k summed over the convs (the 1x1 shortcuts are segments of
        their block's second conv: 18 launches); bytes = every weight once (``weight_bytes`` per
        element) + every fp32 activation a conv reads (input window, identity residual) and
        writes, + the latent in / out of the step."""
        flops = 0
        wbytes = 0
        abytes = 0
        for (_, ci, co, k, Lin, Lout, ident) in self.conv_list():
            flops += 2 * n * co * Lout * ci * k
            wbytes += weight_bytes * co * ci * k
            abytes += 4 * n * (ci * Lin + co * Lout + (co * Lout if ident else 0))
        return {"flops": float(flops), "bytes": float(wbytes + abytes),
                "weight_bytes": float(wbytes), "activation_bytes": float(abytes),
                "launches": 18}

    def invalidate(self) -> None:
        self._dev.clear()

    # ------------------------------------------------------------------------- device pack
    def device_pack(self, dtype: str, device) -> Dict[str, object]:
        """Weights in ``dtype`` (fp32 | bf16; biases fp32) on ``device`` plus the per-block
        E tables ``[T, Cout_i]`` computed on the device (ldm_linear)."""
        device = torch.device(device)
        key = (dtype, device)
        if key in self._dev:
            return self._dev[key]
        wdt = {"fp32": torch.float32, "bf16": torch.bfloat16}[dtype]
        dev: Dict[str, object] = {}
        for n, v in self.params.items():
            v = v.to(device)
            if n.endswith((".w", ".w1", ".w2", ".ws")):        # conv: matrix-core packing
                dev[n] = ops.pack_conv_weight(v.to(wdt))
            elif n.startswith("W") or n.endswith(".p"):       # linear [out][in]
                dev[n] = v.to(wdt).contiguous()
            else:
                dev[n] = v.to(torch.float32).contiguous()
        emb = self.emb_table.to(device).contiguous()
        temb = ops.temb_forward(dev, emb, self.HT)                      # [T, HT]
        for i, (_, co) in enumerate(unet_res_specs(self.C)):
            E = torch.empty(self.T, co, device=device, dtype=torch.float32)
            ops.linear(temb, dev[f"res{i}.p"], E, epi=capi.EPI_BIAS, bias=dev[f"res{i}.b1"])
            dev[f"etab{i}"] = E
        self._dev[key] = dev
        return dev

    # ------------------------------------------------------------------------- forward
    def buffers(self, n: int, device) -> Dict[str, torch.Tensor]:
        """Activation buffers for a batch of ``n`` (allocated once per sampler)."""
        c0, c1, c2 = self.C
        D = self.D
        f = lambda *s: torch.empty(*s, device=device, dtype=torch.float32)  # noqa: E731
        b = {"h0": f(n, c0, D), "a0": f(n, c0, D), "s0": f(n, c0, D),
             "d0": f(n, c1, D // 2), "a1": f(n, c1, D // 2), "s1": f(n, c1, D // 2),
             "d1": f(n, c2, D // 4), "a2": f(n, c2, D // 4), "m0": f(n, c2, D // 4),
             "m1": f(n, c2, D // 4), "u1": f(n, c1, D // 2), "a4": f(n, c1, D // 2),
             "r4": f(n, c1, D // 2), "u0": f(n, c0, D), "a5": f(n, c0, D),
             "r5": f(n, c0, D), "eps": f(n, 1, D)}
        if n == 1:
            # the decoder-side skip concats [u || s] as ONE buffer whose halves the producers
            # write: res4 / res5 then read it as one segment (one staging segment fewer in
            # their two convs); a channel slice is contiguous only at n = 1
            for lvl, c in ((1, c1), (0, c0)):
                cat = f(1, 2 * c, D >> lvl)
                b[f"cat{lvl}"], b[f"u{lvl}"], b[f"s{lvl}"] = cat, cat[:, :c], cat[:, c:]
        return b

    def step_args(self, dev: Dict[str, object], buf: Dict[str, torch.Tensor], x: torch.Tensor,
                  t: int, *, out: torch.Tensor, sched=None, z: Optional[torch.Tensor] = None,
                  cbias: Optional[List[torch.Tensor]] = None) -> List[capi.ConvArgs]:
        """The 18 ``ldm_conv1d`` calls of one forward at a batch-uniform ``t``.

        With ``sched`` the last call writes the A8 reverse step ``x_{t-1}`` into ``out``
        ([n, D]); without, it writes eps_hat.  ``cbias`` overrides the tabulated per-block
        bias rows (training: per-sample ``[n, Cout_i]``)."""
        S = ops.ConvSegment
        UP2 = capi.CONV_UP2
        n = x.shape[0]
        calls: List[capi.ConvArgs] = []

        def cb(i):
            if cbias is not None:
                return dict(cbias=cbias[i], scb=cbias[i].shape[1])
            return dict(cbias=dev[f"etab{i}"][t], scb=0)

        def res(i, xin: List[torch.Tensor], a, y):
            w1, w2 = dev[f"res{i}.w1"], dev[f"res{i}.w2"]
            segs, off = [], 0
            for xi in xin:
                segs.append(S(xi, w1, c_off=off, silu=True))
                off += xi.shape[1]
            calls.append(ops.conv1d_args(segs, a, **cb(i)))
            segs2 = [S(a, w2, silu=True)]
            if f"res{i}.ws" in dev:
                ws, off = dev[f"res{i}.ws"], 0
                for xi in xin:
                    segs2.append(S(xi, ws, c_off=off))
                    off += xi.shape[1]
                calls.append(ops.conv1d_args(segs2, y, bias=dev[f"res{i}.b2"],
                                             bias2=dev[f"res{i}.bs"]))
            else:
                calls.append(ops.conv1d_args(segs2, y, bias=dev[f"res{i}.b2"], R=xin[0]))

        b = buf
        x3 = x.view(n, 1, self.D)
        calls.append(ops.conv1d_args([S(x3, dev["conv_in.w"])], b["h0"], bias=dev["conv_in.b"]))
        res(0, [b["h0"]], b["a0"], b["s0"])
        calls.append(ops.conv1d_args([S(b["s0"], dev["down0.w"], stride=2)], b["d0"],
                                     bias=dev["down0.b"]))
        res(1, [b["d0"]], b["a1"], b["s1"])
        calls.append(ops.conv1d_args([S(b["s1"], dev["down1.w"], stride=2)], b["d1"],
                                     bias=dev["down1.b"]))
        res(2, [b["d1"]], b["a2"], b["m0"])
        res(3, [b["m0"]], b["a2"], b["m1"])
        calls.append(ops.conv1d_args([S(b["m1"], dev["up1.w"], mode=UP2)], b["u1"],
                                     bias=dev["up1.b"]))
        res(4, [b["cat1"]] if "cat1" in b else [b["u1"], b["s1"]], b["a4"], b["r4"])
        calls.append(ops.conv1d_args([S(b["r4"], dev["up0.w"], mode=UP2)], b["u0"],
                                     bias=dev["up0.b"]))
        res(5, [b["cat0"]] if "cat0" in b else [b["u0"], b["s0"]], b["a5"], b["r5"])
        last = [S(b["r5"], dev["conv_out.w"], silu=True)]
        if sched is not None:
            calls.append(ops.conv1d_args(last, out.view(n, 1, self.D), bias=dev["conv_out.b"],
                                         epi=capi.CONV_EPI_DDPM, xlat=x, z=z, sched=sched, t=t))
        else:
            calls.append(ops.conv1d_args(last, out.view(n, 1, self.D), bias=dev["conv_out.b"]))
        return calls

    def forward_uniform_t(self, x: torch.Tensor, t: int, dtype: str = "bf16") -> torch.Tensor:
        """eps_hat = UNet(x, t) for a batch sharing one timestep (device tensors)."""
        capi.require_device(x)
        dev = self.device_pack(dtype, x.device)
        buf = self.buffers(x.shape[0], x.device)
        eps = torch.empty(x.shape[0], self.D, device=x.device, dtype=torch.float32)
        x = x.float().contiguous()
        for a in self.step_args(dev, buf, x, t, out=eps):
            ops.conv1d_launch(a, x.device)
        return eps

    def make_stepper(self, n: int, dtype: str, device, sched_desc):
        """Callable ``step(x, z, t, x_out)`` = one fused reverse step (for ``api.Sampler``)."""
        dev = self.device_pack(dtype, device)
        buf = self.buffers(n, device)

        def step(x, z, t, x_out):
            for a in self.step_args(dev, buf, x, t, out=x_out, sched=sched_desc, z=z):
                ops.conv1d_launch(a, device)
        return step
