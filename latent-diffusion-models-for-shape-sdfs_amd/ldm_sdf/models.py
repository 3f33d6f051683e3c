"""Model containers for the hot path: parameters on the host in canonical
form, plus device-resident packed copies handed to ``libldm_sdf.so`` as POD descriptors.

* ``SDFDecoder``   -- DeepSDF auto-decoder MLP (8x512, latent re-injected at layer 4, tanh).
* ``DDPMSchedule`` -- linear-beta DDPM tables (A4), computed in fp64, stored fp32.
* ``MLPDenoiser``  -- eps-prediction MLP over latent codes with timestep-embedded residual
                      blocks (A5/A6): ``h <- h + SiLU(W_k h + U_k temb(t) + b_k)``.

Canonical parameter shapes follow ``torch.nn.Linear`` (``[out, in]``).  Initialisers match
``oracle/ref_cpu.py`` (He-normal decoder, 1/sqrt(fan_in) denoiser) so synthetic benchmark
weights and test weights are the same family.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _capi as capi
from .pack import pack_decoder

# ----------------------------------------------------------------------------------------
# decoder
# ----------------------------------------------------------------------------------------


def decoder_layer_dims(L: int, H: int = 512, n_hidden: int = 8, skip: int = 4,
                       widen_skip: bool = False) -> List[Tuple[int, int]]:
    """(in, out) per linear -- DeepSDF ``Decoder.__init__`` with ``latent_in=[skip]``.
    ``widen_skip`` (needed when L+3 >= H, config 5) keeps layer skip-1 at width H and widens
    layer skip's input to H + L + 3 instead."""
    dims = []
    d_in = L + 3
    for l in range(n_hidden):
        if l + 1 == skip:
            out = H if widen_skip else H - (L + 3)
            if out <= 0:
                raise ValueError(f"latent {L} too wide for hidden {H}: use widen_skip=True")
        else:
            out = H
        dims.append((d_in + (L + 3 if l == skip else 0), out))
        d_in = out
    dims.append((d_in, 1))
    return dims


class SDFDecoder:
    """DeepSDF decoder.  ``weights[l]``/``biases[l]`` are canonical fp32 CPU tensors."""

    def __init__(self, latent_dim: int = 256, hidden: int = 512, n_hidden: int = 8,
                 skip: int = 4, widen_skip: Optional[bool] = None,
                 weights: Optional[List[torch.Tensor]] = None,
                 biases: Optional[List[torch.Tensor]] = None, seed: int = 1234):
        if widen_skip is None:
            widen_skip = latent_dim + 3 >= hidden
        self.latent_dim, self.hidden, self.n_hidden, self.skip = latent_dim, hidden, n_hidden, skip
        self.widen_skip = widen_skip
        dims = decoder_layer_dims(latent_dim, hidden, n_hidden, skip, widen_skip)
        if weights is None:
            g = torch.Generator().manual_seed(seed)
            weights, biases = [], []
            for (i, o) in dims:   # He-normal
                weights.append(torch.randn(o, i, generator=g, dtype=torch.float64)
                               * math.sqrt(2.0 / i))
                biases.append(torch.randn(o, generator=g, dtype=torch.float64) * 0.01)
        for l, (i, o) in enumerate(dims):
            if tuple(weights[l].shape) != (o, i) or tuple(biases[l].shape) != (o,):
                raise ValueError(f"layer {l}: expected W[{o},{i}], b[{o}]")
        self.weights = [w.detach().to("cpu", torch.float32).contiguous() for w in weights]
        self.biases = [b.detach().to("cpu", torch.float32).contiguous() for b in biases]
        self._dev: Dict[Tuple[str, torch.device, str], Dict[str, object]] = {}

    @property
    def skip_width(self) -> int:
        return self.weights[self.skip - 1].shape[0]

    def gpu_supported(self) -> bool:
        return (self.hidden == 512 and self.n_hidden == 8 and self.skip == 4
                and self.skip_width in (253, 512))

    # the feature-split kernel (csrc/decoder_fs.hip; the 16x16x32 "split16" variant was deleted
    # in ABI 7, 5.5 % slower)
    DEFAULT_LAYOUT = "split"

    def invalidate(self) -> None:
        """Call after the weights changed (auto-decoder training): drops the packed copies."""
        self._dev.clear()

    def device_pack(self, dtype: str, device: torch.device,
                    layout: Optional[str] = None) -> Dict[str, object]:
        """Packed device arrays + ``ldm_decoder_t`` (cached per dtype/device/layout)."""
        device = torch.device(device)
        layout = layout or self.DEFAULT_LAYOUT
        key = (dtype, device, layout)
        if key not in self._dev:
            if not self.gpu_supported():
                raise capi.LdmError("GPU decoder kernels support DeepSDF 8x512 with skip at 4")
            host = pack_decoder(self.weights, self.biases, self.latent_dim, dtype, layout)
            dev = {k: (v.to(device) if isinstance(v, torch.Tensor) else v)
                   for k, v in host.items()}
            desc = capi.Decoder()
            desc.abi_version = capi.ABI_VERSION
            desc.dtype = capi.DTYPE_CODES[dtype]
            desc.hidden = self.hidden
            desc.skip_width = host["skip_width"]
            desc.latent_dim = self.latent_dim
            desc.n_stages = host["n_stages"]
            desc.weights = dev["weights"].data_ptr()
            desc.wz = dev["wz"].data_ptr()
            desc.bz = dev["bz"].data_ptr()
            desc.wxyz = dev["wxyz"].data_ptr()
            desc.w_last = dev["w_last"].data_ptr()
            desc.b_last = host["b_last"]
            desc.layout = capi.LAYOUT_CODES[layout]
            dev["desc"] = desc
            self._dev[key] = dev
        return self._dev[key]

    def state_dict(self) -> Dict[str, torch.Tensor]:
        sd = {}
        for l, (w, b) in enumerate(zip(self.weights, self.biases)):
            sd[f"lin{l}.weight"] = w
            sd[f"lin{l}.bias"] = b
        return sd

    @classmethod
    def from_state_dict(cls, sd: Dict[str, torch.Tensor], latent_dim: int, **kw) -> "SDFDecoder":
        """Accepts DeepSDF-style keys ``lin{l}.weight`` / ``lin{l}.bias`` or weight-norm pairs
        ``lin{l}.weight_g`` / ``lin{l}.weight_v`` (folded here)."""
        from .pack import fold_weight_norm
        ws, bs = [], []
        l = 0
        while f"lin{l}.bias" in sd:
            if f"lin{l}.weight" in sd:
                ws.append(sd[f"lin{l}.weight"])
            else:
                ws.append(fold_weight_norm(sd[f"lin{l}.weight_g"], sd[f"lin{l}.weight_v"]))
            bs.append(sd[f"lin{l}.bias"])
            l += 1
        H = ws[0].shape[0]
        return cls(latent_dim, H, len(ws) - 1, weights=ws, biases=bs, **kw)


# ----------------------------------------------------------------------------------------
# DDPM schedule (A4) and timestep embedding (A5)
# ----------------------------------------------------------------------------------------


def timestep_embedding_table(T: int, dim: int) -> np.ndarray:
    """DDPM sinusoidal embedding for all t (fp64 -> fp32) ``[T, dim]``."""
    half = dim // 2
    freqs = np.exp(-math.log(10000.0) * np.arange(half, dtype=np.float64) / (half - 1))
    ang = np.arange(T, dtype=np.float64)[:, None] * freqs[None, :]
    return np.concatenate([np.sin(ang), np.cos(ang)], axis=1).astype(np.float32)


class DDPMSchedule:
    """Linear beta schedule; tables computed in fp64 on the host, stored fp32 (A4)."""

    NAMES = ("sqrt_ab", "sqrt_1mab", "c1", "c2", "sigma")

    def __init__(self, T: int = 1000, beta_start: float = 1e-4, beta_end: float = 0.02):
        self.T = T
        betas = np.linspace(beta_start, beta_end, T, dtype=np.float64)
        alphas = 1.0 - betas
        ab = np.cumprod(alphas)
        self.tables64 = {
            "betas": betas, "alphas_cumprod": ab,
            "sqrt_ab": np.sqrt(ab), "sqrt_1mab": np.sqrt(1.0 - ab),
            "c1": 1.0 / np.sqrt(alphas), "c2": betas / np.sqrt(1.0 - ab),
            "sigma": np.sqrt(betas),
        }
        self._dev: Dict[torch.device, Dict[str, object]] = {}

    def table(self, name: str) -> torch.Tensor:
        return torch.from_numpy(self.tables64[name].astype(np.float32))

    def device(self, device: torch.device) -> Dict[str, object]:
        device = torch.device(device)
        if device not in self._dev:
            d = {n: self.table(n).to(device) for n in self.NAMES}
            desc = capi.Sched()
            desc.abi_version = capi.ABI_VERSION
            desc.T = self.T
            for n in self.NAMES:
                setattr(desc, n, d[n].data_ptr())
            d["desc"] = desc
            self._dev[device] = d
        return self._dev[device]


# ----------------------------------------------------------------------------------------
# MLP denoiser (A5-A7)
# ----------------------------------------------------------------------------------------


class MLPDenoiser:
    """eps-prediction MLP (SURVEY.md §8 defaults: D=256, H=1024, 4 blocks, TE=128).

    ``e = table[t]``; ``temb = Wt2 SiLU(Wt1 e + bt1) + bt2``; ``h = Win x + bin``;
    block k: ``h <- h + SiLU(Wblk[k] [h || temb] + bblk[k])`` with ``Wblk[k] = [W_k | U_k]``;
    ``eps = Wout h + bout``.  Parameters are fp32 master copies (``self.params``).
    """

    PARAM_ORDER = ("Wt1", "bt1", "Wt2", "bt2", "Win", "bin", "Wout", "bout")

    def __init__(self, D: int = 256, H: int = 1024, n_blocks: int = 4, TE: int = 128,
                 T: int = 1000, seed: int = 4321, params: Optional[Dict[str, torch.Tensor]] = None):
        if n_blocks > capi.MAX_BLOCKS:
            raise ValueError(f"n_blocks <= {capi.MAX_BLOCKS}")
        self.D, self.H, self.n_blocks, self.TE, self.T = D, H, n_blocks, TE, T
        if params is None:
            g = torch.Generator().manual_seed(seed)

            def lin(o, i, scale=1.0):
                w = torch.randn(o, i, generator=g, dtype=torch.float64) * (scale / math.sqrt(i))
                b = torch.randn(o, generator=g, dtype=torch.float64) * 0.01
                return w.float(), b.float()

            params = {}
            params["Wt1"], params["bt1"] = lin(H, TE)
            params["Wt2"], params["bt2"] = lin(H, H)
            params["Win"], params["bin"] = lin(H, D)
            for k in range(n_blocks):
                params[f"Wblk{k}"], params[f"bblk{k}"] = lin(
                    H, 2 * H, 1.0 / math.sqrt(2 * n_blocks) * math.sqrt(2.0))
            params["Wout"], params["bout"] = lin(D, H)
        self.params = {k: v.detach().to(torch.float32).contiguous() for k, v in params.items()}
        self.emb_table = torch.from_numpy(timestep_embedding_table(T, TE))
        self._dev: Dict[Tuple[str, torch.device], Dict[str, object]] = {}
        # bumped whenever packed weights or E tables change under a descriptor handed out
        # earlier: a Sampler compares it and re-packs / re-captures
        self.table_gen = 0

    def names(self) -> List[str]:
        return list(self.PARAM_ORDER) + [f"Wblk{k}" for k in range(self.n_blocks)] + \
            [f"bblk{k}" for k in range(self.n_blocks)]

    def to_device(self, device) -> None:
        self.params = {k: v.to(device) for k, v in self.params.items()}
        self.emb_table = self.emb_table.to(device)
        self._dev.clear()
        self._train_ws = {}

    def train_workspace(self, B: int, device) -> torch.Tensor:
        """The ``saved`` activations workspace of the bf16 C-ABI training path (cached per
        batch size and device; contents are per call)."""
        from . import ops
        key = (torch.device(device), int(B))
        ws = getattr(self, "_train_ws", {})
        self._train_ws = ws
        if key not in ws:
            ws[key] = ops.train_workspace(self.device_pack("bf16", device, with_tables=False)["desc"],
                                          B, device)
        return ws[key]

    def grads_struct(self, grads: Dict[str, torch.Tensor]):
        from . import ops
        return ops.grads_struct(grads, self.n_blocks)

    def invalidate(self) -> None:
        """Call after the fp32 masters changed (training): drops packed copies / E tables."""
        self._dev.clear()
        self.table_gen += 1

    def invalidate_tables(self) -> None:
        """Call after training that kept the working copies current (the built-in AdamW
        rewrites them every step): drops only the E tables, which the next sampling pack
        rebuilds from the trained weights; the working copies (and graphs that captured their
        addresses) stay valid.

        Retention: the tables of the PREVIOUS generation stay allocated here; beyond that,
        every stepper / loop closure (``make_stepper`` / ``make_loop``) holds the tensors its
        descriptor pointed at when it was made, so a graph captured from one replays on valid
        (old) memory however many ``train`` calls later, and calling a stale closure raises
        ``LdmError``.  ``Sampler`` re-packs and re-captures on a ``table_gen``
        change before its next launch."""
        for dev in self._dev.values():
            old = [dev.pop(f"etab{k}") for k in range(self.n_blocks) if f"etab{k}" in dev]
            if old:
                dev["_stale_etab"] = old      # replaces (frees) the generation before it
        self.table_gen += 1

    def _pinned_pack(self, dtype: str, device):
        """(desc, keep, gen): the pack's descriptor, the device tensors its pointers name (held by
        a stepper / loop closure, so a graph captured from the closure never replays on freed
        memory, whatever ``invalidate_tables`` drops later), and the table generation."""
        pack = self.device_pack(dtype, device)
        keep = [v for k, v in pack.items() if isinstance(v, torch.Tensor)]
        return pack["desc"], keep, self.table_gen

    def _check_gen(self, gen: int, what: str) -> None:
        if self.table_gen != gen:
            raise capi.LdmError(f"{what}: the denoiser was trained or re-packed since this "
                                "callable was made (its E tables / weights are stale); make a "
                                "new one (Sampler does so itself)")

    def make_stepper(self, n: int, dtype: str, device, sched_desc):
        """Callable ``step(x, z, t, x_out)``: one fused reverse step (``ldm_sample_step``).
        Raises ``LdmError`` once the denoiser's tables changed under it (``table_gen``)."""
        from . import ops
        desc, keep, gen = self._pinned_pack(dtype, device)
        ws = torch.empty(2 * n * self.H, device=device)

        def step(x, z, t, x_out):
            self._check_gen(gen, "sampling stepper")
            ops.sample_step(desc, sched_desc, x, z, t, x_out, ws)
        step.keep = keep
        return step

    def make_loop(self, n: int, dtype: str, device, sched_desc):
        """Callable ``loop(x2, noise, t_hi, steps)`` running the whole reverse loop as one
        persistent launch (``ldm_sample_loop``), or None when the shape has no persistent
        kernel (the per-step stepper is used then)."""
        from . import ops
        desc, keep, gen = self._pinned_pack(dtype, device)
        if not ops.sample_loop_supported(desc, n):
            return None
        ws = ops.sample_loop_workspace(desc, n, device)

        def loop(x2, noise, t_hi, steps):
            self._check_gen(gen, "sampling loop")
            ops.sample_loop(desc, sched_desc, x2, noise, t_hi, steps, ws)
            return ws
        loop.keep = keep
        loop.status = lambda: ops.sample_loop_status(desc, ws, n)
        loop.form = ops.sample_loop_last_form     # which kernel the last launch ran
        # status 2 (replica placement mismatch) switches this device to the chip-wide loop
        # inside the library, so the Sampler keeps launching the loop
        loop.placement_fallback = True
        return loop

    def device_pack(self, dtype: str, device, with_tables: bool = True) -> Dict[str, object]:
        """Weights in ``dtype`` on ``device`` + the per-block E tables (A5):
        ``E_k[t] = U_k temb(t) + b_k`` for all t, computed with the device GEMM kernel."""
        device = torch.device(device)
        key = (dtype, device)
        if key in self._dev and ("etab0" in self._dev[key] or not with_tables):
            return self._dev[key]
        if key in self._dev:                    # tables dropped by invalidate_tables
            dev = self._dev[key]
            from .ops import build_e_tables
            tabs = build_e_tables(self, dev, dtype)
            for k in range(self.n_blocks):
                dev[f"etab{k}"] = tabs[k]
                dev["desc"].e_tab[k] = tabs[k].data_ptr()
            return dev
        wdt = {"fp32": torch.float32, "bf16": torch.bfloat16}[dtype]
        dev: Dict[str, object] = {}
        for n, v in self.params.items():
            v = v.to(device)
            dev[n] = v.to(wdt).contiguous() if n.startswith("W") else v.contiguous()
        dev["emb_table"] = self.emb_table.to(device).contiguous()
        desc = capi.Denoiser()
        desc.abi_version = capi.ABI_VERSION
        desc.dtype = capi.DTYPE_CODES[dtype]
        desc.D, desc.H, desc.n_blocks, desc.TE, desc.T = self.D, self.H, self.n_blocks, self.TE, self.T
        desc.w_in, desc.b_in = dev["Win"].data_ptr(), dev["bin"].data_ptr()
        desc.w_t1, desc.b_t1 = dev["Wt1"].data_ptr(), dev["bt1"].data_ptr()
        desc.w_t2, desc.b_t2 = dev["Wt2"].data_ptr(), dev["bt2"].data_ptr()
        for k in range(self.n_blocks):
            desc.w_blk[k] = dev[f"Wblk{k}"].data_ptr()
            desc.b_blk[k] = dev[f"bblk{k}"].data_ptr()
        desc.w_out, desc.b_out = dev["Wout"].data_ptr(), dev["bout"].data_ptr()
        desc.emb_table = dev["emb_table"].data_ptr()
        if dtype == "bf16":
            # transposed bf16 copies for the backward's G W products (ldm_denoiser_bwd /
            # _train_step read every operand k-contiguous); ldm_adamw_multi keeps them current
            for n in ["Win", "Wt2", "Wout"] + [f"Wblk{k}" for k in range(self.n_blocks)]:
                dev[n + "_T"] = dev[n].t().contiguous()
            desc.wt_in, desc.wt_t2 = dev["Win_T"].data_ptr(), dev["Wt2_T"].data_ptr()
            desc.wt_out = dev["Wout_T"].data_ptr()
            for k in range(self.n_blocks):
                desc.wt_blk[k] = dev[f"Wblk{k}_T"].data_ptr()
        dev["desc"] = desc
        self._dev[key] = dev
        if with_tables:
            from .ops import build_e_tables
            tabs = build_e_tables(self, dev, dtype)
            for k in range(self.n_blocks):
                dev[f"etab{k}"] = tabs[k]
                desc.e_tab[k] = tabs[k].data_ptr()
        return dev
