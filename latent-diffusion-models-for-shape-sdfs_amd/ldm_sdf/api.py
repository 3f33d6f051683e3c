"""Public train / sample / decode API (SURVEY.md §8(b) 'Python API').

The reference (/root/reference/README.md:1, a title only) defines no API; this is the
build-defined surface a caller drops in:

    decode(decoder, latents[B,L], resolution, *, bbox, dtype, group)  -> sdf[B,N,N,N]
    decode_points(decoder, latents[B,L], xyz[B,P,3], *, dtype)        -> sdf[B,P]
    sample(denoiser, schedule, n, *, steps, dtype, x_T, noise, ...)    -> latents[n,D]
    train(denoiser, schedule, latents[M,D], *, steps, batch, lr, ...)  -> TrainState

All tensors live on the GPU.  Every op runs in libldm_sdf.so (HIP, gfx950); there is no CPU
path in the product (the CPU restatement is oracle/, test infrastructure only).
"""
from __future__ import annotations

import warnings
import weakref
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from . import _capi as capi
from . import dist as ldist
from . import ops
from .models import DDPMSchedule, MLPDenoiser, SDFDecoder


# ---------------------------------------------------------------------------------- decode
# The bf16 decode meets SURVEY §8(c)'s 1e-2 bound (vs the fp64 decoder) only while the
# activations stay near the scale it was calibrated at: its rounding error grows with the
# latents' scale (He-init DeepSDF, CPU oracle at the 16-bit contract: 3.5e-3 at latent RMS
# 0.1, 5.9e-3 at 0.2, 1.1e-2 at 0.5).  fp16 has 3 more mantissa bits (6e-4 / 1.4e-3 at RMS
# 0.1 / 0.5, inside its 2e-3 bound) at the same MFMA rate, so dtype="auto" decodes latents
# whose largest per-shape RMS exceeds BF16_MAX_LATENT_RMS in fp16.
BF16_MAX_LATENT_RMS = 0.2
# fp16's calibration ends here (CPU oracle at the fp16 contract: 1.4e-3 at RMS 0.5, 2.0e-3 --
# SURVEY §8(c)'s fp16 bound -- at 1.0; larger latents also approach fp16's 65504 range): above
# it "auto" decodes in exact fp32
FP16_MAX_LATENT_RMS = 1.0
# "auto" costs one device->host read of the latents' RMS; it is cached per latents tensor, so
# repeated decodes of the same latents do not sync.  An entry holds a WEAK reference to the
# tensor it was computed for and counts as a hit only while that same object is alive and
# unmodified (storage, in-place version, shape): CPython reuses the id of a freed tensor and the
# caching allocator its block, so (id, data_ptr, _version) alone matched a NEW tensor with other
# values.  Writes made behind torch's back (through a C-ABI data_ptr) do not bump
# _version: after such a write, pass an explicit dtype or call clear_auto_cache().
_AUTO_CACHE: Dict[int, tuple] = {}


def clear_auto_cache() -> None:
    """Forget every cached dtype="auto" decision."""
    _AUTO_CACHE.clear()


def resolve_decode_dtype(dtype: str, latents: torch.Tensor) -> str:
    """``dtype`` itself, or for "auto": bf16 when every shape's latent RMS is within the bf16
    calibration (``BF16_MAX_LATENT_RMS``), fp16 up to ``FP16_MAX_LATENT_RMS``, else fp32 -- one
    device->host read per latents tensor (cached while the tensor is unmodified).  Pass an
    explicit dtype to keep a decode free of host synchronisation (graph capture)."""
    if dtype != "auto":
        return dtype
    key = (latents.data_ptr(), latents._version, tuple(latents.shape), str(latents.device))
    ent = _AUTO_CACHE.get(id(latents))
    if ent is not None and ent[0]() is latents and ent[1] == key:
        return ent[2]
    if latents.is_cuda:
        # the library's own reduction (ldm_latent_rms_max): the first torch pow / mean / sqrt /
        # max of a process load their kernels, ~0.25 s (config 3's first call)
        rms = ops.latent_rms_max(latents)
    else:                         # (host tensors: the decision only; decode itself refuses them)
        lat = latents.float().reshape(latents.shape[0] if latents.dim() > 1 else 1, -1)
        rms = float(lat.pow(2).mean(dim=1).sqrt().max())
    pick = "bf16" if rms <= BF16_MAX_LATENT_RMS else "fp16" if rms <= FP16_MAX_LATENT_RMS \
        else "fp32"
    if len(_AUTO_CACHE) > 64:
        _AUTO_CACHE.clear()
    _AUTO_CACHE[id(latents)] = (weakref.ref(latents), key, pick)
    return pick


def decode(decoder: SDFDecoder, latents: torch.Tensor, resolution: int, *,
           bbox: Tuple[float, float] = (-1.0, 1.0), dtype: str = "auto", group=None,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """SDF of every shape on a dense ``resolution^3`` grid over ``bbox^3``.

    Layout ``[B, z, y, x]`` (z slowest).  With an initialised process group the grid is
    z-slab sharded over its ranks and all-gathered (every rank returns the full volume).
    ``dtype``: "fp32" (exact), "bf16", "fp16" or "auto" (``resolve_decode_dtype``: bf16 for
    latents at the calibrated scale, fp16 above it, fp32 past fp16's calibration, so the result
    stays inside §8(c)'s bound).
    """
    capi.require_device(latents)
    if latents.dim() == 1:
        latents = latents[None]
    if latents.shape[1] != decoder.latent_dim:
        raise ValueError(f"latents must be [B, {decoder.latent_dim}]")
    N = int(resolution)
    if N < 2:
        raise ValueError("resolution must be >= 2")
    dtype = resolve_decode_dtype(dtype, latents)
    pack = decoder.device_pack(dtype, latents.device)
    desc = pack["desc"]
    beta = ops.decoder_fold(desc, latents.float().contiguous())
    B = latents.shape[0]
    world, _ = ldist.world_and_rank(group)

    def slab(k0: int, k1: int, dst: torch.Tensor, b0: int = 0, b1: int = B) -> None:
        ops.decoder_grid_fwd(desc, beta[b0:b1], N, k0, k1, bbox, out=dst)

    if world == 1:
        vol = out if out is not None else torch.empty(B, N, N, N, device=latents.device)
        slab(0, N, vol)
        return vol
    return ldist.decode_sharded(slab, B, N, latents.device, group=group, out=out)


def decode_points(decoder: SDFDecoder, latents: torch.Tensor, xyz: torch.Tensor, *,
                  dtype: str = "auto") -> torch.Tensor:
    """SDF at arbitrary points: xyz ``[B, P, 3]`` (or ``[P, 3]`` shared) -> ``[B, P]``
    (``dtype`` as in ``decode``)."""
    capi.require_device(latents, xyz)
    if latents.dim() == 1:
        latents = latents[None]
    dtype = resolve_decode_dtype(dtype, latents)
    B = latents.shape[0]
    if xyz.dim() == 2:
        xyz = xyz[None].expand(B, -1, -1)
    pack = decoder.device_pack(dtype, latents.device)
    beta = ops.decoder_fold(pack["desc"], latents.float().contiguous())
    return ops.decoder_points_fwd(pack["desc"], beta, xyz.float().contiguous())


# ---------------------------------------------------------------------------------- sample
class Sampler:
    """A10: the T-step reverse loop for a fixed (n, steps, dtype), captured once as a HIP
    graph (``torch.cuda.CUDAGraph`` = hipGraph on ROCm) and replayed.  Each step is the
    denoiser's fused reverse step (``make_stepper``): for the MLP, ``ldm_sample_step``
    (in-projection, n_blocks residual blocks, out-projection with the DDPM update in its
    epilogue); for the 1D-UNet, 18 ``ldm_conv1d`` launches ending in the same update."""

    def __init__(self, denoiser, schedule: DDPMSchedule, n: int, *,
                 steps: Optional[int] = None, dtype: str = "bf16", device=None,
                 use_graph: bool = True, persistent: Optional[bool] = None):
        self.device = torch.device(device or torch.device("cuda", torch.cuda.current_device()))
        self.model, self.schedule, self.n = denoiser, schedule, n
        self.T = schedule.T
        self.steps = self.T if steps is None else int(steps)
        if not (1 <= self.steps <= self.T):
            raise ValueError("steps must be in [1, T]")
        self.sd = schedule.device(self.device)
        self.dtype = dtype
        self._gen = getattr(denoiser, "table_gen", 0)
        D = denoiser.D
        self.x2 = torch.empty(2, n, D, device=self.device)
        self.x = [self.x2[0], self.x2[1]]
        self.noise = torch.empty(self.T, n, D, device=self.device)
        self.step = denoiser.make_stepper(n, dtype, self.device, self.sd["desc"])
        self.graph = None
        self.use_graph = use_graph
        # persistent=None (default): the whole loop as one persistent launch (ldm_sample_loop,
        # bit-identical, +10-13 % on MI355X: DESIGN.md §5) whenever the denoiser has a kernel
        # for this shape, else per-step launches; True: require it; False: per-step launches,
        # graph-replayed when use_graph.
        make_loop = getattr(denoiser, "make_loop", None)
        self.loop = None
        self.loop_fallbacks = 0
        # a denoiser whose loop does not beat its per-step graph at this batch (prefer_loop(n)
        # False) runs the graph unless the loop is asked for; the 1D-UNet has no loop (its
        # one-launch loop was retired in round 4 at 0.53x the graph)
        prefer = getattr(denoiser, "prefer_loop", lambda n_: True)(n)
        if make_loop is not None and (persistent or (persistent is None and prefer)):
            self.loop = make_loop(n, dtype, self.device, self.sd["desc"])
        if persistent and self.loop is None:
            raise RuntimeError("no persistent sampling kernel for this denoiser/batch")

    def _loop(self) -> None:
        cur = 0
        for t in range(self.T - 1, self.T - 1 - self.steps, -1):
            self.step(self.x[cur], self.noise[t], t, self.x[cur ^ 1])
            cur ^= 1

    @property
    def result(self) -> torch.Tensor:
        return self.x[self.steps & 1]

    def run(self, x_T: torch.Tensor, noise: torch.Tensor, *, check: bool = True) -> torch.Tensor:
        """x_T ``[n, D]``, noise ``[T, n, D]`` -> the sampled latents (a view of the ping-pong
        buffer; clone it to keep it across runs).

        The persistent loop's grid barriers are bounded: if one gives up (status 1, e.g. when
        other work on the device kept part of the grid from being resident), the launch has
        left partially updated latents; status 2 (an XCD-replica loop found its workgroups
        placed other than one replica's worth per XCD) left them untouched.  After status 2
        the MLP sampler's library has switched the device to its chip-wide loop
        (``loop.placement_fallback``); a loop without such a fallback is dropped here, so later
        runs stay on the per-step graph instead of retrying the launch.  With ``check`` (default) the status word is read back (one stream
        synchronisation) and such a run is redone on the per-step path, which gives the same
        numbers bit for bit; ``loop_fallbacks`` counts these.  ``check=False`` keeps the call
        asynchronous: the caller then reads ``loop.status()`` itself."""
        gen = getattr(self.model, "table_gen", 0)
        if gen != self._gen:
            # the denoiser was trained (or re-packed) since this sampler was built: re-pack its
            # weights / E tables (descriptors are updated in place) and re-capture the graph,
            # which baked the old table addresses in
            self.model.device_pack(self.dtype, self.device)
            self.step = self.model.make_stepper(self.n, self.dtype, self.device, self.sd["desc"])
            if self.loop is not None:
                self.loop = self.model.make_loop(self.n, self.dtype, self.device, self.sd["desc"])
            self.graph = None
            self._gen = gen
        self.x[0].copy_(x_T)
        self.noise[:noise.shape[0]].copy_(noise)
        if self.loop is not None:
            self.loop(self.x2, self.noise, self.T - 1, self.steps)
            if not check:
                return self.result
            st = self.loop.status()
            if st == 0:
                return self.result
            self.loop_fallbacks += 1
            why = {1: "a grid barrier timed out",
                   2: "replica placement mismatch: workgroups not 1/8 per XCD, nothing computed",
                   3: "launch arguments differ from the prepared program, nothing computed"}
            warnings.warn(f"persistent sampling loop ({type(self.model).__name__}): status {st} "
                          f"({why.get(st, 'unknown')}); "
                          "re-running this sample on the per-step path", RuntimeWarning)
            if st == 2 and not getattr(self.loop, "placement_fallback", False):
                self.loop = None          # nothing to switch to: the graph from now on
            self.x[0].copy_(x_T)
            self._loop()
            return self.result
        if not self.use_graph:
            self._loop()
            return self.result
        if self.graph is None:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._loop()          # warm-up (module load, first-launch costs)
            torch.cuda.current_stream(self.device).wait_stream(s)
            self.x[0].copy_(x_T)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._loop()
            self.graph = g
        self.graph.replay()
        return self.result


def sample(denoiser, schedule: DDPMSchedule, n: int, *,
           steps: Optional[int] = None, dtype: str = "bf16", x_T: Optional[torch.Tensor] = None,
           noise: Optional[torch.Tensor] = None, generator: Optional[torch.Generator] = None,
           device=None, use_graph: bool = True, persistent: Optional[bool] = None,
           group=None) -> torch.Tensor:
    """DDPM ancestral sampling (DDPM Alg. 2) of ``n`` latent codes.

    ``x_T [n, D]`` and ``noise [T, n, D]`` may be given (parity mode: the same numbers the
    CPU oracle consumes); otherwise they are drawn on the device.  With a process group the
    batch is sharded over ranks and the latents all-gathered.
    """
    device = torch.device(device or torch.device("cuda", torch.cuda.current_device()))
    world, rank = ldist.world_and_rank(group)
    lo, hi = ldist.batch_shard(n, rank, world)
    nl = hi - lo
    D, T = denoiser.D, schedule.T
    if x_T is None:
        x_T = torch.randn(n, D, device=device, generator=generator)
    if noise is None:
        noise = torch.randn(T, n, D, device=device, generator=generator)
    x_T = x_T.to(device, torch.float32)[lo:hi].contiguous()
    noise = noise.to(device, torch.float32)[:, lo:hi].contiguous()
    out = Sampler(denoiser, schedule, nl, steps=steps, dtype=dtype, device=device,
                  use_graph=use_graph, persistent=persistent).run(x_T, noise).clone()
    return ldist.all_gather_rows(out, n, group=group)


# ---------------------------------------------------------------------------------- train
@dataclass
class TrainState:
    step: int = 0
    losses: List[float] = field(default_factory=list)
    optimizer: Optional[torch.optim.Optimizer] = None    # a torch optimizer, if one is given
    masters: Optional[Dict[str, torch.Tensor]] = None
    adam: Optional[Dict[str, Tuple[torch.Tensor, torch.Tensor]]] = None   # fused AdamW (m, v)
    hparams: Dict[str, float] = field(default_factory=dict)
    adam_table: Optional[object] = None     # ldm_adamw_multi descriptors (bf16 path)
    adam_grads: Optional[Dict[str, torch.Tensor]] = None
    adam_pack: Optional[Dict[str, object]] = None    # the device pack the table points into
    graphs: Optional[Dict[str, object]] = None       # captured steps (train(graph=True))

    # ---- checkpoint / resume ({denoiser, optimizer, step, rng}) --------------
    FORMAT = "ldm_sdf.TrainState/1"

    def save(self, path: str, generator: Optional[torch.Generator] = None) -> None:
        """Write the training state: the fp32 masters (the denoiser's parameters), the built-in
        AdamW moments or a torch optimizer's state dict, the step count, the losses, the
        hyper-parameters and -- when given -- the random generator's state, so that
        ``TrainState.load`` + ``train(..., state=)`` continues the run bit for bit (resume at a
        multiple of train()'s 32-step draw block).  Derived data (bf16 working copies, E tables,
        AdamW descriptor tables, graphs) is rebuilt after a load, never saved."""
        if self.masters is None:
            raise ValueError("TrainState.save: nothing trained yet")
        ck = {"format": self.FORMAT, "step": int(self.step),
              "losses": [float(l) for l in self.losses], "hparams": dict(self.hparams),
              "masters": {n: v.detach().cpu() for n, v in self.masters.items()}}
        if self.adam is not None:
            ck["adam"] = {n: (m.detach().cpu(), v.detach().cpu())
                          for n, (m, v) in self.adam.items()}
        if self.optimizer is not None:
            ck["optimizer"] = self.optimizer.state_dict()
            # the state dict is positional: record which parameter each position is, so a load
            # can rebuild the groups in this order whatever order the caller's optimizer uses
            ident = {id(t): n for n, t in self.masters.items()}
            if all(id(p) in ident for g in self.optimizer.param_groups for p in g["params"]):
                ck["optimizer_names"] = [[ident[id(p)] for p in g["params"]]
                                         for g in self.optimizer.param_groups]
        if generator is not None:
            ck["rng"] = generator.get_state().cpu()
            ck["rng_device"] = str(generator.device)
        torch.save(ck, path)

    @classmethod
    def load(cls, path: str, denoiser: MLPDenoiser, device=None,
             generator: Optional[torch.Generator] = None,
             optimizer: Optional[torch.optim.Optimizer] = None) -> "TrainState":
        """Restore a state written by ``save`` into ``denoiser`` (its parameters become the
        saved masters, on ``device``) and, when given, ``generator`` (its state) and
        ``optimizer`` (its state dict).  Loaded with ``torch.load(weights_only=True)``: nothing
        in the file is executed."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        if ck.get("format") != cls.FORMAT:
            raise ValueError(f"{path}: not a {cls.FORMAT} checkpoint")
        device = torch.device(device or torch.device("cuda", torch.cuda.current_device()))
        names = denoiser.names()
        if sorted(ck["masters"]) != sorted(names):
            raise ValueError(f"{path}: parameters {sorted(ck['masters'])} do not match the "
                             f"denoiser's {sorted(names)}")
        for n in names:
            if tuple(ck["masters"][n].shape) != tuple(denoiser.params[n].shape):
                raise ValueError(f"{path}: {n} has shape {tuple(ck['masters'][n].shape)}")
        # which parameter each tensor of a caller's optimizer is (by identity, before the
        # denoiser's tensors are replaced): its param_groups are re-pointed at the loaded
        # masters below, so optimizer.step() updates what train() trains
        opt_names = None
        if optimizer is not None:
            ident = {id(t): n for n, t in denoiser.params.items()}
            opt_names = []
            for g in optimizer.param_groups:
                if any(id(p) not in ident for p in g["params"]):
                    raise ValueError("TrainState.load: the optimizer holds tensors that are not "
                                     "this denoiser's parameters")
                opt_names.append([ident[id(p)] for p in g["params"]])
        denoiser.params = {n: ck["masters"][n].to(torch.float32) for n in names}
        denoiser.to_device(device)               # also drops packs, tables, workspaces
        denoiser.invalidate()
        st = cls()
        st.step = int(ck["step"])
        st.losses = list(ck["losses"])
        st.hparams = dict(ck["hparams"])
        st.masters = {n: denoiser.params[n] for n in names}
        for v in st.masters.values():
            v.requires_grad_(False)
        if "adam" in ck:
            st.adam = {n: (m.to(device), v.to(device)) for n, (m, v) in ck["adam"].items()}
        if optimizer is not None:
            if "optimizer" not in ck:
                raise ValueError(f"{path}: no optimizer state saved")
            saved = ck.get("optimizer_names")
            if saved is not None:
                # the saved order (positional state), whatever order the caller built in
                if len(saved) != len(optimizer.param_groups) or \
                        sorted(n for g in saved for n in g) != sorted(n for g in opt_names
                                                                      for n in g):
                    raise ValueError(f"{path}: the optimizer's parameter groups do not match "
                                     "the saved ones")
                opt_names = saved
            for g, gn in zip(optimizer.param_groups, opt_names):
                g["params"] = [st.masters[n] for n in gn]
            optimizer.state.clear()               # keyed by the old tensors; reloaded below
            optimizer.load_state_dict(ck["optimizer"])
            st.optimizer = optimizer
        if generator is not None:
            if "rng" not in ck:
                raise ValueError(f"{path}: no generator state saved")
            generator.set_state(ck["rng"])
        return st


def _reduce_grads(denoiser, grads, loss, B_local: int, global_batch: Optional[int], group):
    """Data-parallel gradient of the GLOBAL batch's mean loss: each rank's gradients (and loss)
    are of its local mean over B_local rows, so rank r scales by B_r / B before one summing
    all-reduce of the flat gradient buffer -- exact for uneven shards (a plain mean over ranks
    is not).  The loss rides in the same all-reduce when the buffer has its ``__loss`` slot.
    ``global_batch`` None: the plain mean over ranks."""
    world, _ = ldist.world_and_rank(group)
    if world == 1:
        return loss
    ts = [grads[n] for n in denoiser.names()]
    lslot = grads.get("__loss")
    if lslot is not None:
        lslot.copy_(loss.reshape(1))
        ts.append(lslot)
    if global_batch is None:
        ldist.allreduce_mean_(ts, group=group)
    else:
        ldist.allreduce_weighted_(ts, B_local / float(global_batch), group=group)
    if lslot is None:
        loss = loss.clone()
        if global_batch is None:
            ldist.allreduce_mean_([loss], group=group)
        else:
            ldist.allreduce_weighted_([loss], B_local / float(global_batch), group=group)
        return loss
    return lslot.clone()


def train_step(denoiser: MLPDenoiser, schedule: DDPMSchedule, x0: torch.Tensor,
               t: torch.Tensor, eps: torch.Tensor, *, dtype: str = "bf16",
               grads: Optional[Dict[str, torch.Tensor]] = None,
               group=None, global_batch: Optional[int] = None
               ) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
    """One DDPM training forward/backward (Alg. 1): q_sample -> eps_hat -> MSE -> grads.
    ``dtype`` "fp32": exact fp32 GEMMs; "bf16": bf16 weights and matrix-core GEMMs with
    operands rounded to bf16 (fp32 accumulate).  Returns (loss [1], grads).  With a group the
    gradients and the loss are those of the mean over the GLOBAL batch of ``global_batch`` rows
    (each rank weighted by its share; None: the plain mean over ranks).  bf16 runs the fused
    forward + backward C call, ``ldm_denoiser_train_step``, in the form
    ``ops.train_step_config`` selects -- the one-launch job DAG (without its AdamW nodes: the
    update waits for the all-reduce) or the launch path."""
    device = x0.device
    dev = denoiser.device_pack(dtype, device, with_tables=False)
    sd = schedule.device(device)
    if grads is None:
        grads = {n: torch.empty_like(denoiser.params[n], device=device) for n in denoiser.names()}
    if dtype == "bf16":
        # the fused C-ABI step (ldm_denoiser_train_step): q_sample, forward, eps-MSE and the
        # whole backward as ldm_gemm_bf16 problems with fused epilogues, one host call
        B = x0.shape[0]
        ws = denoiser.train_workspace(B, device)
        loss = torch.empty(1, device=device, dtype=torch.float32)
        ops.denoiser_train_step(dev["desc"], sd["desc"], x0.float().contiguous(),
                                eps.float().contiguous(), t.to(torch.int32).contiguous(), ws,
                                denoiser.grads_struct(grads), loss)
        loss = _reduce_grads(denoiser, grads, loss, B, global_batch, group)
        return loss, grads
    xt = ops.q_sample(sd["desc"], x0.contiguous(), eps.contiguous(), t.to(torch.int32).contiguous())
    cp = capi.COMPUTE_CODES[dtype]
    eps_hat, sv = ops.denoiser_forward_train(denoiser, dev, xt, t.to(torch.int32).contiguous(),
                                             compute=cp)
    loss, g_out = ops.eps_mse_loss(eps_hat, eps.contiguous())
    ops.denoiser_backward_train(denoiser, dev, sv, g_out, grads, compute=cp)
    loss = _reduce_grads(denoiser, grads, loss, x0.shape[0], global_batch, group)
    return loss, grads


def _adam_table(denoiser: MLPDenoiser, state: TrainState, grads, dtype: str, device):
    """ldm_adamw_multi descriptors: fp32 masters + Adam moments, and the bf16 working copies
    (both layouts) the next step's GEMMs read."""
    work = denoiser.device_pack(dtype, device, with_tables=False)
    return ops.adamw_table(
        [(p, grads[n], *state.adam[n], work[n] if n.startswith("W") else None,
          work.get(n + "_T")) for n, p in state.masters.items()])


def train(denoiser: MLPDenoiser, schedule: DDPMSchedule, latents: torch.Tensor, *, steps: int,
          batch: Optional[int] = None, lr: float = 1e-4, weight_decay: float = 0.0,
          dtype: str = "bf16", generator: Optional[torch.Generator] = None,
          state: Optional[TrainState] = None, group=None, fused_step: bool = True,
          overlap: bool = False, graph: bool = False) -> TrainState:
    """Train the denoiser on latent codes ``[M, D]`` (DDPM Alg. 1, eps-prediction, AdamW).

    fp32 master weights; forward/backward GEMMs read ``dtype`` copies (bf16 by default).
    Data parallel over the group's ranks (each rank its shard of every batch; gradients
    all-reduced in one bucket).  On one rank with the built-in AdamW (bf16) each step is ONE C
    call, ``ldm_denoiser_train_step_adamw`` (``fused_step``); ``overlap`` forks its weight
    updates onto a side stream beside the backward's tail (measured slower at config 2, so off
    by default).  ``graph``: full-batch single-rank steps replay hipGraphs of that call, one
    per slot of a 32-step chunk (t, eps and the AdamW scalars in device buffers refilled per
    chunk), captured once per state; measured 3% slower than the eager calls at config 2
    (3030 vs 3115 steps/s, scripts/train_ab.py), so off by default.  No switch changes the
    results.
    """
    capi.require_device(latents)
    device = latents.device
    world, rank = ldist.world_and_rank(group)
    M, D = latents.shape
    batch = M if batch is None else batch
    if state is None:
        denoiser.to_device(device)
        state = TrainState()
        state.masters = {n: denoiser.params[n] for n in denoiser.names()}
        for v in state.masters.values():
            v.requires_grad_(False)
        # fused AdamW (ldm_adamw_step): one HIP pass per tensor updates the fp32 master and
        # rewrites the bf16 working copy the next step's GEMMs read (no per-step re-pack)
        state.adam = {n: (torch.zeros_like(v), torch.zeros_like(v))
                      for n, v in state.masters.items()}
        state.hparams = dict(lr=lr, weight_decay=weight_decay)
    # gradients live in ONE flat buffer (one view per parameter): the data-parallel all-reduce
    # then reduces that buffer in place, with no per-step concatenation or copy back
    # (+ a one-float "__loss" slot at its end: at world > 1 the loss rides in the gradients'
    # all-reduce)
    grads = state.adam_grads if state.adam_grads is not None else \
        ldist.flat_buffers({**{n: tuple(v.shape) for n, v in state.masters.items()},
                            "__loss": (1,)}, device)[1]
    T = schedule.T
    # single rank, built-in AdamW: the fused C step (no gradient all-reduce to wait for)
    fused = dtype == "bf16" and state.optimizer is None and world == 1 and fused_step
    chunk = 32           # steps whose random draws are made in one launch each
    if dtype == "bf16" and state.optimizer is None:
        pack = denoiser.device_pack(dtype, device, with_tables=False)
        if state.adam_table is None or state.adam_pack is not pack:
            # (re)build the AdamW table for this pack; graphs captured on the old one are void
            state.adam_table = _adam_table(denoiser, state, grads, dtype, device)
            state.adam_grads, state.adam_pack, state.graphs = grads, pack, None
    if fused and graph and batch == M and not overlap:
        _train_graphed(denoiser, schedule, latents, steps, state, grads, generator, chunk)
        steps = 0
    for s in range(steps):
        j = s % chunk
        if j == 0:
            # the draws of the next `chunk` steps (t, eps, and the batch indices when the batch
            # is a sample of the latents) in three launches instead of two or three per step;
            # full-batch steps (batch == M) take the latents as they are: no index, no gather
            n = min(chunk, steps - s)
            idx_all = torch.randint(0, M, (n, batch), device=device, generator=generator) \
                if batch != M else None
            t_all = torch.randint(0, T, (n, batch), device=device, generator=generator,
                                  dtype=torch.int32)
            eps_all = torch.randn(n, batch, D, device=device, generator=generator)
        idx = idx_all[j] if idx_all is not None else None
        t, eps = t_all[j], eps_all[j]
        lo, hi = ldist.batch_shard(batch, rank, world)
        x0 = latents[idx[lo:hi]].contiguous() if idx is not None else \
            latents[lo:hi].float().contiguous()
        if fused:
            # one C call for the whole step: forward, backward and AdamW (same bits as
            # train_step + adamw_multi)
            if state.adam_grads is not grads:
                raise RuntimeError("train: gradient buffers changed under the AdamW table")
            dev = denoiser.device_pack(dtype, device, with_tables=False)
            ws = denoiser.train_workspace(hi - lo, device)
            loss = torch.empty(1, device=device, dtype=torch.float32)
            ops.denoiser_train_step_adamw(
                dev["desc"], schedule.device(device)["desc"], x0.float().contiguous(),
                eps[lo:hi].contiguous(), t[lo:hi].contiguous(), ws,
                denoiser.grads_struct(grads), loss, state.adam_table,
                lr=state.hparams["lr"], weight_decay=state.hparams["weight_decay"],
                step=state.step + 1, overlap=overlap)
            state.step += 1
            state.losses.append(loss)
            continue
        loss, grads = train_step(denoiser, schedule, x0, t[lo:hi], eps[lo:hi], dtype=dtype,
                                 grads=grads, group=group, global_batch=batch)
        if state.optimizer is not None:          # caller-supplied torch optimizer
            for n, p in state.masters.items():
                p.grad = grads[n]
            state.optimizer.step()
            denoiser.invalidate()
        elif dtype == "bf16":
            # one launch for every tensor: fp32 masters + Adam moments, and the bf16 working
            # copies (both layouts) the next step's GEMMs read (table built above)
            if state.adam_grads is not grads:
                raise RuntimeError("train: gradient buffers changed under the AdamW table")
            ops.adamw_multi(state.adam_table, lr=state.hparams["lr"],
                            weight_decay=state.hparams["weight_decay"], step=state.step + 1,
                            device=device)
        else:
            work = denoiser.device_pack(dtype, device, with_tables=False)
            for n, p in state.masters.items():
                w = work[n]
                low = w if (w.dtype == torch.bfloat16 and w.data_ptr() != p.data_ptr()) else None
                m, v = state.adam[n]
                ops.adamw_step(p, grads[n], m, v, low, lr=state.hparams["lr"],
                               weight_decay=state.hparams["weight_decay"], step=state.step + 1)
                if low is None and w.data_ptr() != p.data_ptr():
                    w.copy_(p)                   # an fp32 working copy that is not the master
        state.step += 1
        state.losses.append(loss)
    if dtype == "bf16" and steps > 0 and ops.train_step_last_form() == "dag":
        # the one-launch step's waits are bounded: a non-zero status means a step gave up and
        # the weights are not to be trusted (one read-back per train() call, where the losses
        # are read back anyway) -- the data-parallel path (the DAG without AdamW nodes) too:
        # its workspace is the rank's shard's
        lo_, hi_ = ldist.batch_shard(batch, rank, world)
        dev_ = denoiser.device_pack(dtype, device, with_tables=False)
        st = ops.train_status(dev_["desc"], hi_ - lo_,
                              denoiser.train_workspace(hi_ - lo_, device))
        if st != 0:
            raise capi.LdmError(f"train: the one-launch training step reported status {st} "
                                "(1: a dependency wait timed out, 3: stale job table); the "
                                "parameters are not valid")
    if state.optimizer is None and dtype == "bf16":
        # the built-in AdamW kept every working copy current (bf16 copies in both layouts; an
        # fp32 pack holds the masters themselves): only the E tables (sampling) are rebuilt
        # from the trained weights, so the AdamW table and captured graphs stay valid
        denoiser.invalidate_tables()
    elif state.optimizer is None:
        denoiser.invalidate()    # fp32 training updated the masters only: bf16 packs are stale
    # one device->host transfer for the whole run, not one per step
    pend = [i for i, l in enumerate(state.losses) if isinstance(l, torch.Tensor)]
    if pend:
        vals = torch.cat([state.losses[i].reshape(1).float() for i in pend]).tolist()
        for i, v in zip(pend, vals):
            state.losses[i] = v
    return state


def _train_graphed(denoiser: MLPDenoiser, schedule: DDPMSchedule, latents: torch.Tensor,
                   steps: int, state: TrainState, grads, generator, chunk: int) -> None:
    """Full-batch single-rank bf16 steps as hipGraph replays of
    ``ldm_denoiser_train_step_adamw``: one graph per slot j of a ``chunk``-step block reads
    t / eps / the AdamW scalars of slot j from device buffers that are refilled once per block
    (the same random draws, in the same order, as the eager loop; the scalars from
    ``ldm_adamw_hyper``, the values the argument path uses), so results are bit-identical.
    Slots run eagerly until their graph exists; every slot is captured after the first block."""
    device = latents.device
    M, D = latents.shape
    T = schedule.T
    dev = denoiser.device_pack("bf16", device, with_tables=False)
    ws = denoiser.train_workspace(M, device)
    sdesc = schedule.device(device)["desc"]
    x0 = latents.float().contiguous()
    key = (x0.data_ptr(), ws.data_ptr(), M, D, T, sdesc.sqrt_ab, chunk)
    G = state.graphs
    if G is None or G["key"] != key:
        G = {"key": key, "x0": x0, "ws": ws,
             "t": torch.empty(chunk, M, device=device, dtype=torch.int32),
             "eps": torch.empty(chunk, M, D, device=device, dtype=torch.float32),
             "hyper": torch.zeros(chunk, 8, device=device, dtype=torch.float32),
             "loss": torch.zeros(chunk, device=device, dtype=torch.float32),
             # two pinned host staging buffers for the scalars, each reused only after the
             # event of its previous copy (a pageable copy would stall the host every block)
             "hyper_host": [torch.zeros(chunk, 8, dtype=torch.float32).pin_memory()
                            for _ in range(2)],
             "hyper_ev": [None, None], "block": 0,
             "g": [None] * chunk}
        state.graphs = G
    gstruct = denoiser.grads_struct(grads)
    hp = state.hparams

    def call(j: int, step: int) -> None:
        ops.denoiser_train_step_adamw(
            dev["desc"], sdesc, x0, G["eps"][j], G["t"][j], ws, gstruct, G["loss"][j:j + 1],
            state.adam_table, lr=hp["lr"], weight_decay=hp["weight_decay"], step=step,
            hyper=G["hyper"][j])

    s = 0
    while s < steps:
        n = min(chunk, steps - s)
        torch.randint(0, T, (n, M), generator=generator, out=G["t"][:n])
        torch.randn((n, M, D), generator=generator, out=G["eps"][:n])
        hb = G["block"] & 1
        G["block"] += 1
        if G["hyper_ev"][hb] is not None:
            G["hyper_ev"][hb].synchronize()
        host = G["hyper_host"][hb]
        host[:n] = torch.tensor([ops.adamw_hyper(lr=hp["lr"], weight_decay=hp["weight_decay"],
                                                 step=state.step + 1 + j) + [0.0]
                                 for j in range(n)], dtype=torch.float32)
        G["hyper"][:n].copy_(host[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        G["hyper_ev"][hb] = ev
        for j in range(n):
            if G["g"][j] is None:
                call(j, state.step + 1 + j)
            else:
                G["g"][j].replay()
        losses = G["loss"][:n].clone()
        state.losses.extend(losses[j:j + 1] for j in range(n))
        state.step += n
        s += n
        if any(g is None for g in G["g"]):
            # capture executes nothing; the slots' next use replays
            for j in range(chunk):
                if G["g"][j] is None:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        call(j, 1)
                    G["g"][j] = g
