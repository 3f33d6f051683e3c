"""C19: DeepSDF auto-decoder training.

The step before the hot path: it fits the decoder weights and one latent code per shape to
SDF samples, producing the latents that the diffusion model is then trained on and the
decoder that decodes them.  Objective: ``oracle/ref_autodecoder.py`` (DeepSDF's clamped L1 on
``tanh`` outputs plus the per-sample latent L2 regulariser; no dropout).

Every FLOP runs in ``libldm_sdf.so``:

* the 9 forward linears are ``ldm_linear`` with the ReLU epilogue;
* the backward products are ``ldm_linear`` on transposed views (``G W``, ``G^T X``);
* the bias gradients are ``ldm_colsum``, the per-shape latent gradients ``ldm_colsum_segments``;
* the loss and its gradient are ``ldm_sdf_l1_loss``, the code regulariser ``ldm_latent_l2_reg``.

torch provides memory, the row gather's destination copies and Adam (plumbing), as in
``api.train``.

Working layout (rebuilt from the fp32 masters each step, in the GEMM dtype).  It pads so that
every operand row is a multiple of 16 bytes and the matrix-core path can use vector loads:

* ``Zx`` [N, 264] = ``[z_s || xyz || 0]`` (8-column multiple: 16-byte rows in bf16). It is the
  input of layer 0 and the second segment of layer 4.
* The backward's ``G W`` products apply the ReLU mask in their epilogue (``LDM_EPI_MASK_R``
  with the saved post-activation), so ``relu_bwd`` is a separate pass nowhere.
* Layer ``skip-1`` (253 outputs) is padded to 256 rows with zero weights and biases, so its
  ReLU output ``h3`` [N, 256] has 3 zero columns. Layer ``skip`` is two segments,
  ``h3 · W4h^T + Zx · W4z^T``.
* The master gradients are cut back out of the padded ones.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from . import _capi as capi
from . import dist as ldist
from . import ops
from .models import SDFDecoder

__all__ = ["AutoDecoderState", "autodecoder_train_step", "train_autodecoder", "CLAMP_DIST",
           "CODE_REG_LAMBDA"]

CLAMP_DIST = 0.1          # DeepSDF ClampingDistance
CODE_REG_LAMBDA = 1e-4    # DeepSDF CodeRegularizationLambda


def _check_decoder(dec: SDFDecoder) -> Tuple[int, int]:
    if dec.widen_skip or dec.n_hidden != 8 or dec.skip != 4:
        raise capi.LdmError("auto-decoder training supports the DeepSDF 8-layer decoder with the "
                            "latent re-injected at layer 4 (skip width H - L - 3)")
    return dec.latent_dim, dec.hidden


def _zx_width(L: int) -> int:
    """[z || xyz] padded to a multiple of 8 columns: 16-byte rows in bf16 as well as fp32."""
    return (L + 3 + 7) // 8 * 8


def _pad_rows(n: int) -> int:
    return (n + 3) // 4 * 4


def work_weights(masters: Dict[str, torch.Tensor], L: int, H: int, skip: int,
                 dtype: torch.dtype) -> Dict[str, torch.Tensor]:
    """Padded working copies (see module doc) of the fp32 masters ``W{l}``/``b{l}``.  Pure
    data movement; also used on CPU tensors by the host-logic tests."""
    zw = _zx_width(L)
    hs = masters[f"W{skip - 1}"].shape[0]             # skip width, 253 for L=256, H=512
    hsp = _pad_rows(hs)
    dev = masters["W0"].device
    w: Dict[str, torch.Tensor] = {}
    W0 = torch.zeros(H, zw, device=dev, dtype=dtype)
    W0[:, :L + 3] = masters["W0"]
    w["W0"] = W0
    for l in range(1, 9):
        if l == skip - 1:
            Wp = torch.zeros(hsp, H, device=dev, dtype=dtype)
            Wp[:hs] = masters[f"W{l}"]
            bp = torch.zeros(hsp, device=dev, dtype=torch.float32)
            bp[:hs] = masters[f"b{l}"]
            w[f"W{l}"], w[f"b{l}p"] = Wp, bp
        elif l == skip:
            Ws = masters[f"W{l}"]
            Wh = torch.zeros(H, hsp, device=dev, dtype=dtype)
            Wh[:, :hs] = Ws[:, :hs]
            Wz = torch.zeros(H, zw, device=dev, dtype=dtype)
            Wz[:, :L + 3] = Ws[:, hs:]
            w["W4h"], w["W4z"] = Wh, Wz
        else:
            w[f"W{l}"] = masters[f"W{l}"].to(dtype)
    return w


def master_grads(gw: Dict[str, torch.Tensor], L: int, skip: int, hs: int,
                 out: Dict[str, torch.Tensor]) -> None:
    """Cut the padded working gradients back to the master shapes (into ``out``)."""
    out["W0"].copy_(gw["W0"][:, :L + 3])
    out["b0"].copy_(gw["b0"])
    for l in range(1, 9):
        if l == skip - 1:
            out[f"W{l}"].copy_(gw[f"W{l}"][:hs])
            out[f"b{l}"].copy_(gw[f"b{l}"][:hs])
        elif l == skip:
            out[f"W{l}"][:, :hs].copy_(gw["W4h"][:, :hs])
            out[f"W{l}"][:, hs:].copy_(gw["W4z"][:, :L + 3])
            out[f"b{l}"].copy_(gw[f"b{l}"])
        else:
            out[f"W{l}"].copy_(gw[f"W{l}"])
            out[f"b{l}"].copy_(gw[f"b{l}"])


def autodecoder_train_step(masters: Dict[str, torch.Tensor], z: torch.Tensor, xyz: torch.Tensor,
                           sdf: torch.Tensor, *, latent_dim: int = 256, hidden: int = 512,
                           skip: int = 4, delta: float = CLAMP_DIST,
                           reg_lambda: float = CODE_REG_LAMBDA, epoch: int = 100,
                           dtype: str = "bf16",
                           grads: Optional[Dict[str, torch.Tensor]] = None
                           ) -> Tuple[torch.Tensor, Dict[str, torch.Tensor], torch.Tensor]:
    """One forward/backward of the DeepSDF objective on a batch of S shapes x P samples.

    masters: fp32 device ``W0..W8``, ``b0..b8`` (torch ``nn.Linear`` layout, latent columns
    first: ``[z || xyz]`` and ``[h || z || xyz]`` at the skip).  z: [S, L] the batch's codes,
    xyz: [S, P, 3], sdf: [S, P].  ``dtype`` "fp32": exact fp32 GEMMs; "bf16": matrix-core
    GEMMs with bf16-rounded operands, fp32 accumulation.
    Returns (loss [1], weight grads keyed like ``masters``, latent grads [S, L]).
    """
    capi.require_device(z, xyz, sdf, masters["W0"])
    L, H = latent_dim, hidden
    S, P = sdf.shape
    N = S * P
    if tuple(z.shape) != (S, L) or tuple(xyz.shape) != (S, P, 3):
        raise capi.LdmError(f"autodecoder_train_step: z{tuple(z.shape)} xyz{tuple(xyz.shape)} "
                            f"sdf{tuple(sdf.shape)}")
    dev = z.device
    cp = capi.COMPUTE_CODES[dtype]
    wdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    hs = masters[f"W{skip - 1}"].shape[0]
    hsp, zw = _pad_rows(hs), _zx_width(L)
    w = work_weights(masters, L, H, skip, wdt)
    b = {f"b{l}": masters[f"b{l}"] for l in range(9)}
    b[f"b{skip - 1}"] = w[f"b{skip - 1}p"]
    f32 = dict(device=dev, dtype=torch.float32)

    # ---- inputs: Zx = [z_s || xyz || 0] per sample
    z = z.contiguous()
    owner = torch.arange(S, device=dev, dtype=torch.int32).repeat_interleave(P)
    Zx = torch.zeros(N, zw, **f32)
    Zx[:, :L].copy_(ops.gather_rows(z, owner))
    Zx[:, L:L + 3].copy_(xyz.reshape(N, 3))

    # ---- forward (post-ReLU activations kept for the backward)
    RELU = capi.EPI_RELU
    h: List[torch.Tensor] = []
    x = Zx
    for l in range(8):
        width = hsp if l == skip - 1 else H
        y = torch.empty(N, width, **f32)
        if l == skip:
            ops.linear(x, w["W4h"], y, epi=RELU, bias=b[f"b{l}"], X2=Zx, W2=w["W4z"], compute=cp)
        else:
            ops.linear(x, w[f"W{l}"], y, epi=RELU, bias=b[f"b{l}"], compute=cp)
        h.append(y)
        x = y
    pre = torch.empty(N, 1, **f32)
    ops.linear(x, w["W8"], pre, bias=b["b8"], compute=cp)
    loss, g = ops.sdf_l1_loss(pre, sdf.contiguous(), delta, 1.0 / N)

    # ---- backward
    gw: Dict[str, torch.Tensor] = {}
    dz = torch.empty(N, L, **f32)
    for l in range(8, -1, -1):
        xin = Zx if l == 0 else h[l - 1]
        if l == skip:
            gw["W4h"] = torch.empty(H, hsp, **f32)
            gw["W4z"] = torch.empty(H, zw, **f32)
            ops.linear(g.T, xin.T, gw["W4h"], compute=cp)
            ops.linear(g.T, Zx.T, gw["W4z"], compute=cp)
            ops.linear(g, w["W4z"][:, :L].t().contiguous(), dz, compute=cp)   # latent part, layer 4
        else:
            Wl = w[f"W{l}"]
            gw[f"W{l}"] = torch.empty(Wl.shape[0], Wl.shape[1], **f32)
            ops.linear(g.T, xin.T, gw[f"W{l}"], compute=cp)
        gw[f"b{l}"] = torch.empty(g.shape[1], **f32)
        ops.colsum(g, gw[f"b{l}"])
        if l == 0:
            ops.linear(g, w["W0"][:, :L].t().contiguous(), dz, epi=capi.EPI_ACCUM, compute=cp)
            break
        Wd = w["W4h"] if l == skip else w[f"W{l}"]
        dh = torch.empty(N, Wd.shape[1], **f32)       # ReLU backward fused: R = post-act.
        # G W with W transposed once (a 512 x 512 copy): both operands then run along k, so the
        # GEMM stages them with 16-byte row loads instead of 2-byte transposing LDS stores
        # (4.6 -> ~2.8 ms per 1M x 512 x 512 product; same products, same k order).
        ops.linear(g, Wd.t().contiguous(), dh, epi=capi.EPI_MASK_R, R=h[l - 1], compute=cp)
        g = dh

    gz = torch.empty(S, L, **f32)
    ops.colsum_segments(dz, S, gz)
    coef = reg_lambda * min(1.0, epoch / 100.0) / S
    if coef != 0.0:
        ops.latent_l2_reg(z, coef, loss, gz)
    if grads is None:
        grads = {k: torch.empty_like(v) for k, v in masters.items()}
    master_grads(gw, L, skip, hs, grads)
    return loss, grads, gz


@dataclass
class AutoDecoderState:
    step: int = 0
    losses: List[float] = field(default_factory=list)
    masters: Optional[Dict[str, torch.Tensor]] = None
    latents: Optional[torch.Tensor] = None            # [n_shapes, L] fp32, device
    optimizer: Optional[torch.optim.Optimizer] = None
    lat_optimizer: Optional[torch.optim.Optimizer] = None


def train_autodecoder(decoder: SDFDecoder, xyz: torch.Tensor, sdf: torch.Tensor, *, steps: int,
                      shapes_per_batch: Optional[int] = None,
                      samples_per_shape: Optional[int] = None, lr_decoder: float = 5e-4,
                      lr_latent: float = 1e-3, delta: float = CLAMP_DIST,
                      reg_lambda: float = CODE_REG_LAMBDA, epoch: Optional[int] = None,
                      dtype: str = "bf16", generator: Optional[torch.Generator] = None,
                      state: Optional[AutoDecoderState] = None, group=None) -> AutoDecoderState:
    """Fit the decoder and one latent per shape to SDF samples (DeepSDF auto-decoder).

    xyz: [n_shapes, n_samples, 3], sdf: [n_shapes, n_samples] on the GPU.  Each step draws
    ``shapes_per_batch`` shapes (without replacement) and ``samples_per_shape`` samples of each
    (DeepSDF: 64 scenes x 16384 samples).  Codes start at N(0, 1/L) (CodeInitStdDev 1 / sqrt L);
    both parameter sets use Adam.  Data parallel over the group: every rank draws the same
    shapes, takes its contiguous share of them, and the weight gradients are all-reduced
    (averaged).  The latents are replicated; each rank updates its own shapes' rows and the
    updated rows are all-reduced, so all ranks keep the same table.  ``decoder``'s weights are
    updated in place at the end.
    """
    capi.require_device(xyz, sdf)
    device = xyz.device
    L, H = _check_decoder(decoder)
    n_shapes, n_samples = sdf.shape
    S = min(shapes_per_batch or n_shapes, n_shapes)
    P = min(samples_per_shape or n_samples, n_samples)
    world, rank = ldist.world_and_rank(group)
    if state is None:
        state = AutoDecoderState()
        state.masters = {}
        for l in range(9):
            state.masters[f"W{l}"] = decoder.weights[l].to(device).clone()
            state.masters[f"b{l}"] = decoder.biases[l].to(device).clone()
        seed = 0 if generator is None else int(
            torch.randint(0, 2 ** 31, (1,), generator=generator, device=generator.device))
        gen = torch.Generator().manual_seed(seed)
        state.latents = (torch.randn(n_shapes, L, generator=gen) / math.sqrt(L)).to(device)
        state.optimizer = torch.optim.Adam(list(state.masters.values()), lr=lr_decoder)
        state.lat_optimizer = torch.optim.Adam([state.latents], lr=lr_latent)
    grads = {k: torch.empty_like(v) for k, v in state.masters.items()}
    lat_grad = torch.zeros_like(state.latents)
    for _ in range(steps):
        sidx = torch.randperm(n_shapes, device=device, generator=generator)[:S]
        pidx = torch.randint(0, n_samples, (S, P), device=device, generator=generator)
        lo, hi = ldist.batch_shard(S, rank, world)
        mine = sidx[lo:hi]
        pts = torch.gather(xyz[mine], 1, pidx[lo:hi, :, None].expand(-1, -1, 3)).contiguous()
        tgt = torch.gather(sdf[mine], 1, pidx[lo:hi]).contiguous()
        z = state.latents[mine].contiguous()
        ep = state.step if epoch is None else epoch
        loss, grads, gz = autodecoder_train_step(
            state.masters, z, pts, tgt, latent_dim=L, hidden=H, skip=decoder.skip, delta=delta,
            reg_lambda=reg_lambda, epoch=ep, dtype=dtype, grads=grads)
        ldist.allreduce_mean_([grads[k] for k in state.masters], group=group)
        lat_grad.zero_()
        lat_grad[mine] = gz * ((hi - lo) / S)     # this rank's share of the batch mean
        ldist.allreduce_sum_([lat_grad], group=group)
        for k, p in state.masters.items():
            p.grad = grads[k]
        state.latents.grad = lat_grad
        state.optimizer.step()
        state.lat_optimizer.step()
        state.step += 1
        state.losses.append(loss)
    pend = [i for i, l in enumerate(state.losses) if isinstance(l, torch.Tensor)]
    if pend:                     # one device->host transfer for the whole run
        vals = torch.cat([state.losses[i].reshape(1).float() for i in pend]).tolist()
        for i, v in zip(pend, vals):
            state.losses[i] = v
    for l in range(9):
        decoder.weights[l] = state.masters[f"W{l}"].detach().to("cpu").contiguous()
        decoder.biases[l] = state.masters[f"b{l}"].detach().to("cpu").contiguous()
    decoder.invalidate()
    return state
