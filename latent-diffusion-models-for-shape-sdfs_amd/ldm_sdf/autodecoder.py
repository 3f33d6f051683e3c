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
                           grads: Optional[Dict[str, torch.Tensor]] = None,
                           wgrad_tile: Optional[int] = None
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
    if dtype == "bf16":
        return _train_step_gemm_bf16(masters, z, xyz, sdf, L=L, H=H, skip=skip, delta=delta,
                                     reg_lambda=reg_lambda, epoch=epoch, grads=grads,
                                     wgrad_tile=WGRAD_TILE if wgrad_tile is None else wgrad_tile)
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


_KQ = 128          # row padding of the sample axis (the K of the weight-gradient products)
# ldm_gemm_bf16 tile of the weight-gradient products (128 x 128: each slice walks KT = 8192
# samples, long enough for the bigger tile's per-CU operand economy); tuning runs pass
# ``wgrad_tile`` to autodecoder_train_step (the product reads no environment variable).
# Round 6 sweep (scripts/ad_wgrad_ab.py, profiles/r06am): the persistent 128 x 128 tile on a
# 2-deep ring (17) 30.9-31.1 ms/step, 14 31.0, the earlier 3 31.3-31.9, others 32-34; same bits
WGRAD_TILE = 17
_KSEG = 64         # column padding of [z || xyz] (a GEMM K segment)


def _ad_inputs(z, xyz, S, P, Np, zw, KT, gather=False):
    """The bf16 step's input operand in both layouts: ``Zx`` [Np, zw] = [z_s || xyz || 0] per
    sample (rows >= N zero) and ``ZxT`` [Np / KT, zw, KT], its k-blocked transpose.  Samples are
    shape-major (sample m belongs to shape m // P), so the code columns are a broadcast of z per
    shape: when P is a multiple of KT every block lies in one shape and both layouts are written
    by broadcast copies (round 6: the index gathers of [N, L] took ≈ 1 ms of the 64 x 16384
    step); else (or ``gather``) by the per-sample gathers.  Same values either way
    (``tests/test_autodecoder_inputs.py``)."""
    L = z.shape[1]
    N = S * P
    nblk = Np // KT
    dev = z.device
    bf = dict(device=dev, dtype=torch.bfloat16)
    Zx = torch.zeros(Np, zw, **bf)
    ZxT = torch.zeros(nblk, zw, KT, **bf)
    if not gather and P % KT == 0:
        zb = z.to(torch.bfloat16)
        Zx[:N].view(S, P, zw)[:, :, :L] = zb[:, None, :]
        ZxT[:N // KT].view(S, P // KT, zw, KT)[:, :, :L, :] = zb[:, None, :, None]
    else:
        owner_pad = torch.full((Np,), S, device=dev, dtype=torch.long)
        owner_pad[:N] = torch.arange(S, device=dev).repeat_interleave(P)
        Zx[:N, :L] = z[owner_pad[:N]]
        zT = torch.zeros(L, S + 1, **bf)          # column S: the padding rows' zero code
        zT[:, :S] = z.t()
        ZxT.permute(1, 0, 2)[:L] = zT[:, owner_pad.view(nblk, KT)]
    Zx[:N, L:L + 3] = xyz.reshape(N, 3)
    xyz_pad = torch.zeros(Np, 3, device=dev, dtype=torch.float32)
    xyz_pad[:N] = xyz.reshape(N, 3)
    ZxT.permute(1, 0, 2)[L:L + 3] = xyz_pad.t().reshape(3, nblk, KT).to(torch.bfloat16)
    return Zx, ZxT


def _train_step_gemm_bf16(masters, z, xyz, sdf, *, L, H, skip, delta, reg_lambda, epoch,
                          grads, wgrad_tile=WGRAD_TILE):
    """bf16 matrix-core step on ``ldm_gemm_bf16`` (include/ldm_sdf.h).

    Every activation is kept once in bf16, in both layouts: ``h_l`` [Np, w] (the A operand of
    the next forward product and of the G W products' ReLU mask) and ``h_l^T`` [w, Np] (the B
    operand of the weight gradients, whose sum runs over the samples).  The epilogues write
    them (``Cb`` / ``CbT``), the ReLU backward rides in the G W products (``relu_bwd`` on the
    saved bf16 post-activation), the bias gradients are the epilogues' 32-row column sums, and
    the weight gradients are split-K products over the sample axis.  The latent gradient needs
    no [N, L] product: per shape, ``sum_p g4 W4z + g0 W0`` = (per-shape column sums of g4 and
    g0) x the latent columns, a [S, H] x [H, L] product in fp32.  Numerics: operands rounded to
    bf16 (RNE), fp32 accumulation -- as the ``ldm_linear`` bf16 path."""
    dev = z.device
    S, P = sdf.shape
    N = S * P
    Np = -(-N // _KQ) * _KQ
    hs = masters[f"W{skip - 1}"].shape[0]
    hsp = -(-hs // 64) * 64                      # skip width padded to a GEMM K segment
    zw = -(-(L + 3) // _KSEG) * _KSEG
    bf = dict(device=dev, dtype=torch.bfloat16)
    f32 = dict(device=dev, dtype=torch.float32)

    # ---- working weights (bf16, padded) and their transposes for the G W products
    W = {}
    W0 = torch.zeros(H, zw, **bf)
    W0[:, :L + 3] = masters["W0"]
    W["W0"] = W0
    for l in range(1, 8):
        if l == skip - 1:
            Wp = torch.zeros(hsp, H, **bf)
            Wp[:hs] = masters[f"W{l}"]
            W[f"W{l}"] = Wp
        elif l == skip:
            Ws = masters[f"W{l}"]
            Wh = torch.zeros(H, hsp, **bf)
            Wh[:, :hs] = Ws[:, :hs]
            Wz = torch.zeros(H, zw, **bf)
            Wz[:, :L + 3] = Ws[:, hs:]
            W["W4h"], W["W4z"] = Wh, Wz
        else:
            W[f"W{l}"] = masters[f"W{l}"].to(torch.bfloat16)
    WT = {k: v.t().contiguous() for k, v in W.items() if k != "W0"}
    bias = {f"b{l}": masters[f"b{l}"].contiguous() for l in range(9)}
    bp = torch.zeros(hsp, **f32)
    bp[:hs] = masters[f"b{skip - 1}"]
    bias[f"b{skip - 1}"] = bp
    # the 512 -> 1 layer as a K = 64 product for its backward (g8 in column 0, zeros beside)
    w8 = masters["W8"].reshape(-1)
    W8T = torch.zeros(H, 64, **bf)
    W8T[:, 0] = w8
    W8 = w8.to(torch.bfloat16).reshape(1, H).contiguous()

    # ---- inputs: Zx = [z_s || xyz || 0] per sample, rows >= N zero, both layouts.  The
    # sample-axis (transposed) operands are k-BLOCKED, [nblk][width][KT]: a weight-gradient
    # slice is one block, so the rows it streams lie KT * 2 bytes apart inside one block
    # instead of 2 MB apart (one memory page per row: measured 9 us per k-step, TLB-bound).
    KT = next(kt for kt in (8192, 4096, 2048, 1024, 512, 256, 128) if Np % kt == 0)
    nblk = Np // KT
    Zx, ZxT = _ad_inputs(z, xyz, S, P, Np, zw, KT)

    # ---- forward: h_l = ReLU(...) in bf16, both layouts (rows >= N written as zeros)
    h, hT = [], []
    x = Zx
    for l in range(8):
        width = hsp if l == skip - 1 else H
        y = torch.empty(Np, width, **bf)
        yT = torch.empty(nblk, width, KT, **bf)
        segs = ([(x, W["W4h"]), (Zx, W["W4z"])] if l == skip else [(x, W[f"W{l}"])])
        ops.gemm([ops.gemm_problem(segs, Np, width, mode="relu", M_valid=N, bias=bias[f"b{l}"],
                                   Cb=y, CbT=yT, ct_blk=KT)])
        h.append(y)
        hT.append(yT)
        x = y
    pre = torch.empty(Np, 1, **f32)
    ops.gemm([ops.gemm_problem([(x, W8)], Np, 1, M_valid=N, bias=bias["b8"], C=pre)])
    loss, g8 = ops.sdf_l1_loss(pre[:N].reshape(N, 1), sdf.reshape(N, 1).contiguous(), delta,
                               1.0 / N)

    # ---- backward
    gw = {}
    gb = {}
    ws_cache = {}

    def ws_for(n, slot):
        # keyed by (size, slot in the launch's problem list): two problems of ONE launch must
        # never share partial slabs, even when their sizes agree (e.g. S == zw on the one-hot
        # path); launches run in stream order, so reuse across launches is safe
        t = ws_cache.get((n, slot))
        if t is None:
            t = ws_cache[(n, slot)] = torch.empty(n, **f32)
        return t

    def wgrad(gT, xT, M_, N_, out, slot):
        """out [M_, N_] fp32 = sum over the samples of gT x xT^T; gT [nblk, M_, KT] and
        xT [nblk, N_, KT] blocked: split-K with one slice per block.  `slot` = the problem's
        index within its launch (its own split-K workspace)."""
        if nblk == 1:
            return ops.gemm_problem([(gT[0], xT[0])], M_, N_, C=out)
        return ops.gemm_problem([(gT[0], xT[0])], M_, N_, C=out, k_split=nblk,
                                ws=ws_for(nblk * M_ * N_, slot),
                                slices=(gT.shape[1] * KT, xT.shape[1] * KT))

    # layer 8: dW8 = g8^T h7, db8 = sum g8; g7 = (g8 w8) * [h7 > 0]
    g8b = torch.zeros(Np, 64, **bf)
    g8b[:N, 0] = g8.reshape(N)
    g8row = g8b[:, 0].contiguous().reshape(nblk, 1, KT)      # blocked [nblk][1][KT]
    gw["W8"] = torch.empty(1, H, **f32)
    gb["b8"] = torch.empty(1, **f32)
    ops.colsum(g8.reshape(N, 1), gb["b8"])
    nrow32 = -(-Np // 32)
    g_cur = torch.empty(Np, H, **bf)
    gT_cur = torch.empty(nblk, H, KT, **bf)
    cs = torch.empty(nrow32, H, **f32)
    ops.gemm([ops.gemm_problem([(g8b, W8T)], Np, H, mode="relu_bwd", M_valid=N, Rb=h[7],
                               Cb=g_cur, CbT=gT_cur, colsum=cs, ct_blk=KT)])
    ops.gemm([wgrad(g8row, hT[7], 1, H, gw["W8"], 0)], tile=wgrad_tile)
    colsums = {7: cs}
    gcs = {}                                       # g_l per 32-row block sums (bias / latent)
    Gs = {}                                        # per-shape column sums of g_skip and g_0
    onehot = None
    if P % 32:                                     # 32-row blocks straddle shapes: a one-hot
        sid = torch.arange(S, device=dev)[:, None, None]   # product sums each shape's rows
        owner_pad = torch.full((Np,), S, device=dev, dtype=torch.long)
        owner_pad[:N] = torch.arange(S, device=dev).repeat_interleave(P)
        onehot = (owner_pad.view(1, nblk, KT) == sid).to(torch.bfloat16).permute(1, 0, 2)
        onehot = onehot.contiguous()               # blocked [nblk][S][KT]
    for l in range(7, -1, -1):
        # g_cur = dL/d pre_l (bf16, both layouts); its column sums are colsums[l]
        gcs[l] = colsums[l]
        wout = hsp if l == skip - 1 else H
        if l == skip:
            gw["W4h"] = torch.empty(H, hsp, **f32)
            gw["W4z"] = torch.empty(H, zw, **f32)
            probs = [wgrad(gT_cur, hT[l - 1], H, hsp, gw["W4h"], 0),
                     wgrad(gT_cur, ZxT, H, zw, gw["W4z"], 1)]
        elif l == 0:
            gw["W0"] = torch.empty(H, zw, **f32)
            probs = [wgrad(gT_cur, ZxT, H, zw, gw["W0"], 0)]
        else:
            win = h[l - 1].shape[1]
            gw[f"W{l}"] = torch.empty(wout, win, **f32)
            probs = [wgrad(gT_cur, hT[l - 1], wout, win, gw[f"W{l}"], 0)]
        if onehot is not None and l in (skip, 0):
            Gs[l] = torch.empty(S, H, **f32)
            probs.append(wgrad(onehot, gT_cur, S, H, Gs[l], len(probs)))
        # weight gradients (long K per slice): larger tiles than the 1M-row G W product, so
        # their own launch
        ops.gemm(probs, tile=wgrad_tile)
        if l > 0:
            win = h[l - 1].shape[1]
            WdT = WT["W4h"] if l == skip else WT[f"W{l}"]          # [win, wout]
            g_nxt = torch.empty(Np, win, **bf)
            gT_nxt = torch.empty(nblk, win, KT, **bf)
            cs = torch.empty(nrow32, win, **f32)
            ops.gemm([ops.gemm_problem([(g_cur, WdT)], Np, win, mode="relu_bwd", M_valid=N,
                                       Rb=h[l - 1], Cb=g_nxt, CbT=gT_nxt, colsum=cs,
                                       ct_blk=KT)])
            colsums[l - 1] = cs
        if l > 0:
            g_prev_keep = (g_cur, gT_cur)            # noqa: F841 (alive until the launch is queued)
            g_cur, gT_cur = g_nxt, gT_nxt
    for l in range(8):
        width = gcs[l].shape[1]
        gb[f"b{l}"] = torch.empty(width, **f32)
        ops.colsum(gcs[l], gb[f"b{l}"])

    # ---- latent gradient: per shape sum_p (g4 W4z + g0 W0)[:, :L]
    if onehot is None:                             # shape s = 32-row blocks [s P/32, (s+1) P/32)
        for l in (skip, 0):
            Gs[l] = torch.empty(S, H, **f32)
            ops.colsum_segments(gcs[l][:N // 32].contiguous(), S, Gs[l])
    G4, G0 = Gs[skip], Gs[0]
    gz = torch.empty(S, L, **f32)
    Wm = masters[f"W{skip}"]
    ops.linear(G4, Wm[:, hs:hs + L].t(), gz, compute=capi.COMPUTE_FP32)
    ops.linear(G0, masters["W0"][:, :L].t(), gz, epi=capi.EPI_ACCUM, compute=capi.COMPUTE_FP32)
    coef = reg_lambda * min(1.0, epoch / 100.0) / S
    if coef != 0.0:
        ops.latent_l2_reg(z, coef, loss, gz)

    if grads is None:
        grads = {k: torch.empty_like(v) for k, v in masters.items()}
    grads["W0"].copy_(gw["W0"][:, :L + 3])
    for l in range(1, 9):
        if l == skip - 1:
            grads[f"W{l}"].copy_(gw[f"W{l}"][:hs])
            grads[f"b{l}"].copy_(gb[f"b{l}"][:hs])
            continue
        if l == skip:
            grads[f"W{l}"][:, :hs].copy_(gw["W4h"][:, :hs])
            grads[f"W{l}"][:, hs:].copy_(gw["W4z"][:, :L + 3])
        else:
            grads[f"W{l}"].copy_(gw[f"W{l}"].reshape(grads[f"W{l}"].shape))
        grads[f"b{l}"].copy_(gb[f"b{l}"].reshape(grads[f"b{l}"].shape))
    grads["b0"].copy_(gb["b0"])
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
