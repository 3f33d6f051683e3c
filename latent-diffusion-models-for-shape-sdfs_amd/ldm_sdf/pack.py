"""Host-side weight packing for the decoder kernels.

Canonical DeepSDF weights (``[out, in]`` per linear, weight-norm already folded -- see
``fold_weight_norm``) are turned into what ``libldm_sdf.so`` streams:

* bf16/f16 MFMA kernel: a *stage blob*.  Every stage is 8 KiB = 8 A-fragments of
  ``v_mfma_f32_32x32x16`` (8 output m-chunks of 32 rows x one 16-wide k-step), stored
  ``[chunk i][lane l][element j]``: element ``(i, l, j)`` of the main stage (layer, pass p,
  k-step ks) is ``W[(8p+i)*32 + (l&31), 16*ks + PERM[8*(l>>5) + j]]``.  ``PERM`` is the row
  order in which a 32x32 accumulator, converted pairwise to 16-bit, becomes the next layer's
  B fragment (cdna_hip_programming.md §3, 'accumulator tile as the next MFMA's operand').
  Each pass ends with one *aux* stage whose columns ``[wx,wy,wz,wx,wy,wz,b_hi,b_lo]`` meet the
  B fragment ``[x_hi,y_hi,z_hi,x_lo,y_lo,z_lo,1,1]``: bias (and xyz for layers 0/4) enter the
  MFMA with ~16 significant bits.  Aux stages of layers 0 and 4 depend on the shape (they
  carry the folded latent) and are written per call into the workspace by ``aux_pack_kernel``.
* fp32 parity kernel: ``W_l^T`` blocks (``[K_l][M_l]``) followed by ``b_l`` for l = 1..7.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

H = 512
STAGE_BYTES = 8192

# k' = 8h + j  ->  feature offset inside a 16-wide k-step (see module docstring)
PERM = np.array([8 * (j >> 2) + 4 * h + (j & 3) for h in range(2) for j in range(8)],
                dtype=np.int64)


def fold_weight_norm(g: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """``torch.nn.utils.weight_norm`` (dim=0) folded: ``w = g * v / ||v||_row``.
    DeepSDF trains with weight-norm on every hidden layer; inference uses the folded w."""
    norm = v.flatten(1).norm(dim=1).reshape(-1, *([1] * (v.dim() - 1)))
    return g.reshape(norm.shape) * v / norm


def skip_pad(skip_width: int) -> int:
    if skip_width == 253:
        return 256
    if skip_width == 512:
        return 512
    raise ValueError(f"GPU decoder supports skip width 253 or 512, got {skip_width}")


@dataclass(frozen=True)
class StageRef:
    layer: int
    pass_: int
    ks: int          # -1 = aux stage
    per_shape: bool  # aux stage of layer 0 / 4 (filled per call from the folded latent)


def stage_plan(skip_width: int) -> List[StageRef]:
    """The per-tile stage sequence the kernel consumes (csrc/decoder.hip Passes<S>)."""
    S = skip_pad(skip_width)
    # (layer, passes, main k-steps)
    layers = [(0, 2, 0), (1, 2, 32), (2, 2, 32), (3, S // 256, 32), (4, 2, S // 16),
              (5, 2, 32), (6, 2, 32), (7, 2, 32)]
    plan = []
    for (l, npass, ks_n) in layers:
        for p in range(npass):
            for ks in range(ks_n):
                plan.append(StageRef(l, p, ks, False))
            plan.append(StageRef(l, p, -1, l in (0, 4)))
    return plan


def n_stages(skip_width: int, layout: str = "pass8") -> int:
    return len(stage_plan_quarter(skip_width) if layout == "quarter" else stage_plan(skip_width))


def stage_plan_quarter(skip_width: int) -> List[StageRef]:
    """Stage sequence of the quarter-pipelined kernel (csrc/decoder_q.hip): per layer, quarters
    of 4 m-chunks; per quarter, K/32 pair-stages (4 chunks x k-steps 2j, 2j+1) then one aux
    stage.  ``pass_`` holds the quarter index and ``ks`` the pair index j (-1 = aux)."""
    S = skip_pad(skip_width)
    layers = [(0, 4, 0), (1, 4, 16), (2, 4, 16), (3, S // 128, 16), (4, 4, S // 32),
              (5, 4, 16), (6, 4, 16), (7, 4, 16)]
    plan = []
    for (l, nq, kp) in layers:
        for q in range(nq):
            for j in range(kp):
                plan.append(StageRef(l, q, j, False))
            plan.append(StageRef(l, q, -1, l in (0, 4)))
    return plan


def _round(x: torch.Tensor, dt: torch.dtype) -> torch.Tensor:
    return x.to(torch.float32).to(dt)


def _hi_lo(b: torch.Tensor, dt: torch.dtype) -> Tuple[torch.Tensor, torch.Tensor]:
    b = b.to(torch.float32)
    hi = b.to(dt)
    lo = (b - hi.to(torch.float32)).to(dt)
    return hi, lo


def canonical_pieces(weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor],
                     latent_dim: int) -> Dict[str, torch.Tensor]:
    """Split canonical DeepSDF weights into the h-part / latent / xyz pieces (float64)."""
    W = [w.detach().to("cpu", torch.float64) for w in weights]
    b = [x.detach().to("cpu", torch.float64) for x in biases]
    L = latent_dim
    if len(W) != 9 or W[0].shape[0] != H:
        raise ValueError("GPU decoder packing expects DeepSDF 8x512 (9 linears)")
    sw = W[3].shape[0]
    if W[4].shape[1] != sw + L + 3:
        raise ValueError("layer 4 input must be [h3 || z || xyz]")
    return {
        "main": [None, W[1], W[2], W[3], W[4][:, :sw], W[5], W[6], W[7]],
        "bias": [b[0], b[1], b[2], b[3], b[4], b[5], b[6], b[7]],
        "wz": torch.stack([W[0][:, :L], W[4][:, sw:sw + L]]),
        "bz": torch.stack([b[0], b[4]]),
        "wxyz": torch.stack([W[0][:, L:L + 3], W[4][:, sw + L:sw + L + 3]]),
        "w_last": W[8][0],
        "b_last": b[8][0],
        "skip_width": sw,
    }


def pack_stage_blob(pieces: Dict[str, torch.Tensor], dt: torch.dtype) -> torch.Tensor:
    """bf16/f16 stage blob ``[n_stages, 8, 64, 8]`` (see module docstring)."""
    sw = pieces["skip_width"]
    S = skip_pad(sw)
    plan = stage_plan(sw)
    lanes = np.arange(64)
    rows_l = lanes & 31                                  # [64]
    kcols = np.array([[PERM[8 * (l >> 5) + j] for j in range(8)] for l in lanes])  # [64, 8]
    padded = {}
    for l in range(1, 8):
        w = pieces["main"][l]
        M = S if l == 3 else H
        K = S if l == 4 else H
        wp = torch.zeros(M, K, dtype=torch.float64)
        wp[:w.shape[0], :w.shape[1]] = w
        padded[l] = _round(wp, dt)
    out = torch.zeros(len(plan), 8, 64, 8, dtype=dt)
    for si, st in enumerate(plan):
        if st.per_shape:
            continue   # filled per call in the workspace
        if st.ks >= 0:
            wp = padded[st.layer]
            rows = (st.pass_ * 8 + np.arange(8))[:, None] * 32 + rows_l[None, :]   # [8, 64]
            cols = st.ks * 16 + kcols                                                # [64, 8]
            out[si] = wp[torch.from_numpy(rows)[:, :, None], torch.from_numpy(cols)[None, :, :]]
        else:
            b = pieces["bias"][st.layer]
            M = b.shape[0]
            bp = torch.zeros(S if st.layer == 3 else H, dtype=torch.float64)
            bp[:M] = b
            hi, lo = _hi_lo(bp, dt)
            f = (st.pass_ * 8 + np.arange(8))[:, None] * 32 + np.arange(32)[None, :]  # [8, 32]
            ft = torch.from_numpy(f)
            out[si, :, :32, 6] = hi[ft]
            out[si, :, :32, 7] = lo[ft]
    return out


def pack_stage_blob_quarter(pieces: Dict[str, torch.Tensor], dt: torch.dtype) -> torch.Tensor:
    """Quarter-layout blob ``[n_stages, 8, 64, 8]``: main stage (layer, quarter q, pair j) frag
    ``i = e*4 + c`` is the A fragment of m-chunk ``4q + c`` at k-step ``2j + e``; the aux stage
    has ``[0,0,0,0,0,0,b_hi,b_lo]`` in frags 0..3 (lanes < 32) and zero frags 4..7."""
    sw = pieces["skip_width"]
    S = skip_pad(sw)
    plan = stage_plan_quarter(sw)
    lanes = np.arange(64)
    rows_l = lanes & 31
    kcols = np.array([[PERM[8 * (l >> 5) + j] for j in range(8)] for l in lanes])  # [64, 8]
    padded = {}
    for l in range(1, 8):
        w = pieces["main"][l]
        M = S if l == 3 else H
        K = S if l == 4 else H
        wp = torch.zeros(M, K, dtype=torch.float64)
        wp[:w.shape[0], :w.shape[1]] = w
        padded[l] = _round(wp, dt)
    out = torch.zeros(len(plan), 8, 64, 8, dtype=dt)
    fr = np.arange(8)
    chunk_of = fr % 4            # frag i = e*4 + c
    e_of = fr // 4
    for si, st in enumerate(plan):
        if st.per_shape:
            continue
        q = st.pass_
        if st.ks >= 0:
            wp = padded[st.layer]
            rows = (4 * q + chunk_of)[:, None] * 32 + rows_l[None, :]              # [8, 64]
            ks = 2 * st.ks + e_of                                                   # [8]
            cols = ks[:, None, None] * 16 + kcols[None, :, :]                       # [8, 64, 8]
            out[si] = wp[torch.from_numpy(rows)[:, :, None], torch.from_numpy(cols)]
        else:
            b = pieces["bias"][st.layer]
            bp = torch.zeros(S if st.layer == 3 else H, dtype=torch.float64)
            bp[:b.shape[0]] = b
            hi, lo = _hi_lo(bp, dt)
            f = (4 * q + np.arange(4))[:, None] * 32 + np.arange(32)[None, :]      # [4, 32]
            ft = torch.from_numpy(f)
            out[si, :4, :32, 6] = hi[ft]
            out[si, :4, :32, 7] = lo[ft]
    return out


def permute_w_last(w_last: torch.Tensor) -> torch.Tensor:
    """``wl[(mc*2 + h)*16 + r] = w8[32 mc + (r&3) + 8 (r>>2) + 4 h]`` (accumulator row order)."""
    idx = [32 * mc + (r & 3) + 8 * (r >> 2) + 4 * h
           for mc in range(16) for h in range(2) for r in range(16)]
    return w_last.to(torch.float32)[torch.tensor(idx)]


def pack_f32_blob(pieces: Dict[str, torch.Tensor]) -> torch.Tensor:
    """fp32 parity-kernel blob: for l = 1..7, ``W_l^T`` then ``b_l`` (b_4 slot zeroed)."""
    parts = []
    for l in range(1, 8):
        w = pieces["main"][l]
        parts.append(w.T.contiguous().reshape(-1))
        parts.append(torch.zeros(w.shape[0], dtype=torch.float64) if l == 4
                     else pieces["bias"][l])
    return torch.cat(parts).to(torch.float32)


def pack_decoder(weights, biases, latent_dim: int, dtype: str,
                 layout: str = "quarter") -> Dict[str, object]:
    """All host-side arrays of an ``ldm_decoder_t`` for ``dtype`` in {fp32, bf16, fp16}; the
    16-bit stage blob in ``layout`` ("quarter": csrc/decoder_q.hip, "pass8": decoder.hip)."""
    pieces = canonical_pieces(weights, biases, latent_dim)
    out = {
        "skip_width": pieces["skip_width"],
        "latent_dim": latent_dim,
        "wz": pieces["wz"].to(torch.float32).contiguous(),
        "bz": pieces["bz"].to(torch.float32).contiguous(),
        "wxyz": pieces["wxyz"].to(torch.float32).contiguous(),
        "b_last": float(pieces["b_last"]),
    }
    out["layout"] = layout
    if dtype == "fp32":
        out["weights"] = pack_f32_blob(pieces)
        out["w_last"] = pieces["w_last"].to(torch.float32).contiguous()
        out["n_stages"] = 0
    elif dtype in ("bf16", "fp16"):
        dt = torch.bfloat16 if dtype == "bf16" else torch.float16
        blob = (pack_stage_blob_quarter(pieces, dt) if layout == "quarter"
                else pack_stage_blob(pieces, dt))
        out["weights"] = blob.contiguous()
        out["w_last"] = permute_w_last(pieces["w_last"]).contiguous()
        out["n_stages"] = n_stages(pieces["skip_width"], layout)
    else:
        raise ValueError(f"unknown decoder dtype {dtype!r}")
    return out
