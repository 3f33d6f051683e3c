"""Host-side weight packing for the decoder kernels.

Canonical DeepSDF weights (``[out, in]`` per linear, weight-norm already folded -- see
``fold_weight_norm``) are turned into what ``libldm_sdf.so`` streams:

* bf16/f16 MFMA kernel: per-wave weight streams of ``v_mfma_f32_32x32x16`` A fragments
  ("split", csrc/decoder_fs.hip, ``pack_split``), each fragment stored ``[lane l][element j]``.
  ``PERM`` is the row order in which a 32x32 accumulator, converted pairwise to 16-bit,
  becomes the next layer's B fragment (cdna_hip_programming.md §3, 'accumulator tile as the
  next MFMA's operand').  Bias (and xyz for layers 0/4) enter as an *aux* k-step whose columns
  ``[wx,wy,wz,wx,wy,wz,b_hi,b_lo]`` meet the B fragment ``[x_hi,y_hi,z_hi,x_lo,y_lo,z_lo,1,1]``
  (~16 significant bits); the aux fragments of layers 0 and 4 carry the folded latent and are
  written per call into the workspace by the kernel's aux pack.
* fp32 parity kernel: ``W_l^T`` blocks (``[K_l][M_l]``) followed by ``b_l`` for l = 1..7.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

H = 512

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


def n_stages(skip_width: int, layout: str = "split") -> int:
    """``ldm_decoder_t.n_stages`` of a 16-bit blob in ``layout`` (split: k-steps per wave)."""
    if layout == "split":
        return split_stream_steps(skip_width)
    raise ValueError(f"unknown decoder layout {layout!r} (pass8 / quarter were removed in ABI "
                     "5, split16 in ABI 7)")


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


# ------------------------------------------------------------------------------------------
# "split" layout (csrc/decoder_fs.hip): the FEATURES of every layer are split
# over the 4 waves of a workgroup, the 128 points of a tile are shared through an LDS activation
# buffer.  Wave w owns output rows [128w, 128w+128) of every 512-wide layer, as two PARTS of
# 64 rows (2 m-chunks); layer 3 at skip width 253 (padded 256) has one part of rows
# [64w, 64w+64).  Each wave streams ITS OWN weight fragments (2 per k-step) from L2 straight
# into registers: every weight byte still feeds the tile's 128 points, but each A fragment read
# feeds 4 MFMAs (4 point chunks) instead of 1.
# ------------------------------------------------------------------------------------------
SPLIT_WAVES = 4


def split_parts(skip_width: int) -> List[Tuple[int, int]]:
    """(layer, part) in the kernel's order (csrc/decoder_fs.hip)."""
    S = skip_pad(skip_width)
    parts = [(0, 0), (0, 1), (1, 0), (1, 1), (2, 0), (2, 1)]
    parts += [(3, 0)] if S == 256 else [(3, 0), (3, 1)]
    parts += [(l, p) for l in (4, 5, 6, 7) for p in (0, 1)]
    return parts


def split_nk(layer: int, skip_width: int) -> int:
    """Ring k-steps (16 features each) of one part of ``layer`` (the aux step not counted)."""
    return 0 if layer == 0 else (skip_pad(skip_width) // 16 if layer == 4 else 32)


def split_kidx(layer: int, skip_width: int) -> np.ndarray:
    """Input k-step consumed at ring step j of ``layer``.  The previous layer's activations sit
    in LDS as 32 k-steps of 16 features; when it was 512 wide (two parts per wave) its part 0
    ("early", k-steps 8w..8w+3) is written at the layer boundary and its part 1 ("late",
    8w+4..8w+7) during this layer's first steps, so early k-steps are consumed first:
    step j = 16u + 4g + r reads k-step 8g + 4u + r.  After the one-part layer 3 (skip 253) the
    16 k-steps are read in order."""
    nk = split_nk(layer, skip_width)
    j = np.arange(nk)
    if layer == 4 and skip_pad(skip_width) == 256:
        return j
    return 8 * ((j >> 2) & 3) + 4 * (j >> 4) + (j & 3)


def split_row_base(layer: int, part: int, wave: int, skip_width: int) -> int:
    if layer == 3 and skip_pad(skip_width) == 256:
        return 64 * wave
    return 128 * wave + 64 * part


def split_stream_steps(skip_width: int) -> int:
    return sum(split_nk(l, skip_width) for (l, _) in split_parts(skip_width))


def pack_split(pieces: Dict[str, torch.Tensor], dt: torch.dtype) -> Tuple[torch.Tensor, int]:
    """Split-layout blob: ``stream [4 waves][n_steps][2 frags][64 lanes][8]`` then
    ``bias_aux [4 waves][n_parts][2 frags][64 lanes][8]``.  Stream element (wave w, step s of
    part (l, p) at ring step j, m-chunk i, lane ln, elem e) =
    ``W_l[row_base + 32 i + (ln & 31), 16 kidx_l(j) + PERM[8 (ln >> 5) + e]]``.  The bias aux
    fragment of a part (lanes < 32, row ``row_base + 32 i + ln``) is
    ``[0,0,0,0,0,0,b_hi,b_lo]``; the parts of layers 0 and 4 are per shape (workspace, filled
    by the kernel's aux pack) and stay zero here.  Returns (flat blob, n_steps)."""
    sw = pieces["skip_width"]
    S = skip_pad(sw)
    parts = split_parts(sw)
    nsteps = split_stream_steps(sw)
    lanes = np.arange(64)
    rows_l = torch.from_numpy(lanes & 31)
    kcols = torch.from_numpy(np.array([[PERM[8 * (l >> 5) + j] for j in range(8)]
                                       for l in lanes]))                          # [64, 8]
    padded = {}
    for l in range(1, 8):
        w = pieces["main"][l]
        M = S if l == 3 else H
        K = S if l == 4 else H
        wp = torch.zeros(M, K, dtype=torch.float64)
        wp[:w.shape[0], :w.shape[1]] = w
        padded[l] = _round(wp, dt)
    stream = torch.zeros(SPLIT_WAVES, nsteps, 2, 64, 8, dtype=dt)
    aux = torch.zeros(SPLIT_WAVES, len(parts), 2, 64, 8, dtype=dt)
    for w in range(SPLIT_WAVES):
        s0 = 0
        for pi, (l, p) in enumerate(parts):
            rb = split_row_base(l, p, w, sw)
            rows = (rb + 32 * torch.arange(2))[:, None] + rows_l[None, :]           # [2, 64]
            if l not in (0, 4):
                b = pieces["bias"][l]
                bp = torch.zeros(S if l == 3 else H, dtype=torch.float64)
                bp[:b.shape[0]] = b
                hi, lo = _hi_lo(bp, dt)
                aux[w, pi, :, :32, 6] = hi[rows[:, :32]]
                aux[w, pi, :, :32, 7] = lo[rows[:, :32]]
            if l == 0:
                continue
            kidx = torch.from_numpy(split_kidx(l, sw))
            nk = kidx.numel()
            cols = kidx[:, None, None] * 16 + kcols[None]                           # [nk, 64, 8]
            wp = padded[l]
            # [nk, 2, 64, 8]: W[rows[i, ln], cols[j, ln, e]]
            stream[w, s0:s0 + nk] = wp[rows[None, :, :, None], cols[:, None, :, :]]
            s0 += nk
        assert s0 == nsteps
    return torch.cat([stream.reshape(-1), aux.reshape(-1)]), nsteps


def permute_w_last_split(w_last: torch.Tensor) -> torch.Tensor:
    """Final-layer weights in the split kernel's accumulator order:
    ``wl[w][p][i][h][v] = w8[128 w + 64 p + 32 i + (v & 3) + 8 (v >> 2) + 4 h]``."""
    idx = [128 * w + 64 * p + 32 * i + (v & 3) + 8 * (v >> 2) + 4 * h
           for w in range(4) for p in range(2) for i in range(2) for h in range(2)
           for v in range(16)]
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
                 layout: str = "split") -> Dict[str, object]:
    """All host-side arrays of an ``ldm_decoder_t`` for ``dtype`` in {fp32, bf16, fp16}; the
    16-bit weights in ``layout`` ("split": csrc/decoder_fs.hip, the only one since ABI 7)."""
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
    elif dtype in ("bf16", "fp16") and layout == "split":
        dt = torch.bfloat16 if dtype == "bf16" else torch.float16
        blob, nst = pack_split(pieces, dt)
        out["weights"] = blob.contiguous()
        out["w_last"] = permute_w_last_split(pieces["w_last"]).contiguous()
        out["n_stages"] = nst
    elif dtype in ("bf16", "fp16"):
        raise ValueError(f"unknown decoder layout {layout!r} (pass8 / quarter were removed in "
                         "ABI 5, split16 in ABI 7; use 'split')")
    else:
        raise ValueError(f"unknown decoder dtype {dtype!r}")
    return out
