"""CPU oracle for C19, DeepSDF auto-decoder training.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  It is the checker, never the product: ``ldm_sdf.autodecoder`` runs the
training step through ``libldm_sdf.so`` and raises if that library is missing.

PARITY STATUS: unpinned by the reference, like the rest of ``oracle/``.  ``/root/reference``
is a one-line README.  This module restates the published DeepSDF
training objective (Park et al., CVPR 2019, Eq. 9 and the authors' ``train_deep_sdf.py`` loop
as SURVEY.md §8(f) rank 3 / C19 describes it).  Per batch of S shapes with P SDF samples
each (N = S P):

    pred   = tanh(decoder([z_s || x]))                (decoder_forward, ref_cpu.py A3)
    loss   = sum |clamp(pred, δ) - clamp(sdf, δ)| / N  (L1 "sum" reduction / num_sdf_samples,
                                                       enforce_minmax clamps the prediction)
           + λ min(1, epoch / 100) sum_samples |z_s(sample)|_2 / N    (code_reg, per sample)

δ = ClampingDistance = 0.1, λ = CodeRegularizationLambda = 1e-4 (DeepSDF's example specs).
Deviations, stated: dropout (DeepSDF specs: p = 0.2 on every hidden layer) is not modelled,
so a step is deterministic, and the weights are the effective (weight-norm folded) ones.

Gradients are float64 torch autograd of exactly this function, pinned by finite differences
(``tests/test_autodecoder_oracle.py``).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

from .ref_cpu import DecoderParams, decoder_forward

__all__ = ["autodecoder_loss", "autodecoder_grads", "CLAMP_DIST", "CODE_REG_LAMBDA"]

CLAMP_DIST = 0.1
CODE_REG_LAMBDA = 1e-4


def autodecoder_loss(p: DecoderParams, z: torch.Tensor, xyz: torch.Tensor, sdf: torch.Tensor,
                     delta: float = CLAMP_DIST, reg_lambda: float = CODE_REG_LAMBDA,
                     epoch: int = 100) -> torch.Tensor:
    """z: [S, L] (the batch's latent codes), xyz: [S, P, 3], sdf: [S, P].  Scalar loss."""
    S, P = sdf.shape
    N = S * P
    pred = decoder_forward(p, z, xyz)                               # [S, P], tanh applied
    l1 = (pred.clamp(-delta, delta) - sdf.to(pred.dtype).clamp(-delta, delta)).abs().sum() / N
    reg = reg_lambda * min(1.0, epoch / 100.0) * (z.norm(dim=1) * P).sum() / N
    return l1 + reg


def autodecoder_grads(p: DecoderParams, z: torch.Tensor, xyz: torch.Tensor, sdf: torch.Tensor,
                      delta: float = CLAMP_DIST, reg_lambda: float = CODE_REG_LAMBDA,
                      epoch: int = 100) -> Tuple[float, Dict[str, torch.Tensor]]:
    """(loss, grads) with grads ``W{l}``, ``b{l}`` (per linear) and ``z`` ([S, L])."""
    ws = [w.detach().clone().requires_grad_(True) for w in p.weights]
    bs = [b.detach().clone().requires_grad_(True) for b in p.biases]
    zz = z.detach().clone().to(ws[0].dtype).requires_grad_(True)
    q = DecoderParams(p.latent_dim, p.hidden, p.n_hidden, p.skip, p.widen_skip, ws, bs)
    loss = autodecoder_loss(q, zz, xyz.to(ws[0].dtype), sdf, delta, reg_lambda, epoch)
    loss.backward()
    g = {f"W{l}": w.grad for l, w in enumerate(ws)}
    g.update({f"b{l}": b.grad for l, b in enumerate(bs)})
    g["z"] = zz.grad
    return float(loss.detach()), g
