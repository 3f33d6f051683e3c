"""Thin wrappers: one Python function per ``libldm_sdf.so`` entry point (include/ldm_sdf.h).

Every wrapper checks devices/shapes/contiguity on the host, launches on torch's current
stream and raises ``LdmError`` on a non-zero status.  No compute happens here.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Tuple

import torch

from . import _capi as capi


def _contig(*ts: torch.Tensor) -> None:
    for t in ts:
        if t is not None and not t.is_contiguous():
            raise capi.LdmError("tensors passed to libldm_sdf must be contiguous")


def _f32(*ts: torch.Tensor) -> None:
    for t in ts:
        if t is not None and t.dtype != torch.float32:
            raise capi.LdmError(f"expected float32, got {t.dtype}")


# ---------------------------------------------------------------------------------------- A1
def grid_coords(N: int, k0: int = 0, k1: Optional[int] = None, bbox=(-1.0, 1.0),
                device=None) -> torch.Tensor:
    """Device grid coordinates ``[(k1-k0)*N*N, 3]`` (z slowest, x fastest)."""
    k1 = N if k1 is None else k1
    device = device or torch.device("cuda", torch.cuda.current_device())
    out = torch.empty((k1 - k0) * N * N, 3, device=device, dtype=torch.float32)
    vs, origin = voxel_size(N, bbox), float(bbox[0])
    capi.check(capi.load().ldm_grid_coords(N, k0, k1, vs, origin, out.data_ptr(),
                                           capi.stream_handle(device)), "ldm_grid_coords")
    return out


def voxel_size(N: int, bbox=(-1.0, 1.0)) -> float:
    """fl32((hi - lo)/(N - 1)), computed on the host (A1; never divided on the device)."""
    import numpy as np
    return float(np.float32((bbox[1] - bbox[0]) / (N - 1))) if N > 1 else 0.0


# ---------------------------------------------------------------------------------------- A2
def decoder_fold(desc: capi.Decoder, z: torch.Tensor) -> torch.Tensor:
    capi.require_device(z)
    _f32(z)
    _contig(z)
    B = z.shape[0]
    beta = torch.empty(B, 2, desc.hidden, device=z.device, dtype=torch.float32)
    capi.check(capi.load().ldm_decoder_fold(C.byref(desc), z.data_ptr(), B, beta.data_ptr(),
                                            capi.stream_handle(z.device)), "ldm_decoder_fold")
    return beta


def latent_rms_max(z: torch.Tensor) -> float:
    """max over shapes of the latent RMS (``ldm_latent_rms_max``; one read-back)."""
    capi.require_device(z)
    z = z.float().contiguous()
    zz = z.reshape(z.shape[0] if z.dim() > 1 else 1, -1)
    out = torch.empty(1, device=z.device, dtype=torch.float32)
    capi.check(capi.load().ldm_latent_rms_max(zz.data_ptr(), zz.shape[0], zz.shape[1],
                                              out.data_ptr(), capi.stream_handle(z.device)),
               "ldm_latent_rms_max")
    return float(out.item())


# ---------------------------------------------------------------------------------------- A3
def decoder_grid_fwd(desc: capi.Decoder, beta: torch.Tensor, N: int, k0: int, k1: int,
                     bbox=(-1.0, 1.0), out: Optional[torch.Tensor] = None,
                     ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    capi.require_device(beta)
    _contig(beta)
    B = beta.shape[0]
    npts = (k1 - k0) * N * N
    if out is None:
        out = torch.empty(B, k1 - k0, N, N, device=beta.device, dtype=torch.float32)
    if out.numel() != B * npts or not out.is_contiguous():
        raise capi.LdmError("decoder_grid_fwd: out must be a contiguous [B, k1-k0, N, N]")
    lib = capi.load()
    wsb = lib.ldm_workspace_bytes_layout(capi.LDM_OP_DECODER_GRID, B, N, desc.dtype, desc.layout)
    if ws is None or ws.numel() < wsb:
        ws = torch.empty(max(wsb, 16), device=beta.device, dtype=torch.uint8)
    capi.check(lib.ldm_decoder_grid_fwd(C.byref(desc), beta.data_ptr(), B, N, k0, k1,
                                        voxel_size(N, bbox), float(bbox[0]), out.data_ptr(),
                                        ws.data_ptr(), ws.numel(),
                                        capi.stream_handle(beta.device)), "ldm_decoder_grid_fwd")
    return out


def decoder_points_fwd(desc: capi.Decoder, beta: torch.Tensor, xyz: torch.Tensor,
                       out: Optional[torch.Tensor] = None,
                       ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    capi.require_device(beta, xyz)
    _f32(xyz)
    _contig(beta, xyz)
    B, P = xyz.shape[0], xyz.shape[1]
    if xyz.shape != (B, P, 3) or beta.shape[0] != B:
        raise capi.LdmError("decoder_points_fwd: xyz must be [B, P, 3] matching beta [B, 2, H]")
    if out is None:
        out = torch.empty(B, P, device=xyz.device, dtype=torch.float32)
    lib = capi.load()
    wsb = lib.ldm_workspace_bytes_layout(capi.LDM_OP_DECODER_POINTS, B, P, desc.dtype,
                                         desc.layout)
    if ws is None or ws.numel() < wsb:
        ws = torch.empty(max(wsb, 16), device=xyz.device, dtype=torch.uint8)
    capi.check(lib.ldm_decoder_points_fwd(C.byref(desc), beta.data_ptr(), xyz.data_ptr(), B, P,
                                          out.data_ptr(), ws.data_ptr(), ws.numel(),
                                          capi.stream_handle(xyz.device)),
               "ldm_decoder_points_fwd")
    return out


# ---------------------------------------------------------------------------------------- A8/A9
def ddpm_step(sched_desc: capi.Sched, x: torch.Tensor, eps: torch.Tensor,
              z: Optional[torch.Tensor], t: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    capi.require_device(x, eps)
    _contig(x, eps, z)
    out = torch.empty_like(x) if out is None else out
    capi.check(capi.load().ldm_ddpm_step(C.byref(sched_desc), x.data_ptr(), eps.data_ptr(),
                                         capi.ptr(z), int(t), x.numel(), out.data_ptr(),
                                         capi.stream_handle(x.device)), "ldm_ddpm_step")
    return out


def q_sample(sched_desc: capi.Sched, x0: torch.Tensor, eps: torch.Tensor,
             t: torch.Tensor) -> torch.Tensor:
    capi.require_device(x0, eps, t)
    _contig(x0, eps, t)
    if t.dtype != torch.int32:
        raise capi.LdmError("t must be int32")
    B, D = x0.shape
    out = torch.empty_like(x0)
    capi.check(capi.load().ldm_q_sample(C.byref(sched_desc), x0.data_ptr(), eps.data_ptr(),
                                        t.data_ptr(), B, D, out.data_ptr(),
                                        capi.stream_handle(x0.device)), "ldm_q_sample")
    return out


def eps_mse_loss(eps_hat: torch.Tensor, eps: torch.Tensor,
                 with_grad: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    capi.require_device(eps_hat, eps)
    _contig(eps_hat, eps)
    loss = torch.empty(1, device=eps.device, dtype=torch.float32)
    grad = torch.empty_like(eps_hat) if with_grad else None
    capi.check(capi.load().ldm_eps_mse_loss(eps_hat.data_ptr(), eps.data_ptr(), eps.numel(),
                                            loss.data_ptr(), capi.ptr(grad),
                                            capi.stream_handle(eps.device)), "ldm_eps_mse_loss")
    return loss, grad


# ---------------------------------------------------------------------------------------- A6
def denoiser_fwd_uniform_t(desc: capi.Denoiser, x: torch.Tensor, t: int,
                           ws: Optional[torch.Tensor] = None) -> torch.Tensor:
    capi.require_device(x)
    _contig(x)
    B = x.shape[0]
    if ws is None:
        ws = torch.empty(2 * B * desc.H, device=x.device, dtype=torch.float32)
    eps = torch.empty(B, desc.D, device=x.device, dtype=torch.float32)
    capi.check(capi.load().ldm_denoiser_fwd_uniform_t(C.byref(desc), x.data_ptr(), int(t), B,
                                                      eps.data_ptr(), ws.data_ptr(),
                                                      capi.stream_handle(x.device)),
               "ldm_denoiser_fwd_uniform_t")
    return eps


def sample_step(desc: capi.Denoiser, sched_desc: capi.Sched, x: torch.Tensor,
                z: Optional[torch.Tensor], t: int, out: torch.Tensor, ws: torch.Tensor) -> None:
    capi.check(capi.load().ldm_sample_step(C.byref(desc), C.byref(sched_desc), x.data_ptr(),
                                           capi.ptr(z), int(t), x.shape[0], out.data_ptr(),
                                           ws.data_ptr(), capi.stream_handle(x.device)),
               "ldm_sample_step")


def adamw_step(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
               p_low: Optional[torch.Tensor], *, lr: float, betas=(0.9, 0.999), eps: float = 1e-8,
               weight_decay: float = 0.0, step: int) -> None:
    """Fused AdamW (``ldm_adamw_step``) on contiguous fp32 tensors; ``p_low`` (bf16, same shape)
    receives the updated weights rounded to nearest even, or None."""
    for t in (p, g, m, v):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.shape != p.shape:
            raise capi.LdmError("adamw_step: p, g, m, v must be contiguous fp32 of one shape")
    if p_low is not None and (p_low.dtype != torch.bfloat16 or not p_low.is_contiguous()
                              or p_low.shape != p.shape):
        raise capi.LdmError("adamw_step: p_low must be contiguous bf16 of p's shape")
    capi.check(capi.load().ldm_adamw_step(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
                                          capi.ptr(p_low), p.numel(), float(lr), float(betas[0]),
                                          float(betas[1]), float(eps), float(weight_decay),
                                          int(step), capi.stream_handle(p.device)),
               "ldm_adamw_step")


def sample_loop_supported(desc: capi.Denoiser, B: int) -> bool:
    return bool(capi.load().ldm_sample_loop_supported(C.byref(desc), int(B)))


def sample_loop_workspace(desc: capi.Denoiser, B: int, device) -> torch.Tensor:
    nbytes = int(capi.load().ldm_sample_loop_ws_bytes(int(B), desc.H))
    return torch.empty((nbytes + 3) // 4, device=device, dtype=torch.float32)


def sample_loop(desc: capi.Denoiser, sched_desc: capi.Sched, x2: torch.Tensor,
                noise: torch.Tensor, t_hi: int, steps: int, ws: torch.Tensor) -> None:
    """A10 in one persistent launch (``ldm_sample_loop``): ``x2 [2, B, D]`` holds x_T in
    ``x2[0]`` and the result in ``x2[steps & 1]``; ``noise [T, B, D]``."""
    B = x2.shape[1]
    capi.check(capi.load().ldm_sample_loop(C.byref(desc), C.byref(sched_desc), x2.data_ptr(),
                                           noise.data_ptr(), int(t_hi), int(steps), B,
                                           ws.data_ptr(), ws.numel() * 4,
                                           capi.stream_handle(x2.device)),
               "ldm_sample_loop")


def sample_loop_status(desc: capi.Denoiser, ws: torch.Tensor, B: int) -> int:
    """0 when the last ``sample_loop`` on ``ws`` completed, 1 when a barrier timed out.
    Synchronises the stream."""
    st = C.c_uint(0)
    capi.check(capi.load().ldm_sample_loop_status(ws.data_ptr(), int(B), desc.H, C.byref(st),
                                                  capi.stream_handle(ws.device)),
               "ldm_sample_loop_status")
    return int(st.value)


LOOP_FORMS = {"auto": 0, "replica": 1, "xcd": 2, "direct": 3, "flat": 4}
LOOP_FORM_NAMES = {v: k for k, v in LOOP_FORMS.items()}


def sample_loop_config(form: str = "auto", spin_limit: int = 0, tagged: bool = True) -> None:
    """Explicit A/B / fault-injection control of the persistent sampling loop on the current
    device (``ldm_sample_loop_config``): the library reads no environment variable."""
    capi.check(capi.load().ldm_sample_loop_config(LOOP_FORMS[form], int(spin_limit),
                                                  1 if tagged else 0),
               "ldm_sample_loop_config")


def sample_loop_last_form() -> str:
    """Which loop kernel the last ``sample_loop`` on the current device ran ("replica", "xcd",
    "direct", "flat"; "auto" before any launch)."""
    return LOOP_FORM_NAMES[int(capi.load().ldm_sample_loop_last_form())]


# ---------------------------------------------------------------------------------------- GEMM
def linear(X: torch.Tensor, W: torch.Tensor, Y: torch.Tensor, *, epi: int = capi.EPI_BIAS,
           bias: Optional[torch.Tensor] = None, X2: Optional[torch.Tensor] = None,
           W2: Optional[torch.Tensor] = None, R: Optional[torch.Tensor] = None,
           A_out: Optional[torch.Tensor] = None, compute: int = capi.COMPUTE_FP32) -> torch.Tensor:
    """``Y = epi(X @ W.T [+ X2 @ W2.T] + bias)`` on strided 2-D views (any strides).
    ``compute``: COMPUTE_FP32 (exact fp32, VALU) or COMPUTE_BF16 (matrix cores, operands
    rounded to bf16, fp32 accumulate).

    X: [Bn, K] view, W: [M, K] view (fp32 or bf16), Y: [Bn, M] view.  Transposed views give
    the backward products, e.g. ``linear(G.T, X.T, dW)`` = ``G^T X``.
    """
    Bn, K = X.shape
    M = W.shape[0]
    if W.shape[1] != K or Y.shape != (Bn, M):
        raise capi.LdmError(f"linear: shapes X{tuple(X.shape)} W{tuple(W.shape)} Y{tuple(Y.shape)}")
    a = capi.LinearArgs()
    a.Bn, a.M, a.K = Bn, M, K
    a.epi = epi
    a.compute = compute
    if W.dtype == torch.bfloat16:
        a.w_dtype = capi.LDM_BF16
    elif W.dtype == torch.float32:
        a.w_dtype = capi.LDM_F32
    else:
        raise capi.LdmError(f"linear: W dtype {W.dtype}")
    _f32(X, Y, bias, R, A_out, X2)
    a.X, a.sxb, a.sxk = X.data_ptr(), X.stride(0), X.stride(1)
    a.W, a.swm, a.swk = W.data_ptr(), W.stride(0), W.stride(1)
    if X2 is not None:
        if W2 is None or W2.dtype != W.dtype or X2.shape[0] != Bn or W2.shape != (M, X2.shape[1]):
            raise capi.LdmError("linear: bad second segment")
        if (X2.stride(1) == 1) != (X.stride(1) == 1) or (W2.stride(1) == 1) != (W.stride(1) == 1):
            raise capi.LdmError("linear: both segments must share contiguity")
        a.K2 = X2.shape[1]
        a.X2, a.sx2b, a.sx2k = X2.data_ptr(), X2.stride(0), X2.stride(1)
        a.W2, a.sw2m, a.sw2k = W2.data_ptr(), W2.stride(0), W2.stride(1)
    if bias is not None:
        a.bias = bias.data_ptr()
    if R is not None:
        if R.stride(1) != 1:
            raise capi.LdmError("linear: R rows must be contiguous")
        a.R, a.srb = R.data_ptr(), R.stride(0)
    a.Y, a.syb, a.sym = Y.data_ptr(), Y.stride(0), Y.stride(1)
    if A_out is not None:
        if A_out.stride(1) != 1:
            raise capi.LdmError("linear: A_out rows must be contiguous")
        a.A_out, a.sab = A_out.data_ptr(), A_out.stride(0)
    lib = capi.load()
    ws = None
    if compute == capi.COMPUTE_BF16:
        n = lib.ldm_linear_workspace_floats(C.byref(a))
        if n > 0:     # split-K partials; freed to the stream-ordered cache after the launch
            ws = torch.empty(n, device=Y.device, dtype=torch.float32)
            a.ws, a.ws_floats = ws.data_ptr(), n
    capi.check(lib.ldm_linear(C.byref(a), capi.stream_handle(Y.device)), "ldm_linear")
    return Y


def silu_bwd(dy: torch.Tensor, a: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _contig(dy, a)
    out = torch.empty_like(dy) if out is None else out
    capi.check(capi.load().ldm_silu_bwd(dy.data_ptr(), a.data_ptr(), dy.numel(), out.data_ptr(),
                                        capi.stream_handle(dy.device)), "ldm_silu_bwd")
    return out


def colsum(G: torch.Tensor, out: torch.Tensor, accumulate: bool = False) -> torch.Tensor:
    """``out (+)= G.sum(0)``, deterministic.  Tall G goes in two passes -- per-segment sums
    over up to 256 row segments in parallel, then their sum -- because the one-pass kernel has
    only ceil(M/64) workgroups: >= 64k rows (C19's 1M samples), and since round 6 >= 16k rows
    when that is under 64 workgroups (C19's per-32-row bias partials, 32k x 512: 8 workgroups,
    0.27 ms a call, 5 % of the auto-decoder step).  Config 2's partials (ceil(B/32) rows) stay
    one-pass, so the one-launch training step still sums them in this order."""
    _contig(G)
    Bn, M = G.shape
    if Bn >= 65536 or (Bn >= 16384 and (M + 63) // 64 < 64):
        segs = next((s for s in (256, 128, 64, 32, 16) if Bn % s == 0), 0)
        if segs:
            part = torch.empty(segs, M, device=G.device, dtype=torch.float32)
            colsum_segments(G, segs, part)
            G, Bn = part, segs
    capi.check(capi.load().ldm_colsum(G.data_ptr(), Bn, M, out.data_ptr(), int(accumulate),
                                      capi.stream_handle(G.device)), "ldm_colsum")
    return out


def gather_rows(table: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    _contig(table, idx)
    Bn, Cc = idx.shape[0], table.shape[1]
    out = torch.empty(Bn, Cc, device=table.device, dtype=torch.float32)
    capi.check(capi.load().ldm_gather_rows(table.data_ptr(), idx.data_ptr(), Bn, Cc,
                                           out.data_ptr(), capi.stream_handle(table.device)),
               "ldm_gather_rows")
    return out


# ---------------------------------------------------------------------------------------- C19
def relu_bwd(dy: torch.Tensor, y: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``dy * (y > 0)`` on the post-activation ``y``."""
    _contig(dy, y)
    out = torch.empty_like(dy) if out is None else out
    capi.check(capi.load().ldm_relu_bwd(dy.data_ptr(), y.data_ptr(), dy.numel(), out.data_ptr(),
                                        capi.stream_handle(dy.device)), "ldm_relu_bwd")
    return out


def sdf_l1_loss(pre: torch.Tensor, gt: torch.Tensor, delta: float, scale: float,
                with_grad: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """DeepSDF clamped L1 on ``tanh(pre)`` (see ``ldm_sdf_l1_loss``): (loss [1], d/d pre)."""
    capi.require_device(pre, gt)
    _contig(pre, gt)
    if pre.numel() != gt.numel():
        raise capi.LdmError(f"sdf_l1_loss: {pre.numel()} predictions vs {gt.numel()} targets")
    loss = torch.empty(1, device=pre.device, dtype=torch.float32)
    grad = torch.empty_like(pre) if with_grad else None
    capi.check(capi.load().ldm_sdf_l1_loss(pre.data_ptr(), gt.data_ptr(), pre.numel(), delta,
                                           scale, loss.data_ptr(), capi.ptr(grad),
                                           capi.stream_handle(pre.device)), "ldm_sdf_l1_loss")
    return loss, grad


def colsum_segments(G: torch.Tensor, S: int, out: torch.Tensor,
                    accumulate: bool = False) -> torch.Tensor:
    """``out[s] (+)= G[s*P:(s+1)*P].sum(0)`` for ``G`` [S*P, M] (rows grouped by segment)."""
    _contig(G, out)
    N, M = G.shape
    if N % S or tuple(out.shape) != (S, M):
        raise capi.LdmError(f"colsum_segments: G{tuple(G.shape)} S={S} out{tuple(out.shape)}")
    capi.check(capi.load().ldm_colsum_segments(G.data_ptr(), S, N // S, M, out.data_ptr(),
                                               int(accumulate), capi.stream_handle(G.device)),
               "ldm_colsum_segments")
    return out


def latent_l2_reg(z: torch.Tensor, coef: float, loss_io: torch.Tensor,
                  grad_io: Optional[torch.Tensor]) -> None:
    """``loss_io += coef * sum_s |z_s|``, ``grad_io += coef * z_s / |z_s|`` (DeepSDF code_reg)."""
    _contig(z, loss_io)
    S, L = z.shape
    capi.check(capi.load().ldm_latent_l2_reg(z.data_ptr(), S, L, coef, loss_io.data_ptr(),
                                             capi.ptr(grad_io), capi.stream_handle(z.device)),
               "ldm_latent_l2_reg")


# ---------------------------------------------------------------------------------------- GEMM
_GEMM_MODES = {"store": capi.GEMM_STORE, "silu": capi.GEMM_SILU,
               "resid_silu": capi.GEMM_RESID_SILU, "relu": capi.GEMM_RELU,
               "accum": capi.GEMM_ACCUM, "dgrad_silu": capi.GEMM_DGRAD_SILU,
               "loss": capi.GEMM_LOSS, "add_r": capi.GEMM_ADD_R,
               "relu_bwd": capi.GEMM_RELU_BWD}


def _rowmajor(t: Optional[torch.Tensor], what: str, dtype=None) -> int:
    """Row stride of a 2-D view whose rows are contiguous (0 for None)."""
    if t is None:
        return 0
    if t.dim() != 2 or t.stride(1) != 1:
        raise capi.LdmError(f"gemm: {what} must be a 2-D view with contiguous rows")
    if dtype is not None and t.dtype != dtype:
        raise capi.LdmError(f"gemm: {what} must be {dtype}, got {t.dtype}")
    return t.stride(0)


def gemm_problem(segs, M: int, N: int, *, mode: str = "store", M_valid: Optional[int] = None,
                 bias=None, R=None, P_in=None, C=None, P=None, Cb=None, CbT=None, colsum=None,
                 loss_part=None, scale: float = 1.0, Rb=None, k_split: int = 1,
                 ws=None, ct_blk: int = 0, slices=None) -> capi.GemmProb:
    """One problem of ``ldm_gemm_bf16`` (include/ldm_sdf.h): ``segs`` = [(A [M,K] bf16,
    B [N,K] bf16), ...] as row-contiguous views; outputs / operands as documented there.
    ``Rb``: bf16 [M,N] post-activation of mode "relu_bwd"; ``k_split`` > 1 with ``ws``
    (fp32, >= k_split * M * N elements): split-K into that workspace.  ``ct_blk`` > 0: CbT
    is written blocked, [ceil(M/ct_blk), N, ct_blk].  ``slices`` = (slice_a, slice_b): split-K
    over blocked operands -- ``segs`` holds ONE block of each ([M, kb] / [N, kb] views) and
    slice s reads the block s * slice_a (s * slice_b) elements further; K = k_split * kb."""
    pr = capi.GemmProb()
    pr.M, pr.N = int(M), int(N)
    pr.M_valid = int(M if M_valid is None else M_valid)
    if not 1 <= len(segs) <= capi.GEMM_MAX_SEGS:
        raise capi.LdmError(f"gemm: 1..{capi.GEMM_MAX_SEGS} segments")
    pr.n_seg = len(segs)
    for i, (A, B) in enumerate(segs):
        la = _rowmajor(A, "A", torch.bfloat16)
        lb = _rowmajor(B, "B", torch.bfloat16)
        if A.shape[0] < M or B.shape[0] < N or A.shape[1] != B.shape[1]:
            raise capi.LdmError(f"gemm seg {i}: A{tuple(A.shape)} B{tuple(B.shape)} vs M={M} N={N}")
        g = pr.seg[i]
        g.A, g.B, g.lda, g.ldb = A.data_ptr(), B.data_ptr(), la, lb
        g.K = A.shape[1] * (k_split if slices else 1)
    pr.mode = _GEMM_MODES[mode]
    pr.scale = float(scale)
    for name, t, dt in (("R", R, torch.float32), ("P_in", P_in, torch.float32),
                        ("C", C, torch.float32), ("P", P, torch.float32),
                        ("Cb", Cb, torch.bfloat16), ("CbT", CbT, torch.bfloat16)):
        if name == "CbT" and ct_blk and t is not None:   # blocked [nblk, N, ct_blk]
            if (t.dtype != torch.bfloat16 or not t.is_contiguous()
                    or t.numel() < -(-M // ct_blk) * N * ct_blk):
                raise capi.LdmError("gemm: blocked CbT must be contiguous bf16 "
                                    "[ceil(M/ct_blk), N, ct_blk]")
            pr.CbT, pr.ldct = t.data_ptr(), 0
            continue
        ld = _rowmajor(t, name, dt)
        setattr(pr, name, capi.ptr(t))
        if t is not None:
            setattr(pr, {"R": "ldr", "P_in": "ldp_in", "C": "ldc", "P": "ldp", "Cb": "ldcb",
                         "CbT": "ldct"}[name], ld)
    if Rb is not None:
        pr.ldrb = _rowmajor(Rb, "Rb", torch.bfloat16)
        pr.Rb = Rb.data_ptr()
    pr.k_split = int(k_split)
    pr.ct_blk = int(ct_blk)
    if slices:
        pr.slice_a, pr.slice_b = int(slices[0]), int(slices[1])
    if k_split > 1:
        if ws is None or ws.dtype != torch.float32 or ws.numel() < k_split * M * N:
            raise capi.LdmError(f"gemm: split-K {k_split} needs an fp32 ws of "
                                f"{k_split * M * N} elements")
    for name, t in (("bias", bias), ("colsum", colsum), ("loss_part", loss_part), ("ws", ws)):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise capi.LdmError(f"gemm: {name} must be contiguous fp32")
        setattr(pr, name, capi.ptr(t))
    return pr


def gemm_args(problems, tile: int = 0) -> capi.GemmArgs:
    a = capi.GemmArgs()
    if not 1 <= len(problems) <= capi.GEMM_MAX_PROBS:
        raise capi.LdmError("gemm: 1..4 problems per launch")
    a.n_prob, a.tile = len(problems), int(tile)
    for i, pr in enumerate(problems):
        a.prob[i] = pr
    return a


def gemm_launch(a: capi.GemmArgs, device) -> None:
    capi.check(capi.load().ldm_gemm_bf16(C.byref(a), capi.stream_handle(device)), "ldm_gemm_bf16")


def gemm(problems, tile: int = 0, device=None) -> None:
    """Launch ``ldm_gemm_bf16`` on torch's current stream (problems from ``gemm_problem``)."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    gemm_launch(gemm_args(problems, tile), device)


# ---------------------------------------------------------------------------------------- C17
def _r16(n: int) -> int:
    return (n + 15) // 16 * 16


def perm16_index(C: int) -> torch.Tensor:
    """``perm16``: position of channel ci inside its group of 16 (include/ldm_sdf.h)."""
    ci = torch.arange(C)
    return (ci & ~15) | ((ci & 3) << 2) | ((ci >> 2) & 3)


def pack_conv_weight(W: torch.Tensor) -> torch.Tensor:
    """torch conv weight ``[Cout, Cw, K]`` -> the matrix-core packing ldm_conv1d reads:
    ``[Cout16, K, Cw16]`` (zero-padded to multiples of 16) with channel ci at perm16(ci)."""
    Cout, Cw, K = W.shape
    out = torch.zeros(_r16(Cout), K, _r16(Cw), dtype=W.dtype, device=W.device)
    out[:Cout, :, perm16_index(_r16(Cw))[:Cw].to(W.device)] = W.permute(0, 2, 1)
    return out


class ConvSegment:
    """One operand segment of ``ldm_conv1d``: input ``X [B, C, L_in]`` (fp32, contiguous),
    packed weight ``Wp [Cout16, ksize, Cw16]`` (``pack_conv_weight``; fp32/bf16; the segment
    uses input channels ``[c_off, c_off + C)``, c_off a multiple of 16), tap geometry and the
    SiLU-on-input flag."""

    __slots__ = ("X", "W", "c_off", "ksize", "stride", "pad", "mode", "silu")

    def __init__(self, X, Wp, *, c_off=0, stride=1, pad=None, mode=capi.CONV_DIRECT, silu=False):
        self.X, self.W, self.c_off = X, Wp, c_off
        self.ksize = Wp.shape[1]
        self.stride, self.mode, self.silu = stride, mode, silu
        self.pad = (self.ksize - 1) // 2 if pad is None else pad


def conv1d_args(segs, Y: torch.Tensor, *, bias=None, bias2=None, cbias=None, scb: int = 0,
                R=None, epi: int = capi.CONV_EPI_STORE, xlat=None, z=None, sched=None,
                t: int = 0) -> capi.ConvArgs:
    """Validated ``ldm_conv1d_args_t`` (kept alive by the caller for graph capture)."""
    B, Cout, L_out = Y.shape
    if not 1 <= len(segs) <= capi.CONV_MAX_SEGS:
        raise capi.LdmError("conv1d: 1..4 segments")
    _f32(Y, bias, bias2, cbias, R, xlat, z)
    _contig(Y, bias, bias2, cbias, R, xlat, z)
    a = capi.ConvArgs()
    a.B, a.Cout, a.L_out, a.n_seg, a.epi = B, Cout, L_out, len(segs), epi
    wdt = segs[0].W.dtype
    a.w_dtype = {torch.float32: capi.LDM_F32, torch.bfloat16: capi.LDM_BF16}.get(wdt, -1)
    if a.w_dtype < 0:
        raise capi.LdmError(f"conv1d: weight dtype {wdt}")
    for i, s in enumerate(segs):
        X, W = s.X, s.W
        _f32(X)
        _contig(X, W)
        if W.dtype != wdt or W.dim() != 3 or W.shape[0] != _r16(Cout) or X.shape[0] != B \
                or W.shape[2] % 16:
            raise capi.LdmError(f"conv1d seg {i}: packed weight [{_r16(Cout)}, K, Cw16] / "
                                f"batch mismatch (got {tuple(W.shape)})")
        Cs = X.shape[1]
        if s.c_off % 16 or s.c_off + Cs > W.shape[2]:
            raise capi.LdmError(f"conv1d seg {i}: channels {s.c_off}+{Cs} vs {W.shape[2]}")
        Lsrc = 2 * X.shape[2] if s.mode == capi.CONV_UP2 else X.shape[2]
        if (Lsrc + 2 * s.pad - s.ksize) // s.stride + 1 != L_out:
            raise capi.LdmError(f"conv1d seg {i}: L_in {X.shape[2]} does not give L_out {L_out}")
        g = a.seg[i]
        g.X = X.data_ptr()
        g.W = W.data_ptr() + s.c_off * W.element_size()
        g.C, g.L_in, g.ksize, g.stride, g.pad = Cs, X.shape[2], s.ksize, s.stride, s.pad
        g.mode, g.silu_in = s.mode, int(bool(s.silu))
        g.ldw, g.kstride = s.ksize * W.shape[2], W.shape[2]
    for name, v in (("bias", bias), ("bias2", bias2), ("R", R), ("xlat", xlat), ("z", z)):
        setattr(a, name, capi.ptr(v))
    if R is not None and R.shape != Y.shape:
        raise capi.LdmError("conv1d: R must match Y")
    if cbias is not None:
        a.cbias, a.scb = cbias.data_ptr(), int(scb)
    a.Y = Y.data_ptr()
    if epi == capi.CONV_EPI_DDPM:
        if sched is None or xlat is None or xlat.shape != (B, Cout * L_out):
            raise capi.LdmError("conv1d DDPM epilogue: needs sched and xlat [B, L]")
        a.c1, a.c2, a.sigma, a.t = sched.c1, sched.c2, sched.sigma, int(t)
    return a


def conv1d_launch(a: capi.ConvArgs, device) -> None:
    capi.check(capi.load().ldm_conv1d(C.byref(a), capi.stream_handle(device)), "ldm_conv1d")


def conv1d(segs, Y: torch.Tensor, **kw) -> torch.Tensor:
    """``Y = epi(sum_seg conv(act(X_seg); W_seg) + biases (+ R))`` -- see include/ldm_sdf.h."""
    capi.require_device(Y, *[s.X for s in segs])
    conv1d_launch(conv1d_args(segs, Y, **kw), Y.device)
    return Y


# ---------------------------------------------------------------------------------------- A5
def temb_forward(dev: Dict[str, object], e: torch.Tensor, H: int,
                 save: Optional[dict] = None, compute: int = capi.COMPUTE_FP32) -> torch.Tensor:
    """temb = Wt2 SiLU(Wt1 e + bt1) + bt2 for a batch of embeddings e [Bn, TE]."""
    Bn = e.shape[0]
    u = torch.empty(Bn, H, device=e.device, dtype=torch.float32)
    a_t = torch.empty_like(u) if save is not None else None
    linear(e, dev["Wt1"], u, epi=capi.EPI_SILU, bias=dev["bt1"], A_out=a_t, compute=compute)
    temb = torch.empty(Bn, H, device=e.device, dtype=torch.float32)
    linear(u, dev["Wt2"], temb, epi=capi.EPI_BIAS, bias=dev["bt2"], compute=compute)
    if save is not None:
        save.update(e=e, u=u, a_t=a_t, temb=temb)
    return temb


def build_e_tables(model, dev: Dict[str, object], dtype: str) -> List[torch.Tensor]:
    """A5 inference tables: ``E_k[t] = U_k temb(t) + b_k`` for every t (fp32 [T, H])."""
    H, T = model.H, model.T
    emb = dev["emb_table"]
    temb = temb_forward(dev, emb, H)
    tabs = []
    for k in range(model.n_blocks):
        W = dev[f"Wblk{k}"]
        E = torch.empty(T, H, device=emb.device, dtype=torch.float32)
        linear(temb, W[:, H:], E, epi=capi.EPI_BIAS, bias=dev[f"bblk{k}"])
        tabs.append(E)
    return tabs


# ---------------------------------------------------------------------------------------- A6/A7
# bf16 training through the C ABI (csrc/denoiser_train.hip): one call per forward / backward /
# fused step; every product is an ldm_gemm_bf16 problem with fused epilogues.
def grads_struct(grads: Dict[str, torch.Tensor], n_blocks: int) -> capi.DenoiserGrads:
    """``ldm_denoiser_grads_t`` over fp32 tensors named like MLPDenoiser.params."""
    g = capi.DenoiserGrads()
    for fld, name in (("w_in", "Win"), ("b_in", "bin"), ("w_t1", "Wt1"), ("b_t1", "bt1"),
                      ("w_t2", "Wt2"), ("b_t2", "bt2"), ("w_out", "Wout"), ("b_out", "bout")):
        t = grads[name]
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise capi.LdmError(f"{name}: fp32 contiguous tensor expected")
        setattr(g, fld, t.data_ptr())
    for k in range(n_blocks):
        g.w_blk[k] = grads[f"Wblk{k}"].data_ptr()
        g.b_blk[k] = grads[f"bblk{k}"].data_ptr()
    return g


def train_workspace(desc: capi.Denoiser, B: int, device) -> torch.Tensor:
    """The ``saved`` workspace of ldm_denoiser_fwd / _bwd / _train_step for batch B."""
    n = int(capi.load().ldm_denoiser_train_ws_bytes(C.byref(desc), int(B)))
    if n == 0:
        raise capi.LdmError("ldm_denoiser_train_ws_bytes: unsupported denoiser shape")
    ws = torch.empty(n + 256, device=device, dtype=torch.uint8)
    off = (-ws.data_ptr()) % 256
    ws = ws[off:off + n]
    # a fresh allocation may lie where a freed workspace did: zero its sync words and drop the
    # host's record of a job table uploaded there (ldm_denoiser_train_ws_init)
    capi.check(capi.load().ldm_denoiser_train_ws_init(C.byref(desc), int(B), ws.data_ptr(),
                                                      capi.stream_handle(ws.device)),
               "ldm_denoiser_train_ws_init")
    return ws


def denoiser_train_step(desc: capi.Denoiser, sched_desc: capi.Sched, x0: torch.Tensor,
                        eps: torch.Tensor, t: torch.Tensor, ws: torch.Tensor,
                        gstruct: capi.DenoiserGrads, loss: torch.Tensor) -> None:
    """q_sample -> net -> eps-MSE -> every gradient (``ldm_denoiser_train_step``)."""
    _f32(x0, eps, loss)
    _contig(x0, eps, t)
    if t.dtype != torch.int32:
        raise capi.LdmError("t must be int32")
    capi.check(capi.load().ldm_denoiser_train_step(C.byref(desc), C.byref(sched_desc),
                                                   x0.data_ptr(), eps.data_ptr(), t.data_ptr(),
                                                   x0.shape[0], ws.data_ptr(), C.byref(gstruct),
                                                   loss.data_ptr(),
                                                   capi.stream_handle(x0.device)),
               "ldm_denoiser_train_step")


_side_streams: Dict[int, "torch.cuda.Stream"] = {}


def side_stream(device: torch.device) -> "torch.cuda.Stream":
    """The second stream ``denoiser_train_step_adamw`` forks the early AdamW updates onto."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _side_streams:
        _side_streams[idx] = torch.cuda.Stream(device=torch.device("cuda", idx))
    return _side_streams[idx]


def denoiser_train_step_adamw(desc: capi.Denoiser, sched_desc: capi.Sched, x0: torch.Tensor,
                              eps: torch.Tensor, t: torch.Tensor, ws: torch.Tensor,
                              gstruct: capi.DenoiserGrads, loss: torch.Tensor, table, *,
                              lr: float, betas=(0.9, 0.999), adam_eps: float = 1e-8,
                              weight_decay: float = 0.0, step: int, overlap: bool = False,
                              hyper: Optional[torch.Tensor] = None) -> None:
    """One single-rank step: ``denoiser_train_step`` + ``adamw_multi`` over ``table`` in one
    call (``ldm_denoiser_train_step_adamw``); ``overlap`` forks the updates onto a side stream
    as their gradients become final.  ``hyper``: device fp32 [7] AdamW scalars
    (``adamw_hyper``) read by the kernels instead of lr / step (graph replays).  Same bits as
    the two calls in sequence."""
    _f32(x0, eps, loss)
    _contig(x0, eps, t)
    if t.dtype != torch.int32:
        raise capi.LdmError("t must be int32")
    side = side_stream(x0.device).cuda_stream if overlap else None
    capi.check(capi.load().ldm_denoiser_train_step_adamw(
        C.byref(desc), C.byref(sched_desc), x0.data_ptr(), eps.data_ptr(), t.data_ptr(),
        x0.shape[0], ws.data_ptr(), C.byref(gstruct), loss.data_ptr(), table, len(table),
        float(lr), float(betas[0]), float(betas[1]), float(adam_eps), float(weight_decay),
        int(step), capi.ptr(hyper), capi.stream_handle(x0.device), side),
        "ldm_denoiser_train_step_adamw")


TRAIN_FORMS = {"auto": 0, "launches": 1, "dag": 2}


def train_step_config(form: str = "auto", spin_limit: int = 0) -> None:
    """Form of ``denoiser_train_step_adamw`` on the current device (``ldm_train_step_config``):
    "auto" (the form measured faster for the configuration: denoiser_train.hip ``dag_auto``),
    "launches" (one launch per GEMM group + AdamW), "dag" (the one-launch step, required).  Same
    bits either way.  ``spin_limit``: MICROSECONDS (s_memrealtime time) one DAG dependency wait
    may take before the launch gives up (0 = the default, 2 s; 1 us makes waits give up at once
    and exercises the timeout path)."""
    capi.check(capi.load().ldm_train_step_config(TRAIN_FORMS[form], int(spin_limit)),
               "ldm_train_step_config")


def train_step_last_form() -> str:
    """The form the last ``denoiser_train_step_adamw`` on this device ran ("" before any)."""
    f = capi.load().ldm_train_step_last_form()
    return {0: "", 1: "launches", 2: "dag"}.get(f, str(f))


def train_status(desc: capi.Denoiser, B: int, ws: torch.Tensor) -> int:
    """The DAG step's status word in ``ws`` (read and cleared; one stream synchronisation):
    0 ok, 1 a wait timed out (that step's results are garbage), 3 stale job table."""
    st = C.c_uint(0)
    capi.check(capi.load().ldm_denoiser_train_status(C.byref(desc), B, ws.data_ptr(),
                                                     C.byref(st), capi.stream_handle(ws.device)),
               "ldm_denoiser_train_status")
    return int(st.value)


def adamw_hyper(*, lr: float, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                step: int) -> List[float]:
    """The 7 AdamW scalars of one step exactly as the library derives them
    (``ldm_adamw_hyper``), for a device ``hyper`` buffer."""
    out = (C.c_float * 7)()
    capi.load().ldm_adamw_hyper(float(lr), float(betas[0]), float(betas[1]), float(eps),
                                float(weight_decay), int(step), C.addressof(out))
    return list(out)


def denoiser_fwd(desc: capi.Denoiser, x: torch.Tensor, t: torch.Tensor, ws: torch.Tensor,
                 eps_out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Training forward with per-sample t (``ldm_denoiser_fwd``), activations saved in ws."""
    _f32(x, eps_out)
    _contig(x, t, eps_out)
    if t.dtype != torch.int32:
        raise capi.LdmError("t must be int32")
    capi.check(capi.load().ldm_denoiser_fwd(C.byref(desc), x.data_ptr(), t.data_ptr(),
                                            x.shape[0], capi.ptr(eps_out), ws.data_ptr(),
                                            capi.stream_handle(x.device)), "ldm_denoiser_fwd")
    return eps_out


def denoiser_bwd(desc: capi.Denoiser, ws: torch.Tensor, deps: torch.Tensor,
                 gstruct: capi.DenoiserGrads, dx: Optional[torch.Tensor] = None) -> None:
    """Backward of the last ``denoiser_fwd`` on ws (``ldm_denoiser_bwd``)."""
    _f32(deps, dx)
    _contig(deps, dx)
    capi.check(capi.load().ldm_denoiser_bwd(C.byref(desc), ws.data_ptr(), deps.data_ptr(),
                                            deps.shape[0], C.byref(gstruct), capi.ptr(dx),
                                            capi.stream_handle(deps.device)), "ldm_denoiser_bwd")


def q_sample_loss(sched_desc: capi.Sched, eps: torch.Tensor, *, x0=None, t=None, xt_out=None,
                  eps_hat=None, loss_out=None, grad_out=None) -> None:
    """A9 head (``ldm_q_sample_loss``): x_t and/or the eps-MSE loss and its gradient."""
    _f32(eps, x0, xt_out, eps_hat, loss_out, grad_out)
    _contig(eps, x0, t, xt_out, eps_hat, grad_out)
    B, D = eps.shape
    capi.check(capi.load().ldm_q_sample_loss(C.byref(sched_desc), capi.ptr(x0), eps.data_ptr(),
                                             capi.ptr(t), B, D, capi.ptr(xt_out),
                                             capi.ptr(eps_hat), capi.ptr(loss_out),
                                             capi.ptr(grad_out),
                                             capi.stream_handle(eps.device)), "ldm_q_sample_loss")


def adamw_table(entries) -> "C.Array":
    """Host ``ldm_adamw_tensor_t`` array for ``adamw_multi``: entries are tuples
    (p, g, m, v, p_bf16 or None, p_bf16_t or None) of tensors with 1-D or 2-D shapes."""
    arr = (capi.AdamwTensor * len(entries))()
    for i, (p, g, m, v, pb, pbt) in enumerate(entries):
        for t in (p, g, m, v):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.shape != p.shape:
                raise capi.LdmError("adamw_multi: p, g, m, v must be contiguous fp32 of one shape")
        rows, cols = (p.shape[0], p.shape[1]) if p.dim() == 2 else (1, p.numel())
        for t, shp in ((pb, (rows, cols)), (pbt, (cols, rows))):
            if t is not None and (t.dtype != torch.bfloat16 or not t.is_contiguous()
                                  or t.numel() != rows * cols):
                raise capi.LdmError("adamw_multi: bf16 copies must be contiguous, p's size")
        e = arr[i]
        e.p, e.g, e.m, e.v = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
        e.p_bf16, e.p_bf16_t = capi.ptr(pb), capi.ptr(pbt)
        e.rows, e.cols = rows, cols
    return arr


def adamw_multi(table, *, lr: float, betas=(0.9, 0.999), eps: float = 1e-8,
                weight_decay: float = 0.0, step: int, device=None) -> None:
    """Every tensor of ``table`` (``adamw_table``) in one launch (``ldm_adamw_multi``)."""
    capi.check(capi.load().ldm_adamw_multi(table, len(table), float(lr), float(betas[0]),
                                           float(betas[1]), float(eps), float(weight_decay),
                                           int(step), capi.stream_handle(device)),
               "ldm_adamw_multi")


def denoiser_forward_train(model, dev: Dict[str, object], xt: torch.Tensor,
                           t: torch.Tensor, compute: int = capi.COMPUTE_FP32
                           ) -> Tuple[torch.Tensor, dict]:
    """Training forward (per-sample t) saving what the backward needs."""
    H, nb = model.H, model.n_blocks
    Bn = xt.shape[0]
    cp = compute
    sv: dict = {"xt": xt}
    e = gather_rows(dev["emb_table"], t)
    temb = temb_forward(dev, e, H, save=sv, compute=cp)
    h = torch.empty(Bn, H, device=xt.device, dtype=torch.float32)
    linear(xt, dev["Win"], h, epi=capi.EPI_BIAS, bias=dev["bin"], compute=cp)
    hs, pre = [h], []
    for k in range(nb):
        W = dev[f"Wblk{k}"]
        a = torch.empty(Bn, H, device=xt.device, dtype=torch.float32)
        hn = torch.empty(Bn, H, device=xt.device, dtype=torch.float32)
        linear(h, W[:, :H], hn, epi=capi.EPI_RESID_SILU, bias=dev[f"bblk{k}"], X2=temb,
               W2=W[:, H:], R=h, A_out=a, compute=cp)
        hs.append(hn)
        pre.append(a)
        h = hn
    eps_hat = torch.empty(Bn, model.D, device=xt.device, dtype=torch.float32)
    linear(h, dev["Wout"], eps_hat, epi=capi.EPI_BIAS, bias=dev["bout"], compute=cp)
    sv.update(hs=hs, pre=pre)
    return eps_hat, sv


def denoiser_backward_train(model, dev: Dict[str, object], sv: dict,
                            g_out: torch.Tensor, grads: Dict[str, torch.Tensor],
                            compute: int = capi.COMPUTE_FP32) -> None:
    """A7: gradients of every parameter given dL/d eps_hat (written into ``grads``)."""
    H, nb = model.H, model.n_blocks
    cp = compute
    Bn = g_out.shape[0]
    hs, pre = sv["hs"], sv["pre"]
    # eps_hat = Wout h + bout
    linear(g_out.T, hs[-1].T, grads["Wout"], compute=cp)
    colsum(g_out, grads["bout"])
    dh = torch.empty(Bn, H, device=g_out.device, dtype=torch.float32)
    linear(g_out, dev["Wout"].T, dh, compute=cp)
    dtemb = torch.zeros(Bn, H, device=g_out.device, dtype=torch.float32)
    g = torch.empty_like(dh)
    for k in range(nb - 1, -1, -1):
        W = dev[f"Wblk{k}"]
        silu_bwd(dh, pre[k], out=g)                                  # g = dh * silu'(a)
        dW = grads[f"Wblk{k}"]
        linear(g.T, hs[k].T, dW[:, :H], compute=cp)                  # dW_k = g^T h_k
        linear(g.T, sv["temb"].T, dW[:, H:], compute=cp)             # dU_k = g^T temb
        colsum(g, grads[f"bblk{k}"])
        linear(g, W[:, H:].T, dtemb, epi=capi.EPI_ACCUM, compute=cp)  # dtemb += g U_k
        dh_new = torch.empty_like(dh)
        linear(g, W[:, :H].T, dh_new, epi=capi.EPI_ADD_R, R=dh, compute=cp)  # dh += g W_k
        dh = dh_new
    # h0 = Win xt + bin
    linear(dh.T, sv["xt"].T, grads["Win"], compute=cp)
    colsum(dh, grads["bin"])
    # temb = Wt2 u + bt2 ; u = silu(a_t) ; a_t = Wt1 e + bt1
    linear(dtemb.T, sv["u"].T, grads["Wt2"], compute=cp)
    colsum(dtemb, grads["bt2"])
    du = torch.empty(Bn, H, device=g_out.device, dtype=torch.float32)
    linear(dtemb, dev["Wt2"].T, du, compute=cp)
    gt = silu_bwd(du, sv["a_t"])
    linear(gt.T, sv["e"].T, grads["Wt1"], compute=cp)
    colsum(gt, grads["bt1"])
