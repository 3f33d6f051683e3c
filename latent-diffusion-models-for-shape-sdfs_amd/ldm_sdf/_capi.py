"""ctypes binding of ``libldm_sdf.so`` (C ABI: ``include/ldm_sdf.h``).

torch is imported first so that the HIP runtime torch bundles (``libamdhip64.so.7``) is the
one the library binds to (same SONAME; SURVEY.md §7 'One HIP runtime per process').
The library is built in-tree by ``__graft_entry__.build()`` (``csrc/Makefile``).  There is
no fallback: if the library is missing or a call fails, this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import torch  # noqa: F401  (must precede the CDLL load)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libldm_sdf.so")
# diagnostic builds only (scripts/ablate_decoder.sh): an alternative in-tree library file
LIB_PATH = os.environ.get("LDM_SDF_LIB", LIB_PATH)
HEADER_PATH = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                            "..", "..", "include", "ldm_sdf.h"))

ABI_VERSION = 7   # 6: ldm_unet_loop* retired; 7: split16 removed, ldm_denoiser_train_step_dag
LDM_F32, LDM_BF16, LDM_F16 = 0, 1, 2
LDM_OP_DECODER_GRID, LDM_OP_DECODER_POINTS = 1, 2
LAYOUT_PASS8, LAYOUT_QUARTER, LAYOUT_SPLIT, LAYOUT_SPLIT16 = 0, 1, 2, 3
LAYOUT_CODES = {"split": LAYOUT_SPLIT}   # pass8 / quarter: removed in ABI 5, split16 in ABI 7
EPI_BIAS, EPI_SILU, EPI_RESID_SILU, EPI_ACCUM, EPI_ADD_R, EPI_RELU, EPI_MASK_R = range(7)
COMPUTE_FP32, COMPUTE_BF16 = 0, 1
COMPUTE_CODES = {"fp32": COMPUTE_FP32, "bf16": COMPUTE_BF16}
MAX_BLOCKS = 8

DTYPE_CODES = {"fp32": LDM_F32, "bf16": LDM_BF16, "fp16": LDM_F16}

_vp = C.c_void_p
_fp = C.c_void_p  # device float* passed as raw address


class Decoder(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("dtype", C.c_int32), ("hidden", C.c_int32),
                ("skip_width", C.c_int32), ("latent_dim", C.c_int32), ("n_stages", C.c_int32),
                ("weights", _vp), ("wz", _vp), ("bz", _vp), ("wxyz", _vp), ("w_last", _vp),
                ("b_last", C.c_float), ("layout", C.c_int32)]


class Sched(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("T", C.c_int32), ("sqrt_ab", _vp),
                ("sqrt_1mab", _vp), ("c1", _vp), ("c2", _vp), ("sigma", _vp)]


class Denoiser(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("dtype", C.c_int32), ("D", C.c_int32),
                ("H", C.c_int32), ("n_blocks", C.c_int32), ("TE", C.c_int32), ("T", C.c_int32),
                ("reserved", C.c_int32),
                ("w_in", _vp), ("b_in", _vp), ("w_t1", _vp), ("b_t1", _vp), ("w_t2", _vp),
                ("b_t2", _vp), ("w_blk", _vp * MAX_BLOCKS), ("b_blk", _vp * MAX_BLOCKS),
                ("e_tab", _vp * MAX_BLOCKS), ("w_out", _vp), ("b_out", _vp),
                ("emb_table", _vp), ("wt_in", _vp), ("wt_t2", _vp),
                ("wt_blk", _vp * MAX_BLOCKS), ("wt_out", _vp)]


class DenoiserGrads(C.Structure):
    """fp32 tensors in the denoiser's parameter shapes (ldm_denoiser_grads_t)."""
    _fields_ = [("w_in", _vp), ("b_in", _vp), ("w_t1", _vp), ("b_t1", _vp), ("w_t2", _vp),
                ("b_t2", _vp), ("w_blk", _vp * MAX_BLOCKS), ("b_blk", _vp * MAX_BLOCKS),
                ("w_out", _vp), ("b_out", _vp)]


ADAMW_MAX_TENSORS = 40


class AdamwTensor(C.Structure):
    _fields_ = [("p", _vp), ("g", _vp), ("m", _vp), ("v", _vp), ("p_bf16", _vp),
                ("p_bf16_t", _vp), ("rows", C.c_int32), ("cols", C.c_int32)]


class LinearArgs(C.Structure):
    _fields_ = [("Bn", C.c_int32), ("M", C.c_int32), ("K", C.c_int32), ("K2", C.c_int32),
                ("epi", C.c_int32), ("w_dtype", C.c_int32),
                ("X", _vp), ("sxb", C.c_int64), ("sxk", C.c_int64),
                ("W", _vp), ("swm", C.c_int64), ("swk", C.c_int64),
                ("X2", _vp), ("sx2b", C.c_int64), ("sx2k", C.c_int64),
                ("W2", _vp), ("sw2m", C.c_int64), ("sw2k", C.c_int64),
                ("bias", _vp), ("R", _vp), ("srb", C.c_int64),
                ("Y", _vp), ("syb", C.c_int64), ("sym", C.c_int64),
                ("A_out", _vp), ("sab", C.c_int64), ("compute", C.c_int32),
                ("ws", _vp), ("ws_floats", C.c_int64)]


GEMM_MAX_SEGS, GEMM_MAX_PROBS = 8, 4
(GEMM_STORE, GEMM_SILU, GEMM_RESID_SILU, GEMM_RELU, GEMM_ACCUM, GEMM_DGRAD_SILU, GEMM_LOSS,
 GEMM_ADD_R, GEMM_RELU_BWD) = range(9)


class GemmSeg(C.Structure):
    _fields_ = [("A", _vp), ("B", _vp), ("lda", C.c_int64), ("ldb", C.c_int64),
                ("K", C.c_int32), ("reserved", C.c_int32)]


class GemmProb(C.Structure):
    _fields_ = [("M", C.c_int32), ("N", C.c_int32), ("M_valid", C.c_int32), ("n_seg", C.c_int32),
                ("seg", GemmSeg * GEMM_MAX_SEGS), ("mode", C.c_int32), ("scale", C.c_float),
                ("bias", _vp), ("R", _vp), ("ldr", C.c_int64), ("P_in", _vp),
                ("ldp_in", C.c_int64), ("C", _vp), ("ldc", C.c_int64), ("P", _vp),
                ("ldp", C.c_int64), ("Cb", _vp), ("ldcb", C.c_int64), ("CbT", _vp),
                ("ldct", C.c_int64), ("colsum", _vp), ("loss_part", _vp),
                ("k_split", C.c_int32), ("ct_blk", C.c_int32), ("ws", _vp), ("Rb", _vp),
                ("ldrb", C.c_int64), ("slice_a", C.c_int64), ("slice_b", C.c_int64)]


class GemmArgs(C.Structure):
    _fields_ = [("n_prob", C.c_int32), ("tile", C.c_int32), ("prob", GemmProb * GEMM_MAX_PROBS)]


CONV_DIRECT, CONV_UP2 = 0, 1
CONV_MAX_SEGS = 4
CONV_EPI_STORE, CONV_EPI_DDPM = 0, 1


class ConvSeg(C.Structure):
    _fields_ = [("X", _vp), ("W", _vp), ("C", C.c_int32), ("L_in", C.c_int32),
                ("ksize", C.c_int32), ("stride", C.c_int32), ("pad", C.c_int32),
                ("mode", C.c_int32), ("silu_in", C.c_int32), ("ldw", C.c_int32),
                ("kstride", C.c_int32)]


class ConvArgs(C.Structure):
    _fields_ = [("B", C.c_int32), ("Cout", C.c_int32), ("L_out", C.c_int32),
                ("n_seg", C.c_int32), ("w_dtype", C.c_int32), ("epi", C.c_int32),
                ("seg", ConvSeg * CONV_MAX_SEGS),
                ("bias", _vp), ("bias2", _vp), ("cbias", _vp), ("scb", C.c_int64),
                ("R", _vp), ("Y", _vp), ("xlat", _vp), ("z", _vp),
                ("c1", _vp), ("c2", _vp), ("sigma", _vp), ("t", C.c_int32)]


# (name, restype, argtypes) -- every symbol include/ldm_sdf.h declares.
_i, _sz, _f = C.c_int, C.c_size_t, C.c_float
SIGNATURES = [
    ("ldm_abi_version", _i, []),
    ("ldm_last_error", C.c_char_p, []),
    ("ldm_workspace_bytes", _sz, [_i, _i, _i, _i]),
    ("ldm_workspace_bytes_layout", _sz, [_i, _i, _i, _i, _i]),
    ("ldm_grid_coords", _i, [_i, _i, _i, _f, _f, _fp, _vp]),
    ("ldm_decoder_fold", _i, [C.POINTER(Decoder), _fp, _i, _fp, _vp]),
    ("ldm_latent_rms_max", _i, [_fp, _i, _i, _fp, _vp]),
    ("ldm_decoder_grid_fwd", _i, [C.POINTER(Decoder), _fp, _i, _i, _i, _i, _f, _f, _fp, _vp,
                                  _sz, _vp]),
    ("ldm_decoder_points_fwd", _i, [C.POINTER(Decoder), _fp, _fp, _i, _i, _fp, _vp, _sz, _vp]),
    ("ldm_ddpm_step", _i, [C.POINTER(Sched), _fp, _fp, _fp, _i, _i, _fp, _vp]),
    ("ldm_q_sample", _i, [C.POINTER(Sched), _fp, _fp, _vp, _i, _i, _fp, _vp]),
    ("ldm_eps_mse_loss", _i, [_fp, _fp, _i, _fp, _fp, _vp]),
    ("ldm_denoiser_fwd_uniform_t", _i, [C.POINTER(Denoiser), _fp, _i, _i, _fp, _fp, _vp]),
    ("ldm_sample_step", _i, [C.POINTER(Denoiser), C.POINTER(Sched), _fp, _fp, _i, _i, _fp,
                             _fp, _vp]),
    ("ldm_sample_loop_supported", _i, [C.POINTER(Denoiser), _i]),
    ("ldm_sample_loop_ws_bytes", _sz, [_i, _i]),
    ("ldm_sample_loop", _i, [C.POINTER(Denoiser), C.POINTER(Sched), _fp, _fp, _i, _i, _i, _fp,
                             _sz, _vp]),
    ("ldm_sample_loop_status", _i, [_fp, _i, _i, C.POINTER(C.c_uint), _vp]),
    ("ldm_sample_loop_config", _i, [_i, C.c_uint, _i]),
    ("ldm_sample_loop_last_form", _i, []),
    ("ldm_adamw_step", _i, [_fp, _fp, _fp, _fp, _vp, C.c_int64, C.c_double, C.c_double,
                            C.c_double, C.c_double, C.c_double, _i, _vp]),
    ("ldm_linear", _i, [C.POINTER(LinearArgs), _vp]),
    ("ldm_linear_workspace_floats", C.c_int64, [C.POINTER(LinearArgs)]),
    ("ldm_silu_bwd", _i, [_fp, _fp, _i, _fp, _vp]),
    ("ldm_colsum", _i, [_fp, _i, _i, _fp, _i, _vp]),
    ("ldm_gather_rows", _i, [_fp, _vp, _i, _i, _fp, _vp]),
    ("ldm_relu_bwd", _i, [_fp, _fp, _i, _fp, _vp]),
    ("ldm_sdf_l1_loss", _i, [_fp, _fp, _i, _f, _f, _fp, _fp, _vp]),
    ("ldm_colsum_segments", _i, [_fp, _i, _i, _i, _fp, _i, _vp]),
    ("ldm_latent_l2_reg", _i, [_fp, _i, _i, _f, _fp, _fp, _vp]),
    ("ldm_conv1d", _i, [C.POINTER(ConvArgs), _vp]),
    ("ldm_gemm_bf16", _i, [C.POINTER(GemmArgs), _vp]),
    ("ldm_denoiser_train_ws_bytes", _sz, [C.POINTER(Denoiser), _i]),
    ("ldm_denoiser_fwd", _i, [C.POINTER(Denoiser), _fp, _vp, _i, _fp, _vp, _vp]),
    ("ldm_denoiser_bwd", _i, [C.POINTER(Denoiser), _vp, _fp, _i, C.POINTER(DenoiserGrads), _fp,
                              _vp]),
    ("ldm_q_sample_loss", _i, [C.POINTER(Sched), _fp, _fp, _vp, _i, _i, _fp, _fp, _fp, _fp, _vp]),
    ("ldm_denoiser_train_step", _i, [C.POINTER(Denoiser), C.POINTER(Sched), _fp, _fp, _vp, _i,
                                     _vp, C.POINTER(DenoiserGrads), _fp, _vp]),
    ("ldm_adamw_multi", _i, [C.POINTER(AdamwTensor), _i, C.c_double, C.c_double, C.c_double,
                             C.c_double, C.c_double, _i, _vp]),
    ("ldm_denoiser_train_step_adamw", _i, [C.POINTER(Denoiser), C.POINTER(Sched), _fp, _fp, _vp,
                                           _i, _vp, C.POINTER(DenoiserGrads), _fp,
                                           C.POINTER(AdamwTensor), _i, C.c_double, C.c_double,
                                           C.c_double, C.c_double, C.c_double, _i, _vp, _vp,
                                           _vp]),
    ("ldm_train_step_config", _i, [_i, C.c_uint]),
    ("ldm_train_step_last_form", _i, []),
    ("ldm_denoiser_train_status", _i, [C.POINTER(Denoiser), _i, _vp, C.POINTER(C.c_uint), _vp]),
    ("ldm_denoiser_train_ws_init", _i, [C.POINTER(Denoiser), _i, _vp, _vp]),
    ("ldm_denoiser_train_dag_describe", _i, [C.POINTER(Denoiser), C.POINTER(Sched), _i, _vp,
                                             C.POINTER(DenoiserGrads), C.POINTER(AdamwTensor),
                                             _i, C.c_char_p, _sz]),
    ("ldm_adamw_hyper", None, [C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, _i,
                               _fp]),
    ("ldm_mc_workspace_bytes", _sz, [_i]),
    ("ldm_mc_count", _i, [_fp, _i, _f, _vp, _sz, _vp, _vp]),
    ("ldm_mc_emit", _i, [_fp, _i, _f, _f, _f, _vp, _sz, _fp, _vp, _vp]),
    ("ldm_mc_table", _i, [_vp, _vp]),
]

_lib: Optional[C.CDLL] = None


class LdmError(RuntimeError):
    pass


def load() -> C.CDLL:
    """Load libldm_sdf.so (raises if it is not built -- there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LdmError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                           f"(make -C csrc).  The HIP path has no fallback.")
        lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.ldm_abi_version() != ABI_VERSION:
            raise LdmError(f"libldm_sdf ABI {lib.ldm_abi_version()} != {ABI_VERSION}")
        _lib = lib
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().ldm_last_error().decode(errors="replace")
        raise LdmError(f"{what} failed (rc={rc}): {msg}")


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device: Optional[torch.device] = None) -> Optional[int]:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise LdmError("ldm_sdf runs on the GPU only (HIP kernels); got a CPU tensor. "
                           "The CPU restatement lives in oracle/ and is test infrastructure.")
