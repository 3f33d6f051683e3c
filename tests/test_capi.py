"""CPU checks of the drop-in boundary: libldm_sdf.so loads and exports every symbol that
include/ldm_sdf.h declares; the ctypes structs match the C layout (compiled with gcc)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ldm_sdf.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ldm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from ldm_sdf import _capi as capi
    lib = capi.load()
    names = declared_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    # and the ctypes binding covers all of them
    assert sorted(n for n, _, _ in capi.SIGNATURES) == names


def test_abi_version_and_error_path_without_gpu():
    from ldm_sdf import _capi as capi
    lib = capi.load()
    assert lib.ldm_abi_version() == 7
    # argument validation runs before any device work
    assert lib.ldm_grid_coords(0, 0, 0, 0.0, 0.0, None, None) == -22
    assert b"bad grid slab" in lib.ldm_last_error()
    assert lib.ldm_decoder_grid_fwd(None, None, 1, 8, 0, 8, 0.1, -1.0, None, None, 0, None) != 0
    assert lib.ldm_workspace_bytes(1, 4, 256, 1) == 4 * 4 * 8192            # the split layout
    assert lib.ldm_workspace_bytes_layout(1, 4, 256, 1, 2) == 4 * 4 * 8192   # split layout
    assert lib.ldm_workspace_bytes_layout(1, 4, 256, 1, 3) == 0   # split16: removed in ABI 7


def test_struct_layouts_match_c():
    from ldm_sdf import _capi as capi
    code = r'''
    #include <stdio.h>
    #include <stddef.h>
    #include "ldm_sdf.h"
    int main(void) {
      printf("%zu %zu %zu %zu\n", sizeof(ldm_decoder_t), sizeof(ldm_sched_t),
             sizeof(ldm_denoiser_t), sizeof(ldm_linear_args_t));
      printf("%zu %zu %zu %zu\n", offsetof(ldm_decoder_t, weights), offsetof(ldm_decoder_t, b_last),
             offsetof(ldm_denoiser_t, e_tab), offsetof(ldm_linear_args_t, A_out));
      printf("%zu %zu %zu %zu\n", sizeof(ldm_conv1d_seg_t), sizeof(ldm_conv1d_args_t),
             offsetof(ldm_conv1d_args_t, bias), offsetof(ldm_conv1d_args_t, t));
      printf("%zu %zu %zu %zu\n", sizeof(ldm_denoiser_grads_t), sizeof(ldm_adamw_tensor_t),
             offsetof(ldm_denoiser_t, wt_blk), offsetof(ldm_denoiser_grads_t, b_out));
      printf("%zu %zu %zu %zu %zu\n", sizeof(ldm_gemm_seg_t), sizeof(ldm_gemm_prob_t),
             sizeof(ldm_gemm_args_t), offsetof(ldm_gemm_prob_t, bias),
             offsetof(ldm_gemm_prob_t, loss_part));
      printf("%zu %zu %zu\n", offsetof(ldm_gemm_prob_t, ws), offsetof(ldm_gemm_prob_t, ldrb),
             offsetof(ldm_gemm_prob_t, slice_b));
      return 0; }
    '''
    tmp = "/tmp/ldm_layout_check"
    with open(tmp + ".c", "w") as f:
        f.write(code)
    r = subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), tmp + ".c", "-o", tmp],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("gcc unavailable: " + r.stderr[:200])
    out = subprocess.run([tmp], capture_output=True, text=True).stdout.split()
    sizes = [int(x) for x in out]
    assert sizes[:4] == [ctypes.sizeof(capi.Decoder), ctypes.sizeof(capi.Sched),
                         ctypes.sizeof(capi.Denoiser), ctypes.sizeof(capi.LinearArgs)]
    assert sizes[4:8] == [capi.Decoder.weights.offset, capi.Decoder.b_last.offset,
                          capi.Denoiser.e_tab.offset, capi.LinearArgs.A_out.offset]
    assert sizes[8:12] == [ctypes.sizeof(capi.ConvSeg), ctypes.sizeof(capi.ConvArgs),
                           capi.ConvArgs.bias.offset, capi.ConvArgs.t.offset]
    assert sizes[12:16] == [ctypes.sizeof(capi.DenoiserGrads), ctypes.sizeof(capi.AdamwTensor),
                            capi.Denoiser.wt_blk.offset, capi.DenoiserGrads.b_out.offset]
    sizes = sizes[4:]
    assert sizes[12:17] == [ctypes.sizeof(capi.GemmSeg), ctypes.sizeof(capi.GemmProb),
                            ctypes.sizeof(capi.GemmArgs), capi.GemmProb.bias.offset,
                            capi.GemmProb.loss_part.offset]
    assert sizes[17:20] == [capi.GemmProb.ws.offset, capi.GemmProb.ldrb.offset,
                            capi.GemmProb.slice_b.offset]
    assert len(sizes) == 20
