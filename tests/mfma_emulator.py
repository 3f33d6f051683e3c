"""CPU emulation of the MFMA decoder kernel's data flow (TEST INFRASTRUCTURE).

Follows csrc/decoder_fs.hip (split layout) at the
fragment level -- the packed per-wave weight streams, the per-shape aux fragments, the B
fragment built from xyz, the v_mfma_f32_32x32x16 operand/result lane maps
(cdna_hip_programming.md §3), the accumulator -> next-B-fragment conversion with 16-bit
rounding + ReLU and the fused fp32 final layer -- so the host packer (ldm_sdf/pack.py) is
validated against the oracle without a GPU.  Accumulation is fp64 here,
so the result differs from the device only by fp32 summation order.
"""
from __future__ import annotations

import numpy as np
import torch

from ldm_sdf import pack

# A operand: Am[r][k'] = frag[lane = r + 32*(k'//8)][k' % 8]   (same map for B with r -> col)
_K = np.arange(16)
_LANE_OF = (np.arange(32)[:, None] + 32 * (_K[None, :] // 8))        # [32 r, 16 k']
_ELEM_OF = np.broadcast_to(_K[None, :] % 8, (32, 16))


def frag_to_A(frag: np.ndarray) -> np.ndarray:
    """frag [64, 8] -> A[32 rows, 16 k]."""
    return frag[_LANE_OF, _ELEM_OF]


def frag_to_B(frag: np.ndarray) -> np.ndarray:
    """frag [64, 8] -> B[16 k, 32 cols]."""
    return frag[_LANE_OF, _ELEM_OF].T


def acc_rows(h: int) -> np.ndarray:
    """Row held by accumulator register v in lane half h: (v&3) + 8(v>>2) + 4h."""
    v = np.arange(16)
    return (v & 3) + 8 * (v >> 2) + 4 * h


def acc_to_Bmats(C: np.ndarray, dt: torch.dtype):
    """C [32 rows, 32 cols] (fp) -> two B matrices [16, 32] for k-steps 2i, 2i+1 after 16-bit
    rounding and ReLU, in the k order the hardware sees (element j of lane half h)."""
    out = []
    for s in range(2):
        Bm = np.zeros((16, 32))
        for h in range(2):
            rows = acc_rows(h)[8 * s:8 * s + 8]                 # element j -> row
            vals = C[rows, :]                                    # [8, 32]
            r = torch.from_numpy(vals).to(torch.float32).to(dt).to(torch.float64).numpy()
            Bm[8 * h:8 * h + 8, :] = np.maximum(r, 0.0)
        out.append(Bm)
    return out


def round_dt(x, dt):
    return torch.as_tensor(x, dtype=torch.float32).to(dt).to(torch.float64).numpy()


def split_aux_shape(beta_b: np.ndarray, wxyz: np.ndarray, skip_width: int, dt) -> np.ndarray:
    """Per-shape aux fragments of the split layout (csrc/decoder_fs.hip fs_aux_pack_kernel):
    ``[4 waves][4 slots: L0p0, L0p1, L4p0, L4p1][2 frags][64][8]``; lane < 32 of frag i holds
    ``[wx,wy,wz,wx,wy,wz,beta_hi,beta_lo]`` of row ``row_base + 32 i + lane``."""
    out = np.zeros((4, 4, 2, 64, 8))
    for w in range(4):
        for slot, (li, l, p) in enumerate([(0, 0, 0), (0, 0, 1), (1, 4, 0), (1, 4, 1)]):
            rb = pack.split_row_base(l, p, w, skip_width)
            for i in range(2):
                f = rb + 32 * i + np.arange(32)
                hi = round_dt(beta_b[li, f], dt)
                lo = round_dt(beta_b[li, f] - hi, dt)
                out[w, slot, i, :32, 0:3] = round_dt(wxyz[li][f], dt)
                out[w, slot, i, :32, 3:6] = round_dt(wxyz[li][f], dt)
                out[w, slot, i, :32, 6] = hi
                out[w, slot, i, :32, 7] = lo
    return out


def emulate_split(packed: dict, beta: np.ndarray, xyz: np.ndarray, dtype: str) -> np.ndarray:
    """Dataflow replay of the split layout (csrc/decoder_fs.hip): per layer, every wave's parts
    read the shared activations ACT[k-step][point chunk] in the part's k order (pack.split_kidx),
    their A fragments from the wave's own stream, the aux step (bias / xyz + folded latent)
    first; outputs convert (16-bit, ReLU) into the next ACT at k-step row_base/16 + 2i + s.
    xyz [B, P, 3] with P a multiple of 128 -> sdf [B, P] (float64 sums)."""
    dt = torch.bfloat16 if dtype == "bf16" else torch.float16
    sw = packed["skip_width"]
    parts = pack.split_parts(sw)
    nst = packed["n_stages"]
    blob = packed["weights"].to(torch.float64).numpy()
    ns = 4 * nst * 2 * 64 * 8
    stream = blob[:ns].reshape(4, nst, 2, 64, 8)
    baux = blob[ns:].reshape(4, len(parts), 2, 64, 8)
    wl = packed["w_last"].numpy().astype(np.float64).reshape(4, 2, 2, 2, 16)
    wxyz = packed["wxyz"].numpy().astype(np.float64)
    B, P, _ = xyz.shape
    out = np.zeros((B, P))
    for b in range(B):
        saux = split_aux_shape(beta[b], wxyz, sw, dt)
        for g0 in range(0, P, 128):
            Bx = []
            for n in range(4):
                x = xyz[b, g0 + 32 * n:g0 + 32 * n + 32].astype(np.float32)
                hi = round_dt(x, dt)
                lo = round_dt(x.astype(np.float64) - hi, dt)
                m = np.zeros((16, 32))
                m[0:3], m[3:6], m[6:8] = hi.T, lo.T, 1.0
                Bx.append(m)
            act = {}
            pos = [0] * 4
            part_acc = np.zeros((4, 64))            # [n][lane]
            for layer in range(8):
                new_act = {}
                for w in range(4):
                    for pi, (l, p) in enumerate(parts):
                        if l != layer:
                            continue
                        if l in (0, 4):
                            afr = saux[w, (0 if l == 0 else 2) + p]
                        else:
                            afr = baux[w, pi]
                        C = [[frag_to_A(afr[i]) @ Bx[n] for n in range(4)] for i in range(2)]
                        kidx = pack.split_kidx(l, sw) if l else []
                        for j, k in enumerate(kidx):
                            fr = stream[w, pos[w] + j]
                            for i in range(2):
                                A = frag_to_A(fr[i])
                                for n in range(4):
                                    C[i][n] = C[i][n] + A @ act[k][n]
                        pos[w] += len(kidx)
                        rb = pack.split_row_base(l, p, w, sw)
                        for i in range(2):
                            for n in range(4):
                                if l == 7:
                                    for h in range(2):
                                        rows = acc_rows(h)
                                        part_acc[n, 32 * h:32 * h + 32] += (
                                            np.maximum(C[i][n][rows, :], 0)
                                            * wl[w, p, i, h][:, None]).sum(0)
                                else:
                                    f0, f1 = acc_to_Bmats(C[i][n], dt)
                                    k0 = rb // 16 + 2 * i
                                    new_act.setdefault(k0, [None] * 4)[n] = f0
                                    new_act.setdefault(k0 + 1, [None] * 4)[n] = f1
                act = new_act
            tot = part_acc[:, :32] + part_acc[:, 32:]                # [n, 32]
            out[b, g0:g0 + 128] = np.tanh(tot.reshape(-1) + packed["b_last"])
    return out
