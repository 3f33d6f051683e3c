// One 64 x 64 tile of the multi-tensor AdamW update (ldm_adamw_multi, denoiser_train.hip), shared
// with the persistent training-step kernel (train_dag.hip) so both update every parameter with
// the same instructions (the update is ldm_adamw_step's, operation for operation: ddpm_common.h
// adamw_update).  The transposed bf16 copy goes through an LDS tile so its stores are 32-byte
// row runs.
#pragma once
#include "ldm_internal.h"
#include "ddpm_common.h"
#include "wt_store.h"

namespace ldm {

// adamw_hyper's 7 scalars: [1 - lr wd, 1 - beta1, beta2, 1 - beta2, eps, lr / bc1, sqrt(bc2)]
struct AdamHyper {
    float decay, omb1, b2, omb2, eps, step_size, bc2_sqrt;
};

// Tile `tl` (row-major over the tensor's 64 x 64 tiles; a 1-D tensor is one row) of tensor T:
// each thread 4 rows x 4 consecutive columns.  TT: ldm_adamw_tensor_t in any address space.
// WT: write-through stores and an sc1 load of the gradient (wt_store.h).
// tid: the thread's index among the tile's 256 (a 512-thread caller runs two tiles at once).
// mode (the one-launch step's split update, train_dag.hip): 0 the whole update; 1 p, m, v only
// (no bf16 copies, no barrier); 2 the bf16 copies only, from the p a mode-1 tile stored (read
// sc1 when WT).  Modes 1 then 2 store exactly what mode 0 stores.
//
// VEC (the dispatcher below): the tile spans 64 whole columns of a row length divisible by 4,
// so every lane's 4 columns are one aligned 16-byte vector -- a tile-uniform property, decided
// once per tile.  (Round 6: decided per lane inside the row loop, the two load forms merged
// into one set of registers, and the compiler waited for each row's first load before issuing
// the next row's -- four serial round trips per tile instead of one.)
template <bool WT, bool VEC, typename TT>
__device__ __forceinline__ void adamw_tile_body(TT& T, const AdamHyper& hy,
                                                unsigned short (&sT)[64][64 + 8], int r0, int c0,
                                                int tid, int mode) {
    const int rows = T.rows, cols = T.cols;
    // extents (wt_store.h): fp32 p, g, m, v and the bf16 copies, rows x cols each
    const uint32_t x4 = ext_bytes(rows, cols, cols, 4), x2 = ext_bytes(rows, cols, cols, 2);
    const int cq = (tid & 15) * 4;
    const float decay = hy.decay, omb1 = hy.omb1, b2 = hy.b2, omb2 = hy.omb2, eps = hy.eps,
                step_size = hy.step_size, bc2_sqrt = hy.bc2_sqrt;
    float* __restrict__ P = T.p;
    const float* __restrict__ Gp = T.g;
    float* __restrict__ M = T.m;
    float* __restrict__ V = T.v;
    // every load of the thread's 4 rows x 4 columns first (16-byte vectors when VEC), then the
    // updates, then the stores: one memory round trip
    constexpr bool vec = VEC;
    // (ragged columns: a lane past the row's end loads the row's last element instead -- its
    // value is never stored -- so no load leaves the tensor; round 6, found by the DEBUG build:
    // the fall-back used to be the lane's first column, itself past the end when c0 + cq >= cols)
    f32x4 p4[4], g4[4], m4[4], v4[4];
    int64_t off[4], in_row[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = min(r0 + (tid >> 4) + 16 * i, rows - 1);
        off[i] = (int64_t)r * cols + c0 + cq;
        in_row[i] = (int64_t)r * cols;
    }
    // the mode test outside the row loop, and a scheduling barrier after the loads: left free,
    // the scheduler started row 0's update (with its waits) before issuing rows 1-3's loads
    if (mode == 2) {                              // the copies: the stored p only
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr (vec) {
                p4[i] = vld_at<WT, f32x4>(P, x4, off[i]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    p4[i][e] = vld_at<WT, float>(P, x4, in_row[i] + min(c0 + cq + e, cols - 1));
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr (vec) {
                p4[i] = *reinterpret_cast<const f32x4*>(P + off[i]);
                g4[i] = vld_at<WT, f32x4>(Gp, x4, off[i]);  // (WT: the handed-off gradient, sc1)
                m4[i] = *reinterpret_cast<const f32x4*>(M + off[i]);
                v4[i] = *reinterpret_cast<const f32x4*>(V + off[i]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int64_t x = in_row[i] + min(c0 + cq + e, cols - 1);
                    p4[i][e] = P[x]; g4[i][e] = vld_at<WT, float>(Gp, x4, x); m4[i][e] = M[x];
                    v4[i][e] = V[x];
                }
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rl = (tid >> 4) + 16 * i;
        const bool rin = r0 + rl < rows;
        unsigned short q[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float pi = p4[i][e], mi = m4[i][e], vi = v4[i][e];
            if (mode != 2)
                adamw_update(pi, g4[i][e], mi, vi, decay, omb1, b2, omb2, eps, step_size,
                             bc2_sqrt);
            p4[i][e] = pi; m4[i][e] = mi; v4[i][e] = vi;
            const unsigned u = __builtin_bit_cast(unsigned, pi);
            q[e] = (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
            sT[cq + e][rl] = rin ? q[e] : (unsigned short)0;
        }
        if (!rin) continue;
        if constexpr (vec) {
            if (mode != 2) {
                vst_at<WT>(P, x4, off[i], p4[i]);
                vst_at<WT>(M, x4, off[i], m4[i]);
                vst_at<WT>(V, x4, off[i], v4[i]);
            }
            if (T.p_bf16 && mode != 1) {
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 w = {(unsigned)q[0] | ((unsigned)q[1] << 16),
                                 (unsigned)q[2] | ((unsigned)q[3] << 16)};
                vst_at<WT>(reinterpret_cast<unsigned short*>(T.p_bf16), x2, off[i], w);
            }
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (c0 + cq + e >= cols) continue;
                if (mode != 2) {
                    vst_at<WT>(P, x4, off[i] + e, p4[i][e]);
                    vst_at<WT>(M, x4, off[i] + e, m4[i][e]);
                    vst_at<WT>(V, x4, off[i] + e, v4[i][e]);
                }
                if (T.p_bf16 && mode != 1)
                    vst_at<WT>(reinterpret_cast<unsigned short*>(T.p_bf16), x2, off[i] + e, q[e]);
            }
        }
    }
    if (!T.p_bf16_t || mode == 1) return;
    __syncthreads();
    // transposed: [c][r], 16 consecutive rows per thread (4 threads per column)
    const int cl = tid >> 2, rb = (tid & 3) * 16;
    const int c = c0 + cl;
    if (c >= cols) return;
    unsigned short* dst = reinterpret_cast<unsigned short*>(T.p_bf16_t);   // (uniform base)
    const int64_t cr = (int64_t)c * rows;
    if ((rows & 7) == 0 && r0 + rb + 16 <= rows) {
        u32x4 w0, w1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            w0[e] = (unsigned)sT[cl][rb + 2 * e] | ((unsigned)sT[cl][rb + 2 * e + 1] << 16);
            w1[e] = (unsigned)sT[cl][rb + 8 + 2 * e] | ((unsigned)sT[cl][rb + 9 + 2 * e] << 16);
        }
        vst_at<WT>(dst, x2, cr + r0 + rb, w0);
        vst_at<WT>(dst, x2, cr + r0 + rb + 8, w1);
    } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int r = r0 + rb + e;
            if (r < rows) vst_at<WT>(dst, x2, cr + r, sT[cl][rb + e]);
        }
    }
}

template <bool WT = false, typename TT>
__device__ __forceinline__ void adamw_tile(TT& T, const AdamHyper& hy,
                                           unsigned short (&sT)[64][64 + 8], int tl,
                                           int tid = threadIdx.x, int mode = 0) {
    const int cols = T.cols;
    const int tcn = (cols + 63) / 64;
    const int r0 = (tl / tcn) * 64, c0 = (tl % tcn) * 64;
    LDM_DASSERT(tl >= 0 && r0 < T.rows);                // the tile lies inside the tensor
    if ((cols & 3) == 0 && c0 + 64 <= cols)
        adamw_tile_body<WT, true>(T, hy, sT, r0, c0, tid, mode);
    else
        adamw_tile_body<WT, false>(T, hy, sT, r0, c0, tid, mode);
}

}  // namespace ldm
