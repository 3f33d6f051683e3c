// Grouped bf16 GEMM with fused training epilogues (ldm_gemm_bf16): the matrix-core engine of
// the DDPM denoiser's training step (A6/A7 at batch 1000, config 2) and of the C19 auto-decoder.
//
//   C[m][n] = sum_seg sum_{k < K_seg} A_seg[m][k] * B_seg[n][k]      (both operands bf16,
//                                                                     k contiguous: "NT")
// then one epilogue per problem (include/ldm_sdf.h LDM_GEMM_*): bias, SiLU / residual+SiLU /
// ReLU, the SiLU backward of the layer below, the eps-MSE gradient, accumulation; outputs in
// fp32, bf16 and bf16 TRANSPOSED ([n][m]), plus per-32-row column sums (bias gradients) and
// per-tile loss sums -- all written from the accumulators, so every operand the next GEMM
// needs is produced here in the layout it wants (k contiguous).  No GEMM reads a transposed
// view; no separate cast / transpose / colsum / silu-backward launch exists.
//
// Why this shape (PMC in profiles/r02a/pmc_train): the generic ldm_linear MFMA
// kernel staged fp32 operands through registers one 128-deep chunk at a time and sat at 3-4 %
// MFMA busy, 51-59 % of wave time parked on memory.  Here
//   * operands are bf16 in HBM (half the bytes) and arrive by LDS-DMA (global_load_lds, 16 B
//     per lane, no VGPR staging) into a STAGES-deep ring: STAGES-1 k-steps in flight across raw
//     s_barriers, retired by a counted vmcnt (never 0 in the steady state);
//   * the LDS image is lane-linear per DMA instruction (8 rows x 128 B) with the 16-byte chunks
//     of row r XOR-permuted by (r >> 1) & 7 on the SOURCE address, so the ds_read_b128 fragment
//     reads of 16 rows are conflict-free (guide T2, rule 21);
//   * several independent GEMMs can share one launch (problems), so small backward products
//     fill the chip together.
// Tiles: BM x BN per 4-wave workgroup (64 or 128 each), each wave (BM/2) x (BN/2) as
// RM x RN v_mfma_f32_32x32x16_bf16 tiles; k-step 64.
#include "ldm_internal.h"

#include <mutex>
#include "ddpm_common.h"
#include "gemm_tile.h"

#include <algorithm>
#include <type_traits>
#include <stdlib.h>
#include <string.h>

namespace ldm {
namespace {
using namespace gtile;

// The launch's argument block: the caller's problems plus the tile bookkeeping the host
// resolves once (first tile and tile counts per problem, k-steps per tile, split-K slices), so
// a workgroup finds its problem with one batch of scalar loads instead of a dependent chain.
struct GemmKArgs {
    int n_prob, total;
    int first[LDM_GEMM_MAX_PROBS];      // first tile of each problem (INT_MAX when unused)
    int tiles_m[LDM_GEMM_MAX_PROBS], tiles_n[LDM_GEMM_MAX_PROBS];
    int nk[LDM_GEMM_MAX_PROBS];         // k-steps per tile (per slice when split)
    int ksplit[LDM_GEMM_MAX_PROBS];     // slices (1: whole K)
    ldm_gemm_prob_t prob[LDM_GEMM_MAX_PROBS];
};
typedef const __attribute__((address_space(4))) GemmKArgs KArgs;
typedef const __attribute__((address_space(4))) ldm_gemm_prob_t KProb;


// Tile t of the launch -> (problem, output origin, split-K slice).  Tiles of a problem are
// slice-major; inside a slice, groups of 4 tile-rows, column-major inside a group (L2 reuse of
// both panels).
template <int BM, int BN>
__device__ __forceinline__ TileLoc locate(KArgs* ka, int t) {
    const int p = (t >= ka->first[1]) + (t >= ka->first[2]) + (t >= ka->first[3]);
    const int tm_n = ka->tiles_m[p], tn_n = ka->tiles_n[p];
    int tl = t - ka->first[p];
    const int slice = tl / (tm_n * tn_n);
    tl -= slice * tm_n * tn_n;
    const int tg = tl / (4 * tn_n), gh = min(4, tm_n - tg * 4), in = tl - tg * 4 * tn_n;
    return {p, (tg * 4 + in % gh) * BM, (in / gh) * BN, slice};
}

// KG = 1: 4 waves, 2 x 2 over the output tile, every wave walks every k-step.
// KG = 2: 8 waves = two k-groups of 4; group g computes the k-steps of parity g (two waves per
// SIMD working on different stages, so one's LDS reads overlap the other's MFMAs) and the two
// partial tiles are summed through LDS before the epilogue.  The ring holds STAGES / KG
// "super-stages" of KG consecutive k-steps.
// PERSIST: one workgroup per resident slot walks a list of tiles (the XCD's contiguous share
// of the launch, strided by the XCD's workgroup count, so the tiles an XCD runs at once share
// their operand panels in its L2).  The ring is one continuous stream of k-steps across tile
// boundaries: the next tile's first stages are in flight while the current tile finishes its
// MFMAs and runs its epilogue (which touches no LDS), so no workgroup pays the pipeline fill of
// a short-K tile (C19: K = 512, 8 k-steps) and the epilogue of one tile overlaps loads of the
// next.
// Diagnostic build only (-DGEMM_STAMP=1, scripts/stamp_gemm.py): workgroup 0 of every
// non-persistent, LDS-DMA launch keeps s_memrealtime marks in registers -- entry, prologue
// stages issued, first stage landed, k-loop done, epilogue issued, stores drained -- and writes
// them at its end into a ring of 256 launches (ldm_dev_gemm_stamps).
#ifndef GEMM_STAMP
#define GEMM_STAMP 0
#endif
#if GEMM_STAMP
__device__ uint64_t g_gemm_stamp[256][8];
__device__ unsigned g_gemm_stamp_n;
#endif
struct GStamp {
    bool on;
    uint64_t t[8];
    __device__ __forceinline__ void mark(int k) {
        if (GEMM_STAMP && on) t[k] = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ void flush(int grid, int tiles) {
#if GEMM_STAMP
        if (!on) return;
        uint64_t* p = g_gemm_stamp[atomicAdd(&g_gemm_stamp_n, 1u) & 255u];
        t[6] = (uint64_t)grid;
        t[7] = (uint64_t)tiles;
        for (int i = 0; i < 8; ++i) p[i] = t[i];
#endif
    }
};

template <int BM, int BN, int STAGES, int KG, bool RS, bool PERSIST, int KB>
__global__ __launch_bounds__(256 * KG) void gemm_bf16_kernel(GemmKArgs a) {
    GStamp gs;
    gs.on = GEMM_STAMP && !PERSIST && !RS && blockIdx.x == 0 && threadIdx.x == 0;
    gs.mark(0);
    extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
    constexpr int RM = BM / 64, RN = BN / 64, NW = 4 * KG;
    constexpr int A_ELEMS = BM * KB, STAGE_ELEMS = (BM + BN) * KB;
    constexpr int G = TileSrc<BM, NW, KB>::NP + TileSrc<BN, NW, KB>::NP;   // DMA pieces/wave/stage
    constexpr int SS = STAGES / KG;                   // super-stages in the ring
    static_assert(STAGES % KG == 0 && SS >= 2, "ring of whole super-stages");
    static_assert(!PERSIST || (KG == 1 && !RS), "persistent: one k-group, LDS-DMA ring");
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int grp = wave >> 2, w4 = wave & 3;
    const int wr = w4 >> 1, wc = w4 & 1;
    const int r32 = lane & 31, h = lane >> 5;

    // The argument block is read through the kernarg segment pointer (scalar loads at a
    // runtime offset); indexing the by-value parameter by a runtime problem id would copy it
    // to scratch.
    KArgs* ka = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    const int lid = blockIdx.x, tot_all = ka->total;

    // ---- tile walk --------------------------------------------------------------------------
    // non-persistent: one tile, XCD-aware deal of the linear workgroup id (bijective);
    // persistent: tiles t0, t0 + tstep, ... < tend (the XCD's contiguous chunk)
    int t0, tstep, tend;
    if constexpr (PERSIST) {
        // XCD x (= lid % 8 under round-robin dispatch) has nx workgroups; its chunk of the
        // tiles is proportional to nx (any grid size, also below 8)
        const int Gd = gridDim.x, q = Gd >> 3, r = Gd & 7, x = lid & 7;
        const int nx = q + (x < r), cum = x * q + min(x, r);
        t0 = (int)((int64_t)tot_all * cum / Gd) + (lid >> 3);
        tend = (int)((int64_t)tot_all * (cum + nx) / Gd);
        tstep = nx;
        if (t0 >= tend) return;                       // no tile (whole workgroup, uniform)
    } else {
        const int q = tot_all / 8, r = tot_all % 8, x = lid % 8;
        t0 = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lid / 8;
        tstep = 1;
        tend = t0 + 1;
    }

    // ---- DMA issue cursor: tile ti, k-step ki of nki; sources re-seated per tile / segment --
    TileSrc<BM, NW, KB> srcA;
    TileSrc<BN, NW, KB> srcB;
    int ti = t0, ki = 0, nki = 0, seg = -1, seg_left = 0, qi = 0;
    TileLoc il{};
    auto seat = [&](int sg, int kofs) {       // sources of segment sg, kofs k-steps in
        KProb& P = ka->prob[il.p];
        const __attribute__((address_space(4))) ldm_gemm_seg_t& S = P.seg[sg];
        srcA.init(reinterpret_cast<const unsigned short*>(S.A), S.lda, il.m0, P.M, wave, lane);
        srcB.init(reinterpret_cast<const unsigned short*>(S.B), S.ldb, il.n0, P.N, wave, lane);
        if (P.slice_a) {                      // split-K slice = one block of a blocked operand
            srcA.base += 2 * P.slice_a * il.slice;
            srcB.base += 2 * P.slice_b * il.slice;
            seg_left = ka->nk[il.p];
        } else {
            srcA.base += 2 * KB * kofs;
            srcB.base += 2 * KB * kofs;
            seg_left = S.K / KB - kofs;
        }
    };
    auto issue = [&]() {                      // the next stage (past the last tile: a dummy)
        const bool again = ti >= tend;
        if (!again) {
            if (ki == 0) {
                il = locate<BM, BN>(ka, ti);
                nki = ka->nk[il.p];
                seg = 0;
                seat(0, il.slice * nki);
            } else if (seg_left == 0) {
                seat(++seg, 0);
            }
        }
        unsigned short* st = smem + (qi % STAGES) * STAGE_ELEMS;
        ++qi;
        srcA.issue(st, wave, again);
        srcB.issue(st + A_ELEMS, wave, again);
        if (!again) {
            --seg_left;
            if (++ki == nki) {
                ki = 0;
                ti += tstep;
            }
        }
    };

    f32x16 acc[RM][RN];
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
    };
    zero_acc();

    auto compute = [&](const unsigned short* sa) {
        const unsigned short* sb = sa + A_ELEMS;
        // every fragment of the stage first (one LDS round trip), then the MFMAs
        u32x4 af[KB / 16][RM], bf[KB / 16][RN];
#pragma unroll
        for (int s = 0; s < KB / 16; ++s) {
#pragma unroll
            for (int i = 0; i < RM; ++i)
                af[s][i] = read_frag<KB>(sa, wr * (BM / 2) + i * 32 + r32, 2 * s + h);
#pragma unroll
            for (int j = 0; j < RN; ++j)
                bf[s][j] = read_frag<KB>(sb, wc * (BN / 2) + j * 32 + r32, 2 * s + h);
        }
        __builtin_amdgcn_sched_barrier(0);     // keep the reads batched ahead of the MFMAs
#pragma unroll
        for (int s = 0; s < KB / 16; ++s)
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int j = 0; j < RN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, af[s][i]),
                        __builtin_bit_cast(bf16x8, bf[s][j]), acc[i][j], 0, 0, 0);
    };

    // ---- LDS-transposed epilogue (non-persistent kernels) -------------------------------------
    // The accumulator layout gives a lane ONE column of 16 rows, so the row-major outputs above
    // take one 4-byte (bf16: 2-byte) store per element: 16-52 store instructions per 32 x 32
    // block, and a one-tile-per-CU launch ends in that store-issue tail (the block GEMM: 11 us
    // with a plain store, 18.7 us with RESID_SILU's four outputs, profiles/r02f).  Here the
    // block goes through a per-wave 4 KiB LDS tile first, so a lane holds 4 consecutive columns
    // of 4 rows: every row-major operand moves as 16-byte (bf16: 8-byte) vectors, 4 per output.
    // The element-wise arithmetic is the same expression per element as epi(), so the outputs
    // are bit-identical; the column sums and the transposed bf16 copy are formed from the
    // results read back in accumulator layout, in epi()'s order (bit-identical too).
    // Falls back to the accumulator-layout stores for a block that crosses N, or operands whose
    // pointers / strides do not allow the vectors.
    constexpr int EPI_LDS_OFF = KG == 2 ? RM * 4 * RN * 16 * 64 * 4 : 0;   // past KG's `red`
    static_assert(PERSIST || EPI_LDS_OFF + NW * 4096 <= STAGES * STAGE_ELEMS * 2,
                  "epilogue scratch fits the ring");
    // LDS-transposed epilogue of one 32 x 32 block (gemm_tile.h epi_lds_block)
    auto epi_lds = [&](const TileLoc& L, const f32x16& c, const int i, const int nb,
                       const EpiArgs& e) __attribute__((always_inline)) {
        epi_lds_block<BM>(smem, EPI_LDS_OFF, wave, lane, wr, h, r32, L, c, i, nb, e);
    };

    // ---- epilogue ------------------------------------------------------------------------
    // Called once per accumulator tile with compile-time (i, j), so every acc index stays a
    // constant (a runtime-indexed accumulator array goes to scratch: guide rule 20).
    // Every field of the problem is read ONCE into scalar registers and pinned there (an empty
    // asm makes the value opaque, so the compiler cannot re-materialise it as a kernarg load),
    // and the mode is dispatched once per tile to a body specialised at compile time.  The
    // generic form re-read the argument block after every store and branched on the mode per
    // element: an s_load round trip per element, ~20 us per 128 x 128 tile (profiles/r02*).
    auto epi = [&](const TileLoc& L, const f32x16& c, const int i, const int j)
                   __attribute__((always_inline)) {
        KProb& P = ka->prob[L.p];
        int mode = P.mode, Mv = P.M_valid, Mr = P.M, Nc = P.N, ksp = ka->ksplit[L.p];
        int kt = P.ct_blk;
        float scale = P.scale;
        const float* bias_p = P.bias;
        const float* Rp = P.R;
        const float* Pin = P.P_in;
        const unsigned short* Rbp = reinterpret_cast<const unsigned short*>(P.Rb);
        float* Cp = P.C;
        float* Pp = P.P;
        unsigned short* Cbp = reinterpret_cast<unsigned short*>(P.Cb);
        unsigned short* CbTp = reinterpret_cast<unsigned short*>(P.CbT);
        float* csp = P.colsum;
        float* lpp = P.loss_part;
        float* wsp = P.ws;
        int64_t ldr = P.ldr, ldpin = P.ldp_in, ldrb = P.ldrb, ldc = P.ldc, ldp = P.ldp,
                ldcb = P.ldcb, ldct = P.ldct;
        const int m0 = L.m0, n0 = L.n0;
        // (128 x 128 tiles keep the accumulator-layout stores: with the LDS path inlined four
        // times the compiler put 460 B per lane in scratch)
        if constexpr (!PERSIST && !(RM == 2 && RN == 2)) {
            // LDS-transposed path (see the note above epi): uniform eligibility test
            const int nb = n0 + wc * (BN / 2) + j * 32;        // first column of the block
            auto al = [](const void* p, int a) {
                return ((uintptr_t)p & (uintptr_t)(a - 1)) == 0;
            };
            bool ok = nb + 32 <= Nc;
            if (ksp > 1) {
                ok = ok && (Nc & 3) == 0 && al(wsp, 16);
            } else {
                ok = ok && (!Cp || (al(Cp, 16) && (ldc & 3) == 0)) &&
                     (!Pp || (al(Pp, 16) && (ldp & 3) == 0)) &&
                     (mode == LDM_GEMM_ACCUM || !Rp || (al(Rp, 16) && (ldr & 3) == 0)) &&
                     (!Pin || (al(Pin, 16) && (ldpin & 3) == 0)) &&
                     (!Cbp || (al(Cbp, 8) && (ldcb & 3) == 0)) &&
                     (!Rbp || (al(Rbp, 8) && (ldrb & 3) == 0)) && (!bias_p || al(bias_p, 16));
            }
            if (ok) {
                const EpiArgs ea = {mode, Mv, Mr, Nc, ksp, kt, scale, bias_p, Rp, Pin, Rbp, Cp,
                                    Pp, Cbp, CbTp, csp, lpp, wsp, ldr, ldpin, ldrb, ldc, ldp,
                                    ldcb, ldct};
                epi_lds(L, c, i, nb, ea);
                return;
            }
        }
        // accumulator-layout path: pin every field in SGPRs (see above; readfirstlane rather
        // than an empty "+s" asm, which the build rejected next to the LDS path)
        mode = pin_s(mode); Mv = pin_s(Mv); Mr = pin_s(Mr); Nc = pin_s(Nc); ksp = pin_s(ksp);
        kt = pin_s(kt); scale = pin_s(scale); bias_p = pin_s(bias_p); Rp = pin_s(Rp);
        Pin = pin_s(Pin); Rbp = pin_s(Rbp); Cp = pin_s(Cp); Pp = pin_s(Pp); Cbp = pin_s(Cbp);
        CbTp = pin_s(CbTp); csp = pin_s(csp); lpp = pin_s(lpp); wsp = pin_s(wsp);
        ldr = pin_s(ldr); ldpin = pin_s(ldpin); ldrb = pin_s(ldrb); ldc = pin_s(ldc);
        ldp = pin_s(ldp); ldcb = pin_s(ldcb); ldct = pin_s(ldct);
        const int rb = m0 + wr * (BM / 2) + i * 32;           // first row of this 32-row block
        const int n = n0 + wc * (BN / 2) + j * 32 + r32;
        const bool ncol = n < Nc;
        const int nn = ncol ? n : Nc - 1;
        auto row = [&](int v) { return rb + (v & 3) + 8 * (v >> 2) + 4 * h; };
        if (ksp > 1) {                                         // split-K: raw partial slab
            float* dst = wsp + (int64_t)L.slice * Mr * Nc;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int b = row(v);
                if (ncol && b < Mv) dst[(int64_t)b * Nc + n] = c[v];
            }
            return;
        }
        const float bias = bias_p ? bias_p[nn] : 0.f;
        auto body = [&](auto mc) {
            constexpr int MODE = decltype(mc)::value;
            constexpr bool X1R = MODE == LDM_GEMM_RESID_SILU || MODE == LDM_GEMM_ADD_R ||
                                 MODE == LDM_GEMM_DGRAD_SILU;
            constexpr bool X1C = MODE == LDM_GEMM_ACCUM;
            constexpr bool X2 = MODE == LDM_GEMM_DGRAD_SILU || MODE == LDM_GEMM_LOSS;
            constexpr bool XB = MODE == LDM_GEMM_RELU_BWD;
            // operands for all 16 rows in one batch (padding rows read row 0, a valid
            // address, and drop the value): no per-element load-use round trip
            float v1[16], v2[16];
            unsigned short vb[16];
            const bool has1 = X1C || (X1R && Rp != nullptr);
            const float* x1 = X1C ? Cp : Rp;
            const int64_t ld1 = X1C ? ldc : ldr;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int b = row(v);
                const int bb = (ncol && b < Mv) ? b : 0;
                v1[v] = 0.f;
                v2[v] = 0.f;
                vb[v] = 0;
                if constexpr (X1R || X1C) {
                    if (has1) v1[v] = x1[(int64_t)bb * ld1 + nn];
                }
                if constexpr (X2) v2[v] = Pin[(int64_t)bb * ldpin + nn];
                if constexpr (XB) vb[v] = Rbp[(int64_t)bb * ldrb + nn];
            }
            float out[16], pre_v[16], dh[16];
            float lsum = 0.f;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const bool live = ncol && row(v) < Mv;
                const float pre = c[v] + bias;
                pre_v[v] = pre;
                float o = pre;
                if constexpr (MODE == LDM_GEMM_SILU) o = silu(pre);
                if constexpr (MODE == LDM_GEMM_RESID_SILU) o = v1[v] + silu(pre);
                if constexpr (MODE == LDM_GEMM_RELU) o = fmaxf(pre, 0.f);
                if constexpr (MODE == LDM_GEMM_ACCUM || MODE == LDM_GEMM_ADD_R) o = v1[v] + pre;
                if constexpr (MODE == LDM_GEMM_DGRAD_SILU) {
                    dh[v] = v1[v] + pre;                       // v1 = 0 without R
                    o = dh[v] * silu_grad(v2[v]);
                }
                if constexpr (MODE == LDM_GEMM_LOSS) {
                    const float d = pre - v2[v];
                    lsum += live ? d * d : 0.f;
                    o = scale * d;
                }
                if constexpr (MODE == LDM_GEMM_RELU_BWD) {   // bf16 > 0: sign clear, not +0
                    const unsigned short u = vb[v];
                    o = (u != 0 && (u & 0x8000u) == 0) ? pre : 0.f;
                }
                out[v] = live ? o : 0.f;
            }
            // stores: one uniform branch per output, per-lane row predicates inside
            if (Cp) {
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const int b = row(v);
                    if (ncol && b < Mv)
                        Cp[(int64_t)b * ldc + n] = MODE == LDM_GEMM_DGRAD_SILU ? dh[v] : out[v];
                }
            }
            if constexpr (MODE == LDM_GEMM_SILU || MODE == LDM_GEMM_RESID_SILU) {
                if (Pp) {
#pragma unroll
                    for (int v = 0; v < 16; ++v) {
                        const int b = row(v);
                        if (ncol && b < Mv) Pp[(int64_t)b * ldp + n] = pre_v[v];
                    }
                }
            }
            if (Cbp) {
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const int b = row(v);
                    if (ncol && b < Mr)
                        Cbp[(int64_t)b * ldcb + n] =
                            (unsigned short)(pack2_bf16(out[v], 0.f) & 0xffffu);
                }
            }
            if (CbTp && ncol) {               // [n][b]: 4 consecutive rows per 8-byte store
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int b = rb + 8 * g + 4 * h;
                    if (b < Mr) {
                        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                        const u32x2 w = {pack2_bf16(out[4 * g], out[4 * g + 1]),
                                         pack2_bf16(out[4 * g + 2], out[4 * g + 3])};
                        const int64_t at = kt ? ((int64_t)(b / kt) * Nc + n) * kt + b % kt
                                              : (int64_t)n * ldct + b;
                        *reinterpret_cast<u32x2*>(CbTp + at) = w;
                    }
                }
            }
            if (csp) {                        // one partial per 32-row block and column
                float cs = 0.f;
#pragma unroll
                for (int v = 0; v < 16; ++v) cs += out[v];
                cs += __shfl_xor(cs, 32);
                if (h == 0 && ncol && rb < Mr) csp[(int64_t)(rb / 32) * Nc + n] = cs;
            }
            if constexpr (MODE == LDM_GEMM_LOSS) {
                if (lpp) {
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) lsum += __shfl_xor(lsum, o);
                    const int cb = n0 + wc * (BN / 2) + j * 32;     // first column of the block
                    if (lane == 0 && rb < Mr && cb < Nc)    // (a block wholly past N: no slot)
                        lpp[(int64_t)(rb / 32) * ((Nc + 31) / 32) + cb / 32] = lsum;
                }
            }
        };
        typedef std::integral_constant<int, LDM_GEMM_STORE> E0;
        switch (mode) {
            case LDM_GEMM_SILU: body(std::integral_constant<int, LDM_GEMM_SILU>{}); break;
            case LDM_GEMM_RESID_SILU:
                body(std::integral_constant<int, LDM_GEMM_RESID_SILU>{});
                break;
            case LDM_GEMM_RELU: body(std::integral_constant<int, LDM_GEMM_RELU>{}); break;
            case LDM_GEMM_ACCUM: body(std::integral_constant<int, LDM_GEMM_ACCUM>{}); break;
            case LDM_GEMM_DGRAD_SILU:
                body(std::integral_constant<int, LDM_GEMM_DGRAD_SILU>{});
                break;
            case LDM_GEMM_LOSS: body(std::integral_constant<int, LDM_GEMM_LOSS>{}); break;
            case LDM_GEMM_ADD_R: body(std::integral_constant<int, LDM_GEMM_ADD_R>{}); break;
            case LDM_GEMM_RELU_BWD:
                body(std::integral_constant<int, LDM_GEMM_RELU_BWD>{});
                break;
            default: body(E0{}); break;
        }
    };
        auto epilogue = [&](const TileLoc& L, bool do0, bool do1) {
        if (do0) {
            epi(L, acc[0][0], 0, 0);
            if constexpr (RN > 1) epi(L, acc[0][RN - 1], 0, 1);
        }
        if constexpr (RM > 1) {
            if (do1) {
                epi(L, acc[RM - 1][0], 1, 0);
                if constexpr (RN > 1) epi(L, acc[RM - 1][RN - 1], 1, 1);
            }
        }
    };

    if constexpr (PERSIST) {
        // ---- persistent walk: one continuous k-step stream over the workgroup's tiles -------
        // Every iteration issues one stage (a dummy re-issue once the tiles run out), so the
        // counted wait below is the same every time: this wave's pieces of the stage about to
        // be computed landed while SS-2 younger stages may still fly.  Epilogue stores also
        // count in vmcnt: the wait after an epilogue over-waits for them (never under-waits).
        for (int u = 0; u < SS - 1; ++u) issue();
        int tc = t0, kc = 0, qc = 0;
        TileLoc cl = locate<BM, BN>(ka, tc);
        int nkc = ka->nk[cl.p];
        for (;;) {
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((SS - 2) * G) : "memory");
            issue();
            compute(smem + (qc % STAGES) * STAGE_ELEMS);
            ++qc;
            if (++kc == nkc) {
                epilogue(cl, true, true);
                zero_acc();
                tc += tstep;
                if (tc >= tend) break;
                cl = locate<BM, BN>(ka, tc);
                nkc = ka->nk[cl.p];
                kc = 0;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // dummies land before LDS is freed
        return;
    } else {
    const TileLoc L0 = locate<BM, BN>(ka, t0);
    const int nk = ka->nk[L0.p];

    if constexpr (RS) {
        // register-staged double buffer: stage it+1 waits in VGPRs while stage it computes
        static_assert(KG == 1 && STAGES == 2, "register staging: 2 LDS buffers, one k-group");
        u32x4 ra[TileSrc<BM, NW, KB>::NP], rb[TileSrc<BN, NW, KB>::NP];
        il = L0;
        seg = 0;
        seat(0, L0.slice * nk);
        auto load = [&]() {
            if (seg_left == 0) seat(++seg, 0);
            srcA.load(ra);
            srcB.load(rb);
            --seg_left;
        };
        auto store = [&](int q) {
            unsigned short* st = smem + (q & 1) * STAGE_ELEMS;
            srcA.store(st, ra, wave, lane);
            srcB.store(st + A_ELEMS, rb, wave, lane);
        };
        load();
        store(0);
        if (nk > 1) load();
        __syncthreads();
        for (int it = 0; it < nk; ++it) {
            compute(smem + (it & 1) * STAGE_ELEMS);
            if (it + 1 < nk) {
                store(it + 1);
                if (it + 2 < nk) load();
            }
            __syncthreads();
        }
    } else {
    const int nks = (nk + KG - 1) / KG;                 // super-steps
    // issue() re-issues a dummy past the tile's last k-step (keeps vmcnt arithmetic uniform)
    for (int ss = 0; ss < SS - 1; ++ss)
        if (ss < nks)
#pragma unroll
            for (int u = 0; u < KG; ++u) issue();
    gs.mark(1);

    for (int it = 0; it < nks; ++it) {
        // RAW: this wave's pieces of super-stage it landed (SS-2 younger ones may still fly),
        // then the barrier makes every wave's pieces visible and retires every wave's reads of
        // super-stage it-1, whose slots the issue below refills (WAR).
        if (it + SS - 2 < nks)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((SS - 2) * KG * G) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (GEMM_STAMP && it == 0) gs.mark(2);
        if (it + SS - 1 < nks)
#pragma unroll
            for (int u = 0; u < KG; ++u) issue();
        const int q = it * KG + grp;
        if (KG == 1 || q < nk) compute(smem + (q % STAGES) * STAGE_ELEMS);
    }
    }

    // ---- k-groups: sum the two partial tiles through LDS ---------------------------------
    // RM == 2: group g keeps accumulator row-block i = g and receives the other group's;
    // RM == 1: group 0 receives everything and runs the whole epilogue.
    if constexpr (KG == 2) {
        __syncthreads();                                // every DMA landed, every read done
        float* red = reinterpret_cast<float*>(smem);    // [4 waves][RN][16][64] per block
        constexpr int BLK = 4 * RN * 16 * 64;
#pragma unroll
        for (int i = 0; i < RM; ++i) {
            const int owner = RM == 2 ? i : 0;
            if (grp != owner) {
#pragma unroll
                for (int j = 0; j < RN; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v)
                        red[i * BLK + ((w4 * RN + j) * 16 + v) * 64 + lane] = acc[i][j][v];
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < RM; ++i) {
            const int owner = RM == 2 ? i : 0;
            if (grp == owner) {
#pragma unroll
                for (int j = 0; j < RN; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v)
                        acc[i][j][v] += red[i * BLK + ((w4 * RN + j) * 16 + v) * 64 + lane];
            }
        }
        if (RM == 1 && grp != 0) return;
    }
    gs.mark(3);
    // the epilogue's LDS tiles overwrite ring slots other waves may still be reading
    if constexpr (KG == 1 && !RS) __syncthreads();
    epilogue(L0, KG == 1 || RM == 1 || grp == 0, KG == 1 || grp == 1);
    if (GEMM_STAMP && !RS) {
        gs.mark(4);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gs.mark(5);
        gs.flush(gridDim.x, tot_all);
    }
    }
}

// Split-K combine: C[m][n] = (ACCUM ? C[m][n] : 0) + sum_s ws[s][m][n] + bias[n], slices summed
// in order 0..S-1 (deterministic).  4 consecutive columns per thread.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(ldm_gemm_prob_t P, int S) {
    const int64_t n4 = (P.N + 3) / 4;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)P.M_valid * n4) return;
    const int m = (int)(i / n4), c0 = (int)(i - (int64_t)m * n4) * 4;
    const int64_t slab = (int64_t)P.M * P.N;
    float v[4];
    int nc = min(4, P.N - c0);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = 0.f;
    for (int s = 0; s < S; ++s) {
        const float* src = P.ws + s * slab + (int64_t)m * P.N + c0;
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (c < nc) v[c] += src[c];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (c >= nc) break;
        float o = v[c] + (P.bias ? P.bias[c0 + c] : 0.f);
        float* dst = P.C + (int64_t)m * P.ldc + c0 + c;
        if (P.mode == LDM_GEMM_ACCUM) o = *dst + o;
        *dst = o;
    }
}

template <int BM, int BN, int STAGES, int KG = 1, bool RS = false, bool PERSIST = false,
          int KB = 64>
int launch_gemm(const ldm_gemm_args_t& a, hipStream_t s) {
    auto* k = &gemm_bf16_kernel<BM, BN, STAGES, KG, RS, PERSIST, KB>;
    GemmKArgs ka;
    memset(&ka, 0, sizeof(ka));
    ka.n_prob = a.n_prob;
    int acc = 0;
    for (int p = 0; p < LDM_GEMM_MAX_PROBS; ++p) {
        if (p < a.n_prob) {
            const ldm_gemm_prob_t& P = a.prob[p];
            ka.prob[p] = P;
            ka.first[p] = acc;
            ka.tiles_m[p] = (P.M + BM - 1) / BM;
            ka.tiles_n[p] = (P.N + BN - 1) / BN;
            ka.ksplit[p] = P.k_split > 1 ? P.k_split : 1;
            int nk = 0;
            for (int g = 0; g < P.n_seg; ++g) nk += P.seg[g].K / KB;
            ka.nk[p] = nk / ka.ksplit[p];
            acc += ka.tiles_m[p] * ka.tiles_n[p] * ka.ksplit[p];
        } else {
            ka.first[p] = 0x7fffffff;
        }
    }
    ka.total = acc;
    constexpr int lds = STAGES * (BM + BN) * KB * 2;
    // once per (template instance, device), thread-safe: the LDS attribute and, persistent,
    // the resident-workgroup cap of THIS device (was once per process)
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    static int grid_cap[kMaxDev];
    static int init_err[kMaxDev];
    int dev = 0;
    LDM_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDev, LDM_EINVAL,
                "ldm_gemm_bf16: no current device");
    std::call_once(once[dev], [&] {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        int per_cu = 0, cus = 0;
        if (e == hipSuccess && PERSIST) {
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per_cu, reinterpret_cast<const void*>(k), 256 * KG, lds);
            if (e == hipSuccess)
                e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            if (e == hipSuccess && per_cu < 1) e = hipErrorInvalidConfiguration;
        }
        init_err[dev] = (int)e;
        grid_cap[dev] = PERSIST ? per_cu * cus : 1;
    });
    LDM_REQUIRE(init_err[dev] == 0, init_err[dev],
                "ldm_gemm_bf16: kernel attribute / persistent occupancy query failed: %s",
                hipGetErrorString((hipError_t)init_err[dev]));
    const int grid = PERSIST ? std::min(acc, grid_cap[dev]) : acc;
    hipLaunchKernelGGL(k, dim3(grid), dim3(256 * KG), lds, s, ka);
    LDM_TRY(launch_status("ldm_gemm_bf16"));
    for (int p = 0; p < a.n_prob; ++p) {
        const ldm_gemm_prob_t& P = a.prob[p];
        if (ka.ksplit[p] <= 1 || P.M_valid == 0) continue;
        const int64_t n = (int64_t)P.M_valid * ((P.N + 3) / 4);
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                           s, P, ka.ksplit[p]);
        LDM_TRY(launch_status("ldm_gemm_bf16 (split-K combine)"));
    }
    return 0;
}

}  // namespace

int gemm_tiles(const ldm_gemm_args_t& a, int bm, int bn) {
    int total = 0;
    for (int p = 0; p < a.n_prob; ++p)
        total += ((a.prob[p].M + bm - 1) / bm) * ((a.prob[p].N + bn - 1) / bn) *
                 (a.prob[p].k_split > 1 ? a.prob[p].k_split : 1);
    return total;
}

int env_int(const char* name) { return dev_knob(name, 0); }

// The tile ldm_gemm_bf16 runs a launch on (a.tile, or the automatic rule below).  Exposed so the
// persistent training step (train_dag.hip) can reproduce each launch's k-group split.
int gemm_tile_choice(const ldm_gemm_args_t& a) {
    const int forced = dev_knob("LDM_GEMM_TILE", 0);
    int tile = a.tile;
    if (tile == 0) {
        bool k128 = true;
        for (int p = 0; p < a.n_prob; ++p)
            for (int g = 0; g < a.prob[p].n_seg; ++g) k128 = k128 && a.prob[p].seg[g].K % 128 == 0;
        const int t64 = gemm_tiles(a, 64, 64);
        // tuning knobs per launch size class (tile counts at 64 x 64): <= 256, <= 512, < 2048,
        // >= 2048
        const int by_size[4] = {env_int("LDM_GEMM_TILE_SMALL"),
                                       env_int("LDM_GEMM_TILE_MID"), env_int("LDM_GEMM_TILE_BIG"),
                                       env_int("LDM_GEMM_TILE_HUGE")};
        const int cls = t64 <= 256 ? 0 : t64 <= 512 ? 1 : t64 < 2048 ? 2 : 3;
        tile = forced ? forced : by_size[cls] ? by_size[cls] : t64 >= 2048 ? 15
             : (k128 && t64 <= 256) ? 24 : 4;
    }
    return tile;
}

// 0 for a tile on one k-group; for the two-k-group tiles (KG = 2: 5, 6, 7, 11 with 64-deep
// stages, 24 with 128-deep ones) the number of 64-deep k-steps a group takes in a row: group g
// sums the k-steps q with (q / period) % 2 == g and the tile's result is group 0's sum + group
// 1's (the reduction above) -- what train_dag.hip reproduces to stay bit-identical.
int gemm_tile_kgroup_period(int tile) {
    switch (tile) {
        case 5: case 6: case 7: case 11: return 1;
        case 24: return 2;
        default: return 0;
    }
}

int gemm_bf16(const ldm_gemm_args_t& a, hipStream_t s) {
    LDM_REQUIRE(a.n_prob >= 1 && a.n_prob <= LDM_GEMM_MAX_PROBS, LDM_EINVAL,
                "ldm_gemm_bf16: n_prob %d", a.n_prob);
    for (int p = 0; p < a.n_prob; ++p) {
        const ldm_gemm_prob_t& P = a.prob[p];
        LDM_REQUIRE(P.M >= 1 && P.N >= 1 && P.M_valid >= 0 && P.M_valid <= P.M &&
                        P.n_seg >= 1 && P.n_seg <= LDM_GEMM_MAX_SEGS,
                    LDM_EINVAL, "ldm_gemm_bf16: problem %d: M=%d N=%d M_valid=%d n_seg=%d", p,
                    P.M, P.N, P.M_valid, P.n_seg);
        for (int s = 0; s < P.n_seg; ++s) {
            const ldm_gemm_seg_t& S = P.seg[s];
            LDM_REQUIRE(S.A && S.B && S.K > 0 && S.K % kBK == 0, LDM_EINVAL,
                        "ldm_gemm_bf16: problem %d seg %d: K=%d must be a positive multiple of 64",
                        p, s, S.K);
            const int kmin = P.k_split > 1 && P.slice_a ? S.K / P.k_split : S.K;
            LDM_REQUIRE(LDM_ALIGNED(S.A, 16) && LDM_ALIGNED(S.B, 16) && S.lda % 8 == 0 &&
                            S.ldb % 8 == 0 && S.lda >= kmin && S.ldb >= kmin,
                        LDM_EALIGN, "ldm_gemm_bf16: problem %d seg %d: operands must be 16-B "
                        "aligned with row strides a multiple of 8 elements", p, s);
        }
        LDM_REQUIRE(P.mode >= LDM_GEMM_STORE && P.mode <= LDM_GEMM_RELU_BWD, LDM_EINVAL,
                    "ldm_gemm_bf16: problem %d: mode %d", p, P.mode);
        LDM_REQUIRE(P.mode != LDM_GEMM_RELU_BWD || P.Rb, LDM_EINVAL,
                    "ldm_gemm_bf16: problem %d: RELU_BWD needs Rb", p);
        if (P.k_split > 1 && P.slice_a) {
            LDM_REQUIRE(P.slice_b && P.seg[0].lda >= P.seg[0].K / P.k_split &&
                            P.seg[0].ldb >= P.seg[0].K / P.k_split,
                        LDM_EINVAL, "ldm_gemm_bf16: problem %d: sliced split-K needs both "
                        "slice strides and row strides >= K / k_split", p);
        }
        if (P.k_split > 1) {
            LDM_REQUIRE(P.n_seg == 1 && P.seg[0].K % (2 * kBK * P.k_split) == 0 && P.ws && P.C &&
                            (P.mode == LDM_GEMM_STORE || P.mode == LDM_GEMM_ACCUM) && !P.Cb &&
                            !P.CbT && !P.colsum && !P.P,
                        LDM_EINVAL, "ldm_gemm_bf16: problem %d: split-K %d needs one segment, "
                        "K a multiple of 128 * k_split, ws, C, mode STORE/ACCUM and no other "
                        "output", p, P.k_split);
        }
        const bool needR = P.mode == LDM_GEMM_RESID_SILU || P.mode == LDM_GEMM_ADD_R;
        const bool needPin = P.mode == LDM_GEMM_DGRAD_SILU || P.mode == LDM_GEMM_LOSS;
        LDM_REQUIRE((!needR || P.R) && (!needPin || P.P_in) &&
                        (P.mode != LDM_GEMM_ACCUM || P.C),
                    LDM_EINVAL, "ldm_gemm_bf16: problem %d: mode %d operand missing", p, P.mode);
        LDM_REQUIRE(!P.CbT || (LDM_ALIGNED(P.CbT, 8) && P.ldct % 4 == 0 && P.M % 4 == 0 &&
                               P.ct_blk % 4 == 0 && P.ct_blk >= 0),
                    LDM_EALIGN, "ldm_gemm_bf16: problem %d: transposed output needs 8-B "
                    "alignment, ldct and M multiples of 4", p);
    }
    // Automatic tile (profiles/r02k, gemm_bench.py; LDM_GEMM_TILE replaces it for tuning):
    //  * >= 2048 64 x 64 tiles (C19's 1M-row products): 128 x 64, register-staged (1.10 ms for
    //    1M x 512 x 512, 64 x 64 DMA 1.39 ms; larger tiles cut the per-CU operand bytes);
    //  * <= 256 tiles with every K a multiple of 128 (config 2's forward): 128-deep stages on
    //    8 waves in two k-groups with a 4-deep ring (11.1 us for the block GEMM 1000 x 1024 x
    //    2048);
    //  * else 64 x 64 on a 3-deep 64-k ring (48 KiB: 3 workgroups per CU, so config 2's
    //    768-tile backward launches run in ONE wave of workgroups; the 128-deep 2-stage tile at
    //    2 per CU left half a wave: the step 0.348 -> 0.317-0.326 ms, scripts/rounds/train_tiles2.sh,
    //    profiles/r02h/train_tiles2.log).
    const int tile = gemm_tile_choice(a);
    if (tile >= 20) {                          // 128-deep stages: every K a multiple of 128
        for (int p = 0; p < a.n_prob; ++p)
            for (int g = 0; g < a.prob[p].n_seg; ++g)
                LDM_REQUIRE(a.prob[p].seg[g].K % (2 * kBK) == 0, LDM_EINVAL,
                            "ldm_gemm_bf16: tile %d needs every K a multiple of 128", tile);
    }
    switch (tile) {
        case 1: return launch_gemm<64, 64, 4>(a, s);
        case 2: return launch_gemm<128, 64, 4>(a, s);
        case 3: return launch_gemm<128, 128, 3>(a, s);
        case 4: return launch_gemm<64, 64, 3>(a, s);
        case 5: return launch_gemm<64, 64, 6, 2>(a, s);
        case 6: return launch_gemm<128, 128, 4, 2>(a, s);
        case 7: return launch_gemm<128, 64, 6, 2>(a, s);
        case 8: return launch_gemm<64, 64, 8>(a, s);
        case 9: return launch_gemm<128, 64, 5>(a, s);
        case 10: return launch_gemm<64, 64, 2>(a, s);
        case 11: return launch_gemm<64, 64, 4, 2>(a, s);
        case 12: return launch_gemm<128, 64, 3>(a, s);
        case 13: return launch_gemm<64, 64, 2, 1, true>(a, s);
        case 14: return launch_gemm<128, 128, 2, 1, true>(a, s);
        case 15: return launch_gemm<128, 64, 2, 1, true>(a, s);
        case 16: return launch_gemm<128, 128, 4, 1, false, true>(a, s);
        case 17: return launch_gemm<128, 128, 2, 1, false, true>(a, s);
        case 18: return launch_gemm<64, 64, 3, 1, false, true>(a, s);
        case 20: return launch_gemm<64, 64, 2, 1, false, false, 128>(a, s);
        case 21: return launch_gemm<64, 64, 3, 1, false, false, 128>(a, s);
        case 22: return launch_gemm<128, 64, 2, 1, false, false, 128>(a, s);
        case 23: return launch_gemm<128, 128, 2, 1, false, false, 128>(a, s);
        case 24: return launch_gemm<64, 64, 4, 2, false, false, 128>(a, s);
        case 25: return launch_gemm<64, 64, 2, 1, false, true, 128>(a, s);
        case 26: return launch_gemm<128, 128, 2, 1, false, true, 128>(a, s);
        case 27: return launch_gemm<64, 64, 2, 1, true, false, 128>(a, s);
        case 28: return launch_gemm<128, 64, 2, 1, true, false, 128>(a, s);
        default: break;
    }
    set_error("ldm_gemm_bf16: tile %d", tile);
    return LDM_EINVAL;
}

}  // namespace ldm

extern "C" int ldm_gemm_bf16(const ldm_gemm_args_t* a, ldm_stream_t s) {
    LDM_REQUIRE(a != nullptr, LDM_EINVAL, "ldm_gemm_bf16: null args");
    return ldm::gemm_bf16(*a, (hipStream_t)s);
}

#if GEMM_STAMP
// diagnostic build only: the GEMM stamp ring (256 x 8: six s_memrealtime marks, grid, tiles)
extern "C" int ldm_dev_gemm_stamps(uint64_t* host, unsigned* n) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(ldm::g_gemm_stamp), sizeof(ldm::g_gemm_stamp)) !=
            hipSuccess ||
        hipMemcpyFromSymbol(n, HIP_SYMBOL(ldm::g_gemm_stamp_n), sizeof(unsigned)) != hipSuccess)
        return -1;
    return 0;
}
#endif
