// C17: the 1D-UNet denoiser's fused conv1d on MI355X (gfx950), DESIGN.md §9.
//
// One kernel, ldm_conv1d, runs every conv of the UNet as an implicit GEMM on the matrix cores
//   Y[b][co][l] = sum_seg sum_{k,ci} W(co,ci,k) act(X[b][ci][src(l,k)]) + biases (+ R)
// with the block structure fused into its operands and epilogue:
//   * SiLU of the input is applied while staging the input window (no separate pass);
//   * a channel concat [u || s] is two segments of one weight (no concat copy);
//   * the ResBlock's 1x1 shortcut conv is an extra k=1 segment of its second conv, and an
//     identity shortcut is the residual operand R;
//   * the timestep-embedding projection enters as a per-(b, co) bias (a [T][Cout] table row
//     for the batch-uniform t of sampling);
//   * nearest-2x upsampling is an index map of the staging loads (LDM_CONV_UP2);
//   * the output conv carries the DDPM reverse step (A8) in its epilogue.
//
// Arithmetic: v_mfma_f32_16x16x4_f32 -- fp32 activations and fp32 (or bf16-stored) weights,
// fp32 products and accumulation, so the bf16 path differs from fp32 only by its weights.
// The UNet at the sampling batch is a chain of small, latency-bound launches, so the design
// minimises per-launch latency rather than maximising MFMA occupancy:
//   * a workgroup (4 waves) owns 16 output channels x TP positions of one shape (TP = 16 for
//     small grids, 32/64 for large ones); the 4 waves split the contraction (tap x channel
//     chunks of 16) and their partial tiles are summed in a fixed order through LDS, so the
//     result is deterministic;
//   * every input window and weight slice of the launch is staged in LDS in ONE round trip
//     (the direct staging below: every segment's loads issued before any LDS store; the
//     generic staging, for other shapes, one round trip per segment part), then one barrier,
//     then the MFMA loop runs from LDS only;
//   * LDS layouts put each lane's operands for 4 consecutive MFMAs in one ds_read_b128:
//     channels are permuted inside every group of 16 (perm16) on staging, and the weights
//     arrive already permuted from the host packing (ldm_sdf/ops.py pack_conv_weight).
#include "ldm_internal.h"
#include "ddpm_common.h"

#include <string.h>

#include <type_traits>
#include <vector>
#include <algorithm>

// Diagnostic build only (-DUNET_STAMP=1, scripts/stamp_conv.py): workgroup (0, 0, 0) of every
// ldm_conv1d launch stamps s_memrealtime (100 MHz) at its phase boundaries (StampRegs).
#ifndef UNET_STAMP
#define UNET_STAMP 0
#endif

namespace ldm {
namespace {

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__host__ __device__ constexpr int round16(int c) { return (c + 15) & ~15; }
// Position of channel ci inside its 16-group so that lane group g reads channels
// 16c + 4m + g (m = 0..3: four consecutive MFMAs) as one 16-byte vector.
__host__ __device__ constexpr int perm16(int ci) {
    return (ci & ~15) | ((ci & 3) << 2) | ((ci >> 2) & 3);
}

// LDS row pitches (floats) of the staged operands.  The contraction's ds_read_b128 fragment
// reads take 16 rows (lanes c16 = 0..15) x four lane quarters g at +4 floats; the instruction
// serves lanes in groups of 16 (MI355X guide, LDS table: {0-3,12-15,20-27}, ...), which meet
// distinct 16-byte bank quads exactly when the row pitch is 2 mod 4 quads -- the quarters then
// fall on the even and the odd quads.  The round-4 pitch (+4 floats: 1 mod 4) put two lanes of
// every group on one quad (SQ_LDS_BANK_CONFLICT 38-50 % of LDS-active cycles, profiles/r04p).
// A stride-2 conv reads every second window row, so its window keeps the odd pitch.
__host__ __device__ constexpr int xpitch(int cinp, int stride) {
    return cinp + (stride == 1 ? 8 : 4);
}
__host__ __device__ constexpr int wpitch(int ksize, int cinp) { return ksize * cinp + 8; }

struct SegPlan {
    int cinp;   // channels rounded up to 16
    int win;    // input window (positions) of one tile
    int xoff;   // LDS float offset of the window  [win][xpitch(cinp, stride)]
    int woff;   // LDS float offset of the weights [16][wpitch(ksize, cinp)]
    int ch0;    // first contraction chunk (16 channels x one tap) of this segment
    // the launch kernel's direct staging (fast_* below; make_plan): every index a shift or mask
    int lgv;    // log2 of the 16-byte weight vectors per (row, tap): cinp / (16 / sizeof(TW))
    int nw;     // weight vectors of the tile: 16 rows x ksize taps x (1 << lgv)
    int lgng;   // log2 of the 4-position source groups staged per channel (>= the window's)
    int nx;     // window items (4 channels x 4 positions each): cinp / 4 << lgng
    // the contraction's geometry packed for the launch kernel (FastGeo): ch0 | ksize << 12 |
    // (stride - 1) << 15 | cinp << 16, and woff | xoff << 16
    int geo0, geo1;
};
struct ConvPlan {
    SegPlan s[LDM_CONV_MAX_SEGS];
    int nchunks;
    int lds_floats;
    int fast;         // every segment fits the direct staging (make_plan)
};

// The device code reads a call's arguments and plan through the CONSTANT address space (the
// kernarg segment), so every field is a scalar load into SGPRs; through a generic pointer each
// field was a vector load with its own memory wait (15.7 us per conv in the round-3 one-launch
// loop, since retired: DESIGN.md §9).
#define LDM_KC __attribute__((address_space(4)))
typedef const LDM_KC ldm_conv1d_args_t KConv;
typedef const LDM_KC ldm_conv1d_seg_t KSeg;
typedef const LDM_KC SegPlan KSegPlan;
typedef const LDM_KC ConvPlan KPlan;

// Staging issues every load of a segment before the first LDS store (one global round trip),
// branch-free: out-of-range slots load a clamped in-bounds address and select 0; their stores
// are skipped (exec-masked: a store needs no wait where the branch rejoins, and a common scratch
// address made the idle lanes' stores one LDS bank-conflict chain).  The slot count NB is picked per segment from the
// real item count (4 / 8 / 16 / 32), so a small segment does not pay a 32-slot unroll.
// SiLU of a staged input: x * rcp(1 + 2^(-x log2 e)) on the transcendental unit (a few
// instructions; the IEEE expf + division form was the dominant cost of staging, which is
// VALU-latency-bound at one wave per SIMD).  Within 2 ulp of x / (1 + e^-x); the oracle
// tolerances of DESIGN.md §9 hold with it.
__device__ __forceinline__ float silu_stage(float x) {
    return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}

// The input window of one segment, [win][perm16(ci)] (pitch xpitch), flat over (ci, j)
// with j fastest: thread tid stages items tid, tid + 256, ... with (ci, j) advanced
// incrementally (no per-item division), every load of a pass issued before its LDS stores
// (one global round trip per pass), branch-free (clamped address + select).  Channels
// C..cinp-1 and positions outside [0, Lsrc) stage zeros.
template <int NB>
__device__ __forceinline__ void stage_x_nb(float* __restrict__ xs,
                                           KSeg& s, const float* Xs, KSegPlan& p, int b,
                                           int pos0) {
    const int tid = threadIdx.x;
    const bool up2 = s.mode == LDM_CONV_UP2;
    const int Lsrc = up2 ? 2 * s.L_in : s.L_in;
    const int pstart = pos0 * s.stride - s.pad;
    const float* X = Xs + (int64_t)b * s.C * s.L_in;
    const int win = p.win, cinp = p.cinp, C = s.C, L_in = s.L_in, ld = xpitch(cinp, s.stride);
    const bool act = s.silu_in != 0;
    const int dq = 256 / win, dr = 256 - dq * win;    // per-item advance of (ci, j); win < 256
    int ci = tid / win, j = tid - ci * win;
    const int nitem = cinp * win;
    for (int base = 0; base < nitem; base += 256 * NB) {
        float v[NB];
        int dst[NB];
        uint64_t okm = 0;                    // item u's value is a real input (else zero)
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int pp = pstart + j;
            const bool in = ci < cinp;
            const bool ok = ci < C && pp >= 0 && pp < Lsrc;
            const int src = ok ? ci * L_in + (up2 ? (pp >> 1) : pp) : 0;
            v[u] = *(X + src);      // consumed only in the store pass below
            okm |= (uint64_t)ok << u;
            dst[u] = in ? j * ld + perm16(ci) : -1;
            // branch-free advance: a divergent branch here made the compiler drain every load
            // issued so far (vmcnt(0)) at its join
            j += dr;
            const int wrap = j >= win ? 1 : 0;
            j -= wrap * win;
            ci += dq + wrap;
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            if (dst[u] < 0) continue;        // exec-masked store (see fast_w_store)
            const float x = (okm >> u) & 1 ? v[u] : 0.f;
            xs[dst[u]] = act ? silu_stage(x) : x;
        }
    }
}

// The same window from 16-byte loads (rows of L_in % 4 == 0 floats, 16-byte aligned): item =
// (channel ci, 4-position source group g) with the groups aligned in the source row, so the
// address and index arithmetic is paid once per 4 elements (the scalar form above was
// VALU-bound at ~38 instructions per element, one wave per SIMD).  Raw buffer loads over the
// shape's [C][L_in] block: channels ci >= C fall outside it and read 0; positions outside
// [0, L_in) are masked per element.  UP2 writes every source element to its two window
// positions.
template <int NB>
__device__ __forceinline__ void stage_x_vec_nb(float* __restrict__ xs,
                                               KSeg& s, const float* Xs, KSegPlan& p, int b,
                                               int pos0) {
    const int tid = threadIdx.x;
    const bool up2 = s.mode == LDM_CONV_UP2;
    const int pstart = pos0 * s.stride - s.pad;               // window origin (>= -3)
    const int win = p.win, cinp = p.cinp, L_in = s.L_in, ld = xpitch(cinp, s.stride);
    const bool act = s.silu_in != 0;
    const int s0 = up2 ? (pstart >> 1) : pstart;               // floor: arithmetic shift
    const int s1 = up2 ? ((pstart + win - 1) >> 1) : pstart + win - 1;
    const int a0 = s0 & ~3;
    const int ng = ((s1 - a0) >> 2) + 1;                       // <= 34 < 256
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(Xs) + (int64_t)b * s.C * L_in, (short)0, s.C * L_in * 4,
        0x00020000);
    const int dq = 256 / ng, dr = 256 - dq * ng;
    int ci = tid / ng, g = tid - ci * ng;
    const int nitem = cinp * ng;
    for (int base = 0; base < nitem; base += 256 * NB) {
        f32x4 v[NB];
        int cg[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int off = ci * L_in + a0 + 4 * g;            // < 0 only for ci = 0: OOB -> 0
            v[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rs, (uint32_t)off * 4u, 0, 0));
            cg[u] = ci < cinp ? (ci << 8) | g : -1;
            g += dr;
            const int wrap = g >= ng ? 1 : 0;
            g -= wrap * ng;
            ci += dq + wrap;
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int c = cg[u] >> 8, sp0 = a0 + 4 * (cg[u] & 0xff);
            const int pc = perm16(c);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int sp = sp0 + e;
                const float x0 = (unsigned)sp < (unsigned)L_in ? v[u][e] : 0.f;
                const float y = act ? silu_stage(x0) : x0;
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    if (r == 1 && !up2) break;
                    const int j = (up2 ? 2 * sp + r : sp) - pstart;
                    const bool in = cg[u] >= 0 && (unsigned)j < (unsigned)win;
                    if (in) xs[j * ld + pc] = y;   // exec-masked store (see fast_w_store)
                }
            }
        }
    }
}

__device__ __forceinline__ void stage_x(float* xs, KSeg& s, const float* X,
                                        KSegPlan& p, int b, int pos0) {
    if ((s.L_in & 3) == 0 && ((uintptr_t)X & 15) == 0) {
        const int ng = (p.win + 6) / 4 + 2;               // bound of the source groups per row
        const int n = (p.cinp * ng + 255) / 256;
        if (n <= 2) stage_x_vec_nb<2>(xs, s, X, p, b, pos0);
        else if (n <= 5) stage_x_vec_nb<5>(xs, s, X, p, b, pos0);
        else if (n <= 10) stage_x_vec_nb<10>(xs, s, X, p, b, pos0);
        else stage_x_vec_nb<18>(xs, s, X, p, b, pos0);
        return;
    }
    const int n = (p.cinp * p.win + 255) / 256;      // items per thread
    if (n <= 4) stage_x_nb<4>(xs, s, X, p, b, pos0);
    else if (n <= 9) stage_x_nb<9>(xs, s, X, p, b, pos0);
    else if (n <= 17) stage_x_nb<17>(xs, s, X, p, b, pos0);
    else stage_x_nb<34>(xs, s, X, p, b, pos0);
}

// Weights: 16-byte vector loads along a packed row (4 fp32 or 8 bf16 channels per load).
// Item it (< nitem = 16 rows x taps x cinp / EPV) -> (co, tap k, element e) of the LDS row.
template <typename TW>
__device__ __forceinline__ void w_item(int it, int per_row, int nvec, int& co, int& k, int& e) {
    constexpr int EPV = 16 / sizeof(TW);
    co = it / per_row;
    const int r = it - co * per_row;
    k = r / nvec;
    e = (r - k * nvec) * EPV;
}

template <typename TW, int NB>
__device__ __forceinline__ void w_load(u32x4 (&v)[NB], KSeg& s, KSegPlan& p, int co0, int base) {
    constexpr int EPV = 16 / sizeof(TW);
    const int nvec = p.cinp / EPV, per_row = s.ksize * nvec, nitem = 16 * per_row;
    const char* W = reinterpret_cast<const char*>(s.W);
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int it = base + u * 256 + (int)threadIdx.x;
        int co, k, e;
        w_item<TW>(it < nitem ? it : 0, per_row, nvec, co, k, e);
        const int64_t gi = (int64_t)(co0 + co) * s.ldw + (int64_t)k * s.kstride + e;
        v[u] = *reinterpret_cast<const u32x4*>(W + gi * (int64_t)sizeof(TW));
    }
}

template <typename TW, int NB>
__device__ __forceinline__ void w_store(const u32x4 (&v)[NB], float* __restrict__ ws, KSeg& s,
                                        KSegPlan& p, int base) {
    constexpr int EPV = 16 / sizeof(TW);
    const int nvec = p.cinp / EPV, per_row = s.ksize * nvec, nitem = 16 * per_row;
    const int ld = wpitch(s.ksize, p.cinp);
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int it = base + u * 256 + (int)threadIdx.x;
        if (it >= nitem) continue;
        int co, k, e;
        w_item<TW>(it, per_row, nvec, co, k, e);
        float* d = ws + co * ld + k * p.cinp + e;
        if constexpr (sizeof(TW) == 2) {
            const u32x4 w = v[u];
            *reinterpret_cast<f32x4*>(d) = f32x4{
                __builtin_bit_cast(float, w[0] << 16), __builtin_bit_cast(float, w[0] & 0xffff0000u),
                __builtin_bit_cast(float, w[1] << 16), __builtin_bit_cast(float, w[1] & 0xffff0000u)};
            *reinterpret_cast<f32x4*>(d + 4) = f32x4{
                __builtin_bit_cast(float, w[2] << 16), __builtin_bit_cast(float, w[2] & 0xffff0000u),
                __builtin_bit_cast(float, w[3] << 16), __builtin_bit_cast(float, w[3] & 0xffff0000u)};
        } else {
            *reinterpret_cast<u32x4*>(d) = v[u];
        }
    }
}

template <typename TW, int NB>
__device__ __forceinline__ void stage_w_nb(float* __restrict__ ws, KSeg& s, KSegPlan& p,
                                           int co0) {
    const int nitem = 16 * s.ksize * (p.cinp / (16 / (int)sizeof(TW)));
    for (int base = 0; base < nitem; base += 256 * NB) {
        u32x4 v[NB];
        w_load<TW, NB>(v, s, p, co0, base);
        w_store<TW, NB>(v, ws, s, p, base);
    }
}

template <typename TW>
__device__ __forceinline__ void stage_w(float* ws, KSeg& s, KSegPlan& p,
                                        int co0) {
    const int n = (16 * s.ksize * (p.cinp / (16 / (int)sizeof(TW))) + 255) / 256;
    if (n <= 1) stage_w_nb<TW, 1>(ws, s, p, co0);
    else if (n <= 2) stage_w_nb<TW, 2>(ws, s, p, co0);
    else if (n <= 4) stage_w_nb<TW, 4>(ws, s, p, co0);
    else stage_w_nb<TW, 8>(ws, s, p, co0);
}

// The epilogue-side operands of one conv call: seg[0]'s input, the per-channel bias row, and
// the output / x_t / noise / t of the DDPM epilogue.
struct ConvIO {
    const float* x0;
    const float* cbias;
    float* Y;
    const float* xlat;
    const float* z;
    int t;
};

__device__ __forceinline__ ConvIO conv_io(KConv& a) {
    return {a.seg[0].X, a.cbias, a.Y, a.xlat, a.z, a.t};
}

// Diagnostic stamps (UNET_STAMP builds only; every mark compiles away otherwise): workgroup
// (0, 0, 0) keeps s_memrealtime marks in registers and writes them at the kernel's end, so the
// slot's atomic and the stores stay out of the timed path.
struct StampRegs {
    bool on;
    uint64_t t[16];
    __device__ __forceinline__ void mark(int k) {
        if (UNET_STAMP && on) t[k] = __builtin_amdgcn_s_memrealtime();
    }
};

// The epilogue's own operands (biases, residual, x_t / noise of the DDPM step, the step's
// schedule coefficients) for thread tid's outputs o = tid + 256 k of the tile, ISSUED early so
// their latency hides under other work and consumed only in conv_finish: every load is
// unconditional (an absent operand reads a valid dummy address and is zeroed there), because a
// load under a branch, or a sum right after the loads, made the compiler wait for every load in
// flight (vmcnt(0)) -- three serial round trips in the launch kernel's staging.
// Out-of-tile outputs read index 0 (valid) and are not stored.
template <int TP>
struct EpiOps {
    static constexpr int NE = TP / 16;           // 16 x TP outputs over 256 threads
    float b1[NE], b2[NE], b3[NE], r[NE], x[NE], z[NE];
    float c1, c2, sg;
};

template <int TP>
__device__ __forceinline__ void epi_load(EpiOps<TP>& e, KConv& a, const ConvIO& io, int pos0,
                                         int co0, int b) {
    const int tid = threadIdx.x;
    const bool ddpm = a.epi == LDM_CONV_EPI_DDPM;
    const bool noise = ddpm && io.t > 0;
    const float* dummy = a.seg[0].X;             // any valid address
#pragma unroll
    for (int k = 0; k < EpiOps<TP>::NE; ++k) {
        const int o = tid + 256 * k;
        const int r = o / TP, pc = o % TP;
        const int co = co0 + r, l = pos0 + pc;
        const bool ok = co < a.Cout && l < a.L_out;
        const int coc = ok ? co : 0;
        const int64_t idx = ok ? ((int64_t)b * a.Cout + co) * a.L_out + l : 0;
        e.b1[k] = *(a.bias ? a.bias + coc : dummy);
        e.b2[k] = *(a.bias2 ? a.bias2 + coc : dummy);
        e.b3[k] = *(io.cbias ? io.cbias + (int64_t)b * a.scb + coc : dummy);
        e.r[k] = *(a.R ? a.R + idx : dummy);
        e.x[k] = *(ddpm ? io.xlat + idx : dummy);
        e.z[k] = *(noise ? io.z + idx : dummy);
    }
    // batch-uniform: scalar loads (the tables are not written during the launch)
    e.c1 = *(const LDM_KC float*)(ddpm ? a.c1 + io.t : dummy);
    e.c2 = *(const LDM_KC float*)(ddpm ? a.c2 + io.t : dummy);
    e.sg = *(const LDM_KC float*)(ddpm ? a.sigma + io.t : dummy);
}

// The contraction's segment geometry, two providers for conv_finish:
//   PlanGeo: read from the plan (scalar loads) where the contraction needs it (generic kernel);
//   FastGeo<NS>: the NS segments' fields read at kernel entry, with the staging's own argument
//     reads, and selected by segment with scalar selects -- read after the staging barrier they
//     were a chain of dependent scalar loads, ~0.45 us per conv (profiles/r04g stamps).
struct PlanGeo {
    KConv& a;
    KPlan& pl;
    __device__ __forceinline__ int n_seg() const { return a.n_seg; }
    __device__ __forceinline__ int nchunks() const { return pl.nchunks; }
    __device__ __forceinline__ int ch0(int s) const { return pl.s[s].ch0; }
    __device__ __forceinline__ int cinp(int s) const { return pl.s[s].cinp; }
    __device__ __forceinline__ int ks(int s) const { return a.seg[s].ksize; }
    __device__ __forceinline__ int st(int s) const { return a.seg[s].stride; }
    __device__ __forceinline__ int woff(int s) const { return pl.s[s].woff; }
    __device__ __forceinline__ int xoff(int s) const { return pl.s[s].xoff; }
};

template <int NS>
struct FastGeo {
    int nch, g0[NS], g1[NS];          // SegPlan::geo0 / geo1: 2 SGPRs per segment (six
                                      // separate fields made the 3-segment kernels spill)
    __device__ __forceinline__ void load(KPlan& pl) {
        nch = pl.nchunks;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            g0[i] = pl.s[i].geo0;
            g1[i] = pl.s[i].geo1;
        }
    }
    // v[s] for a wave-uniform s as a select chain (an indexed register array would go to scratch)
    __device__ __forceinline__ static int pick(const int (&v)[NS], int s) {
        int r = v[0];
#pragma unroll
        for (int i = 1; i < NS; ++i) r = s == i ? v[i] : r;
        return r;
    }
    __device__ __forceinline__ int n_seg() const { return NS; }
    __device__ __forceinline__ int nchunks() const { return nch; }
    __device__ __forceinline__ int ch0(int s) const { return pick(g0, s) & 0xfff; }
    __device__ __forceinline__ int ks(int s) const { return (pick(g0, s) >> 12) & 7; }
    __device__ __forceinline__ int st(int s) const { return ((pick(g0, s) >> 15) & 1) + 1; }
    __device__ __forceinline__ int cinp(int s) const { return (unsigned)pick(g0, s) >> 16; }
    __device__ __forceinline__ int woff(int s) const { return pick(g1, s) & 0xffff; }
    __device__ __forceinline__ int xoff(int s) const { return (unsigned)pick(g1, s) >> 16; }
};

template <typename G>
__device__ __forceinline__ G make_geo(KConv& a, KPlan& pl) {
    if constexpr (std::is_same<G, PlanGeo>::value) {
        return PlanGeo{a, pl};
    } else {
        G g;
        g.load(pl);
        return g;
    }
}

// The tile after its operands are staged (and the staging barrier passed): the MFMA
// contraction split over the 4 waves, the partial tiles summed in wave order, the fused
// epilogue.
// A chunk's A fragment held in registers (MAXC > 0, the fast kernel's register weights): the
// lane's 4 consecutive weights of row co0 + c16 -- 8 bytes of bf16 or 16 of fp32 -- as loaded.
template <typename TW>
struct WFrag {
    typedef typename std::conditional<sizeof(TW) == 2, u32x2, u32x4>::type V;
};
template <typename TW>
__device__ __forceinline__ f32x4 wfrag_unpack(const typename WFrag<TW>::V& w) {
    if constexpr (sizeof(TW) == 2)
        return f32x4{__builtin_bit_cast(float, w[0] << 16), __builtin_bit_cast(float, w[0] & 0xffff0000u),
                     __builtin_bit_cast(float, w[1] << 16), __builtin_bit_cast(float, w[1] & 0xffff0000u)};
    else
        return __builtin_bit_cast(f32x4, w);
}

template <typename TW, int TP, int MAXC = 0, typename GEO, typename ST>
__device__ __forceinline__ void conv_finish(KConv& a, const GEO& geo, const ConvIO& io,
                                            float* sm, int pos0, int co0, int b,
                                            const EpiOps<TP>& e, ST& st_,
                                            const typename WFrag<TW>::V* aw = nullptr) {
    constexpr int NT = TP / 16;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c16 = lane & 15;
    const bool ddpm = a.epi == LDM_CONV_EPI_DDPM;
    const bool noise = ddpm && io.t > 0;

    // The contraction: this wave's chunks (16 channels x one tap) [c_beg, c_end), TWO at a time
    // on two accumulator sets (chunk pairs alternate, so the MFMA chains interleave instead of
    // each MFMA waiting out its predecessor's 40-cycle latency), the next pair's operands read
    // from LDS before this pair's MFMAs, and the segment geometry (plan fields: scalar loads)
    // re-read only when a segment changes -- the first form read them per chunk and waited on
    // every LDS read (the MFMA phase was ~25 % of the step).  The two sets
    // are added at the end, so per output the sum order is fixed (deterministic).
    f32x4 acc0[NT], acc1[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        acc0[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc1[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int nchunks = geo.nchunks(), n_seg = geo.n_seg();
    // wave-uniform (scalar) chunk range: the loop below branches on it with scalar branches
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int c_beg = nchunks * wv / 4, c_end = nchunks * (wv + 1) / 4;
    // chunk iterator: (segment, tap, channel group) with the lane's operand offsets (floats)
    int si = 0;
    while (si + 1 < n_seg && c_beg >= geo.ch0(si + 1)) ++si;
    int ng = 0, ks = 0, st = 0, cinp = 0, wrow = 0, xbase = 0, xld = 0, k = 0, cg = 0;
    auto set_seg = [&](int s_) {
        cinp = geo.cinp(s_);
        ng = cinp >> 4;
        ks = geo.ks(s_);
        st = geo.st(s_);
        wrow = geo.woff(s_) + c16 * wpitch(ks, cinp) + 4 * g;
        xbase = geo.xoff(s_) + 4 * g;
        xld = xpitch(cinp, st);
    };
    set_seg(si);
    {
        int q = c_beg - geo.ch0(si);
        while (q >= ng) { q -= ng; ++k; }
        cg = q;
    }
    // The chunk iterator reads the current chunk's operands and then advances only while a
    // chunk of this wave is left (past the end it re-reads the last one): every LDS read of the
    // loop is unconditional, so the compiler can wait for exactly the pair an MFMA group needs
    // while the next pair is in flight.  (The first form loaded the next pair under branches
    // and rotated registers, so every pair waited for ALL reads, the prefetch included.)
    int left = c_end - c_beg - 1;           // chunks after the current one
    auto load_chunk = [&](f32x4& av, f32x4 (&bv)[NT]) {
        av = *reinterpret_cast<const f32x4*>(sm + wrow + k * cinp + cg * 16);
#pragma unroll
        for (int t = 0; t < NT; ++t)
            bv[t] = *reinterpret_cast<const f32x4*>(
                sm + xbase + ((t * 16 + c16) * st + k) * xld + cg * 16);
        if (left > 0) {
            --left;
            if (++cg == ng) {
                cg = 0;
                if (++k == ks && si + 1 < n_seg) {
                    k = 0;
                    set_seg(++si);
                }
            }
        }
    };
    auto mfma4 = [&](f32x4 (&acc)[NT], const f32x4& av, const f32x4 (&bv)[NT]) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int t = 0; t < NT; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[t][m], acc[t], 0, 0, 0);
    };
    const int n = c_end - c_beg;
    if constexpr (MAXC > 0) {
        // register weights: chunk j of this wave takes its A fragment from aw[j] (loaded at the
        // kernel's start) and its B fragments from LDS; the same accumulator set per chunk
        // parity and the same order within a set as the LDS form below, so the same bits
#pragma unroll
        for (int j = 0; j < MAXC; ++j) {
            if (j >= n) break;
            const f32x4 av = wfrag_unpack<TW>(aw[j]);
            f32x4 bv[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t)
                bv[t] = *reinterpret_cast<const f32x4*>(
                    sm + xbase + ((t * 16 + c16) * st + k) * xld + cg * 16);
            if (++cg == ng) {
                cg = 0;
                if (++k == ks && si + 1 < n_seg) {
                    k = 0;
                    set_seg(++si);
                }
            }
            if (j & 1) mfma4(acc1, av, bv);
            else mfma4(acc0, av, bv);
        }
        st_.mark(8);
    } else {
    // two pairs in flight (ping-pong, no register copies), chunks alternating between the two
    // accumulator sets so consecutive MFMAs are independent
    f32x4 pa0, pa1, pb0, pb1, qa0[NT], qa1[NT], qb0[NT], qb1[NT];
    if (n > 0) {
        load_chunk(pa0, qa0);
        load_chunk(pa1, qa1);
    }
    st_.mark(8);
    for (int i = 0; i < n; i += 4) {
        load_chunk(pb0, qb0);               // chunks i + 2, i + 3
        load_chunk(pb1, qb1);
        if (i + 1 < n) {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    acc0[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa0[m], qa0[t][m], acc0[t], 0, 0, 0);
                    acc1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa1[m], qa1[t][m], acc1[t], 0, 0, 0);
                }
        } else {
            mfma4(acc0, pa0, qa0);
        }
        if (i + 2 >= n) break;
        load_chunk(pa0, qa0);               // chunks i + 4, i + 5
        load_chunk(pa1, qa1);
        if (i + 3 < n) {
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    acc0[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(pb0[m], qb0[t][m], acc0[t], 0, 0, 0);
                    acc1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(pb1[m], qb1[t][m], acc1[t], 0, 0, 0);
                }
        } else {
            mfma4(acc0, pb0, qb0);
        }
    }
    }
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = acc0[t] + acc1[t];
    st_.mark(9);
    __syncthreads();                    // every wave is done reading the staged operands
    st_.mark(2);
    float* red = sm;                    // [wave][t][reg][lane]
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[((wave * NT + t) * 4 + i) * 64 + lane] = acc[t][i];
    __syncthreads();
    st_.mark(6);

#pragma unroll
    for (int k = 0; k < EpiOps<TP>::NE; ++k) {
        const int o = tid + 256 * k;
        const int r = o / TP, pc = o % TP;
        const int co = co0 + r, l = pos0 + pc;
        if (co >= a.Cout || l >= a.L_out) continue;
        const int t = pc >> 4, ln = 16 * (r >> 2) + (pc & 15), i = r & 3;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) v += red[((w * NT + t) * 4 + i) * 64 + ln];
        const int64_t idx = ((int64_t)b * a.Cout + co) * a.L_out + l;
        float bb = 0.f;                              // the summation order of every path
        if (a.bias) bb += e.b1[k];
        if (a.bias2) bb += e.b2[k];
        if (io.cbias) bb += e.b3[k];
        float pre = v + bb;
        if (a.R) pre += e.r[k];
        float y = pre;
        if (ddpm) y = ddpm_update(e.x[k], pre, noise ? e.z[k] : 0.f, e.c1, e.c2, e.sg, noise);
        io.Y[idx] = y;
    }
    st_.mark(10);
    if (UNET_STAMP) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_.mark(7);
    }
}

// ---- direct staging: the ldm_conv1d launch kernel -----------------
// A launch is latency-bound: the generic staging above spent ~45 VALU (two integer divisions,
// 64-bit address arithmetic) per 16-byte weight vector and per-element index arithmetic on
// the window, at one wave per SIMD, before and after ONE round trip per part (segment weights,
// segment window): 1.0-2.3 us per part in the stamps (profiles/r04f/stamp_conv_b1_fine.log).
// Here make_plan has checked that every count is a power of two, so an item's indices are
// shifts and masks of its number, the loads are raw buffer loads at 32-bit offsets, and every
// segment's weights and window are ISSUED before any LDS store (one round trip for the whole
// tile, the epilogue operands in flight under the stores).  The LDS image is the generic
// staging's, value for value (same SiLU), so the contraction and the results are unchanged.
//   weights: item i -> vector v = i & (nvec - 1) of row co = (i >> lgv) & 15, tap k = i >>
//            (lgv + 4): 16 bytes of the packed row (co0 + co, k), stored (fp32) at
//            woff + co wpitch(ksize, cinp) + k cinp + v EPV;
//   window:  item i -> source group gi = i & (NG - 1) (4 aligned positions a0 + 4 gi), channel
//            quad q = i >> lgng = 4 cg + g: the 4 channels 16 cg + g + 4 m (m = 0..3), i.e. the
//            4 consecutive perm16 columns 4 q.  Four 16-byte loads (one per channel), stored as
//            one 16-byte LDS vector per position (4 channels): 4 (8 for UP2) stores per item.
//            Rows L_in % 4 == 0, so a group lies wholly inside or outside [0, L_in): one test.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes,
                                             0x00020000);
}

template <typename TW, int NBW>
__device__ __forceinline__ void fast_w_issue(u32x4 (&v)[NBW], KSeg& s, KSegPlan& p, int co0,
                                             int base) {
    const __amdgpu_buffer_rsrc_t rs = rsrc(s.W, 0x7ffffff0u);
    const int lgv = p.lgv, nw = p.nw;
    const uint32_t ldw_b = (uint32_t)s.ldw * sizeof(TW), kst_b = (uint32_t)s.kstride * sizeof(TW);
#pragma unroll
    for (int u = 0; u < NBW; ++u) {
        const int i = base + u * 256 + (int)threadIdx.x;
        const uint32_t vv = i & ((1 << lgv) - 1), co = (i >> lgv) & 15, k = i >> (lgv + 4);
        uint32_t off = (uint32_t)(co0 + co) * ldw_b + k * kst_b + vv * 16u;
        off = i < nw ? off : 0xfffffff0u;          // absent item: out of range, no memory access
        v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
}

// Stores of absent items are skipped (exec-masked; a store needs no wait at the join): a common
// scratch address instead made every idle lane of a small conv write the same 16 bytes, one LDS
// bank conflict chain per instruction (~2 us per launch, profiles/r04g).
template <typename TW, int NBW>
__device__ __forceinline__ void fast_w_store(const u32x4 (&v)[NBW], float* sm, KSeg& s,
                                             KSegPlan& p, int base) {
    constexpr int EPV = 16 / sizeof(TW);
    const int lgv = p.lgv, nw = p.nw, cinp = p.cinp, wld = wpitch(s.ksize, cinp);
    float* ws = sm + p.woff;
#pragma unroll
    for (int u = 0; u < NBW; ++u) {
        const int i = base + u * 256 + (int)threadIdx.x;
        if (i >= nw) continue;
        const int vv = i & ((1 << lgv) - 1), co = (i >> lgv) & 15, k = i >> (lgv + 4);
        float* d = ws + co * wld + k * cinp + vv * EPV;
        if constexpr (sizeof(TW) == 2) {
            const u32x4 w = v[u];
            *reinterpret_cast<f32x4*>(d) = f32x4{
                __builtin_bit_cast(float, w[0] << 16), __builtin_bit_cast(float, w[0] & 0xffff0000u),
                __builtin_bit_cast(float, w[1] << 16), __builtin_bit_cast(float, w[1] & 0xffff0000u)};
            *reinterpret_cast<f32x4*>(d + 4) = f32x4{
                __builtin_bit_cast(float, w[2] << 16), __builtin_bit_cast(float, w[2] & 0xffff0000u),
                __builtin_bit_cast(float, w[3] << 16), __builtin_bit_cast(float, w[3] & 0xffff0000u)};
        } else {
            *reinterpret_cast<u32x4*>(d) = v[u];
        }
    }
}

// the window's source origin: a0 = the aligned group start at or below the first source
// position (UP2: positions of the upsampled row map to source p >> 1)
__device__ __forceinline__ int fast_x_a0(KSeg& s, int pos0) {
    const int pstart = pos0 * s.stride - s.pad;
    const int s0 = s.mode == LDM_CONV_UP2 ? (pstart >> 1) : pstart;   // floor (arithmetic shift)
    return s0 & ~3;
}

template <int NBX>
__device__ __forceinline__ void fast_x_issue(f32x4 (&v)[NBX][4], KSeg& s, KSegPlan& p,
                                             const float* X, int b, int pos0, int base) {
    const int L_in = s.L_in, lgng = p.lgng, nx = p.nx;
    const __amdgpu_buffer_rsrc_t rs =
        rsrc(X + (int64_t)b * s.C * L_in, (uint32_t)s.C * (uint32_t)L_in * 4u);
    const int a0 = fast_x_a0(s, pos0);
#pragma unroll
    for (int u = 0; u < NBX; ++u) {
        const int i = base + u * 256 + (int)threadIdx.x;
        const int gi = i & ((1 << lgng) - 1), q = i >> lgng;
        const int row0 = 16 * (q >> 2) + (q & 3);
        // channels >= C lie past the buffer's end and read 0; a group left of position 0 reads
        // the previous row (or nothing: negative offsets wrap past the end) and is masked; an
        // absent item reads out of range (no memory access)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            uint32_t off = (uint32_t)(((row0 + 4 * m) * L_in + a0 + 4 * gi) * 4);
            off = i < nx ? off : 0xfffffff0u;
            v[u][m] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        }
    }
}

template <int NBX>
__device__ __forceinline__ void fast_x_store(const f32x4 (&v)[NBX][4], float* sm, KSeg& s,
                                             KSegPlan& p, int pos0, int base) {
    const bool up2 = s.mode == LDM_CONV_UP2, act = s.silu_in != 0;
    const int L_in = s.L_in, lgng = p.lgng, nx = p.nx, win = p.win,
              ldx = xpitch(p.cinp, s.stride);
    const int pstart = pos0 * s.stride - s.pad;
    const int a0 = fast_x_a0(s, pos0);
    float* xs = sm + p.xoff;
#pragma unroll
    for (int u = 0; u < NBX; ++u) {
        const int i = base + u * 256 + (int)threadIdx.x;
        const int gi = i & ((1 << lgng) - 1), q = i >> lgng;
        const int sp0 = a0 + 4 * gi;
        if (i >= nx) continue;
        const bool inb = sp0 >= 0 && sp0 < L_in;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            f32x4 x = {v[u][0][e], v[u][1][e], v[u][2][e], v[u][3][e]};
            if (!inb) x = f32x4{0.f, 0.f, 0.f, 0.f};
            if (act)
                x = f32x4{silu_stage(x[0]), silu_stage(x[1]), silu_stage(x[2]), silu_stage(x[3])};
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                if (r == 1 && !up2) break;
                const int j = (up2 ? 2 * (sp0 + e) + r : sp0 + e) - pstart;
                if ((unsigned)j < (unsigned)win)
                    *reinterpret_cast<f32x4*>(xs + j * ldx + 4 * q) = x;
            }
        }
    }
}

struct ConvKArgs {
    ldm_conv1d_args_t a;
    ConvPlan pl;
};

#if UNET_STAMP
// diagnostic build: workgroup (0, 0, 0) of every ldm_conv1d launch stamps entry, staging done,
// MFMA done, reduction done and stores drained into a ring of 256 launches (ldm_dev_conv_stamps)
__device__ uint64_t g_conv_stamp[256][16];
__device__ unsigned g_conv_stamp_n;
#endif

#if UNET_STAMP
__device__ __forceinline__ void stamps_flush(const StampRegs& sr) {
    if (!sr.on) return;
    uint64_t* p = g_conv_stamp[atomicAdd(&g_conv_stamp_n, 1u) & 255u];
    for (int i = 0; i < 16; ++i) p[i] = sr.t[i];
}
#endif

// The generic launch kernel: conv_tile's staging (any channel count / alignment).
template <typename TW, int TP>
__global__ __launch_bounds__(256) void conv1d_mfma_kernel(ConvKArgs ka) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const LDM_KC ConvKArgs* k = (const LDM_KC ConvKArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    KConv& a = k->a;
    KPlan& pl = k->pl;
    StampRegs sr;
    sr.on = UNET_STAMP && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 &&
            threadIdx.x == 0;
    sr.mark(0);
    const int pos0 = blockIdx.x * TP, co0 = blockIdx.y * 16, b = blockIdx.z;
    const ConvIO io = conv_io(a);
    for (int si = 0; si < a.n_seg; ++si) {
        stage_w<TW>(sm + pl.s[si].woff, a.seg[si], pl.s[si], co0);
        if (si == 0) sr.mark(3);
        stage_x(sm + pl.s[si].xoff, a.seg[si], a.seg[si].X, pl.s[si], b, pos0);
        if (si == 0) sr.mark(4);
    }
    sr.mark(5);
    __syncthreads();
    sr.mark(1);
    EpiOps<TP> e;
    epi_load<TP>(e, a, io, pos0, co0, b);
    conv_finish<TW, TP>(a, PlanGeo{a, pl}, io, sm, pos0, co0, b, e, sr);
#if UNET_STAMP
    stamps_flush(sr);
#endif
}

// Register weights (MAXC > 0, round 6): instead of staging the tile's weights into LDS (fp32,
// 16 rows x every tap and channel: loads, bf16 unpack, LDS stores and the barrier's share), every
// lane loads exactly the A fragments its wave's chunks use -- 4 consecutive weights of its row
// per chunk, 8 bytes (bf16) -- straight from the packed rows into registers, in the staging's
// single round trip.  The weights are the same values, the contraction the same order: the same
// bits.  Chunk iteration as conv_finish's.
template <typename TW, int MAXC, typename GEO>
__device__ __forceinline__ void wreg_issue(typename WFrag<TW>::V (&aw)[MAXC], KConv& a,
                                           const GEO& geo, int co0) {
    const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int nch = geo.nchunks(), n_seg = geo.n_seg();
    const int c_beg = nch * wv / 4, c_end = nch * (wv + 1) / 4;
    int si = 0;
    while (si + 1 < n_seg && c_beg >= geo.ch0(si + 1)) ++si;
    int ng = geo.cinp(si) >> 4, ks = geo.ks(si), k = 0, cg = c_beg - geo.ch0(si);
    while (cg >= ng) { cg -= ng; ++k; }
#pragma unroll
    for (int j = 0; j < MAXC; ++j) {
        const bool live = c_beg + j < c_end;
        KSeg& sg = a.seg[si];
        const __amdgpu_buffer_rsrc_t rs = rsrc(sg.W, 0x7ffffff0u);
        uint32_t off = ((uint32_t)(co0 + c16) * (uint32_t)sg.ldw + (uint32_t)(k * sg.kstride) +
                        (uint32_t)(cg * 16 + 4 * g)) * (uint32_t)sizeof(TW);
        off = live ? off : 0xfffffff0u;               // past the chunks: no memory access
        if constexpr (sizeof(TW) == 2)
            aw[j] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
        else
            aw[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        if (live && ++cg == ng) {
            cg = 0;
            if (++k == ks && si + 1 < n_seg) {
                k = 0;
                ++si;
                ng = geo.cinp(si) >> 4;
                ks = geo.ks(si);
            }
        }
    }
}

// The direct-staging launch kernel (see fast_* above): NS segments, all staged in one round
// trip when they fit the per-thread budgets (the first round of every segment is issued before
// any store; a segment with more items runs extra rounds after), then conv_finish.
template <typename TW, int TP, int NS, int NBW, int MAXC = 0>
__global__ __launch_bounds__(256) void conv1d_fast_kernel(ConvKArgs ka) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const LDM_KC ConvKArgs* k = (const LDM_KC ConvKArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    KConv& a = k->a;
    KPlan& pl = k->pl;
    StampRegs sr;
    sr.on = UNET_STAMP && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 &&
            threadIdx.x == 0;
    sr.mark(0);
    const int pos0 = blockIdx.x * TP, co0 = blockIdx.y * 16, b = blockIdx.z;
    const ConvIO io = conv_io(a);
    sr.mark(13);                             // entry code done (block ids, io)
    // (3 segments: the plan read lazily -- preloaded, its SGPRs pushed the kernel into scratch)
    typedef typename std::conditional<NS <= 2, FastGeo<NS>, PlanGeo>::type Geo;
    Geo geo = make_geo<Geo>(a, pl);
    // per-thread items of a segment's first round: weights (16 B each; NBW picked per launch
    // from the segments' counts) and window items (4 x 16 B each: TP / 16 covers 128 channels).
    // Every slot is a load instruction even when its item is absent (out of range: no memory
    // access, but TA issue), so the slots match the launch: 4-slot weights and windows at every
    // size cost ~1 us per small conv (profiles/r04g).
    constexpr int NBX = TP / 16;
    constexpr bool WREG = MAXC > 0;
    constexpr int NBWS = WREG ? 1 : NBW;               // (no weight staging slots)
    u32x4 wv[NS][NBWS];
    typename WFrag<TW>::V aw[WREG ? MAXC : 1];
    f32x4 xv[NS][NBX][4];
    if constexpr (WREG) wreg_issue<TW, MAXC>(aw, a, geo, co0);
#pragma unroll
    for (int si = 0; si < NS; ++si) {
        if constexpr (!WREG) fast_w_issue<TW, NBW>(wv[si], a.seg[si], pl.s[si], co0, 0);
        fast_x_issue<NBX>(xv[si], a.seg[si], pl.s[si], a.seg[si].X, b, pos0, 0);
    }
    EpiOps<TP> e;
    epi_load<TP>(e, a, io, pos0, co0, b);
    sr.mark(11);
    // keep every load above issued before the first use of any of them below: the scheduler
    // otherwise pairs each segment's stores with its loads, or hoists the first bf16 unpack
    // above the window loads -- either is a wait for the data in the middle of the issue, one
    // round trip per part again.  (Empty asm: a memory clobber orders the loads; the register
    // operands make every use of the loaded values come after it.)
    asm volatile("" ::: "memory");
    if constexpr (WREG) {
#pragma unroll
        for (int j = 0; j < MAXC; ++j) asm volatile("" : "+v"(aw[j]));
    }
#pragma unroll
    for (int si = 0; si < NS; ++si) {
        if constexpr (!WREG) {
#pragma unroll
            for (int u = 0; u < NBW; ++u) asm volatile("" : "+v"(wv[si][u]));
        }
#pragma unroll
        for (int u = 0; u < NBX; ++u)
#pragma unroll
            for (int m = 0; m < 4; ++m) asm volatile("" : "+v"(xv[si][u][m]));
    }
    if (UNET_STAMP && sr.on) {               // diagnostic: every staging load has landed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sr.mark(12);
    }
#pragma unroll
    for (int si = 0; si < NS; ++si) {
        if constexpr (!WREG) fast_w_store<TW, NBW>(wv[si], sm, a.seg[si], pl.s[si], 0);
        fast_x_store<NBX>(xv[si], sm, a.seg[si], pl.s[si], pos0, 0);
    }
    sr.mark(3);
    sr.mark(4);
#pragma unroll
    for (int si = 0; si < NS; ++si) {
        if constexpr (!WREG)
        for (int base = 256 * NBW; base < pl.s[si].nw; base += 256 * NBW) {
            u32x4 v[NBW];
            fast_w_issue<TW, NBW>(v, a.seg[si], pl.s[si], co0, base);
            fast_w_store<TW, NBW>(v, sm, a.seg[si], pl.s[si], base);
        }
        for (int base = 256 * NBX; base < pl.s[si].nx; base += 256 * NBX) {
            f32x4 v[NBX][4];
            fast_x_issue<NBX>(v, a.seg[si], pl.s[si], a.seg[si].X, b, pos0, base);
            fast_x_store<NBX>(v, sm, a.seg[si], pl.s[si], pos0, base);
        }
    }
    sr.mark(5);
    __syncthreads();
    sr.mark(1);
    conv_finish<TW, TP, MAXC>(a, geo, io, sm, pos0, co0, b, e, sr, aw);
#if UNET_STAMP
    stamps_flush(sr);
#endif
}

constexpr int kMaxLdsBytes = 160 * 1024;

__host__ __device__ constexpr bool pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }
inline int ilog2(int x) { int l = 0; while ((1 << l) < x) ++l; return l; }

int make_plan(const ldm_conv1d_args_t& a, int TP, ConvPlan* pl, int* lds_bytes) {
    int off = 0, ch = 0;
    const int epv = a.w_dtype == LDM_BF16 ? 8 : 4;
    bool fast = true;
    for (int i = 0; i < a.n_seg; ++i) {
        const ldm_conv1d_seg_t& g = a.seg[i];
        SegPlan& p = pl->s[i];
        p.cinp = round16(g.C);
        p.win = (TP - 1) * g.stride + g.ksize;
        p.xoff = off;
        off += p.win * xpitch(p.cinp, g.stride);
        p.woff = off;
        off += 16 * wpitch(g.ksize, p.cinp);
        p.ch0 = ch;
        ch += g.ksize * (p.cinp / 16);
        // direct staging: power-of-two item counts, 16-byte source groups, 32-bit offsets
        p.lgv = ilog2(p.cinp / epv);
        p.nw = 16 * g.ksize * (p.cinp / epv);
        const int span = g.mode == LDM_CONV_UP2 ? p.win / 2 + 3 : p.win + 2;
        p.lgng = ilog2(span / 4 + 1);
        p.nx = (p.cinp / 4) << p.lgng;
        p.geo0 = p.ch0 | g.ksize << 12 | (g.stride - 1) << 15 | p.cinp << 16;
        p.geo1 = p.woff | p.xoff << 16;
        const int64_t wbytes = (int64_t)(a.Cout + 15) / 16 * 16 * g.ldw * (epv == 8 ? 2 : 4);
        fast = fast && pow2(p.cinp) && g.L_in % 4 == 0 && ((uintptr_t)g.X & 15) == 0 &&
               p.ch0 < 4096 && p.cinp < 65536 && p.woff < 65536 && p.xoff < 65536 &&
               ((uintptr_t)g.W & 15) == 0 && (g.ldw * (16 / epv)) % 16 == 0 &&
               (g.kstride * (16 / epv)) % 16 == 0 &&
               // the window offsets run over PADDED channel rows (row0 + 4m < cinp) in signed
               // 32-bit arithmetic, and the weight resource spans 0x7ffffff0 bytes
               (int64_t)p.cinp * g.L_in * 4 < (1ll << 31) && wbytes <= 0x7ffffff0ll;
    }
    pl->nchunks = ch;
    pl->fast = fast;
    const int red = 4 * (TP / 16) * 4 * 64;
    pl->lds_floats = off > red ? off : red;
    *lds_bytes = 4 * pl->lds_floats;
    return *lds_bytes <= kMaxLdsBytes ? 0 : LDM_ENOSPC;
}

template <typename TW, int TP, int NS, int NBW, int MAXC = 0>
int launch_fast(const ConvKArgs& ka, dim3 grid, int lds, hipStream_t s) {
    LDM_TRY((set_max_lds_once<&conv1d_fast_kernel<TW, TP, NS, NBW, MAXC>>(kMaxLdsBytes, "conv1d")));
    hipLaunchKernelGGL((conv1d_fast_kernel<TW, TP, NS, NBW, MAXC>), grid, dim3(256), lds, s, ka);
    return launch_status("ldm_conv1d");
}

// register weights (conv1d_fast_kernel MAXC) when every wave's chunks fit kWregChunks
// (UNET_WREG 0: the LDS-staged weights, the round-5 form)
#ifndef UNET_WREG
#define UNET_WREG 1
#endif
constexpr int kWregChunks = 8;

template <typename TW, int TP, int NS>
int launch_fast_nbw(const ConvKArgs& ka, dim3 grid, int lds, hipStream_t s) {
    if (UNET_WREG && ka.pl.nchunks <= 4 * kWregChunks && dev_knob("LDM_CONV_WREG", 1))
        return launch_fast<TW, TP, NS, 1, kWregChunks>(ka, grid, lds, s);
    int nw = 0;
    for (int i = 0; i < NS; ++i) nw = ka.pl.s[i].nw > nw ? ka.pl.s[i].nw : nw;
    if (nw <= 256) return launch_fast<TW, TP, NS, 1>(ka, grid, lds, s);
    if (nw <= 512) return launch_fast<TW, TP, NS, 2>(ka, grid, lds, s);
    return launch_fast<TW, TP, NS, 4>(ka, grid, lds, s);   // more: extra rounds
}

template <typename TW, int TP>
int launch_tp(const ldm_conv1d_args_t& a, hipStream_t s) {
    ConvPlan pl = {};
    int lds = 0;
    LDM_REQUIRE(make_plan(a, TP, &pl, &lds) == 0, LDM_ENOSPC,
                "conv1d: staged operands need %d B of LDS (> %d); split the channels", lds,
                kMaxLdsBytes);
    const dim3 grid((a.L_out + TP - 1) / TP, (a.Cout + 15) / 16, a.B);
    ConvKArgs ka;
    ka.a = a;
    ka.pl = pl;
    // dev A/B: LDM_CONV_FAST=0 forces the generic staging
    if (pl.fast && a.n_seg <= 3 && dev_knob("LDM_CONV_FAST", 1)) {
        switch (a.n_seg) {
            case 1: return launch_fast_nbw<TW, TP, 1>(ka, grid, lds, s);
            case 2: return launch_fast_nbw<TW, TP, 2>(ka, grid, lds, s);
            default: return launch_fast_nbw<TW, TP, 3>(ka, grid, lds, s);
        }
    }
    LDM_TRY((set_max_lds_once<&conv1d_mfma_kernel<TW, TP>>(kMaxLdsBytes, "conv1d")));
    hipLaunchKernelGGL((conv1d_mfma_kernel<TW, TP>), grid, dim3(256), lds, s, ka);
    return launch_status("ldm_conv1d");
}

template <typename TW>
int launch_conv(const ldm_conv1d_args_t& a, hipStream_t s) {
    // Widest tile that still leaves >= 512 workgroups (latency: small grids get TP = 16).
    const long tiles16 = (long)((a.L_out + 15) / 16) * ((a.Cout + 15) / 16) * a.B;
    if (tiles16 >= 4 * 512) return launch_tp<TW, 64>(a, s);
    if (tiles16 >= 2 * 512) return launch_tp<TW, 32>(a, s);
    return launch_tp<TW, 16>(a, s);
}

// The checks ldm_conv1d makes on one call.
int check_conv_args(const ldm_conv1d_args_t* a) {
    LDM_REQUIRE(a && a->Y && a->B >= 1 && a->Cout >= 1 && a->L_out >= 1, LDM_EINVAL,
                "bad conv1d args");
    LDM_REQUIRE(a->B <= 65535, LDM_EINVAL, "conv1d: B %d > 65535", a->B);
    LDM_REQUIRE(a->n_seg >= 1 && a->n_seg <= LDM_CONV_MAX_SEGS, LDM_EINVAL, "bad n_seg %d",
                a->n_seg);
    LDM_REQUIRE(a->w_dtype == LDM_F32 || a->w_dtype == LDM_BF16, LDM_EINVAL, "bad w_dtype");
    LDM_REQUIRE(a->epi == LDM_CONV_EPI_STORE || a->epi == LDM_CONV_EPI_DDPM, LDM_EINVAL,
                "bad conv epilogue %d", a->epi);
    if (a->epi == LDM_CONV_EPI_DDPM)
        LDM_REQUIRE(a->xlat && a->c1 && a->c2 && a->sigma && a->t >= 0 && (a->t == 0 || a->z),
                    LDM_EINVAL, "conv1d DDPM epilogue needs xlat, tables, t and z");
    for (int i = 0; i < a->n_seg; ++i) {
        const ldm_conv1d_seg_t& g = a->seg[i];
        LDM_REQUIRE(g.X && g.W && g.C >= 1 && g.L_in >= 1 && g.pad >= 0, LDM_EINVAL,
                    "conv1d seg %d: bad operand", i);
        const bool ok = (g.ksize == 3 && (g.stride == 1 || g.stride == 2)) ||
                        (g.ksize == 1 && g.stride == 1) || (g.ksize == 4 && g.stride == 2);
        LDM_REQUIRE(ok, LDM_EINVAL, "conv1d seg %d: unsupported ksize %d / stride %d", i,
                    g.ksize, g.stride);
        LDM_REQUIRE(g.mode == LDM_CONV_DIRECT || (g.mode == LDM_CONV_UP2 && g.stride == 1),
                    LDM_EINVAL, "conv1d seg %d: bad mode %d", i, g.mode);
        LDM_REQUIRE(g.kstride >= ((g.C + 15) & ~15) && g.ldw >= g.ksize * g.kstride,
                    LDM_EINVAL, "conv1d seg %d: packed weight pitches (ldw %d, kstride %d)",
                    i, g.ldw, g.kstride);
        LDM_REQUIRE(g.pad < g.ksize, LDM_EINVAL, "conv1d seg %d: pad %d >= ksize", i, g.pad);
    }
    return 0;
}

}  // namespace
}  // namespace ldm

extern "C" int ldm_conv1d(const ldm_conv1d_args_t* a, ldm_stream_t s) {
    using namespace ldm;
    LDM_TRY(check_conv_args(a));
    if (a->w_dtype == LDM_BF16) return launch_conv<unsigned short>(*a, (hipStream_t)s);
    return launch_conv<float>(*a, (hipStream_t)s);
}

#if UNET_STAMP
// diagnostic build only: the conv stamp ring (256 x 16 s_memrealtime values) and its counter
extern "C" int ldm_dev_conv_stamps(uint64_t* host, unsigned* n) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(ldm::g_conv_stamp), sizeof(ldm::g_conv_stamp)) !=
            hipSuccess ||
        hipMemcpyFromSymbol(n, HIP_SYMBOL(ldm::g_conv_stamp_n), sizeof(unsigned)) != hipSuccess)
        return -1;
    return 0;
}
#endif
