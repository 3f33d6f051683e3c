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
//     (loads of a segment issued back to back before their LDS stores), then one barrier,
//     then the MFMA loop runs from LDS only;
//   * LDS layouts put each lane's operands for 4 consecutive MFMAs in one ds_read_b128:
//     channels are permuted inside every group of 16 (perm16) on staging, and the weights
//     arrive already permuted from the host packing (ldm_sdf/ops.py pack_conv_weight).
#include "ldm_internal.h"
#include "ddpm_common.h"

namespace ldm {
namespace {

__host__ __device__ constexpr int round16(int c) { return (c + 15) & ~15; }
// Position of channel ci inside its 16-group so that lane group g reads channels
// 16c + 4m + g (m = 0..3: four consecutive MFMAs) as one 16-byte vector.
__host__ __device__ constexpr int perm16(int ci) {
    return (ci & ~15) | ((ci & 3) << 2) | ((ci >> 2) & 3);
}

struct SegPlan {
    int cinp;   // channels rounded up to 16
    int win;    // input window (positions) of one tile
    int xoff;   // LDS float offset of the window  [win][cinp + 4]
    int woff;   // LDS float offset of the weights [16][ksize * cinp + 4]
    int ch0;    // first contraction chunk (16 channels x one tap) of this segment
};
struct ConvPlan {
    SegPlan s[LDM_CONV_MAX_SEGS];
    int nchunks;
    int lds_floats;   // including 4 scratch floats at the end (stores of out-of-range slots)
};

// Staging issues every load of a segment before the first LDS store (one global round trip),
// branch-free: out-of-range slots load a clamped in-bounds address and select 0, and store
// to a scratch word past the operands.  The slot count NB is picked per segment from the
// real item count (4 / 8 / 16 / 32), so a small segment does not pay a 32-slot unroll.
template <int TP, int NB>
__device__ __forceinline__ void stage_x_nb(float* __restrict__ xs, float* __restrict__ trash,
                                           const ldm_conv1d_seg_t& s, const SegPlan& p, int b,
                                           int pos0) {
    constexpr int CW = TP <= 16 ? 32 : 64;            // window columns per pass
    constexpr int RPP = 256 / CW;                     // channel rows per pass
    const int tid = threadIdx.x;
    const int col = tid % CW, row = tid / CW;
    const bool up2 = s.mode == LDM_CONV_UP2;
    const int Lsrc = up2 ? 2 * s.L_in : s.L_in;
    const int pstart = pos0 * s.stride - s.pad;
    const float* X = s.X + (int64_t)b * s.C * s.L_in;
    const int ncolp = (p.win + CW - 1) / CW;
    const int nitem = ncolp * ((p.cinp + RPP - 1) / RPP);
    const int ld = p.cinp + 4;
    for (int base = 0; base < nitem; base += NB) {
        float v[NB];
        int dst[NB];
        int rp = base / ncolp, cp = base - rp * ncolp;
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int ci = rp * RPP + row, j = cp * CW + col, pp = pstart + j;
            const bool in = base + u < nitem && ci < p.cinp && j < p.win;
            const bool ok = in && ci < s.C && pp >= 0 && pp < Lsrc;
            const int src = ok ? ci * s.L_in + (up2 ? (pp >> 1) : pp) : 0;
            v[u] = X[src];
            v[u] = ok ? v[u] : 0.f;
            dst[u] = in ? j * ld + perm16(ci) : -1;
            if (++cp == ncolp) { cp = 0; ++rp; }
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            float* d = dst[u] >= 0 ? xs + dst[u] : trash;
            *d = s.silu_in ? silu(v[u]) : v[u];
        }
    }
}

template <int TP>
__device__ __forceinline__ void stage_x(float* xs, float* trash, const ldm_conv1d_seg_t& s,
                                        const SegPlan& p, int b, int pos0) {
    constexpr int CW = TP <= 16 ? 32 : 64;
    const int n = ((p.win + CW - 1) / CW) * ((p.cinp + 256 / CW - 1) / (256 / CW));
    if (n <= 4) stage_x_nb<TP, 4>(xs, trash, s, p, b, pos0);
    else if (n <= 8) stage_x_nb<TP, 8>(xs, trash, s, p, b, pos0);
    else if (n <= 16) stage_x_nb<TP, 16>(xs, trash, s, p, b, pos0);
    else stage_x_nb<TP, 32>(xs, trash, s, p, b, pos0);
}

// Weights: 16-byte vector loads along a packed row (4 fp32 or 8 bf16 channels per load).
template <typename TW, int NB>
__device__ __forceinline__ void stage_w_nb(float* __restrict__ ws, const ldm_conv1d_seg_t& s,
                                           const SegPlan& p, int co0) {
    constexpr int EPV = 16 / sizeof(TW);              // elements per 16-byte vector
    const int tid = threadIdx.x;
    const int nvec = p.cinp / EPV;                    // vectors per (row, tap)
    const int per_row = s.ksize * nvec;
    const int nitem = 16 * per_row;
    const int ld = s.ksize * p.cinp + 4;
    const char* W = reinterpret_cast<const char*>(s.W);
    for (int base = 0; base < nitem; base += 256 * NB) {
        u32x4 v[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int it = base + u * 256 + tid;
            const int itc = it < nitem ? it : 0;
            const int co = itc / per_row, r = itc - co * per_row;
            const int k = r / nvec, e = (r - k * nvec) * EPV;
            const int64_t gi = (int64_t)(co0 + co) * s.ldw + (int64_t)k * s.kstride + e;
            v[u] = *reinterpret_cast<const u32x4*>(W + gi * (int64_t)sizeof(TW));
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int it = base + u * 256 + tid;
            if (it >= nitem) continue;
            const int co = it / per_row, r = it - co * per_row;
            const int k = r / nvec, e = (r - k * nvec) * EPV;
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
}

template <typename TW>
__device__ __forceinline__ void stage_w(float* ws, const ldm_conv1d_seg_t& s, const SegPlan& p,
                                        int co0) {
    const int n = (16 * s.ksize * (p.cinp / (16 / (int)sizeof(TW))) + 255) / 256;
    if (n <= 1) stage_w_nb<TW, 1>(ws, s, p, co0);
    else if (n <= 2) stage_w_nb<TW, 2>(ws, s, p, co0);
    else if (n <= 4) stage_w_nb<TW, 4>(ws, s, p, co0);
    else stage_w_nb<TW, 8>(ws, s, p, co0);
}

template <typename TW, int TP>
__global__ __launch_bounds__(256) void conv1d_mfma_kernel(ldm_conv1d_args_t a, ConvPlan pl) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    constexpr int NT = TP / 16;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g = lane >> 4, c16 = lane & 15;
    const int pos0 = blockIdx.x * TP, co0 = blockIdx.y * 16, b = blockIdx.z;

    float* trash = sm + pl.lds_floats - 4;
    for (int si = 0; si < a.n_seg; ++si) {
        stage_w<TW>(sm + pl.s[si].woff, a.seg[si], pl.s[si], co0);
        stage_x<TP>(sm + pl.s[si].xoff, trash, a.seg[si], pl.s[si], b, pos0);
    }
    __syncthreads();

    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int c_beg = pl.nchunks * wave / 4, c_end = pl.nchunks * (wave + 1) / 4;
    // walk this wave's chunks with carried (segment, tap, channel group) counters
    int si = 0;
    while (si + 1 < a.n_seg && c_beg >= pl.s[si + 1].ch0) ++si;
    int ng = pl.s[si].cinp >> 4;
    int q = c_beg - pl.s[si].ch0;
    int k = 0;
    while (q >= ng) { q -= ng; ++k; }
    int cg = q;
    for (int ch = c_beg; ch < c_end; ++ch) {
        const SegPlan& p = pl.s[si];
        const int ks = a.seg[si].ksize, st = a.seg[si].stride;
        const f32x4 av = *reinterpret_cast<const f32x4*>(
            sm + p.woff + c16 * (ks * p.cinp + 4) + k * p.cinp + cg * 16 + 4 * g);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int j = (t * 16 + c16) * st + k;
            const f32x4 bv = *reinterpret_cast<const f32x4*>(
                sm + p.xoff + j * (p.cinp + 4) + cg * 16 + 4 * g);
#pragma unroll
            for (int m = 0; m < 4; ++m)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[m], acc[t], 0, 0, 0);
        }
        if (++cg == ng) {
            cg = 0;
            if (++k == ks && si + 1 < a.n_seg) { k = 0; ++si; ng = pl.s[si].cinp >> 4; }
        }
    }
    __syncthreads();                    // every wave is done reading the staged operands
    float* red = sm;                    // [wave][t][reg][lane]
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[((wave * NT + t) * 4 + i) * 64 + lane] = acc[t][i];
    __syncthreads();

    for (int o = tid; o < 16 * TP; o += 256) {
        const int r = o / TP, pc = o % TP;
        const int co = co0 + r, l = pos0 + pc;
        if (co >= a.Cout || l >= a.L_out) continue;
        const int t = pc >> 4, ln = 16 * (r >> 2) + (pc & 15), i = r & 3;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) v += red[((w * NT + t) * 4 + i) * 64 + ln];
        float bb = 0.f;
        if (a.bias) bb += a.bias[co];
        if (a.bias2) bb += a.bias2[co];
        if (a.cbias) bb += a.cbias[(int64_t)b * a.scb + co];
        const int64_t idx = ((int64_t)b * a.Cout + co) * a.L_out + l;
        float pre = v + bb;
        if (a.R) pre += a.R[idx];
        if (a.epi == LDM_CONV_EPI_DDPM) {
            const bool noise = a.t > 0;
            a.Y[idx] = ddpm_update(a.xlat[idx], pre, noise ? a.z[idx] : 0.f, a.c1[a.t],
                                   a.c2[a.t], a.sigma[a.t], noise);
        } else {
            a.Y[idx] = pre;
        }
    }
}

constexpr int kMaxLdsBytes = 160 * 1024;

int make_plan(const ldm_conv1d_args_t& a, int TP, ConvPlan* pl, int* lds_bytes) {
    int off = 0, ch = 0;
    for (int i = 0; i < a.n_seg; ++i) {
        const ldm_conv1d_seg_t& g = a.seg[i];
        SegPlan& p = pl->s[i];
        p.cinp = round16(g.C);
        p.win = (TP - 1) * g.stride + g.ksize;
        p.xoff = off;
        off += p.win * (p.cinp + 4);
        p.woff = off;
        off += 16 * (g.ksize * p.cinp + 4);
        p.ch0 = ch;
        ch += g.ksize * (p.cinp / 16);
    }
    pl->nchunks = ch;
    const int red = 4 * (TP / 16) * 4 * 64;
    pl->lds_floats = (off > red ? off : red) + 4;
    *lds_bytes = 4 * pl->lds_floats;
    return *lds_bytes <= kMaxLdsBytes ? 0 : LDM_ENOSPC;
}

template <typename TW, int TP>
int launch_tp(const ldm_conv1d_args_t& a, hipStream_t s) {
    ConvPlan pl = {};
    int lds = 0;
    LDM_REQUIRE(make_plan(a, TP, &pl, &lds) == 0, LDM_ENOSPC,
                "conv1d: staged operands need %d B of LDS (> %d); split the channels", lds,
                kMaxLdsBytes);
    static bool attr_set = false;     // one per instantiation; idempotent if raced
    if (!attr_set) {
        const hipError_t e = hipFuncSetAttribute(
            reinterpret_cast<const void*>(&conv1d_mfma_kernel<TW, TP>),
            hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLdsBytes);
        LDM_REQUIRE(e == hipSuccess, (int)e, "conv1d: hipFuncSetAttribute: %s",
                    hipGetErrorString(e));
        attr_set = true;
    }
    const dim3 grid((a.L_out + TP - 1) / TP, (a.Cout + 15) / 16, a.B);
    hipLaunchKernelGGL((conv1d_mfma_kernel<TW, TP>), grid, dim3(256), lds, s, a, pl);
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

}  // namespace
}  // namespace ldm

extern "C" int ldm_conv1d(const ldm_conv1d_args_t* a, ldm_stream_t s) {
    using namespace ldm;
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
    if (a->w_dtype == LDM_BF16) return launch_conv<unsigned short>(*a, (hipStream_t)s);
    return launch_conv<float>(*a, (hipStream_t)s);
}
