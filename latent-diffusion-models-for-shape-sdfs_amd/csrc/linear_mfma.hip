// Matrix-core path of ldm_linear (compute = LDM_COMPUTE_BF16): the training GEMMs of the DDPM
// denoiser (A6/A7 at the training batch, config 2) -- forward X W^T, input gradient G W and
// weight gradient G^T X through the same strided-view interface as the fp32 VALU kernel
// (denoiser.hip linear_tiled_kernel), with the same epilogues.
//
// Arithmetic: operands are rounded to bf16 (RNE) on their way into LDS, products and sums are
// fp32 (v_mfma_f32_32x32x16_bf16): mixed-precision training.  The fp32 VALU kernel stays the
// exact path (compute = LDM_COMPUTE_FP32) that the fp64 gradient parity test pins.
//
// Tiling: a workgroup (4 waves) owns a 64 (rows b) x 64 (cols m) tile, each wave a 32 x 32
// MFMA tile.  K advances in KCH-deep chunks (64 or 128, see Chunk) through two LDS buffers
// per operand: the next chunk's global loads are issued into registers before the current chunk's MFMAs (one barrier
// per chunk).  At the training shapes (1000 x 1024 x 1024..2048, 256 workgroups = one per CU)
// each workgroup walks K alone; 128-deep chunks (vs 64) and the XCD-grouped tile order below
// each took ~5-10 % off.  Operand tiles load with 16-byte vectors along
// the contiguous dimension when strides and alignment allow (vec_ok), else element-wise; every
// load is unconditional (clamped index, value selected) so a wave keeps them all in flight.
// LDS rows are 128 + 8 bf16 (272 B): the 16-byte fragment reads of 16 consecutive rows land
// 4 banks apart, conflict-free.
#include "ldm_internal.h"
#include "ddpm_common.h"

#include <algorithm>

namespace ldm {
namespace {

// Chunk depth KCH (k per LDS chunk) is a template parameter, picked per call (launch_mfma3):
// 128 for few workgroups with long K (training, 1 workgroup per CU: deeper chunks amortise
// the barrier), 64 for many workgroups (auto-decoder, 1M rows: 37 KiB of LDS instead of
// 68 KiB doubles the workgroups per CU, which hides the operand-load latency).
constexpr int kKCSplit = 128;        // split-K slice granularity (a multiple of every KCH)
template <int KCH>
struct Chunk {
    static constexpr int Ld = KCH + 8;                               // LDS row pitch (bf16)
    static constexpr int Buf = 64 * Ld;                              // one operand buffer
    static constexpr int LdsBytes = 4 * Buf * (int)sizeof(unsigned short);   // X0 X1 W0 W1
};

__device__ __forceinline__ unsigned pack_bf16(float a, float b) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 v = {a, b};
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}

template <typename T>
__device__ __forceinline__ float ld_elem(const T* p, int64_t i) {
    if constexpr (sizeof(T) == 2) return bf16_to_f32(p[i]);
    else return p[i];
}

// One operand tile: rows [r0, r0+64) x k [k0, k0+kKC) of a strided matrix, E values per thread
// held in registers between the load and the LDS store.  A "line" is a run along the
// contiguous dimension: a row (KC, contiguous along k) or a k column (rows contiguous).
// VEC: 16-byte vector loads along the line (its stride 1, the other stride and the base
// 16-byte aligned, the line extent a multiple of the vector); lanes of a wave then cover whole
// 256-byte (fp32) / 128-byte (bf16) segments.  Otherwise TPL threads per line, E consecutive
// elements each.
template <typename T, bool KC, bool VEC, int KCH>
struct Tile {
    static constexpr int kKC = KCH, kLd = Chunk<KCH>::Ld;
    static constexpr int E = 64 * kKC / 256;          // values per thread
    static constexpr int EPV = 16 / sizeof(T);        // elements per 16-byte vector
    static constexpr int LEN = KC ? kKC : 64;         // line length
    static constexpr int VPL = LEN / EPV;             // vectors per line
    static constexpr int NV = E / EPV;                // vectors per thread
    static constexpr int TPL = LEN / E;               // scalar path: threads per line
    static constexpr int RG = 64 / EPV;               // !KC vector path: row groups
    static_assert(KC || !VEC || NV * (256 / RG) == kKC, "!KC vector tile covers the chunk");
    float v[E];

    __device__ __forceinline__ void load(const T* __restrict__ P, int64_t sr, int64_t sk,
                                         int rows, int K, int r0, int k0) {
        const int t = threadIdx.x;
        if constexpr (VEC && !KC) {
            // rows contiguous: thread owns EPV rows x NV consecutive k (one 16-byte load per
            // k; 64/EPV lanes cover one k's 64 rows), so store() writes whole k-runs per row
#pragma unroll
            for (int u = 0; u < NV; ++u) {
                const int r = r0 + (t % RG) * EPV, k = k0 + (t / RG) * NV + u;
                const bool ok = r < rows && k < K;
                const int64_t gi = ok ? (int64_t)r * sr + (int64_t)k * sk : 0;
                u32x4 w = *reinterpret_cast<const u32x4*>(P + gi);
                if (!ok) w = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const unsigned wq = w[q];
                    if constexpr (sizeof(T) == 2) {
                        v[u * 8 + 2 * q] = __builtin_bit_cast(float, wq << 16);
                        v[u * 8 + 2 * q + 1] = __builtin_bit_cast(float, wq & 0xffff0000u);
                    } else {
                        v[u * 4 + q] = __builtin_bit_cast(float, wq);
                    }
                }
            }
        } else if constexpr (VEC) {
#pragma unroll
            for (int u = 0; u < NV; ++u) {
                const int id = u * 256 + t;
                const int line = id / VPL, e = (id % VPL) * EPV;
                const int r = KC ? r0 + line : r0 + e, k = KC ? k0 + e : k0 + line;
                const bool ok = r < rows && k < K;
                const int64_t gi = ok ? (int64_t)r * sr + (int64_t)k * sk : 0;
                u32x4 w = *reinterpret_cast<const u32x4*>(P + gi);
                if (!ok) w = u32x4{0u, 0u, 0u, 0u};
                // copy each element out first: __builtin_bit_cast of an ext-vector element
                // lvalue (w[q]) reads element 0 whatever q is
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const unsigned wq = w[q];
                    if constexpr (sizeof(T) == 2) {
                        v[u * 8 + 2 * q] = __builtin_bit_cast(float, wq << 16);
                        v[u * 8 + 2 * q + 1] = __builtin_bit_cast(float, wq & 0xffff0000u);
                    } else {
                        v[u * 4 + q] = __builtin_bit_cast(float, wq);
                    }
                }
            }
        } else {
            const int line = t / TPL, eb = (t % TPL) * E;
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const int r = KC ? r0 + line : r0 + eb + j, k = KC ? k0 + eb + j : k0 + line;
                const bool ok = r < rows && k < K;
                const float x = ld_elem(P, ok ? (int64_t)r * sr + (int64_t)k * sk : 0);
                v[j] = ok ? x : 0.f;
            }
        }
    }

    // S: [64 rows][kLd] bf16, row-major in (row, k) whatever the source layout.
    __device__ __forceinline__ void store(unsigned short* __restrict__ S) const {
        const int t = threadIdx.x;
        if constexpr (VEC && !KC) {   // per row: NV consecutive k -> one 16-B (fp32 source,
                                      // NV = 8) or 8-B (bf16 source, NV = 4) LDS store
            const int rl = (t % RG) * EPV, kl = (t / RG) * NV;
#pragma unroll
            for (int q = 0; q < EPV; ++q) {
                unsigned short* d = S + (rl + q) * kLd + kl;
                if constexpr (NV == 8) {
                    u32x4 w;
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        w[c] = pack_bf16(v[(2 * c) * EPV + q], v[(2 * c + 1) * EPV + q]);
                    *reinterpret_cast<u32x4*>(d) = w;
                } else if constexpr (NV == 4) {
                    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                    u32x2 w;
#pragma unroll
                    for (int c = 0; c < 2; ++c)
                        w[c] = pack_bf16(v[(2 * c) * EPV + q], v[(2 * c + 1) * EPV + q]);
                    *reinterpret_cast<u32x2*>(d) = w;
                } else {
                    static_assert(NV == 2, "k-run of 2, 4 or 8");
                    *reinterpret_cast<unsigned*>(d) = pack_bf16(v[q], v[EPV + q]);
                }
            }
        } else if constexpr (VEC) {
#pragma unroll
            for (int u = 0; u < NV; ++u) {
                const int id = u * 256 + t;
                const int line = id / VPL, e = (id % VPL) * EPV;
                const float* x = v + u * EPV;
                if constexpr (KC) {      // EPV consecutive k of one row -> one 8/16-byte store
                    if constexpr (EPV == 8) {
                        u32x4 w;
#pragma unroll
                        for (int q = 0; q < 4; ++q) w[q] = pack_bf16(x[2 * q], x[2 * q + 1]);
                        *reinterpret_cast<u32x4*>(S + line * kLd + e) = w;
                    } else {
                        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                        const u32x2 w = {pack_bf16(x[0], x[1]), pack_bf16(x[2], x[3])};
                        *reinterpret_cast<u32x2*>(S + line * kLd + e) = w;
                    }
                } else {                 // EPV consecutive rows of one k -> 2-byte stores
#pragma unroll
                    for (int q = 0; q < EPV; q += 2) {
                        const unsigned p = pack_bf16(x[q], x[q + 1]);
                        S[(e + q) * kLd + line] = (unsigned short)(p & 0xffffu);
                        S[(e + q + 1) * kLd + line] = (unsigned short)(p >> 16);
                    }
                }
            }
        } else {
            const int line = t / TPL, eb = (t % TPL) * E;
            if constexpr (KC) {
#pragma unroll
                for (int c = 0; c < E / 8; ++c) {
                    u32x4 w;
#pragma unroll
                    for (int q = 0; q < 4; ++q) w[q] = pack_bf16(v[8 * c + 2 * q], v[8 * c + 2 * q + 1]);
                    *reinterpret_cast<u32x4*>(S + line * kLd + eb + 8 * c) = w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < E; j += 2) {
                    const unsigned p = pack_bf16(v[j], v[j + 1]);
                    S[(eb + j) * kLd + line] = (unsigned short)(p & 0xffffu);
                    S[(eb + j + 1) * kLd + line] = (unsigned short)(p >> 16);
                }
            }
        }
    }
};

template <typename TW, bool XK, bool WK, bool XV, bool WV, int KCH>
__device__ __forceinline__ void mfma_segment(f32x16& acc, unsigned short* __restrict__ sm,
                                             const float* X, int64_t sxb, int64_t sxk,
                                             const void* Wv, int64_t swm, int64_t swk, int K,
                                             int Bn, int M, int b0, int m0) {
    const TW* W = reinterpret_cast<const TW*>(Wv);
    // buffers addressed as sm + offset (not through a pointer array, which loses the LDS
    // address space and turns the fragment reads into flat loads): X0 X1 W0 W1
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
    const int r = lane & 31, h = lane >> 5;
    constexpr int kKC = KCH, kLd = Chunk<KCH>::Ld, kBuf = Chunk<KCH>::Buf;
    Tile<float, XK, XV, KCH> tx;
    Tile<TW, WK, WV, KCH> tw;
    const int nk = (K + kKC - 1) / kKC;
    tx.load(X, sxb, sxk, Bn, K, b0, 0);
    tw.load(W, swm, swk, M, K, m0, 0);
    tx.store(sm);
    tw.store(sm + 2 * kBuf);
    __syncthreads();
    for (int kc = 0; kc < nk; ++kc) {
        const int cur = (kc & 1) * kBuf, nxt = kBuf - cur;
        if (kc + 1 < nk) {
            tx.load(X, sxb, sxk, Bn, K, b0, (kc + 1) * kKC);
            tw.load(W, swm, swk, M, K, m0, (kc + 1) * kKC);
        }
        const unsigned short* xa = sm + cur + (wr + r) * kLd + 8 * h;
        const unsigned short* wb = sm + 2 * kBuf + cur + (wc + r) * kLd + 8 * h;
#pragma unroll
        for (int ks = 0; ks < kKC / 16; ++ks) {
            const u32x4 af = *reinterpret_cast<const u32x4*>(xa + ks * 16);
            const u32x4 bf = *reinterpret_cast<const u32x4*>(wb + ks * 16);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af),
                                                          __builtin_bit_cast(bf16x8, bf), acc, 0,
                                                          0, 0);
        }
        if (kc + 1 < nk) {
            tx.store(sm + nxt);
            tw.store(sm + 2 * kBuf + nxt);
        }
        __syncthreads();
    }
}

__device__ __forceinline__ void apply_epi(const ldm_linear_args_t& a, int b, int m, float pre) {
    float* y = a.Y + (int64_t)b * a.syb + (int64_t)m * a.sym;
    switch (a.epi) {
        case LDM_EPI_BIAS: *y = pre; break;
        case LDM_EPI_SILU:
            if (a.A_out) a.A_out[(int64_t)b * a.sab + m] = pre;
            *y = silu(pre);
            break;
        case LDM_EPI_RESID_SILU:
            if (a.A_out) a.A_out[(int64_t)b * a.sab + m] = pre;
            *y = a.R[(int64_t)b * a.srb + m] + silu(pre);
            break;
        case LDM_EPI_ACCUM: *y = *y + pre; break;
        case LDM_EPI_RELU: *y = fmaxf(pre, 0.f); break;
        case LDM_EPI_MASK_R: *y = a.R[(int64_t)b * a.srb + m] > 0.f ? pre : 0.f; break;
        default: *y = a.R[(int64_t)b * a.srb + m] + pre; break;
    }
}

// gridDim.z > 1: split-K.  Slice z covers k in [z*kc_len, min(K, (z+1)*kc_len)) (kc_len a
// multiple of kKC, every slice non-empty) and stores its raw partial to ws[z][b][m]; the
// epilogue is split_reduce_kernel's.
template <typename TW, bool XK, bool WK, bool XV, bool WV, int KCH>
__global__ __launch_bounds__(256) void linear_mfma_kernel(ldm_linear_args_t a, int kc_len) {
    extern __shared__ __attribute__((aligned(16))) unsigned short sm[];   // kLdsBytes
    // XCD-aware tile order.  Workgroups are dealt round-robin to the 8 XCDs (linear id % 8),
    // each with its own L2.  Give XCD x the contiguous logical tiles [x*T/8, (x+1)*T/8) and
    // walk logical tiles in groups of kGH tile-rows, column-major inside a group: the 32
    // tiles an XCD holds at the training shapes form a 4 x 8 block, so its L2 fetches 4 X
    // row-panels and 8 W column-panels instead of (up to) 32 of each.
    constexpr int kGH = 4;
    const int nx = gridDim.x, ny = gridDim.y, T = nx * ny;
    const int lid = blockIdx.x + nx * blockIdx.y;
    const int t = (T % 8 == 0) ? (lid % 8) * (T / 8) + lid / 8 : lid;
    const int g = t / (kGH * nx), gh = min(kGH, ny - g * kGH), i = t - g * kGH * nx;
    const int b0 = (g * kGH + i % gh) * 64, m0 = (i / gh) * 64;
    const bool split = gridDim.z > 1;
    const int kb = blockIdx.z * kc_len, kl = min(a.K - kb, kc_len);
    const TW* W = reinterpret_cast<const TW*>(a.W);
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    mfma_segment<TW, XK, WK, XV, WV, KCH>(acc, sm, a.X + (int64_t)kb * a.sxk, a.sxb, a.sxk,
                                     W + (int64_t)kb * a.swk, a.swm, a.swk, kl, a.Bn, a.M, b0,
                                     m0);
    if (a.K2 > 0)
        mfma_segment<TW, XK, WK, XV, WV, KCH>(acc, sm, a.X2, a.sx2b, a.sx2k, a.W2, a.sw2m, a.sw2k,
                                         a.K2, a.Bn, a.M, b0, m0);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m = m0 + (wave & 1) * 32 + (lane & 31);
    if (m >= a.M) return;
    float* part = a.ws + (size_t)blockIdx.z * a.Bn * a.M;
    const float bias = (!split && a.bias) ? a.bias[m] : 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int b = b0 + (wave >> 1) * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
        if (b >= a.Bn) continue;
        if (split) part[(size_t)b * a.M + m] = acc[v];
        else apply_epi(a, b, m, acc[v] + bias);
    }
}

// Split-K second pass: the slices' partials summed in slice order, then the epilogue.
__global__ void split_reduce_kernel(ldm_linear_args_t a, int nz) {
    const int64_t n = (int64_t)a.Bn * a.M;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.f;
    for (int z = 0; z < nz; ++z) s += a.ws[(size_t)z * n + i];
    const int b = (int)(i / a.M), m = (int)(i - (int64_t)b * a.M);
    apply_epi(a, b, m, s + (a.bias ? a.bias[m] : 0.f));
}

// Split plan: slices so that tiles x slices reaches ~4 workgroups per CU, each slice at
// least 8 chunks deep.  {slices, slice length}; slices == 1: no split.
struct SplitPlan { int nz, kc_len; };
SplitPlan split_plan(const ldm_linear_args_t& a) {
    const int64_t tiles = (int64_t)((a.M + 63) / 64) * ((a.Bn + 63) / 64);
    if (a.compute != LDM_COMPUTE_BF16 || a.K2 > 0 || tiles >= 256) return {1, a.K};
    int nz = (int)std::min<int64_t>((1024 + tiles - 1) / tiles, a.K / (8 * kKCSplit));
    nz = std::min(nz, 256);
    if (nz < 2) return {1, a.K};
    const int kc = ((a.K + nz - 1) / nz + kKCSplit - 1) / kKCSplit * kKCSplit;
    return {(a.K + kc - 1) / kc, kc};
}

// Can an operand use 16-byte vector loads?  Its contiguous dimension must have stride 1 and
// an extent that is a multiple of the vector, the other stride and the base 16-byte aligned.
bool vec_ok(const void* P, int64_t s_row, int64_t s_k, int rows, int K, int esize) {
    const int epv = 16 / esize;
    const bool kc = s_k == 1;
    const int64_t other = kc ? s_row : s_k;
    const int ext = kc ? K : rows;
    return (kc || s_row == 1) && (((uintptr_t)P) & 15) == 0 && other % epv == 0 &&
           ext % epv == 0;
}

template <typename TW, bool XK, bool WK, bool XV, bool WV, int KCH>
int launch_one(const ldm_linear_args_t& a, const SplitPlan& sp, hipStream_t s) {
    auto* k = &linear_mfma_kernel<TW, XK, WK, XV, WV, KCH>;
    constexpr int kLdsBytes = Chunk<KCH>::LdsBytes;
    LDM_TRY((set_max_lds_once<&linear_mfma_kernel<TW, XK, WK, XV, WV, KCH>>(
        kLdsBytes, "ldm_linear (mfma)")));
    const dim3 grid((a.M + 63) / 64, (a.Bn + 63) / 64, sp.nz);
    hipLaunchKernelGGL(k, grid, dim3(256), kLdsBytes, s, a, sp.kc_len);
    if (sp.nz > 1) {
        const int64_t n = (int64_t)a.Bn * a.M;
        hipLaunchKernelGGL(split_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                           s, a, sp.nz);
    }
    return 0;
}

template <typename TW, bool XK, bool WK, int KCH>
int launch_mfma4(const ldm_linear_args_t& a, const SplitPlan& sp, bool xv, bool wv,
                 hipStream_t s) {
    if (xv && wv) return launch_one<TW, XK, WK, true, true, KCH>(a, sp, s);
    if (xv) return launch_one<TW, XK, WK, true, false, KCH>(a, sp, s);
    if (wv) return launch_one<TW, XK, WK, false, true, KCH>(a, sp, s);
    return launch_one<TW, XK, WK, false, false, KCH>(a, sp, s);
}

// Chunk depth by grid size (measured: auto-decoder 1M x 512 x 512 products, 131k workgroups,
// 96.9 -> 81.2 ms/step with 64; config-2 training, 256 workgroups, 1012 -> 911 steps/s with 64).
constexpr int64_t kShallowChunkMinWG = 2048;

template <typename TW, bool XK, bool WK>
int launch_mfma3(const ldm_linear_args_t& a, bool xv, bool wv, hipStream_t s) {
    SplitPlan sp = split_plan(a);
    if (sp.nz > 1 && (!a.ws || a.ws_floats < (int64_t)sp.nz * a.Bn * a.M)) sp = {1, a.K};
    const int64_t wgs = (int64_t)((a.M + 63) / 64) * ((a.Bn + 63) / 64) * sp.nz;
    if (wgs >= kShallowChunkMinWG) return launch_mfma4<TW, XK, WK, 64>(a, sp, xv, wv, s);
    return launch_mfma4<TW, XK, WK, 128>(a, sp, xv, wv, s);
}

template <typename TW>
int launch_mfma(const ldm_linear_args_t& a, bool xk, bool wk, hipStream_t s) {
    const int es = (int)sizeof(TW);
    const bool vec_on = dev_knob("LDM_LINEAR_VEC", 1) != 0;   // dev A/B: 0 -> scalar tiles
    bool xv = vec_on && vec_ok(a.X, a.sxb, a.sxk, a.Bn, a.K, 4);
    bool wv = vec_on && vec_ok(a.W, a.swm, a.swk, a.M, a.K, es);
    if (a.K2 > 0) {
        xv = xv && vec_ok(a.X2, a.sx2b, a.sx2k, a.Bn, a.K2, 4);
        wv = wv && vec_ok(a.W2, a.sw2m, a.sw2k, a.M, a.K2, es);
    }
    if (xk && wk) return launch_mfma3<TW, true, true>(a, xv, wv, s);
    if (xk) return launch_mfma3<TW, true, false>(a, xv, wv, s);
    if (wk) return launch_mfma3<TW, false, true>(a, xv, wv, s);
    return launch_mfma3<TW, false, false>(a, xv, wv, s);
}

}  // namespace

int64_t linear_mfma_ws_floats(const ldm_linear_args_t& a) {
    const SplitPlan sp = split_plan(a);
    return sp.nz > 1 ? (int64_t)sp.nz * a.Bn * a.M : 0;
}

namespace {
// K == 1 (a rank-1 product, e.g. the auto-decoder's last-layer input gradient g W8): one
// product per output, so no tile, LDS or MFMA.  Same numbers as the matrix-core kernel: the
// operands rounded to bf16 (RNE) and multiplied in fp32 (exact for two bf16 values), then the
// shared epilogue with the bias.  Memory-bound; one thread per output, m fastest.
template <typename TW>
__global__ __launch_bounds__(256) void outer_k1_kernel(ldm_linear_args_t a) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)a.Bn * a.M) return;
    const int b = (int)(i / a.M), m = (int)(i - (int64_t)b * a.M);
    const float x = bf16_to_f32((unsigned short)(pack_bf16(a.X[(int64_t)b * a.sxb], 0.f) & 0xffffu));
    const float w = bf16_to_f32((unsigned short)(pack_bf16(
        ld_elem(reinterpret_cast<const TW*>(a.W), (int64_t)m * a.swm), 0.f) & 0xffffu));
    apply_epi(a, b, m, x * w + (a.bias ? a.bias[m] : 0.f));
}
}  // namespace

int linear_mfma(const ldm_linear_args_t& a, hipStream_t s) {
    if (a.K == 1 && a.K2 == 0) {
        const int64_t n = (int64_t)a.Bn * a.M;
        const dim3 grid((unsigned)((n + 255) / 256));
        if (a.w_dtype == LDM_BF16) hipLaunchKernelGGL(outer_k1_kernel<unsigned short>, grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL(outer_k1_kernel<float>, grid, dim3(256), 0, s, a);
        return launch_status("ldm_linear (mfma, K=1)");
    }
    const bool xk = a.sxk == 1, wk = a.swk == 1;
    const int e = a.w_dtype == LDM_BF16 ? launch_mfma<unsigned short>(a, xk, wk, s)
                                        : launch_mfma<float>(a, xk, wk, s);
    if (e) return e;
    return launch_status("ldm_linear (mfma)");
}

}  // namespace ldm
