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
// MFMA tile.  K advances in 64-wide chunks through two LDS buffers: the next chunk's global
// loads are issued into registers before the current chunk's MFMAs (one barrier per chunk).
// An operand contiguous along k is loaded 8 k per thread (one 16-byte LDS store); a
// transposed view (contiguous along rows) is loaded 8 rows per thread and scattered.
// LDS rows are 64 + 8 bf16 (144 B), so the 16-byte fragment reads of a 16-lane group land
// in distinct banks.
#include "ldm_internal.h"
#include "ddpm_common.h"

namespace ldm {
namespace {

constexpr int kKC = 64;              // k per chunk
constexpr int kLd = kKC + 8;         // LDS row pitch (bf16 elements)

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

// One operand tile: rows [r0, r0+64) x k [k0, k0+64) of a strided matrix, 16 values per
// thread held in registers between the load and the LDS store.
template <typename T, bool KC>
struct Tile {
    float v[16];
    __device__ __forceinline__ void load(const T* __restrict__ P, int64_t sr, int64_t sk,
                                         int rows, int K, int r0, int k0) {
        const int t = threadIdx.x;
        if (KC) {   // contiguous along k: thread -> (row t/4, k 16*(t%4) .. +15)
            const int r = r0 + (t >> 2), kb = k0 + (t & 3) * 16;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int k = kb + j;
                v[j] = (r < rows && k < K) ? ld_elem(P, (int64_t)r * sr + (int64_t)k * sk) : 0.f;
            }
        } else {    // contiguous along rows: thread -> (k t/4, rows 16*(t%4) .. +15)
            const int k = k0 + (t >> 2), rb = r0 + (t & 3) * 16;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int r = rb + j;
                v[j] = (r < rows && k < K) ? ld_elem(P, (int64_t)r * sr + (int64_t)k * sk) : 0.f;
            }
        }
    }
    __device__ __forceinline__ void store(unsigned short* __restrict__ S) const {
        const int t = threadIdx.x;
        if (KC) {
            const int r = t >> 2, kb = (t & 3) * 16;
            u32x4 w0, w1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w0[q] = pack_bf16(v[2 * q], v[2 * q + 1]);
                w1[q] = pack_bf16(v[8 + 2 * q], v[8 + 2 * q + 1]);
            }
            *reinterpret_cast<u32x4*>(S + r * kLd + kb) = w0;
            *reinterpret_cast<u32x4*>(S + r * kLd + kb + 8) = w1;
        } else {
            const int k = t >> 2, rb = (t & 3) * 16;
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                const unsigned p = pack_bf16(v[j], v[j + 1]);
                S[(rb + j) * kLd + k] = (unsigned short)(p & 0xffffu);
                S[(rb + j + 1) * kLd + k] = (unsigned short)(p >> 16);
            }
        }
    }
};

template <typename TW, bool XK, bool WK>
__device__ __forceinline__ void mfma_segment(f32x16& acc, unsigned short* __restrict__ sm,
                                             const float* X, int64_t sxb, int64_t sxk,
                                             const void* Wv, int64_t swm, int64_t swk, int K,
                                             int Bn, int M, int b0, int m0) {
    const TW* W = reinterpret_cast<const TW*>(Wv);
    unsigned short* Xs[2] = {sm, sm + 64 * kLd};
    unsigned short* Ws[2] = {sm + 2 * 64 * kLd, sm + 3 * 64 * kLd};
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
    const int r = lane & 31, h = lane >> 5;
    Tile<float, XK> tx;
    Tile<TW, WK> tw;
    const int nk = (K + kKC - 1) / kKC;
    tx.load(X, sxb, sxk, Bn, K, b0, 0);
    tw.load(W, swm, swk, M, K, m0, 0);
    tx.store(Xs[0]);
    tw.store(Ws[0]);
    __syncthreads();
    for (int kc = 0; kc < nk; ++kc) {
        const int cur = kc & 1;
        if (kc + 1 < nk) {
            tx.load(X, sxb, sxk, Bn, K, b0, (kc + 1) * kKC);
            tw.load(W, swm, swk, M, K, m0, (kc + 1) * kKC);
        }
#pragma unroll
        for (int ks = 0; ks < kKC / 16; ++ks) {
            const u32x4 af = *reinterpret_cast<const u32x4*>(Xs[cur] + (wr + r) * kLd + ks * 16 + 8 * h);
            const u32x4 bf = *reinterpret_cast<const u32x4*>(Ws[cur] + (wc + r) * kLd + ks * 16 + 8 * h);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af),
                                                          __builtin_bit_cast(bf16x8, bf), acc, 0,
                                                          0, 0);
        }
        if (kc + 1 < nk) {
            tx.store(Xs[cur ^ 1]);
            tw.store(Ws[cur ^ 1]);
        }
        __syncthreads();
    }
}

template <typename TW, bool XK, bool WK>
__global__ __launch_bounds__(256) void linear_mfma_kernel(ldm_linear_args_t a) {
    __shared__ __attribute__((aligned(16))) unsigned short sm[4 * 64 * kLd];
    const int b0 = blockIdx.y * 64, m0 = blockIdx.x * 64;
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    mfma_segment<TW, XK, WK>(acc, sm, a.X, a.sxb, a.sxk, a.W, a.swm, a.swk, a.K, a.Bn, a.M, b0, m0);
    if (a.K2 > 0)
        mfma_segment<TW, XK, WK>(acc, sm, a.X2, a.sx2b, a.sx2k, a.W2, a.sw2m, a.sw2k, a.K2, a.Bn,
                                 a.M, b0, m0);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m = m0 + (wave & 1) * 32 + (lane & 31);
    if (m >= a.M) return;
    const float bias = a.bias ? a.bias[m] : 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int b = b0 + (wave >> 1) * 32 + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
        if (b >= a.Bn) continue;
        const float pre = acc[v] + bias;
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
            default: *y = a.R[(int64_t)b * a.srb + m] + pre; break;
        }
    }
}

template <typename TW>
void launch_mfma(const ldm_linear_args_t& a, bool xk, bool wk, hipStream_t s) {
    const dim3 grid((a.M + 63) / 64, (a.Bn + 63) / 64);
    if (xk && wk) hipLaunchKernelGGL((linear_mfma_kernel<TW, true, true>), grid, dim3(256), 0, s, a);
    else if (xk) hipLaunchKernelGGL((linear_mfma_kernel<TW, true, false>), grid, dim3(256), 0, s, a);
    else if (wk) hipLaunchKernelGGL((linear_mfma_kernel<TW, false, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((linear_mfma_kernel<TW, false, false>), grid, dim3(256), 0, s, a);
}

}  // namespace

int linear_mfma(const ldm_linear_args_t& a, hipStream_t s) {
    const bool xk = a.sxk == 1, wk = a.swk == 1;
    if (a.w_dtype == LDM_BF16) launch_mfma<unsigned short>(a, xk, wk, s);
    else launch_mfma<float>(a, xk, wk, s);
    return launch_status("ldm_linear (mfma)");
}

}  // namespace ldm
