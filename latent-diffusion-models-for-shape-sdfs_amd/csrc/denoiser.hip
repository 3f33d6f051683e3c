// DDPM side of the hot path on MI355X (gfx950): SURVEY.md §8(a) rows A5-A10.
//
//   ddpm_step_kernel        A8 reverse step (fixed op order, no contraction: bit-exact vs
//                           oracle/ref_cpu.py ddpm_step in fp32)
//   q_sample_kernel         A9 forward noising
//   mse_loss_kernel         A9 eps-MSE loss and its gradient (deterministic single-block sum)
//   small_linear_kernel     A6 for the sampling batch (B <= 16): one wave per output row,
//                           activations staged once in LDS, k split over the 64 lanes, wave
//                           shuffle reduction, fused epilogue (bias | residual+SiLU+E[t] |
//                           out-projection + DDPM step).  VALU fp32 accumulate; MFMA is kept
//                           for the decoder (north star).
//   linear_tiled_kernel     A6/A7 for training batches: 64x64 register-tiled VALU GEMM with
//                           LDS-staged operand tiles, arbitrary strides (X W^T, G W, G^T X).
//   silu_bwd / colsum / gather_rows   A7 elementwise pieces, A5 embedding lookup.
#include "ldm_internal.h"
#include "ddpm_common.h"

#include <math.h>
#include <stdlib.h>

namespace ldm {
namespace {

__global__ void ddpm_step_kernel(const float* __restrict__ c1t, const float* __restrict__ c2t,
                                 const float* __restrict__ sgt, int t,
                                 const float* __restrict__ x, const float* __restrict__ eps,
                                 const float* __restrict__ z, int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = ddpm_update(x[i], eps[i], t > 0 ? z[i] : 0.f, c1t[t], c2t[t], sgt[t], t > 0);
}

__global__ void q_sample_kernel(const float* __restrict__ sab, const float* __restrict__ s1mab,
                                const float* __restrict__ x0, const float* __restrict__ eps,
                                const int32_t* __restrict__ t, int B, int D,
                                float* __restrict__ xt) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * D) return;
    const int tb = t[i / D];
    const float a = sab[tb] * x0[i];
    const float b = s1mab[tb] * eps[i];
    xt[i] = a + b;
}

// One block, fixed summation order (deterministic).  The loads of U groups are issued before
// any is consumed (index clamped, use predicated) so the block pays one memory round trip per
// U x 1024 groups instead of one per group.  V4: groups of 4 via 16-byte loads (all pointers
// 16-byte aligned), the n % 4 tail scalar.
template <bool V4>
__global__ __launch_bounds__(1024) void mse_loss_kernel(const float* __restrict__ eh,
                                                        const float* __restrict__ e, int n,
                                                        float* __restrict__ loss,
                                                        float* __restrict__ grad) {
    __shared__ float red[1024];
    constexpr int U = 8;
    constexpr int G = V4 ? 4 : 1;
    typedef float vec_t __attribute__((ext_vector_type(G)));
    float s = 0.f;
    const float g = 2.f / (float)n;
    const int ng = n / G;
    const vec_t* A = reinterpret_cast<const vec_t*>(eh);
    const vec_t* Bv = reinterpret_cast<const vec_t*>(e);
    const int tid = (int)threadIdx.x;
    for (int base = 0; base < ng; base += 1024 * U) {
        vec_t a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * 1024 + tid;
            const int ii = i < ng ? i : 0;
            a[u] = A[ii];
            b[u] = Bv[ii];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * 1024 + tid;
            if (i < ng) {
                const vec_t d = a[u] - b[u];
#pragma unroll
                for (int q = 0; q < G; ++q) s = fmaf(d[q], d[q], s);
                if (grad) reinterpret_cast<vec_t*>(grad)[i] = g * d;
            }
        }
    }
    if (tid < n - ng * G) {
        const int i = ng * G + tid;
        const float d = eh[i] - e[i];
        s = fmaf(d, d, s);
        if (grad) grad[i] = g * d;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = red[0] / (float)n;
}

// ------------------------------------------------------------------------------------------
// Small-batch fused linear (sampling).  Y[b][m] = epi(sum_k X[b][k] W[m*ldw + k]).
// ------------------------------------------------------------------------------------------
enum SmallEpi { SE_BIAS = 0, SE_BLOCK = 1, SE_STEP = 2 };

struct SmallArgs {
    const float* X;      // [B][K]
    const void* W;       // rows of length >= K, row stride ldw
    const float* bias;   // [M]: b (SE_BIAS / SE_STEP) or E_k[t] (SE_BLOCK, includes b_k)
    float* Y;            // [B][M]
    const float* xlat;   // SE_STEP: x_t [B][M]
    const float* z;      // SE_STEP: noise [B][M]
    const float* c1t;    // SE_STEP: schedule tables (device), read at index t
    const float* c2t;
    const float* sgt;
    int B, M, K, ldw;
    int t;
};

constexpr int kSmallMaxB = 16;

template <typename TW, int EPI>
__global__ __launch_bounds__(256) void small_linear_kernel(SmallArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs[];   // [B][K]
    const int nx = a.B * a.K;
    for (int i = threadIdx.x * 4; i < nx; i += 256 * 4)
        *reinterpret_cast<f32x4*>(xs + i) = *reinterpret_cast<const f32x4*>(a.X + i);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= a.M) return;
    float acc[kSmallMaxB];
#pragma unroll
    for (int b = 0; b < kSmallMaxB; ++b) acc[b] = 0.f;
    const int nch = a.K >> 3;   // 8-element chunks
    for (int c = lane; c < nch; c += 64) {
        float w[8];
        if (sizeof(TW) == 2) {
            const uint4 u = *reinterpret_cast<const uint4*>(
                reinterpret_cast<const unsigned short*>(a.W) + (size_t)m * a.ldw + c * 8);
            w[0] = bf16_to_f32(u.x & 0xffff); w[1] = bf16_to_f32(u.x >> 16);
            w[2] = bf16_to_f32(u.y & 0xffff); w[3] = bf16_to_f32(u.y >> 16);
            w[4] = bf16_to_f32(u.z & 0xffff); w[5] = bf16_to_f32(u.z >> 16);
            w[6] = bf16_to_f32(u.w & 0xffff); w[7] = bf16_to_f32(u.w >> 16);
        } else {
            const float* wp = reinterpret_cast<const float*>(a.W) + (size_t)m * a.ldw + c * 8;
            const f32x4 w0 = *reinterpret_cast<const f32x4*>(wp);
            const f32x4 w1 = *reinterpret_cast<const f32x4*>(wp + 4);
            w[0] = w0[0]; w[1] = w0[1]; w[2] = w0[2]; w[3] = w0[3];
            w[4] = w1[0]; w[5] = w1[1]; w[6] = w1[2]; w[7] = w1[3];
        }
#pragma unroll
        for (int b = 0; b < kSmallMaxB; ++b) {
            if (b < a.B) {
                const f32x4 x0 = *reinterpret_cast<const f32x4*>(xs + b * a.K + c * 8);
                const f32x4 x1 = *reinterpret_cast<const f32x4*>(xs + b * a.K + c * 8 + 4);
                float s = acc[b];
                s = fmaf(w[0], x0[0], s); s = fmaf(w[1], x0[1], s);
                s = fmaf(w[2], x0[2], s); s = fmaf(w[3], x0[3], s);
                s = fmaf(w[4], x1[0], s); s = fmaf(w[5], x1[1], s);
                s = fmaf(w[6], x1[2], s); s = fmaf(w[7], x1[3], s);
                acc[b] = s;
            }
        }
    }
    float mine = 0.f;   // lane b keeps row b's total
#pragma unroll
    for (int b = 0; b < kSmallMaxB; ++b) {
        if (b < a.B) {
            float v = acc[b];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == b) mine = v;
        }
    }
    if (lane < a.B) {
        const int b = lane;
        const float pre = mine + a.bias[m];
        if (EPI == SE_BIAS) {
            a.Y[(size_t)b * a.M + m] = pre;
        } else if (EPI == SE_BLOCK) {
            a.Y[(size_t)b * a.M + m] = xs[b * a.K + m] + silu(pre);
        } else {
            const size_t i = (size_t)b * a.M + m;
            const bool noise = a.t > 0;
            a.Y[i] = ddpm_update(a.xlat[i], pre, noise ? a.z[i] : 0.f, a.c1t[a.t], a.c2t[a.t],
                                 a.sgt[a.t], noise);
        }
    }
}

// v2: one wave per block owns R rows.  All weight and activation loads are issued up front
// (registers, no LDS staging, no barrier), then R*MB partial dot products per lane are
// reduce-scattered across the wave (each butterfly level exchanges only the half a lane gives
// away: 32 shuffles for 4 rows x 8 samples instead of 192), and the lanes that end up owning a
// (row, sample) total run the fused epilogue.  Latency-bound by design.
template <typename TW, int EPI, int R, int MB>
__global__ __launch_bounds__(64) void small_linear_v2(SmallArgs a) {
    constexpr int V = R * MB;                 // values to reduce per lane (power of 2, <= 64)
    static_assert((V & (V - 1)) == 0 && V <= 64, "R*MB must be a power of two <= 64");
    const int lane = threadIdx.x;
    const int m0 = blockIdx.x * R;
    const int nch = a.K >> 3;                 // 8-element chunks; lane takes c = lane + 64 j
    constexpr int MAXJ = 4;                   // K <= 2048
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
        const int c = lane + 64 * j;
        if (64 * j >= nch) break;             // uniform
        const bool on = c < nch;
        float w[R][8];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int m = (m0 + r < a.M) ? m0 + r : a.M - 1;
            if (sizeof(TW) == 2) {
                uint4 u = {0, 0, 0, 0};
                if (on) u = *reinterpret_cast<const uint4*>(
                    reinterpret_cast<const unsigned short*>(a.W) + (size_t)m * a.ldw + c * 8);
                w[r][0] = bf16_to_f32(u.x & 0xffff); w[r][1] = bf16_to_f32(u.x >> 16);
                w[r][2] = bf16_to_f32(u.y & 0xffff); w[r][3] = bf16_to_f32(u.y >> 16);
                w[r][4] = bf16_to_f32(u.z & 0xffff); w[r][5] = bf16_to_f32(u.z >> 16);
                w[r][6] = bf16_to_f32(u.w & 0xffff); w[r][7] = bf16_to_f32(u.w >> 16);
            } else {
                f32x4 w0 = {0, 0, 0, 0}, w1 = {0, 0, 0, 0};
                if (on) {
                    const float* wp = reinterpret_cast<const float*>(a.W) + (size_t)m * a.ldw + c * 8;
                    w0 = *reinterpret_cast<const f32x4*>(wp);
                    w1 = *reinterpret_cast<const f32x4*>(wp + 4);
                }
                w[r][0] = w0[0]; w[r][1] = w0[1]; w[r][2] = w0[2]; w[r][3] = w0[3];
                w[r][4] = w1[0]; w[r][5] = w1[1]; w[r][6] = w1[2]; w[r][7] = w1[3];
            }
        }
#pragma unroll
        for (int b = 0; b < MB; ++b) {
            f32x4 x0 = {0, 0, 0, 0}, x1 = {0, 0, 0, 0};
            if (on && b < a.B) {
                x0 = *reinterpret_cast<const f32x4*>(a.X + (size_t)b * a.K + c * 8);
                x1 = *reinterpret_cast<const f32x4*>(a.X + (size_t)b * a.K + c * 8 + 4);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float s = acc[r * MB + b];
                s = fmaf(w[r][0], x0[0], s); s = fmaf(w[r][1], x0[1], s);
                s = fmaf(w[r][2], x0[2], s); s = fmaf(w[r][3], x0[3], s);
                s = fmaf(w[r][4], x1[0], s); s = fmaf(w[r][5], x1[1], s);
                s = fmaf(w[r][6], x1[2], s); s = fmaf(w[r][7], x1[3], s);
                acc[r * MB + b] = s;
            }
        }
    }
    // reduce-scatter: at level lv (offset o = 32 >> lv) a lane keeps the half of its n = V >> lv
    // values selected by lane & o and adds its partner's copy of that half.
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {
        const int o = 32 >> lv;
        const int n = V >> lv;                // compile-time after unrolling
        const bool upper = (lane & o) != 0;
        if (n > 1) {
            const int half = n >> 1;
#pragma unroll
            for (int i = 0; i < half; ++i) {
                const float send = upper ? acc[i] : acc[i + half];
                const float keep = upper ? acc[i + half] : acc[i];
                acc[i] = keep + xor_lane(send, o, lane);
            }
        } else {
            acc[0] += xor_lane(acc[0], o, lane);
        }
    }
    // lane owns value index idx = (lane >> (6 - log2 V)) in natural order: idx = r*MB + b
    constexpr int LV = (V >= 64) ? 6 : (V >= 32) ? 5 : (V >= 16) ? 4 : (V >= 8) ? 3 : (V >= 4) ? 2 : (V >= 2) ? 1 : 0;
    const int idx = lane >> (6 - LV);
    const bool writer = (lane & ((1 << (6 - LV)) - 1)) == 0;
    const int r = idx / MB, b = idx - (idx / MB) * MB;
    const int m = m0 + r;
    if (writer && b < a.B && m < a.M) {
        const float pre = acc[0] + a.bias[m];
        const size_t i = (size_t)b * a.M + m;
        if (EPI == SE_BIAS) {
            a.Y[i] = pre;
        } else if (EPI == SE_BLOCK) {
            a.Y[i] = a.X[(size_t)b * a.K + m] + silu(pre);
        } else {
            const bool noise = a.t > 0;
            a.Y[i] = ddpm_update(a.xlat[i], pre, noise ? a.z[i] : 0.f, a.c1t[a.t], a.c2t[a.t],
                                 a.sgt[a.t], noise);
        }
    }
}

// v3: v1's shape (one wave per output row, 4 rows per 256-thread block, activations staged
// once per block in LDS) with the row's weight loads issued BEFORE the activation staging and
// its barrier (the two memory latencies overlap), and a reduce-scatter over the MB samples.
template <typename TW, int EPI, int MB>
__global__ __launch_bounds__(256) void small_linear_v3(SmallArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs[];   // [B][K]
    const int lane = threadIdx.x & 63;
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int mm = m < a.M ? m : a.M - 1;
    const int nch = a.K >> 3;
    constexpr int MAXJ = 4;                    // K <= 2048
    float w[MAXJ][8];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
        const int c = lane + 64 * j;
        const bool on = c < nch;
        if (sizeof(TW) == 2) {
            uint4 u = {0, 0, 0, 0};
            if (on) u = *reinterpret_cast<const uint4*>(
                reinterpret_cast<const unsigned short*>(a.W) + (size_t)mm * a.ldw + c * 8);
            w[j][0] = bf16_to_f32(u.x & 0xffff); w[j][1] = bf16_to_f32(u.x >> 16);
            w[j][2] = bf16_to_f32(u.y & 0xffff); w[j][3] = bf16_to_f32(u.y >> 16);
            w[j][4] = bf16_to_f32(u.z & 0xffff); w[j][5] = bf16_to_f32(u.z >> 16);
            w[j][6] = bf16_to_f32(u.w & 0xffff); w[j][7] = bf16_to_f32(u.w >> 16);
        } else {
            f32x4 w0 = {0, 0, 0, 0}, w1 = {0, 0, 0, 0};
            if (on) {
                const float* wp = reinterpret_cast<const float*>(a.W) + (size_t)mm * a.ldw + c * 8;
                w0 = *reinterpret_cast<const f32x4*>(wp);
                w1 = *reinterpret_cast<const f32x4*>(wp + 4);
            }
            w[j][0] = w0[0]; w[j][1] = w0[1]; w[j][2] = w0[2]; w[j][3] = w0[3];
            w[j][4] = w1[0]; w[j][5] = w1[1]; w[j][6] = w1[2]; w[j][7] = w1[3];
        }
    }
    const int nx = a.B * a.K;
    for (int i = threadIdx.x * 4; i < nx; i += 256 * 4)
        *reinterpret_cast<f32x4*>(xs + i) = *reinterpret_cast<const f32x4*>(a.X + i);
    __syncthreads();
    float acc[MB];
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[b] = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
        const int c = lane + 64 * j;
        if (64 * j >= nch) break;
        if (c < nch) {
#pragma unroll
            for (int b = 0; b < MB; ++b) {
                if (b < a.B) {
                    const f32x4 x0 = *reinterpret_cast<const f32x4*>(xs + b * a.K + c * 8);
                    const f32x4 x1 = *reinterpret_cast<const f32x4*>(xs + b * a.K + c * 8 + 4);
                    float t = acc[b];
                    t = fmaf(w[j][0], x0[0], t); t = fmaf(w[j][1], x0[1], t);
                    t = fmaf(w[j][2], x0[2], t); t = fmaf(w[j][3], x0[3], t);
                    t = fmaf(w[j][4], x1[0], t); t = fmaf(w[j][5], x1[1], t);
                    t = fmaf(w[j][6], x1[2], t); t = fmaf(w[j][7], x1[3], t);
                    acc[b] = t;
                }
            }
        }
    }
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {
        const int o = 32 >> lv;
        const int n = MB >> lv;
        const bool upper = (lane & o) != 0;
        if (n > 1) {
            const int half = n >> 1;
#pragma unroll
            for (int i = 0; i < half; ++i) {
                const float send = upper ? acc[i] : acc[i + half];
                const float keep = upper ? acc[i + half] : acc[i];
                acc[i] = keep + xor_lane(send, o, lane);
            }
        } else {
            acc[0] += xor_lane(acc[0], o, lane);
        }
    }
    constexpr int LB = (MB >= 16) ? 4 : 3;
    const int b = lane >> (6 - LB);
    const bool writer = (lane & ((1 << (6 - LB)) - 1)) == 0;
    if (m < a.M && writer && b < a.B) {
        const float pre = acc[0] + a.bias[m];
        const size_t i = (size_t)b * a.M + m;
        if (EPI == SE_BIAS) {
            a.Y[i] = pre;
        } else if (EPI == SE_BLOCK) {
            a.Y[i] = xs[b * a.K + m] + silu(pre);
        } else {
            const bool noise = a.t > 0;
            a.Y[i] = ddpm_update(a.xlat[i], pre, noise ? a.z[i] : 0.f, a.c1t[a.t], a.c2t[a.t],
                                 a.sgt[a.t], noise);
        }
    }
}

// v4: v3 with every global load unconditional (index clamped, value selected afterwards) so a
// wave issues all of its loads back to back -- a load under a divergent branch makes hipcc
// wait vmcnt(0) before leaving the branch, one round trip per load -- and the activation
// staging batched 8 x 16 B per thread before any LDS store.  NJ = ceil(K / 8 / 64) weight
// chunks per lane (K <= 2048).
template <typename TW, int EPI, int MB, int NJ>
__global__ __launch_bounds__(256) void small_linear_v4(SmallArgs a) {
    extern __shared__ __attribute__((aligned(16))) float xs[];   // [B][K]
    const int lane = threadIdx.x & 63;
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int mm = m < a.M ? m : a.M - 1;
    const int nch = a.K >> 3;
    float w[NJ][8];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int c = lane + 64 * j;
        const bool on = c < nch;
        const size_t off = (size_t)mm * a.ldw + (on ? c : 0) * 8;
        if constexpr (sizeof(TW) == 2) {
            uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const unsigned short*>(a.W) + off);
            const unsigned q[4] = {on ? u.x : 0u, on ? u.y : 0u, on ? u.z : 0u, on ? u.w : 0u};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[j][2 * i] = __builtin_bit_cast(float, q[i] << 16);
                w[j][2 * i + 1] = __builtin_bit_cast(float, q[i] & 0xffff0000u);
            }
        } else {
            const float* wp = reinterpret_cast<const float*>(a.W) + off;
            const f32x4 w0 = *reinterpret_cast<const f32x4*>(wp);
            const f32x4 w1 = *reinterpret_cast<const f32x4*>(wp + 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[j][i] = on ? w0[i] : 0.f;
                w[j][4 + i] = on ? w1[i] : 0.f;
            }
        }
    }
    const int n4 = (a.B * a.K) >> 2;
    const f32x4* X4 = reinterpret_cast<const f32x4*>(a.X);
    for (int base = 0; base < n4; base += 256 * 8) {
        f32x4 t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = base + u * 256 + (int)threadIdx.x;
            t[u] = X4[i < n4 ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = base + u * 256 + (int)threadIdx.x;
            if (i < n4) reinterpret_cast<f32x4*>(xs)[i] = t[u];
        }
    }
    __syncthreads();
    float acc[MB];
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[b] = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int c = lane + 64 * j;
        const int cc = c < nch ? c : 0;       // off lanes: zero weights times a valid row
#pragma unroll
        for (int b = 0; b < MB; ++b) {
            const int bb = b < a.B ? b : 0;   // rows past B are never written out
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(xs + bb * a.K + cc * 8);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(xs + bb * a.K + cc * 8 + 4);
            float t = acc[b];
            t = fmaf(w[j][0], x0[0], t); t = fmaf(w[j][1], x0[1], t);
            t = fmaf(w[j][2], x0[2], t); t = fmaf(w[j][3], x0[3], t);
            t = fmaf(w[j][4], x1[0], t); t = fmaf(w[j][5], x1[1], t);
            t = fmaf(w[j][6], x1[2], t); t = fmaf(w[j][7], x1[3], t);
            acc[b] = t;
        }
    }
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {
        const int o = 32 >> lv;
        const int n = MB >> lv;
        const bool upper = (lane & o) != 0;
        if (n > 1) {
            const int half = n >> 1;
#pragma unroll
            for (int i = 0; i < half; ++i) {
                const float send = upper ? acc[i] : acc[i + half];
                const float keep = upper ? acc[i + half] : acc[i];
                acc[i] = keep + xor_lane(send, o, lane);
            }
        } else {
            acc[0] += xor_lane(acc[0], o, lane);
        }
    }
    constexpr int LB = (MB >= 16) ? 4 : 3;
    const int b = lane >> (6 - LB);
    const bool writer = (lane & ((1 << (6 - LB)) - 1)) == 0;
    if (m < a.M && writer && b < a.B) {
        const float pre = acc[0] + a.bias[m];
        const size_t i = (size_t)b * a.M + m;
        if (EPI == SE_BIAS) {
            a.Y[i] = pre;
        } else if (EPI == SE_BLOCK) {
            a.Y[i] = xs[b * a.K + m] + silu(pre);
        } else {
            const bool noise = a.t > 0;
            a.Y[i] = ddpm_update(a.xlat[i], pre, noise ? a.z[i] : 0.f, a.c1t[a.t], a.c2t[a.t],
                                 a.sgt[a.t], noise);
        }
    }
}

template <typename TW, int EPI, int MB>
void launch_small_v4_nj(const SmallArgs& a, hipStream_t s) {
    const size_t lds = (size_t)a.B * a.K * sizeof(float);
    const dim3 grid((a.M + 3) / 4);
    const int nj = ((a.K >> 3) + 63) / 64;
    if (nj <= 1) hipLaunchKernelGGL((small_linear_v4<TW, EPI, MB, 1>), grid, dim3(256), lds, s, a);
    else if (nj <= 2) hipLaunchKernelGGL((small_linear_v4<TW, EPI, MB, 2>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((small_linear_v4<TW, EPI, MB, 4>), grid, dim3(256), lds, s, a);
}

template <typename TW, int EPI>
void launch_small_v4(const SmallArgs& a, hipStream_t s) {
    if (a.B <= 8) launch_small_v4_nj<TW, EPI, 8>(a, s);
    else launch_small_v4_nj<TW, EPI, 16>(a, s);
}

template <typename TW, int EPI>
void launch_small_v3(const SmallArgs& a, hipStream_t s) {
    const size_t lds = (size_t)a.B * a.K * sizeof(float);
    const dim3 grid((a.M + 3) / 4);
    if (a.B <= 8)
        hipLaunchKernelGGL((small_linear_v3<TW, EPI, 8>), grid, dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL((small_linear_v3<TW, EPI, 16>), grid, dim3(256), lds, s, a);
}

int small_version() {
    const int v = dev_knob("LDM_SMALL_LINEAR", 4);   // development A/B knob: 1, 2, 3, 4 (default)
    return (v >= 1 && v <= 4) ? v : 4;
}

template <typename TW, int EPI>
void launch_small_v2(const SmallArgs& a, hipStream_t s) {
    constexpr int R = 4;
    const dim3 grid((a.M + R - 1) / R);
    if (a.B <= 8)
        hipLaunchKernelGGL((small_linear_v2<TW, EPI, R, 8>), grid, dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((small_linear_v2<TW, EPI, R, 16>), grid, dim3(64), 0, s, a);
}

template <int EPI>
int launch_small(const SmallArgs& a, int w_dtype, hipStream_t s) {
    const int ver = small_version();
    if (ver == 2) {
        if (w_dtype == LDM_BF16) launch_small_v2<unsigned short, EPI>(a, s);
        else launch_small_v2<float, EPI>(a, s);
        return launch_status("small_linear_v2");
    }
    if (ver == 4) {
        if (w_dtype == LDM_BF16) launch_small_v4<unsigned short, EPI>(a, s);
        else launch_small_v4<float, EPI>(a, s);
        return launch_status("small_linear_v4");
    }
    if (ver == 3) {
        if (w_dtype == LDM_BF16) launch_small_v3<unsigned short, EPI>(a, s);
        else launch_small_v3<float, EPI>(a, s);
        return launch_status("small_linear_v3");
    }
    const size_t lds = (size_t)a.B * a.K * sizeof(float);
    const dim3 grid((a.M + 3) / 4);
    if (w_dtype == LDM_BF16)
        hipLaunchKernelGGL((small_linear_kernel<unsigned short, EPI>), grid, dim3(256), lds, s, a);
    else
        hipLaunchKernelGGL((small_linear_kernel<float, EPI>), grid, dim3(256), lds, s, a);
    return launch_status("small_linear");
}

// ------------------------------------------------------------------------------------------
// Tiled fused linear (training).  64 (b) x 64 (m) tile, 16-deep k tiles in LDS, 4x4 per thread.
// XK / WK: operand contiguous along the contraction index (stride 1) -> k-major tile loads;
// otherwise row-contiguous loads.  Both segments (X,W) and (X2,W2) share the flags.
// ------------------------------------------------------------------------------------------
template <typename TW>
__device__ __forceinline__ float ldw(const void* W, int64_t i) {
    if (sizeof(TW) == 2) return bf16_to_f32(reinterpret_cast<const unsigned short*>(W)[i]);
    return reinterpret_cast<const float*>(W)[i];
}

template <typename TW, bool XK, bool WK>
__device__ __forceinline__ void tiled_segment(float (&acc)[4][4], float (*xs)[68], float (*ws)[68],
                                              const float* X, int64_t sxb, int64_t sxk,
                                              const void* W, int64_t swm, int64_t swk, int K,
                                              int b0, int m0, int Bn, int M) {
    const int tid = threadIdx.x;
    const int ty = tid >> 4, tx = tid & 15;
    for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int r, kk;
            if (XK) { r = tid >> 2; kk = (tid & 3) * 4 + i; }
            else    { r = (tid & 15) * 4 + i; kk = tid >> 4; }
            const int b = b0 + r, k = k0 + kk;
            xs[kk][r] = (b < Bn && k < K) ? X[(int64_t)b * sxb + (int64_t)k * sxk] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int r, kk;
            if (WK) { r = tid >> 2; kk = (tid & 3) * 4 + i; }
            else    { r = (tid & 15) * 4 + i; kk = tid >> 4; }
            const int m = m0 + r, k = k0 + kk;
            ws[kk][r] = (m < M && k < K) ? ldw<TW>(W, (int64_t)m * swm + (int64_t)k * swk) : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            const f32x4 xv = *reinterpret_cast<const f32x4*>(&xs[kk][ty * 4]);
            const f32x4 wv = *reinterpret_cast<const f32x4*>(&ws[kk][tx * 4]);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(xv[i], wv[j], acc[i][j]);
        }
        __syncthreads();
    }
}

template <typename TW, bool XK, bool WK>
__global__ __launch_bounds__(256) void linear_tiled_kernel(ldm_linear_args_t a) {
    __shared__ __attribute__((aligned(16))) float xs[16][68];
    __shared__ __attribute__((aligned(16))) float ws[16][68];
    const int b0 = blockIdx.y * 64, m0 = blockIdx.x * 64;
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    tiled_segment<TW, XK, WK>(acc, xs, ws, a.X, a.sxb, a.sxk, a.W, a.swm, a.swk, a.K, b0, m0,
                              a.Bn, a.M);
    if (a.K2 > 0)
        tiled_segment<TW, XK, WK>(acc, xs, ws, a.X2, a.sx2b, a.sx2k, a.W2, a.sw2m, a.sw2k, a.K2,
                                  b0, m0, a.Bn, a.M);
    const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int b = b0 + ty * 4 + i;
        if (b >= a.Bn) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int m = m0 + tx * 4 + j;
            if (m >= a.M) continue;
            const float pre = acc[i][j] + (a.bias ? a.bias[m] : 0.f);
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
    }
}

template <typename TW>
void launch_tiled(const ldm_linear_args_t& a, bool xk, bool wk, hipStream_t s) {
    const dim3 grid((a.M + 63) / 64, (a.Bn + 63) / 64);
    if (xk && wk) hipLaunchKernelGGL((linear_tiled_kernel<TW, true, true>), grid, dim3(256), 0, s, a);
    else if (xk) hipLaunchKernelGGL((linear_tiled_kernel<TW, true, false>), grid, dim3(256), 0, s, a);
    else if (wk) hipLaunchKernelGGL((linear_tiled_kernel<TW, false, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((linear_tiled_kernel<TW, false, false>), grid, dim3(256), 0, s, a);
}

__global__ void silu_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ a, int n,
                                float* __restrict__ g) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) g[i] = dy[i] * silu_grad(a[i]);
}

// Column sums, 64 columns per workgroup of 1024 threads: 16 row groups x 64 columns, each
// thread 4 interleaved partial sums over rows r = ty + 16 i, then a fixed-order LDS reduce
// (deterministic; one column per thread serialised ~1000 dependent loads before).
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ G, int Bn, int M,
                                                     float* __restrict__ out, int accumulate) {
    __shared__ float red[16][65];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int m = blockIdx.x * 64 + tx;
    G += (size_t)blockIdx.y * Bn * M;       // segment (ldm_colsum_segments); 0 for ldm_colsum
    out += (size_t)blockIdx.y * M;
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    if (m < M) {
        int b = ty;
        for (; b + 48 < Bn; b += 64) {
#pragma unroll
            for (int q = 0; q < 4; ++q) p[q] += G[(size_t)(b + 16 * q) * M + m];
        }
        for (int q = 0; b < Bn; b += 16, ++q) p[q & 3] += G[(size_t)b * M + m];
    }
    red[ty][tx] = (p[0] + p[1]) + (p[2] + p[3]);
    __syncthreads();
    if (ty == 0 && m < M) {
        float s = 0.f;
        for (int r = 0; r < 16; ++r) s += red[r][tx];
        out[m] = accumulate ? out[m] + s : s;
    }
}

__global__ void gather_rows_kernel(const float* __restrict__ table, const int32_t* __restrict__ idx,
                                   int Bn, int C, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Bn * C) return;
    const int b = i / C, c = i - b * C;
    out[i] = table[(size_t)idx[b] * C + c];
}

int check_sched(const ldm_sched_t* sc, int t) {
    LDM_REQUIRE(sc && sc->abi_version == LDM_ABI_VERSION, LDM_EINVAL, "bad schedule descriptor");
    LDM_REQUIRE(t >= 0 && t < sc->T, LDM_EINVAL, "timestep %d outside [0,%d)", t, sc->T);
    return 0;
}

int check_denoiser(const ldm_denoiser_t* w, int B) {
    LDM_REQUIRE(w && w->abi_version == LDM_ABI_VERSION, LDM_EINVAL, "bad denoiser descriptor");
    LDM_REQUIRE(w->dtype == LDM_F32 || w->dtype == LDM_BF16, LDM_EINVAL, "bad denoiser dtype");
    LDM_REQUIRE(B >= 1 && B <= kSmallMaxB, LDM_ENOSYS, "sampling batch %d outside [1,%d]", B,
                kSmallMaxB);
    LDM_REQUIRE(w->n_blocks >= 1 && w->n_blocks <= LDM_MAX_BLOCKS, LDM_EINVAL, "bad n_blocks");
    LDM_REQUIRE(w->D % 8 == 0 && w->H % 8 == 0, LDM_EINVAL, "D and H must be multiples of 8");
    LDM_REQUIRE(w->D <= 2048 && w->H <= 2048, LDM_ENOSYS,
                "D and H must be <= 2048 for the sampling GEMV (8 k per lane, 4 chunks)");
    LDM_REQUIRE((size_t)B * (w->H > w->D ? w->H : w->D) * 4 <= 64 * 1024, LDM_ENOSYS,
                "B*H too large for the LDS-staged sampling kernel");
    return 0;
}

// Runs in -> blocks; leaves h in ws[(n_blocks & 1) * B*H].  Returns status.
int denoiser_trunk(const ldm_denoiser_t* w, const float* x, int t, int B, float* ws,
                   hipStream_t s, const float** h_out) {
    float* buf[2] = {ws, ws + (size_t)B * w->H};
    SmallArgs a = {};
    a.B = B;
    a.X = x; a.W = w->w_in; a.bias = w->b_in; a.Y = buf[0];
    a.M = w->H; a.K = w->D; a.ldw = w->D;
    if (int e = launch_small<SE_BIAS>(a, w->dtype, s)) return e;
    for (int k = 0; k < w->n_blocks; ++k) {
        a.X = buf[k & 1]; a.Y = buf[(k + 1) & 1];
        a.W = w->w_blk[k]; a.ldw = 2 * w->H;
        a.bias = w->e_tab[k] + (size_t)t * w->H;
        a.M = w->H; a.K = w->H;
        if (int e = launch_small<SE_BLOCK>(a, w->dtype, s)) return e;
    }
    *h_out = buf[w->n_blocks & 1];
    return 0;
}

// AdamW (decoupled weight decay; torch.optim.AdamW's update order) on fp32 masters, with the
// low-precision working copy the next step's GEMMs read written in the same pass:
//   p *= 1 - lr*wd;  m += (1-b1)(g - m);  v = b2 v + (1-b2) g^2;
//   p -= step_size * m / (sqrt(v)/bc2_sqrt + eps);  p_bf16 = RNE(p)
// One read of p, g, m, v and one write of p, m, v (+ 2 B) per parameter: HBM-bound.
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    unsigned short* __restrict__ pb, int64_t n,
                                                    float decay, float omb1, float b2, float omb2,
                                                    float eps, float step_size, float bc2_sqrt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_update(pi, g[i], mi, vi, decay, omb1, b2, omb2, eps, step_size, bc2_sqrt);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (pb) {   // round to nearest even
        const unsigned u = __builtin_bit_cast(unsigned, pi);
        pb[i] = (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
    }
}

}  // namespace
}  // namespace ldm

using namespace ldm;

extern "C" int ldm_adamw_step(float* p, const float* g, float* m, float* v, void* p_bf16,
                              int64_t n, double lr, double beta1, double beta2, double eps,
                              double weight_decay, int step, ldm_stream_t s) {
    LDM_REQUIRE(p && g && m && v && n >= 0 && step >= 1, LDM_EINVAL, "adamw: bad arguments");
    if (n == 0) return 0;
    // scalars derived in double and rounded once, as torch does with its Python-float betas
    const double bc1 = 1.0 - pow(beta1, step), bc2 = 1.0 - pow(beta2, step);
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)s, p, g, m, v, (unsigned short*)p_bf16, n,
                       (float)(1.0 - lr * weight_decay), (float)(1.0 - beta1), (float)beta2,
                       (float)(1.0 - beta2), (float)eps, (float)(lr / bc1), (float)sqrt(bc2));
    return launch_status("adamw");
}

extern "C" int ldm_ddpm_step(const ldm_sched_t* sc, const float* x, const float* eps,
                             const float* z, int t, int n, float* x_out, ldm_stream_t s) {
    if (int e = check_sched(sc, t)) return e;
    LDM_REQUIRE(x && eps && x_out && n >= 1 && (t == 0 || z), LDM_EINVAL, "bad step arguments");
    hipLaunchKernelGGL(ddpm_step_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s,
                       sc->c1, sc->c2, sc->sigma, t, x, eps, z, n, x_out);
    return launch_status("ldm_ddpm_step");
}

extern "C" int ldm_q_sample(const ldm_sched_t* sc, const float* x0, const float* eps,
                            const int32_t* t, int B, int D, float* xt_out, ldm_stream_t s) {
    LDM_REQUIRE(sc && sc->abi_version == LDM_ABI_VERSION, LDM_EINVAL, "bad schedule");
    LDM_REQUIRE(x0 && eps && t && xt_out && B >= 1 && D >= 1, LDM_EINVAL, "bad q_sample args");
    const int n = B * D;
    hipLaunchKernelGGL(q_sample_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s,
                       sc->sqrt_ab, sc->sqrt_1mab, x0, eps, t, B, D, xt_out);
    return launch_status("ldm_q_sample");
}

extern "C" int ldm_eps_mse_loss(const float* eps_hat, const float* eps, int n, float* loss_out,
                                float* grad_out, ldm_stream_t s) {
    LDM_REQUIRE(eps_hat && eps && loss_out && n >= 1, LDM_EINVAL, "bad loss args");
    const bool v4 = LDM_ALIGNED(eps_hat, 16) && LDM_ALIGNED(eps, 16) && LDM_ALIGNED(grad_out, 16);
    if (v4)
        hipLaunchKernelGGL(mse_loss_kernel<true>, dim3(1), dim3(1024), 0, (hipStream_t)s, eps_hat,
                           eps, n, loss_out, grad_out);
    else
        hipLaunchKernelGGL(mse_loss_kernel<false>, dim3(1), dim3(1024), 0, (hipStream_t)s, eps_hat,
                           eps, n, loss_out, grad_out);
    return launch_status("ldm_eps_mse_loss");
}

extern "C" int ldm_denoiser_fwd_uniform_t(const ldm_denoiser_t* w, const float* x, int t, int B,
                                          float* eps_out, float* ws, ldm_stream_t s) {
    if (int e = check_denoiser(w, B)) return e;
    LDM_REQUIRE(t >= 0 && t < w->T, LDM_EINVAL, "timestep %d outside [0,%d)", t, w->T);
    LDM_REQUIRE(x && eps_out && ws && LDM_ALIGNED(x, 16) && LDM_ALIGNED(ws, 16), LDM_EALIGN,
                "x/ws must be 16-byte aligned");
    const float* h = nullptr;
    if (int e = denoiser_trunk(w, x, t, B, ws, (hipStream_t)s, &h)) return e;
    SmallArgs a = {};
    a.B = B; a.X = h; a.W = w->w_out; a.bias = w->b_out; a.Y = eps_out;
    a.M = w->D; a.K = w->H; a.ldw = w->H;
    return launch_small<SE_BIAS>(a, w->dtype, (hipStream_t)s);
}

extern "C" int ldm_sample_step(const ldm_denoiser_t* w, const ldm_sched_t* sc, const float* x,
                               const float* z, int t, int B, float* x_out, float* ws,
                               ldm_stream_t s) {
    if (int e = check_denoiser(w, B)) return e;
    if (int e = check_sched(sc, t)) return e;
    LDM_REQUIRE(x && x_out && ws && x != x_out && (t == 0 || z), LDM_EINVAL,
                "bad sample_step args");
    LDM_REQUIRE(LDM_ALIGNED(x, 16) && LDM_ALIGNED(ws, 16), LDM_EALIGN, "x/ws misaligned");
    const float* h = nullptr;
    if (int e = denoiser_trunk(w, x, t, B, ws, (hipStream_t)s, &h)) return e;
    // out-projection with the A8 update fused into its epilogue (tables read on device at t:
    // no host round trip, so the whole T-step loop can be captured as one hipGraph).
    SmallArgs a = {};
    a.B = B; a.X = h; a.W = w->w_out; a.bias = w->b_out; a.Y = x_out;
    a.M = w->D; a.K = w->H; a.ldw = w->H;
    a.xlat = x; a.z = z; a.t = t;
    a.c1t = sc->c1; a.c2t = sc->c2; a.sgt = sc->sigma;
    return launch_small<SE_STEP>(a, w->dtype, (hipStream_t)s);
}

extern "C" int ldm_linear(const ldm_linear_args_t* a, ldm_stream_t s) {
    LDM_REQUIRE(a && a->X && a->W && a->Y && a->Bn >= 1 && a->M >= 1 && a->K >= 1, LDM_EINVAL,
                "bad linear args");
    LDM_REQUIRE(a->K2 == 0 || (a->X2 && a->W2), LDM_EINVAL, "second segment NULL");
    LDM_REQUIRE(a->epi >= 0 && a->epi <= LDM_EPI_MASK_R, LDM_EINVAL, "bad epilogue %d", a->epi);
    LDM_REQUIRE((a->epi != LDM_EPI_RESID_SILU && a->epi != LDM_EPI_ADD_R && a->epi != LDM_EPI_MASK_R) || a->R, LDM_EINVAL,
                "epilogue needs R");
    LDM_REQUIRE(a->w_dtype == LDM_F32 || a->w_dtype == LDM_BF16, LDM_EINVAL, "bad w_dtype");
    LDM_REQUIRE(a->compute == LDM_COMPUTE_FP32 || a->compute == LDM_COMPUTE_BF16, LDM_EINVAL,
                "bad compute mode %d", a->compute);
    if (a->compute == LDM_COMPUTE_BF16) return linear_mfma(*a, (hipStream_t)s);
    const bool xk = a->sxk == 1, wk = a->swk == 1;
    if (a->w_dtype == LDM_BF16) launch_tiled<unsigned short>(*a, xk, wk, (hipStream_t)s);
    else launch_tiled<float>(*a, xk, wk, (hipStream_t)s);
    return launch_status("ldm_linear");
}

extern "C" int64_t ldm_linear_workspace_floats(const ldm_linear_args_t* a) {
    if (!a || a->Bn < 1 || a->M < 1 || a->K < 1) return 0;
    return linear_mfma_ws_floats(*a);
}

extern "C" int ldm_silu_bwd(const float* dy, const float* a, int n, float* g_out, ldm_stream_t s) {
    LDM_REQUIRE(dy && a && g_out && n >= 1, LDM_EINVAL, "bad silu_bwd args");
    hipLaunchKernelGGL(silu_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, dy, a,
                       n, g_out);
    return launch_status("ldm_silu_bwd");
}

extern "C" int ldm_colsum(const float* G, int Bn, int M, float* out, int accumulate,
                          ldm_stream_t s) {
    LDM_REQUIRE(G && out && Bn >= 1 && M >= 1, LDM_EINVAL, "bad colsum args");
    hipLaunchKernelGGL(colsum_kernel, dim3((M + 63) / 64), dim3(1024), 0, (hipStream_t)s, G, Bn, M,
                       out, accumulate);
    return launch_status("ldm_colsum");
}

extern "C" int ldm_colsum_segments(const float* G, int S, int P, int M, float* out,
                                   int accumulate, ldm_stream_t s) {
    LDM_REQUIRE(G && out && S >= 1 && P >= 1 && M >= 1, LDM_EINVAL, "bad colsum_segments args");
    LDM_REQUIRE(S <= 65535, LDM_EINVAL, "too many segments (%d)", S);
    hipLaunchKernelGGL(colsum_kernel, dim3((M + 63) / 64, S), dim3(1024), 0, (hipStream_t)s, G, P,
                       M, out, accumulate);
    return launch_status("ldm_colsum_segments");
}

extern "C" int ldm_gather_rows(const float* table, const int32_t* idx, int Bn, int C, float* out,
                               ldm_stream_t s) {
    LDM_REQUIRE(table && idx && out && Bn >= 1 && C >= 1, LDM_EINVAL, "bad gather args");
    const int n = Bn * C;
    hipLaunchKernelGGL(gather_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s,
                       table, idx, Bn, C, out);
    return launch_status("ldm_gather_rows");
}
