// C17: the 1D-UNet denoiser's fused conv1d on MI355X (gfx950), DESIGN.md §9.
//
// One kernel, ldm_conv1d, runs every conv of the UNet as an implicit GEMM
//   Y[b][co][l] = sum_seg sum_{ci,k} W(co,ci,k) act(X[b][ci][src(l,k)]) + biases (+ R)
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
// Tiling: a workgroup (256 threads = 4 waves) owns 32 output channels x 64 positions of one
// shape.  The input window (16 channels x (63*stride + ksize) positions) and the weight slice
// (16 channels x ksize taps x 32 outputs) are staged in LDS per 16-channel chunk; each thread
// accumulates 2 channels x 4 consecutive positions in fp32 (VALU FMA: the UNet is a small,
// latency-bound GEMV-like op at the sampling batch, MFMA is reserved for the decoder as the
// north star asks).  Stores are 4 consecutive positions per thread.
#include "ldm_internal.h"
#include "ddpm_common.h"

namespace ldm {
namespace {

constexpr int kCoT = 32;          // output channels per workgroup
constexpr int kLT = 64;           // output positions per workgroup
constexpr int kCiT = 16;          // input channels per LDS chunk
constexpr int kMaxWin = 63 * 2 + 4;
constexpr int kXsLd = kMaxWin + 2;   // 132
constexpr int kWsLd = kCoT + 1;      // 33
constexpr int kMaxKs = 4;

template <typename TW>
__device__ __forceinline__ float ldw(const void* W, int64_t i) {
    if (sizeof(TW) == 2) return bf16_to_f32(reinterpret_cast<const unsigned short*>(W)[i]);
    return reinterpret_cast<const float*>(W)[i];
}

template <typename TW, int KS, int ST>
__device__ __forceinline__ void conv_segment(float (&acc)[2][4], float* __restrict__ xs,
                                             float* __restrict__ ws, const ldm_conv1d_seg_t& s,
                                             int b, int co0, int l0, int Cout) {
    constexpr int WIN = (kLT - 1) * ST + KS;
    const int tid = threadIdx.x;
    const int tx = tid & 15, ty = tid >> 4;
    const bool up2 = s.mode == LDM_CONV_UP2;
    const int Lsrc = up2 ? 2 * s.L_in : s.L_in;
    const int p0 = l0 * ST - s.pad;
    for (int ci0 = 0; ci0 < s.C; ci0 += kCiT) {
        for (int i = tid; i < kCiT * WIN; i += 256) {
            const int ci = i / WIN, j = i - ci * WIN;
            const int c = ci0 + ci, p = p0 + j;
            float v = 0.f;
            if (c < s.C && p >= 0 && p < Lsrc) {
                v = s.X[((int64_t)b * s.C + c) * s.L_in + (up2 ? (p >> 1) : p)];
                if (s.silu_in) v = silu(v);
            }
            xs[ci * kXsLd + j] = v;
        }
        for (int i = tid; i < kCoT * kCiT * KS; i += 256) {
            const int co = i / (kCiT * KS), r = i - co * (kCiT * KS);
            const int ci = r / KS;
            float v = 0.f;
            if (co0 + co < Cout && ci0 + ci < s.C)
                v = ldw<TW>(s.W, (int64_t)(co0 + co) * s.ldw + (int64_t)ci0 * KS + r);
            ws[r * kWsLd + co] = v;
        }
        __syncthreads();
#pragma unroll 4
        for (int ci = 0; ci < kCiT; ++ci) {
#pragma unroll
            for (int k = 0; k < KS; ++k) {
                const float w0 = ws[(ci * KS + k) * kWsLd + ty * 2];
                const float w1 = ws[(ci * KS + k) * kWsLd + ty * 2 + 1];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float x = xs[ci * kXsLd + (tx * 4 + i) * ST + k];
                    acc[0][i] = fmaf(w0, x, acc[0][i]);
                    acc[1][i] = fmaf(w1, x, acc[1][i]);
                }
            }
        }
        __syncthreads();
    }
}

template <typename TW>
__global__ __launch_bounds__(256) void conv1d_kernel(ldm_conv1d_args_t a) {
    __shared__ __attribute__((aligned(16))) float xs[kCiT * kXsLd];
    __shared__ __attribute__((aligned(16))) float ws[kCiT * kMaxKs * kWsLd];
    const int l0 = blockIdx.x * kLT, co0 = blockIdx.y * kCoT, b = blockIdx.z;
    float acc[2][4];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[r][i] = 0.f;
    for (int si = 0; si < a.n_seg; ++si) {
        const ldm_conv1d_seg_t& s = a.seg[si];
        if (s.ksize == 3 && s.stride == 1)
            conv_segment<TW, 3, 1>(acc, xs, ws, s, b, co0, l0, a.Cout);
        else if (s.ksize == 3 && s.stride == 2)
            conv_segment<TW, 3, 2>(acc, xs, ws, s, b, co0, l0, a.Cout);
        else if (s.ksize == 1)
            conv_segment<TW, 1, 1>(acc, xs, ws, s, b, co0, l0, a.Cout);
        else if (s.ksize == 4 && s.stride == 2)
            conv_segment<TW, 4, 2>(acc, xs, ws, s, b, co0, l0, a.Cout);
    }
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int co = co0 + ty * 2 + r;
        if (co >= a.Cout) continue;
        float bb = 0.f;
        if (a.bias) bb += a.bias[co];
        if (a.bias2) bb += a.bias2[co];
        if (a.cbias) bb += a.cbias[(int64_t)b * a.scb + co];
        const int64_t row = ((int64_t)b * a.Cout + co) * a.L_out;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int l = l0 + tx * 4 + i;
            if (l >= a.L_out) continue;
            float pre = acc[r][i] + bb;
            if (a.R) pre += a.R[row + l];
            if (a.epi == LDM_CONV_EPI_DDPM) {
                const bool noise = a.t > 0;
                a.Y[row + l] = ddpm_update(a.xlat[row + l], pre, noise ? a.z[row + l] : 0.f,
                                           a.c1[a.t], a.c2[a.t], a.sigma[a.t], noise);
            } else {
                a.Y[row + l] = pre;
            }
        }
    }
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
        LDM_REQUIRE(g.ldw >= g.C * g.ksize, LDM_EINVAL, "conv1d seg %d: ldw %d < C*ksize", i,
                    g.ldw);
        LDM_REQUIRE(g.pad < g.ksize, LDM_EINVAL, "conv1d seg %d: pad %d >= ksize", i, g.pad);
    }
    const dim3 grid((a->L_out + kLT - 1) / kLT, (a->Cout + kCoT - 1) / kCoT, a->B);
    if (a->w_dtype == LDM_BF16)
        hipLaunchKernelGGL(conv1d_kernel<unsigned short>, grid, dim3(256), 0, (hipStream_t)s, *a);
    else
        hipLaunchKernelGGL(conv1d_kernel<float>, grid, dim3(256), 0, (hipStream_t)s, *a);
    return launch_status("ldm_conv1d");
}
