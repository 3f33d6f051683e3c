// C19 auto-decoder training pieces (DeepSDF): the
// loss, the ReLU backward and the latent-code regulariser.  The decoder's forward/backward
// GEMMs run through ldm_linear (denoiser.hip / linear_mfma.hip, LDM_EPI_RELU forward) and the
// bias / per-shape latent gradients through ldm_colsum(_segments).
//
//   relu_bwd_kernel        g = dy * (y > 0) on the post-activation
//   sdf_l1_kernel          pred = tanh(pre); clamped L1 vs the ground-truth SDF and its
//                          gradient w.r.t. pre (one workgroup, fixed summation order)
//   latent_reg_kernel      DeepSDF code_reg: coef * sum_s |z_s|, gradient coef * z_s / |z_s|
#include "ldm_internal.h"

#include <math.h>

namespace ldm {
namespace {

__global__ void relu_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y, int n,
                                float* __restrict__ g) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) g[i] = y[i] > 0.f ? dy[i] : 0.f;
}

// Fixed-order reduction of one float per thread over a 1024-thread block; result in red[0].
__device__ __forceinline__ void block_sum_1024(float* red, float s) {
    red[threadIdx.x] = s;
    __syncthreads();
#pragma unroll
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
}

__device__ __forceinline__ float clampd(float x, float d) { return fminf(fmaxf(x, -d), d); }

// Per element: loss term and d/d pre.  Written out (no fast-math intrinsics) so the tanh
// matches the C library's within an ulp or two.
__device__ __forceinline__ float sdf_l1_term(float pre, float gt, float delta, float scale,
                                             float& grad) {
    const float pred = tanhf(pre);
    const float diff = clampd(pred, delta) - clampd(gt, delta);
    const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
    const bool pass = pred >= -delta && pred <= delta;
    grad = pass ? scale * sg * (1.f - pred * pred) : 0.f;
    return fabsf(diff);
}

// One workgroup; U groups of loads in flight per thread (clamped index, predicated use).
__global__ __launch_bounds__(1024) void sdf_l1_kernel(const float* __restrict__ pre,
                                                      const float* __restrict__ gt, int n,
                                                      float delta, float scale,
                                                      float* __restrict__ loss,
                                                      float* __restrict__ grad) {
    __shared__ float red[1024];
    constexpr int U = 8;
    const int tid = (int)threadIdx.x;
    float s = 0.f;
    for (int base = 0; base < n; base += 1024 * U) {
        float a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * 1024 + tid;
            const int ii = i < n ? i : 0;
            a[u] = pre[ii];
            b[u] = gt[ii];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * 1024 + tid;
            if (i < n) {
                float g;
                s += sdf_l1_term(a[u], b[u], delta, scale, g);
                if (grad) grad[i] = g;
            }
        }
    }
    block_sum_1024(red, s);
    if (tid == 0) loss[0] = scale * red[0];
}

// One workgroup of 1024; codes in order, each norm a fixed-order block sum.
__global__ __launch_bounds__(1024) void latent_reg_kernel(const float* __restrict__ z, int S,
                                                          int L, float coef,
                                                          float* __restrict__ loss,
                                                          float* __restrict__ grad) {
    __shared__ float red[1024];
    float total = 0.f;       // thread 0's running sum
    for (int sidx = 0; sidx < S; ++sidx) {
        const float* zs = z + (size_t)sidx * L;
        float q = 0.f;
        for (int c = threadIdx.x; c < L; c += 1024) q = fmaf(zs[c], zs[c], q);
        block_sum_1024(red, q);
        const float nrm = sqrtf(red[0]);
        __syncthreads();     // everyone has read red[0] before the next code reuses red
        if (grad && nrm > 0.f) {
            const float f = coef / nrm;
            for (int c = threadIdx.x; c < L; c += 1024) grad[(size_t)sidx * L + c] += f * zs[c];
        }
        total += nrm;
    }
    if (threadIdx.x == 0) loss[0] += coef * total;
}

}  // namespace
}  // namespace ldm

using namespace ldm;

extern "C" int ldm_relu_bwd(const float* dy, const float* y, int n, float* g_out, ldm_stream_t s) {
    LDM_REQUIRE(dy && y && g_out && n >= 1, LDM_EINVAL, "bad relu_bwd args");
    hipLaunchKernelGGL(relu_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, dy, y,
                       n, g_out);
    return launch_status("ldm_relu_bwd");
}

extern "C" int ldm_sdf_l1_loss(const float* pre, const float* gt, int n, float delta, float scale,
                               float* loss_out, float* grad_out, ldm_stream_t s) {
    LDM_REQUIRE(pre && gt && loss_out && n >= 1, LDM_EINVAL, "bad sdf_l1_loss args");
    LDM_REQUIRE(delta > 0.f, LDM_EINVAL, "clamp distance must be > 0 (got %g)", (double)delta);
    hipLaunchKernelGGL(sdf_l1_kernel, dim3(1), dim3(1024), 0, (hipStream_t)s, pre, gt, n, delta,
                       scale, loss_out, grad_out);
    return launch_status("ldm_sdf_l1_loss");
}

extern "C" int ldm_latent_l2_reg(const float* z, int S, int L, float coef, float* loss_io,
                                 float* grad_io, ldm_stream_t s) {
    LDM_REQUIRE(z && loss_io && S >= 1 && L >= 1, LDM_EINVAL, "bad latent_l2_reg args");
    hipLaunchKernelGGL(latent_reg_kernel, dim3(1), dim3(1024), 0, (hipStream_t)s, z, S, L, coef,
                       loss_io, grad_io);
    return launch_status("ldm_latent_l2_reg");
}
