// Device helpers shared by the DDPM-side translation units (denoiser.hip, unet.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace ldm {

__device__ __forceinline__ float silu(float a) { return a / (1.f + expf(-a)); }
__device__ __forceinline__ float silu_grad(float a) {
    const float s = 1.f / (1.f + expf(-a));
    return s * (1.f + a * (1.f - s));
}

__device__ __forceinline__ float bf16_to_f32(unsigned short u) {
    return __builtin_bit_cast(float, (unsigned)u << 16);
}

// AdamW element update in torch.optim.AdamW's order (exp_avg.lerp_, exp_avg_sq.mul_.addcmul_,
// param.mul_(1 - lr wd).addcdiv_), every rounding spelled out so that ldm_adamw_step and
// ldm_adamw_multi produce the same bits whatever the surrounding code lets the compiler contract.
__device__ __forceinline__ void adamw_update(float& p, float g, float& m, float& v, float decay,
                                             float omb1, float b2, float omb2, float eps,
                                             float step_size, float bc2_sqrt) {
#pragma clang fp contract(off)
    const float mi = m + omb1 * (g - m);
    const float vi = v * b2 + (omb2 * g) * g;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p = p * decay - step_size * (mi / denom);
    m = mi;
    v = vi;
}

// A8: x' = c1*(x - c2*eps) + sigma*z  (rounded exactly as the CPU oracle: each op once).
__device__ __forceinline__ float ddpm_update(float x, float eps, float z, float c1, float c2,
                                             float sg, bool add_noise) {
#pragma clang fp contract(off)
    float y = c1 * (x - c2 * eps);
    if (add_noise) y = y + sg * z;
    return y;
}

}  // namespace ldm
