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

// A8: x' = c1*(x - c2*eps) + sigma*z  (rounded exactly as the CPU oracle: each op once).
__device__ __forceinline__ float ddpm_update(float x, float eps, float z, float c1, float c2,
                                             float sg, bool add_noise) {
#pragma clang fp contract(off)
    float y = c1 * (x - c2 * eps);
    if (add_noise) y = y + sg * z;
    return y;
}

}  // namespace ldm
