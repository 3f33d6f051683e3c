// Device helpers shared by the DDPM-side translation units (denoiser.hip, unet.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace ldm {

// v of lane (lane ^ o).  Inside a 16-lane row (o <= 8) through DPP moves, a VALU operation,
// instead of ds_bpermute's LDS round trip (the reduce-scatters below chain 7 of them per layer
// on the loop's critical path).  The partner value is the same either
// way, so every sum keeps its operands and order (the loops stay bit-identical to the graph).
// Across rows (o = 16, 32): gfx950's v_permlane16_swap / v_permlane32_swap.
// DPP: quad_perm [1,0,3,2] = 0xB1, [2,3,0,1] = 0x4E; row_ror:n (0x120 + n) gives lane i the
// value of lane (i - n) mod 16 of its row, so xor 4 is ror 12 (bit 2 clear) or ror 4 (set)
// and xor 8 is ror 8.
__device__ __forceinline__ float xor_lane(float v, int o, int lane) {
    const int x = __builtin_bit_cast(int, v);
    switch (o) {
        case 1: return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));
        case 2: return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false));
        case 4: {
            const int lo = __builtin_amdgcn_mov_dpp(x, 0x12C, 0xF, 0xF, false);   // from i + 4
            const int hi = __builtin_amdgcn_mov_dpp(x, 0x124, 0xF, 0xF, false);   // from i - 4
            return __builtin_bit_cast(float, (lane & 4) ? hi : lo);
        }
        case 8: return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false));
        case 16: {      // v_permlane16_swap(x, x): {even rows doubled, odd rows doubled}
            const auto r = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
            return __builtin_bit_cast(float, (lane & 16) ? r[0] : r[1]);
        }
        case 32: {      // v_permlane32_swap(x, x): {lower half doubled, upper half doubled}
            const auto r = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
            return __builtin_bit_cast(float, (lane & 32) ? r[0] : r[1]);
        }
        default: return __shfl_xor(v, o);
    }
}

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
