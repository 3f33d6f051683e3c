// Device helpers shared by the decoder kernels (decoder.hip, decoder_fs.hip).
#pragma once
#include "ldm_internal.h"

#include <math.h>

namespace ldm {
namespace dec {

#define LDM_STR2(x) #x
#define LDM_STR(x) LDM_STR2(x)

// ------------------------------------------------------------------------------------------
// A1: one grid axis value, x = fl32(fl32(i * vs) + origin).  Contraction is disabled so the
// device rounds twice exactly like the CPU oracle (SURVEY.md §7 'Bit-exact coordinates').
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float grid_axis(int i, float vs, float origin) {
#pragma clang fp contract(off)
    float t = (float)i * vs;
    return t + origin;
}

__device__ __forceinline__ void grid_point(int p, int N, int k0, float vs, float origin,
                                           float& x, float& y, float& z) {
    const int nn = N * N;
    const int k = k0 + p / nn;
    const int r = p - (p / nn) * nn;
    const int j = r / N;
    const int i = r - j * N;
    x = grid_axis(i, vs, origin);
    y = grid_axis(j, vs, origin);
    z = grid_axis(k, vs, origin);
}


// ------------------------------------------------------------------------------------------
// Element conversion + MFMA per 16-bit type.
// ------------------------------------------------------------------------------------------
template <typename T>
struct Elem;
template <>
struct Elem<__bf16> {
    static __device__ __forceinline__ unsigned pack(float a, float b) {
        // one v_cvt_pk_bf16_f32 (RNE); the element-wise {(__bf16)a, (__bf16)b} form costs two
        // single conversions + a v_perm
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const f32x2 v = {a, b};
        return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
    }
    static __device__ __forceinline__ float round(float x) { return (float)(__bf16)x; }
    static __device__ __forceinline__ f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                       __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
    static __device__ __forceinline__ f32x4 mfma16(u32x4 a, u32x4 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                       __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
};
template <>
struct Elem<_Float16> {
    static __device__ __forceinline__ unsigned pack(float a, float b) {
        f16x2 v = {(_Float16)a, (_Float16)b};
        return __builtin_bit_cast(unsigned, v);
    }
    static __device__ __forceinline__ float round(float x) { return (float)(_Float16)x; }
    static __device__ __forceinline__ f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                      __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    }
    static __device__ __forceinline__ f32x4 mfma16(u32x4 a, u32x4 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                      __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    }
};


// ReLU in the 16-bit domain: bf16 and f16 order like sign-magnitude, so max with +0 as signed
// int16 is ReLU (rounding commutes with ReLU).
__device__ __forceinline__ unsigned relu2(unsigned v) {
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    s16x2 x = __builtin_bit_cast(s16x2, v);
    const s16x2 z = {0, 0};
    x = __builtin_elementwise_max(x, z);
    return __builtin_bit_cast(unsigned, x);
}

// Accumulator m-chunk (rows = features, cols = points) -> two B fragments (k-steps 2i, 2i+1).
template <typename T>
__device__ __forceinline__ void acc_to_frags(const f32x16& a, u32x4& f0, u32x4& f1) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        f0[q] = relu2(Elem<T>::pack(a[2 * q], a[2 * q + 1]));
        f1[q] = relu2(Elem<T>::pack(a[8 + 2 * q], a[8 + 2 * q + 1]));
    }
}

}  // namespace dec
}  // namespace ldm
