// Microbenchmark: the decoder's weight stream (csrc/decoder_fs.hip) in isolation.  One
// workgroup per CU (LDS-forced), 4 waves; each wave streams its own 768 KiB region of a 3 MiB
// L2-resident blob (the split layout's per-wave streams: 384 k-steps x 2 KiB) with raw buffer
// loads straight into a register ring D k-steps deep, and per k-step issues M bf16 MFMAs
// (v_mfma_f32_32x32x16_bf16; A = the two streamed fragments, B fixed).  Reports cycles per
// k-step (s_memtime over 3 passes of the stream, median over workgroups) and the CU's stream
// rate in bytes per cycle.
//   D in {2, 4, 6, 8} k-steps in flight, M in {0, 8}: M = 0 is the bare L2 -> VGPR rate a CU
//   gets with 4 waves x 2 D KiB in flight; M = 8 is the decoder's plain k-step (8 MFMAs = 256
//   cycles of matrix pipe per SIMD).
// Build (here): hipcc --offload-arch=gfx950 -O3 weight_stream.hip -o weight_stream
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kSteps = 384;            // k-steps per wave stream
constexpr int kStepBytes = 2048;       // 2 A fragments
constexpr int kPasses = 3;
constexpr int kLds = 140 * 1024;       // one workgroup per CU

__device__ __forceinline__ u32x4 bld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

template <int D, int M>
__global__ __launch_bounds__(256, 1) void stream_kernel(const uint8_t* blob, float* sink,
                                                        long long* cyc) {
    __shared__ char smem[kLds];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x == 0) smem[0] = 0;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)blob, (short)0, 0x7ffffff0, 0x00020000);
    const uint32_t voff = lane * 16u;
    const uint32_t beg = (uint32_t)wave * kSteps * kStepBytes, end = beg + kSteps * kStepBytes;
    u32x4 ring[D][2];
    uint32_t iss = beg;
#pragma unroll
    for (int r = 0; r < D; ++r) {
        ring[r][0] = bld(rs, voff, iss);
        ring[r][1] = bld(rs, voff + 1024u, iss);
        iss += kStepBytes;
    }
    bf16x8 b;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = (__bf16)(0.001f * (lane + i));
    f32x16 acc[4] = {};
    u32x4 x = {0, 0, 0, 0};
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int s = 0; s < kPasses * kSteps; s += D) {
#pragma unroll
        for (int r = 0; r < D; ++r) {
            // wait for slot r (the oldest two loads), use it, refill it D steps ahead
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (D - 1)) : "memory");
            const u32x4 a0 = ring[r][0], a1 = ring[r][1];
            if (M == 0) {
                x ^= a0 ^ a1;
            } else {
#pragma unroll
                for (int m = 0; m < M / 2; ++m) {
                    acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, a0), b, acc[m & 3], 0, 0, 0);
                    acc[(m + 1) & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, a1), b, acc[(m + 1) & 3], 0, 0, 0);
                }
            }
            ring[r][0] = bld(rs, voff, iss);
            ring[r][1] = bld(rs, voff + 1024u, iss);
            iss += kStepBytes;
            if (iss == end) iss = beg;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t1 = __builtin_amdgcn_s_memtime();
    float v = (float)(x[0] ^ x[1] ^ x[2] ^ x[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) v += acc[i][e];
    if (v == 1234.5f) sink[threadIdx.x] = v + smem[0];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

template <int D, int M>
int run(const uint8_t* blob, float* sink, long long* d_cyc, int grid) {
    for (int rep = 0; rep < 3; ++rep)
        hipLaunchKernelGGL((stream_kernel<D, M>), dim3(grid), dim3(256), 0, 0, blob, sink, d_cyc);
    CK(hipDeviceSynchronize());
    std::vector<long long> c(grid);
    CK(hipMemcpy(c.data(), d_cyc, grid * sizeof(long long), hipMemcpyDeviceToHost));
    std::sort(c.begin(), c.end());
    const double per_step = (double)c[grid / 2] / (kPasses * kSteps);
    printf("{\"D\": %d, \"M\": %d, \"grid\": %d, \"cycles_per_step\": %.1f, "
           "\"cu_bytes_per_cycle\": %.2f, \"min\": %.1f, \"max\": %.1f}\n",
           D, M, grid, per_step, 4.0 * kStepBytes / per_step,
           (double)c[0] / (kPasses * kSteps), (double)c[grid - 1] / (kPasses * kSteps));
    fflush(stdout);
    return 0;
}

int main() {
    uint8_t* blob;
    float* sink;
    long long* d_cyc;
    const size_t bytes = 4ull * kSteps * kStepBytes;
    CK(hipMalloc(&blob, bytes));
    CK(hipMemset(blob, 0x11, bytes));
    CK(hipMalloc(&sink, 4096));
    CK(hipMalloc(&d_cyc, 4096 * sizeof(long long)));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int grid : {cus, 8}) {
        if (run<2, 0>(blob, sink, d_cyc, grid)) return 1;
        if (run<4, 0>(blob, sink, d_cyc, grid)) return 1;
        if (run<6, 0>(blob, sink, d_cyc, grid)) return 1;
        if (run<8, 0>(blob, sink, d_cyc, grid)) return 1;
        if (run<2, 8>(blob, sink, d_cyc, grid)) return 1;
        if (run<4, 8>(blob, sink, d_cyc, grid)) return 1;
        if (run<6, 8>(blob, sink, d_cyc, grid)) return 1;
        if (run<8, 8>(blob, sink, d_cyc, grid)) return 1;
    }
    return 0;
}
