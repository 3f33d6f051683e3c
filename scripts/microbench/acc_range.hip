// Does a k-step cost more on one of the split decoder's two accumulator sets?  (DESIGN.md §4
// round 6: the plain k-steps of every layer's part 0 -- accumulators accA, a[128:255] in the
// decoder's code -- run ~320 cycles, those of part 1 -- accB, a[0:127] -- ~278, with the same
// instructions, and scripts/microbench/lds_half_latency showed the LDS address is not it.)
// One workgroup of 4 waves per CU (one per SIMD, as dec_fs_kernel), each wave with TWO sets of
// 8 32x32 accumulators (2 x 128 registers, both live), 4 lane-linear ds_read_b128 B fragments
// per step behind the MFMAs (the decoder's rolling schedule); phases of 16 steps alternate
// between the sets, wave 0 of each workgroup stamps s_memtime at every phase boundary.
// hipcc --offload-arch=gfx950 -O3 acc_range.hip -o acc_range && ./acc_range
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void step16(f32x16 (&acc)[2][4], u32x4 (&b)[4], const u32x4& a0,
                                       const u32x4& a1, const char* p) {
#pragma unroll 1
    for (int j = 0; j < 16; j += 4) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const char* q = p + ((j + r + 1) & 15) * 4096;
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                acc[0][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                    __builtin_bit_cast(bf16x8, a0), __builtin_bit_cast(bf16x8, b[n]), acc[0][n], 0, 0, 0);
                acc[1][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                    __builtin_bit_cast(bf16x8, a1), __builtin_bit_cast(bf16x8, b[n]), acc[1][n], 0, 0, 0);
                b[n] = *reinterpret_cast<const u32x4*>(q + n * 1024);
            }
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

__global__ __launch_bounds__(256, 1) void acc_sets(int reps, unsigned long long* out, float* sink) {
    __shared__ __attribute__((aligned(16))) char smem[64 * 1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4096; i += 256)
        reinterpret_cast<u32x4*>(smem)[i] = u32x4{0x3f803f80u ^ (unsigned)i, 0x3f80u, 0u, 0x3f800000u};
    __syncthreads();
    f32x16 X[2][4], Y[2][4];
    for (int i = 0; i < 2; ++i)
        for (int n = 0; n < 4; ++n) { X[i][n] = f32x16{}; Y[i][n] = f32x16{}; }
    const u32x4 a0 = {0x3f803f80u, 0x3c003c00u, 0u, 0x3f80u}, a1 = {0u, 0x3f803f80u, 0x3f00u, 0u};
    u32x4 b[4];
    const char* p = smem + lane * 16;
    for (int n = 0; n < 4; ++n) b[n] = *reinterpret_cast<const u32x4*>(p + n * 1024);
    unsigned long long t0 = 0, t1 = 0, t2 = 0;
    for (int r = 0; r < reps; ++r) {
        t0 = __builtin_readcyclecounter();
        step16(X, b, a0, a1, p);
        t1 = __builtin_readcyclecounter();
        step16(Y, b, a0, a1, p);
        t2 = __builtin_readcyclecounter();
    }
    float s = 0.f;
    for (int i = 0; i < 2; ++i)
        for (int n = 0; n < 4; ++n) s += X[i][n][lane & 15] + Y[i][n][(lane + 3) & 15];
    sink[blockIdx.x * 256 + threadIdx.x] = s;
    if (lane == 0 && wave == 0) {
        out[blockIdx.x * 2 + 0] = t1 - t0;   // (the last rep's phases)
        out[blockIdx.x * 2 + 1] = t2 - t1;
    }
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned long long* d;
    float* sink;
    CHECK(hipMalloc(&d, (size_t)cus * 2 * 8));
    CHECK(hipMalloc(&sink, (size_t)cus * 256 * 4));
    for (int reps : {1, 4, 16}) {
        for (int it = 0; it < 2; ++it) {
            hipLaunchKernelGGL(acc_sets, dim3(cus), dim3(256), 0, 0, reps, d, sink);
            CHECK(hipDeviceSynchronize());
        }
        std::vector<unsigned long long> h((size_t)cus * 2);
        CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
        std::vector<double> x, y;
        for (int i = 0; i < cus; ++i) { x.push_back(h[2 * i] / 16.0); y.push_back(h[2 * i + 1] / 16.0); }
        std::sort(x.begin(), x.end());
        std::sort(y.begin(), y.end());
        printf("{\"reps\": %d, \"set_X_cycles_per_step\": %.1f, \"set_Y_cycles_per_step\": %.1f, "
               "\"mfma_floor\": 256}\n", reps, x[x.size() / 2], y[y.size() / 2]);
    }
    return 0;
}
