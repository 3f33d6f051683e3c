// Does an LDS read cost more above 64 KiB?  (the split decoder's plain
// k-steps run ~320 cycles when they read activation positions 16..31 -- LDS bytes 64..128 KiB --
// and ~278 when they read positions 0..15, with the same instructions.)
//   chase: one wave, a dependent chain of ds_read_b32 (every lane the same address, the value
//          read is the next address), starting in a 16 KiB window at byte offset `base`:
//          cycles per read = the load-to-use latency there;
//   stream: 4 waves (one per SIMD), each 4 lane-linear ds_read_b128 (1 KiB per instruction,
//          the decoder's B-fragment read) per step with 8 v_mfma_f32_32x32x16_bf16 between, the
//          reads of step j+1 issued behind step j's MFMAs (the decoder's rolling schedule), over
//          a 64 KiB window at `base`: cycles per step.
// hipcc --offload-arch=gfx950 -O3 lds_half_latency.hip -o lds_half_latency && ./lds_half_latency
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int kLds = 160 * 1024;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void chase(unsigned base, int n, unsigned long long* out) {
    extern __shared__ unsigned lds[];
    // a ring of 4096 dwords at base: lds[base/4 + i] = byte address of the next element (stride
    // 260 bytes: a new bank and line every hop)
    const unsigned w0 = base / 4;
    for (int i = threadIdx.x; i < 4096; i += 64) lds[w0 + i] = base + ((i * 65 + 65) % 4096) * 4;
    __syncthreads();
    unsigned a = base;
    // warm
    for (int i = 0; i < 64; ++i) a = *reinterpret_cast<volatile unsigned*>(reinterpret_cast<char*>(lds) + (a - 0));
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int i = 0; i < n; ++i) a = *reinterpret_cast<volatile unsigned*>(reinterpret_cast<char*>(lds) + a);
    const unsigned long long t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = a; }
}

__global__ __launch_bounds__(256, 1) void stream(unsigned base, int steps, unsigned long long* out,
                                                 float* sink) {
    extern __shared__ char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kLds / 16; i += 256)
        reinterpret_cast<u32x4*>(smem)[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
    __syncthreads();
    f32x16 acc[2][4];
    for (int i = 0; i < 2; ++i)
        for (int n = 0; n < 4; ++n) acc[i][n] = f32x16{};
    const u32x4 a0 = {0x3f803f80u, 0u, 0u, 0u}, a1 = {0u, 0x3f803f80u, 0u, 0u};
    u32x4 b[4];
    const char* p = smem + base + lane * 16;
    for (int n = 0; n < 4; ++n) b[n] = *reinterpret_cast<const u32x4*>(p + n * 1024);
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int j = 0; j < steps; ++j) {
        const char* q = p + ((j + 1) & 15) * 4096;       // the next position (16 x 4 KiB window)
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
    const unsigned long long t1 = __builtin_readcyclecounter();
    float s = 0.f;
    for (int i = 0; i < 2; ++i)
        for (int n = 0; n < 4; ++n) s += acc[i][n][lane & 15];
    sink[blockIdx.x * 256 + threadIdx.x] = s;
    if (lane == 0) out[blockIdx.x * 4 + wave] = t1 - t0;
}

int main() {
    unsigned long long* d;
    float* sink;
    CHECK(hipMalloc(&d, 4096 * 8));
    CHECK(hipMalloc(&sink, 256 * 256 * 4));
    CHECK(hipFuncSetAttribute((const void*)chase, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
    CHECK(hipFuncSetAttribute((const void*)stream, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
    const unsigned bases[] = {0u, 32u << 10, 48u << 10, 64u << 10, 80u << 10, 96u << 10, 128u << 10, 144u << 10};
    for (unsigned base : bases) {
        unsigned long long h[2];
        const int n = 4096;
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), kLds, 0, base, n, d);
        CHECK(hipDeviceSynchronize());
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), kLds, 0, base, n, d);
        CHECK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
        printf("{\"test\": \"chase\", \"base_kib\": %u, \"cycles_per_read\": %.1f}\n", base >> 10,
               (double)h[0] / n);
    }
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned sbases[] = {0u, 32u << 10, 64u << 10, 96u << 10};
    for (unsigned base : sbases) {
        const int steps = 4096;
        hipLaunchKernelGGL(stream, dim3(cus), dim3(256), kLds, 0, base, steps, d, sink);
        CHECK(hipDeviceSynchronize());
        hipLaunchKernelGGL(stream, dim3(cus), dim3(256), kLds, 0, base, steps, d, sink);
        CHECK(hipDeviceSynchronize());
        unsigned long long h[4096];
        CHECK(hipMemcpy(h, d, (size_t)cus * 4 * 8, hipMemcpyDeviceToHost));
        double s = 0;
        for (int i = 0; i < cus * 4; ++i) s += (double)h[i];
        printf("{\"test\": \"stream\", \"base_kib\": %u, \"window_kib\": 64, \"cycles_per_step\": %.1f, "
               "\"mfma_floor\": 256}\n", base >> 10, s / (cus * 4) / steps);
    }
    return 0;
}
