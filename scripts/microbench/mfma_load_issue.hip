// Microbenchmark: issue cost of vector-memory loads interleaved with
// v_mfma_f32_32x32x16_bf16 at one wave per SIMD (4 waves/CU, LDS-forced 1 WG/CU).
// MODE 0: no loads; 1: global_load_dwordx4 -> VGPR; 2: global_load_lds_dwordx4 (LDS-DMA).
// NL loads per 8 MFMAs.  Prints cycles per 8-MFMA step (s_memtime, median over WGs).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(4 * sizeof(unsigned)))) unsigned u32x4;

constexpr int ITERS = 4096;

template <int MODE, int NL>
__global__ __launch_bounds__(256, 1) void kern(const u32x4* __restrict__ src, float* out,
                                               long long* cyc) {
    __shared__ __attribute__((aligned(16))) char smem[160 * 1024 - 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    f32x16 acc[4] = {};
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(0.01f * (lane + i)); b[i] = (__bf16)(0.02f * i); }
    u32x4 sink = {0, 0, 0, 0};
    u32x4 buf[NL > 0 ? NL : 1][4];
    const u32x4* p = src + ((blockIdx.x * 4 + wave) * 64 + lane);
    const uint32_t lds = (uint32_t)(uintptr_t)smem + wave * 16384;
    long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[m & 3], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (m < NL) {
                const u32x4* q = p + ((it * NL + m) & 1023) * 1024;   // 16 MiB window, L2/MALL
                if (MODE == 1) {
                    sink ^= buf[m][it & 3];
                    buf[m][it & 3] = *q;
                } else if (MODE == 2) {
                    unsigned keep;
                    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                                 : "=&s"(keep) : "v"(q), "s"(lds + (m & 15) * 1024) : "memory");
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (MODE == 2 && NL > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL * 3) : "memory");
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc[0][i] + acc[1][i] + acc[2][i] + acc[3][i];
    s += (float)(sink[0] ^ sink[1] ^ sink[2] ^ sink[3]);
    if (MODE == 2) s += (float)smem[lane];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int NL>
void run(const u32x4* src, float* out, long long* cyc, int nwg) {
    kern<MODE, NL><<<nwg, 256>>>(src, out, cyc);   // warm
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    kern<MODE, NL><<<nwg, 256>>>(src, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(nwg);
    hipMemcpy(h.data(), cyc, nwg * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("mode %d loads/8mfma %d: %.1f cyc per 8-MFMA step (median WG), wall %.3f ms, "
           "%.1f TF/s\n", MODE, NL, (double)h[nwg / 2] / ITERS, ms,
           (double)nwg * 4 * ITERS * 8 * 32768.0 / (ms * 1e-3) / 1e12);
}

int main() {
    const int nwg = 256;
    u32x4* src; float* out; long long* cyc;
    hipMalloc(&src, (size_t)64 << 20);
    hipMemset(src, 0x3c, (size_t)64 << 20);
    hipMalloc(&out, nwg * 256 * 4);
    hipMalloc(&cyc, nwg * 8);
    run<0, 0>(src, out, cyc, nwg);
    run<1, 1>(src, out, cyc, nwg);
    run<1, 2>(src, out, cyc, nwg);
    run<1, 4>(src, out, cyc, nwg);
    run<2, 1>(src, out, cyc, nwg);
    run<2, 2>(src, out, cyc, nwg);
    run<2, 4>(src, out, cyc, nwg);
    return 0;
}
