// Microbenchmark: cost of streaming A fragments through LDS beside v_mfma_f32_32x32x16_bf16 at
// one wave per SIMD, the decoder's step shape: 8 MFMAs per step, each A fragment re-read from
// an LDS ring by ds_read_b128 (rolling, 1 per MFMA), plus the fill of 8 KiB per step per CU.
//   FILL 0: no fill                     1: 2 LDS-DMA pieces / wave / step (global_load_lds)
//   FILL 2: 1 LDS-DMA piece / step      3: register staging (2 global_load_dwordx4 + 2 ds_write_b128)
//   SRC  = source window in KiB (L2-hot 512 KiB vs 8 MiB)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(4 * sizeof(unsigned)))) unsigned u32x4;

constexpr int ITERS = 2048;
constexpr int RING = 7;

__device__ __forceinline__ bf16x8 as_bf(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

template <int FILL, int READS, int SRC_KB>
__global__ __launch_bounds__(256, 1) void kern(const uint8_t* __restrict__ src, float* out,
                                               long long* cyc) {
    __shared__ __attribute__((aligned(16))) char smem[RING * 8192 + 96 * 1024];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int i = threadIdx.x; i < RING * 8192 / 16; i += 256)
        reinterpret_cast<u32x4*>(smem)[i] = u32x4{0x3c003c00u, 0x3c003c00u, 0, 0};
    __syncthreads();
    f32x16 acc[4] = {};
    bf16x8 b;
    for (int i = 0; i < 8; ++i) b[i] = (__bf16)(0.02f * i);
    u32x4 acur[8];
    for (int i = 0; i < 8; ++i) acur[i] = reinterpret_cast<const u32x4*>(smem)[i * 64 + lane];
    const uint32_t ring_beg = (uint32_t)(uintptr_t)smem + wave * 2048;
    uint32_t islot = ring_beg, coff = 0;
    const uint8_t* isrc = src;
    const uint8_t* send = src + SRC_KB * 1024;
    const uint32_t voff = wave * 2048 + lane * 16;
    u32x4 st0 = {}, st1 = {};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
        const u32x4* sl;
        coff = (coff + 8192 == RING * 8192) ? 0 : coff + 8192;
        sl = reinterpret_cast<const u32x4*>(smem + coff);
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(acur[m]), b, acc[m & 3], 0, 0, 0);
            if (READS) acur[m] = sl[m * 64 + lane];
            if (m == 2) {
                __builtin_amdgcn_sched_barrier(0);
                if (FILL == 1 || FILL == 2) {
                    if (FILL == 1)
                        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\t"
                                     "global_load_lds_dwordx4 %0, %1\n\t"
                                     "global_load_lds_dwordx4 %0, %1 offset:1024"
                                     :: "v"(voff), "s"(isrc), "s"(islot) : "memory");
                    else
                        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\t"
                                     "global_load_lds_dwordx4 %0, %1"
                                     :: "v"(voff), "s"(isrc), "s"(islot) : "memory");
                } else if (FILL == 3) {
                    // write the pair loaded one step ago, then load the next pair
                    char* d = smem + (islot - (uint32_t)(uintptr_t)smem) + lane * 16;
                    *reinterpret_cast<u32x4*>(d) = st0;
                    *reinterpret_cast<u32x4*>(d + 1024) = st1;
                    const u32x4* g = reinterpret_cast<const u32x4*>(isrc + voff);
                    st0 = g[0];
                    st1 = g[64];
                }
                islot = (islot + 8192 == ring_beg + RING * 8192) ? ring_beg : islot + 8192;
                isrc = (isrc + 8192 == send) ? src : isrc + 8192;
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (FILL == 1 && (it & 1)) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
        if (FILL == 2 && (it & 1)) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
        if ((FILL == 0 || FILL == 3) && (it & 1)) asm volatile("s_barrier" ::: "memory");
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc[0][i] + acc[1][i] + acc[2][i] + acc[3][i];
    out[blockIdx.x * 256 + threadIdx.x] = s + (float)(st0[0] ^ st1[1]);
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int FILL, int READS, int SRC_KB>
void run(const uint8_t* src, float* out, long long* cyc, int nwg, const char* what) {
    kern<FILL, READS, SRC_KB><<<nwg, 256>>>(src, out, cyc);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    kern<FILL, READS, SRC_KB><<<nwg, 256>>>(src, out, cyc);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(nwg);
    (void)hipMemcpy(h.data(), cyc, nwg * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("%-44s %6.1f cyc/step  %7.1f TF/s  (%.1f GB/s/CU fill)\n", what,
           (double)h[nwg / 2] / ITERS, (double)nwg * 4 * ITERS * 8 * 32768.0 / (ms * 1e-3) / 1e12,
           FILL == 0 ? 0.0 : (FILL == 2 ? 4096.0 : 8192.0) * ITERS / (ms * 1e-3) / 1e9);
}

int main() {
    const int nwg = 256;
    uint8_t* src; float* out; long long* cyc;
    (void)hipMalloc(&src, (size_t)64 << 20);
    (void)hipMemset(src, 0x3c, (size_t)64 << 20);
    (void)hipMalloc(&out, nwg * 256 * 4);
    (void)hipMalloc(&cyc, nwg * 8);
    run<0, 0, 512>(src, out, cyc, nwg, "MFMA only");
    run<0, 1, 512>(src, out, cyc, nwg, "MFMA + 8 ds_read_b128");
    run<1, 0, 512>(src, out, cyc, nwg, "MFMA + 2 glds (512K src)");
    run<1, 1, 512>(src, out, cyc, nwg, "MFMA + reads + 2 glds (512K src)");
    run<1, 1, 4096>(src, out, cyc, nwg, "MFMA + reads + 2 glds (4M src)");
    run<1, 1, 16384>(src, out, cyc, nwg, "MFMA + reads + 2 glds (16M src)");
    run<2, 1, 512>(src, out, cyc, nwg, "MFMA + reads + 1 glds (512K src)");
    run<3, 1, 512>(src, out, cyc, nwg, "MFMA + reads + reg staging (512K src)");
    run<3, 0, 512>(src, out, cyc, nwg, "MFMA + reg staging (512K src)");
    return 0;
}
