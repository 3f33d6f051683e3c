// Microbenchmark: the quarter decoder's steady-state k-loop step in isolation (no epilogue,
// no layer structure), to bisect where a step's cycles go.  One wave per SIMD, LDS ring of 7
// x 8 KiB filled by LDS-DMA (2 pieces per wave per step) from a 3.3 MB random weight blob,
// A fragments re-read by ds_read_b128 one per MFMA, B fragments from 32 resident registers,
// barrier + vmcnt every 2 steps.  Variants (template flags):
//   DMA   : issue the LDS-DMA pieces          RD  : re-read A fragments from LDS
//   BAR   : barrier + vmcnt(6) every 2 steps  POS : DMA placement (0 after MFMA 2, 1 at step end)
//   HOT   : DMA from a 512 KiB window instead of the 3.3 MB blob
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(16 * sizeof(float)))) float f32x16;
typedef __attribute__((__vector_size__(4 * sizeof(unsigned)))) unsigned u32x4;

constexpr int STEPS = 4096;
constexpr int RING = 7;
constexpr int NST = 414;

__device__ __forceinline__ bf16x8 bf(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

template <int DMA, int RD, int BAR, int POS, int HOT>
__global__ __launch_bounds__(256, 1) void kern(const uint8_t* __restrict__ blob, float* out,
                                               long long* cyc) {
    __shared__ __attribute__((aligned(16))) char smem[RING * 8192 + 96 * 1024];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t voff = wave * 2048 + lane * 16;
    const uint32_t ring_beg = (uint32_t)(uintptr_t)smem + wave * 2048;
    const uint32_t ring_end = ring_beg + RING * 8192;
    const int nst = HOT ? 64 : NST;
    int is = (blockIdx.x * 37) % nst;
    const uint8_t* isrc = blob + (size_t)is * 8192;
    uint32_t islot = ring_beg, coff = 0;
    // prologue: 6 stages ahead
    for (int j = 0; j < 6; ++j) {
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1\n\t"
                     "global_load_lds_dwordx4 %0, %1 offset:1024" ::"v"(voff), "s"(isrc), "s"(islot) : "memory");
        islot = (islot + 8192 == ring_end) ? ring_beg : islot + 8192;
        isrc += 8192;
        if (++is == nst) { is = 0; isrc = blob; }
    }
    asm volatile("s_waitcnt vmcnt(10)\n\ts_barrier" ::: "memory");
    u32x4 acur[8], hb[32];
    const u32x4* hsrc = reinterpret_cast<const u32x4*>(blob + 5 * 8192);
    for (int i = 0; i < 32; ++i) hb[i] = hsrc[i * 64 + lane];
    {
        const u32x4* sl = reinterpret_cast<const u32x4*>(smem);
        for (int i = 0; i < 8; ++i) acur[i] = sl[i * 64 + lane];
    }
    f32x16 acc[4] = {};
    long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int g = 0; g < STEPS; g += 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const u32x4 b0 = hb[2 * j], b1 = hb[2 * j + 1];
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(acur[0]), bf(b0), acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(acur[1]), bf(b0), acc[1], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (BAR && (j & 1) == 0) asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            coff = (coff + 8192 == RING * 8192) ? 0u : coff + 8192;
            const u32x4* sl = reinterpret_cast<const u32x4*>(smem + coff);
            if (RD) { acur[0] = sl[0 * 64 + lane]; acur[1] = sl[1 * 64 + lane]; }
            const u32x4 f2 = acur[2];
            acc[2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(f2), bf(b0), acc[2], 0, 0, 0);
            if (RD) acur[2] = sl[2 * 64 + lane];
            __builtin_amdgcn_sched_barrier(0);
            if (DMA && POS == 0) {
                asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1\n\t"
                             "global_load_lds_dwordx4 %0, %1 offset:1024" ::"v"(voff), "s"(isrc), "s"(islot) : "memory");
            }
            islot = (islot + 8192 == ring_end) ? ring_beg : islot + 8192;
            __builtin_amdgcn_sched_barrier(0);
            const u32x4 f3 = acur[3];
            acc[3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(f3), bf(b0), acc[3], 0, 0, 0);
            if (RD) acur[3] = sl[3 * 64 + lane];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const u32x4 f = acur[4 + i];
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(f), bf(b1), acc[i], 0, 0, 0);
                if (RD) acur[4 + i] = sl[(4 + i) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
            if (DMA && POS == 1) {
                asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1\n\t"
                             "global_load_lds_dwordx4 %0, %1 offset:1024" ::"v"(voff), "s"(isrc - 0), "s"(islot) : "memory");
            }
            __builtin_amdgcn_sched_barrier(0);
            isrc += 8192;
            if (++is == nst) { is = 0; isrc = blob; }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc[0][i] + acc[1][i] + acc[2][i] + acc[3][i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int DMA, int RD, int BAR, int POS, int HOT>
void run(const uint8_t* blob, float* out, long long* cyc, int nwg, const char* what) {
    kern<DMA, RD, BAR, POS, HOT><<<nwg, 256>>>(blob, out, cyc);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    kern<DMA, RD, BAR, POS, HOT><<<nwg, 256>>>(blob, out, cyc);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(nwg);
    (void)hipMemcpy(h.data(), cyc, nwg * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("%-40s %6.1f cyc/step  %7.1f TF/s  clock %.2f GHz\n", what, (double)h[nwg / 2] / STEPS,
           (double)nwg * 4 * STEPS * 8 * 32768.0 / (ms * 1e-3) / 1e12,
           (double)h[nwg / 2] / (ms * 1e-3) / 1e9);
}

int main() {
    const int nwg = 256;
    uint8_t* blob; float* out; long long* cyc;
    const size_t bytes = (size_t)NST * 8192;
    (void)hipMalloc(&blob, bytes);
    std::vector<uint16_t> h(bytes / 2);
    uint32_t x = 12345;
    for (auto& v : h) { x = x * 1664525u + 1013904223u; v = 0x3c00 + ((x >> 16) & 0x3ff) - 0x200; v ^= (x & 0x8000); }
    (void)hipMemcpy(blob, h.data(), bytes, hipMemcpyHostToDevice);
    (void)hipMalloc(&out, nwg * 256 * 4);
    (void)hipMalloc(&cyc, nwg * 8);
    run<0, 0, 0, 0, 0>(blob, out, cyc, nwg, "MFMA only (B from 32 regs)");
    run<0, 1, 0, 0, 0>(blob, out, cyc, nwg, "+ A reads");
    run<0, 1, 1, 0, 0>(blob, out, cyc, nwg, "+ A reads + barrier/2");
    run<1, 1, 0, 0, 0>(blob, out, cyc, nwg, "+ A reads + DMA");
    run<1, 1, 1, 0, 0>(blob, out, cyc, nwg, "+ A reads + DMA + barrier (kernel)");
    run<1, 1, 1, 0, 1>(blob, out, cyc, nwg, "kernel, DMA from 512K window");
    run<1, 1, 1, 1, 0>(blob, out, cyc, nwg, "kernel, DMA at step end");
    run<1, 0, 1, 0, 0>(blob, out, cyc, nwg, "DMA + barrier, no A reads");
    return 0;
}
