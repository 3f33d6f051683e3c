// Microbenchmark: the per-layer hand-off of the XCD-replica sampler (csrc/sample_loop.hip,
// sample_replica_kernel with tagged granules) WITHOUT its arithmetic: every phase, each of an
// XCD's 32 workgroups (8 waves, as kRepWaves) publishes its 32 rows of the layer as 8-byte
// {value, tag} agent-scope stores, then stages ALL 1024 granules of the layer (agent-scope
// 8-byte polls until the tag is the phase's) into LDS and passes a workgroup barrier -- an
// all-gather inside one XCD, which is what a layer boundary of the sampler is.  All 8 XCDs run
// their own replica at once (B = 8 in the bench).  Time per phase = a workgroup's elapsed
// s_memrealtime (100 MHz) / NPHASE, median over workgroups.
//
// Placement is checked, not assumed: a census gives each workgroup its XCD and rank; if an XCD
// holds other than 32 workgroups the run is flagged.  Every poll is bounded (2^22 tries).
//
// Build (here): hipcc --offload-arch=gfx950 -O3 allgather_latency.hip -o allgather_latency
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef unsigned long long u64;
constexpr int NPHASE = 6000;          // 1000 sampler steps x 6 layers
constexpr int H = 1024;               // granules per layer (rows)
constexpr int NT = 512;               // threads per workgroup
constexpr int G = 256;                // workgroups: 8 XCDs x 32
constexpr unsigned kLimit = 1u << 22;

__global__ __launch_bounds__(NT) void allgather(u64* gran, unsigned* census, long long* out,
                                                 int* flag) {
    __shared__ unsigned s_xcc, s_rank;
    __shared__ float xs[H];
    __shared__ int s_ok;
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;
        s_xcc = xcc;
        s_rank = atomicAdd(&census[xcc], 1u);
        atomicAdd(&census[8], 1u);
        unsigned spins = 0;
        while (__hip_atomic_load(&census[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < G)
            if (++spins > kLimit) break;
        bool even = true;
        for (int x = 0; x < 8; ++x)
            even = even && __hip_atomic_load(&census[x], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) == G / 8;
        s_ok = even ? 1 : 0;
        if (!even) *flag = 2;
    }
    __syncthreads();
    if (!s_ok) return;
    const unsigned xcc = s_xcc, rank = s_rank;
    u64* g = gran + (size_t)xcc * 2 * H;                 // [2][H] per replica
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    bool good = true;
    for (int p = 1; p <= NPHASE && good; ++p) {
        u64* buf = g + (p & 1) * H;
        if (threadIdx.x < 32) {                           // this workgroup's 32 rows
            const float v = xs[(rank * 32 + threadIdx.x) & (H - 1)] + 1.0f;
            const u64 w = ((u64)p << 32) | __builtin_bit_cast(unsigned, v);
            __hip_atomic_store(buf + rank * 32 + threadIdx.x, w, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        // stage every granule: all loads first, then re-poll the ones not yet tagged
        u64 t[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
            t[u] = __hip_atomic_load(buf + threadIdx.x + NT * u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            unsigned spins = 0;
            while ((unsigned)(t[u] >> 32) != (unsigned)p) {
                if (++spins > kLimit) { good = false; break; }
                t[u] = __hip_atomic_load(buf + threadIdx.x + NT * u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
            }
            xs[threadIdx.x + NT * u] = __builtin_bit_cast(float, (unsigned)t[u]);
        }
        __syncthreads();
    }
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) out[blockIdx.x] = r1 - r0;
    if (!good) *flag = 1;
}

int main() {
    u64* gran;
    unsigned* census;
    long long* out;
    int* flag;
    hipMalloc(&gran, (size_t)8 * 2 * H * sizeof(u64));
    hipMalloc(&census, 64);
    hipMalloc(&out, G * sizeof(long long));
    hipMalloc(&flag, sizeof(int));
    for (int rep = 0; rep < 4; ++rep) {
        hipMemset(gran, 0, (size_t)8 * 2 * H * sizeof(u64));
        hipMemset(census, 0, 64);
        hipMemset(out, 0, G * sizeof(long long));
        hipMemset(flag, 0, sizeof(int));
        hipLaunchKernelGGL(allgather, dim3(G), dim3(NT), 0, 0, gran, census, out, flag);
        hipDeviceSynchronize();
        std::vector<long long> h(G);
        int f = 0;
        hipMemcpy(h.data(), out, G * sizeof(long long), hipMemcpyDeviceToHost);
        hipMemcpy(&f, flag, sizeof(int), hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        const double med_ns = h[G / 2] * 10.0 / NPHASE, max_ns = h[G - 1] * 10.0 / NPHASE;
        printf("{\"pattern\": \"allgather-32wg-xcd\", \"rep\": %d, \"ok\": %d, "
               "\"phase_ns_median\": %.1f, \"phase_ns_max\": %.1f, \"granules\": %d, "
               "\"phases\": %d}\n", rep, f == 0, med_ns, max_ns, H, NPHASE);
    }
    return 0;
}
