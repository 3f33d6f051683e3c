// Microbenchmark: one-way latency of the XCD-replica sampler's hand-off primitive
// (csrc/sample_loop.hip publish_tagged / stage_tagged): an 8-byte {value, tag} agent-scope
// relaxed store, observed by an agent-scope relaxed 8-byte poll in another workgroup.
//
// Two single-wave workgroups on ONE XCD ping-pong NROUND times: A publishes tag 2i+1 into
// g[0] and polls g[1] for 2i+2; B polls g[0] for 2i+1 and publishes 2i+2 into g[1].  One-way
// latency = A's elapsed time / (2 NROUND), from s_memrealtime (100 MHz) and s_memtime.
// The grid is 64 workgroups (8 per XCD under round-robin placement); the pair is picked on the
// device: the first two workgroups that report the same HW_REG_XCC_ID (found through an
// atomic claim), so placement is checked, never assumed.  Every other workgroup exits.
// Bounded: every poll gives up after 2^22 tries and the result is flagged.
//
// Build + run (GPU box):  hipcc --offload-arch=gfx950 -O3 handoff_latency.hip -o /tmp/hl && /tmp/hl
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned long long u64;
constexpr int NROUND = 20000;
constexpr unsigned kLimit = 1u << 22;

__device__ __forceinline__ void publish(u64* g, unsigned tag) {
    __hip_atomic_store(g, ((u64)tag << 32) | 0x3f800000u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool wait_tag(const u64* g, unsigned tag) {
    unsigned spins = 0;
    while ((unsigned)(__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) !=
           tag)
        if (++spins > kLimit) return false;
    return true;
}

// claim[x]: workgroups of XCD x that arrived (first two form the pair); role via the count
__global__ void pingpong(u64* g, unsigned* claim, long long* out, int cross) {
    if (threadIdx.x != 0) return;
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;
    // cross = 0: both on XCD 0's first two arrivals; cross = 1: first arrival on XCD 0 (A)
    // and first arrival on XCD 1 (B)
    int role = -1;
    if (!cross) {
        if (xcc == 0) {
            const unsigned k = atomicAdd(&claim[0], 1u);
            role = k < 2 ? (int)k : -1;
        }
    } else if (xcc <= 1) {
        const unsigned k = atomicAdd(&claim[xcc], 1u);
        role = k == 0 ? (int)xcc : -1;
    }
    if (role < 0) return;
    u64* ping = g;
    u64* pong = g + 32;       // another 256-B line
    bool ok = true;
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < NROUND && ok; ++i) {
        if (role == 0) {
            publish(ping, 2 * i + 1);
            ok = wait_tag(pong, 2 * i + 2);
        } else {
            ok = wait_tag(ping, 2 * i + 1);
            publish(pong, 2 * i + 2);
        }
    }
    const long long c1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if (role == 0) {
        out[0] = r1 - r0;
        out[1] = c1 - c0;
        out[2] = ok;
        out[3] = xcc;
    }
}

int main() {
    u64* g;
    unsigned* claim;
    long long* out;
    hipMalloc(&g, 4096);
    hipMalloc(&claim, 64);
    hipMalloc(&out, 64);
    for (int cross = 0; cross < 2; ++cross) {
        for (int rep = 0; rep < 4; ++rep) {
            hipMemset(g, 0, 4096);
            hipMemset(claim, 0, 64);
            hipMemset(out, 0, 64);
            hipLaunchKernelGGL(pingpong, dim3(64), dim3(64), 0, 0, g, claim, out, cross);
            hipDeviceSynchronize();
            long long h[4];
            hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
            const double ns = h[0] * 10.0 / (2.0 * NROUND);
            const double cyc = (double)h[1] / (2.0 * NROUND);
            printf("{\"pair\": \"%s\", \"rep\": %d, \"ok\": %lld, \"one_way_ns\": %.1f, "
                   "\"one_way_cycles\": %.0f, \"clock_ghz\": %.3f}\n",
                   cross ? "cross-XCD" : "same-XCD", rep, h[2], ns, cyc,
                   h[0] ? (double)h[1] / (h[0] * 10.0) : 0.0);
        }
    }
    return 0;
}
