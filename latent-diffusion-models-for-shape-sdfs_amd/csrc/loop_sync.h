// Device-side synchronisation of the persistent XCD-replica loop (the MLP sampler's
// sample_replica_kernel in sample_loop.hip; the 1D-UNet's loop that also used it was retired
// in round 4):
// bounded spins, the start-up census that places a workgroup on its XCD, and the XCD-local
// barrier between dependent phases.  Hand-off rules (MI355X guide, Guideline 16 table row 1):
// every handed-off byte is stored sc1 and drained (s_waitcnt vmcnt(0)) before ONE lane of the
// workgroup adds to its XCD's arrival counter; every load of handed-off bytes is an sc1 load
// issued after the barrier, so no acquire fence is needed.
#pragma once

#include <hip/hip_runtime.h>

#ifndef LDM_LOOP_SLEEP
#define LDM_LOOP_SLEEP 1     // s_sleep units (64 clocks) between polls of the XCD barrier
#endif

namespace ldm {
namespace lsync {

constexpr size_t kSyncBytes = 4096;

// Sync words of a replica loop, one 128-byte line each (zeroed by the host before every
// launch): start counter, status (0 ok, 1 a wait timed out, 2 placement other than G/8
// workgroups per XCD), per-XCD census counts, arrival counters and generation words.
enum ReplicaLine { R_START = 0, R_STATUS = 1, R_CNT = 2, R_ARR = 10, R_GEN = 18, R_COUNT = 26 };
static_assert(R_COUNT * 128 <= (int)kSyncBytes, "replica sync words overflow");

// Poll *w (relaxed, agent scope: an sc1 load) until it reaches target.  Bounded: after `limit`
// polls the status word is raised (1); a status raised by anyone else also ends the wait.
__device__ __forceinline__ bool spin_until(const unsigned* w, unsigned target, unsigned* status,
                                           unsigned limit) {
    unsigned spins = 0;
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if ((spins & 63) == 63 &&
            __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
            return false;
        if (++spins > limit) {
            __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
#if LDM_LOOP_SLEEP > 0
        __builtin_amdgcn_s_sleep(LDM_LOOP_SLEEP);
#endif
    }
    return true;
}

// Start-up census, thread 0 only: the workgroup's XCD (HW_REG_XCC_ID, hwreg 20 bits [3:0]) and
// its rank among that XCD's workgroups; then one flat barrier over the G workgroups, after which
// every XCD must hold exactly G/8 of them (else status 2: the caller returns before any
// compute and the host falls back).  Returns false on a timeout or a placement mismatch.
__device__ __forceinline__ bool replica_census(unsigned* sync, unsigned G, unsigned limit,
                                               unsigned* xcc_out, unsigned* rank_out) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;
    const unsigned rank = __hip_atomic_fetch_add(sync + 32 * (R_CNT + xcc), 1u,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(sync + 32 * R_START, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const bool good = spin_until(sync + 32 * R_START, G, sync + 32 * R_STATUS, limit);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");        // once per launch
    bool even = true;
    for (unsigned x = 0; x < 8; ++x)
        even = even && __hip_atomic_load(sync + 32 * (R_CNT + x), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) == G / 8;
    if (good && !even)
        __hip_atomic_store(sync + 32 * R_STATUS, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *xcc_out = xcc;
    *rank_out = rank;
    return good && even;
}

// XCD-local barrier of the nloc workgroups of replica xcc (every storing wave drained its sc1
// stores; one lane adds; the last arriver of the phase publishes the generation word).
__device__ __forceinline__ bool replica_sync(unsigned* sync, unsigned xcc, unsigned nloc,
                                            unsigned phase, int* ok, unsigned limit) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned* status = sync + 32 * R_STATUS;
        unsigned* gen = sync + 32 * (R_GEN + xcc);
        const unsigned t = __hip_atomic_fetch_add(sync + 32 * (R_ARR + xcc), 1u,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool good = true;
        if (t + 1 == phase * nloc)
            __hip_atomic_store(gen, phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            good = spin_until(gen, phase, status, limit);
        *ok = good;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
    return *ok != 0;
}

}  // namespace lsync
}  // namespace ldm
