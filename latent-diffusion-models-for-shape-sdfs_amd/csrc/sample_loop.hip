// A10 as ONE launch: the whole T-step DDPM reverse loop of the MLP denoiser in a persistent,
// kernel whose whole grid is resident (SURVEY.md §8(a) A6 + A8 + A10).
//
// Why: the graph-replayed loop (denoiser.hip small_linear_v4) is 6 dependent launches per step
// at the ~5 us floor of a dependent launch; the GEMVs themselves are far from any bandwidth
// limit.  Here the grid is H/4 workgroups of 4 waves, one wave per output row, and
//   * every wave keeps ITS weight rows in registers for the whole loop (in-proj row, one row of
//     each block, one out-proj row when gw < D: 88 fp32 values per lane at D=256, H=1024), so
//     the 9.45 MB of bf16 weights are read from HBM once per loop instead of once per step;
//   * the layer boundary is a grid barrier (write-through sc1 activation stores, one agent
//     atomic per workgroup, sc1 polling with s_sleep, sc1 loads of the activations) instead of
//     a kernel boundary;
//   * per layer each workgroup stages the [B][K] activations into LDS once.
// Arithmetic is the v4 GEMV's exactly (same k-to-lane mapping, same fma order, same shuffle
// reduce-scatter, same epilogues), so the loop is bit-identical to the graph path
// (tests/test_gpu_ddpm.py::test_sample_loop_persistent_matches_graph).
//
// Termination: every barrier wait is bounded (kSpinLimit polls); a workgroup that times out
// raises an abort flag that every other waiter also polls, so all waves exit and the host
// sees LDM_ETIMEOUT-style failure through the status word instead of a hung GPU.
#include "ldm_internal.h"
#include "ddpm_common.h"
#include "loop_sync.h"

#include <stdlib.h>

#include <atomic>
#include <type_traits>

namespace ldm {
namespace {
using lsync::kSyncBytes;
using lsync::spin_until;
using lsync::replica_sync;
using lsync::replica_census;
using namespace lsync;   // ReplicaLine

constexpr unsigned kSpinLimit = 1u << 22;   // x s_sleep(2) ~ 0.3 s per barrier, worst case
// The limit travels in LoopArgs::spin_limit (default kSpinLimit).  ldm_sample_loop_config()
// lowers it for the timeout test (tests/test_gpu_ddpm.py): a tiny limit makes barriers give up,
// which must surface as status 1, never as silently wrong latents.

struct LoopArgs {
    const void* w_in;  const float* b_in;     // [H][D]
    const void* w_blk[4];                     // [H][2H] (the W_k half is read; U_k is in e_tab)
    const float* e_tab[4];                    // [T][H]
    const void* w_out; const float* b_out;    // [D][H]
    const float* c1; const float* c2; const float* sg;
    float* x;              // [2][B][D] ping-pong, x[0] = x_T; result in x[steps & 1]
    const float* noise;    // [T][B][D]
    float* h;              // [2][B][H]
    unsigned* ctr;         // sync words (kSyncBytes, zeroed by the host before the launch):
                           // one 128-B line each (32 words): see SyncLine
    unsigned* status;      // abort flag (ctr + 32 * L_STATUS)
    int B, D, H, t_hi, steps;
    int hier;              // 1: XCD-hierarchical, 2: hierarchical arrival + direct poll,
                           // 0: one flat counter
    unsigned spin_limit;   // polls before a barrier wait gives up (status 1)
    unsigned long long* hg;  // replica loop: tagged h granules [8 XCDs][2][MBX][H]
    unsigned long long* xg;  // replica loop: tagged x granules [8 XCDs][2][MBX][D]
    int tagged;              // replica loop: 1 = tagged-granule hand-offs, 0 = XCD barriers
};

template <typename TW, int NJ>
__device__ __forceinline__ void load_row(float (&w)[NJ][8], const void* W, int row, int ldw,
                                         int K, int lane) {
    const int nch = K >> 3;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int c = lane + 64 * j;
        const bool on = c < nch;
        const size_t off = (size_t)row * ldw + (on ? c : 0) * 8;
        if constexpr (sizeof(TW) == 2) {
            uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const unsigned short*>(W) + off);
            const unsigned q[4] = {on ? u.x : 0u, on ? u.y : 0u, on ? u.z : 0u, on ? u.w : 0u};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[j][2 * i] = __builtin_bit_cast(float, q[i] << 16);
                w[j][2 * i + 1] = __builtin_bit_cast(float, q[i] & 0xffff0000u);
            }
        } else {
            const float* wp = reinterpret_cast<const float*>(W) + off;
            const f32x4 w0 = *reinterpret_cast<const f32x4*>(wp);
            const f32x4 w1 = *reinterpret_cast<const f32x4*>(wp + 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[j][i] = on ? w0[i] : 0.f;
                w[j][4 + i] = on ? w1[i] : 0.f;
            }
        }
    }
}

// [B][K] fp32 activations -> LDS.  The activations were written by other workgroups in this
// launch, so EVERY load of them is an agent-scope relaxed 8-byte load (global_load_dwordx2 sc1:
// bypasses this CU's L1, served coherently; Guideline 16 table row 1), 16 in flight per
// thread: one round trip for B*K <= 8192 (B=8, K=1024).
typedef unsigned long long u64;
#ifndef LDM_STAGE_IN_FLIGHT
#define LDM_STAGE_IN_FLIGHT 16
#endif
constexpr int kStageInFlight = LDM_STAGE_IN_FLIGHT;   // 8-B loads per thread per round
template <int NT = 256>
__device__ __forceinline__ void stage(float* xs, const float* X, int n2) {
    constexpr int U = kStageInFlight * 256 / NT;
    const u64* X2 = reinterpret_cast<const u64*>(X);
    for (int base = 0; base < n2; base += NT * U) {
        u64 t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * NT + (int)threadIdx.x;
            t[u] = __hip_atomic_load(X2 + (i < n2 ? i : 0), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * NT + (int)threadIdx.x;
            if (i < n2) reinterpret_cast<u64*>(xs)[i] = t[u];
        }
    }
}

// Hand-off store of one activation: write-through (sc1) 4-byte store, no release fence needed.
__device__ __forceinline__ void publish(float* p, float v) {
    __hip_atomic_store(reinterpret_cast<unsigned*>(p), __builtin_bit_cast(unsigned, v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave's row dot products for all batch rows, reduced so that lane `writer` of group b
// holds acc[0] = sum_k X[b][k] w[k] (v4's reduce-scatter).  Returns acc[0].
template <int MB, int NJ>
__device__ __forceinline__ float row_dot(const float (&w)[NJ][8], const float* xs, int B, int K,
                                         int lane) {
    const int nch = K >> 3;
    float acc[MB];
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[b] = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int c = lane + 64 * j;
        const int cc = c < nch ? c : 0;
#pragma unroll
        for (int b = 0; b < MB; ++b) {
            const int bb = b < B ? b : 0;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(xs + bb * K + cc * 8);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(xs + bb * K + cc * 8 + 4);
            float t = acc[b];
            t = fmaf(w[j][0], x0[0], t); t = fmaf(w[j][1], x0[1], t);
            t = fmaf(w[j][2], x0[2], t); t = fmaf(w[j][3], x0[3], t);
            t = fmaf(w[j][4], x1[0], t); t = fmaf(w[j][5], x1[1], t);
            t = fmaf(w[j][6], x1[2], t); t = fmaf(w[j][7], x1[3], t);
            acc[b] = t;
        }
    }
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {
        const int o = 32 >> lv;
        const int n = MB >> lv;
        const bool upper = (lane & o) != 0;
        if (n > 1) {
            const int half = n >> 1;
#pragma unroll
            for (int i = 0; i < half; ++i) {
                const float send = upper ? acc[i] : acc[i + half];
                const float keep = upper ? acc[i + half] : acc[i];
                acc[i] = keep + xor_lane(send, o, lane);
            }
        } else {
            acc[0] += xor_lane(acc[0], o, lane);
        }
    }
    return acc[0];
}

// Grid barrier (MI355X guide, Guideline 16 table row 1): every wave drains its sc1 stores,
// workgroup barrier, ONE lane adds to the monotonic counter (agent atomic) and polls it with
// relaxed sc1 loads + s_sleep; the other waves wait at the workgroup barrier.  All later loads
// of handed-off bytes are sc1 loads (stage()), so no acquire fence is needed.  Bounded: a
// timeout raises status[0], which every poller also watches, so every workgroup exits.
__device__ __forceinline__ bool grid_sync(unsigned* ctr, unsigned* status, unsigned target,
                                          int* ok, unsigned limit) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int good = 1;
        unsigned spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if ((spins & 63) == 63 &&
                __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                good = 0;
                break;
            }
            if (++spins > limit) {
                __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                good = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *ok = good;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: no hoisting
    __syncthreads();
    return *ok != 0;
}

// XCD-hierarchical variant (the guide's barrier-xcd shape): only the last arriver of each XCD
// touches the chip-wide counter; the others poll their XCD's generation word.  Arrival counts
// per XCD come from a start-up census (every workgroup adds 1 to its XCD's count, then one flat
// barrier).  Data hand-off rules are the flat barrier's (sc1 stores drained before the first
// add, sc1 loads after the last poll).
enum SyncLine { L_TOP = 0, L_STATUS = 1, L_START = 2, L_CNT = 3, L_ARR = 11, L_GEN = 19,
                L_COUNT = 27 };
static_assert(L_COUNT * 128 <= (int)kSyncBytes, "sync words overflow");


struct XcdState { unsigned xcc, n_local, n_active; };

__device__ __forceinline__ bool grid_sync_xcd(unsigned* sync, const XcdState& xs_,
                                              unsigned phase, int* ok, bool direct,
                                              unsigned limit) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned* status = sync + 32 * L_STATUS;
        unsigned* gen = sync + 32 * (L_GEN + xs_.xcc);
        const unsigned t = __hip_atomic_fetch_add(sync + 32 * (L_ARR + xs_.xcc), 1u,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool good;
        const bool last = t + 1 == phase * xs_.n_local;   // last of this XCD: go chip-wide
        if (last)
            __hip_atomic_fetch_add(sync + 32 * L_TOP, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (direct) {                                  // everyone polls the chip-wide word
            good = spin_until(sync + 32 * L_TOP, phase * xs_.n_active, status, limit);
        } else if (last) {
            good = spin_until(sync + 32 * L_TOP, phase * xs_.n_active, status, limit);
            if (good) __hip_atomic_store(gen, phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            good = spin_until(gen, phase, status, limit);
        }
        *ok = good;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
    return *ok != 0;
}

// Start-up census for grid_sync_xcd: thread 0 of every workgroup learns its XCD, the number of
// workgroups on it and the number of XCDs holding any.  Returns false on timeout.
__device__ __forceinline__ bool xcd_census(unsigned* sync, unsigned G, XcdState* st, int* ok,
                                           unsigned a_spin) {
    if (threadIdx.x == 0) {
        // HW_REG_XCC_ID (hwreg 20), bits [3:0]
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 7u;
        __hip_atomic_fetch_add(sync + 32 * (L_CNT + xcc), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        // release: the L_CNT add above is performed (visible at agent scope) before L_START
        // counts this workgroup, so a waiter that sees L_START == G reads every final count
        __hip_atomic_fetch_add(sync + 32 * L_START, 1u, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
        bool good = spin_until(sync + 32 * L_START, G, sync + 32 * L_STATUS, a_spin);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // once per launch
        unsigned n_act = 0, n_loc = 0;
        for (unsigned x = 0; x < 8; ++x) {
            const unsigned c = __hip_atomic_load(sync + 32 * (L_CNT + x), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            n_act += c > 0;
            if (x == xcc) n_loc = c;
        }
        st->xcc = xcc; st->n_local = n_loc; st->n_active = n_act;
        *ok = good;
    }
    __syncthreads();
    return *ok != 0;
}

template <typename TW, int MB, int NJD, int NJH, int NB>
__global__ __launch_bounds__(256) void sample_loop_kernel(LoopArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];  // [4] flag words, [B][max(D,H)]
    int* ok = reinterpret_cast<int*>(smem);
    float* xs = smem + 4;
    const int lane = threadIdx.x & 63;
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);           // this wave's row
    const bool has_out = m < a.D;
    const int mo = has_out ? m : a.D - 1;
    const int B = a.B, D = a.D, H = a.H;

    float wi[NJD][8], wb[NB][NJH][8], wo[NJH][8];
    load_row<TW, NJD>(wi, a.w_in, m, D, D, lane);
#pragma unroll
    for (int k = 0; k < NB; ++k) load_row<TW, NJH>(wb[k], a.w_blk[k], m, 2 * H, H, lane);
    load_row<TW, NJH>(wo, a.w_out, mo, H, H, lane);
    const float bi = a.b_in[m];
    const float bo = a.b_out[mo];

    constexpr int LB = (MB >= 16) ? 4 : 3;
    const int b = lane >> (6 - LB);
    const bool writer = (lane & ((1 << (6 - LB)) - 1)) == 0 && b < B;
    const unsigned G = gridDim.x;
    unsigned phase = 0;
    XcdState xst = {0, 0, 0};
    if (a.hier && !xcd_census(a.ctr, G, &xst, ok, a.spin_limit)) return;

    for (int s = 0; s < a.steps; ++s) {
        const int t = a.t_hi - s;
        const float* xin = a.x + (size_t)(s & 1) * B * D;
        float* xout = a.x + (size_t)((s & 1) ^ 1) * B * D;
        // This step's epilogue operands, loaded now so that their latency overlaps the
        // in-projection's staging instead of sitting behind each layer's barrier: E_k[t][m],
        // noise[t][b][m], x_t[b][m] (written by this same lane last step), c1/c2/sigma[t].
        // Every lane loads (clamped index); only writer lanes use the values.
        const int bq = b < B ? b : 0;
        const size_t io = (size_t)bq * D + mo;
        float ep[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) ep[k] = a.e_tab[k][(size_t)t * H + m];
        const float zp = a.noise[(size_t)t * B * D + io];
        const float xp = __builtin_bit_cast(float, __hip_atomic_load(
            reinterpret_cast<const unsigned*>(xin + io), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT));
        const float c1 = a.c1[t], c2 = a.c2[t], sg = a.sg[t];
        // in-projection: h0 = W_in x + b_in
        stage(xs, xin, (B * D) >> 1);
        __syncthreads();
        {
            const float acc = row_dot<MB, NJD>(wi, xs, B, D, lane);
            if (writer) publish(a.h + (size_t)b * H + m, acc + bi);
        }
        ++phase;
        if (!(a.hier ? grid_sync_xcd(a.ctr, xst, phase, ok, a.hier == 2, a.spin_limit)
                     : grid_sync(a.ctr + 32 * L_TOP, a.status, phase * G, ok, a.spin_limit))) return;
        // residual blocks: h <- h + SiLU(W_k h + E_k[t])
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const float* hin = a.h + (size_t)(k & 1) * B * H;
            float* hout = a.h + (size_t)((k + 1) & 1) * B * H;
            stage(xs, hin, (B * H) >> 1);
            __syncthreads();
            const float acc = row_dot<MB, NJH>(wb[k], xs, B, H, lane);
            if (writer) {
                const float pre = acc + ep[k];
                publish(hout + (size_t)b * H + m, xs[b * H + m] + silu(pre));
            }
            ++phase;
        if (!(a.hier ? grid_sync_xcd(a.ctr, xst, phase, ok, a.hier == 2, a.spin_limit)
                     : grid_sync(a.ctr + 32 * L_TOP, a.status, phase * G, ok, a.spin_limit))) return;
        }
        // out-projection with the A8 update fused
        stage(xs, a.h + (size_t)(NB & 1) * B * H, (B * H) >> 1);
        __syncthreads();
        if (has_out) {
            const float acc = row_dot<MB, NJH>(wo, xs, B, H, lane);
            if (writer) {
                const float pre = acc + bo;
                const size_t i = (size_t)b * D + m;
                const bool noise = t > 0;
                publish(xout + i, ddpm_update(xp, pre, noise ? zp : 0.f, c1, c2, sg, noise));
            }
        }
        ++phase;
        if (!(a.hier ? grid_sync_xcd(a.ctr, xst, phase, ok, a.hier == 2, a.spin_limit)
                     : grid_sync(a.ctr + 32 * L_TOP, a.status, phase * G, ok, a.spin_limit))) return;
    }
}

// ------------------------------------------------------------------------------------------
// XCD-replica loop (bf16 weights).  Each of the 8 XCDs holds a FULL copy of the network in its
// G/8 workgroups' registers (bf16 pairs, ~300 VGPRs per lane) and samples the shapes
// b == xcd (mod 8) on its own, so a layer boundary is a barrier of the G/8 workgroups of one
// XCD instead of the whole chip (no chip-wide hop).  Wave gw (0..127) of a
// replica owns rows gw*8 .. gw*8+7 of the in-projection and of every block, and D/128 rows of
// the out-projection.  Per row the arithmetic is the per-step kernels' exactly: the same
// k-to-lane map and fma order, and a reduce-scatter over (row, shape) pairs whose butterfly
// visits the lanes in the same order as the batch reduce-scatter (floating-point addition is
// commutative, so each sum is the same bits) -- the loop stays bit-identical to the graph path.
// Placement: workgroups learn their XCD from HW_REG_XCC_ID; if an XCD holds other than G/8 of
// them the launch reports status 2 and returns before any compute (the host then uses the
// chip-wide loop), so correctness never rests on the dispatch order.

template <int NR, int NJ>
__device__ __forceinline__ void load_rows_bf16(u32x4 (&w)[NR][NJ], const void* W, int row0,
                                               int ldw, int K, int lane) {
    const int nch = K >> 3;
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int c = lane + 64 * j;
            const bool on = c < nch;
            const u32x4 u = *reinterpret_cast<const u32x4*>(
                reinterpret_cast<const unsigned short*>(W) + (size_t)(row0 + r) * ldw +
                (on ? c : 0) * 8);
            w[r][j] = on ? u : u32x4{0u, 0u, 0u, 0u};
        }
}

// vals[r * MBX + b] = this lane's partial dot product of row r with shape b (row_dot's chain);
// rows NW..NR-1 have no weights and stay 0 (padding of the reduce-scatter).  wget(r, j) returns
// the lane's 8 bf16 weights (u32x4) of row r, chunk j -- registers or LDS.
template <int NR, int NW, int NJ, int MBX, typename WGet>
__device__ __forceinline__ void rows_partial(float (&vals)[NR * MBX], WGet wget, const float* xs,
                                             int K, int lane) {
    const int nch = K >> 3;
#pragma unroll
    for (int q = 0; q < NR * MBX; ++q) vals[q] = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int c = lane + 64 * j;
        const int cc = c < nch ? c : 0;
#pragma unroll
        for (int b = 0; b < MBX; ++b) {
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(xs + b * K + cc * 8);
            const f32x4 x1 = *reinterpret_cast<const f32x4*>(xs + b * K + cc * 8 + 4);
#pragma unroll
            for (int r = 0; r < NW; ++r) {
                u32x4 u4 = wget(r, j);
                // opaque to the optimiser: the bf16 -> fp32 unpack then stays here instead of
                // being hoisted out of the step loop as 2x the registers (which spilled)
                asm volatile("" : "+v"(u4));
                float wf[8];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const unsigned u = u4[i];
                    wf[2 * i] = __builtin_bit_cast(float, u << 16);
                    wf[2 * i + 1] = __builtin_bit_cast(float, u & 0xffff0000u);
                }
                float t = vals[r * MBX + b];
                t = fmaf(wf[0], x0[0], t); t = fmaf(wf[1], x0[1], t);
                t = fmaf(wf[2], x0[2], t); t = fmaf(wf[3], x0[3], t);
                t = fmaf(wf[4], x1[0], t); t = fmaf(wf[5], x1[1], t);
                t = fmaf(wf[6], x1[2], t); t = fmaf(wf[7], x1[3], t);
                vals[r * MBX + b] = t;
            }
        }
    }
}

// row_dot's reduce-scatter over NV values: lane group q = lane >> (6 - log2 NV) ends with
// vals[0] = the full sum of value q.
template <int NV>
__device__ __forceinline__ float reduce_scatter(float (&acc)[NV], int lane) {
    static_assert(NV == 2 || NV == 4 || NV == 8 || NV == 16, "power-of-two value count");
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {
        const int o = 32 >> lv;
        const int n = NV >> lv;
        const bool upper = (lane & o) != 0;
        if (n > 1) {
            const int half = n >> 1;
#pragma unroll
            for (int i = 0; i < half; ++i) {
                const float send = upper ? acc[i] : acc[i + half];
                const float keep = upper ? acc[i + half] : acc[i];
                acc[i] = keep + xor_lane(send, o, lane);
            }
        } else {
            acc[0] += xor_lane(acc[0], o, lane);
        }
    }
    return acc[0];
}


// Data-tagged granule hand-off (MI355X guide: handoff-1to1 / allgather rows, "keep 8-byte
// granules, flat sweep").  A producer stores {value, tag} as ONE 8-byte agent-scope store
// (single-copy atomic: a reader sees the old pair or the new one); a consumer sweeps the
// granules it needs with agent-scope (L1-bypassing) 8-byte loads and re-polls any whose tag is
// not yet the layer's.  The data is its own flag: no arrival counter, no generation word, no
// drain before a flag -- one L2 round trip after the last producer's store instead of the
// barrier's three.  Tags are the launch's phase numbers (1, 2, ...); the host zeroes the
// granules before every launch, so no stale tag can match.  Double buffering is WAR-safe by
// data dependence: a workgroup can only hold every granule of layer k+1 once every workgroup
// has published its layer-k+1 rows, i.e. finished reading layer k; layer k+2 then overwrites
// layer k's buffer (the same argument holds for the x ping-pong between steps).
__device__ __forceinline__ void publish_tagged(u64* g, float v, unsigned tag) {
    const u64 w = ((u64)tag << 32) | __builtin_bit_cast(unsigned, v);
    __hip_atomic_store(g, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// n granules -> xs[0..n), every thread granules tid, tid + NT, ... (all loads issued before any
// tag test).  Returns false (and sets the status word) if a granule never arrives.
// Re-polls a missing granule back to back (LDM_GRAN_SLEEP = 0): measured at B = 8, 74.5k steps/s
// vs 72.0-72.7k with s_sleep 1 and 64.3k with s_sleep 3 (profiles/r03l/ab_sleep.log).
#ifndef LDM_GRAN_SLEEP
#define LDM_GRAN_SLEEP 0
#endif
template <int NT, int U>
__device__ __forceinline__ bool stage_tagged(float* xs, const u64* G, int n, unsigned tag,
                                             unsigned* status, unsigned limit) {
    bool good = true;
    for (int base = 0; base < n; base += NT * U) {
        u64 t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * NT + (int)threadIdx.x;
            t[u] = __hip_atomic_load(G + (i < n ? i : 0), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * NT + (int)threadIdx.x;
            if (i < n) {
                unsigned spins = 0;
                while ((unsigned)(t[u] >> 32) != tag) {
                    if ((spins & 63) == 63 &&
                        __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        good = false;
                        break;
                    }
                    if (++spins > limit) {
                        __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        good = false;
                        break;
                    }
#if LDM_GRAN_SLEEP > 0
                    __builtin_amdgcn_s_sleep(LDM_GRAN_SLEEP);
#endif
                    t[u] = __hip_atomic_load(G + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                xs[i] = __builtin_bit_cast(float, (unsigned)t[u]);
            }
        }
    }
    return good;
}

constexpr int kRepWaves = 8;      // 2 waves per SIMD: 4 rows of each layer per wave

// Phase stamps (scripts/stamp_sampler.py reads them through ldm_dev_sample_stamps): every wave
// of the replica loop keeps per-phase sums of s_memrealtime ticks (100 MHz) in registers over
// all its layers -- 0 own granules landed, 1 the workgroup's staging barrier (the slowest wave's
// granules), 2 the row dot products, 3 the reduce-scatter, 4 epilogue + publish -- and writes
// them at its end (g_sl_stamp[workgroup][wave]); slot 5 counts the layers.
// Diagnostic builds only (-DSL_STAMP=1).  Round 5 shipped them ON because the stamped build ran
// 86.5-88.2k steps/s at B = 8 against 72.0-74.4k without; its explanation (index products in
// SALU instead of VALU) was wrong -- those v_mul_lo_u32 sit in the barrier form's arrival code,
// which the tagged hand-offs never run.  Round 6 found the real difference in the assembly: both
// builds SPILLED (116-132 bytes of scratch at 255-256 VGPRs), and each step reloaded 5-6 of a
// residual block's register-resident weight vectors from scratch, one serial
// scratch_load + s_waitcnt vmcnt(0) after another; the stamps merely moved one reload.  The fix
// is SL_LDSBLK below: no spills at all, with or without stamps (tests/test_sampler_codegen.py
// pins it).
#ifndef SL_STAMP
#define SL_STAMP 0
#endif
// Residual blocks whose weights live in LDS instead of registers (the LAST SL_LDSBLK blocks):
// the 4 blocks' register-resident weights (128 VGPRs) + the loop's state overflowed the 256
// VGPRs a wave has at 2 waves per SIMD, so the compiler spilled weight vectors and reloaded them
// serially every step.  One block in LDS (64 KiB per workgroup, read as 8 ds_read_b128 per wave
// per step) frees 32 VGPRs: no scratch at all.  Same arithmetic (the
// lane's 8 bf16 weights, the same fma chain), so the loop stays bit-identical to the graph path.
#ifndef SL_LDSBLK
#define SL_LDSBLK 1
#endif
// After a layer's publish: the publishing store stays ahead of the next layer's granule polls
// in issue order (a scheduling barrier), and the wave sleeps one interval (64 cycles) before it
// starts polling -- fewer polls hit the lines the other producers are still writing (the
// pause's length: SL_PUBSLEEP below).  What the
// round-5 stamps did by accident (their mark after the publish: SL_MARKS = 16 alone carried the
// whole gain, profiles/r06d), now on purpose.  A/B on one box (profiles/r06f, B = 8, steps/s):
// 0 nothing 84.9-85.9k; 1 the barrier alone 92.4-93.0k; 2 an s_memrealtime read instead 92.9-
// 93.6k; 3 barrier + s_sleep 1 96.5-99.0k (the product form); 4 the stamp's clock arithmetic kept in a
// register 97.1-98.1k; the round-5 mark itself 96.7-98.1k.  tests/test_sampler_codegen.py pins
// the sleep behind every publish.
#ifndef SL_PUBFENCE
#define SL_PUBFENCE 3
#endif
// The pause, in s_sleep units of 64 cycles.  Swept on one box (profiles/r06s, r06t, B = 8,
// steps/s): 1 96.3-98.6k, 2 100.6-101.8k, 3 101.8-104.5k, 4 104.1-104.7k, 6 102.1-103.0k,
// 8 99.7-100.3k, 12 94.8-95.2k; a sleep between re-polls of a missing granule instead
// (LDM_GRAN_SLEEP 1) 90-94k.
// Double-buffered activation stage (SL_XSDB 1): layer L stages into xs[L & 1] and its abort
// flag is slot L % 3, so the workgroup barrier BEFORE a layer's granule polls (the WAR guard on
// the single xs buffer, and the flag reset) goes.  WAR on xs[L & 1]: its last reads were layer
// L - 2's rows, and every wave finishes those before it arrives at layer L - 1's post-poll
// barrier, which every writer of layer L has passed.  Flag slot (L + 1) % 3 is reset during
// layer L by thread 0: its last readers (layer L - 2, right after their post-poll barrier)
// passed layer L - 1's barrier before thread 0 could get here, and any layer-(L + 1) failure
// write comes after layer L's barrier, which thread 0 reaches only after the reset.
#ifndef SL_XSDB
#define SL_XSDB 0
#endif
#ifndef SL_POLLW
#define SL_POLLW 8
#endif
#ifndef SL_PUBSLEEP
#define SL_PUBSLEEP 4
#endif
__device__ __forceinline__ void after_publish() {
    if (SL_PUBFENCE == 1) __builtin_amdgcn_sched_barrier(0);
    if (SL_PUBFENCE == 2) {
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        asm volatile("" ::"s"(t));
    }
    if (SL_PUBFENCE == 3) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_sleep(SL_PUBSLEEP);
    }
}
// SL_PUBFENCE 4: the round-5 stamp's mark 4 alone, kept in a register (no global stamp buffer):
// the elapsed time since the previous publish accumulated per wave, consumed at the end
struct PubClock {
    uint64_t t = 0, acc = 0;
    __device__ __forceinline__ void start() {
        if (SL_PUBFENCE == 4) t = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ void mark() {
        if (SL_PUBFENCE == 4) {
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            acc += now - t;
            t = now;
        }
    }
    __device__ __forceinline__ void end() {
        if (SL_PUBFENCE == 4) asm volatile("" ::"s"(acc));
    }
};
// SL_MARKS (A/B builds only): a bit mask of the marks to keep without the rest of the stamps
#ifndef SL_MARKS
#define SL_MARKS 0
#endif
#define SL_ANY (SL_STAMP || SL_MARKS)
#ifndef SL_PRIO
#define SL_PRIO 0
#endif
#ifndef SL_NAPS
#define SL_NAPS 0
#endif
#if SL_ANY
__device__ unsigned long long g_sl_stamp[256][kRepWaves][8];
#endif
struct SlStamp {
    uint64_t acc[6] = {0, 0, 0, 0, 0, 0};
    uint64_t t = 0;
    __device__ __forceinline__ void start() {
        if (SL_ANY) t = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ void mark(int k) {
        if ((SL_NAPS >> k) & 1) __builtin_amdgcn_s_sleep(1);
        if (SL_STAMP || ((SL_MARKS >> k) & 1)) {
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            acc[k] += now - t;
            t = now;
        }
    }
    __device__ __forceinline__ void flush(int wave) {
#if SL_ANY
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 256)
            for (int i = 0; i < 6; ++i) g_sl_stamp[blockIdx.x][wave][i] = acc[i];
#endif
    }
};

template <int D_, int MBX>
__global__ __launch_bounds__(64 * kRepWaves) void sample_replica_kernel(LoopArgs a) {
    constexpr int H = 1024, NB = 4, NWV = kRepWaves, R = H / (32 * NWV), RO = D_ / (32 * NWV);
    constexpr int NJD = (D_ + 511) / 512, NJH = 2;
    constexpr int NV = R * MBX, LB = NV >= 16 ? 4 : NV >= 8 ? 3 : NV >= 4 ? 2 : 1;
    constexpr int NT = 64 * NWV;
    static_assert(RO * MBX <= NV, "out-projection values fit the reduce-scatter");
    // LDS: [4] flags | xs [1 + SL_XSDB][MBX][H] | in-proj weights [8 waves][R][NJD][64 lanes] u32x4 |
    //      out-proj weights [8 waves][RO][NJH][64] u32x4 | the last SL_LDSBLK blocks' weights
    //      [SL_LDSBLK][8 waves][R][NJH][64] u32x4.  The other residual blocks' weights (32 VGPRs
    //      of bf16 pairs each) live in registers.
    extern __shared__ __attribute__((aligned(16))) float smem[];
    int* ok = reinterpret_cast<int*>(smem);
    float* const xsb = smem + 4;                         // [1 + SL_XSDB][MBX][H]
    float* xs = xsb;
    u32x4* lwi = reinterpret_cast<u32x4*>(smem + 4 + (1 + SL_XSDB) * MBX * H);
    u32x4* lwo = lwi + NWV * R * NJD * 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned* sync = a.ctr;
    const unsigned G = gridDim.x;

    // ---- census: XCD id, local rank, equal split check -----------------------------------
    __shared__ unsigned s_xcc, s_rank, s_nloc;
    if (threadIdx.x == 0) {
        unsigned xcc, rank;
        const bool good = replica_census(sync, G, a.spin_limit, &xcc, &rank);
        s_xcc = xcc; s_rank = rank; s_nloc = G / 8;
        *ok = good;
    }
    __syncthreads();
    if (!*ok) return;
    const unsigned xcc = s_xcc, nloc = s_nloc;
    // every wave has read ok[0] above; the slots are set before the first layer's barrier
    // (the step-0 in-projection stage's)
    if (threadIdx.x == 0) ok[0] = ok[1] = ok[2] = 1;
    const int B = a.B, D = D_;
    const int nsh = (B > (int)xcc) + (B > (int)xcc + 8);     // shapes of this replica
    if (nsh == 0) return;                                     // idle replica (B < 8)
    const int gw = (int)s_rank * NWV + wave;                  // 0 .. 32 NWV - 1
    const int row0 = gw * R, orow0 = gw * RO;

    constexpr int NBR = NB - SL_LDSBLK;                  // blocks with register weights
    static_assert(NBR >= 1 && NBR <= NB, "SL_LDSBLK in 0..3");
    u32x4 wb[NBR][R][NJH];
#pragma unroll
    for (int k = 0; k < NBR; ++k) load_rows_bf16<R, NJH>(wb[k], a.w_blk[k], row0, 2 * H, H, lane);
    // blocks NBR.. in LDS: [block][wave][R][NJH][64 lanes] u32x4, past the projections
    u32x4* lwb = lwi + NWV * R * NJD * 64 + NWV * RO * NJH * 64;
#pragma unroll
    for (int k = NBR; k < NB; ++k) {
        u32x4 wl[R][NJH];
        load_rows_bf16<R, NJH>(wl, a.w_blk[k], row0, 2 * H, H, lane);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < NJH; ++j)
                lwb[((((k - NBR) * NWV + wave) * R + r) * NJH + j) * 64 + lane] = wl[r][j];
    }
    {
        u32x4 wi[R][NJD], wo[RO][NJH];
        load_rows_bf16<R, NJD>(wi, a.w_in, row0, D, D, lane);
        load_rows_bf16<RO, NJH>(wo, a.w_out, orow0, H, H, lane);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < NJD; ++j) lwi[((wave * R + r) * NJD + j) * 64 + lane] = wi[r][j];
#pragma unroll
        for (int r = 0; r < RO; ++r)
#pragma unroll
            for (int j = 0; j < NJH; ++j) lwo[((wave * RO + r) * NJH + j) * 64 + lane] = wo[r][j];
    }
    auto get_in = [&](int r, int j) { return lwi[((wave * R + r) * NJD + j) * 64 + lane]; };
    auto get_out = [&](int r, int j) { return lwo[((wave * RO + r) * NJH + j) * 64 + lane]; };

    const int q = lane >> (6 - LB);                     // value index this lane finishes
    const bool qlead = (lane & ((1 << (6 - LB)) - 1)) == 0;
    const int qr = q / MBX, qb = q % MBX;                 // (row, shape) of value q
    const int sb = (int)xcc + 8 * qb;                    // global shape index
    const bool wr_h = qlead && qb < nsh;                 // writes an H-wide row
    const bool wr_o = wr_h && qr < RO;                   // writes an out-projection row
    const int mh = row0 + qr, mo = orow0 + (qr < RO ? qr : 0);
    const float bi = a.b_in[mh];
    const float bo = a.b_out[mo];
    float* hrep = a.h + (size_t)xcc * 2 * MBX * H;       // [2][MBX][H] per replica
    u64* hgr = a.hg + (size_t)xcc * 2 * MBX * H;          // tagged: [2][MBX][H] per replica
    u64* xgr = a.xg + (size_t)xcc * 2 * MBX * D_;         // tagged: [2][MBX][D] per replica
    const bool tagged = a.tagged != 0;
    unsigned* status = sync + 32 * R_STATUS;
    unsigned phase = 0;
    // layer boundary: the barrier form publishes, then waits for the XCD's workgroups; the
    // tagged form has nothing to wait for here (the next layer's stage polls the data)
    auto boundary = [&]() -> bool {
        if (tagged) return true;
        return replica_sync(sync, xcc, nloc, phase, ok, a.spin_limit);
    };
    // stage this replica's [MBX][K] activations of the layer that published under tag `tg`
    SlStamp stp;
    // each staged layer's buffer and abort-flag slot (SL_XSDB), in the order every wave stages
    int lyr = 0;
    int* okc = ok;
    auto begin_layer = [&]() {
        if (SL_XSDB) {
            xs = xsb + (size_t)(lyr & 1) * MBX * H;
            okc = ok + lyr % 3;
            if (threadIdx.x == 0) ok[(lyr + 1) % 3] = 1;
        }
        ++lyr;
    };
    auto stage_act = [&](float* dst, const float* plain, const u64* gran, int K, unsigned tg) {
        if (!tagged || gran == nullptr) {
#pragma unroll
            for (int b = 0; b < MBX; ++b) stage<NT>(dst + b * K, plain + (size_t)b * K, K >> 1);
            __syncthreads();
            return true;
        }
        if (!SL_XSDB) {
            if (threadIdx.x == 0) *okc = 1;
            __syncthreads();
        }
        // only this replica's nsh shapes are published (rows of a missing second shape are
        // computed on whatever the LDS holds and never written)
#if SL_PRIO
        __builtin_amdgcn_s_setprio(0);           // (A/B) polling waves yield issue to computing ones
#endif
        // (SL_POLLW < 8, A/B builds: only the first SL_POLLW waves poll, more granules each)
        bool good = true;
        if constexpr (SL_POLLW >= kRepWaves) {
            good = stage_tagged<NT, 2>(dst, gran, nsh * K, tg, status, a.spin_limit);
        } else {
            if (wave < SL_POLLW)
                good = stage_tagged<64 * SL_POLLW, 2 * kRepWaves / SL_POLLW>(
                    dst, gran, nsh * K, tg, status, a.spin_limit);
        }
#if SL_PRIO
        __builtin_amdgcn_s_setprio(SL_PRIO);
#endif
        stp.mark(0);
        if (!good) *okc = 0;
        __syncthreads();
        stp.mark(1);
        return *okc != 0;
    };
    stp.start();
    PubClock pclk;
    pclk.start();

    for (int s = 0; s < a.steps; ++s) {
        const int t = a.t_hi - s;
        const float* xin = a.x + (size_t)(s & 1) * B * D;
        float* xout = a.x + (size_t)((s & 1) ^ 1) * B * D;
        const int sq = qb < nsh ? sb : (int)xcc;
        float ep[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) ep[k] = a.e_tab[k][(size_t)t * H + mh];
        const float zp = a.noise[(size_t)t * B * D + (size_t)sq * D + mo];
        const float xp = __builtin_bit_cast(float, __hip_atomic_load(
            reinterpret_cast<const unsigned*>(xin + (size_t)sq * D + mo), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT));
        const float c1 = a.c1[t], c2 = a.c2[t], sg = a.sg[t];
        // in-projection over this replica's shapes (step 0: the caller's x; later: the
        // previous out-projection's tagged granules)
        begin_layer();
        if (tagged && s > 0) {
            if (!stage_act(xs, nullptr, xgr + (size_t)(s & 1) * MBX * D, D, phase)) return;
        } else {
#pragma unroll
            for (int b = 0; b < MBX; ++b)
                stage<NT>(xs + b * D, xin + (size_t)((int)xcc + 8 * (b < nsh ? b : 0)) * D, D >> 1);
            __syncthreads();
        }
        {
            float v[NV];
            rows_partial<R, R, NJD, MBX>(v, get_in, xs, D, lane);
            stp.mark(2);
            const float acc = reduce_scatter<NV>(v, lane);
            stp.mark(3);
            ++phase;
            if (wr_h) {
                if (tagged) publish_tagged(hgr + (size_t)qb * H + mh, acc + bi, phase);
                else publish(hrep + (size_t)qb * H + mh, acc + bi);
            }
            after_publish();
            pclk.mark();
            stp.mark(4);
            if (SL_STAMP) stp.acc[5] += 1;
        }
        if (!boundary()) return;
        // the four blocks as four compile-time copies (a runtime block index into wb would
        // put the register-resident weights in scratch)
        bool alive = true;
        auto block = [&](auto KC) {
            constexpr int k = decltype(KC)::value;
            if (!alive) return;
            const float* hin = hrep + (size_t)(k & 1) * MBX * H;
            float* hout = hrep + (size_t)((k + 1) & 1) * MBX * H;
            begin_layer();
            if (!stage_act(xs, hin, tagged ? hgr + (size_t)(k & 1) * MBX * H : nullptr, H,
                           phase)) {
                alive = false;
                return;
            }
            float v[NV];
            if constexpr (k < NBR)
                rows_partial<R, R, NJH, MBX>(v, [&](int r, int j) { return wb[k][r][j]; }, xs,
                                             H, lane);
            else
                rows_partial<R, R, NJH, MBX>(v, [&](int r, int j) {
                    return lwb[((((k - NBR) * NWV + wave) * R + r) * NJH + j) * 64 + lane];
                }, xs, H, lane);
            stp.mark(2);
            const float acc = reduce_scatter<NV>(v, lane);
            stp.mark(3);
            ++phase;
            if (wr_h) {
                const float pre = acc + ep[k];
                const float hv = xs[qb * H + mh] + silu(pre);
                if (tagged) publish_tagged(hgr + (size_t)((k + 1) & 1) * MBX * H + (size_t)qb * H + mh, hv, phase);
                else publish(hout + (size_t)qb * H + mh, hv);
            }
            after_publish();
            pclk.mark();
            stp.mark(4);
            if (SL_STAMP) stp.acc[5] += 1;
            alive = boundary();
        };
        static_assert(NB == 4, "four residual blocks");
        block(std::integral_constant<int, 0>{});
        block(std::integral_constant<int, 1>{});
        block(std::integral_constant<int, 2>{});
        block(std::integral_constant<int, 3>{});
        if (!alive) return;
        begin_layer();
        if (!stage_act(xs, hrep + (size_t)(NB & 1) * MBX * H,
                       tagged ? hgr + (size_t)(NB & 1) * MBX * H : nullptr, H, phase))
            return;
        {
            float v[NV];
            // out-projection: RO rows, zero-padded to the R-row reduce-scatter
            rows_partial<R, RO, NJH, MBX>(v, get_out, xs, H, lane);
            stp.mark(2);
            const float acc = reduce_scatter<NV>(v, lane);
            stp.mark(3);
            ++phase;
            if (wr_o) {
                const float pre = acc + bo;
                const bool noise = t > 0;
                const float xv = ddpm_update(xp, pre, noise ? zp : 0.f, c1, c2, sg, noise);
                publish(xout + (size_t)sb * D + mo, xv);          // the caller's ping-pong
                if (tagged)
                    publish_tagged(xgr + (size_t)((s & 1) ^ 1) * MBX * D + (size_t)qb * D + mo,
                                   xv, phase);
            }
            after_publish();
            pclk.mark();
            stp.mark(4);
            if (SL_STAMP) stp.acc[5] += 1;
        }
        if (!boundary()) return;
    }
    stp.flush(wave);
    pclk.end();
}

// Residency: every workgroup of the grid must be resident at once (the grid barriers wait for
// all of them).  Checked against the occupancy query x CU count before each plain launch; a
// cooperative launch would make the same check at +15-19 us per call (MI355X guide,
// coop-launch) and crashed rocprofv3 at process exit here.  Spins stay bounded regardless.
template <typename TW, int MB>
bool loop_resident(int B, int D, int H) {
    const size_t lds = 16 + (size_t)B * (H > D ? H : D) * sizeof(float);
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return false;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, (const void*)sample_loop_kernel<TW, MB, 1, 2, 4>, 256, lds) != hipSuccess)
        return false;
    return (long)per_cu * cus >= H / 4;
}

bool loop_resident_any(int dtype, int B, int D, int H) {
    if (dtype == LDM_BF16)
        return B <= 8 ? loop_resident<unsigned short, 8>(B, D, H)
                      : loop_resident<unsigned short, 16>(B, D, H);
    return B <= 8 ? loop_resident<float, 8>(B, D, H) : loop_resident<float, 16>(B, D, H);
}

// The replica loop needs exactly H/4 = 256 workgroups resident, G/8 per XCD (checked in the
// kernel: status 2 otherwise).  Once a launch has reported status 2 on a device, later
// launches on that device take the chip-wide loop.  Per-device host state (device ordinals
// < kMaxDev; the library is re-entrant per device, and these words are only ever flipped one
// way or set by the explicit debug call ldm_sample_loop_config).
constexpr int kMaxDev = 64;
std::atomic<bool> g_replica_off[kMaxDev];
// ldm_sample_loop_config (A/B and fault-injection tests only): form, spin limit, tagged
struct LoopConfig {
    std::atomic<int> form{LDM_LOOP_AUTO};
    std::atomic<unsigned> spin_limit{0};
    std::atomic<int> tagged{1};
};
LoopConfig g_cfg[kMaxDev];
std::atomic<int> g_last_form[kMaxDev];

int cur_dev() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDev) d = 0;
    return d;
}

size_t replica_lds(int D, int MBX) {
    const int H = 1024, W = kRepWaves, R = H / (32 * W), RO = D / (32 * W);
    const int NJD = (D + 511) / 512, NJH = 2;
    return 16 + (size_t)(1 + SL_XSDB) * MBX * H * 4 +
           (size_t)W * (R * NJD + RO * NJH + SL_LDSBLK * R * NJH) * 64 * 16;
}

template <int D_, int MBX>
bool replica_resident() {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return false;
    const size_t lds = replica_lds(D_, MBX);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, (const void*)sample_replica_kernel<D_, MBX>, 64 * kRepWaves, lds) != hipSuccess)
        return false;
    return per_cu >= 1 && (long)per_cu * cus >= 256;
}

bool replica_ok(const ldm_denoiser_t* w, int B) {
    if (g_replica_off[cur_dev()].load() || w->dtype != LDM_BF16 || w->H != 1024 || w->n_blocks != 4) return false;
    if (w->D == 256) return B <= 8 ? replica_resident<256, 1>() : replica_resident<256, 2>();
    if (w->D == 512) return B <= 8 ? replica_resident<512, 1>() : replica_resident<512, 2>();
    return false;
}

int launch_replica(const LoopArgs& a, hipStream_t s) {
    const size_t lds = replica_lds(a.D, a.B <= 8 ? 1 : 2);
    const dim3 grid(a.H / 4), blk(64 * kRepWaves);
    if (a.D == 256) {
        if (a.B <= 8) hipLaunchKernelGGL((sample_replica_kernel<256, 1>), grid, blk, lds, s, a);
        else hipLaunchKernelGGL((sample_replica_kernel<256, 2>), grid, blk, lds, s, a);
    } else {
        if (a.B <= 8) hipLaunchKernelGGL((sample_replica_kernel<512, 1>), grid, blk, lds, s, a);
        else hipLaunchKernelGGL((sample_replica_kernel<512, 2>), grid, blk, lds, s, a);
    }
    return launch_status("sample_loop (replica)");
}

template <typename TW, int MB>
int launch_loop(const LoopArgs& a, hipStream_t s) {
    const size_t lds = 16 + (size_t)a.B * (a.H > a.D ? a.H : a.D) * sizeof(float);
    hipLaunchKernelGGL((sample_loop_kernel<TW, MB, 1, 2, 4>), dim3(a.H / 4), dim3(256), lds, s, a);
    return launch_status("sample_loop");
}

}  // namespace
}  // namespace ldm

using namespace ldm;

// ws = [activations: 32 H floats (chip-wide loop: [2][B][H], B <= 16; replica loop:
// [8 XCDs][2][MBX <= 2][H])] [sync words: kSyncBytes] [replica loop's tagged granules:
// h [8][2][2][H] then x [8][2][2][512], 8 bytes each; zeroed with the sync words per launch]
static size_t act_floats(int H) { return (size_t)32 * H; }
static size_t gran_bytes(int H) { return (size_t)8 * 2 * 2 * (H + 512) * 8; }

extern "C" size_t ldm_sample_loop_ws_bytes(int B, int H) {
    (void)B;
    return act_floats(H) * sizeof(float) + kSyncBytes + gran_bytes(H);
}

extern "C" int ldm_sample_loop_supported(const ldm_denoiser_t* w, int B) {
    if (!w || B < 1 || B > 16) return 0;
    if (w->n_blocks != 4 || w->H != 1024) return 0;
    if (w->D != 256 && w->D != 512) return 0;
    if (w->dtype != LDM_BF16 && w->dtype != LDM_F32) return 0;
    return loop_resident_any(w->dtype, B, w->D, w->H) ? 1 : 0;
}

extern "C" int ldm_sample_loop(const ldm_denoiser_t* w, const ldm_sched_t* sc, float* x,
                               const float* noise, int t_hi, int steps, int B, float* ws,
                               size_t ws_bytes, ldm_stream_t s) {
    LDM_REQUIRE(w && sc && x && noise && ws, LDM_EINVAL, "sample_loop: null argument");
    LDM_REQUIRE(ldm_sample_loop_supported(w, B), LDM_ENOSYS,
                "sample_loop: persistent path needs H=1024, D in {256,512}, 4 blocks, B<=16 "
                "(got H=%d D=%d blocks=%d B=%d)", w->H, w->D, w->n_blocks, B);
    LDM_REQUIRE(steps >= 1 && t_hi >= 0 && t_hi < w->T && t_hi < sc->T && t_hi - steps + 1 >= 0,
                LDM_EINVAL, "sample_loop: steps %d from t=%d outside the schedule", steps, t_hi);
    LDM_REQUIRE(ws_bytes >= ldm_sample_loop_ws_bytes(B, w->H), LDM_EINVAL,
                "sample_loop: workspace %zu B < %zu B", ws_bytes, ldm_sample_loop_ws_bytes(B, w->H));
    LDM_REQUIRE(LDM_ALIGNED(x, 16) && LDM_ALIGNED(ws, 256) && LDM_ALIGNED(noise, 16),
                LDM_EALIGN, "sample_loop: misaligned buffers");
    LoopArgs a = {};
    a.w_in = w->w_in; a.b_in = w->b_in;
    for (int k = 0; k < 4; ++k) { a.w_blk[k] = w->w_blk[k]; a.e_tab[k] = w->e_tab[k]; }
    a.w_out = w->w_out; a.b_out = w->b_out;
    a.c1 = sc->c1; a.c2 = sc->c2; a.sg = sc->sigma;
    a.x = x; a.noise = noise;
    a.h = ws;
    a.ctr = reinterpret_cast<unsigned*>(ws + act_floats(w->H));
    a.status = a.ctr + 32 * L_STATUS;
    const int dev = cur_dev();
    const LoopConfig& cfg = g_cfg[dev];
    const int form = cfg.form.load();
    // AUTO / REPLICA: one network copy per XCD, XCD-local hand-offs (bf16 weights; else the
    // chip-wide loop with the XCD barrier); XCD: chip-wide loop, XCD-hierarchical barrier with
    // per-XCD generation words; DIRECT: hierarchical arrival, every workgroup polls the
    // chip-wide word; FLAT: one counter for everything
    const bool replica = (form == LDM_LOOP_AUTO || form == LDM_LOOP_REPLICA) && replica_ok(w, B);
    a.hier = form == LDM_LOOP_FLAT ? 0 : form == LDM_LOOP_DIRECT ? 2 : 1;
    a.B = B; a.D = w->D; a.H = w->H; a.t_hi = t_hi; a.steps = steps;
    a.spin_limit = kSpinLimit;
    {
        const unsigned v = cfg.spin_limit.load();
        if (v >= 1 && v < kSpinLimit) a.spin_limit = v;
    }
    for (int k = 0; k < 4; ++k)
        LDM_REQUIRE(a.w_blk[k] && a.e_tab[k], LDM_EINVAL, "sample_loop: block %d missing", k);
    a.hg = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(a.ctr) + kSyncBytes);
    a.xg = a.hg + (size_t)8 * 2 * 2 * w->H;
    // replica hand-offs: tagged granules (default) or XCD-local barriers (tagged = 0, A/B)
    a.tagged = cfg.tagged.load() ? 1 : 0;
    hipStream_t st = (hipStream_t)s;
    const size_t zero = kSyncBytes + (replica && a.tagged ? gran_bytes(w->H) : 0);
    if (hipMemsetAsync(a.ctr, 0, zero, st) != hipSuccess) return launch_status("sample_loop memset");
    g_last_form[dev].store(replica ? LDM_LOOP_REPLICA
                           : a.hier == 0 ? LDM_LOOP_FLAT : a.hier == 2 ? LDM_LOOP_DIRECT
                                                                       : LDM_LOOP_XCD);
    if (replica) return launch_replica(a, st);
    if (w->dtype == LDM_BF16)
        return B <= 8 ? launch_loop<unsigned short, 8>(a, st) : launch_loop<unsigned short, 16>(a, st);
    return B <= 8 ? launch_loop<float, 8>(a, st) : launch_loop<float, 16>(a, st);
}

extern "C" int ldm_sample_loop_status(const float* ws, int B, int H, unsigned* status_host,
                                      ldm_stream_t s) {
    (void)B;
    const unsigned* st = reinterpret_cast<const unsigned*>(ws + act_floats(H)) + 32 * L_STATUS;
    hipError_t e = hipMemcpyAsync(status_host, st, sizeof(unsigned), hipMemcpyDeviceToHost,
                                  (hipStream_t)s);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)s);
    if (e == hipSuccess && *status_host == 2)
        g_replica_off[cur_dev()].store(true);          // placement: chip-wide loop from now on
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int ldm_sample_loop_config(int form, unsigned spin_limit, int tagged) {
    LDM_REQUIRE(form >= LDM_LOOP_AUTO && form <= LDM_LOOP_FLAT, LDM_EINVAL,
                "sample_loop_config: form %d", form);
    LoopConfig& c = g_cfg[cur_dev()];
    c.form.store(form);
    c.spin_limit.store(spin_limit);
    c.tagged.store(tagged ? 1 : 0);
    return 0;
}

extern "C" int ldm_sample_loop_last_form(void) { return g_last_form[cur_dev()].load(); }

#if SL_STAMP
// diagnostic build only: the replica loop's per-wave phase sums [256][8 waves][8]
extern "C" int ldm_dev_sample_stamps(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(ldm::g_sl_stamp), sizeof(ldm::g_sl_stamp)) ==
                   hipSuccess
               ? 0
               : -1;
}
#endif
