// Quarter-pipelined MFMA decoder (stage layout LDM_LAYOUT_QUARTER): SURVEY.md §8(a) A1+A3.
//
// Same math and operand maps as dec_mfma_kernel (decoder.hip), different work
// order so that the per-chunk epilogue (AGPR read, cvt_pk, ReLU, store) overlaps matrix work:
//   * a layer's output rows are split in quarters of 4 m-chunks (128 features);
//   * one 8 KiB stage = 4 m-chunks x 2 k-steps (frag i = e*4 + c: chunk c, k-step 2j+e);
//   * the accumulators alternate between two 4-chunk sets A/B (2 x 64 AGPRs);
//   * quarter q's epilogue runs inside the first 4 steps of quarter q+1 (one chunk per step,
//     between that step's MFMAs), on the other accumulator set;
//   * quarters 0..nq-2 of a layer park their outputs in a per-wave LDS area (24 KiB/wave) that
//     is reloaded into the B fragments hb[] at the next layer's start; the last quarter writes
//     hb directly (the next layer only reads those k-steps 4+ steps later).
// Layer 0 (aux only) and the final quarter of the tile (layer-7 dot + tanh + store) run
// serialized.  DMA ring: 7 x 8 KiB, barrier every 2 steps, 6 stages ahead.
#include "decoder_common.h"

#include <stdlib.h>

namespace ldm {
namespace {
using namespace dec;

// Timing ablations for diagnostic builds only (scripts/ablate_decoder.sh; results are wrong):
// 1 = no s_barrier/vmcnt wait, 2 = no DMA issue either, 4 = no epilogue (MFMAs then dead-code
// eliminated: invalid), 8 = no A reads, 16 = epilogue reduced to one live element per chunk.
#ifndef QABL
#define QABL 0
#endif

// Diagnostic build only: wave 0 stamps s_memtime around the quarters of its second tile into
// LDS and dumps them over the output at the end (scripts/stamp_decoder.py; results are wrong).
#ifndef QSTAMP
#define QSTAMP 0
#endif

#ifndef QRELOAD_BRANCH
#define QRELOAD_BRANCH 0
#endif

#define QRD(sl, i) ((QABL & 8) ? acur[i] : (sl)[(i) * 64 + c.lane])

constexpr int QRING = 7;
constexpr int QQ = 2;                         // barrier period (steps)
constexpr int QD = 6;                         // stages issued ahead
constexpr int QVM = 2 * (QD - 1 - QQ);        // vmcnt at a barrier
static_assert(QRING >= QD + QQ - 1, "WAR distance");
static_assert(QVM >= 0, "RAW distance");
constexpr int QLDS_RING = QRING * kStageBytes;        // 56 KiB
constexpr int QLDS_TMP = 4 * 24 * 1024;               // 96 KiB (3 quarters x 8 frags x 1 KiB x 4 waves)
constexpr int QLDS_WL = 16 * 2 * 16 * 4;              // 2 KiB
constexpr int QLDS_STAMP = QSTAMP ? 1024 : 0;
constexpr int QLDS_TOTAL = QLDS_RING + QLDS_TMP + QLDS_WL + QLDS_STAMP;
static_assert(QLDS_TOTAL <= 160 * 1024, "LDS");

__host__ __device__ constexpr int q_nq3(int S) { return S / 128; }     // quarters of layer 3
__host__ __device__ constexpr int q_kp4(int S) { return S / 32; }      // pair-stages of layer 4
__host__ __device__ constexpr int q_base4(int S) { return 4 + 68 + 68 + q_nq3(S) * 17; }
__host__ __device__ constexpr int q_len4(int S) { return q_kp4(S) + 1; }
__host__ __device__ constexpr int q_nstages(int S) { return q_base4(S) + 4 * q_len4(S) + 3 * 68; }
__host__ __device__ constexpr int q_nquarters(int S) { return 4 + 4 + q_nq3(S) + 4 + 12; }
static_assert(q_nstages(256) == 414 && q_nstages(512) == 480, "stage plan");

// ------------------------------------------------------------------------------------------
// per-shape aux stages (8 per shape): layer-0 quarters q = 0..3 -> stages 0..3, layer-4
// quarters -> 4..7.  Frag c (0..3), lane l < 32: [wx, wy, wz, wx, wy, wz, beta_hi, beta_lo] of
// feature (4q + c)*32 + l; frags 4..7 and lanes >= 32 are zero.
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void qaux_pack_kernel(const float* __restrict__ beta, const float* __restrict__ wxyz,
                                 int B, T* __restrict__ aux) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;   // (b, stage, frag, lane)
    if (id >= B * 8 * 8 * 64) return;
    const int lane = id & 63;
    const int i = (id >> 6) & 7;
    const int st = (id >> 9) & 7;
    const int b = id >> 12;
    const int layer = st >> 2;
    const int q = st & 3;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (lane < 32 && i < 4) {
        const int f = (4 * q + i) * 32 + lane;
        const float* w = wxyz + ((size_t)layer * kHidden + f) * 3;
        const float bb = beta[((size_t)b * 2 + layer) * kHidden + f];
        const float hi = Elem<T>::round(bb);
        v[0] = w[0]; v[1] = w[1]; v[2] = w[2];
        v[3] = w[0]; v[4] = w[1]; v[5] = w[2];
        v[6] = hi;   v[7] = bb - hi;
    }
    T* o = aux + (size_t)id * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (T)v[e];
}

// ------------------------------------------------------------------------------------------
// DMA pipeline (lean issue path; source pattern changes only around the 8 per-shape stages)
// ------------------------------------------------------------------------------------------
struct QPipe {
    const uint8_t* blob;
    const uint8_t* isrc;        // source of the next stage to issue (wave-uniform)
    const uint8_t* aux_sh;      // per-shape aux stages of the tile being issued (null: past the end)
    const uint8_t* next_aux_sh; // ... of the following tile (set by the consumer at tile start)
    uint32_t islot, ring_beg, ring_end;   // LDS byte address of this wave's piece of that slot
    int is, inext, k4;          // stage being issued, next switch point, layer-4 aux stages done
    int nst, base4, len4;
};

// Slow path, at the 17 per-tile points where the source switches between the blob and the
// shape's aux stages (stages 0..3 and the last stage of each layer-4 quarter) and at the tile
// seam.  Compact on purpose: it is inlined into every step.  Past the last tile every stage
// comes from the blob (dummy copies keep every wave's vmcnt arithmetic exact).
__device__ __forceinline__ void qpipe_boundary(QPipe& p) {
    if (p.is == p.nst) {
        p.is = 0;
        p.k4 = 0;
        p.aux_sh = p.next_aux_sh;
    }
    const int s = p.is;
    const int apos = (p.k4 < 4) ? p.base4 + p.k4 * p.len4 + p.len4 - 1 : p.nst;
    if (p.aux_sh != nullptr && (s < 4 || s == apos)) {
        const int ai = (s < 4) ? s : 4 + p.k4;
        p.k4 += (s < 4) ? 0 : 1;
        p.isrc = p.aux_sh + ai * kStageBytes;
        p.inext = s + 1;
    } else {
        p.isrc = p.blob + s * kStageBytes;
        p.inext = (p.aux_sh != nullptr) ? apos : p.nst;
    }
}

// Fast path: ~12 instructions (2 LDS-DMA pieces, one M0 write, scalar pointer bumps).
__device__ __forceinline__ void qpipe_issue(QPipe& p, uint32_t voff) {
    glds2_saddr(p.isrc, voff, p.islot);
    p.islot = (p.islot + kStageBytes == p.ring_end) ? p.ring_beg : p.islot + kStageBytes;
    p.isrc += kStageBytes;
    if (__builtin_expect(++p.is == p.inext, 0)) qpipe_boundary(p);   // 17 of 414 steps
}

__device__ __forceinline__ void qread_stage(const char* smem, int slot, int lane, u32x4 (&a)[8]) {
    const u32x4* s = reinterpret_cast<const u32x4*>(smem + slot * kStageBytes);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = s[i * 64 + lane];
}

// ------------------------------------------------------------------------------------------
// Per-wave state
// ------------------------------------------------------------------------------------------
struct QCtx {
    QPipe p;
    const char* smem;
    uint32_t coff;       // LDS byte offset of the stage being consumed
    uint32_t voff;       // wave * 2 KiB + lane * 16: this lane's bytes of a stage
    int wave, lane, h;
    u32x4* tmp;          // this wave's parked quarter outputs: [24 frags][64 lanes]
    const float* wl;     // permuted final weights [16 mc][2 h][16]
    float part;          // final-layer partial dot product
    unsigned long long* st;   // QSTAMP: stamp area (LDS)
    bool stamp_on;
};

#define QST(k)                                                                   \
    do {                                                                         \
        if (QSTAMP && c.stamp_on && c.lane == 0) c.st[(k)] = __builtin_readcyclecounter(); \
    } while (0)
// stamp after the MFMAs issued so far have retired (reads the last-written accumulator)
#define QSTS(k, accv)                                                            \
    do {                                                                         \
        if (QSTAMP) {                                                            \
            __builtin_amdgcn_sched_barrier(0);                                   \
            const float _d = (accv)[3][0];                                       \
            asm volatile("; stamp sync %0" ::"v"(_d));                           \
            __builtin_amdgcn_sched_barrier(0);                                   \
            QST(k);                                                              \
            __builtin_amdgcn_sched_barrier(0);                                   \
        }                                                                        \
    } while (0)

// Pending epilogue kinds.  Every converted quarter is parked in the wave's LDS area (slot
// 0..2); the last quarter of a layer reuses slot 0, whose previous contents the next layer
// has already reloaded (see run_quarter), so no B fragment is ever written inside a step.
enum QEpi { QE_NONE = 0, QE_TMP = 1, QE_FIN = 2 };

// Convert chunk c of a finished accumulator set into its parking slot (CVT) or fold it into
// the final-layer dot product (FIN).  Pure VALU/LDS work that fills MFMA issue gaps.
template <typename T, int KIND>
__device__ __forceinline__ void qepi_chunk(QCtx& c, const f32x16& a, int chunk, int slot,
                                           int fin_q) {
    if (QABL & 16) {            // timing ablation: keep the MFMA chains live, no epilogue work
        if (KIND == QE_FIN) c.part += a[0];
        else reinterpret_cast<float*>(c.tmp)[(slot * 8 + 2 * chunk) * 256 + c.lane] = a[0];
        return;
    }
    if (KIND == QE_FIN) {
        const f32x4* w = reinterpret_cast<const f32x4*>(c.wl + ((fin_q * 4 + chunk) * 2 + c.h) * 16);
        float part = c.part;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 wv = w[q];
#pragma unroll
            for (int e = 0; e < 4; ++e) part = fmaf(fmaxf(a[4 * q + e], 0.f), wv[e], part);
        }
        c.part = part;
    } else if (KIND == QE_TMP) {
        u32x4 f0, f1;
        acc_to_frags<T>(a, f0, f1);
        c.tmp[(slot * 8 + 2 * chunk) * 64 + c.lane] = f0;
        c.tmp[(slot * 8 + 2 * chunk + 1) * 64 + c.lane] = f1;
    }
}

// Consumer side of a step: advance to the next ring slot (byte offset, wraps at QRING).
__device__ __forceinline__ const u32x4* qnext_slot(QCtx& c) {
    c.coff = (c.coff + kStageBytes == QRING * kStageBytes) ? 0u : c.coff + kStageBytes;
    return reinterpret_cast<const u32x4*>(c.smem + c.coff);
}

// Barrier + RAW wait, every QQ = 2 steps.  `bar` is a compile-time constant after inlining:
// every quarter has an odd number of steps, so quarter A of a pair starts on an even step and
// quarter B on an odd one (run_quarter's PAR).
__device__ __forceinline__ void qbarrier(bool bar) {
    if (!(QABL & 3) && bar)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(QVM) : "memory");
}

// One pipeline step on a pair-stage: 8 MFMAs (4 chunks x k-steps 2j, 2j+1) into accX, plus
// (KIND != QE_NONE) chunk `ec` of the pending epilogue on accY, interleaved with the last 5.
template <typename T, bool FIRST, int KIND>
__device__ __forceinline__ void qstep(QCtx& c, u32x4 (&acur)[8], const u32x4 b0, const u32x4 b1,
                                      f32x16 (&accX)[4], const f32x16 (&accY)[4], int ec,
                                      int slot, int fin_q, bool bar) {
    const f32x16 zero = {};
    accX[0] = Elem<T>::mfma(acur[0], b0, FIRST ? zero : accX[0]);
    accX[1] = Elem<T>::mfma(acur[1], b0, FIRST ? zero : accX[1]);
    __builtin_amdgcn_sched_barrier(0);
    qbarrier(bar);
    __builtin_amdgcn_sched_barrier(0);
    // rolling fragment buffer: fragment i of the next stage is read right after fragment i of
    // this stage has been consumed (>= 6 MFMAs of latency cover, ~40 live fragment VGPRs)
    const u32x4* sl = qnext_slot(c);
    acur[0] = QRD(sl, 0);
    acur[1] = QRD(sl, 1);
    const u32x4 f2 = acur[2];
    accX[2] = Elem<T>::mfma(f2, b0, FIRST ? zero : accX[2]);
    acur[2] = QRD(sl, 2);
    const u32x4 f3 = acur[3];
    accX[3] = Elem<T>::mfma(f3, b0, FIRST ? zero : accX[3]);
    acur[3] = QRD(sl, 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const u32x4 f = acur[4 + i];
        accX[i] = Elem<T>::mfma(f, b1, accX[i]);
        acur[4 + i] = QRD(sl, 4 + i);
    }
    // LDS-DMA issue after the step's fragment reads: measured in the qstep skeleton
    // (scripts/microbench/qstep_skeleton.hip) 333 vs 363 cycles/step against issuing it
    // between MFMAs 2 and 3.  The barrier still precedes it, so the ring distances hold.
    __builtin_amdgcn_sched_barrier(0);
    if (!(QABL & 2)) qpipe_issue(c.p, c.voff);
    __builtin_amdgcn_sched_barrier(0);
    if (KIND != QE_NONE && !(QABL & 4)) qepi_chunk<T, KIND>(c, accY[ec], ec, slot, fin_q);
}

// The aux step of a quarter: frags 0..3 x bfrag (frags 4..7 of the stage are zero padding).
template <typename T, bool FIRST>
__device__ __forceinline__ void qstep_aux(QCtx& c, u32x4 (&acur)[8], const u32x4 bfrag,
                                          f32x16 (&accX)[4], bool bar) {
    const f32x16 zero = {};
    accX[0] = Elem<T>::mfma(acur[0], bfrag, FIRST ? zero : accX[0]);
    accX[1] = Elem<T>::mfma(acur[1], bfrag, FIRST ? zero : accX[1]);
    __builtin_amdgcn_sched_barrier(0);
    qbarrier(bar);
    __builtin_amdgcn_sched_barrier(0);
    const u32x4* sl = qnext_slot(c);
    acur[0] = QRD(sl, 0);
    acur[1] = QRD(sl, 1);
    const u32x4 f2 = acur[2];
    accX[2] = Elem<T>::mfma(f2, bfrag, FIRST ? zero : accX[2]);
    acur[2] = QRD(sl, 2);
    const u32x4 f3 = acur[3];
    accX[3] = Elem<T>::mfma(f3, bfrag, FIRST ? zero : accX[3]);
#pragma unroll
    for (int i = 3; i < 8; ++i) acur[i] = QRD(sl, i);
    __builtin_amdgcn_sched_barrier(0);
    if (!(QABL & 2)) qpipe_issue(c.p, c.voff);
    __builtin_amdgcn_sched_barrier(0);
}

// k-loop remainder j = 4 .. KP-1 (no epilogue work).  KP == 8 only occurs for layer 4 with a
// 2-quarter layer 3 (K = 256), whose k-steps 8..15 were parked into hb[24..31].
template <typename T, int KP, int PAR>
__device__ __forceinline__ void qkloop_rest(QCtx& c, u32x4 (&acur)[8], u32x4 (&hb)[32],
                                            f32x16 (&accX)[4], const f32x16 (&accY)[4]) {
    constexpr int OFF = (KP == 8) ? 16 : 0;
#pragma unroll
    for (int j = 4; j < KP; ++j)
        qstep<T, false, QE_NONE>(c, acur, hb[OFF + 2 * j], hb[OFF + 2 * j + 1], accX, accY, 0,
                                 0, 0, ((j + PAR) & 1) == 0);
}

struct QPend {
    int kind, slot, fin_q;
};

// Quarter metadata (layers 1..7).  qi is the quarter index over the 26 (28) quarters.
template <int S>
__device__ __forceinline__ void quarter_info(int qi, int& layer, int& q, int& nq) {
    constexpr int n3 = q_nq3(S);
    if (qi < 4) { layer = 1; q = qi; nq = 4; }
    else if (qi < 8) { layer = 2; q = qi - 4; nq = 4; }
    else if (qi < 8 + n3) { layer = 3; q = qi - 8; nq = n3; }
    else { const int r = qi - 8 - n3; layer = 4 + r / 4; q = r & 3; nq = 4; }
}

// One quarter: accumulate into accX (static set), run the pending epilogue of accY inside the
// first 4 steps, then return this quarter's pending epilogue.
template <typename T, int S, int PAR, int KP>
__device__ __forceinline__ void run_quarter(QCtx& c, int qi, u32x4 (&acur)[8], u32x4 (&hb)[32],
                                            const u32x4 bfrag, f32x16 (&accX)[4],
                                            f32x16 (&accY)[4], QPend& pend) {
    int layer, q, nq;
    quarter_info<S>(qi, layer, q, nq);
    // layer boundary: reload the parked quarters 0..2 of the previous layer into hb[0..23]
    // (after a 2-quarter layer 3, slots 1-2 are stale and land in hb[8..23], which layer 4's
    // K = 256 k-loop never reads: it takes k-steps 8..15 from hb[24..31])
    if (q == 0 && layer >= 2) {   // layer 1's reload was done right after layer 0
#pragma unroll
        for (int i = 0; i < 24; ++i) hb[i] = c.tmp[i * 64 + c.lane];
    }
    QSTS(2 + 3 * qi, accY);
    const int kind = pend.kind, slot = pend.slot, fq = pend.fin_q;
    if (kind == QE_TMP) {
        qstep<T, true, QE_TMP>(c, acur, hb[0], hb[1], accX, accY, 0, slot, 0, ((0 + PAR) & 1) == 0);
        qstep<T, false, QE_TMP>(c, acur, hb[2], hb[3], accX, accY, 1, slot, 0, ((1 + PAR) & 1) == 0);
        qstep<T, false, QE_TMP>(c, acur, hb[4], hb[5], accX, accY, 2, slot, 0, ((2 + PAR) & 1) == 0);
        qstep<T, false, QE_TMP>(c, acur, hb[6], hb[7], accX, accY, 3, slot, 0, ((3 + PAR) & 1) == 0);
    } else if (kind == QE_FIN) {
        qstep<T, true, QE_FIN>(c, acur, hb[0], hb[1], accX, accY, 0, 0, fq, ((0 + PAR) & 1) == 0);
        qstep<T, false, QE_FIN>(c, acur, hb[2], hb[3], accX, accY, 1, 0, fq, ((1 + PAR) & 1) == 0);
        qstep<T, false, QE_FIN>(c, acur, hb[4], hb[5], accX, accY, 2, 0, fq, ((2 + PAR) & 1) == 0);
        qstep<T, false, QE_FIN>(c, acur, hb[6], hb[7], accX, accY, 3, 0, fq, ((3 + PAR) & 1) == 0);
    }
    QSTS(3 + 3 * qi, accX);
    // first quarter of a layer: the previous layer's last quarter was just parked in slot 0
    // by the 4 steps above; it always lands in hb[24..31] (k-steps 24..31; a K=256 layer 4
    // reads its k-steps 8..15 from there, see qkloop_rest<8>), first read at pair j >= 4.
    // A predicated select (not a branch) keeps hb's register assignment stable.
#if QRELOAD_BRANCH
    if (q == 0) {         // uniform branch: the other 3 quarters skip the 8 KiB of LDS reads
#pragma unroll
        for (int i = 0; i < 8; ++i) hb[24 + i] = c.tmp[i * 64 + c.lane];
    }
#else
    {
        const bool rl = (q == 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const u32x4 v = c.tmp[i * 64 + c.lane];
            hb[24 + i] = rl ? v : hb[24 + i];
        }
    }
#endif
    qkloop_rest<T, KP, PAR>(c, acur, hb, accX, accY);
    QSTS(4 + 3 * qi, accX);
    qstep_aux<T, false>(c, acur, bfrag, accX, PAR == 0);     // step KP (even)
    // this quarter's epilogue, deferred to the next quarter's first 4 steps
    if (layer == 7) {
        pend.kind = QE_FIN;
        pend.fin_q = q;
    } else {
        pend.kind = QE_TMP;
        pend.slot = (q < nq - 1) ? q : 0;
    }
}

struct QArgs {
    const uint8_t* blob;
    const uint8_t* aux;
    const float* w_last;
    const float* xyz;
    float* out;
    float b_last;
    int npts, tiles_per_shape, n_tiles;
    int N, k0;
    float vs, origin;
};

template <typename T, int S, bool POINTS>
__global__ __launch_bounds__(256, 1) void dec_q_kernel(QArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[QLDS_TOTAL];
    QCtx c;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.voff = (uint32_t)c.wave * 2048u + (uint32_t)c.lane * 16u;
    c.h = c.lane >> 5;
    c.smem = smem;
    c.coff = 0;
    c.tmp = reinterpret_cast<u32x4*>(smem + QLDS_RING + c.wave * 24576);
    float* wl = reinterpret_cast<float*>(smem + QLDS_RING + QLDS_TMP);
    c.wl = wl;
    c.st = reinterpret_cast<unsigned long long*>(smem + QLDS_RING + QLDS_TMP + QLDS_WL);
    c.stamp_on = false;
    for (int i = threadIdx.x; i < 512; i += 256) wl[i] = a.w_last[i];
    __syncthreads();
    if ((int)blockIdx.x >= a.n_tiles) return;

    QPipe& p = c.p;
    p.blob = a.blob;
    p.ring_beg = (uint32_t)(uintptr_t)smem + (uint32_t)c.wave * 2048u;
    p.ring_end = p.ring_beg + QRING * kStageBytes;
    p.islot = p.ring_beg;
    p.nst = q_nstages(S);
    p.base4 = q_base4(S);
    p.len4 = q_len4(S);
    p.aux_sh = a.aux + (size_t)(blockIdx.x / a.tiles_per_shape) * 8 * kStageBytes;
    p.next_aux_sh = nullptr;
    p.is = 0;
    p.k4 = 0;
    qpipe_boundary(p);
#pragma unroll 1
    for (int j = 0; j < QD; ++j) qpipe_issue(p, c.voff);
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * (QD - 1)) : "memory");
    u32x4 acur[8];
    qread_stage(smem, 0, c.lane, acur);

#pragma unroll 1
    for (int tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
        const int shape = tile / a.tiles_per_shape;
        const int local = tile - shape * a.tiles_per_shape;
        {   // the DMA stream crosses into the next tile QD stages before this tile ends
            const int nt = tile + (int)gridDim.x;
            p.next_aux_sh = (nt < a.n_tiles)
                ? a.aux + (size_t)(nt / a.tiles_per_shape) * 8 * kStageBytes : nullptr;
        }
        int pt = local * kTilePoints + c.wave * 32 + (c.lane & 31);
        const bool valid = pt < a.npts;
        if (!valid) pt = a.npts - 1;
        float x, y, z;
        if (POINTS) {
            const float* qq = a.xyz + ((size_t)shape * a.npts + pt) * 3;
            x = qq[0];
            y = qq[1];
            z = qq[2];
        } else {
            grid_point(pt, a.N, a.k0, a.vs, a.origin, x, y, z);
        }
        u32x4 bfrag = {0u, 0u, 0u, 0u};
        {
            const float xh = Elem<T>::round(x), yh = Elem<T>::round(y), zh = Elem<T>::round(z);
            const unsigned w0 = Elem<T>::pack(xh, yh);
            const unsigned w1 = Elem<T>::pack(zh, x - xh);
            const unsigned w2 = Elem<T>::pack(y - yh, z - zh);
            const unsigned w3 = Elem<T>::pack(1.f, 1.f);
            bfrag[0] = c.h ? 0u : w0;
            bfrag[1] = c.h ? 0u : w1;
            bfrag[2] = c.h ? 0u : w2;
            bfrag[3] = c.h ? 0u : w3;
        }
        u32x4 hb[32];
        f32x16 accA[4], accB[4];
        c.part = 0.f;
        c.stamp_on = QSTAMP && c.wave == 0 && tile == (int)blockIdx.x + (int)gridDim.x;
        QST(0);

        // ---- layer 0: four aux-only quarters; 0..2 converted at once into parking slots
        // 0..2, quarter 3 deferred like any layer's last quarter (slot 0, into hb[24..31]).
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            qstep_aux<T, true>(c, acur, bfrag, accA, (q & 1) == 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) qepi_chunk<T, QE_TMP>(c, accA[i], i, q, 0);
        }
        qstep_aux<T, true>(c, acur, bfrag, accB, false);      // step 3
#pragma unroll
        for (int i = 0; i < 24; ++i) hb[i] = c.tmp[i * 64 + c.lane];

        // ---- layers 1..7: quarters alternate A / B; epilogues deferred by one quarter
        QSTS(1, accB);
        QPend pend = {QE_TMP, 0, 0};     // layer 0 quarter 3 (in accB) -> slot 0
        // Pairs of quarters.  K is a compile-time property of each run_quarter instance (a
        // runtime K made the compiler re-home all 64 accumulator AGPRs at the k-loop join).
        // Pairs of quarters.  K is a compile-time property of each run_quarter instance (a
        // runtime K made the compiler re-home all 64 accumulator AGPRs at the k-loop join),
        // and each pair body exists once in the code (the kernel must stay well inside the
        // instruction cache: a 75 KB variant with three pair loops ran 30 % slower).
        constexpr int L4B = 8 + q_nq3(S);              // first layer-4 quarter
        int qi = 0;
#pragma unroll 1
        for (int phase = 0; phase < 2; ++phase) {
            const int qend = (phase == 0 && q_kp4(S) != 16) ? L4B : q_nquarters(S);
#pragma unroll 1
            for (; qi < qend; qi += 2) {               // layers 1..3, then 5..7 (all K = 512)
                run_quarter<T, S, 0, 16>(c, qi, acur, hb, bfrag, accA, accB, pend);
                run_quarter<T, S, 1, 16>(c, qi + 1, acur, hb, bfrag, accB, accA, pend);
            }
            if (q_kp4(S) == 16) break;
#pragma unroll 1
            for (; phase == 0 && qi < L4B + 4; qi += 2) {   // layer 4 (K = 256)
                run_quarter<T, S, 0, q_kp4(S)>(c, qi, acur, hb, bfrag, accA, accB, pend);
                run_quarter<T, S, 1, q_kp4(S)>(c, qi + 1, acur, hb, bfrag, accB, accA, pend);
            }
        }
        // ---- last quarter (layer 7, q = 3, set B): dot product, combine halves, tanh, store
#pragma unroll
        for (int i = 0; i < 4; ++i) qepi_chunk<T, QE_FIN>(c, accB[i], i, 0, 3);
        const float tot = c.part + __shfl_xor(c.part, 32);
        const float sdf = tanhf(tot + a.b_last);
        if (c.h == 0 && valid) a.out[(size_t)shape * a.npts + pt] = sdf;
        QST(2 + 3 * q_nquarters(S));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (QSTAMP && c.wave == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        for (int k = c.lane; k < 96; k += 64)
            reinterpret_cast<unsigned long long*>(a.out)[(size_t)blockIdx.x * 96 + k] = c.st[k];
    }
}

template <typename T, int S>
void launch_q(const QArgs& a, bool points, hipStream_t s, int grid) {
    if (points)
        hipLaunchKernelGGL((dec_q_kernel<T, S, true>), dim3(grid), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((dec_q_kernel<T, S, false>), dim3(grid), dim3(256), 0, s, a);
}

}  // namespace

size_t decoder_q_aux_bytes(int B) { return (size_t)B * 8 * kStageBytes; }

int decoder_q_n_stages(int skip_width) { return q_nstages(skip_width == 253 ? 256 : 512); }

int decoder_q_fwd(const ldm_decoder_t* w, const float* beta, const float* xyz, int B, int npts,
                  int N, int k0, float vs, float origin, float* out, void* ws, size_t ws_bytes,
                  hipStream_t s, int num_cus) {
    const int S = w->skip_width == 253 ? 256 : 512;
    LDM_REQUIRE(w->n_stages == q_nstages(S), LDM_EINVAL, "quarter layout: n_stages %d != %d",
                w->n_stages, q_nstages(S));
    LDM_REQUIRE(ws != nullptr && ws_bytes >= decoder_q_aux_bytes(B) && LDM_ALIGNED(ws, 16),
                LDM_ENOSPC, "workspace too small: need %zu bytes, got %zu",
                decoder_q_aux_bytes(B), ws_bytes);
    {
        const int n = B * 8 * 8 * 64;
        if (w->dtype == LDM_BF16)
            hipLaunchKernelGGL(qaux_pack_kernel<__bf16>, dim3((n + 255) / 256), dim3(256), 0, s,
                               beta, w->wxyz, B, (__bf16*)ws);
        else
            hipLaunchKernelGGL(qaux_pack_kernel<_Float16>, dim3((n + 255) / 256), dim3(256), 0, s,
                               beta, w->wxyz, B, (_Float16*)ws);
        if (int e = launch_status("qaux_pack")) return e;
    }
    QArgs a;
    a.blob = (const uint8_t*)w->weights;
    a.aux = (const uint8_t*)ws;
    a.w_last = w->w_last;
    a.xyz = xyz;
    a.out = out;
    a.b_last = w->b_last;
    a.npts = npts;
    a.tiles_per_shape = (npts + kTilePoints - 1) / kTilePoints;
    a.n_tiles = B * a.tiles_per_shape;
    a.N = N;
    a.k0 = k0;
    a.vs = vs;
    a.origin = origin;
    const int grid = a.n_tiles < num_cus ? a.n_tiles : num_cus;
    const bool points = xyz != nullptr;
    if (w->dtype == LDM_BF16) {
        if (S == 256) launch_q<__bf16, 256>(a, points, s, grid);
        else launch_q<__bf16, 512>(a, points, s, grid);
    } else {
        if (S == 256) launch_q<_Float16, 256>(a, points, s, grid);
        else launch_q<_Float16, 512>(a, points, s, grid);
    }
    return launch_status("ldm_decoder_fwd(quarter)");
}

}  // namespace ldm
