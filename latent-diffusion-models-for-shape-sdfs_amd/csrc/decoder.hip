// DeepSDF decoder on MI355X (gfx950): SURVEY.md §8(a) rows A1 (grid coords), A2 (latent
// fold) and A3 (fused 9-layer MLP), in grid mode and point-list mode.
//
// The reference ships no implementation (/root/reference/README.md:1 is its only line); the
// math follows oracle/ref_cpu.py (decoder_forward_folded, grid_coords_np, latent_fold).
//
// Kernels:
//   dec_mfma_kernel<T,S,POINTS>  bf16/f16 MFMA kernel (the hot path).  DESIGN.md §3-4.
//   dec_f32_kernel<POINTS>       exact-fp32 parity kernel (VALU, correctness first).
//   grid_coords_kernel           A1 on its own (bit-exactness test surface).
//   fold_kernel                  A2 per-shape biases.
//   aux_pack_kernel<T>           per-shape "aux" weight stages (xyz + folded biases).
#include "decoder_common.h"

#include <math.h>
#include <stdlib.h>

namespace ldm {
namespace {
using namespace dec;

__global__ void grid_coords_kernel(int N, int k0, int npts, float vs, float origin,
                                   float* __restrict__ out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npts) return;
    float x, y, z;
    grid_point(p, N, k0, vs, origin, x, y, z);
    out[3 * (size_t)p + 0] = x;
    out[3 * (size_t)p + 1] = y;
    out[3 * (size_t)p + 2] = z;
}

// ------------------------------------------------------------------------------------------
// A2: beta[b][l][f] = sum_k wz[l][f][k] z[b][k] + bz[l][f]   (l = 0: layer 0, 1: layer 4)
// ------------------------------------------------------------------------------------------
__global__ void fold_kernel(const float* __restrict__ wz, const float* __restrict__ bz,
                            const float* __restrict__ z, int B, int L, int H,
                            float* __restrict__ beta) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= B * 2 * H) return;
    const int f = id % H;
    const int l = (id / H) % 2;
    const int b = id / (2 * H);
    const float* w = wz + ((size_t)l * H + f) * L;
    const float* zz = z + (size_t)b * L;
    float acc = 0.f;
    for (int k = 0; k < L; ++k) acc = fmaf(w[k], zz[k], acc);
    beta[id] = acc + bz[l * H + f];
}

// ------------------------------------------------------------------------------------------
// Per-shape aux stages: for layer 0 (stages 0,1) and layer 4 (stages 2,3), fragment i, lane
// l, element e of pass p is  A[row=(8p+i)*32 + (l&31)][k=8*(l>>5)+e]  with columns
// [wx, wy, wz, wx, wy, wz, beta_hi, beta_lo] for lanes 0..31 and zeros for lanes 32..63.
// The matching B fragment is [x_hi, y_hi, z_hi, x_lo, y_lo, z_lo, 1, 1].
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void aux_pack_kernel(const float* __restrict__ beta, const float* __restrict__ wxyz,
                                int B, T* __restrict__ aux) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;  // one (b, stage, frag, lane)
    if (id >= B * 4 * 8 * 64) return;
    const int lane = id & 63;
    const int i = (id >> 6) & 7;
    const int st = (id >> 9) & 3;
    const int b = id >> 11;
    const int layer = st >> 1;  // 0: decoder layer 0, 1: decoder layer 4
    const int pass = st & 1;
    const int f = (pass * 8 + i) * 32 + (lane & 31);
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (lane < 32) {
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
// The fused MFMA decoder.
//
// Workgroup = 4 waves (one per SIMD), tile = 128 points (32 per wave).  Per wave the
// activations of its 32 points live in registers as MFMA B fragments (hb[32]: 512 features x
// 32 points, 16-bit).  Weights stream from L2 through an LDS ring of 8 KiB stages, filled by
// LDS-DMA (global_load_lds_dwordx4) DEPTH stages ahead, one s_barrier per stage; each stage
// feeds 8 v_mfma_f32_32x32x16 per wave.  Biases and xyz enter as one extra "aux" k-step per
// pass.  Persistent grid (one workgroup per CU) walks the tiles; the DMA ring runs across
// tile boundaries without draining.  DESIGN.md §4 has the schedule and its vmcnt accounting.
// ------------------------------------------------------------------------------------------
constexpr int RING = 10;                  // LDS ring slots
constexpr int DEPTH = 8;                  // stages issued ahead (DEPTH <= RING - 2)
#define LDM_VM_STEADY 10                  // 2 * (DEPTH - 3)
#define LDM_VM_PROLOGUE 12                // 2 * (DEPTH - 2)
#define LDM_VM_PAIR 8                     // SCHED 1: 4 * (DEPTH/2 - 2) (pairs P+2..P+3 younger)
#define LDM_VM_PROLOGUE_PAIR 14           // SCHED 1 prologue: 16 issued, stage 0 = oldest 2
static_assert(2 * (DEPTH - 3) == LDM_VM_STEADY, "vmcnt");
static_assert(2 * (DEPTH - 2) == LDM_VM_PROLOGUE, "vmcnt");
static_assert(4 * (DEPTH / 2 - 2) == LDM_VM_PAIR && DEPTH % 2 == 0 && RING % 2 == 0, "pairs");
static_assert(DEPTH / 2 <= RING / 2 - 1, "pair WAR distance");
static_assert(2 * DEPTH - 2 == LDM_VM_PROLOGUE_PAIR, "vmcnt");
constexpr int LDS_RING = RING * kStageBytes;
constexpr int LDS_TMP = 4 * 16 * 1024;    // per-wave spill of a layer's first-pass output
constexpr int LDS_WL = 16 * 2 * 16 * 4;   // final-layer weights (permuted)
constexpr int LDS_TOTAL = LDS_RING + LDS_TMP + LDS_WL;
static_assert(LDS_TOTAL <= 160 * 1024, "LDS");

enum PassMode { M_LO = 0, M_HI = 1, M_TMP = 2, M_MERGE = 3, M_FIN0 = 4, M_FIN1 = 5 };

// Pass table: k-steps (0/16/32) and epilogue mode per pass, 4 bits each.
template <int S>
struct Passes;
template <>
struct Passes<256> {
    static constexpr int NP = 15;
    // L0p0 L0p1 | L1 | L2 | L3 | L4 | L5 | L6 | L7
    static __device__ __forceinline__ int ks(int p) {
        return (p < 2) ? 0 : (p == 7 || p == 8) ? 16 : 32;
    }
    static __device__ __forceinline__ int mode(int p) {
        if (p == 0) return M_LO;
        if (p == 1) return M_HI;
        if (p == 6) return M_LO;   // layer 3: one pass, 256 outputs -> hb[0..15]
        if (p == 13) return M_FIN0;
        if (p == 14) return M_FIN1;
        if (p < 6) return (p & 1) ? M_MERGE : M_TMP;   // 2,3 4,5
        return (p & 1) ? M_TMP : M_MERGE;               // 7,8 9,10 11,12
    }
};
template <>
struct Passes<512> {
    static constexpr int NP = 16;
    static __device__ __forceinline__ int ks(int p) { return (p < 2) ? 0 : 32; }
    static __device__ __forceinline__ int mode(int p) {
        if (p == 0) return M_LO;
        if (p == 1) return M_HI;
        if (p == 14) return M_FIN0;
        if (p == 15) return M_FIN1;
        return (p & 1) ? M_MERGE : M_TMP;
    }
};

struct DecArgs {
    const uint8_t* blob;   // [n_stages][8 KiB]
    const uint8_t* aux;    // [B][4][8 KiB]
    const float* w_last;   // [16][2][16] permuted
    const float* xyz;      // points mode [B][npts][3]
    float* out;            // [B][npts]
    float b_last;
    int npts, tiles_per_shape, n_tiles;
    int N, k0;
    float vs, origin;
};

// DMA pipeline state (wave-uniform; lives in SGPRs).
struct Pipe {
    const uint8_t* blob;
    const uint8_t* aux;
    int g;          // stage being computed (WG-local sequence number; parity drives SCHED 1)
    int islot;      // ring slot of the next issue
    int cslot;      // ring slot of the stage whose fragments are being read next
    int is;         // stage-within-tile of the next issue
    int itile;      // tile of the next issue
    int ishape;     // shape of itile
    int nst, aux4a, aux4b, n_tiles, tps, tstride;
    const uint8_t* isrc;   // SCHED 3: source of the next issue
    int inext;             // SCHED 3: next stage index where the source pattern changes
};

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_dst)
        : "memory");
}

// Issue this wave's share (2 x 1 KiB) of the next stage, then advance the issue cursor.
// Past the last tile a dummy copy of stage 0 keeps every wave's vmcnt arithmetic uniform.
__device__ __forceinline__ void pipe_issue(Pipe& p, uint32_t ring_lds, int wave, int lane) {
    const uint8_t* src = p.blob;
    if (p.itile < p.n_tiles) {
        const int s = p.is;
        const bool sp = (s < 2) | (s == p.aux4a) | (s == p.aux4b);
        const int ai = (s < 2) ? s : (s == p.aux4a ? 2 : 3);
        src = sp ? p.aux + ((size_t)p.ishape * 4 + ai) * kStageBytes
                 : p.blob + (size_t)s * kStageBytes;
    }
    const uint32_t dst = ring_lds + (uint32_t)p.islot * kStageBytes + (uint32_t)wave * 2048u;
    const uint8_t* g = src + wave * 2048 + lane * 16;
    glds16(g, dst);
    glds16(g + 1024, dst + 1024u);
    p.islot = (p.islot + 1 == RING) ? 0 : p.islot + 1;
    if (++p.is == p.nst) {
        p.is = 0;
        p.itile += p.tstride;
        p.ishape = p.itile / p.tps;
    }
}

// SCHED 3 issue path: the common case is "next 8 KiB of the blob"; the source pattern only
// changes at 8 boundaries per tile (per-shape aux stages 0,1,aux4a,aux4b; their successors;
// the tile wrap), handled by pipe_boundary().
__device__ __forceinline__ void pipe_boundary(Pipe& p) {
    if (p.is == p.nst) {
        p.is = 0;
        p.itile += p.tstride;
        p.ishape = p.itile / p.tps;
    }
    const int s = p.is;
    const int ai = (s < 2) ? s : (s == p.aux4a ? 2 : (s == p.aux4b ? 3 : -1));
    p.isrc = (ai >= 0) ? p.aux + ((size_t)p.ishape * 4 + ai) * kStageBytes
                       : p.blob + (size_t)s * kStageBytes;
    p.inext = (s < 2) ? s + 1
            : (s < p.aux4a) ? p.aux4a
            : (s == p.aux4a) ? p.aux4a + 1
            : (s < p.aux4b) ? p.aux4b
            : (s == p.aux4b) ? p.aux4b + 1 : p.nst;
}


__device__ __forceinline__ void pipe_issue_lean(Pipe& p, uint32_t ring_lds, int wave, int lane) {
    const uint8_t* src = (p.itile < p.n_tiles) ? p.isrc : p.blob;   // dummy past the end
    glds16x2(src + wave * 2048 + lane * 16,
             ring_lds + (uint32_t)p.islot * kStageBytes + (uint32_t)wave * 2048u);
    p.islot = (p.islot + 1 == RING) ? 0 : p.islot + 1;
    p.isrc += kStageBytes;
    if (++p.is == p.inext) pipe_boundary(p);
}

__device__ __forceinline__ void read_stage(const char* smem, int slot, int lane, u32x4 (&a)[8]) {
    const u32x4* s = reinterpret_cast<const u32x4*>(smem + slot * kStageBytes);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = s[i * 64 + lane];
}

// Lean schedules: barrier period Q, prefetch depth D (stages issued ahead).
// WAR: the slot refilled at step g held stage g+D-RING, read at step g+D-RING-1; the last
// barrier (>= g-Q+1) must follow it  =>  RING >= D + Q - 1.
// RAW: the barrier at step b certifies stages <= b+Q; stages b+Q+1..b+D-1 may still be in
// flight  =>  vmcnt(2*(D-1-Q)) (2 DMAs per wave per stage); flight time D-Q steps.
template <int SCHED> struct SchedCfg { static constexpr int Q = 2, D = 8, VM_STEADY = 2 * (D - 1 - Q); };
template <> struct SchedCfg<4> { static constexpr int Q = 4, D = 7, VM_STEADY = 2 * (D - 1 - Q); };
static_assert(RING >= SchedCfg<3>::D + SchedCfg<3>::Q - 1, "WAR distance");   // Q=2, D=8
static_assert(RING >= SchedCfg<4>::D + SchedCfg<4>::Q - 1, "WAR distance");

// One pipeline step: certify the next stage(s) (vmcnt + barrier), refill the ring, prefetch
// the next stage's fragments and run this stage's 8 MFMAs.
//   SCHED 0: one barrier + one stage of DMA per step.
//   SCHED 1: one barrier + two stages of DMA every EVEN step (pair P = stages 2P, 2P+1; the
//            barrier of step 2P certifies pair P+1), and the step's first MFMA is issued
//            before the barrier so the barrier wait overlaps matrix work.  DESIGN.md §4.
template <typename T, bool FIRST, int SCHED>
__device__ __forceinline__ void step(Pipe& p, const char* smem, uint32_t ring_lds, int wave,
                                     int lane, u32x4 (&acur)[8], const u32x4 bfrag,
                                     f32x16 (&acc)[8]) {
    const f32x16 zero = {};
    if (SCHED == 0) {
        asm volatile("s_waitcnt vmcnt(" LDM_STR(LDM_VM_STEADY) ")\n\ts_barrier" ::: "memory");
        pipe_issue(p, ring_lds, wave, lane);
        p.cslot = (p.cslot + 1 == RING) ? 0 : p.cslot + 1;
        u32x4 an[8];
        read_stage(smem, p.cslot, lane, an);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = Elem<T>::mfma(acur[i], bfrag, FIRST ? zero : acc[i]);
#pragma unroll
        for (int i = 0; i < 8; ++i) acur[i] = an[i];
    } else if (SCHED == 2) {
        // explicit register double buffer: next stage's 8 fragment reads are issued before
        // this stage's MFMAs (which only touch acur), so LDS latency hides under matrix work.
        acc[0] = Elem<T>::mfma(acur[0], bfrag, FIRST ? zero : acc[0]);
        acc[1] = Elem<T>::mfma(acur[1], bfrag, FIRST ? zero : acc[1]);
        __builtin_amdgcn_sched_barrier(0);
        if ((p.g & 1) == 0)
            asm volatile("s_waitcnt vmcnt(" LDM_STR(LDM_VM_PAIR) ")\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        p.cslot = (p.cslot + 1 == RING) ? 0 : p.cslot + 1;
        u32x4 an[8];
        read_stage(smem, p.cslot, lane, an);
        __builtin_amdgcn_sched_barrier(0);
        if ((p.g & 1) == 0) {
            pipe_issue(p, ring_lds, wave, lane);
            pipe_issue(p, ring_lds, wave, lane);
        }
        p.g++;
#pragma unroll
        for (int i = 2; i < 8; ++i) acc[i] = Elem<T>::mfma(acur[i], bfrag, FIRST ? zero : acc[i]);
#pragma unroll
        for (int i = 0; i < 8; ++i) acur[i] = an[i];
    } else {
        // SCHED 3/4: barrier every Q steps certifying the stages read until the next one,
        // one lean DMA stage per step (stage g+D into the slot of stage g+D-RING), fragment
        // double buffer, scalar issue work pinned between MFMAs (it fills their issue gaps).
        constexpr int Q = SchedCfg<SCHED>::Q;
        constexpr int VM = SchedCfg<SCHED>::VM_STEADY;
        acc[0] = Elem<T>::mfma(acur[0], bfrag, FIRST ? zero : acc[0]);
        acc[1] = Elem<T>::mfma(acur[1], bfrag, FIRST ? zero : acc[1]);
        __builtin_amdgcn_sched_barrier(0);
        if ((p.g & (Q - 1)) == 0)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(VM) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        p.cslot = (p.cslot + 1 == RING) ? 0 : p.cslot + 1;
        u32x4 an[8];
        read_stage(smem, p.cslot, lane, an);
        __builtin_amdgcn_sched_barrier(0);
        acc[2] = Elem<T>::mfma(acur[2], bfrag, FIRST ? zero : acc[2]);
        __builtin_amdgcn_sched_barrier(0);
        pipe_issue_lean(p, ring_lds, wave, lane);
        p.g++;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 3; i < 8; ++i) acc[i] = Elem<T>::mfma(acur[i], bfrag, FIRST ? zero : acc[i]);
#pragma unroll
        for (int i = 0; i < 8; ++i) acur[i] = an[i];
    }
}

template <typename T, int KS, int SCHED>
__device__ __forceinline__ void kloop(Pipe& p, const char* smem, uint32_t ring_lds, int wave,
                                      int lane, u32x4 (&acur)[8], const u32x4 (&hb)[32],
                                      f32x16 (&acc)[8]) {
    step<T, true, SCHED>(p, smem, ring_lds, wave, lane, acur, hb[0], acc);
#pragma unroll
    for (int ks = 1; ks < KS; ++ks)
        step<T, false, SCHED>(p, smem, ring_lds, wave, lane, acur, hb[ks], acc);
}



template <typename T, int S, bool POINTS, int SCHED>
__global__ __launch_bounds__(256, 1) void dec_mfma_kernel(DecArgs a, int nst, int aux4a,
                                                          int aux4b) {
    __shared__ __attribute__((aligned(16))) char smem[LDS_TOTAL];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const uint32_t ring_lds = (uint32_t)(uintptr_t)smem;
    float* wl = reinterpret_cast<float*>(smem + LDS_RING + LDS_TMP);
    u32x4* tmp = reinterpret_cast<u32x4*>(smem + LDS_RING + wave * 16384);

    for (int i = threadIdx.x; i < 512; i += 256) wl[i] = a.w_last[i];
    __syncthreads();
    if ((int)blockIdx.x >= a.n_tiles) return;

    Pipe p;
    p.blob = a.blob;
    p.aux = a.aux;
    p.g = 0;
    p.islot = 0;
    p.cslot = 0;
    p.is = 0;
    p.itile = blockIdx.x;
    p.ishape = p.itile / a.tiles_per_shape;
    p.nst = nst;
    p.aux4a = aux4a;
    p.aux4b = aux4b;
    p.n_tiles = a.n_tiles;
    p.tps = a.tiles_per_shape;
    p.tstride = gridDim.x;

    // prologue: SCHED 0 prefetches DEPTH-1 stages, SCHED 1 DEPTH/2 whole pairs; both then
    // wait for stage 0 (2 x DEPTH-2 younger DMAs resp. 4 x (DEPTH/2-1) = the same 12).
    p.is = 0;
    p.inext = 0;
    p.isrc = p.blob;
    if (SCHED >= 3) {
        constexpr int D = SchedCfg<SCHED >= 3 ? SCHED : 3>::D;
        pipe_boundary(p);
#pragma unroll 1
        for (int j = 0; j < D; ++j) pipe_issue_lean(p, ring_lds, wave, lane);
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * (D - 1)) : "memory");
    } else {
#pragma unroll 1
        for (int j = 0; j < (SCHED ? DEPTH : DEPTH - 1); ++j) pipe_issue(p, ring_lds, wave, lane);
        if (SCHED)
            asm volatile("s_waitcnt vmcnt(" LDM_STR(LDM_VM_PROLOGUE_PAIR) ")\n\ts_barrier" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(" LDM_STR(LDM_VM_PROLOGUE) ")\n\ts_barrier" ::: "memory");
    }
    u32x4 acur[8];
    read_stage(smem, 0, lane, acur);

#pragma unroll 1
    for (int tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
        const int shape = tile / a.tiles_per_shape;
        const int local = tile - shape * a.tiles_per_shape;
        int pt = local * kTilePoints + wave * 32 + (lane & 31);
        const bool valid = pt < a.npts;
        if (!valid) pt = a.npts - 1;
        float x, y, z;
        if (POINTS) {
            const float* q = a.xyz + ((size_t)shape * a.npts + pt) * 3;
            x = q[0];
            y = q[1];
            z = q[2];
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
            bfrag[0] = h ? 0u : w0;
            bfrag[1] = h ? 0u : w1;
            bfrag[2] = h ? 0u : w2;
            bfrag[3] = h ? 0u : w3;
        }

        u32x4 hb[32];   // every k-step is written by an epilogue before a k-loop reads it
        f32x16 acc[8];
        float part = 0.f;

#pragma unroll 1
        for (int pi = 0; pi < Passes<S>::NP; ++pi) {
            const int ks = Passes<S>::ks(pi);
            if (ks == 32) {
                kloop<T, 32, SCHED>(p, smem, ring_lds, wave, lane, acur, hb, acc);
                step<T, false, SCHED>(p, smem, ring_lds, wave, lane, acur, bfrag, acc);
            } else if (ks == 16) {
                kloop<T, 16, SCHED>(p, smem, ring_lds, wave, lane, acur, hb, acc);
                step<T, false, SCHED>(p, smem, ring_lds, wave, lane, acur, bfrag, acc);
            } else {
                step<T, true, SCHED>(p, smem, ring_lds, wave, lane, acur, bfrag, acc);
            }
            const int mode = Passes<S>::mode(pi);
            if (mode == M_LO) {
#pragma unroll
                for (int i = 0; i < 8; ++i) acc_to_frags<T>(acc[i], hb[2 * i], hb[2 * i + 1]);
            } else if (mode == M_HI) {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc_to_frags<T>(acc[i], hb[16 + 2 * i], hb[16 + 2 * i + 1]);
            } else if (mode == M_TMP) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    u32x4 f0, f1;
                    acc_to_frags<T>(acc[i], f0, f1);
                    tmp[(2 * i) * 64 + lane] = f0;
                    tmp[(2 * i + 1) * 64 + lane] = f1;
                }
            } else if (mode == M_MERGE) {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    acc_to_frags<T>(acc[i], hb[16 + 2 * i], hb[16 + 2 * i + 1]);
#pragma unroll
                for (int i = 0; i < 16; ++i) hb[i] = tmp[i * 64 + lane];
            } else {
                // final 512 -> 1 layer fused as an fp32 dot product of ReLU(h7).
                const int pass = (mode == M_FIN0) ? 0 : 1;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const f32x4* w = reinterpret_cast<const f32x4*>(wl + ((pass * 8 + i) * 2 + h) * 16);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const f32x4 wv = w[q];
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            part = fmaf(fmaxf(acc[i][4 * q + e], 0.f), wv[e], part);
                    }
                }
                if (mode == M_FIN1) {
                    const float tot = part + __shfl_xor(part, 32);
                    const float sdf = tanhf(tot + a.b_last);
                    if (h == 0 && valid) a.out[(size_t)shape * a.npts + pt] = sdf;
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------------
// fp32 parity kernel: 32 points per workgroup, activations in LDS [512][32], weights W^T
// streamed from L2 with coalesced loads, 8x8 register tile per thread, fmaf accumulation.
// Blob layout: for l = 1..7: WT_l [K_l][M_l] then b_l [M_l].
// ------------------------------------------------------------------------------------------
struct F32Args {
    const float* blob;
    const float* wxyz;     // [2][512][3]
    const float* beta;     // [B][2][512]
    const float* w_last;   // [512] natural order
    const float* xyz;      // points mode
    float* out;
    float b_last;
    int npts, tiles_per_shape, N, k0, sw;
    float vs, origin;
};

__global__ __launch_bounds__(256) void dec_f32_kernel_impl(F32Args a, int points) {
    __shared__ float hs[512 * 32];
    __shared__ float pxyz[32 * 3];
    const int t = threadIdx.x;
    const int shape = blockIdx.x / a.tiles_per_shape;
    const int local = blockIdx.x - shape * a.tiles_per_shape;
    const int p0 = local * 32;
    if (t < 32) {
        int pt = p0 + t;
        if (pt >= a.npts) pt = a.npts - 1;
        float x, y, z;
        if (points) {
            const float* q = a.xyz + ((size_t)shape * a.npts + pt) * 3;
            x = q[0]; y = q[1]; z = q[2];
        } else {
            grid_point(pt, a.N, a.k0, a.vs, a.origin, x, y, z);
        }
        pxyz[t * 3 + 0] = x;
        pxyz[t * 3 + 1] = y;
        pxyz[t * 3 + 2] = z;
    }
    __syncthreads();
    const float* beta0 = a.beta + (size_t)shape * 2 * 512;
    const float* beta4 = beta0 + 512;
    // layer 0: h = relu(Wxyz0 xyz + beta0)
    for (int e = t; e < 512 * 32; e += 256) {
        const int f = e >> 5, pp = e & 31;
        const float* w = a.wxyz + f * 3;
        float v = beta0[f];
        v = fmaf(w[0], pxyz[pp * 3 + 0], v);
        v = fmaf(w[1], pxyz[pp * 3 + 1], v);
        v = fmaf(w[2], pxyz[pp * 3 + 2], v);
        hs[e] = fmaxf(v, 0.f);
    }
    __syncthreads();
    const int tf = t & 63, tp = t >> 6;
    const float* blob = a.blob;
    for (int l = 1; l <= 7; ++l) {
        const int K = (l == 4) ? a.sw : 512;
        const int M = (l == 3) ? a.sw : 512;
        const float* WT = blob;
        const float* bias = blob + (size_t)K * M;
        blob = bias + M;
        float acc[8][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = tf + 64 * i;
            const float bv = (f < M) ? (l == 4 ? beta4[f] : bias[f]) : 0.f;
            float wx = 0.f, wy = 0.f, wzz = 0.f;
            if (l == 4 && f < M) {
                const float* w = a.wxyz + (512 + f) * 3;
                wx = w[0]; wy = w[1]; wzz = w[2];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float v = bv;
                if (l == 4) {
                    const int pp = tp * 8 + j;
                    v = fmaf(wx, pxyz[pp * 3 + 0], v);
                    v = fmaf(wy, pxyz[pp * 3 + 1], v);
                    v = fmaf(wzz, pxyz[pp * 3 + 2], v);
                }
                acc[i][j] = v;
            }
        }
        for (int k = 0; k < K; ++k) {
            float w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int f = tf + 64 * i;
                w[i] = (f < M) ? WT[(size_t)k * M + f] : 0.f;
            }
            const f32x4 h0 = *reinterpret_cast<const f32x4*>(hs + k * 32 + tp * 8);
            const f32x4 h1 = *reinterpret_cast<const f32x4*>(hs + k * 32 + tp * 8 + 4);
            const float hv[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(w[i], hv[j], acc[i][j]);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = tf + 64 * i;
            if (f < M) {
#pragma unroll
                for (int j = 0; j < 8; ++j) hs[f * 32 + tp * 8 + j] = fmaxf(acc[i][j], 0.f);
            }
        }
        __syncthreads();
    }
    if (t < 32) {
        float s = 0.f;
        for (int f = 0; f < 512; ++f) s = fmaf(a.w_last[f], hs[f * 32 + t], s);
        const int pt = p0 + t;
        if (pt < a.npts) a.out[(size_t)shape * a.npts + pt] = tanhf(s + a.b_last);
    }
}

int g_num_cus = 0;
int num_cus() {
    if (g_num_cus == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            n > 0)
            g_num_cus = n;
        else
            g_num_cus = 256;
    }
    return g_num_cus;
}

size_t aux_bytes(int B) { return (size_t)B * 4 * kStageBytes; }

int check_decoder(const ldm_decoder_t* w) {
    LDM_REQUIRE(w != nullptr, LDM_EINVAL, "decoder descriptor is NULL");
    LDM_REQUIRE(w->abi_version == LDM_ABI_VERSION, LDM_EINVAL, "decoder abi_version %d != %d",
                w->abi_version, LDM_ABI_VERSION);
    LDM_REQUIRE(w->hidden == kHidden, LDM_ENOSYS, "GPU decoder supports hidden=512 (got %d)",
                w->hidden);
    LDM_REQUIRE(w->skip_width == 253 || w->skip_width == 512, LDM_ENOSYS,
                "skip_width must be 253 or 512 (got %d)", w->skip_width);
    LDM_REQUIRE(w->dtype == LDM_F32 || w->dtype == LDM_BF16 || w->dtype == LDM_F16, LDM_EINVAL,
                "bad decoder dtype %d", w->dtype);
    LDM_REQUIRE(w->weights && w->wxyz && w->w_last, LDM_EINVAL, "decoder weights are NULL");
    LDM_REQUIRE(LDM_ALIGNED(w->weights, 16) && LDM_ALIGNED(w->w_last, 16), LDM_EALIGN,
                "decoder weights must be 16-byte aligned");
    if (w->dtype != LDM_F32) {
        LDM_REQUIRE(w->layout == LDM_LAYOUT_PASS8 || w->layout == LDM_LAYOUT_QUARTER ||
                        w->layout == LDM_LAYOUT_SPLIT || w->layout == LDM_LAYOUT_SPLIT16,
                    LDM_EINVAL, "bad decoder layout %d", w->layout);
        const int S = w->skip_width == 253 ? 256 : 512;
        const int want = w->layout == LDM_LAYOUT_PASS8     ? dec_n_stages(S)
                         : w->layout == LDM_LAYOUT_QUARTER ? decoder_q_n_stages(w->skip_width)
                         : w->layout == LDM_LAYOUT_SPLIT   ? decoder_fs_n_stages(w->skip_width)
                                                           : decoder_fs16_n_stages(w->skip_width);
        LDM_REQUIRE(w->n_stages == want, LDM_EINVAL, "n_stages %d != %d for skip width %d",
                    w->n_stages, want, w->skip_width);
    }
    return 0;
}

// Schedule variant (development A/B knob; LDM_DECODER_SCHED=0|1, default 1).
int decoder_sched() {
    const int v = dev_knob("LDM_DECODER_SCHED", 4);   // read per launch: same-process A/B
    return (v >= 0 && v <= 4) ? v : 4;
}

template <typename T, int S, int SCHED>
void launch_mfma_s(const DecArgs& a, bool points, hipStream_t s, int grid) {
    const int nst = dec_n_stages(S);
    const int b4 = dec_base4(S);
    const int aux4a = b4 + S / 16;
    const int aux4b = b4 + 2 * (S / 16) + 1;
    if (points)
        hipLaunchKernelGGL((dec_mfma_kernel<T, S, true, SCHED>), dim3(grid), dim3(256), 0, s, a,
                           nst, aux4a, aux4b);
    else
        hipLaunchKernelGGL((dec_mfma_kernel<T, S, false, SCHED>), dim3(grid), dim3(256), 0, s, a,
                           nst, aux4a, aux4b);
}

template <typename T, int S>
void launch_mfma(const DecArgs& a, bool points, hipStream_t s, int grid) {
    switch (decoder_sched()) {
        case 0: launch_mfma_s<T, S, 0>(a, points, s, grid); break;
        case 2: launch_mfma_s<T, S, 2>(a, points, s, grid); break;
        case 4: launch_mfma_s<T, S, 4>(a, points, s, grid); break;
        case 3: launch_mfma_s<T, S, 3>(a, points, s, grid); break;
        default: launch_mfma_s<T, S, 4>(a, points, s, grid); break;
    }
}

int decoder_fwd(const ldm_decoder_t* w, const float* beta, const float* xyz, int B, int npts,
                int N, int k0, float vs, float origin, float* out, void* ws, size_t ws_bytes,
                hipStream_t s) {
    if (int e = check_decoder(w)) return e;
    LDM_REQUIRE(B >= 1 && npts >= 1, LDM_EINVAL, "empty decode (B=%d, npts=%d)", B, npts);
    LDM_REQUIRE((long long)B * npts < (1ll << 31), LDM_EINVAL, "B*npts too large");
    LDM_REQUIRE(beta && out, LDM_EINVAL, "beta/out NULL");
    LDM_REQUIRE(LDM_ALIGNED(beta, 16) && LDM_ALIGNED(out, 4), LDM_EALIGN, "misaligned buffers");
    const bool points = xyz != nullptr;
    if (w->dtype == LDM_F32) {
        F32Args a;
        a.blob = (const float*)w->weights;
        a.wxyz = w->wxyz;
        a.beta = beta;
        a.w_last = w->w_last;
        a.xyz = xyz;
        a.out = out;
        a.b_last = w->b_last;
        a.npts = npts;
        a.tiles_per_shape = (npts + 31) / 32;
        a.N = N;
        a.k0 = k0;
        a.sw = w->skip_width;
        a.vs = vs;
        a.origin = origin;
        hipLaunchKernelGGL(dec_f32_kernel_impl, dim3(B * a.tiles_per_shape), dim3(256), 0, s, a,
                           points ? 1 : 0);
        return launch_status("ldm_decoder_fwd(f32)");
    }
    if (w->layout == LDM_LAYOUT_SPLIT16)
        return decoder_fs16_fwd(w, beta, xyz, B, npts, N, k0, vs, origin, out, ws, ws_bytes, s,
                                num_cus());
    if (w->layout == LDM_LAYOUT_SPLIT)
        return decoder_fs_fwd(w, beta, xyz, B, npts, N, k0, vs, origin, out, ws, ws_bytes, s,
                              num_cus());
    if (w->layout == LDM_LAYOUT_QUARTER)
        return decoder_q_fwd(w, beta, xyz, B, npts, N, k0, vs, origin, out, ws, ws_bytes, s,
                             num_cus());
    LDM_REQUIRE(ws != nullptr && ws_bytes >= aux_bytes(B) && LDM_ALIGNED(ws, 16), LDM_ENOSPC,
                "workspace too small: need %zu bytes, got %zu", aux_bytes(B), ws_bytes);
    // per-shape aux stages (folded biases + xyz columns) into the workspace
    {
        const int n = B * 4 * 8 * 64;
        if (w->dtype == LDM_BF16)
            hipLaunchKernelGGL(aux_pack_kernel<__bf16>, dim3((n + 255) / 256), dim3(256), 0, s,
                               beta, w->wxyz, B, (__bf16*)ws);
        else
            hipLaunchKernelGGL(aux_pack_kernel<_Float16>, dim3((n + 255) / 256), dim3(256), 0, s,
                               beta, w->wxyz, B, (_Float16*)ws);
        if (int e = launch_status("aux_pack")) return e;
    }
    DecArgs a;
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
    const int grid = a.n_tiles < num_cus() ? a.n_tiles : num_cus();
    const int S = w->skip_width == 253 ? 256 : 512;
    if (w->dtype == LDM_BF16) {
        if (S == 256) launch_mfma<__bf16, 256>(a, points, s, grid);
        else launch_mfma<__bf16, 512>(a, points, s, grid);
    } else {
        if (S == 256) launch_mfma<_Float16, 256>(a, points, s, grid);
        else launch_mfma<_Float16, 512>(a, points, s, grid);
    }
    return launch_status("ldm_decoder_fwd(mfma)");
}

}  // namespace

size_t decoder_workspace_bytes(int B, int dtype, int layout) {
    if (dtype == LDM_F32) return 0;
    return layout == LDM_LAYOUT_PASS8    ? aux_bytes(B)
           : layout == LDM_LAYOUT_SPLIT ? decoder_fs_aux_bytes(B)
           : layout == LDM_LAYOUT_SPLIT16 ? decoder_fs16_aux_bytes(B)
                                        : decoder_q_aux_bytes(B);
}

}  // namespace ldm

using namespace ldm;

extern "C" int ldm_grid_coords(int N, int k0, int k1, float vs, float origin, float* xyz_out,
                               ldm_stream_t s) {
    LDM_REQUIRE(N >= 1 && k0 >= 0 && k1 > k0 && k1 <= N, LDM_EINVAL,
                "bad grid slab N=%d [%d,%d)", N, k0, k1);
    LDM_REQUIRE(xyz_out != nullptr && LDM_ALIGNED(xyz_out, 4), LDM_EINVAL, "xyz_out NULL");
    const long long npts = (long long)(k1 - k0) * N * N;
    LDM_REQUIRE(npts < (1ll << 31), LDM_EINVAL, "grid too large");
    hipLaunchKernelGGL(grid_coords_kernel, dim3((unsigned)((npts + 255) / 256)), dim3(256), 0,
                       (hipStream_t)s, N, k0, (int)npts, vs, origin, xyz_out);
    return launch_status("ldm_grid_coords");
}

extern "C" int ldm_decoder_fold(const ldm_decoder_t* w, const float* z, int B, float* beta_out,
                                ldm_stream_t s) {
    LDM_REQUIRE(w && w->abi_version == LDM_ABI_VERSION, LDM_EINVAL, "bad decoder descriptor");
    LDM_REQUIRE(w->wz && w->bz && z && beta_out && B >= 1 && w->latent_dim >= 1, LDM_EINVAL,
                "bad fold arguments");
    const int n = B * 2 * w->hidden;
    hipLaunchKernelGGL(fold_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, w->wz,
                       w->bz, z, B, w->latent_dim, w->hidden, beta_out);
    return launch_status("ldm_decoder_fold");
}

extern "C" int ldm_decoder_grid_fwd(const ldm_decoder_t* w, const float* beta, int B, int N,
                                    int k0, int k1, float vs, float origin, float* out, void* ws,
                                    size_t ws_bytes, ldm_stream_t s) {
    LDM_REQUIRE(N >= 2 && k0 >= 0 && k1 > k0 && k1 <= N, LDM_EINVAL,
                "bad grid slab N=%d [%d,%d)", N, k0, k1);
    const long long npts = (long long)(k1 - k0) * N * N;
    LDM_REQUIRE(npts < (1ll << 31), LDM_EINVAL, "grid slab too large");
    return decoder_fwd(w, beta, nullptr, B, (int)npts, N, k0, vs, origin, out, ws, ws_bytes,
                       (hipStream_t)s);
}

extern "C" int ldm_decoder_points_fwd(const ldm_decoder_t* w, const float* beta, const float* xyz,
                                      int B, int P, float* out, void* ws, size_t ws_bytes,
                                      ldm_stream_t s) {
    LDM_REQUIRE(xyz != nullptr && LDM_ALIGNED(xyz, 4), LDM_EINVAL, "xyz NULL");
    return decoder_fwd(w, beta, xyz, B, P, 0, 0, 0.f, 0.f, out, ws, ws_bytes, (hipStream_t)s);
}
