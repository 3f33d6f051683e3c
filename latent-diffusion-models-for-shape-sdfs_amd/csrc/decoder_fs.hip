// Feature-split MFMA decoder (weight layout LDM_LAYOUT_SPLIT): SURVEY.md §8(a) A1+A3.
//
// Same math and operand maps as the quarter kernel (decoder_q.hip), a
// different split of the work inside a workgroup (DESIGN.md §4 "split kernel"):
//   * a tile is 128 points = 4 point chunks (n) of 32, shared by the workgroup's 4 waves;
//   * wave w owns the OUTPUT FEATURES [128w, 128w+128) of every 512-wide layer as two parts of
//     64 rows (2 m-chunks of 32); the one-part layer 3 of DeepSDF (253 -> 256) gives each wave
//     rows [64w, 64w+64);
//   * the tile's activations live once, in LDS, as B fragments (128 KiB, 32 positions of 4
//     point chunks x 1 KiB); every wave reads every position's 4 B fragments;
//   * each wave streams ITS OWN weight fragments (2 per k-step, 2 KiB) from L2 straight into a
//     register ring (raw buffer loads, FS_D k-steps ahead): no LDS ring, no DMA barrier.
//     Per k-step a wave reads 2 A fragments (L2) + 4 B fragments (LDS) for 8 MFMAs: each
//     fragment feeds 4 (A) or 2 (B) MFMAs, where the quarter kernel read one LDS fragment per
//     MFMA; the weight bytes per point are unchanged (each feeds the tile's 128 points).
//   * a part's accumulators (2 m x 4 n tiles = 128 fp32) alternate between two sets A and B,
//     and a finished set is converted (16-bit + ReLU) straight into LDS inside 8 k-steps of a
//     LATER part, one tile per step, between its MFMAs:
//       - a layer's part 1 (set B) -> the "late" positions 16..31, during the next layer's
//         part 0 steps 0-7; that part meets a barrier at its step 16 before reading them;
//       - a layer's part 0 (set A) -> the "early" positions 0..15, during the SAME layer's
//         part 1 steps 16-23: part 1 reads the early positions in steps 0-15, so after a
//         barrier at its step 16 no wave reads them any more; the next layer's part 0
//         publishes them with a barrier after its aux step;
//       - layer 7's parts fold into the final 512 -> 1 dot product instead (fp32, w_last).
//     No activation is parked in registers and no layer boundary writes LDS serially.
//   * the bias (and, for layers 0 and 4, xyz + the folded latent) enters as one aux MFMA step
//     at the START of each part (A = [wx,wy,wz,wx,wy,wz,b_hi,b_lo], B = [x_hi,y_hi,z_hi,x_lo,
//     y_lo,z_lo,1,1]), which also zero-initialises the accumulators.
// Barriers per tile: 3 per layer (the quarter kernel: one per 2 k-steps, ~207).
#include "decoder_common.h"

namespace ldm {
namespace {
using namespace dec;

// FS_D: k-steps of A fragments in flight per wave (register ring depth), 4 or 8; the product
// uses kFsDefaultD, the other depth is instantiated for A/B runs of the dev build
constexpr int kFsDefaultD = 4;

constexpr int kFsStep = 2048;                       // one wave's A fragments of one k-step
constexpr int kFsAct = 32 * 4 * 1024;               // 128 KiB activation buffer
constexpr int kFsRed = 4 * 4 * 32 * 4;              // final partials [wave][n][32] fp32
constexpr int kFsWl = 512 * 4;                      // permuted final-layer weights
constexpr int kFsXyz = 4 * 4 * 1024;                // per-wave aux B fragments [wave][n][64]
// Diagnostic build only (-DFS_STAMP=1, scripts/stamp_split.py; results are wrong): wave 0 of
// every workgroup stamps s_memtime at part and layer boundaries of its second tile, dumped over
// the output at the end.
#ifndef FS_STAMP
#define FS_STAMP 0
#endif
constexpr int kFsStamp = FS_STAMP ? 128 * 8 : 0;
constexpr int kFsLds = kFsAct + kFsRed + kFsWl + kFsXyz + kFsStamp;
static_assert(kFsLds <= 160 * 1024, "LDS");

__host__ __device__ constexpr int fs_nparts(int S) { return S == 256 ? 15 : 16; }
__host__ __device__ constexpr int fs_nsteps(int S) { return S == 256 ? 384 : 448; }

// ------------------------------------------------------------------------------------------
// per-shape aux fragments: [B][4 waves][4 slots: L0p0, L0p1, L4p0, L4p1][2 frags][64][8].
// Lane < 32 of frag i: [wx, wy, wz, wx, wy, wz, beta_hi, beta_lo] of row 128w + 64p + 32i +
// lane (layers 0 and 4 are 512 wide); lanes >= 32 zero (they meet zero B rows: must be finite).
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void fs_aux_pack_kernel(const float* __restrict__ beta, const float* __restrict__ wxyz,
                                   int B, T* __restrict__ aux) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;   // (b, w, slot, i, lane)
    if (id >= B * 4 * 4 * 2 * 64) return;
    const int lane = id & 63;
    const int i = (id >> 6) & 1;
    const int slot = (id >> 7) & 3;
    const int w = (id >> 9) & 3;
    const int b = id >> 11;
    const int li = slot >> 1;                 // 0: layer 0, 1: layer 4
    const int p = slot & 1;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (lane < 32) {
        const int f = 128 * w + 64 * p + 32 * i + lane;
        const float* wx = wxyz + ((size_t)li * kHidden + f) * 3;
        const float bb = beta[((size_t)b * 2 + li) * kHidden + f];
        const float hi = Elem<T>::round(bb);
        v[0] = wx[0]; v[1] = wx[1]; v[2] = wx[2];
        v[3] = wx[0]; v[4] = wx[1]; v[5] = wx[2];
        v[6] = hi;    v[7] = bb - hi;
    }
    T* o = aux + (size_t)id * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (T)v[e];
}

struct FArgs {
    const uint8_t* stream;   // [4 waves][nsteps][2 KiB] then bias aux [4 waves][nparts][2 KiB]
    const uint8_t* aux;      // workspace [B][4 waves][4 slots][2 KiB]
    const float* w_last;     // [4 w][2 p][2 i][2 h][16] (pack.permute_w_last_split)
    const float* xyz;
    float* out;
    float b_last;
    int npts, tiles_per_shape, n_tiles;
    int N, k0;
    float vs, origin;
};

// Epilogue kinds run inside 8 k-steps of a part (on the OTHER accumulator set)
enum FsEpi { FE_NONE = 0, FE_LATE = 1, FE_EARLY = 2, FE_FIN = 3 };

// A fragment source: a buffer resource (SGPRs) + a byte offset (SGPR); the lane's 16 bytes at
// voffset lane*16 (+1024: the second fragment, an immediate).  Raw buffer loads keep every
// address in scalar registers: plain global loads made the compiler materialise (and hoist,
// then spill) a 64-bit VGPR address per load site.
struct FSrc {
    bool shape;               // per-shape aux (workspace) or the weight blob
    uint32_t off;             // byte offset in that buffer
};

template <int FS_D>
struct FCtx {
    int lane, wave, h;
    uint32_t voff;            // lane * 16
    char* smem;
    __amdgpu_buffer_rsrc_t rw;   // the weight blob: streams then bias aux fragments
    __amdgpu_buffer_rsrc_t ra;   // the per-shape aux workspace
    uint32_t s_beg, s_end;    // this wave's stream [s_beg, s_end) in rw
    uint32_t s_iss;           // next 4-step stream group to issue
    uint32_t baux_w;          // this wave's bias aux fragments [nparts][2 KiB] in rw
    uint32_t aux_w;           // this tile's per-shape aux of this wave [4 slots][2 KiB] in ra
    uint32_t aux_next;        // ... of the next tile
    u32x4 auxn[2];            // aux A fragments of the part about to start
    u32x4 ring[FS_D][2];
    float part[4];
    unsigned long long* st;   // FS_STAMP
    int st_i;
    bool st_on;
};

template <int FS_D>
__device__ __forceinline__ void stamp(FCtx<FS_D>& c) {
    if (FS_STAMP) {
        if (c.st_on && c.lane == 0 && c.st_i < 128) c.st[c.st_i] = __builtin_readcyclecounter();
        ++c.st_i;
    }
}

__device__ __forceinline__ u32x4 bld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

template <int FS_D>
__device__ __forceinline__ void load_aux(FCtx<FS_D>& c, FSrc s) {
    const __amdgpu_buffer_rsrc_t r = s.shape ? c.ra : c.rw;
    c.auxn[0] = bld(r, c.voff, s.off);
    c.auxn[1] = bld(r, c.voff + 1024u, s.off);
}

// A lane's LDS byte address `voff + off` (off wave-uniform) as an OPAQUE VGPR: LDS immediates
// are 16 bits, so positions past 64 KiB need a register base; left to itself the compiler
// materialised one VGPR per (position, chunk) constant, hoisted them out of the tile loop and
// spilled them.  The empty volatile asm is neither folded nor hoisted: one v_add per use site,
// and every per-tile offset below it fits the immediate.
template <int FS_D>
__device__ __forceinline__ char* lds_at(const FCtx<FS_D>& c, uint32_t off) {
    uint32_t v = c.voff + off;
    asm volatile("" : "+v"(v));
    return c.smem + v;
}

// LDS barrier: LDS writes done (lgkmcnt), then s_barrier.  The weight loads in flight
// (vmcnt) are NOT waited for: they feed registers only.
__device__ __forceinline__ void fs_bar() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The activation buffer is kept in CONSUMPTION order: position j (4 KiB: 4 point chunks x
// 1 KiB) holds the k-step that ring step j of the next layer reads (pack.split_kidx): after a
// 512-wide layer, k-step 8w + 4u + 2i + s sits at position 16u + 4w + 2i + s (u = 0: part 0,
// the "early" positions; u = 1: part 1, the "late" ones); after layer 3 at skip 253, k-step
// 4w + 2i + s at position 16 + 4w + 2i + s (layer 4 reads positions 16 + j).  Step j reads
// position pos0 + j: the addresses are immediates from one group base.
template <int FS_D>
__device__ __forceinline__ void read_b(const FCtx<FS_D>& c, int pos, u32x4 (&b)[4]) {
    const u32x4* p = reinterpret_cast<const u32x4*>(lds_at(c, pos * 4096));
#pragma unroll
    for (int n = 0; n < 4; ++n) b[n] = p[n * 64];
}

// Stream step r (0..3) of the 4-step stream group at c.s_iss into ring slot `slot`: the
// (r & 1) * 2 KiB + fragment offset folds into the load's immediate, the (r >> 1) * 4 KiB into
// the scalar offset, so a group costs one wrap test instead of one per step.
template <int FS_D>
__device__ __forceinline__ void issue(FCtx<FS_D>& c, int slot, int r) {
    const uint32_t so = c.s_iss + (uint32_t)(r >> 1) * 2u * kFsStep;
    const uint32_t vo = c.voff + (uint32_t)(r & 1) * kFsStep;
    c.ring[slot][0] = bld(c.rw, vo, so);
    c.ring[slot][1] = bld(c.rw, vo + 1024u, so);
}

template <int FS_D>
__device__ __forceinline__ void next_group(FCtx<FS_D>& c) {
    c.s_iss += 4u * kFsStep;
    if (c.s_iss == c.s_end) c.s_iss = c.s_beg;
}

// one accumulator tile -> its two B fragments at LDS position pos, pos + 1 (point chunk n)
template <typename T, int FS_D>
__device__ __forceinline__ void tile_to_lds(FCtx<FS_D>& c, const f32x16& acc, int pos, int n) {
    u32x4 f0, f1;
    acc_to_frags<T>(acc, f0, f1);
    u32x4* p = reinterpret_cast<u32x4*>(lds_at(c, (pos * 4 + n) * 1024));
    p[0] = f0;
    p[4 * 64] = f1;
}

// One tile t = 4i + n of the other accumulator set's epilogue.
template <typename T, int EK, int FS_D>
__device__ __forceinline__ void epi_tile(FCtx<FS_D>& c, const f32x16 (&accY)[2][4], int t) {
    const int i = t >> 2, n = t & 3;
    if (EK == FE_LATE || EK == FE_EARLY) {   // part 1 of the previous layer / part 0 of this
        u32x4 f0, f1;
        acc_to_frags<T>(accY[i][n], f0, f1);
        u32x4* p = reinterpret_cast<u32x4*>(
            lds_at(c, (uint32_t)((EK == FE_LATE ? 16 : 0) + 4 * c.wave) * 4096u));
        p[(2 * i * 4 + n) * 64] = f0;
        p[((2 * i + 1) * 4 + n) * 64] = f1;
    } else if (EK == FE_FIN) {     // part 0 of layer 7 -> the final dot product
        const f32x4* w = reinterpret_cast<const f32x4*>(
            c.smem + kFsAct + kFsRed + (((c.wave * 2 * 2 + i) * 2 + c.h) * 16) * 4);
        float part = c.part[n];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 wv = w[q];
#pragma unroll
            for (int e = 0; e < 4; ++e) part = fmaf(fmaxf(accY[i][n][4 * q + e], 0.f), wv[e], part);
        }
        c.part[n] = part;
    }
}

// Four k-steps reading positions p0..p0+3 (ring slots RO..RO+3).  E work: tiles T0..T0+3 of the
// other set (EK != FE_NONE).  The next position's B fragments are read unconditionally (no
// selects in the loop): at a barrier and at a part's end that read is stale or unused and the
// caller reads again (position 32 is still inside the LDS allocation).
template <typename T, int EK, int T0, int RO, int FS_D>
__device__ __forceinline__ void group4(FCtx<FS_D>& c, f32x16 (&acc)[2][4], const f32x16 (&accY)[2][4],
                                       u32x4 (&b)[4], int p0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        // rolling B fragments: chunk n of step j+1 is read as soon as step j's two MFMAs on
        // chunk n are issued, ~6 MFMAs (~190 cycles) before it is needed (a read after the
        // step's last MFMA left ~32 cycles of cover: an LDS round trip exposed per step)
        const u32x4* nb = reinterpret_cast<const u32x4*>(lds_at(c, (p0 + r + 1) * 4096));
        const u32x4 a0 = c.ring[RO + r][0], a1 = c.ring[RO + r][1];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            acc[0][n] = Elem<T>::mfma(a0, b[n], acc[0][n]);
            acc[1][n] = Elem<T>::mfma(a1, b[n], acc[1][n]);
            b[n] = nb[n * 64];
        }
        issue(c, RO + r, r);
        if (EK != FE_NONE) epi_tile<T, EK>(c, accY, T0 + r);
        // pin the step's order for the scheduler (left free it sank the B reads and weight
        // loads below the last MFMA: one step of latency cover instead of FS_D): per point
        // chunk n, MFMA, [VALU], MFMA, B read, [VALU]; then the 2 weight loads.  E steps
        // spread their VALU (AGPR reads, cvt, ReLU) 4 per MFMA gap (the guide: <= 5 fillers
        // per 32x32x16 gap hide).
        constexpr int V = EK == FE_NONE ? 0 : 4;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (V) __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            if (V) __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    next_group(c);
}

// 8 k-steps from position p0 (ring slots 0..7 mod FS_D); E work (tiles 0..7) when EK != NONE
template <typename T, int EK, int FS_D>
__device__ __forceinline__ void steps8(FCtx<FS_D>& c, f32x16 (&acc)[2][4], const f32x16 (&accY)[2][4],
                                       u32x4 (&b)[4], int p0) {
    group4<T, EK, 0, 0, FS_D>(c, acc, accY, b, p0);
    group4<T, EK, 4, (FS_D == 8 ? 4 : 0), FS_D>(c, acc, accY, b, p0 + 4);
}

// One part: the aux step (zero-initialises acc; loads the NEXT part's aux fragments), then nk
// ring steps reading positions pos0 + j.  E work (the other set, EK) in steps 0-7 (E16 false)
// or 16-23 (E16 true).  `mid`: a barrier before step 16 (the late positions were written
// during steps 0-7 by every wave / no wave reads the early positions any more).  `bar0`: the
// part follows LDS writes of the previous layer still to be published: the barrier comes after
// its aux step (which reads only the wave's own xyz fragments).
template <typename T, int EK, bool E16, int FS_D>
__device__ __forceinline__ void run_part(FCtx<FS_D>& c, f32x16 (&acc)[2][4], const f32x16 (&accY)[2][4],
                                         int nk, bool mid, FSrc naux, int pos0, bool bar0) {
    const f32x16 zero = {};
    u32x4 b[4];
    // the aux B fragments (xyz of the tile's points) sit in this wave's LDS copy
    const u32x4* xb = reinterpret_cast<const u32x4*>(
        lds_at(c, kFsAct + kFsRed + kFsWl + c.wave * 4096));
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const u32x4 x = xb[n * 64];
        acc[0][n] = Elem<T>::mfma(c.auxn[0], x, zero);
        acc[1][n] = Elem<T>::mfma(c.auxn[1], x, zero);
    }
    load_aux(c, naux);
    if (bar0) fs_bar();
    stamp(c);
    if (nk == 0) return;
    read_b(c, pos0, b);
    // code size: the E steps are unrolled per kind, the plain steps run as ONE runtime loop of
    // 4-step groups (the kernel must stay well inside the instruction cache)
    int j = 0;
    if (!E16) {
        steps8<T, EK, FS_D>(c, acc, accY, b, pos0);
        j = 8;
    }
    stamp(c);
#pragma unroll 1
    for (; j < nk; j += FS_D) {
        if (j == 16) {
            if (E16) break;
            if (mid) {
                stamp(c);
                fs_bar();
                read_b(c, pos0 + 16, b);
            }
        }
        group4<T, FE_NONE, 0, 0, FS_D>(c, acc, accY, b, pos0 + j);
        if (FS_D == 8) group4<T, FE_NONE, 0, 4, FS_D>(c, acc, accY, b, pos0 + j + 4);
    }
    if (E16) {               // j == 16 here (E16 parts have nk = 32 and a mid barrier)
        stamp(c);
        fs_bar();
        read_b(c, pos0 + 16, b);
        steps8<T, EK, FS_D>(c, acc, accY, b, pos0 + 16);
        stamp(c);
#pragma unroll 1
        for (j = 24; j < nk; j += FS_D) {
            group4<T, FE_NONE, 0, 0, FS_D>(c, acc, accY, b, pos0 + j);
            if (FS_D == 8) group4<T, FE_NONE, 0, 4, FS_D>(c, acc, accY, b, pos0 + j + 4);
        }
    }
    stamp(c);
}

// a whole set into LDS positions kbase + 2i + s (serial: layer 0, layer 3 at skip 253)
template <typename T, int FS_D>
__device__ __forceinline__ void acc_to_lds(FCtx<FS_D>& c, const f32x16 (&acc)[2][4], int kbase) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int n = 0; n < 4; ++n) tile_to_lds<T>(c, acc[i][n], kbase + 2 * i, n);
}

// final layer of part 1 of layer 7 (after its MFMAs): w read once per m-chunk, shared by the 4
// point chunks; four independent fma chains per tile, summed in fixed order
template <int FS_D>
__device__ __forceinline__ void fin_serial(FCtx<FS_D>& c, const f32x16 (&acc)[2][4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const f32x4* wp = reinterpret_cast<const f32x4*>(
            c.smem + kFsAct + kFsRed + ((((c.wave * 2 + 1) * 2 + i) * 2 + c.h) * 16) * 4);
        f32x4 w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = wp[q];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            float s[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                s[q] = fmaxf(acc[i][n][4 * q], 0.f) * w[q][0];
#pragma unroll
                for (int e = 1; e < 4; ++e) s[q] = fmaf(fmaxf(acc[i][n][4 * q + e], 0.f), w[q][e], s[q]);
            }
            c.part[n] += (s[0] + s[1]) + (s[2] + s[3]);
        }
    }
}

template <typename T, int S, bool POINTS, int FS_D>
__global__ __launch_bounds__(256, 1) void dec_fs_kernel(FArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[kFsLds];
    FCtx<FS_D> c;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.h = c.lane >> 5;
    c.voff = (uint32_t)c.lane * 16u;
    c.smem = smem;
    c.st = reinterpret_cast<unsigned long long*>(smem + kFsAct + kFsRed + kFsWl + kFsXyz);
    c.st_i = 0;
    c.st_on = false;
    float* wl = reinterpret_cast<float*>(smem + kFsAct + kFsRed);
    float* red = reinterpret_cast<float*>(smem + kFsAct);
    u32x4* xyz_l = reinterpret_cast<u32x4*>(smem + kFsAct + kFsRed + kFsWl + c.wave * 4096 +
                                            c.voff);
    for (int i = threadIdx.x; i < 512; i += 256) wl[i] = a.w_last[i];
    __syncthreads();
    if ((int)blockIdx.x >= a.n_tiles) return;

    constexpr int NST = fs_nsteps(S);
    constexpr int NP = fs_nparts(S);
    constexpr uint32_t kFlags = 0x00020000u;     // raw dword buffer (gfx9 word 3)
    c.rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.stream, (short)0, 0x7ffffff0, kFlags);
    c.ra = __builtin_amdgcn_make_buffer_rsrc((void*)a.aux, (short)0, 0x7ffffff0, kFlags);
    c.s_beg = (uint32_t)c.wave * NST * kFsStep;
    c.s_end = c.s_beg + NST * kFsStep;
    c.s_iss = c.s_beg;
    c.baux_w = (uint32_t)(4 * NST + c.wave * NP) * kFsStep;
    auto shape_aux = [&](int tile) -> uint32_t {
        return ((uint32_t)(tile / a.tiles_per_shape) * 4u + (uint32_t)c.wave) * 4u * kFsStep;
    };
    auto bias = [&](int pi) -> FSrc { return FSrc{false, c.baux_w + (uint32_t)pi * kFsStep}; };
    auto shp = [&](int slot) -> FSrc { return FSrc{true, c.aux_w + (uint32_t)slot * kFsStep}; };
    c.aux_w = shape_aux(blockIdx.x);
#pragma unroll
    for (int r = 0; r < FS_D; ++r) {
        issue(c, r, r & 3);
        if ((r & 3) == 3) next_group(c);
    }
    load_aux(c, shp(0));                                // layer 0 part 0 of the first tile

    f32x16 accA[2][4], accB[2][4];
#pragma unroll 1
    for (int tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
        const int shape = tile / a.tiles_per_shape;
        const int local = tile - shape * a.tiles_per_shape;
        {
            const int nt = tile + (int)gridDim.x;
            c.aux_next = nt < a.n_tiles ? shape_aux(nt) : c.aux_w;
        }
        c.st_on = FS_STAMP && c.wave == 0 && tile == (int)blockIdx.x + (int)gridDim.x;
        c.st_i = 0;
        stamp(c);
        // ---- aux B fragments [x_hi,y_hi,z_hi,x_lo,y_lo,z_lo,1,1] of point 32n + (lane&31),
        // into this wave's LDS copy
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            int pt = local * kTilePoints + 32 * n + (c.lane & 31);
            if (pt >= a.npts) pt = a.npts - 1;
            float x, y, z;
            if (POINTS) {
                const float* qq = a.xyz + ((size_t)shape * a.npts + pt) * 3;
                x = qq[0];
                y = qq[1];
                z = qq[2];
            } else {
                grid_point(pt, a.N, a.k0, a.vs, a.origin, x, y, z);
            }
            const float xh = Elem<T>::round(x), yh = Elem<T>::round(y), zh = Elem<T>::round(z);
            u32x4 f;
            f[0] = c.h ? 0u : Elem<T>::pack(xh, yh);
            f[1] = c.h ? 0u : Elem<T>::pack(zh, x - xh);
            f[2] = c.h ? 0u : Elem<T>::pack(y - yh, z - zh);
            f[3] = c.h ? 0u : Elem<T>::pack(1.f, 1.f);
            xyz_l[n * 64] = f;
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) c.part[n] = 0.f;

        // ---- layer 0 (aux only): part 0 -> A -> early positions now (the previous tile's
        // readers all passed its final barrier), part 1 -> B -> late positions during L1p0
        run_part<T, FE_NONE, false, FS_D>(c, accA, accB, 0, false, shp(1), 0, false);
        run_part<T, FE_NONE, false, FS_D>(c, accB, accA, 0, false, bias(2), 0, false);
        acc_to_lds<T, FS_D>(c, accA, 4 * c.wave);
        stamp(c);

        // ---- two-part layers 1, 2 (and 3 when 512 wide)
        constexpr int L2P = S == 256 ? 3 : 4;
        int pi = 2;
#pragma unroll 1
        for (int l = 1; l < L2P; ++l, pi += 2) {
            // the part after layer 3 (512 wide) is layer 4's: per-shape aux
            const FSrc nx = (S == 512 && l == 3) ? shp(2) : bias(pi + 2);
            run_part<T, FE_LATE, false, FS_D>(c, accA, accB, 32, true, bias(pi + 1), 0, true);
            run_part<T, FE_EARLY, true, FS_D>(c, accB, accA, 32, true, nx, 0, false);
        }
        if (S == 256) {
            // layer 3: one part of rows 64w..64w+63 -> positions 16 + 4w + 2i + s (serial,
            // once every wave is done reading layer 3's inputs)
            run_part<T, FE_LATE, false, FS_D>(c, accA, accB, 32, true, shp(2), 0, true);
            fs_bar();
            acc_to_lds<T, FS_D>(c, accA, 16 + 4 * c.wave);
            stamp(c);
            // layer 4 (K = 256, positions 16..31); part 0 -> early positions during part 1
            run_part<T, FE_NONE, false, FS_D>(c, accA, accB, 16, false, shp(3), 16, true);
            run_part<T, FE_EARLY, false, FS_D>(c, accB, accA, 16, false, bias(pi + 3), 16, false);
            pi += 3;
        } else {
            run_part<T, FE_LATE, false, FS_D>(c, accA, accB, 32, true, shp(3), 0, true);
            run_part<T, FE_EARLY, true, FS_D>(c, accB, accA, 32, true, bias(pi + 2), 0, false);
            pi += 2;
        }
        // ---- layers 5, 6
#pragma unroll 1
        for (int l = 5; l < 7; ++l, pi += 2) {
            run_part<T, FE_LATE, false, FS_D>(c, accA, accB, 32, true, bias(pi + 1), 0, true);
            run_part<T, FE_EARLY, true, FS_D>(c, accB, accA, 32, true, bias(pi + 2), 0, false);
        }
        // ---- layer 7: part 0 folds into the dot product during part 1; part 1 after it
        run_part<T, FE_LATE, false, FS_D>(c, accA, accB, 32, true, bias(pi + 1), 0, true);
        run_part<T, FE_FIN, false, FS_D>(c, accB, accA, 32, false, FSrc{true, c.aux_next}, 0,
                                         false);
        fin_serial(c, accB);
        // ---- final layer across waves: lanes l and l^32 hold the same point
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const float tot = c.part[n] + __shfl_xor(c.part[n], 32);
            if (c.h == 0) red[(c.wave * 4 + n) * 32 + c.lane] = tot;
        }
        stamp(c);
        fs_bar();
        if (c.h == 0) {
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) s += red[(w * 4 + c.wave) * 32 + c.lane];
            const int pt = local * kTilePoints + 32 * c.wave + c.lane;
            if (pt < a.npts)
                __builtin_nontemporal_store(tanhf(s + a.b_last), a.out + (size_t)shape * a.npts + pt);
        }
        stamp(c);
        c.aux_w = c.aux_next;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (FS_STAMP && c.wave == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        for (int k = c.lane; k < 128; k += 64)
            reinterpret_cast<unsigned long long*>(a.out)[(size_t)blockIdx.x * 128 + k] = c.st[k];
    }
}

template <typename T, int S, int D>
void launch_fs_d(const FArgs& a, bool points, hipStream_t s, int grid) {
    if (points)
        hipLaunchKernelGGL((dec_fs_kernel<T, S, true, D>), dim3(grid), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((dec_fs_kernel<T, S, false, D>), dim3(grid), dim3(256), 0, s, a);
}

template <typename T, int S>
void launch_fs(const FArgs& a, bool points, hipStream_t s, int grid) {
#ifdef LDM_DEV_KNOBS
    if (dev_knob("LDM_FS_D", kFsDefaultD) == 8) return launch_fs_d<T, S, 8>(a, points, s, grid);
    if (dev_knob("LDM_FS_D", kFsDefaultD) == 4) return launch_fs_d<T, S, 4>(a, points, s, grid);
#endif
    launch_fs_d<T, S, kFsDefaultD>(a, points, s, grid);
}

}  // namespace

size_t decoder_fs_aux_bytes(int B) { return (size_t)B * 4 * 4 * kFsStep; }

int decoder_fs_n_stages(int skip_width) { return fs_nsteps(skip_width == 253 ? 256 : 512); }

int decoder_fs_fwd(const ldm_decoder_t* w, const float* beta, const float* xyz, int B, int npts,
                   int N, int k0, float vs, float origin, float* out, void* ws, size_t ws_bytes,
                   hipStream_t s, int num_cus) {
    const int S = w->skip_width == 253 ? 256 : 512;
    LDM_REQUIRE(w->n_stages == fs_nsteps(S), LDM_EINVAL, "split layout: n_stages %d != %d",
                w->n_stages, fs_nsteps(S));
    LDM_REQUIRE(ws != nullptr && ws_bytes >= decoder_fs_aux_bytes(B) && LDM_ALIGNED(ws, 16),
                LDM_ENOSPC, "workspace too small: need %zu bytes, got %zu",
                decoder_fs_aux_bytes(B), ws_bytes);
    LDM_REQUIRE((size_t)B * 4 * 4 * kFsStep < 0x7ffffff0u, LDM_EINVAL,
                "split layout: %d shapes exceed the aux buffer range", B);
    {
        const int n = B * 4 * 4 * 2 * 64;
        if (w->dtype == LDM_BF16)
            hipLaunchKernelGGL(fs_aux_pack_kernel<__bf16>, dim3((n + 255) / 256), dim3(256), 0, s,
                               beta, w->wxyz, B, (__bf16*)ws);
        else
            hipLaunchKernelGGL(fs_aux_pack_kernel<_Float16>, dim3((n + 255) / 256), dim3(256), 0,
                               s, beta, w->wxyz, B, (_Float16*)ws);
        if (int e = launch_status("fs_aux_pack")) return e;
    }
    FArgs a;
    a.stream = (const uint8_t*)w->weights;
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
        if (S == 256) launch_fs<__bf16, 256>(a, points, s, grid);
        else launch_fs<__bf16, 512>(a, points, s, grid);
    } else {
        if (S == 256) launch_fs<_Float16, 256>(a, points, s, grid);
        else launch_fs<_Float16, 512>(a, points, s, grid);
    }
    return launch_status("ldm_decoder_fwd(split)");
}

}  // namespace ldm
