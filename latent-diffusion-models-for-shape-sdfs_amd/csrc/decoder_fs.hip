// Feature-split MFMA decoder (weight layout LDM_LAYOUT_SPLIT): SURVEY.md §8(a) A1+A3.
//
// The operand maps of DESIGN.md §3 (v_mfma_f32_32x32x16, accumulator rows as the next layer's B
// fragment) with the work inside a workgroup split by output feature (DESIGN.md §4 "split
// kernel"; it superseded the round-1/2 pass8 and quarter kernels, removed in ABI 5):
//   * a tile is 128 points = 4 point chunks (n) of 32, shared by the workgroup's 4 waves;
//   * wave w owns the OUTPUT FEATURES [128w, 128w+128) of every 512-wide layer as two parts of
//     64 rows (2 m-chunks of 32); the one-part layer 3 of DeepSDF (253 -> 256) gives each wave
//     rows [64w, 64w+64);
//   * the tile's activations live once, in LDS, as B fragments (128 KiB, 32 positions of 4
//     point chunks x 1 KiB; position 32 = the tile's xyz fragments of the aux steps); every
//     wave reads every position's 4 B fragments;
//   * each wave streams ITS OWN weight fragments (2 per k-step, 2 KiB) from L2 straight into a
//     register ring (raw buffer loads, kFsD k-steps ahead): no LDS ring, no DMA barrier.
//     Per k-step a wave reads 2 A fragments (L2) + 4 B fragments (LDS) for 8 MFMAs: each
//     fragment feeds 4 (A) or 2 (B) MFMAs (the removed quarter kernel read one LDS fragment
//     per MFMA); each weight byte feeds the tile's 128 points.
//   * a part's accumulators (2 m x 4 n tiles = 128 fp32) alternate between two sets A and B,
//     and a finished set is converted (16-bit + ReLU) straight into LDS inside a 16-step
//     window of a LATER part, half a tile per step, between its MFMAs:
//       - a layer's part 1 (set B) -> the "late" positions 16..31, during the next layer's
//         part 0 steps 0-14; a barrier inside its step 15 publishes them;
//       - a layer's part 0 (set A) -> the "early" positions 0..15, during the SAME layer's
//         part 1 steps 16-30: part 1 reads the early positions in steps 0-15, so after the
//         barrier inside its step 15 no wave reads them any more; the barrier inside its
//         step 31 publishes them to the next layer;
//       - layer 7's parts fold into the final 512 -> 1 dot product instead (fp32, w_last):
//         part 0 during part 1, part 1 during the NEXT tile's layer 1 part 0 (which also
//         stores the previous tile's outputs).
//     The barriers sit INSIDE a step, after its first MFMA pair, so the next position's reads
//     after them stay covered by the step's remaining MFMAs.  Serial LDS writes: layer 0
//     (both parts) and layer 3 of DeepSDF.
//   * the bias (and, for layers 0 and 4, xyz + the folded latent) enters as one aux MFMA step
//     at the START of each part (A = [wx,wy,wz,wx,wy,wz,b_hi,b_lo], B = [x_hi,y_hi,z_hi,x_lo,
//     y_lo,z_lo,1,1]), which also zero-initialises the accumulators.
// Barriers per tile: 3 per layer.
#include "decoder_common.h"

namespace ldm {
namespace {
using namespace dec;

// k-steps of A fragments in flight per wave (register ring depth = one 4-step stream group)
constexpr int kFsD = 4;
// FV (kernel variant, template): bit 0 = an in-stream barrier sits after the step's SECOND
// MFMA pair instead of its first; bit 1 = one LDS base per 4-step group (dev-build A/B:
// LDM_FS_V=<FV>).  Measured and dropped: layers 2..7 as one runtime loop with every part kind
// inlined once (74 -> 50 KB of code, 1.2 % slower: profiles/r04b/ab_decoder_v.log).
constexpr int kFsDefaultV = 2;   // group base: +0.5 % (profiles/r04b/ab_decoder_v.log)

constexpr int kFsStep = 2048;                       // one wave's A fragments of one k-step
// activation buffer: 32 positions of 4 KiB + position 32 = the tile's aux B fragments
// [x_hi,y_hi,z_hi,x_lo,y_lo,z_lo,1,1] (every part's last step reads it for the next aux step)
constexpr int kFsAct = 33 * 4 * 1024;
constexpr int kFsRed = 4 * 4 * 64 * 4;              // final partials [wave][n][64 lanes] fp32
constexpr int kFsWl = 512 * 4;                      // permuted final-layer weights
// Diagnostic build only (-DFS_STAMP=1, scripts/stamp_split.py; results are wrong): wave 0 of
// every workgroup stamps s_memtime at part and layer boundaries of its second tile, dumped over
// the output at the end.
#ifndef FS_STAMP
#define FS_STAMP 0
#endif
constexpr int kFsStamp = FS_STAMP ? 128 * 8 : 0;
// Diagnostic ablations (stamp builds only, results wrong; scripts/stamp_split.py, DESIGN.md §4
// round 6): FS_ABL bit 0 = no weight stream (the ring keeps its registers), bit 1 = no epilogue
// units, bit 2 = no in-stream barriers
#ifndef FS_ABL
#define FS_ABL 0
#endif
static_assert(FS_ABL == 0 || FS_STAMP, "ablations are diagnostic builds");
constexpr int kFsLds = kFsAct + kFsRed + kFsWl + kFsStamp;
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
//   FE_FIN0: layer 7 part 0 (set A) -> the final dot product, during layer 7 part 1;
//   FE_FIN1: layer 7 part 1 of the PREVIOUS tile (set B) -> the dot product, during layer 1 part
//            0 of this one; its step 14 publishes the partials (the mid barrier) and the part
//            sums them and stores the previous tile's outputs after that barrier
enum FsEpi { FE_NONE = 0, FE_LATE = 1, FE_EARLY = 2, FE_FIN0 = 3, FE_FIN1 = 4 };

// A fragment source: a buffer resource (SGPRs) + a byte offset (SGPR); the lane's 16 bytes at
// voffset lane*16 (+1024: the second fragment, an immediate).  Raw buffer loads keep every
// address in scalar registers: plain global loads made the compiler materialise (and hoist,
// then spill) a 64-bit VGPR address per load site.
struct FSrc {
    bool shape;               // per-shape aux (workspace) or the weight blob
    uint32_t off;             // byte offset in that buffer
    bool none = false;        // nothing to prefetch (the tile's last part)
};

template <int FV>
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
    u32x4 ring[kFsD][2];
    u32x4 b[4];               // the B fragments of the step about to run (rolling)
    float part[4];            // final-layer partial sums of point chunk n
    float* out;               // the previous tile's outputs (FE_FIN1): [shape][npts]
    int npts, prev_shape, prev_local;   // prev_local < 0: no previous tile
    float b_last;
    unsigned long long* st;   // FS_STAMP
    int st_i;
    bool st_on;
};

template <int FV>
__device__ __forceinline__ void stamp(FCtx<FV>& c) {
    if (FS_STAMP) {
        if (c.st_on && c.lane == 0 && c.st_i < 128) c.st[c.st_i] = __builtin_readcyclecounter();
        ++c.st_i;
    }
}

__device__ __forceinline__ u32x4 bld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

template <int FV>
__device__ __forceinline__ void load_aux(FCtx<FV>& c, FSrc s) {
    if (s.none) return;
    const __amdgpu_buffer_rsrc_t r = s.shape ? c.ra : c.rw;
    c.auxn[0] = bld(r, c.voff, s.off);
    c.auxn[1] = bld(r, c.voff + 1024u, s.off);
}

// A lane's LDS byte address `voff + off` (off wave-uniform: one v_add).
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ int opaque_s(int v) {
    asm volatile("" : "+s"(v));
    return v;
}

// LDS addressing.  Immediates are 16 bits, so most accesses need a register base past 64 KiB;
// left to itself the compiler materialised one VGPR per constant address, hoisted them out of
// the tile loop and spilled them -- and every spill reload waits vmcnt(0), i.e. for the whole
// weight ring in flight.  So every address is formed AT ITS USE from an opaque copy of voff
// (a volatile asm is neither hoisted nor folded): one or two VALU per use, nothing long-lived
// but voff itself.
template <int FV>
__device__ __forceinline__ char* lds_at(const FCtx<FV>& c, uint32_t off) {
    return c.smem + (opaque(c.voff) + off);
}
// this wave's early (0) / late (16) positions: + (2i + s) * 4 KiB + n * 1 KiB immediates
template <int FV>
__device__ __forceinline__ u32x4* act_w(const FCtx<FV>& c, int late) {
    return reinterpret_cast<u32x4*>(lds_at(c, (uint32_t)(late + 4 * c.wave) * 4096u));
}
// final-layer weights of (this wave, part p, m-chunk i, this lane half)
template <int FV>
__device__ __forceinline__ const f32x4* wl_at(const FCtx<FV>& c, int p, int i) {
    const uint32_t h = opaque(c.voff) >> 9;           // lane >> 5
    return reinterpret_cast<const f32x4*>(
        c.smem + kFsAct + kFsRed + (((c.wave * 2 + p) * 2 + i) * 2) * 64 + h * 64);
}

// this lane's final partials red[wave][n][lane] (+ n * 64 floats)
template <int FV>
__device__ __forceinline__ float* red_w(const FCtx<FV>& c) {
    return reinterpret_cast<float*>(c.smem + kFsAct + c.wave * 4 * 64 * 4 + (opaque(c.voff) >> 2));
}

// LDS barrier: LDS writes done (lgkmcnt), then s_barrier.  The weight loads in flight
// (vmcnt) are NOT waited for: they feed registers only.
__device__ __forceinline__ void fs_bar() {
    if (FS_ABL & 4) return;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The activation buffer is kept in CONSUMPTION order: position j (4 KiB: 4 point chunks x
// 1 KiB) holds the k-step that ring step j of the next layer reads (pack.split_kidx): after a
// 512-wide layer, k-step 8w + 4u + 2i + s sits at position 16u + 4w + 2i + s (u = 0: part 0,
// the "early" positions; u = 1: part 1, the "late" ones); after layer 3 at skip 253, k-step
// 4w + 2i + s at position 16 + 4w + 2i + s (layer 4 reads positions 16 + j).  Step j reads
// position pos0 + j: the addresses are immediates from one group base.
template <int FV>
__device__ __forceinline__ void read_b(FCtx<FV>& c, int pos) {
    const u32x4* p = reinterpret_cast<const u32x4*>(lds_at(c, pos * 4096));
#pragma unroll
    for (int n = 0; n < 4; ++n) c.b[n] = p[n * 64];
}

// Stream step r (0..3) of the 4-step stream group at c.s_iss into ring slot r: the
// (r & 1) * 2 KiB + fragment offset folds into the load's immediate, the (r >> 1) * 4 KiB into
// the scalar offset, so a group costs one wrap test instead of one per step.
template <int FV>
__device__ __forceinline__ void issue(FCtx<FV>& c, int r) {
    const uint32_t so = c.s_iss + (uint32_t)(r >> 1) * 2u * kFsStep;
    const uint32_t vo = c.voff + (uint32_t)(r & 1) * kFsStep;
    if (FS_ABL & 1) return;
    c.ring[r][0] = bld(c.rw, vo, so);
    c.ring[r][1] = bld(c.rw, vo + 1024u, so);
}

template <int FV>
__device__ __forceinline__ void next_group(FCtx<FV>& c) {
    c.s_iss += 4u * kFsStep;
    if (c.s_iss == c.s_end) c.s_iss = c.s_beg;
}

// ReLU of an fp32 value as ONE integer max: a negative float is a negative int32 (sign bit),
// so max(bits, 0) is +0 for it and the value itself otherwise (fmaxf costs a NaN-quieting
// v_max plus the max under IEEE mode: two instructions per element)
__device__ __forceinline__ float relu_f(float x) {
    return __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));
}

// One epilogue unit u = 2t + s of the other accumulator set: HALF of tile t = 4i + n (its
// accumulator registers 8s..8s+7 = the B fragment of k-step 2i + s).
template <typename T, int EK, int FV>
__device__ __forceinline__ void epi_unit(FCtx<FV>& c, const f32x16 (&accY)[2][4], int u) {
    const int t = u >> 1, s = u & 1;
    const int i = t >> 2, n = t & 3;
    if (FS_ABL & 2) return;
    if (EK == FE_LATE || EK == FE_EARLY) {   // part 1 of the previous layer / part 0 of this
        u32x4 f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            f[q] = relu2(Elem<T>::pack(accY[i][n][8 * s + 2 * q], accY[i][n][8 * s + 2 * q + 1]));
        u32x4* p = act_w(c, EK == FE_LATE ? 16 : 0);
        p[((2 * i + s) * 4 + n) * 64] = f;
    } else if (EK == FE_FIN0 || EK == FE_FIN1) {     // layer 7 -> the final dot product
        const f32x4* w = wl_at(c, EK == FE_FIN0 ? 0 : 1, i);
        float part = c.part[n];
#pragma unroll
        for (int q = 2 * s; q < 2 * s + 2; ++q) {
            const f32x4 wv = w[q];
#pragma unroll
            for (int e = 0; e < 4; ++e) part = fmaf(relu_f(accY[i][n][4 * q + e]), wv[e], part);
        }
        c.part[n] = part;
    }
}

// The 16 units of an epilogue window of 16 steps k = 0..15: unit k in step k < 14, units 14
// and 15 in step 14, none in step 15 -- so the window's LDS writes are all issued before the
// barrier that closes it (inside step 15, see group4).
template <typename T, int EK, int FV>
__device__ __forceinline__ void epi_step(FCtx<FV>& c, const f32x16 (&accY)[2][4], int k) {
    if (EK == FE_NONE || k == 15) return;
    epi_unit<T, EK>(c, accY, k);
    if (k == 14) epi_unit<T, EK>(c, accY, 15);
    if (EK == FE_FIN1 && k == 14) {         // the partials -> red[wave][n][lane], published by
        float* rw = red_w(c);               // the barrier inside step 15
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            rw[n * 64] = c.part[n];
            c.part[n] = 0.f;
        }
    }
}

// the final layer across waves and lane halves (lanes l and l^32 hold the same point): lanes
// < 32 of wave w sum point chunk w's 8 partials (after the barrier that published them), add
// the bias, tanh, store
template <int FV>
__device__ __forceinline__ void fin_store(const FCtx<FV>& c, int shape, int local) {
    const int lane = (int)(opaque(c.voff) >> 4);     // formed here: nothing kept live (spills)
    if (local < 0 || lane >= 32) return;
    const float* rr = reinterpret_cast<const float*>(
        c.smem + kFsAct + c.wave * 64 * 4 + (opaque(c.voff) >> 2));
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) s += rr[w * 4 * 64] + rr[w * 4 * 64 + 32];
    const int pt = local * kTilePoints + 32 * c.wave + lane;
    if (pt < c.npts) {
        // a buffer store off the shape's row (scalar base, 32-bit lane offset): a 64-bit VGPR
        // address here was kept live across the tile loop and spilled
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(c.out + (size_t)shape * c.npts), (short)0, 0x7ffffff0, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, tanhf(s + c.b_last)),
                                              ro, (uint32_t)pt * 4u, 0, 2 /* nt */);
    }
}

// scheduling slot of v VALU instructions (0, 2 or 4; v is a constant once unrolled)
__device__ __forceinline__ void valu_slot(int v) {
    if (v == 2) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
    else if (v == 4) __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
}

// MFMA pair of point chunk n of one step (both m-chunks of the wave's part)
template <typename T>
__device__ __forceinline__ void mfma_pair(f32x16 (&acc)[2][4], const u32x4& a0, const u32x4& a1,
                                          const u32x4& b, int n) {
    acc[0][n] = Elem<T>::mfma(a0, b, acc[0][n]);
    acc[1][n] = Elem<T>::mfma(a1, b, acc[1][n]);
}

// Four k-steps reading positions p0..p0+3 (ring slots 0..3), epilogue window steps K0..K0+3.
// Rolling B fragments: chunk n of step j+1 is read as soon as step j's two MFMAs on chunk n are
// issued (~6 MFMAs, ~190 cycles, before it is needed).  BAR = r: an LDS barrier INSIDE step r,
// after its first (FV & 1: second) MFMA pair and before its first read of the next position:
// the waves wait on each other with the step's remaining MFMAs still to issue and the next
// position's reads still covered by them (a barrier between steps exposed one LDS round trip
// plus the pipeline drain, ~500-750 cycles per barrier).
template <typename T, int EK, int K0, int BAR, int FV>
__device__ __forceinline__ void group4(FCtx<FV>& c, f32x16 (&acc)[2][4], const f32x16 (&accY)[2][4],
                                       int p0) {
    constexpr int BP = (FV & 1) ? 2 : 1;     // MFMA pairs before the in-stream barrier
    // FV bit 1: ONE LDS base for the group's four next positions (r * 4 KiB + n * 1 KiB fold
    // into the ds_read immediates) instead of an address formed per step
    const char* gbase = (FV & 2) ? lds_at(c, (p0 + 1) * 4096) : nullptr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const u32x4* nb = reinterpret_cast<const u32x4*>(
            (FV & 2) ? gbase + r * 4096 : lds_at(c, (p0 + r + 1) * 4096));
        const u32x4 a0 = c.ring[r][0], a1 = c.ring[r][1];
        const int k = K0 + r;
        // the step's VALU (epilogue: AGPR reads, cvt, ReLU, LDS address) 2 per MFMA gap, 4 in
        // the double-unit step 14 (the guide: <= 5 fillers per 32x32x16 gap hide)
        const int V = (EK == FE_NONE || k == 15) ? 0 : (k == 14 ? 4 : 2);
        if (r == BAR) {
#pragma unroll
            for (int n = 0; n < BP; ++n) mfma_pair<T>(acc, a0, a1, c.b[n], n);
            for (int n = 0; n < BP; ++n) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            fs_bar();
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int n = 0; n < BP; ++n) c.b[n] = nb[n * 64];
#pragma unroll
            for (int n = BP; n < 4; ++n) {
                mfma_pair<T>(acc, a0, a1, c.b[n], n);
                c.b[n] = nb[n * 64];
            }
            issue(c, r);
            epi_step<T, EK>(c, accY, k);
            for (int n = 0; n < BP; ++n) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            for (int n = BP; n < 4; ++n) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                valu_slot(V);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                valu_slot(V);
            }
        } else {
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                mfma_pair<T>(acc, a0, a1, c.b[n], n);
                c.b[n] = nb[n * 64];
            }
            issue(c, r);
            epi_step<T, EK>(c, accY, k);
            // pin the step's order for the scheduler (left free it sank the B reads and weight
            // loads below the last MFMA): per point chunk n, MFMA, [VALU], MFMA, B read,
            // [VALU]; then the 2 weight loads
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                valu_slot(V);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                valu_slot(V);
            }
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    next_group(c);
}

// 16 k-steps from position p0 carrying the 16 epilogue units of the other set; BAR: the
// window's closing barrier inside its step 15
template <typename T, int EK, bool BAR, int FV>
__device__ __forceinline__ void steps16e(FCtx<FV>& c, f32x16 (&acc)[2][4],
                                         const f32x16 (&accY)[2][4], int p0) {
    group4<T, EK, 0, -1, FV>(c, acc, accY, p0);
    group4<T, EK, 4, -1, FV>(c, acc, accY, p0 + 4);
    group4<T, EK, 8, -1, FV>(c, acc, accY, p0 + 8);
    group4<T, EK, 12, BAR ? 3 : -1, FV>(c, acc, accY, p0 + 12);
}

// plain k-steps [j0, j1) from position pos0 as ONE runtime loop of 4-step groups (code size:
// the kernel must stay well inside the instruction cache)
template <typename T, int FV>
__device__ __forceinline__ void steps_plain(FCtx<FV>& c, f32x16 (&acc)[2][4],
                                            const f32x16 (&accY)[2][4], int pos0, int j0, int j1) {
#pragma unroll 1
    for (int j = j0; j < j1; j += 4) group4<T, FE_NONE, 0, -1, FV>(c, acc, accY, pos0 + j);
}

// One part: the aux step, then nk ring steps reading positions pos0 .. pos0 + nk - 1 = 31
// (the last one reads position 32, the tile's aux B fragments, for the next part's aux step).
//   * aux step: zero-initialises acc with [wx,wy,wz,wx,wy,wz,b_hi,b_lo] x xyz (c.b on entry)
//     and, per point chunk, reads the first position's B fragment behind its MFMA pair -- or,
//     `bar0`, after a barrier (the part follows serial LDS writes: layers 1 and 4 at skip 253);
//     then it loads the NEXT part's aux A fragments (naux).
//   * E work (the other set, EK) in steps 0-15 (E16 false) or 16-31 (E16 true).
//   * `mid`: the barrier inside step 15 (the late positions written during steps 0-14 by
//     every wave / no wave reads the early positions any more before E16 writes them);
//     `endbar` (E work parts): the barrier inside the part's last step, publishing the window's
//     writes to the next part, whose aux step then reads on without a barrier.
template <typename T, int EK, bool E16, int FV>
__device__ __forceinline__ void run_part(FCtx<FV>& c, f32x16 (&acc)[2][4], const f32x16 (&accY)[2][4],
                                         int nk, bool mid, bool endbar, FSrc naux, int pos0,
                                         bool bar0) {
    const f32x16 zero = {};
    const u32x4 a0 = c.auxn[0], a1 = c.auxn[1];
    if (nk == 0) {             // layer 0: the aux step only, c.b stays the xyz fragments
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            acc[0][n] = Elem<T>::mfma(a0, c.b[n], zero);
            acc[1][n] = Elem<T>::mfma(a1, c.b[n], zero);
        }
        load_aux(c, naux);
        stamp(c);
        return;
    }
    if (bar0) {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            acc[0][n] = Elem<T>::mfma(a0, c.b[n], zero);
            acc[1][n] = Elem<T>::mfma(a1, c.b[n], zero);
        }
        load_aux(c, naux);
        fs_bar();
        read_b(c, pos0);
    } else {
        const u32x4* p = reinterpret_cast<const u32x4*>(lds_at(c, pos0 * 4096));
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            acc[0][n] = Elem<T>::mfma(a0, c.b[n], zero);
            acc[1][n] = Elem<T>::mfma(a1, c.b[n], zero);
            c.b[n] = p[n * 64];
        }
        load_aux(c, naux);
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    stamp(c);
    if (!E16 && EK != FE_NONE) {        // E work in steps 0-15
        // the barrier inside step 15: mid (nk 32), or the end barrier of a 16-step part
        if (mid || (endbar && nk == 16)) steps16e<T, EK, true>(c, acc, accY, pos0);
        else steps16e<T, EK, false>(c, acc, accY, pos0);
        if (EK == FE_FIN1) fin_store(c, c.prev_shape, c.prev_local);
        stamp(c);
        if (endbar && nk == 32) {       // the end barrier inside step 31
            steps_plain<T>(c, acc, accY, pos0, 16, 28);
            group4<T, FE_NONE, 0, 3, FV>(c, acc, accY, pos0 + 28);
        } else {
            steps_plain<T>(c, acc, accY, pos0, 16, nk);
        }
    } else if (E16) {                   // nk 32, mid
        steps_plain<T>(c, acc, accY, pos0, 0, 12);
        group4<T, FE_NONE, 0, 3, FV>(c, acc, accY, pos0 + 12);
        stamp(c);
        if (endbar) steps16e<T, EK, true>(c, acc, accY, pos0 + 16);
        else steps16e<T, EK, false>(c, acc, accY, pos0 + 16);
    } else {                            // plain part, no barrier (layer 4 part 0 at skip 253)
        steps_plain<T>(c, acc, accY, pos0, 0, nk < 16 ? nk : 16);
        stamp(c);
        steps_plain<T>(c, acc, accY, pos0, 16, nk);
    }
    stamp(c);
}

// a whole set into this wave's early (LATE = false) or late positions 16u + 4w + 2i + s
// (serial: layer 0, layer 3 at skip 253); the per-wave base and immediates per tile
template <typename T, bool LATE, int FV>
__device__ __forceinline__ void acc_to_lds(FCtx<FV>& c, const f32x16 (&acc)[2][4]) {
    u32x4* p = act_w(c, LATE ? 16 : 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            u32x4 f0, f1;
            acc_to_frags<T>(acc[i][n], f0, f1);
            p[(2 * i * 4 + n) * 64] = f0;
            p[((2 * i + 1) * 4 + n) * 64] = f1;
        }
}

template <typename T, int S, bool POINTS, int FV>
__global__ __launch_bounds__(256, 1) void dec_fs_kernel(FArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[kFsLds];
    FCtx<FV> c;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.h = c.lane >> 5;
    c.voff = (uint32_t)c.lane * 16u;
    c.smem = smem;
    c.out = a.out;
    c.npts = a.npts;
    c.b_last = a.b_last;
    c.prev_shape = 0;
    c.prev_local = -1;
    c.st = reinterpret_cast<unsigned long long*>(smem + kFsAct + kFsRed + kFsWl);
    c.st_i = 0;
    c.st_on = false;
    float* wl = reinterpret_cast<float*>(smem + kFsAct + kFsRed);

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
    for (int r = 0; r < kFsD; ++r) issue(c, r);
    next_group(c);

    f32x16 accA[2][4], accB[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int n = 0; n < 4; ++n) accB[i][n] = f32x16{};    // the first tile's FE_FIN1 input
#pragma unroll
    for (int n = 0; n < 4; ++n) c.part[n] = 0.f;
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
        load_aux(c, shp(0));            // L0p0's aux fragments (latency under the xyz setup)
        // ---- aux B fragments [x_hi,y_hi,z_hi,x_lo,y_lo,z_lo,1,1] of point 32n + (lane&31) at
        // position 32.  Every wave writes the same bytes (no barrier: a wave reads back its own
        // writes, the others only ever replace them with equal values; every read of the
        // previous tile's position 32 came before its final barrier)
        // lane values formed here from an opaque voff (kept live across the tile loop, they
        // were spilled and reloaded behind the whole weight ring)
        const uint32_t lv = opaque(c.voff);
        const bool hi = lv >= 512u;                       // lane >= 32
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            int pt = local * kTilePoints + 32 * n + (int)((lv >> 4) & 31u);
            if (pt >= a.npts) pt = a.npts - 1;
            float x, y, z;
            if (POINTS) {
                const float* qq = a.xyz + ((size_t)shape * a.npts + pt) * 3;
                x = qq[0];
                y = qq[1];
                z = qq[2];
            } else {
                // N through an opaque SGPR: the divisions' reciprocals are formed per tile
                // instead of hoisted out of the loop (and spilled)
                grid_point(pt, opaque_s(a.N), a.k0, a.vs, a.origin, x, y, z);
            }
            const float xh = Elem<T>::round(x), yh = Elem<T>::round(y), zh = Elem<T>::round(z);
            u32x4 f;
            f[0] = hi ? 0u : Elem<T>::pack(xh, yh);
            f[1] = hi ? 0u : Elem<T>::pack(zh, x - xh);
            f[2] = hi ? 0u : Elem<T>::pack(y - yh, z - zh);
            f[3] = hi ? 0u : Elem<T>::pack(1.f, 1.f);
            reinterpret_cast<u32x4*>(lds_at(c, 32u * 4096u))[n * 64] = f;
        }
        read_b(c, 32);

        // ---- layer 0 (aux only), both parts through set A into LDS serially (set B still
        // holds the previous tile's layer 7 part 1, folded into the output during L1p0); the
        // previous tile's readers all passed the end barrier of its layer 7
        run_part<T, FE_NONE, false, FV>(c, accA, accB, 0, false, false, shp(1), 0, false);
        acc_to_lds<T, false, FV>(c, accA);
        stamp(c);
        run_part<T, FE_NONE, false, FV>(c, accA, accB, 0, false, false, bias(2), 0, false);
        acc_to_lds<T, true, FV>(c, accA);
        stamp(c);

        // ---- two-part layers 1, 2 (and 3 when 512 wide).  L1p0 folds the previous tile's
        // layer 7 part 1 into its outputs (FE_FIN1); p1 of layer l publishes with its end barrier
        int pi = 2;
        run_part<T, FE_FIN1, false, FV>(c, accA, accB, 32, true, false, bias(pi + 1), 0, true);
        run_part<T, FE_EARLY, true, FV>(c, accB, accA, 32, true, true, bias(pi + 2), 0, false);
        pi += 2;
        constexpr int L2P = S == 256 ? 3 : 4;
#pragma unroll 1
        for (int l = 2; l < L2P; ++l, pi += 2) {
            // the part after layer 3 (512 wide) is layer 4's: per-shape aux
            const FSrc nx = (S == 512 && l == 3) ? shp(2) : bias(pi + 2);
            run_part<T, FE_LATE, false, FV>(c, accA, accB, 32, true, false, bias(pi + 1), 0, false);
            run_part<T, FE_EARLY, true, FV>(c, accB, accA, 32, true, true, nx, 0, false);
        }
        if (S == 256) {
            // layer 3: one part of rows 64w..64w+63 -> positions 16 + 4w + 2i + s (serial,
            // once every wave is done reading layer 3's inputs)
            run_part<T, FE_LATE, false, FV>(c, accA, accB, 32, true, false, shp(2), 0, false);
            fs_bar();
            acc_to_lds<T, true, FV>(c, accA);
            stamp(c);
            // layer 4 (K = 256, positions 16..31); part 0 -> early positions during part 1
            run_part<T, FE_NONE, false, FV>(c, accA, accB, 16, false, false, shp(3), 16, true);
            run_part<T, FE_EARLY, false, FV>(c, accB, accA, 16, false, true, bias(pi + 3), 16,
                                             false);
            pi += 3;
        } else {
            run_part<T, FE_LATE, false, FV>(c, accA, accB, 32, true, false, shp(3), 0, false);
            run_part<T, FE_EARLY, true, FV>(c, accB, accA, 32, true, true, bias(pi + 2), 0, false);
            pi += 2;
        }
        // ---- layers 5, 6
#pragma unroll 1
        for (int l = 5; l < 7; ++l, pi += 2) {
            run_part<T, FE_LATE, false, FV>(c, accA, accB, 32, true, false, bias(pi + 1), 0, false);
            run_part<T, FE_EARLY, true, FV>(c, accB, accA, 32, true, true, bias(pi + 2), 0, false);
        }
        // ---- layer 7: part 0 folds into the dot product during part 1, part 1 during the
        // next tile's L1p0 (its end barrier lets the next tile overwrite every position)
        run_part<T, FE_LATE, false, FV>(c, accA, accB, 32, true, false, bias(pi + 1), 0, false);
        // (no prefetch of the next tile's first aux fragments here: live across the whole
        // part they were spilled, each spill waiting for the whole ring)
        run_part<T, FE_FIN0, false, FV>(c, accB, accA, 32, false, true, FSrc{true, 0, true}, 0,
                                        false);
        c.prev_shape = shape;
        c.prev_local = local;
        c.aux_w = c.aux_next;
    }
    // the last tile's layer 7 part 1: the FE_FIN1 units in their window order (a point's
    // value must not depend on whether its tile was its workgroup's last)
#pragma unroll
    for (int u = 0; u < 16; ++u) epi_unit<T, FE_FIN1>(c, accB, u);
    {
        float* rw = red_w(c);
#pragma unroll
        for (int n = 0; n < 4; ++n) rw[n * 64] = c.part[n];
    }
    fs_bar();
    fin_store(c, c.prev_shape, c.prev_local);
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
    switch (dev_knob("LDM_FS_V", kFsDefaultV)) {
        case 0: return launch_fs_d<T, S, 0>(a, points, s, grid);
        case 1: return launch_fs_d<T, S, 1>(a, points, s, grid);
        case 3: return launch_fs_d<T, S, 3>(a, points, s, grid);
        default: break;
    }
#endif
    launch_fs_d<T, S, kFsDefaultV>(a, points, s, grid);
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
