// Feature-split MFMA decoder (weight layout LDM_LAYOUT_SPLIT): SURVEY.md §8(a) A1+A3.
//
// Same math and operand maps as the quarter kernel (decoder_q.hip), a
// different split of the work inside a workgroup (DESIGN.md §4 "split kernel"):
//   * a tile is 128 points = 4 point chunks (n) of 32, shared by the workgroup's 4 waves;
//   * wave w owns the OUTPUT FEATURES [128w, 128w+128) of every 512-wide layer as two parts of
//     64 rows (2 m-chunks of 32); the one-part layer 3 of DeepSDF (253 -> 256) gives each wave
//     rows [64w, 64w+64);
//   * the tile's activations live once, in LDS, as B fragments: ACT[32 k-steps][4 n][64 lanes]
//     x 16 B = 128 KiB; every wave reads every k-step's 4 B fragments;
//   * each wave streams ITS OWN weight fragments (2 per k-step, 2 KiB) from L2 straight into a
//     register ring (global_load_dwordx4, FS_D k-steps ahead): no LDS ring, no DMA barrier.
//     Per k-step a wave reads 2 A fragments (L2) + 4 B fragments (LDS) for 8 MFMAs: each
//     fragment feeds 4 (A) or 2 (B) MFMAs, where the quarter kernel read one LDS fragment per
//     MFMA; the weight bytes per point are unchanged (each feeds the tile's 128 points).
//   * a part's accumulators (2 m x 4 n tiles = 128 fp32) alternate between two sets A and B;
//     the epilogue of the previous part (16-bit convert + ReLU) runs inside the first 8 k-steps
//     of the next part, one tile per step, between its MFMAs:
//       - the last part of a layer is converted straight into LDS ("late" k-steps 8w+4..8w+7),
//         so the next layer reads its "early" k-steps (8w..8w+3, written at the layer boundary)
//         first and meets one barrier at its step 16;
//       - part 0 of a layer is parked in registers (64 VGPRs, bf16) and written to LDS at the
//         layer boundary (two barriers: no reader of the old activations is left / all written);
//       - layer 7's parts fold into the final 512 -> 1 dot product instead (fp32, w_last).
//   * the bias (and, for layers 0 and 4, xyz + the folded latent) enters as one aux MFMA step
//     at the START of each part (A = [wx,wy,wz,wx,wy,wz,b_hi,b_lo], B = [x_hi,y_hi,z_hi,x_lo,
//     y_lo,z_lo,1,1]), which also zero-initialises the accumulators.
// Barriers per tile: ~21 (the quarter kernel: one per 2 k-steps, ~207).
#include "decoder_common.h"

namespace ldm {
namespace {
using namespace dec;

#ifndef FS_D
#define FS_D 4        // k-steps of A fragments in flight per wave (register ring depth)
#endif
static_assert(FS_D == 4 || FS_D == 8, "ring depth must divide 16");

constexpr int kFsStep = 2048;                       // one wave's A fragments of one k-step
constexpr int kFsAct = 32 * 4 * 1024;               // 128 KiB activation buffer
constexpr int kFsRed = 4 * 4 * 32 * 4;              // final partials [wave][n][32] fp32
constexpr int kFsWl = 512 * 4;                      // permuted final-layer weights
constexpr int kFsLds = kFsAct + kFsRed + kFsWl;
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
    const uint8_t* stream;   // [4 waves][nsteps][2 KiB]
    const uint8_t* baux;     // [4 waves][nparts][2 KiB] bias aux fragments
    const uint8_t* aux;      // workspace [B][4 waves][4 slots][2 KiB]
    const float* w_last;     // [4 w][2 p][2 i][2 h][16] (pack.permute_w_last_split)
    const float* xyz;
    float* out;
    float b_last;
    int npts, tiles_per_shape, n_tiles;
    int N, k0;
    float vs, origin;
};

// Epilogue kinds run inside a part's first 8 k-steps (on the OTHER accumulator set)
enum FsEpi { FE_NONE = 0, FE_LDS = 1, FE_PARK = 2, FE_FIN = 3 };

// A fragment source: a buffer resource (SGPRs) + a byte offset (SGPR); the lane's 16 bytes at
// voffset lane*16 (+1024: the second fragment, an immediate).  Raw buffer loads keep every
// address in scalar registers: plain global loads made the compiler materialise (and hoist,
// then spill) a 64-bit VGPR address per load site.
struct FSrc {
    bool shape;               // per-shape aux (workspace) or the weight blob
    uint32_t off;             // byte offset in that buffer
};

struct FCtx {
    int lane, wave, h;
    uint32_t voff;            // lane * 16
    char* smem;
    __amdgpu_buffer_rsrc_t rw;   // the weight blob: streams then bias aux fragments
    __amdgpu_buffer_rsrc_t ra;   // the per-shape aux workspace
    uint32_t s_beg, s_end;    // this wave's stream [s_beg, s_end) in rw
    uint32_t s_iss;           // next k-step to issue
    uint32_t baux_w;          // this wave's bias aux fragments [nparts][2 KiB] in rw
    uint32_t aux_w;           // this tile's per-shape aux of this wave [4 slots][2 KiB] in ra
    uint32_t aux_next;        // ... of the next tile
    u32x4 auxn[2];            // aux A fragments of the part about to start
    u32x4 ring[FS_D][2];
    u32x4 park[2][4][2];
    u32x4 xyzf[4];
    float part[4];
};

__device__ __forceinline__ u32x4 bld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

__device__ __forceinline__ void load_aux(FCtx& c, FSrc s) {
    const __amdgpu_buffer_rsrc_t r = s.shape ? c.ra : c.rw;
    c.auxn[0] = bld(r, c.voff, s.off);
    c.auxn[1] = bld(r, c.voff + 1024u, s.off);
}

// LDS barrier: LDS writes done (lgkmcnt), then s_barrier.  The weight loads in flight
// (vmcnt) are NOT waited for: they feed registers only.
__device__ __forceinline__ void fs_bar() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The activation buffer is kept in CONSUMPTION order: position j (4 KiB: 4 point chunks x
// 1 KiB) holds the k-step that ring step j of the next layer reads (pack.split_kidx): after a
// 512-wide layer, k-step 8w + 4u + 2i + s sits at position 16u + 4w + 2i + s (u = 0: part 0,
// written at the layer boundary; u = 1: part 1, written during the next layer's first steps);
// after layer 3 at skip 253, k-step 4w + 2i + s at position 4w + 2i + s.  So step j reads
// position j: the addresses are immediates from one group base.
__device__ __forceinline__ void read_b(const FCtx& c, int pos, u32x4 (&b)[4]) {
    const u32x4* p = reinterpret_cast<const u32x4*>(c.smem + pos * 4096 + c.voff);
#pragma unroll
    for (int n = 0; n < 4; ++n) b[n] = p[n * 64];
}

// Stream step r (0..3) of the 4-step stream group at c.s_iss into ring slot `slot`: the
// (r & 1) * 2 KiB + fragment offset folds into the load's immediate, the (r >> 1) * 4 KiB into
// the scalar offset, so a group costs one wrap test instead of one per step.
__device__ __forceinline__ void issue(FCtx& c, int slot, int r) {
    const uint32_t so = c.s_iss + (uint32_t)(r >> 1) * 2u * kFsStep;
    const uint32_t vo = c.voff + (uint32_t)(r & 1) * kFsStep;
    c.ring[slot][0] = bld(c.rw, vo, so);
    c.ring[slot][1] = bld(c.rw, vo + 1024u, so);
}

__device__ __forceinline__ void next_group(FCtx& c) {
    c.s_iss += 4u * kFsStep;
    if (c.s_iss == c.s_end) c.s_iss = c.s_beg;
}

// One tile t = 4i + n of the other accumulator set's epilogue.
template <typename T, int EK>
__device__ __forceinline__ void epi_tile(FCtx& c, const f32x16 (&accY)[2][4], int t, int fin_p) {
    const int i = t >> 2, n = t & 3;
    if (EK == FE_LDS) {          // last part of the previous layer -> its "late" positions
        u32x4 f0, f1;
        acc_to_frags<T>(accY[i][n], f0, f1);
        const int pos = 16 + 4 * c.wave + 2 * i;
        u32x4* p = reinterpret_cast<u32x4*>(c.smem + (pos * 4 + n) * 1024 + c.voff);
        p[0] = f0;
        p[4 * 64] = f1;            // k-step kk + 1
    } else if (EK == FE_PARK) {
        acc_to_frags<T>(accY[i][n], c.park[i][n][0], c.park[i][n][1]);
    } else if (EK == FE_FIN) {
        const f32x4* w = reinterpret_cast<const f32x4*>(
            c.smem + kFsAct + kFsRed + ((((c.wave * 2 + fin_p) * 2 + i) * 2 + c.h) * 16) * 4);
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

template <typename T>
__device__ __forceinline__ void mfma8(f32x16 (&acc)[2][4], const u32x4 a0, const u32x4 a1,
                                      const u32x4 (&b)[4]) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        acc[0][n] = Elem<T>::mfma(a0, b[n], acc[0][n]);
        acc[1][n] = Elem<T>::mfma(a1, b[n], acc[1][n]);
    }
}

// Four k-steps j0..j0+3 (ring slots RO..RO+3).  E work: tiles T0..T0+3 of the other set
// (EK != FE_NONE).  The next step's B fragments are read unconditionally (no selects in the
// loop): at the mid barrier and at a part's end that read is stale or unused and the caller
// reads again (position 32 is still inside the LDS allocation).  A scheduling barrier closes
// every step: left free, the scheduler sank all of a group's weight loads to its end, which
// left one step of latency cover instead of FS_D.
template <typename T, int EK, int T0, int RO>
__device__ __forceinline__ void group4(FCtx& c, f32x16 (&acc)[2][4], const f32x16 (&accY)[2][4],
                                       u32x4 (&b)[4], int j0, int fin_p) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        // rolling B fragments: chunk n of step j+1 is read as soon as step j's two MFMAs on
        // chunk n are issued, ~6 MFMAs (~190 cycles) before it is needed (a read after the
        // step's last MFMA left ~32 cycles of cover: an LDS round trip exposed per step)
        const u32x4* nb = reinterpret_cast<const u32x4*>(c.smem + (j0 + r + 1) * 4096 + c.voff);
        const u32x4 a0 = c.ring[RO + r][0], a1 = c.ring[RO + r][1];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            acc[0][n] = Elem<T>::mfma(a0, b[n], acc[0][n]);
            acc[1][n] = Elem<T>::mfma(a1, b[n], acc[1][n]);
            b[n] = nb[n * 64];
        }
        issue(c, RO + r, r);
        if (EK != FE_NONE) epi_tile<T, EK>(c, accY, T0 + r, fin_p);
        // pin the step's order for the scheduler (it otherwise sinks the B reads and weight
        // loads below the last MFMA): per point chunk n, MFMA, [VALU], MFMA, B read, [VALU];
        // then the 2 weight loads.  E steps spread their VALU (AGPR reads, cvt, ReLU) 4 per
        // MFMA gap (the guide: <= 5 fillers per 32x32x16 gap hide).
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

// One part: aux step (zero-initialises acc), then nk ring steps; the other set's epilogue
// (EK) in steps 0..7; a barrier before step 16 when `mid` (the late k-steps were written by
// every wave during steps 0..7).  `naux`: aux fragments of the NEXT part (loaded here).
template <typename T, int EK>
__device__ __forceinline__ void run_part(FCtx& c, f32x16 (&acc)[2][4], const f32x16 (&accY)[2][4],
                                         int nk, bool mid, FSrc naux, int fin_p) {
    const f32x16 zero = {};
    u32x4 b[4];
    if (nk > 0) read_b(c, 0, b);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        acc[0][n] = Elem<T>::mfma(c.auxn[0], c.xyzf[n], zero);
        acc[1][n] = Elem<T>::mfma(c.auxn[1], c.xyzf[n], zero);
    }
    load_aux(c, naux);
    if (nk == 0) return;
    // steps 0..7 carry the epilogue of the other set (ring slots 0..7)
    group4<T, EK, 0, 0>(c, acc, accY, b, 0, fin_p);
    group4<T, EK, 4, (FS_D == 8 ? 4 : 0)>(c, acc, accY, b, 4, fin_p);
#pragma unroll 1
    for (int j0 = 8; j0 < nk; j0 += FS_D) {
        if (mid && j0 == 16) {
            fs_bar();
            read_b(c, 16, b);                // the late positions, now written by every wave
        }
        group4<T, FE_NONE, 0, 0>(c, acc, accY, b, j0, 0);
        if (FS_D == 8) group4<T, FE_NONE, 0, 4>(c, acc, accY, b, j0 + 4, 0);
    }
}

// serial epilogue of a whole set into LDS positions kbase + 2i + s
template <typename T>
__device__ __forceinline__ void acc_to_lds(FCtx& c, const f32x16 (&acc)[2][4], int kbase) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            u32x4 f0, f1;
            acc_to_frags<T>(acc[i][n], f0, f1);
            u32x4* p = reinterpret_cast<u32x4*>(c.smem + ((kbase + 2 * i) * 4 + n) * 1024 + c.voff);
            p[0] = f0;
            p[4 * 64] = f1;
        }
}

// layer boundary after a two-part layer: park -> "early" positions 4w + 2i + s
__device__ __forceinline__ void park_to_lds(FCtx& c) {
    fs_bar();                      // every wave is done reading this layer's inputs
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            u32x4* p = reinterpret_cast<u32x4*>(c.smem + ((4 * c.wave + 2 * i) * 4 + n) * 1024 +
                                                c.voff);
            p[0] = c.park[i][n][0];
            p[4 * 64] = c.park[i][n][1];
        }
    fs_bar();                      // early k-steps visible
}

template <typename T, int S, bool POINTS>
__global__ __launch_bounds__(256, 1) void dec_fs_kernel(FArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[kFsLds];
    FCtx c;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.h = c.lane >> 5;
    c.voff = (uint32_t)c.lane * 16u;
    c.smem = smem;
    float* wl = reinterpret_cast<float*>(smem + kFsAct + kFsRed);
    float* red = reinterpret_cast<float*>(smem + kFsAct);
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
        // ---- aux B fragments: [x_hi,y_hi,z_hi,x_lo,y_lo,z_lo,1,1] of point 32n + (lane&31)
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
            c.xyzf[n] = f;
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) c.part[n] = 0.f;

        // ---- layer 0 (aux only): part 0 -> A, part 1 -> B; A parked, B deferred into L1
        run_part<T, FE_NONE>(c, accA, accB, 0, false, shp(1), 0);
        run_part<T, FE_NONE>(c, accB, accA, 0, false, bias(2), 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int n = 0; n < 4; ++n) acc_to_frags<T>(accA[i][n], c.park[i][n][0], c.park[i][n][1]);
        park_to_lds(c);

        // ---- layers 1, 2 (and 3 when 512 wide)
        constexpr int L2P = S == 256 ? 3 : 4;    // two-part layers before layer 4: 1, 2 (, 3)
        int pi = 2;
#pragma unroll 1
        for (int l = 1; l < L2P; ++l, pi += 2) {
            // the part after layer 3 (512 wide) is layer 4's: per-shape aux
            const FSrc nx = (S == 512 && l == 3) ? shp(2) : bias(pi + 2);
            run_part<T, FE_LDS>(c, accA, accB, 32, true, bias(pi + 1), 0);
            run_part<T, FE_PARK>(c, accB, accA, 32, false, nx, 0);
            park_to_lds(c);
        }
        if (S == 256) {
            // layer 3, one part of rows 64w..64w+63 -> LDS k-steps 4w..4w+3 (serial)
            run_part<T, FE_LDS>(c, accA, accB, 32, true, shp(2), 0);
            fs_bar();
            acc_to_lds<T>(c, accA, 4 * c.wave);
            fs_bar();
            // layer 4 (K = 256 in order)
            run_part<T, FE_NONE>(c, accA, accB, 16, false, shp(3), 0);
            run_part<T, FE_PARK>(c, accB, accA, 16, false, bias(pi + 3), 0);
            park_to_lds(c);
            pi += 3;
        } else {
            run_part<T, FE_LDS>(c, accA, accB, 32, true, shp(3), 0);
            run_part<T, FE_PARK>(c, accB, accA, 32, false, bias(pi + 2), 0);
            park_to_lds(c);
            pi += 2;
        }
        // ---- layers 5, 6
#pragma unroll 1
        for (int l = 5; l < 7; ++l, pi += 2) {
            run_part<T, FE_LDS>(c, accA, accB, 32, true, bias(pi + 1), 0);
            run_part<T, FE_PARK>(c, accB, accA, 32, false, bias(pi + 2), 0);
            park_to_lds(c);
        }
        // ---- layer 7: part 0 folds into the dot product during part 1; part 1 after it
        run_part<T, FE_LDS>(c, accA, accB, 32, true, bias(pi + 1), 0);
        run_part<T, FE_FIN>(c, accB, accA, 32, false, FSrc{true, c.aux_next}, 0);
#pragma unroll
        for (int t = 0; t < 8; ++t) epi_tile<T, FE_FIN>(c, accB, t, 1);
        // ---- final layer across waves: lanes l and l^32 hold the same point
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const float tot = c.part[n] + __shfl_xor(c.part[n], 32);
            if (c.h == 0) red[(c.wave * 4 + n) * 32 + c.lane] = tot;
        }
        fs_bar();
        if (c.h == 0) {
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) s += red[(w * 4 + c.wave) * 32 + c.lane];
            const int pt = local * kTilePoints + 32 * c.wave + c.lane;
            if (pt < a.npts)
                __builtin_nontemporal_store(tanhf(s + a.b_last), a.out + (size_t)shape * a.npts + pt);
        }
        c.aux_w = c.aux_next;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <typename T, int S>
void launch_fs(const FArgs& a, bool points, hipStream_t s, int grid) {
    if (points)
        hipLaunchKernelGGL((dec_fs_kernel<T, S, true>), dim3(grid), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((dec_fs_kernel<T, S, false>), dim3(grid), dim3(256), 0, s, a);
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
    a.baux = a.stream + (size_t)4 * fs_nsteps(S) * kFsStep;
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
