// Feature-split decoder on v_mfma_f32_16x16x32 (weight layout LDM_LAYOUT_SPLIT16):
// SURVEY.md §8(a) A1+A3.
//
// The work split of the split kernel (decoder_fs.hip), on the 16x16x32 MFMA
// shape: under load the chip holds a higher clock on it than on 32x32x16 at the same cycles
// per FLOP (MI355X_MICROARCH.md 'DVFS give-back' item 7), and the split kernel is clock-bound
// (measured 1.95 GHz in-kernel).
//   * a tile is 128 points = 8 point chunks (n) of 16, shared by the workgroup's 4 waves;
//   * wave w owns output features [128w, 128w+128) of every 512-wide layer as two parts of 64
//     rows = 4 m-chunks of 16 (layer 3 of DeepSDF: one part, rows [64w, 64w+64));
//   * one k-step is 32 input features: per k-step a wave reads 4 A fragments (its own weight
//     stream, raw buffer loads into a 2-step register ring) and 8 B fragments (LDS) for 32
//     MFMAs: each A fragment feeds 8 MFMAs, each B fragment 4;
//   * activations: 16 LDS positions of 8 KiB (8 chunks x 64 lanes x 16 B), position j = the
//     k-step ring step j reads; after a 512-wide layer, the 32 features 128w + 64u + 32q + k'
//     sit at position 8u + 2w + q (u = 0: part 0, "early"; u = 1: part 1, "late"), k' in the
//     order an accumulator pair becomes a B fragment: k = 8h + e holds feature
//     16(e >> 2) + 4h + (e & 3) (lane group h = lane >> 4 owns accumulator rows 4h..4h+3 of
//     both m-chunks 2q, 2q+1).  Position 16 holds the tile's aux B fragments.
//   * the BIAS is added in fp32 in the epilogue (an exact fp32 add before the 16-bit
//     conversion) instead of an aux MFMA step: only layers 0 and 4 keep the aux step, for xyz
//     (hi/lo) and the folded latent beta (hi/lo): A = [wx,wy,wz,wx,wy,wz,b_hi,b_lo] in k 0..7
//     of lanes 0-15, B = [x_hi,y_hi,z_hi,x_lo,y_lo,z_lo,1,1] (other lanes zero);
//   * epilogues, barriers and the layer-7 folds as in decoder_fs.hip, on 8-step windows (half a
//     part): 16 units (an m-chunk pair x a point chunk: one 16-byte LDS write) in window steps
//     0-6, the closing barrier inside step 7 after its first two point chunks.
#include "decoder_common.h"

namespace ldm {
namespace {
using namespace dec;

constexpr int kGStep = 4096;                      // one wave's 4 A fragments of one k-step
constexpr int kGPos = 8192;                       // one LDS position: 8 chunks x 1 KiB
constexpr int kGAct = 17 * kGPos;                 // 16 positions + the tile's aux B fragments
constexpr int kGRed = 4 * 8 * 64 * 4;             // final partials [wave][n][lane] fp32
constexpr int kGWl = 512 * 4;                     // final-layer weights [w][p][i][h][v]
#ifndef FS_STAMP
#define FS_STAMP 0
#endif
#ifndef G_NOEPI
#define G_NOEPI 0
#endif
// Diagnostic build only (-DFS16_DUMP=k, scripts/dump_split16.py; results are wrong): workgroup
// 0 copies LDS positions 0..15 over the output after point k of its first tile (1: layer 0
// written, 2: L1p1, 3: L2p0, 4: L2p1, 5: layer 3 written (skip 253), 6: L4p1 done) and stops.
#ifndef FS16_DUMP
#define FS16_DUMP 0
#endif
constexpr int kGStamp = FS_STAMP ? 128 * 8 : 0;
constexpr int kGLds = kGAct + kGRed + kGWl + kGStamp;
static_assert(kGLds <= 160 * 1024, "LDS");

__host__ __device__ constexpr int g_nparts(int S) { return S == 256 ? 15 : 16; }
__host__ __device__ constexpr int g_nsteps(int S) { return S == 256 ? 192 : 224; }
constexpr int kGBiasPart = 64 * 4;                // fp32 bias bytes per (wave, part)

// ------------------------------------------------------------------------------------------
// per-shape aux fragments: [B][4 waves][4 slots: L0p0, L0p1, L4p0, L4p1][4 frags][64][8].
// Lane < 16 of frag i: [wx, wy, wz, wx, wy, wz, beta_hi, beta_lo] of row 128w + 64p + 16i +
// lane; other lanes zero (they meet zero B rows: must be finite).
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void fs16_aux_pack_kernel(const float* __restrict__ beta,
                                     const float* __restrict__ wxyz, int B, T* __restrict__ aux) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;   // (b, w, slot, i, lane)
    if (id >= B * 4 * 4 * 4 * 64) return;
    const int lane = id & 63;
    const int i = (id >> 6) & 3;
    const int slot = (id >> 8) & 3;
    const int w = (id >> 10) & 3;
    const int b = id >> 12;
    const int li = slot >> 1;                 // 0: layer 0, 1: layer 4
    const int p = slot & 1;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (lane < 16) {
        const int f = 128 * w + 64 * p + 16 * i + lane;
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

struct GArgs {
    const uint8_t* stream;   // [4 waves][nsteps][4 KiB] then fp32 bias [4 waves][nparts][4 h][4 i][4 v]
    const uint8_t* aux;      // workspace [B][4 waves][4 slots][4 KiB]
    const float* w_last;     // natural order = [w][p][i][h][v]
    const float* xyz;
    float* out;
    float b_last;
    int npts, tiles_per_shape, n_tiles;
    int N, k0;
    float vs, origin;
};

// Epilogue kinds (on the OTHER accumulator set, inside an 8-step window of a later part)
//   FE_LATE: a layer's part 1 -> late positions, during the next layer's part 0;
//   FE_EARLY: a layer's part 0 -> early positions, during the same layer's part 1;
//   FE_FIN0: layer 7 part 0 -> the final dot product, during layer 7 part 1;
//   FE_FIN1: the PREVIOUS tile's layer 7 part 1 -> the dot product, during layer 1 part 0
//            (window step 6 publishes the partials, the part then stores that tile's outputs)
enum GEpi { GE_NONE = 0, GE_LATE = 1, GE_EARLY = 2, GE_FIN0 = 3, GE_FIN1 = 4 };

struct GSrc {
    uint32_t off;             // byte offset in the per-shape aux workspace
    bool none = false;
};

struct GCtx {
    int wave;
    uint32_t voff;            // lane * 16
    char* smem;
    __amdgpu_buffer_rsrc_t rw;   // the weight blob: streams then fp32 biases
    __amdgpu_buffer_rsrc_t ra;   // the per-shape aux workspace
    uint32_t s_beg, s_end, s_iss;
    uint32_t bias_w;          // this wave's bias block in rw
    uint32_t aux_w, aux_next;
    u32x4 auxn[4];            // aux A fragments of the next aux part
    u32x4 ring[2][4];         // A fragments of the next 2 k-steps
    u32x4 b[8];               // B fragments of the step about to run (rolling)
    f32x4 bias_y[4];          // bias of the set whose epilogue runs now: rows 16i + 4h + v
    f32x4 bias_n[4];          // bias of the current part
    float part[8];            // final-layer partial sums of point chunk n
    f32x4 wfin[4];            // final-layer weights of the folding window's part (m-chunk i)
    float* out;
    int npts, prev_shape, prev_local;   // prev_local < 0: no previous tile
    float b_last;
    unsigned long long* st;
    int st_i;
    bool st_on;
};

__device__ __forceinline__ void stamp(GCtx& c) {
    if (FS_STAMP) {
        if (c.st_on && (c.voff >> 4) == 0 && c.st_i < 128) c.st[c.st_i] = __builtin_readcyclecounter();
        ++c.st_i;
    }
}

__device__ __forceinline__ u32x4 bld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

__device__ __forceinline__ uint32_t opaque(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ int opaque_s(int v) {
    asm volatile("" : "+s"(v));
    return v;
}

// every LDS address is formed at its use from an opaque voff (decoder_fs.hip: hoisted constant
// addresses were spilled, and each reload waits for the whole weight ring)
__device__ __forceinline__ char* lds_at(const GCtx& c, uint32_t off) {
    return c.smem + (opaque(c.voff) + off);
}

__device__ __forceinline__ void load_aux(GCtx& c, GSrc s) {
    if (s.none) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) c.auxn[i] = bld(c.ra, c.voff + 1024u * i, s.off);
}

// this part's fp32 bias (rows 16i + 4h + v of lane group h): 4 x 16 B at h * 64
__device__ __forceinline__ void load_bias(GCtx& c, int pi) {
    const uint32_t hv = (opaque(c.voff) >> 8) << 6;
    const uint32_t so = c.bias_w + (uint32_t)pi * kGBiasPart;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        c.bias_n[i] = __builtin_bit_cast(f32x4, bld(c.rw, hv + 16u * i, so));
}

__device__ __forceinline__ void fs_bar() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void read_b(GCtx& c, int pos) {
    const u32x4* p = reinterpret_cast<const u32x4*>(lds_at(c, pos * kGPos));
#pragma unroll
    for (int n = 0; n < 8; ++n) c.b[n] = p[n * 64];
}

// k-step r (0, 1) of the stream group at c.s_iss into ring slot r
__device__ __forceinline__ void issue(GCtx& c, int r) {
    const uint32_t so = c.s_iss + (uint32_t)r * kGStep;
#pragma unroll
    for (int i = 0; i < 4; ++i) c.ring[r][i] = bld(c.rw, c.voff + 1024u * i, so);
}

__device__ __forceinline__ void next_group(GCtx& c) {
    c.s_iss += 2u * kGStep;
    if (c.s_iss == c.s_end) c.s_iss = c.s_beg;
}

__device__ __forceinline__ float relu_f(float x) {
    return __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));
}

// final-layer weights of (this wave, part p, m-chunk i, this lane group): 4 floats
__device__ __forceinline__ f32x4 wl_at(const GCtx& c, int p, int i) {
    const uint32_t h = opaque(c.voff) >> 8;
    return *reinterpret_cast<const f32x4*>(
        c.smem + kGAct + kGRed + (((c.wave * 2 + p) * 4 + i) * 4) * 16 + h * 16);
}

// One epilogue unit u = 8q + n of set Y: m-chunks 2q, 2q+1 of point chunk n (+ bias, ReLU).
// LATE / EARLY / serial: one 16-byte B fragment at position (late ? 8 : 0) + 2w + q, chunk n.
template <typename T, int EK>
__device__ __forceinline__ void epi_unit(GCtx& c, const f32x4 (&accY)[4][8],
                                         const f32x4 (&by)[4], int u, int late) {
    const int q = u >> 3, n = u & 7;
    if (EK == GE_FIN0 || EK == GE_FIN1) {
        float part = c.part[n];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const f32x4 w = c.wfin[2 * q + s];
#pragma unroll
            for (int v = 0; v < 4; ++v)
                part = fmaf(relu_f(accY[2 * q + s][n][v] + by[2 * q + s][v]), w[v], part);
        }
        c.part[n] = part;
    } else {
        const f32x4 y0 = accY[2 * q][n], y1 = accY[2 * q + 1][n];
        const f32x4 b0 = by[2 * q], b1 = by[2 * q + 1];
        u32x4 f;
        f[0] = relu2(Elem<T>::pack(y0[0] + b0[0], y0[1] + b0[1]));
        f[1] = relu2(Elem<T>::pack(y0[2] + b0[2], y0[3] + b0[3]));
        f[2] = relu2(Elem<T>::pack(y1[0] + b1[0], y1[1] + b1[1]));
        f[3] = relu2(Elem<T>::pack(y1[2] + b1[2], y1[3] + b1[3]));
        *reinterpret_cast<u32x4*>(
            lds_at(c, (uint32_t)((late + 2 * c.wave + q) * kGPos + n * 1024))) = f;
    }
}

// this lane's final partials red[wave][n][lane] (+ n * 256 B)
__device__ __forceinline__ float* red_w(const GCtx& c) {
    return reinterpret_cast<float*>(c.smem + kGAct + c.wave * 8 * 256 + opaque(c.voff) / 4);
}

// Window step k (0..7) of an epilogue: units {0,1,2} {3,4,5} {6,7} {8,9} {10,11} {12,13}
// {14,15} in steps 0-6, none in step 7 (its barrier closes the window).
template <typename T, int EK>
__device__ __forceinline__ void epi_step(GCtx& c, const f32x4 (&accY)[4][8], int k) {
    if (EK == GE_NONE || k == 7 || (G_NOEPI == 1) || (G_NOEPI == 2 && (EK == GE_FIN0 || EK == GE_FIN1)) || (G_NOEPI == 3 && !(EK == GE_FIN0 || EK == GE_FIN1)) || (G_NOEPI == 4 && EK == GE_FIN1) || (G_NOEPI == 5 && EK == GE_FIN0)) return;
    const int late = EK == GE_LATE ? 8 : 0;
    if ((EK == GE_FIN0 || EK == GE_FIN1) && k == 0) {     // the window's w_last, read once
#pragma unroll
        for (int i = 0; i < 4; ++i) c.wfin[i] = wl_at(c, EK == GE_FIN0 ? 0 : 1, i);
    }
    const int u0 = k < 2 ? 3 * k : 2 * k + 2;
    const int nu = k < 2 ? 3 : 2;
#pragma unroll
    for (int u = 0; u < 3; ++u)
        if (u < nu) epi_unit<T, EK>(c, accY, c.bias_y, u0 + u, late);
    if (EK == GE_FIN1 && k == 6) {          // the partials, published by the barrier in step 7
        float* rw = red_w(c);
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            rw[n * 64] = c.part[n];
            c.part[n] = 0.f;
        }
    }
}

__device__ __forceinline__ void valu_slot(int v) {
    if (v == 1) __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    else if (v == 2) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
    else if (v == 3) __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
}

// the 4 MFMAs of point chunk n (m-chunks 0..3); ZERO: the part's first k-step (C = 0)
template <typename T>
__device__ __forceinline__ void mfma_n(f32x4 (&acc)[4][8], const u32x4 (&a)[4], const u32x4& b,
                                       int n, bool zero) {
    const f32x4 z = {};
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][n] = Elem<T>::mfma16(a[i], b, zero ? z : acc[i][n]);
}

// Two k-steps reading positions p0, p0 + 1 (ring slots 0, 1), window steps K0, K0 + 1.  Rolling
// B fragments: chunk n of the next position is read right after chunk n's 4 MFMAs (28 MFMAs of
// cover).  The next position after step r = 1 is `np1` (the part's last group: the next part's
// first position, or 16 = the aux B fragments).  BAR = r: an LDS barrier inside step r after its
// first two point chunks, before any read of the next position.  ZERO: step 0 initialises.
template <typename T, int EK, int K0, int BAR, bool ZERO>
__device__ __forceinline__ void group2(GCtx& c, f32x4 (&acc)[4][8], const f32x4 (&accY)[4][8],
                                       int p0, int np1) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int npos = r == 1 ? np1 : p0 + 1;
        const u32x4* nb = reinterpret_cast<const u32x4*>(lds_at(c, (uint32_t)npos * kGPos));
        u32x4 a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = c.ring[r][i];
        const bool zero = ZERO && r == 0;
        const int k = K0 + r;
        // the window step's VALU spread over its MFMA gaps (~26 per unit; 2-3 units per step)
        const int V = (EK == GE_NONE || k == 7) ? 0 : (k < 2 ? 3 : 2);
        if (r == BAR) {
            mfma_n<T>(acc, a, c.b[0], 0, zero);
            mfma_n<T>(acc, a, c.b[1], 1, zero);
            __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
            __builtin_amdgcn_sched_barrier(0);
            fs_bar();
            __builtin_amdgcn_sched_barrier(0);
            c.b[0] = nb[0];
            c.b[1] = nb[64];
#pragma unroll
            for (int n = 2; n < 8; ++n) {
                mfma_n<T>(acc, a, c.b[n], n, zero);
                c.b[n] = nb[n * 64];
            }
            issue(c, r);
            epi_step<T, EK>(c, accY, k);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
            for (int n = 2; n < 8; ++n) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    valu_slot(V);
                }
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
        } else {
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                mfma_n<T>(acc, a, c.b[n], n, zero);
                c.b[n] = nb[n * 64];
            }
            issue(c, r);
            epi_step<T, EK>(c, accY, k);
            // pin the order: per point chunk, 4 x (MFMA, [VALU]), the B read
#pragma unroll
            for (int n = 0; n < 8; ++n) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    valu_slot(V);
                }
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
        }
        __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
    next_group(c);
}

// an 8-step epilogue window from position p0; BAR: its closing barrier inside step 7; np: the
// position after the window's last step
template <typename T, int EK, bool BAR, bool ZERO>
__device__ __forceinline__ void window8(GCtx& c, f32x4 (&acc)[4][8], const f32x4 (&accY)[4][8],
                                        int p0, int np) {
    group2<T, EK, 0, -1, ZERO>(c, acc, accY, p0, p0 + 2);
    group2<T, EK, 2, -1, false>(c, acc, accY, p0 + 2, p0 + 4);
    group2<T, EK, 4, -1, false>(c, acc, accY, p0 + 4, p0 + 6);
    group2<T, EK, 6, BAR ? 1 : -1, false>(c, acc, accY, p0 + 6, np);
}

// plain k-steps [j0, j1) from position pos0 as ONE runtime loop of 2-step groups, the last
// group (steps j1 - 2, j1 - 1) peeled: its next position is np, BAR: a barrier inside its
// second step; ZERO: j0 is the part's first step
template <typename T, bool BAR, bool ZERO>
__device__ __forceinline__ void plain(GCtx& c, f32x4 (&acc)[4][8], const f32x4 (&accY)[4][8],
                                      int pos0, int j0, int j1, int np) {
    int j = j0;
    if (ZERO) {            // (every plain range spans >= 4 steps)
        group2<T, GE_NONE, 0, -1, true>(c, acc, accY, pos0 + j, pos0 + j + 2);
        j += 2;
    }
#pragma unroll 1
    for (; j < j1 - 2; j += 2)
        group2<T, GE_NONE, 0, -1, false>(c, acc, accY, pos0 + j, pos0 + j + 2);
    group2<T, GE_NONE, 0, BAR ? 1 : -1, false>(c, acc, accY, pos0 + j, np);
}

// the final layer across waves and lane groups: lanes < 32 of wave w sum point chunk
// n = 2w + (lane >> 4), point c = lane & 15, over the 4 waves x 4 lane groups, + bias, tanh
__device__ __forceinline__ void fin_store(const GCtx& c, int shape, int local) {
    const int lane = (int)(opaque(c.voff) >> 4);
    if (local < 0 || lane >= 32) return;
    const int n = 2 * c.wave + (lane >> 4), pc = lane & 15;
    const float* rr = reinterpret_cast<const float*>(c.smem + kGAct + n * 256 + pc * 4);
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int h = 0; h < 4; ++h) s += rr[w * 512 + h * 16];
    const int pt = local * kTilePoints + 16 * n + pc;
    if (pt < c.npts) {
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(c.out + (size_t)shape * c.npts), (short)0, 0x7ffffff0, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, tanhf(s + c.b_last)),
                                              ro, (uint32_t)pt * 4u, 0, 2 /* nt */);
    }
}

// One part.  AUX (layers 0 and 4): first the aux step (zero-initialises acc with
// [wx,wy,wz,wx,wy,wz,b_hi,b_lo] x xyz, the xyz fragments in c.b on entry) reading the first
// position behind it -- after a barrier when `bar0` (the part follows serial LDS writes) --
// then loads the next aux part's fragments (naux).  Without AUX the first k-step zero-inits.
// A non-AUX part with naux (the one before layer 4) loads those fragments at its start.
// Every part but layer 0's loads its fp32 bias (part index pi) and hands the previous one to
// the epilogue.  EK work in window steps 0-7 (E8 false) or 8-15 (E8 true).  `mid`: the barrier
// inside step 7; `endbar`: the one inside the last step.  np: the position the last step reads
// (the next part's first, or 16 when the next part has an aux step).
template <typename T, int EK, bool E8, bool AUX>
__device__ __forceinline__ void run_part(GCtx& c, f32x4 (&acc)[4][8], const f32x4 (&accY)[4][8],
                                         int nk, int pos0, bool mid, bool endbar, GSrc naux,
                                         bool bar0, int pi, int np) {
    if (nk > 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) c.bias_y[i] = c.bias_n[i];
        load_bias(c, pi);
    }
    // the part before layer 4's first: fetch its aux fragments now (an AUX part loads its
    // successor's after its own aux step, below)
    if (!AUX) load_aux(c, naux);
    if (AUX) {
        const f32x4 z = {};
        if (nk == 0 || bar0) {
#pragma unroll
            for (int n = 0; n < 8; ++n)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i][n] = Elem<T>::mfma16(c.auxn[i], c.b[n], z);
            load_aux(c, naux);
            if (nk > 0) {
                fs_bar();
                read_b(c, pos0);
            }
        } else {
            const u32x4* p = reinterpret_cast<const u32x4*>(lds_at(c, (uint32_t)pos0 * kGPos));
#pragma unroll
            for (int n = 0; n < 8; ++n) {
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i][n] = Elem<T>::mfma16(c.auxn[i], c.b[n], z);
                c.b[n] = p[n * 64];
            }
            load_aux(c, naux);
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    } else if (bar0) {
        fs_bar();
        read_b(c, pos0);
    }
    stamp(c);
    if (nk == 0) return;
    constexpr bool Z = !AUX;
    if (!E8 && EK != GE_NONE) {          // window in steps 0-7
        const bool last8 = nk == 8;
        if (mid || (endbar && last8)) window8<T, EK, true, Z>(c, acc, accY, pos0, last8 ? np : pos0 + 8);
        else window8<T, EK, false, Z>(c, acc, accY, pos0, last8 ? np : pos0 + 8);
        if (EK == GE_FIN1) fin_store(c, c.prev_shape, c.prev_local);
        stamp(c);
        if (!last8) {
            if (endbar) plain<T, true, false>(c, acc, accY, pos0, 8, nk, np);
            else plain<T, false, false>(c, acc, accY, pos0, 8, nk, np);
        }
    } else if (E8) {                     // nk 16, mid: plain 0-7 (barrier in 7), window 8-15
        plain<T, true, Z>(c, acc, accY, pos0, 0, 8, pos0 + 8);
        stamp(c);
        if (endbar) window8<T, EK, true, false>(c, acc, accY, pos0 + 8, np);
        else window8<T, EK, false, false>(c, acc, accY, pos0 + 8, np);
    } else {                             // plain part (layer 4 part 0 at skip 253)
        plain<T, false, Z>(c, acc, accY, pos0, 0, nk, np);
        stamp(c);
    }
    stamp(c);
}

// a whole set into LDS (serial: layer 0's parts, layer 3 at skip 253) with bias `by`
template <typename T>
__device__ __forceinline__ void acc_to_lds(GCtx& c, const f32x4 (&acc)[4][8], const f32x4 (&by)[4],
                                           int late) {
#pragma unroll
    for (int u = 0; u < 16; ++u) epi_unit<T, GE_LATE>(c, acc, by, u, late);
}

template <typename T, int S, bool POINTS>
__global__ __launch_bounds__(256, 1) void dec_fs16_kernel(GArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[kGLds];
    GCtx c;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.voff = (uint32_t)(threadIdx.x & 63) * 16u;
    c.smem = smem;
    c.out = a.out;
    c.npts = a.npts;
    c.b_last = a.b_last;
    c.prev_shape = 0;
    c.prev_local = -1;
    c.st = reinterpret_cast<unsigned long long*>(smem + kGAct + kGRed + kGWl);
    c.st_i = 0;
    c.st_on = false;
    float* wl = reinterpret_cast<float*>(smem + kGAct + kGRed);
    for (int i = threadIdx.x; i < 512; i += 256) wl[i] = a.w_last[i];
    __syncthreads();
    if ((int)blockIdx.x >= a.n_tiles) return;

    constexpr int NST = g_nsteps(S);
    constexpr uint32_t kFlags = 0x00020000u;     // raw dword buffer (gfx9 word 3)
    c.rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.stream, (short)0, 0x7ffffff0, kFlags);
    c.ra = __builtin_amdgcn_make_buffer_rsrc((void*)a.aux, (short)0, 0x7ffffff0, kFlags);
    c.s_beg = (uint32_t)c.wave * NST * kGStep;
    c.s_end = c.s_beg + NST * kGStep;
    c.s_iss = c.s_beg;
    c.bias_w = (uint32_t)(4 * NST) * kGStep + (uint32_t)(c.wave * g_nparts(S)) * kGBiasPart;
    auto shape_aux = [&](int tile) -> uint32_t {
        return ((uint32_t)(tile / a.tiles_per_shape) * 4u + (uint32_t)c.wave) * 4u * kGStep;
    };
    auto shp = [&](int slot) -> GSrc { return GSrc{c.aux_w + (uint32_t)slot * kGStep}; };
    const GSrc none{0, true};
    c.aux_w = shape_aux(blockIdx.x);
#pragma unroll
    for (int r = 0; r < 2; ++r) issue(c, r);
    next_group(c);

    f32x4 accA[4][8], accB[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        c.bias_n[i] = f32x4{};
#pragma unroll
        for (int n = 0; n < 8; ++n) accB[i][n] = f32x4{};   // the first tile's GE_FIN1 input
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) c.part[n] = 0.f;
    const f32x4 nobias[4] = {};

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
        load_aux(c, shp(0));
        // ---- aux B fragments [x_hi,y_hi,z_hi,x_lo,y_lo,z_lo,1,1] of point 16n + lane (lanes
        // < 16; the others zero) at position 16; every wave writes the same bytes
        {
            const uint32_t lv = opaque(c.voff);
            const bool hi = lv >= 256u;                   // lane >= 16
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                int pt = local * kTilePoints + 16 * n + (int)((lv >> 4) & 15u);
                if (pt >= a.npts) pt = a.npts - 1;
                float x, y, z;
                if (POINTS) {
                    const float* qq = a.xyz + ((size_t)shape * a.npts + pt) * 3;
                    x = qq[0];
                    y = qq[1];
                    z = qq[2];
                } else {
                    grid_point(pt, opaque_s(a.N), a.k0, a.vs, a.origin, x, y, z);
                }
                const float xh = Elem<T>::round(x), yh = Elem<T>::round(y), zh = Elem<T>::round(z);
                u32x4 f;
                f[0] = hi ? 0u : Elem<T>::pack(xh, yh);
                f[1] = hi ? 0u : Elem<T>::pack(zh, x - xh);
                f[2] = hi ? 0u : Elem<T>::pack(y - yh, z - zh);
                f[3] = hi ? 0u : Elem<T>::pack(1.f, 1.f);
                reinterpret_cast<u32x4*>(lds_at(c, 16u * kGPos))[n * 64] = f;
            }
        }
        read_b(c, 16);

        // ---- layer 0: both parts through set A into LDS serially (set B holds the previous
        // tile's layer 7 part 1 until L1p0 folds it)
        run_part<T, GE_NONE, false, true>(c, accA, accB, 0, 0, false, false, shp(1), false, 0, 0);
        acc_to_lds<T>(c, accA, nobias, 0);
        stamp(c);
        run_part<T, GE_NONE, false, true>(c, accA, accB, 0, 0, false, false, none, false, 1, 0);
        acc_to_lds<T>(c, accA, nobias, 8);
        stamp(c);
        if (FS16_DUMP == 1) {
            fs_bar();
            if (blockIdx.x == 0) {
                const u32x4* src = reinterpret_cast<const u32x4*>(smem);
                for (int k = threadIdx.x; k < 16 * kGPos / 16; k += 256)
                    reinterpret_cast<u32x4*>(a.out)[k] = src[k];
            }
            return;
        }

        // ---- layers 1, 2 (and 3 when 512 wide)
        constexpr int L2P = S == 256 ? 3 : 4;
        int pi = 2;
        run_part<T, GE_FIN1, false, false>(c, accA, accB, 16, 0, true, false, none, true, pi, 0);
        run_part<T, GE_EARLY, true, false>(c, accB, accA, 16, 0, true, true, none, false, pi + 1, 0);

        if (FS16_DUMP == 2) {
            fs_bar();
            if (blockIdx.x == 0) {
                const u32x4* src = reinterpret_cast<const u32x4*>(smem);
                for (int k = threadIdx.x; k < 16 * kGPos / 16; k += 256)
                    reinterpret_cast<u32x4*>(a.out)[k] = src[k];
            }
            return;
        }
        pi += 2;
#pragma unroll 1
        for (int l = 2; l < L2P; ++l, pi += 2) {
            const bool to4 = S == 512 && l == 3;      // the next part is layer 4's (aux)
            run_part<T, GE_LATE, false, false>(c, accA, accB, 16, 0, true, false, none, false, pi, 0);
        if (FS16_DUMP == 3) {
            fs_bar();
            if (blockIdx.x == 0) {
                const u32x4* src = reinterpret_cast<const u32x4*>(smem);
                for (int k = threadIdx.x; k < 16 * kGPos / 16; k += 256)
                    reinterpret_cast<u32x4*>(a.out)[k] = src[k];
            }
            return;
        }
            run_part<T, GE_EARLY, true, false>(c, accB, accA, 16, 0, true, true,
                                               to4 ? shp(2) : none, false, pi + 1, to4 ? 16 : 0);
        if (FS16_DUMP == 4) {
            fs_bar();
            if (blockIdx.x == 0) {
                const u32x4* src = reinterpret_cast<const u32x4*>(smem);
                for (int k = threadIdx.x; k < 16 * kGPos / 16; k += 256)
                    reinterpret_cast<u32x4*>(a.out)[k] = src[k];
            }
            return;
        }

        }
        if (S == 256) {
            // layer 3: one part of rows 64w..64w+63 -> positions 8 + 2w + q (serial, once every
            // wave is done reading layer 3's inputs)
            run_part<T, GE_LATE, false, false>(c, accA, accB, 16, 0, true, false, shp(2), false, pi, 16);
            fs_bar();
            acc_to_lds<T>(c, accA, c.bias_n, 8);
            stamp(c);
        if (FS16_DUMP == 5) {
            fs_bar();
            if (blockIdx.x == 0) {
                const u32x4* src = reinterpret_cast<const u32x4*>(smem);
                for (int k = threadIdx.x; k < 16 * kGPos / 16; k += 256)
                    reinterpret_cast<u32x4*>(a.out)[k] = src[k];
            }
            return;
        }

            // layer 4 (K = 256, positions 8..15); part 0 -> early positions during part 1
            run_part<T, GE_NONE, false, true>(c, accA, accB, 8, 8, false, false, shp(3), true, pi + 1, 16);
            run_part<T, GE_EARLY, false, true>(c, accB, accA, 8, 8, false, true, none, false, pi + 2, 0);
        if (FS16_DUMP == 6) {
            fs_bar();
            if (blockIdx.x == 0) {
                const u32x4* src = reinterpret_cast<const u32x4*>(smem);
                for (int k = threadIdx.x; k < 16 * kGPos / 16; k += 256)
                    reinterpret_cast<u32x4*>(a.out)[k] = src[k];
            }
            return;
        }

            pi += 3;
        } else {
            run_part<T, GE_LATE, false, true>(c, accA, accB, 16, 0, true, false, shp(3), false, pi, 16);
            run_part<T, GE_EARLY, true, true>(c, accB, accA, 16, 0, true, true, none, false, pi + 1, 0);
            pi += 2;
        }
        // ---- layers 5, 6
#pragma unroll 1
        for (int l = 5; l < 7; ++l, pi += 2) {
            run_part<T, GE_LATE, false, false>(c, accA, accB, 16, 0, true, false, none, false, pi, 0);
            run_part<T, GE_EARLY, true, false>(c, accB, accA, 16, 0, true, true, none, false, pi + 1, 0);
        }
        // ---- layer 7: part 0 folds into the dot product during part 1, part 1 during the
        // next tile's L1p0 (its end barrier lets the next tile overwrite every position)
        run_part<T, GE_LATE, false, false>(c, accA, accB, 16, 0, true, false, none, false, pi, 0);
        run_part<T, GE_FIN0, false, false>(c, accB, accA, 16, 0, false, true, none, false, pi + 1, 16);
        c.prev_shape = shape;
        c.prev_local = local;
        c.aux_w = c.aux_next;
    }
    // the last tile's layer 7 part 1, in the GE_FIN1 unit order (a point's value must not depend
    // on whether its tile was its workgroup's last)
#pragma unroll
    for (int i = 0; i < 4; ++i) c.wfin[i] = wl_at(c, 1, i);
#pragma unroll
    for (int u = 0; u < 16; ++u) epi_unit<T, GE_FIN1>(c, accB, c.bias_n, u, 0);
    {
        float* rw = red_w(c);
#pragma unroll
        for (int n = 0; n < 8; ++n) rw[n * 64] = c.part[n];
    }
    fs_bar();
    fin_store(c, c.prev_shape, c.prev_local);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (FS_STAMP && c.wave == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        for (int k = threadIdx.x & 63; k < 128; k += 64)
            reinterpret_cast<unsigned long long*>(a.out)[(size_t)blockIdx.x * 128 + k] = c.st[k];
    }
}

template <typename T, int S>
void launch_fs16(const GArgs& a, bool points, hipStream_t s, int grid) {
    if (points)
        hipLaunchKernelGGL((dec_fs16_kernel<T, S, true>), dim3(grid), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((dec_fs16_kernel<T, S, false>), dim3(grid), dim3(256), 0, s, a);
}

}  // namespace

size_t decoder_fs16_aux_bytes(int B) { return (size_t)B * 4 * 4 * kGStep; }

int decoder_fs16_n_stages(int skip_width) { return g_nsteps(skip_width == 253 ? 256 : 512); }

int decoder_fs16_fwd(const ldm_decoder_t* w, const float* beta, const float* xyz, int B, int npts,
                     int N, int k0, float vs, float origin, float* out, void* ws, size_t ws_bytes,
                     hipStream_t s, int num_cus) {
    const int S = w->skip_width == 253 ? 256 : 512;
    LDM_REQUIRE(w->n_stages == g_nsteps(S), LDM_EINVAL, "split16 layout: n_stages %d != %d",
                w->n_stages, g_nsteps(S));
    LDM_REQUIRE(ws != nullptr && ws_bytes >= decoder_fs16_aux_bytes(B) && LDM_ALIGNED(ws, 16),
                LDM_ENOSPC, "workspace too small: need %zu bytes, got %zu",
                decoder_fs16_aux_bytes(B), ws_bytes);
    LDM_REQUIRE(decoder_fs16_aux_bytes(B) < 0x7ffffff0u, LDM_EINVAL,
                "split16 layout: %d shapes exceed the aux buffer range", B);
    {
        const int n = B * 4 * 4 * 4 * 64;
        if (w->dtype == LDM_BF16)
            hipLaunchKernelGGL(fs16_aux_pack_kernel<__bf16>, dim3((n + 255) / 256), dim3(256), 0,
                               s, beta, w->wxyz, B, (__bf16*)ws);
        else
            hipLaunchKernelGGL(fs16_aux_pack_kernel<_Float16>, dim3((n + 255) / 256), dim3(256),
                               0, s, beta, w->wxyz, B, (_Float16*)ws);
        if (int e = launch_status("fs16_aux_pack")) return e;
    }
    GArgs a;
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
        if (S == 256) launch_fs16<__bf16, 256>(a, points, s, grid);
        else launch_fs16<__bf16, 512>(a, points, s, grid);
    } else {
        if (S == 256) launch_fs16<_Float16, 256>(a, points, s, grid);
        else launch_fs16<_Float16, 512>(a, points, s, grid);
    }
    return launch_status("ldm_decoder_fwd(split16)");
}

}  // namespace ldm
