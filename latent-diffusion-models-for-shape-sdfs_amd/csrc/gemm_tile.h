// Shared device machinery of the bf16 GEMM tiles: the operand DMA sources, fragment reads and the
// LDS-transposed fused epilogue.  Used by ldm_gemm_bf16's kernels (gemm_bf16.hip) and by the
// persistent training-step kernel (train_dag.hip), so both compute every output element with
// the same instructions (the DAG step is bit-identical to the launch-per-GEMM step).
#pragma once
#include "ldm_internal.h"
#include "ddpm_common.h"
#include "wt_store.h"

#include <type_traits>

namespace ldm {
namespace gtile {

constexpr int kBK = 64;                 // k per ring stage (128 B per operand row)

// A wave-uniform value made opaque in an SGPR (v_readfirstlane): the compiler can neither
// re-materialise it as a kernarg load nor move it to a VGPR.
template <typename T>
__device__ __forceinline__ T pin_s(T v) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
    } else {
        static_assert(sizeof(T) == 8, "pin_s: 4- or 8-byte values");
        const uint64_t u = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
        return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
    }
}

__device__ __forceinline__ unsigned pack2_bf16(float a, float b) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 v = {a, b};
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}

// Per-lane source pointers of one operand tile (ROWS x KB k): piece i (1 KiB) = tile rows
// RP*i .. RP*i+RP-1 (RP = 1024 / (2 KB): 8 rows of 128 B at KB = 64, 4 rows of 256 B at
// KB = 128); the NW waves of the workgroup issue pieces w, w + NW, ...  Lane L: row
// RP*i + L/(KB/8), LDS chunk L%(KB/8) <- global chunk (L%(KB/8)) ^ swz(row).  Rows past the end
// are clamped (valid bytes, never stored).
// swz: KB = 64 -> (row >> 1) & 7 (two 128-B rows span the 64 banks); KB = 128 -> row & 15.
// Either way the 16 rows one ds_read_b128 lane group reads hit 16 distinct 16-B bank quads.
template <int KB>
__device__ __forceinline__ int swz(int row) {
    return KB == 64 ? (row >> 1) & 7 : row & 15;
}
template <int ROWS, int NW, int KB>
struct TileSrc {
    static constexpr int CPR = KB / 8;                   // 16-B chunks per row
    static constexpr int RP = 64 / CPR;                  // rows per 1 KiB piece
    static constexpr int NP = ROWS / (RP * NW);          // pieces per wave
    static_assert(NP >= 1 && ROWS % (RP * NW) == 0, "tile rows vs issuing waves");
    // Scalar base + 32-bit per-lane byte offsets: the DMA issues in the saddr form (one SGPR
    // pair, no 64-bit vector address math per piece), and the k step is a scalar add.
    const char* base;                                    // wave-uniform
    uint32_t voff[NP];
    __device__ __forceinline__ void init(const unsigned short* src, int64_t ld, int row0,
                                         int nrows, int wave, int lane) {
        const int rl = lane / CPR, cc = lane % CPR;
        base = reinterpret_cast<const char*>(src);
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const int rr = RP * (wave + NW * j) + rl;
            const int row = min(row0 + rr, nrows - 1);
            voff[j] = (uint32_t)(((int64_t)row * ld + 8 * (cc ^ swz<KB>(rr))) * 2);
        }
    }
    // issue the next KB-deep stage into LDS `dst` and step on; `again`: re-issue the previous
    // stage instead (a dummy that keeps every wave's vmcnt arithmetic uniform)
    // CP: the load's cache policy (0; 16 = sc1, the DAG kernel's hand-off loads: wt_store.h)
    template <int CP = 0>
    __device__ __forceinline__ void issue(unsigned short* dst, int wave, bool again) {
        const char* b = again ? base - 2 * KB : base;
#pragma unroll
        for (int j = 0; j < NP; ++j)
            __builtin_amdgcn_global_load_lds(
                (const void*)(b + voff[j]),
                (__attribute__((address_space(3))) void*)(dst + (wave + NW * j) * 512), 16, 0, CP);
        if (!again) base += 2 * KB;
    }
    // register staging (RS kernels): the same pieces through VGPRs, written to the same
    // lane-linear LDS image by ds_write_b128 once the compute of the previous stage is done
    __device__ __forceinline__ void load(u32x4* r) {
#pragma unroll
        for (int j = 0; j < NP; ++j) r[j] = *reinterpret_cast<const u32x4*>(base + voff[j]);
        base += 2 * KB;
    }
    __device__ __forceinline__ void store(unsigned short* dst, const u32x4* r, int wave,
                                          int lane) const {
#pragma unroll
        for (int j = 0; j < NP; ++j)
            *reinterpret_cast<u32x4*>(dst + (wave + NW * j) * 512 + lane * 8) = r[j];
    }
};


template <int KB>
__device__ __forceinline__ u32x4 read_frag(const unsigned short* tile, int row, int chunk) {
    const int c = chunk ^ swz<KB>(row);
    return *reinterpret_cast<const u32x4*>(tile + row * KB + 8 * c);
}

// Tile t of a launch -> (problem, output origin, split-K slice).
struct TileLoc {
    int p, m0, n0, slice;
};

// One problem's epilogue fields, read once per tile into registers (see gemm_bf16.hip epi()).
struct EpiArgs {
    int mode, Mv, Mr, Nc, ksp, kt;
    float scale;
    const float* bias_p;
    const float* Rp;
    const float* Pin;
    const unsigned short* Rbp;
    float* Cp;
    float* Pp;
    unsigned short* Cbp;
    unsigned short* CbTp;
    float* csp;
    float* lpp;
    float* wsp;
    int64_t ldr, ldpin, ldrb, ldc, ldp, ldcb, ldct;
};

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// ---- LDS-transposed epilogue of one 32 x 32 accumulator block ------------------------------
// The accumulator layout gives a lane ONE column of 16 rows, so the row-major outputs would take
// one 4-byte (bf16: 2-byte) store per element: 16-52 store instructions per 32 x 32 block, and a
// one-tile-per-CU launch ends in that store-issue tail (the block GEMM: 11 us with a plain
// store, 18.7 us with RESID_SILU's four outputs, profiles/r02f).  Here the block goes through a
// per-wave 4 KiB LDS tile first (at byte offset `epi_off` of `smem`), so a lane holds 4
// consecutive columns of 4 rows: every row-major operand moves as 16-byte (bf16: 8-byte)
// vectors, 4 per output.  The element-wise arithmetic is the same expression per element as the
// accumulator-layout epilogue (gemm_bf16.hip epi()), so the outputs are bit-identical; the
// column sums and the transposed bf16 copy are formed from the results read back in
// accumulator layout, in that epilogue's order (bit-identical too).  The caller checks
// eligibility (the block lies inside N; pointers / strides allow the vectors).
// Block: rows rb = L.m0 + wr * (BM / 2) + i * 32 .. +32, columns nb .. nb + 32.
template <int BM, bool WT = false>
__device__ __forceinline__ void epi_lds_block(unsigned short* smem, int epi_off, int wave,
                                              int lane, int wr, int h, int r32, const TileLoc& L,
                                              const f32x16& c, const int i, const int nb,
                                              const EpiArgs& e) {
    const int mode = e.mode, Mv = e.Mv, Mr = e.Mr, Nc = e.Nc, ksp = e.ksp, kt = e.kt;
    const float scale = e.scale;
    const float* bias_p = e.bias_p;
    const float* Rp = e.Rp;
    const float* Pin = e.Pin;
    const unsigned short* Rbp = e.Rbp;
    float* Cp = e.Cp;
    float* Pp = e.Pp;
    unsigned short* Cbp = e.Cbp;
    unsigned short* CbTp = e.CbTp;
    float* csp = e.csp;
    float* lpp = e.lpp;
    float* wsp = e.wsp;
    const int64_t ldr = e.ldr, ldpin = e.ldpin, ldrb = e.ldrb, ldc = e.ldc, ldp = e.ldp,
                  ldcb = e.ldcb, ldct = e.ldct;

    const int rb = L.m0 + wr * (BM / 2) + i * 32;      // first row of this 32-row block
    // every operand's extent in bytes (wt_store.h): the rows the problem names, never more --
    // the write-through forms clamp their buffer resources to these, DEBUG builds trap past them.
    // Formed at each use (short live ranges: computed once up front they held 10 scalar
    // registers across the epilogue and pushed the one-launch kernel into spills)
    auto xC = [&]() { return ext_bytes(Mv, ldc, Nc, 4); };
    auto xP = [&]() { return ext_bytes(Mv, ldp, Nc, 4); };
    auto xR = [&]() { return ext_bytes(Mv, ldr, Nc, 4); };
    auto xPin = [&]() { return ext_bytes(Mv, ldpin, Nc, 4); };
    auto xRb = [&]() { return ext_bytes(Mv, ldrb, Nc, 2); };
    auto xCb = [&]() { return ext_bytes(Mr, ldcb, Nc, 2); };
    auto xCbT = [&]() {
        return kt ? ext_bytes((Mr + kt - 1) / kt, (int64_t)Nc * kt, (int64_t)Nc * kt, 2)
                  : ext_bytes(Nc, ldct, Mr, 2);
    };
    auto xcs = [&]() { return ext_bytes((Mr - 1) / 32 + 1, Nc, Nc, 4); };
    auto xlp = [&]() { return ext_bytes((Mr - 1) / 32 + 1, (Nc + 31) / 32, (Nc + 31) / 32, 4); };
    auto xws = [&]() { return ext_bytes(Mv, Nc, Nc, 4); };
    LDM_DASSERT(rb >= 0 && nb >= 0 && nb + 32 <= Nc);
    float* sc = reinterpret_cast<float*>(reinterpret_cast<char*>(smem) + epi_off) +
                wave * 1024;
    auto arow = [&](int v) { return (v & 3) + 8 * (v >> 2) + 4 * h; };   // block-local row
    const int rl = lane >> 3, cq = 4 * (lane & 7);   // row layout: rows rl + 8p, 4 columns
    asm volatile("" ::: "memory");
#pragma unroll
    for (int v = 0; v < 16; ++v) sc[arow(v) * 32 + r32] = c[v];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f32x4 cv[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
        cv[p] = *reinterpret_cast<const f32x4*>(sc + (rl + 8 * p) * 32 + cq);
    const int n4 = nb + cq;
    if (ksp > 1) {                                       // split-K: raw partial slab
        float* dst = wsp + (int64_t)L.slice * Mr * Nc;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int b = rb + rl + 8 * p;
            if (b < Mv) vst_at<WT>(dst, xws(), (int64_t)b * Nc + n4, cv[p]);
        }
        asm volatile("" ::: "memory");
        return;
    }
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    LDM_DASSERT(n4 + 4 <= Nc);
    const f32x4 bias4 = bias_p ? *reinterpret_cast<const f32x4*>(bias_p + n4) : zero4;
    auto body = [&](auto mc) {
        constexpr int MODE = decltype(mc)::value;
        constexpr bool X1R = MODE == LDM_GEMM_RESID_SILU || MODE == LDM_GEMM_ADD_R ||
                             MODE == LDM_GEMM_DGRAD_SILU;
        constexpr bool X1C = MODE == LDM_GEMM_ACCUM;
        constexpr bool X2 = MODE == LDM_GEMM_DGRAD_SILU || MODE == LDM_GEMM_LOSS;
        constexpr bool XB = MODE == LDM_GEMM_RELU_BWD;
        constexpr bool LS = MODE == LDM_GEMM_LOSS;
        f32x4 v1[4], v2[4];
        u32x2 vb[4];
        const bool has1 = X1C || (X1R && Rp != nullptr);
        const float* x1 = X1C ? Cp : Rp;
        const int64_t ld1 = X1C ? ldc : ldr;
        const uint32_t x1x = X1C ? xC() : xR();
#pragma unroll
        for (int p = 0; p < 4; ++p) {    // padding rows read row 0 (valid) and drop it
            const int b = rb + rl + 8 * p;
            const int bb = b < Mv ? b : 0;
            v1[p] = zero4;
            v2[p] = zero4;
            vb[p] = u32x2{0u, 0u};
            if constexpr (X1R || X1C) {
                if (has1)
                    v1[p] = vld_at<WT, f32x4>(x1, x1x, (int64_t)bb * ld1 + n4);
            }
            if constexpr (X2)
                v2[p] = vld_at<WT, f32x4>(Pin, xPin(), (int64_t)bb * ldpin + n4);
            if constexpr (XB)
                vb[p] = vld_at<WT, u32x2>(Rbp, xRb(), (int64_t)bb * ldrb + n4);
        }
        // one row at a time from the batched operand loads: only the values the write-back
        // needs (keep) live across rows (the 128 x 128 kernels spilled with all of it live)
        f32x4 keep[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int b = rb + rl + 8 * p;
            const bool live = b < Mv;
            f32x4 out, pre_v, dh, dd;
#pragma unroll
            for (int e = 0; e < 4; ++e) {      // epi()'s expressions, element for element
                const float pre = cv[p][e] + bias4[e];
                pre_v[e] = pre;
                float o = pre;
                dh[e] = 0.f;
                dd[e] = 0.f;
                if constexpr (MODE == LDM_GEMM_SILU) o = silu(pre);
                if constexpr (MODE == LDM_GEMM_RESID_SILU) o = v1[p][e] + silu(pre);
                if constexpr (MODE == LDM_GEMM_RELU) o = fmaxf(pre, 0.f);
                if constexpr (MODE == LDM_GEMM_ACCUM || MODE == LDM_GEMM_ADD_R)
                    o = v1[p][e] + pre;
                if constexpr (MODE == LDM_GEMM_DGRAD_SILU) {
                    dh[e] = v1[p][e] + pre;
                    o = dh[e] * silu_grad(v2[p][e]);
                }
                if constexpr (LS) {
                    dd[e] = pre - v2[p][e];
                    o = scale * dd[e];
                }
                if constexpr (MODE == LDM_GEMM_RELU_BWD) {
                    const unsigned u = (vb[p][e >> 1] >> (16 * (e & 1))) & 0xffffu;
                    o = (u != 0 && (u & 0x8000u) == 0) ? pre : 0.f;
                }
                out[e] = live ? o : 0.f;
            }
            if (Cp && live)
                vst_at<WT>(Cp, xC(), (int64_t)b * ldc + n4, MODE == LDM_GEMM_DGRAD_SILU ? dh : out);
            if constexpr (MODE == LDM_GEMM_SILU || MODE == LDM_GEMM_RESID_SILU) {
                if (Pp && live) vst_at<WT>(Pp, xP(), (int64_t)b * ldp + n4, pre_v);
            }
            if (Cbp && b < Mr)
                vst_at<WT>(Cbp, xCb(), (int64_t)b * ldcb + n4,
                        u32x2{pack2_bf16(out[0], out[1]), pack2_bf16(out[2], out[3])});
            keep[p] = LS ? dd : out;
        }
        if (CbTp || csp || (LS && lpp)) {   // back to accumulator layout through the tile
            asm volatile("" ::: "memory");
#pragma unroll
            for (int p = 0; p < 4; ++p)
                *reinterpret_cast<f32x4*>(sc + (rl + 8 * p) * 32 + cq) = keep[p];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            float oa[16];
            float lsum = 0.f;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                oa[v] = sc[arow(v) * 32 + r32];
                if constexpr (LS) {             // epi()'s loss expressions, in its order
                    const float d = oa[v];
                    const bool live = rb + arow(v) < Mv;
                    lsum += live ? d * d : 0.f;
                    oa[v] = live ? scale * d : 0.f;
                }
            }
            const int n = nb + r32;
            // [n][b] from the row-layout tile: lane = (column n, 8 consecutive rows), one
            // 16-byte store, so a store instruction writes 16 columns x 64 contiguous bytes
            // instead of 32 columns x 16 bytes (round 6).  Whole blocks whose rows keep 8-row
            // runs together and 16-byte aligned; the others take the accumulator-layout stores
            // below.  Same bf16 values, only the store grouping differs.  Launch kernels only
            // (!WT): in the one-launch step (train_dag.hip) the extra code spilled.
            const bool tvec = !WT && CbTp && !LS && rb + 32 <= Mr &&
                              (kt ? (kt & 7) == 0 : (ldct & 7) == 0) &&
                              ((uintptr_t)CbTp & 15) == 0;
            if (!WT && tvec) {
                const int q8 = (lane & 3) * 8;
#pragma unroll
                for (int half = 0; half < 2; ++half) {
                    const int nl = (lane >> 2) + 16 * half;       // block-local column
                    float t8[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) t8[e] = sc[(q8 + e) * 32 + nl];
                    const u32x4 w = {pack2_bf16(t8[0], t8[1]), pack2_bf16(t8[2], t8[3]),
                                     pack2_bf16(t8[4], t8[5]), pack2_bf16(t8[6], t8[7])};
                    const int b = rb + q8, nn = nb + nl;
                    const int64_t at = kt ? ((int64_t)(b / kt) * Nc + nn) * kt + b % kt
                                          : (int64_t)nn * ldct + b;
                    vst_at<WT>(CbTp, xCbT(), at, w);
                }
            }
            if (CbTp && !tvec) {          // [n][b]: 4 consecutive rows per 8-byte store
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int b = rb + 8 * g + 4 * h;
                    if (b < Mr) {
                        const u32x2 w = {pack2_bf16(oa[4 * g], oa[4 * g + 1]),
                                         pack2_bf16(oa[4 * g + 2], oa[4 * g + 3])};
                        const int64_t at = kt ? ((int64_t)(b / kt) * Nc + n) * kt + b % kt
                                              : (int64_t)n * ldct + b;
                        vst_at<WT>(CbTp, xCbT(), at, w);
                    }
                }
            }
            if (csp) {                    // one partial per 32-row block and column
                float cs = 0.f;
#pragma unroll
                for (int v = 0; v < 16; ++v) cs += oa[v];
                cs += __shfl_xor(cs, 32);
                if (h == 0 && rb < Mr) vst_at<WT>(csp, xcs(), (int64_t)(rb / 32) * Nc + n, cs);
            }
            if constexpr (LS) {
                if (lpp) {
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) lsum += __shfl_xor(lsum, o);
                    if (lane == 0 && rb < Mr)      // the block lies inside N here
                        vst_at<WT>(lpp, xlp(), (int64_t)(rb / 32) * ((Nc + 31) / 32) + nb / 32, lsum);
                }
            }
        }
        asm volatile("" ::: "memory");
    };
    switch (mode) {
        case LDM_GEMM_SILU: body(std::integral_constant<int, LDM_GEMM_SILU>{}); break;
        case LDM_GEMM_RESID_SILU:
            body(std::integral_constant<int, LDM_GEMM_RESID_SILU>{});
            break;
        case LDM_GEMM_RELU: body(std::integral_constant<int, LDM_GEMM_RELU>{}); break;
        case LDM_GEMM_ACCUM: body(std::integral_constant<int, LDM_GEMM_ACCUM>{}); break;
        case LDM_GEMM_DGRAD_SILU:
            body(std::integral_constant<int, LDM_GEMM_DGRAD_SILU>{});
            break;
        case LDM_GEMM_LOSS: body(std::integral_constant<int, LDM_GEMM_LOSS>{}); break;
        case LDM_GEMM_ADD_R: body(std::integral_constant<int, LDM_GEMM_ADD_R>{}); break;
        case LDM_GEMM_RELU_BWD:
            body(std::integral_constant<int, LDM_GEMM_RELU_BWD>{});
            break;
        default: body(std::integral_constant<int, LDM_GEMM_STORE>{}); break;
    }
}

}  // namespace gtile
}  // namespace ldm
