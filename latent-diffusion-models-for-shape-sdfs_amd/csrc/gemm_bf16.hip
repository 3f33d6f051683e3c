// Grouped bf16 GEMM with fused training epilogues (ldm_gemm_bf16): the matrix-core engine of
// the DDPM denoiser's training step (A6/A7 at batch 1000, config 2) and of the C19 auto-decoder.
//
//   C[m][n] = sum_seg sum_{k < K_seg} A_seg[m][k] * B_seg[n][k]      (both operands bf16,
//                                                                     k contiguous: "NT")
// then one epilogue per problem (include/ldm_sdf.h LDM_GEMM_*): bias, SiLU / residual+SiLU /
// ReLU, the SiLU backward of the layer below, the eps-MSE gradient, accumulation; outputs in
// fp32, bf16 and bf16 TRANSPOSED ([n][m]), plus per-32-row column sums (bias gradients) and
// per-tile loss sums -- all written from the accumulators, so every operand the next GEMM
// needs is produced here in the layout it wants (k contiguous).  No GEMM reads a transposed
// view; no separate cast / transpose / colsum / silu-backward launch exists.
//
// Why this shape (PMC in profiles/r02a/pmc_train): the generic ldm_linear MFMA
// kernel staged fp32 operands through registers one 128-deep chunk at a time and sat at 3-4 %
// MFMA busy, 51-59 % of wave time parked on memory.  Here
//   * operands are bf16 in HBM (half the bytes) and arrive by LDS-DMA (global_load_lds, 16 B
//     per lane, no VGPR staging) into a STAGES-deep ring: STAGES-1 k-steps in flight across raw
//     s_barriers, retired by a counted vmcnt (never 0 in the steady state);
//   * the LDS image is lane-linear per DMA instruction (8 rows x 128 B) with the 16-byte chunks
//     of row r XOR-permuted by (r >> 1) & 7 on the SOURCE address, so the ds_read_b128 fragment
//     reads of 16 rows are conflict-free (guide T2, rule 21);
//   * several independent GEMMs can share one launch (problems), so small backward products
//     fill the chip together.
// Tiles: BM x BN per 4-wave workgroup (64 or 128 each), each wave (BM/2) x (BN/2) as
// RM x RN v_mfma_f32_32x32x16_bf16 tiles; k-step 64.
#include "ldm_internal.h"
#include "ddpm_common.h"

#include <algorithm>
#include <stdlib.h>
#include <string.h>

namespace ldm {
namespace {

constexpr int kBK = 64;                 // k per ring stage (128 B per operand row)

__device__ __forceinline__ unsigned pack2_bf16(float a, float b) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 v = {a, b};
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}

// Per-lane source pointers of one operand tile (ROWS x 64 k): piece i (1 KiB) = tile rows
// 8i..8i+7; the NW waves of the workgroup issue pieces w, w + NW, ...  Lane L: row 8i+L/8, LDS
// chunk L%8 <- global chunk (L%8) ^ ((row >> 1) & 7).  Rows past the end are clamped (valid
// bytes, never stored).
template <int ROWS, int NW>
struct TileSrc {
    static constexpr int NP = ROWS / (8 * NW);          // pieces per wave
    static_assert(NP >= 1 && ROWS % (8 * NW) == 0, "tile rows vs issuing waves");
    // Scalar base + 32-bit per-lane byte offsets: the DMA issues in the saddr form (one SGPR
    // pair, no 64-bit vector address math per piece), and the k step is a scalar add.
    const char* base;                                    // wave-uniform
    uint32_t voff[NP];
    __device__ __forceinline__ void init(const unsigned short* src, int64_t ld, int row0,
                                         int nrows, int wave, int lane) {
        const int rl = lane >> 3, cc = lane & 7;
        base = reinterpret_cast<const char*>(src);
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const int rr = 8 * (wave + NW * j) + rl;
            const int row = min(row0 + rr, nrows - 1);
            voff[j] = (uint32_t)(((int64_t)row * ld + 8 * (cc ^ ((rr >> 1) & 7))) * 2);
        }
    }
    // issue the next 64-k stage into LDS `dst` and step on; `again`: re-issue the previous
    // stage instead (a dummy that keeps every wave's vmcnt arithmetic uniform)
    __device__ __forceinline__ void issue(unsigned short* dst, int wave, bool again) {
        const char* b = again ? base - 2 * kBK : base;
#pragma unroll
        for (int j = 0; j < NP; ++j)
            __builtin_amdgcn_global_load_lds(
                (const void*)(b + voff[j]),
                (__attribute__((address_space(3))) void*)(dst + (wave + NW * j) * 512), 16, 0, 0);
        if (!again) base += 2 * kBK;
    }
    // register staging (RS kernels): the same pieces through VGPRs, written to the same
    // lane-linear LDS image by ds_write_b128 once the compute of the previous stage is done
    __device__ __forceinline__ void load(u32x4* r) {
#pragma unroll
        for (int j = 0; j < NP; ++j) r[j] = *reinterpret_cast<const u32x4*>(base + voff[j]);
        base += 2 * kBK;
    }
    __device__ __forceinline__ void store(unsigned short* dst, const u32x4* r, int wave,
                                          int lane) const {
#pragma unroll
        for (int j = 0; j < NP; ++j)
            *reinterpret_cast<u32x4*>(dst + (wave + NW * j) * 512 + lane * 8) = r[j];
    }
};

// The launch's argument block: the caller's problems plus the tile bookkeeping the host
// resolves once (first tile and tile counts per problem, k-steps), so a workgroup finds its
// problem with one batch of scalar loads instead of a dependent chain.
struct GemmKArgs {
    int n_prob, total;
    int first[LDM_GEMM_MAX_PROBS];      // first tile of each problem (INT_MAX when unused)
    int tiles_m[LDM_GEMM_MAX_PROBS], tiles_n[LDM_GEMM_MAX_PROBS], nk[LDM_GEMM_MAX_PROBS];
    ldm_gemm_prob_t prob[LDM_GEMM_MAX_PROBS];
};

__device__ __forceinline__ u32x4 read_frag(const unsigned short* tile, int row, int chunk) {
    const int c = chunk ^ ((row >> 1) & 7);
    return *reinterpret_cast<const u32x4*>(tile + row * kBK + 8 * c);
}

// KG = 1: 4 waves, 2 x 2 over the output tile, every wave walks every k-step.
// KG = 2: 8 waves = two k-groups of 4; group g computes the k-steps of parity g (two waves per
// SIMD working on different stages, so one's LDS reads overlap the other's MFMAs) and the two
// partial tiles are summed through LDS before the epilogue.  The ring holds STAGES / KG
// "super-stages" of KG consecutive k-steps.
template <int BM, int BN, int STAGES, int KG, bool RS>
__global__ __launch_bounds__(256 * KG) void gemm_bf16_kernel(GemmKArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
    constexpr int RM = BM / 64, RN = BN / 64, NW = 4 * KG;
    constexpr int A_ELEMS = BM * kBK, STAGE_ELEMS = (BM + BN) * kBK;
    constexpr int G = (BM + BN) / (8 * NW);           // DMA pieces per wave per stage
    constexpr int SS = STAGES / KG;                   // super-stages in the ring
    static_assert(STAGES % KG == 0 && SS >= 2, "ring of whole super-stages");
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int grp = wave >> 2, w4 = wave & 3;
    const int wr = w4 >> 1, wc = w4 & 1;

    // ---- which problem / tile: XCD-aware deal of the linear workgroup id (bijective) ------
    // The argument block is read through the kernarg segment pointer (scalar loads at a
    // runtime offset); indexing the by-value parameter by a runtime problem id would copy it
    // to scratch.
    typedef const __attribute__((address_space(4))) GemmKArgs KArgs;
    KArgs* ka = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    const int lid = blockIdx.x, tot_all = ka->total;
    int t;
    {
        const int q = tot_all / 8, r = tot_all % 8, x = lid % 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lid / 8;
    }
    const int p = (t >= ka->first[1]) + (t >= ka->first[2]) + (t >= ka->first[3]);
    const __attribute__((address_space(4))) ldm_gemm_prob_t& P = ka->prob[p];
    const int tl = t - ka->first[p], tm_n = ka->tiles_m[p], tn_n = ka->tiles_n[p];
    // tiles in groups of 4 tile-rows, column-major inside a group (L2 reuse of both panels)
    const int tg = tl / (4 * tn_n), gh = min(4, tm_n - tg * 4), in = tl - tg * 4 * tn_n;
    const int m0 = (tg * 4 + in % gh) * BM, n0 = (in / gh) * BN;
    const int nk = ka->nk[p];

    // DMA sources advance 64 k per issued stage; they are re-seated at each segment start.
    TileSrc<BM, NW> srcA;
    TileSrc<BN, NW> srcB;
    int seg = -1, seg_left = 0;
    auto issue = [&](int q) {                 // stage q (q >= nk: dummy re-issue)
        const bool again = q >= nk;
        if (!again && seg_left == 0) {
            ++seg;
            const __attribute__((address_space(4))) ldm_gemm_seg_t& S = P.seg[seg];
            srcA.init(reinterpret_cast<const unsigned short*>(S.A), S.lda, m0, P.M, wave, lane);
            srcB.init(reinterpret_cast<const unsigned short*>(S.B), S.ldb, n0, P.N, wave, lane);
            seg_left = S.K / kBK;
        }
        unsigned short* st = smem + (q % STAGES) * STAGE_ELEMS;
        srcA.issue(st, wave, again);
        srcB.issue(st + A_ELEMS, wave, again);
        if (!again) --seg_left;
    };

    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

    const int r32 = lane & 31, h = lane >> 5;
    auto compute = [&](const unsigned short* sa) {
        const unsigned short* sb = sa + A_ELEMS;
        // every fragment of the stage first (one LDS round trip), then the MFMAs
        u32x4 af[kBK / 16][RM], bf[kBK / 16][RN];
#pragma unroll
        for (int s = 0; s < kBK / 16; ++s) {
#pragma unroll
            for (int i = 0; i < RM; ++i)
                af[s][i] = read_frag(sa, wr * (BM / 2) + i * 32 + r32, 2 * s + h);
#pragma unroll
            for (int j = 0; j < RN; ++j)
                bf[s][j] = read_frag(sb, wc * (BN / 2) + j * 32 + r32, 2 * s + h);
        }
        __builtin_amdgcn_sched_barrier(0);     // keep the reads batched ahead of the MFMAs
#pragma unroll
        for (int s = 0; s < kBK / 16; ++s)
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int j = 0; j < RN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, af[s][i]),
                        __builtin_bit_cast(bf16x8, bf[s][j]), acc[i][j], 0, 0, 0);
    };

    if constexpr (RS) {
        // register-staged double buffer: stage it+1 waits in VGPRs while stage it computes
        static_assert(KG == 1 && STAGES == 2, "register staging: 2 LDS buffers, one k-group");
        u32x4 ra[TileSrc<BM, NW>::NP], rb[TileSrc<BN, NW>::NP];
        auto load = [&]() {
            if (seg_left == 0) {
                ++seg;
                const __attribute__((address_space(4))) ldm_gemm_seg_t& S = P.seg[seg];
                srcA.init(reinterpret_cast<const unsigned short*>(S.A), S.lda, m0, P.M, wave, lane);
                srcB.init(reinterpret_cast<const unsigned short*>(S.B), S.ldb, n0, P.N, wave, lane);
                seg_left = S.K / kBK;
            }
            srcA.load(ra);
            srcB.load(rb);
            --seg_left;
        };
        auto store = [&](int q) {
            unsigned short* st = smem + (q & 1) * STAGE_ELEMS;
            srcA.store(st, ra, wave, lane);
            srcB.store(st + A_ELEMS, rb, wave, lane);
        };
        load();
        store(0);
        if (nk > 1) load();
        __syncthreads();
        for (int it = 0; it < nk; ++it) {
            compute(smem + (it & 1) * STAGE_ELEMS);
            if (it + 1 < nk) {
                store(it + 1);
                if (it + 2 < nk) load();
            }
            __syncthreads();
        }
    } else {
    const int nks = (nk + KG - 1) / KG;                 // super-steps
    for (int ss = 0; ss < SS - 1; ++ss)
        if (ss < nks)
#pragma unroll
            for (int u = 0; u < KG; ++u) issue(ss * KG + u);

    for (int it = 0; it < nks; ++it) {
        // RAW: this wave's pieces of super-stage it landed (SS-2 younger ones may still fly),
        // then the barrier makes every wave's pieces visible and retires every wave's reads of
        // super-stage it-1, whose slots the issue below refills (WAR).
        if (it + SS - 2 < nks)
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((SS - 2) * KG * G) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (it + SS - 1 < nks)
#pragma unroll
            for (int u = 0; u < KG; ++u) issue((it + SS - 1) * KG + u);
        const int q = it * KG + grp;
        if (KG == 1 || q < nk) compute(smem + (q % STAGES) * STAGE_ELEMS);
    }
    }

    // ---- k-groups: sum the two partial tiles through LDS ---------------------------------
    // RM == 2: group g keeps accumulator row-block i = g and receives the other group's;
    // RM == 1: group 0 receives everything and runs the whole epilogue.
    if constexpr (KG == 2) {
        __syncthreads();                                // every DMA landed, every read done
        float* red = reinterpret_cast<float*>(smem);    // [4 waves][RN][16][64] per block
        constexpr int BLK = 4 * RN * 16 * 64;
#pragma unroll
        for (int i = 0; i < RM; ++i) {
            const int owner = RM == 2 ? i : 0;
            if (grp != owner) {
#pragma unroll
                for (int j = 0; j < RN; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v)
                        red[i * BLK + ((w4 * RN + j) * 16 + v) * 64 + lane] = acc[i][j][v];
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < RM; ++i) {
            const int owner = RM == 2 ? i : 0;
            if (grp == owner) {
#pragma unroll
                for (int j = 0; j < RN; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v)
                        acc[i][j][v] += red[i * BLK + ((w4 * RN + j) * 16 + v) * 64 + lane];
            }
        }
        if (RM == 1 && grp != 0) return;
    }

    // ---- epilogue ------------------------------------------------------------------------
    // Called once per accumulator tile with compile-time (i, j), so every acc index stays a
    // constant (a runtime-indexed accumulator array goes to scratch: guide rule 20).
    const int mode = P.mode;
    auto epi = [&](const f32x16& c, const int i, const int j) {
        const int rb = m0 + wr * (BM / 2) + i * 32;           // first row of this 32-row block
        {
            const int n = n0 + wc * (BN / 2) + j * 32 + r32;
            const bool ncol = n < P.N;
            const int nn = ncol ? n : P.N - 1;
            const float bias = P.bias ? P.bias[nn] : 0.f;
            // The fp32 operands the mode reads (R or C; P_in) are fetched for all 16 rows in
            // one batch before any use: padding rows read row 0 (a valid address) and drop the
            // value.  A load guarded per element makes hipcc branch around it and wait for each
            // one in turn (guide §5 "Projection GEMM", trap 4(c)): 16 dependent round trips.
            const float* x1 = nullptr;                           // R (or C for ACCUM)
            int64_t ld1 = 0;
            if (mode == LDM_GEMM_RESID_SILU || mode == LDM_GEMM_ADD_R ||
                (mode == LDM_GEMM_DGRAD_SILU && P.R)) {
                x1 = P.R;
                ld1 = P.ldr;
            } else if (mode == LDM_GEMM_ACCUM) {
                x1 = P.C;
                ld1 = P.ldc;
            }
            const float* x2 = (mode == LDM_GEMM_DGRAD_SILU || mode == LDM_GEMM_LOSS) ? P.P_in
                                                                                  : nullptr;
            float v1[16], v2[16];
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int b = rb + (v & 3) + 8 * (v >> 2) + 4 * h;
                const int bb = (ncol && b < P.M_valid) ? b : 0;
                v1[v] = x1 ? x1[(int64_t)bb * ld1 + nn] : 0.f;
                v2[v] = x2 ? x2[(int64_t)bb * P.ldp_in + nn] : 0.f;
            }
            float out[16];
            float lsum = 0.f;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int b = rb + (v & 3) + 8 * (v >> 2) + 4 * h;
                const bool live = ncol && b < P.M_valid;   // padding rows: nothing read / fp32 kept
                const bool inb = ncol && b < P.M;
                const int bb = live ? b : 0;
                const int64_t ic = (int64_t)bb * P.ldc + nn;
                const float r1 = live ? v1[v] : 0.f, r2 = live ? v2[v] : 0.f;
                const float pre = c[v] + bias;
                float o = pre;
                switch (mode) {
                    case LDM_GEMM_SILU:
                        if (P.P && live) P.P[(int64_t)bb * P.ldp + nn] = pre;
                        o = silu(pre);
                        break;
                    case LDM_GEMM_RESID_SILU:
                        if (P.P && live) P.P[(int64_t)bb * P.ldp + nn] = pre;
                        o = r1 + silu(pre);
                        break;
                    case LDM_GEMM_RELU: o = fmaxf(pre, 0.f); break;
                    case LDM_GEMM_ACCUM: o = r1 + pre; break;
                    case LDM_GEMM_ADD_R: o = r1 + pre; break;
                    case LDM_GEMM_DGRAD_SILU: {
                        const float dh = P.R ? r1 + pre : pre;
                        if (P.C && live) P.C[ic] = dh;
                        o = dh * silu_grad(r2);
                        break;
                    }
                    case LDM_GEMM_LOSS: {
                        const float d = pre - r2;
                        lsum += live ? d * d : 0.f;
                        o = P.scale * d;
                        break;
                    }
                    default: break;
                }
                out[v] = live ? o : 0.f;
                if (mode != LDM_GEMM_DGRAD_SILU && P.C && live) P.C[ic] = out[v];
                if (P.Cb && inb)
                    reinterpret_cast<unsigned short*>(P.Cb)[(int64_t)b * P.ldcb + nn] =
                        (unsigned short)(pack2_bf16(out[v], 0.f) & 0xffffu);
            }
            if (P.CbT && ncol) {                 // [n][b]: 4 consecutive rows per 8-byte store
                unsigned short* T = reinterpret_cast<unsigned short*>(P.CbT) + (int64_t)n * P.ldct;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int b = rb + 8 * g + 4 * h;
                    if (b < P.M) {
                        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                        const u32x2 w = {pack2_bf16(out[4 * g], out[4 * g + 1]),
                                         pack2_bf16(out[4 * g + 2], out[4 * g + 3])};
                        *reinterpret_cast<u32x2*>(T + b) = w;
                    }
                }
            }
            if (P.colsum) {                      // one partial per 32-row block and column
                float cs = 0.f;
#pragma unroll
                for (int v = 0; v < 16; ++v) cs += out[v];
                cs += __shfl_xor(cs, 32);
                if (h == 0 && ncol && rb < P.M) P.colsum[(int64_t)(rb / 32) * P.N + n] = cs;
            }
            if (mode == LDM_GEMM_LOSS && P.loss_part) {
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) lsum += __shfl_xor(lsum, o);
                if (lane == 0 && rb < P.M)
                    P.loss_part[(int64_t)(rb / 32) * ((P.N + 31) / 32) + (n0 + wc * (BN / 2) + j * 32) / 32] = lsum;
            }
        }
    };
    const bool do0 = KG == 1 || RM == 1 || grp == 0;
    const bool do1 = KG == 1 || grp == 1;
    if (do0) {
        epi(acc[0][0], 0, 0);
        if constexpr (RN > 1) epi(acc[0][RN - 1], 0, 1);
    }
    if constexpr (RM > 1) {
        if (do1) {
            epi(acc[RM - 1][0], 1, 0);
            if constexpr (RN > 1) epi(acc[RM - 1][RN - 1], 1, 1);
        }
    }
}

template <int BM, int BN, int STAGES, int KG = 1, bool RS = false>
int launch_gemm(const ldm_gemm_args_t& a, int total, hipStream_t s) {
    auto* k = &gemm_bf16_kernel<BM, BN, STAGES, KG, RS>;
    GemmKArgs ka;
    memset(&ka, 0, sizeof(ka));
    ka.n_prob = a.n_prob;
    int acc = 0;
    for (int p = 0; p < LDM_GEMM_MAX_PROBS; ++p) {
        if (p < a.n_prob) {
            const ldm_gemm_prob_t& P = a.prob[p];
            ka.prob[p] = P;
            ka.first[p] = acc;
            ka.tiles_m[p] = (P.M + BM - 1) / BM;
            ka.tiles_n[p] = (P.N + BN - 1) / BN;
            for (int g = 0; g < P.n_seg; ++g) ka.nk[p] += P.seg[g].K / kBK;
            acc += ka.tiles_m[p] * ka.tiles_n[p];
        } else {
            ka.first[p] = 0x7fffffff;
        }
    }
    ka.total = acc;
    constexpr int lds = STAGES * (BM + BN) * kBK * 2;
    static bool attr = false;
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        LDM_REQUIRE(e == hipSuccess, (int)e, "ldm_gemm_bf16: hipFuncSetAttribute: %s",
                    hipGetErrorString(e));
        attr = true;
    }
    hipLaunchKernelGGL(k, dim3(total), dim3(256 * KG), lds, s, ka);
    return launch_status("ldm_gemm_bf16");
}

}  // namespace

int gemm_tiles(const ldm_gemm_args_t& a, int bm, int bn) {
    int total = 0;
    for (int p = 0; p < a.n_prob; ++p)
        total += ((a.prob[p].M + bm - 1) / bm) * ((a.prob[p].N + bn - 1) / bn);
    return total;
}

int gemm_bf16(const ldm_gemm_args_t& a, hipStream_t s) {
    LDM_REQUIRE(a.n_prob >= 1 && a.n_prob <= LDM_GEMM_MAX_PROBS, LDM_EINVAL,
                "ldm_gemm_bf16: n_prob %d", a.n_prob);
    for (int p = 0; p < a.n_prob; ++p) {
        const ldm_gemm_prob_t& P = a.prob[p];
        LDM_REQUIRE(P.M >= 1 && P.N >= 1 && P.M_valid >= 0 && P.M_valid <= P.M &&
                        P.n_seg >= 1 && P.n_seg <= LDM_GEMM_MAX_SEGS,
                    LDM_EINVAL, "ldm_gemm_bf16: problem %d: M=%d N=%d M_valid=%d n_seg=%d", p,
                    P.M, P.N, P.M_valid, P.n_seg);
        for (int s = 0; s < P.n_seg; ++s) {
            const ldm_gemm_seg_t& S = P.seg[s];
            LDM_REQUIRE(S.A && S.B && S.K > 0 && S.K % kBK == 0, LDM_EINVAL,
                        "ldm_gemm_bf16: problem %d seg %d: K=%d must be a positive multiple of 64",
                        p, s, S.K);
            LDM_REQUIRE(LDM_ALIGNED(S.A, 16) && LDM_ALIGNED(S.B, 16) && S.lda % 8 == 0 &&
                            S.ldb % 8 == 0 && S.lda >= S.K && S.ldb >= S.K,
                        LDM_EALIGN, "ldm_gemm_bf16: problem %d seg %d: operands must be 16-B "
                        "aligned with row strides a multiple of 8 elements", p, s);
        }
        LDM_REQUIRE(P.mode >= LDM_GEMM_STORE && P.mode <= LDM_GEMM_ADD_R, LDM_EINVAL,
                    "ldm_gemm_bf16: problem %d: mode %d", p, P.mode);
        const bool needR = P.mode == LDM_GEMM_RESID_SILU || P.mode == LDM_GEMM_ADD_R;
        const bool needPin = P.mode == LDM_GEMM_DGRAD_SILU || P.mode == LDM_GEMM_LOSS;
        LDM_REQUIRE((!needR || P.R) && (!needPin || P.P_in) &&
                        (P.mode != LDM_GEMM_ACCUM || P.C),
                    LDM_EINVAL, "ldm_gemm_bf16: problem %d: mode %d operand missing", p, P.mode);
        LDM_REQUIRE(!P.CbT || (LDM_ALIGNED(P.CbT, 8) && P.ldct % 4 == 0 && P.M % 4 == 0),
                    LDM_EALIGN, "ldm_gemm_bf16: problem %d: transposed output needs 8-B "
                    "alignment, ldct and M multiples of 4", p);
    }
    // tile: 128 x 128 once the 64 x 64 grid has >= 8 workgroups per CU (C19's 1M-row
    // products); else 64 x 64 (config 2: 256-768 workgroups) on a 3-stage ring (48 KiB, so
    // three workgroups share a CU and a 768-tile launch is resident at once; ring depth
    // beyond 2 buys a lone workgroup nothing -- the per-CU DMA rate bounds it: profiles/r02b)
    // LDM_GEMM_TILE (tuning only) replaces the automatic choice
    static const int forced = [] {
        const char* e = getenv("LDM_GEMM_TILE");
        return e ? atoi(e) : 0;
    }();
    int tile = a.tile;
    if (tile == 0) {
        const int t64 = gemm_tiles(a, 64, 64);
        tile = forced ? forced : t64 >= 2048 ? 3 : 4;
    }
    switch (tile) {
        case 1: return launch_gemm<64, 64, 4>(a, gemm_tiles(a, 64, 64), s);
        case 2: return launch_gemm<128, 64, 4>(a, gemm_tiles(a, 128, 64), s);
        case 3: return launch_gemm<128, 128, 3>(a, gemm_tiles(a, 128, 128), s);
        case 4: return launch_gemm<64, 64, 3>(a, gemm_tiles(a, 64, 64), s);
        case 5: return launch_gemm<64, 64, 6, 2>(a, gemm_tiles(a, 64, 64), s);
        case 6: return launch_gemm<128, 128, 4, 2>(a, gemm_tiles(a, 128, 128), s);
        case 7: return launch_gemm<128, 64, 6, 2>(a, gemm_tiles(a, 128, 64), s);
        case 8: return launch_gemm<64, 64, 8>(a, gemm_tiles(a, 64, 64), s);
        case 9: return launch_gemm<128, 64, 5>(a, gemm_tiles(a, 128, 64), s);
        case 10: return launch_gemm<64, 64, 2>(a, gemm_tiles(a, 64, 64), s);
        case 11: return launch_gemm<64, 64, 4, 2>(a, gemm_tiles(a, 64, 64), s);
        case 12: return launch_gemm<128, 64, 3>(a, gemm_tiles(a, 128, 64), s);
        case 13: return launch_gemm<64, 64, 2, 1, true>(a, gemm_tiles(a, 64, 64), s);
        case 14: return launch_gemm<128, 128, 2, 1, true>(a, gemm_tiles(a, 128, 128), s);
        case 15: return launch_gemm<128, 64, 2, 1, true>(a, gemm_tiles(a, 128, 64), s);
        default: break;
    }
    set_error("ldm_gemm_bf16: tile %d", tile);
    return LDM_EINVAL;
}

}  // namespace ldm

extern "C" int ldm_gemm_bf16(const ldm_gemm_args_t* a, ldm_stream_t s) {
    LDM_REQUIRE(a != nullptr, LDM_EINVAL, "ldm_gemm_bf16: null args");
    return ldm::gemm_bf16(*a, (hipStream_t)s);
}
