// The whole DDPM training step (config 2, SURVEY.md §8(a) A6/A7/A9 + AdamW) as ONE persistent
// launch: train_dag_kernel walks the job DAG that denoiser_train.hip build_dag records from the
// launch-per-GEMM step (train_dag.h).  Why: the launch-per-GEMM step spends two thirds of its
// time in per-launch fixed cost -- argument issue, ring fill, the epilogue tail of the last
// workgroups, the gap to the next launch -- and its AdamW (HBM-bound) starts only after the
// last GEMM (DESIGN.md §5, round-4 stamps).  Here a workgroup that finishes a tile takes the
// next job at once, dependent layers are handed off per 64-row band (kBand) instead of per launch, and
// the weight-gradient tiles, bias sums and AdamW tiles fill the CUs the residual chain leaves
// idle.
//
// Every job computes its outputs with the same instructions as the launch path: the GEMM tile
// runs gemm_bf16.hip's LDS-DMA ring and its LDS-transposed epilogue (gemm_tile.h), reproducing
// the k-group split of the launch's tile choice (two accumulators, summed in the same order),
// the sums are colsum_jobs_kernel's, the updates adamw_tile (adamw_tile.h).  So the step is
// BIT-IDENTICAL to ldm_denoiser_train_step + ldm_adamw_multi (tests/test_gpu_train_dag.py).
//
// Hand-offs (MI355X guide, inter-workgroup visibility, "Valid forms" table row 1: one workgroup
// per CU, hipMalloc memory): EVERY store of a handed-off byte is write-through (sc1, wt_store.h)
// and EVERY load of one is an sc1 load -- the GEMM operands' LDS-DMA, the epilogue operands, the
// bias sums' partials, AdamW's gradients -- so no release or acquire fence is needed.  A job's
// storing waves drain (s_waitcnt vmcnt(0)) and join a workgroup barrier; then ONE lane adds to
// the node's band and all-jobs counters (agent-scope atomics).  A consumer's wave 0 polls the
// counters (relaxed agent loads), drains, and the workgroup joins a barrier before any load of
// the handed-off bytes.  (The release/acquire form stays selectable for A/B:
// ldm_dev_train_dag_flags bit 7; it cost ~95 us per step, profiles/r05m.)  Every spin is
// bounded: a timeout raises the status word, every later wait gives up at once, every
// workgroup still drains its queue and exits, and the host reads the status back.
#include "train_dag.h"
#include "gemm_tile.h"
#include "adamw_tile.h"
#include "ddpm_common.h"

#include <mutex>

// DAG_EPI_WT 0 (timing-only A/B builds, results WRONG): the GEMM jobs' epilogue stores plain
// instead of write-through -- what the plain-store hand-off lever could gain at
// most, before any same-XCD / cross-XCD split of the stores
#ifndef DAG_EPI_WT
#define DAG_EPI_WT 1
#endif
namespace ldm {
namespace dag {
namespace {
using namespace gtile;

typedef const __attribute__((address_space(4))) Table KTab;
typedef const __attribute__((address_space(4))) Node KNode;
typedef const __attribute__((address_space(4))) ldm_gemm_prob_t KProb;

// One workgroup of kThreads (8 waves) per CU, 128 KiB of LDS.  GEMM jobs come in three
// configurations (Node::tile, train_dag.h), each on an LDS-DMA ring of 64-deep stages:
//   * TILE_K2: 64 x 64 in two k-groups of 4 waves (the launch path's two-k-group tile, for the
//     nodes whose launch tile summed two k-groups: k-group period kgp 1 or 2); the groups work
//     on different stages at once and group 1's sum is added to group 0's at the end;
//   * TILE_ROW: 64 x 128 (two 64-wide column halves), the other row nodes (batch rows: the
//     chain, band hand-offs);
//   * TILE_W: 128 x 128 (each wave 64 x 32), the weight-gradient products (half the operand
//     bytes per output of 64 x 64).
// Why 8 waves: a 4-wave workgroup streamed its operands at ~27-30 GB/s per CU, the launch
// path's 8-wave tile at ~47 and 12 waves per CU at ~70 (profiles/r05n): the per-CU operand
// stream scales with the waves issuing it, and fence-free hand-offs need one workgroup per CU.
constexpr int NW = kThreads / 64, kWgPerCu = 1;
// LDS per workgroup (the ring): 128 KiB; DAG_LDS_KB=160 (A/B builds) deepens every ring
#ifndef DAG_LDS_KB
#define DAG_LDS_KB 128
#endif
constexpr int kLdsBytes = DAG_LDS_KB * 1024;
template <int CFG>
struct TileCfg {
    static constexpr int BM = CFG == TILE_W ? 128 : 64;
    static constexpr int BN = CFG == TILE_K2 || CFG == TILE_K2L ? 64 : 128;
    static constexpr int KG = CFG == TILE_K2 || CFG == TILE_K2L ? 2 : 1;   // k-groups
    static constexpr int KB = CFG == TILE_K2L ? 128 : 64;      // k per ring stage
    static constexpr int WR = 2, WC = NW / KG / WR;             // waves per group: WR x WC
    static constexpr int RM = BM / WR / 32, RN = BN / WC / 32;  // 32 x 32 blocks per wave
    static constexpr int A_ELEMS = BM * KB, STAGE_ELEMS = (BM + BN) * KB;
    typedef TileSrc<BM, NW, KB> SrcA;
    typedef TileSrc<BN, NW, KB> SrcB;
    static constexpr int G = SrcA::NP + SrcB::NP;               // DMA pieces per wave per stage
    // as many stages as the LDS holds (128 KiB: TILE_K2 8, TILE_ROW 5, TILE_W / TILE_K2L 4)
    static constexpr int STAGES_LDS = kLdsBytes / (STAGE_ELEMS * 2);
    static constexpr int STAGES = STAGES_LDS < 63 / G + 1 ? STAGES_LDS : 63 / G + 1;
    static_assert(STAGES * STAGE_ELEMS * 2 <= kLdsBytes, "ring fits");
    static_assert((STAGES - 1) * G <= 63, "vmcnt immediate");
    static_assert(RM >= 1 && RN >= 1 && WC >= 1, "wave grid");
};
static_assert(NW * 4096 <= kLdsBytes, "epilogue scratch fits the ring");
static_assert(2 * 64 * (64 + 8) * 2 <= kLdsBytes, "two AdamW transpose tiles fit the ring");
static_assert(kAdamGroup % 2 == 0 && kThreads == 512, "AdamW jobs: two tiles per step");
static_assert(kBand * 66 * 2 <= kLdsBytes, "prep transpose tile fits the ring");
static_assert(kBand == 64, "row-node tiles are kBand rows");

// s_waitcnt vmcnt(y * G) lgkmcnt(0) + s_barrier for a runtime y in 0..7 (vmcnt is an immediate)
template <int G>
__device__ __forceinline__ void wait_younger(int y) {
    switch (y) {
#define LDM_WY(n)                                                                              \
    case n:                                                                                    \
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(n * G) : "memory"); \
        break;
        LDM_WY(7) LDM_WY(6) LDM_WY(5) LDM_WY(4) LDM_WY(3) LDM_WY(2) LDM_WY(1)
#undef LDM_WY
        default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

__device__ __forceinline__ unsigned* ctr(unsigned* sync, int i) {
    return sync + (kSyncCtr0 + i) * kCtrStride;
}

// Poll *w (relaxed agent-scope load) until >= target.  Run by a whole wave with wave-uniform
// arguments: every lane loads the same word and the value is made uniform (readfirstlane), so
// the loop is a scalar loop -- no lane of the wave leaves it before another, which a barrier
// later in the kernel relies on (a one-lane spin let the compiler split the scheduler loop per
// lane around the workgroup barrier: a hang).  Bounded in TIME (s_memrealtime, 100 MHz:
// `limit_us` microseconds), not in polls -- a poll's latency grows with the number of pollers
// -- and abandoned as soon as anyone raised the status word.  The sleep between polls backs off
// (64 -> 512 clocks) so that hundreds of waiting workgroups do not crowd the counters' lines.
__device__ __forceinline__ unsigned poll(const unsigned* w) {
    return __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ bool spin(const unsigned* w, unsigned target, unsigned* status,
                                     unsigned limit_us) {
    if (poll(w) >= target) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t lim = (uint64_t)limit_us * 100u;
    for (unsigned n = 1;; ++n) {
        if (n <= 4) __builtin_amdgcn_s_sleep(1);
        else __builtin_amdgcn_s_sleep(8);
        if (poll(w) >= target) return true;
        if ((n & 15) == 0) {
            if (poll(status) != 0) return false;
            if (__builtin_amdgcn_s_memrealtime() - t0 > lim) {
                if ((threadIdx.x & 63) == 0)
                    __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
    }
}

__device__ __forceinline__ unsigned short to_bf16(float x) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 v = {x, 0.f};
    return (unsigned short)(__builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2)) &
                            0xffffu);
}

// ---- GEMM tile job: tile (tm, tn) of node N's problem in configuration CFG ------------------
// The launch path's LDS-DMA ring and LDS-transposed epilogue (gemm_tile.h).  Every output
// element gets the launch path's arithmetic: per 64-deep k-step the same four 32x32x16 MFMAs in
// order, so the tile shape does not change a bit; kgp > 0 reproduces a launch that ran the
// problem on two k-groups (tile 24: 128-deep stages, kgp = 2; 64-deep, kgp = 1): k-step i
// belongs to group (i / kgp) & 1 and the result is group 0's sum + group 1's, that launch's
// summation exactly.
template <int CFG>
__device__ __forceinline__ void gemm_job(KNode& N, int job, const float* eps,
                                         unsigned short* smem, int wave, int lane, int stat) {
    typedef TileCfg<CFG> C;
    constexpr int BM = C::BM, BN = C::BN, STAGES = C::STAGES, RM = C::RM, RN = C::RN;
    constexpr int KG = C::KG, WC = C::WC, A_ELEMS = C::A_ELEMS, STAGE_ELEMS = C::STAGE_ELEMS;
    constexpr int G = C::G, KB = C::KB, KS = KB / 64;        // KS 64-deep k-steps per stage
    KProb& P = N.P;
    const int tn_n = N.tiles_n;
    const int tm = job / tn_n, tn = job - tm * tn_n;
    const int m0 = tm * BM, n0 = tn * BN;
    // (DEBUG builds) the job's tile lies inside its problem, its k-steps are the segments'
    LDM_DASSERT(tm >= 0 && m0 < P.M && n0 < P.N && P.n_seg >= 1 && N.nk % KS == 0);
    const int grp = wave / (NW / KG), wl = wave % (NW / KG);   // k-group, wave in the group
    const int wr = wl / WC, wc = wl % WC, r32 = lane & 31, h = lane >> 5;
    const int nk = N.nk / KS, kgp = N.kgp / KS;     // in ring stages (TILE_K2L: kgp 2 -> 1)
    typename C::SrcA srcA;
    typename C::SrcB srcB;
    int seg = 0, seg_left = 0, qi = 0;
    auto seat = [&](int sg) {
        LDM_DASSERT(sg < P.n_seg);
        const __attribute__((address_space(4))) ldm_gemm_seg_t& S = P.seg[sg];
        LDM_DASSERT(S.K > 0 && S.K % KB == 0);
        srcA.init(reinterpret_cast<const unsigned short*>(S.A), S.lda, m0, P.M, wave, lane);
        srcB.init(reinterpret_cast<const unsigned short*>(S.B), S.ldb, n0, P.N, wave, lane);
        seg_left = S.K / KB;
    };
    auto issue = [&]() {
        if (seg_left == 0) seat(++seg);
        unsigned short* st = smem + (qi % STAGES) * STAGE_ELEMS;
        ++qi;
        // sc1 operand loads (hand-offs); with kDbgWeightsL2 a weight copy (Node::stat) through the L2
        if (stat & 1) srcA.template issue<0>(st, wave, false);
        else srcA.template issue<16>(st, wave, false);
        if (stat & 2) srcB.template issue<0>(st + A_ELEMS, wave, false);
        else srcB.template issue<16>(st + A_ELEMS, wave, false);
        --seg_left;
    };
    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
    struct Frags {
        u32x4 a[KB / 16][RM], b[KB / 16][RN];
    };
    auto read_frags = [&](int slot, Frags& f) __attribute__((always_inline)) {
        const unsigned short* sa = smem + slot * STAGE_ELEMS;
        const unsigned short* sb = sa + A_ELEMS;
#pragma unroll
        for (int s = 0; s < KB / 16; ++s) {
#pragma unroll
            for (int i = 0; i < RM; ++i)
                f.a[s][i] = read_frag<KB>(sa, wr * (BM / 2) + i * 32 + r32, 2 * s + h);
#pragma unroll
            for (int j = 0; j < RN; ++j)
                f.b[s][j] = read_frag<KB>(sb, wc * (BN / WC) + j * 32 + r32, 2 * s + h);
        }
    };
    auto mfma = [&](const Frags& f) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < KB / 16; ++s)
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int j = 0; j < RN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, f.a[s][i]), __builtin_bit_cast(bf16x8, f.b[s][j]),
                        acc[i][j], 0, 0, 0);
    };
    // The fragment reads of a stage go BEFORE the next DMA issue, and the prologue issues only
    // the first stage(s) a step reads: an LDS read after an LDS-DMA issue makes the compiler
    // wait for every DMA in flight (vmcnt(0): it cannot tell the ring slots apart), so the
    // first read would otherwise wait for the whole prefetched ring.
    seat(0);
    if constexpr (KG == 1) {
        // stage j landed (issued so far: min(nk, j + STAGES - 1) -- the issue after step j's
        // reads refills the slot of stage j - 1, whose reads every wave finished before the
        // barrier); the workgroup's two waves per SIMD hide each other's LDS reads
        issue();
        for (int j = 0; j < nk; ++j) {
            wait_younger<G>(j == 0 ? 0 : min(STAGES - 2, nk - 1 - j));
            Frags f;
            read_frags(j % STAGES, f);
            while (qi < nk && qi < j + STAGES) issue();
            mfma(f);
        }
    } else {
        // Two k-groups: per super-step of 2 kgp stages, group g takes stages s0 + g kgp + u
        // (u < kgp) -- the two groups read and multiply different stages at once.  The issue
        // after the first reads refills the slots of the previous super-step (all its reads
        // done: the barrier).
        while (qi < nk && qi < 2 * kgp) issue();
        for (int s0 = 0; s0 < nk; s0 += 2 * kgp) {
            wait_younger<G>(qi - min(nk, s0 + 2 * kgp));
            for (int u = 0; u < kgp; ++u) {
                const int q = s0 + grp * kgp + u;
                Frags f;
                if (q < nk) read_frags(q % STAGES, f);
                if (u == 0)
                    while (qi < nk && qi < s0 + STAGES) issue();
                if (q < nk) mfma(f);
            }
        }
        // group 1's sums -> LDS (past the epilogue scratch), group 0 adds them: acc0 + acc1
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        float* red = reinterpret_cast<float*>(smem) + NW * 1024;
        const int slot = wl * (RM * RN * 16 * 64) + lane;
        if (grp == 1) {
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int j = 0; j < RN; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v) red[slot + ((i * RN + j) * 16 + v) * 64] = acc[i][j][v];
        }
        __syncthreads();
        if (grp == 1) return;      // (every later barrier of the job is inside this guard's peers)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[i][j][v] += red[slot + ((i * RN + j) * 16 + v) * 64];
    }
    if constexpr (KG == 1) __syncthreads();   // the epilogue overwrites ring slots others read
    EpiArgs e;
    e.mode = P.mode; e.Mv = P.M_valid; e.Mr = P.M; e.Nc = P.N; e.ksp = 1; e.kt = P.ct_blk;
    e.scale = P.scale;
    e.bias_p = P.bias; e.Rp = P.R;
    e.Pin = N.pin_eps ? eps : P.P_in;
    e.Rbp = reinterpret_cast<const unsigned short*>(P.Rb);
    e.Cp = P.C; e.Pp = P.P;
    e.Cbp = reinterpret_cast<unsigned short*>(P.Cb);
    e.CbTp = reinterpret_cast<unsigned short*>(P.CbT);
    e.csp = P.colsum; e.lpp = P.loss_part; e.wsp = nullptr;
    e.ldr = P.ldr; e.ldpin = P.ldp_in; e.ldrb = P.ldrb; e.ldc = P.ldc; e.ldp = P.ldp;
    e.ldcb = P.ldcb; e.ldct = P.ldct;
    const TileLoc L = {0, m0, n0, 0};
    // one inlined epilogue, looped over the wave's blocks (inlined per block it spilled); a
    // block past N (N a multiple of 64) is skipped
#pragma unroll 1
    for (int b = 0; b < RM * RN; ++b) {
        const int i = b / RN, j = b - (b / RN) * RN;
        const int nb = n0 + wc * (BN / WC) + j * 32;
        if (nb >= P.N) continue;
        f32x16 c = acc[0][0];
#pragma unroll
        for (int bb = 1; bb < RM * RN; ++bb)
            if (b == bb) c = acc[bb / RN][bb % RN];
        epi_lds_block<BM, DAG_EPI_WT != 0>(smem, 0, wl, lane, wr, h, r32, L, c, i, nb, e);
    }
}

// ---- input preparation of one kBand-row x 64-column chunk (prep_inputs_kernel<true>'s arithmetic)
// Chunk ch of a band: columns 64 ch .. of xt (ch < ceil(D / 64)) or of e (the rest); a thread
// takes 4 consecutive columns.  The rows go out as they are computed (8-byte write-through
// stores, 128-B runs per 16 lanes); the transposed copy ([c][Bp]) is staged in LDS and goes out
// 4 rows per store, 128-B runs too.  (D and TE are multiples of 4: build_dag.)
__device__ __forceinline__ void prep_job(KNode& N, int job, const float* x0, const float* eps,
                                         const int32_t* t, unsigned short* smem) {
#pragma clang fp contract(off)
    const int B = N.B, Bp = N.Bp, D = N.D, TE = N.TE;
    const int band = job / N.tiles_n, ch = job - band * N.tiles_n;
    const int nd = (D + 63) / 64;
    const bool is_x = ch < nd;
    const int c0 = (is_x ? ch : ch - nd) * 64, width = is_x ? D : TE;
    const float* sab = N.sab;
    const float* s1mab = N.s1mab;
    const float* emb = N.emb;
    unsigned short* rows_out = is_x ? N.xt_b : N.e_b;
    unsigned short* cols_out = is_x ? N.xt_T : N.e_T;
    unsigned short (*tile)[66] = reinterpret_cast<unsigned short (*)[66]>(smem);
    LDM_DASSERT(band * kBand < Bp && c0 < width);
    const uint32_t xrows = ext_bytes(Bp, width, width, 2), xcols = ext_bytes(width, Bp, Bp, 2);
    for (int i = threadIdx.x; i < kBand * 16; i += kThreads) {
        const int r = i >> 4, cl = 4 * (i & 15), c = c0 + cl, b = band * kBand + r;
        if (c >= width || b >= Bp) continue;
        const bool live = b < B;
        const int tb = live ? t[b] : 0;
        unsigned short q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float v = 0.f;
            if (live) {
                if (is_x) {
                    const float a = sab[tb] * x0[(int64_t)b * D + c + u];
                    const float e = s1mab[tb] * eps[(int64_t)b * D + c + u];
                    v = a + e;
                } else {
                    v = emb[(int64_t)tb * TE + c + u];
                }
            }
            q[u] = to_bf16(v);
            tile[r][cl + u] = q[u];
        }
        vst_at<true>(rows_out, xrows, (int64_t)b * width + c,
                  u32x2{(unsigned)q[0] | (unsigned)q[1] << 16, (unsigned)q[2] | (unsigned)q[3] << 16});
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * (kBand / 4); i += kThreads) {
        const int cc = i / (kBand / 4), r = 4 * (i % (kBand / 4));
        if (c0 + cc >= width || band * kBand + r >= Bp) continue;
        vst_at<true>(cols_out, xcols, (int64_t)(c0 + cc) * Bp + band * kBand + r,
                  u32x2{(unsigned)tile[r][cc] | (unsigned)tile[r + 1][cc] << 16,
                        (unsigned)tile[r + 2][cc] | (unsigned)tile[r + 3][cc] << 16});
    }
}

// ---- a bias gradient (or the loss) from the epilogues' partials, + that bias's AdamW --------
// colsum_jobs_kernel's sum (8 loads in flight, summed in row order), then adamw_update on the
// stored gradient, as adamw_multi_kernel does.
__device__ __forceinline__ void sum_job(KTab* tab, KNode& N, float* loss_out,
                                        const AdamHyper& hy) {
    const int rows = N.rows, len = N.len;
    const int64_t ld = N.ld;
    const float scale = N.scale;
    float* dst = N.dst ? N.dst : loss_out;
    const int ti = N.adam;
    const uint32_t xsrc = ext_bytes(rows, ld, len, 4), xdst = ext_bytes(1, len, len, 4);
    for (int c = threadIdx.x; c < len; c += kThreads) {
        const float* src = N.src;                // (uniform base for the sc1 loads)
        float s = 0.f;
        int r = 0;
        for (; r + 8 <= rows; r += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = vld_at<true, float>(src, xsrc, (int64_t)(r + u) * ld + c);
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; r < rows; ++r) s += vld_at<true, float>(src, xsrc, (int64_t)r * ld + c);
        const float g = scale * s;
        vst_at<true>(dst, xdst, c, g);
        if (ti >= 0) {
            const __attribute__((address_space(4))) ldm_adamw_tensor_t& T = tab->tensor[ti];
            float p = T.p[c], m = T.m[c], v = T.v[c];
            adamw_update(p, g, m, v, hy.decay, hy.omb1, hy.b2, hy.omb2, hy.eps, hy.step_size,
                         hy.bc2_sqrt);
            LDM_DASSERT((int64_t)T.rows * T.cols == len);
            vst_at<true>(T.p, xdst, c, p);
            vst_at<true>(T.m, xdst, c, m);
            vst_at<true>(T.v, xdst, c, v);
        }
    }
}

// Diagnostic build only (-DDAG_TRACE=1, scripts/trace_dag.py): per queue entry the workgroup that
// ran it (and its XCD) and the s_memrealtime stamps (100 MHz) of its dequeue, of its inputs being ready and of
// its completion (counters raised); per workgroup its start and exit.
#ifndef DAG_TRACE
#define DAG_TRACE 0
#endif
#if DAG_TRACE
__device__ unsigned long long g_dag_trace[kMaxEntries][4];
__device__ unsigned long long g_dag_wg[4096][2];
#endif

__global__ __launch_bounds__(kThreads, kWgPerCu) void train_dag_kernel(LaunchArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
    __shared__ int s_job;
    __shared__ int s_last;
    typedef const __attribute__((address_space(4))) LaunchArgs KLA;
    KLA* ka = (KLA*)__builtin_amdgcn_kernarg_segment_ptr();
    KTab* tab = (KTab*)ka->tab;
    unsigned* sync = ka->sync;
    unsigned* status = sync + kSyncStatus * kCtrStride;
    const unsigned limit = ka->spin_limit;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int q = blockIdx.x & (kQueues - 1);
    const float* dh = ka->d_hyper;
    const AdamHyper hy = {dh ? dh[0] : ka->hy[0], dh ? dh[1] : ka->hy[1], dh ? dh[2] : ka->hy[2],
                          dh ? dh[3] : ka->hy[3], dh ? dh[4] : ka->hy[4], dh ? dh[5] : ka->hy[5],
                          dh ? dh[6] : ka->hy[6]};
    const bool table_ok = tab->hash == ka->hash;
    if (!table_ok && threadIdx.x == 0)
        __hip_atomic_store(status, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int qlen = tab->qlen[q], qoff = tab->qoff[q];
    const uint32_t* entries = reinterpret_cast<const uint32_t*>(ka->tab + 1);
    unsigned* head = sync + (kSyncHead + q) * kCtrStride;
#if DAG_TRACE
    uint64_t tr_deq = 0, tr_rdy = 0;
    int tr_idx = 0;
    if (threadIdx.x == 0) g_dag_wg[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
#endif
    // The scheduler's control flow is wave-uniform (wave 0 runs it with all its lanes; a lane-0
    // region holds no loop), so every wave meets every workgroup barrier the same number of
    // times.
    const bool claim = (ka->dbg & kDbgClaim) != 0;
    for (;;) {
        if (wave == 0 && claim) {
            // Claim scheduler: a workgroup takes only a job whose inputs are READY -- the head of
            // its queue's chain list first, else the head of the rest -- by compare-and-swap on
            // that list's head; it never holds a job while it waits.  Progress: the earliest
            // unfinished job (node order is topological) has every input, and it heads its list.
            int e = -1;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (unsigned n = 0; table_ok; ++n) {
                bool any = false;
                for (int cls = 0; cls < 2 && e < 0; ++cls) {
                    const int li = q + cls * kQueues;
                    unsigned* hd = sync + (kSyncHead2 + li) * kCtrStride;
                    const int len = tab->qlen2[li], off = tab->qoff2[li];
                    const int h = (int)poll(hd);
                    if (h >= len) continue;
                    any = true;
                    const int ee = (int)__builtin_amdgcn_readfirstlane(entries[off + h]);
                    KNode& Nn = tab->node[ee >> 16];
                    const int jb = (ee & 0xffff) / Nn.tiles_n;
                    bool ready = true;
                    for (int d = 0; d < Nn.ndep && ready; ++d)
                        ready = poll(ctr(sync, Nn.dep_ctr[d] + (Nn.dep_band[d] ? jb : 0))) >=
                                Nn.dep_target[d];
                    if (!ready) continue;
                    unsigned won = 0;
                    if (lane == 0) {
                        unsigned expect = (unsigned)h;
                        won = __hip_atomic_compare_exchange_strong(
                                  hd, &expect, (unsigned)h + 1u, __ATOMIC_RELAXED,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 1u : 0u;
                    }
                    if (__builtin_amdgcn_readfirstlane(won)) {
                        e = ee;
#if DAG_TRACE
                        tr_idx = off + h;
#endif
                    } else {
                        cls = -1;            // lost the race: look at the chain list again
                        any = true;
                    }
                }
                if (e >= 0 || !any) break;
                __builtin_amdgcn_s_sleep(2);
                if ((n & 15) == 15) {
                    if (poll(status) != 0) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)limit * 100u) {
                        if (lane == 0)
                            __hip_atomic_store(status, 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
#if DAG_TRACE
            tr_deq = t0;
            tr_rdy = __builtin_amdgcn_s_memrealtime();
#endif
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) s_job = e;
        } else if (wave == 0) {
            unsigned jl = 0;
            if (lane == 0 && table_ok)
                jl = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int j = table_ok ? (int)__builtin_amdgcn_readfirstlane(jl) : qlen;
            int e = -1;
            if (j < qlen) {
#if DAG_TRACE
                tr_deq = __builtin_amdgcn_s_memrealtime();
                tr_idx = qoff + j;
#endif
                LDM_DASSERT(qoff + j < tab->n_entries);
                e = (int)__builtin_amdgcn_readfirstlane(entries[qoff + j]);
                LDM_DASSERT((e >> 16) < tab->n_nodes);
                // wait for the job's inputs (the consumer side of the hand-off)
                KNode& N = tab->node[e >> 16];
                const int job = e & 0xffff;
                const int band = job / N.tiles_n;      // (GEMM and PREP; others have no band)
                bool ok = true;
                LDM_DASSERT(job < N.tiles_m * N.tiles_n && N.ndep <= kMaxDeps);
                for (int d = 0; d < N.ndep && ok; ++d)
                    ok = spin(ctr(sync, N.dep_ctr[d] + (N.dep_band[d] ? band : 0)),
                              N.dep_target[d], status, limit);
                if (!ok) e = -2 - e;     // skip the job (everything drains after a timeout)
                if (ka->dbg & kDbgFences) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if DAG_TRACE
                tr_rdy = __builtin_amdgcn_s_memrealtime();
#endif
            }
            if (lane == 0) s_job = e;
        }
        __syncthreads();
        const int e = __builtin_amdgcn_readfirstlane(s_job);
        if (e == -1) break;
        if (e >= 0) {
            KNode& N = tab->node[e >> 16];
            const int job = e & 0xffff;
            const int type = N.type;
            if ((ka->dbg >> type) & 1) {
                // diagnostics: this node type's compute skipped
            } else if (type == N_GEMM) {
                const int st = (ka->dbg & kDbgWeightsL2) ? N.stat : 0;
                if (N.tile == TILE_W) gemm_job<TILE_W>(N, job, ka->eps, smem, wave, lane, st);
                else if (N.tile == TILE_K2L)
                    gemm_job<TILE_K2L>(N, job, ka->eps, smem, wave, lane, st);
                else if (N.tile == TILE_ROW)
                    gemm_job<TILE_ROW>(N, job, ka->eps, smem, wave, lane, st);
                else gemm_job<TILE_K2>(N, job, ka->eps, smem, wave, lane, st);
            } else if (type == N_PREP) {
                prep_job(N, job, ka->x0, ka->eps, ka->t, smem);
            } else if (type == N_SUM) {
                sum_job(tab, N, ka->loss_out, hy);
            } else {
                const __attribute__((address_space(4))) ldm_adamw_tensor_t& T =
                    tab->tensor[N.adam];
                // two 64 x 64 tiles at a time, one per 256-thread half, each with its own
                // transpose tile; a half without a tile still meets the tile's barrier
                const int tr = job / N.tiles_n, tg = job - tr * N.tiles_n;
                const int tl0 = tr * ((T.cols + 63) / 64) + N.col_off;
                LDM_DASSERT(tr * 64 < T.rows && N.col_off + N.nk <= (T.cols + 63) / 64);
                const int half = threadIdx.x >> 8;
                unsigned short(&sT)[64][64 + 8] =
                    *reinterpret_cast<unsigned short(*)[64][64 + 8]>(smem + half * 64 * 72);
                for (int k = 0; k < kAdamGroup; k += 2) {
                    const int tc = tg * kAdamGroup + k + half;
                    if (k) __syncthreads();      // the transpose tiles are rewritten
                    if (tc < N.nk)
                        adamw_tile<true>(T, hy, sT, tl0 + tc, threadIdx.x & 255, N.amode);
                    else if (T.p_bf16_t && N.amode != 1)
                        __syncthreads();
                }
            }
            // the producer side of the hand-off: every wave's stores drained, then one lane
            // counts the job (a node no later job waits on skips the count: the launch's end
            // publishes its stores).  (Fetching the next queue index as a job ends, and skipping
            // the drain of unwatched jobs, measured slower together with a tail reorder:
            // profiles/r05s.)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (wave == 0 && N.signal) {
                if (ka->dbg & kDbgFences) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) {
                    LDM_DASSERT(N.out_all < tab->n_counters);
                    if (N.out_band >= 0) {
                        const int band = job / N.tiles_n;
                        LDM_DASSERT(N.out_band + band < tab->n_counters);
                        __hip_atomic_fetch_add(ctr(sync, N.out_band + band), 1u,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    __hip_atomic_fetch_add(ctr(sync, N.out_all), 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }
#if DAG_TRACE
            if (threadIdx.x == 0) {
                // low word: the XCD the workgroup runs on (HW_REG_XCC_ID, read-only) << 16 | blockIdx
                const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;
                g_dag_trace[tr_idx][0] = (uint64_t)(unsigned)e << 32 | xcc << 16 | blockIdx.x;
                g_dag_trace[tr_idx][1] = tr_deq;
                g_dag_trace[tr_idx][2] = tr_rdy;
                g_dag_trace[tr_idx][3] = __builtin_amdgcn_s_memrealtime();
            }
#endif
        }
        // (s_job is rewritten only after the barrier at the top of the next round, which every
        // wave reaches after its read above)
    }
    // exit: the last workgroup out zeroes the heads, the exit counter and every job counter for
    // the next launch (the status word stays for the host to read)
    if (wave == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned nl = 0;
        if (lane == 0)
            nl = __hip_atomic_fetch_add(sync + kSyncExit * kCtrStride, 1u, __ATOMIC_ACQ_REL,
                                        __HIP_MEMORY_SCOPE_AGENT);
        const bool last = __builtin_amdgcn_readfirstlane(nl) + 1 == gridDim.x;
        if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (lane == 0) s_last = last;
    }
    __syncthreads();
#if DAG_TRACE
    if (threadIdx.x == 0) g_dag_wg[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
#endif
    // after a failure the words stay as they are for inspection; ldm_denoiser_train_status
    // zeroes them when it reads a non-zero status
    if (s_last && __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        const int nc = tab->n_counters;
        for (int i = threadIdx.x; i < kSyncCtr0 + nc; i += kThreads)
            if (i != kSyncStatus)
                __hip_atomic_store(sync + i * kCtrStride, 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace

int dag_grid(int* grid) {
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    static int g[kMaxDev], err[kMaxDev];
    int dev = 0;
    LDM_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDev, LDM_EINVAL,
                "train dag: no current device");
    std::call_once(once[dev], [&] {
        const void* k = reinterpret_cast<const void*>(&train_dag_kernel);
        hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           kLdsBytes);
        int per_cu = 0, cus = 0;
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kThreads, kLdsBytes);
        if (e == hipSuccess)
            e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess && per_cu < 1) e = hipErrorInvalidConfiguration;
        err[dev] = (int)e;
        // every workgroup resident (the deadlock-freedom argument needs it): the occupancy
        // answer x CUs, rounded down to whole queues
        g[dev] = (per_cu * cus) / kQueues * kQueues;
    });
    LDM_REQUIRE(err[dev] == 0, err[dev], "train dag: occupancy query failed: %s",
                hipGetErrorString((hipError_t)err[dev]));
    *grid = g[dev];
    return 0;
}

#if DAG_TRACE
int dag_trace(void* entries, void* wgs) {
    if (hipMemcpyFromSymbol(entries, HIP_SYMBOL(g_dag_trace), sizeof(g_dag_trace)) != hipSuccess)
        return 1;
    return hipMemcpyFromSymbol(wgs, HIP_SYMBOL(g_dag_wg), sizeof(g_dag_wg)) == hipSuccess ? 0 : 1;
}
#endif

int dag_launch(const LaunchArgs& a, int grid, hipStream_t s) {
    LDM_REQUIRE(grid >= kQueues && grid % kQueues == 0, LDM_EINVAL, "train dag: grid %d", grid);
    hipLaunchKernelGGL(train_dag_kernel, dim3(grid), dim3(kThreads), kLdsBytes, s, a);
    return launch_status("ldm_denoiser_train_step (dag)");
}

}  // namespace dag
}  // namespace ldm

#if DAG_TRACE
// diagnostic build: the last launch's trace (entries: kMaxEntries x {workgroup, dequeue, inputs
// ready, done}; workgroups: 4096 x {start, exit}), s_memrealtime ticks
extern "C" int ldm_dev_train_dag_trace(void* entries, void* wgs) {
    return ldm::dag::dag_trace(entries, wgs);
}
#endif
