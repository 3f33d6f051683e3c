// A6/A7/A9 training of the MLP denoiser through the C ABI (SURVEY.md §8(b):
// ldm_denoiser_fwd / ldm_denoiser_bwd / ldm_q_sample_loss, plus the fused
// ldm_denoiser_train_step and the multi-tensor ldm_adamw_multi).
//
// Every matrix product is one problem of ldm_gemm_bf16 (gemm_bf16.hip) whose epilogue writes
// the operands the NEXT products need, in bf16, in both layouts ([b][f] for products over f,
// [f][b] for the weight gradients, whose sum runs over the batch b).  So the backward of a
// residual block is two launches' worth of problems and no elementwise pass:
//   * G W  with epilogue DGRAD_SILU:  dh_k = dh_{k+1} + g_k W_k  (fp32, the residual stream)
//                                      g_{k-1} = dh_k * SiLU'(a_{k-1})  (bf16 [b][f] + [f][b])
//                                      + the column sums of g_{k-1} (the bias gradient)
//   * G^T [h || temb]  as two problems (dW_k, dU_k) in the same launch;
//   * dtemb = sum_k g_k U_k as ONE product over 4 K-segments (one per block) at the end;
// and the eps-MSE gradient is the out-projection's epilogue (LOSS) in the fused step.
// Launches per fused step: prep 1, forward 3 + n_blocks, backward 4 + n_blocks, finalize 1.
//
// Rows are padded to Bp = ceil(B/64)*64; padding rows of every bf16 operand are written as 0
// by the producing epilogue (M_valid = B), so K = Bp weight-gradient products see zeros there.
#include "ldm_internal.h"
#include "ddpm_common.h"
#include "adamw_tile.h"
#include "train_dag.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace ldm {

int gemm_bf16(const ldm_gemm_args_t& a, hipStream_t s);
int gemm_tile_choice(const ldm_gemm_args_t& a);
int gemm_tile_kgroup_period(int tile);

namespace {

typedef unsigned short bf16_t;

__device__ __forceinline__ bf16_t to_bf16(float x) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 v = {x, 0.f};
    return (bf16_t)(__builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2)) & 0xffffu);
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// ---- workspace layout ----------------------------------------------------------------------
struct TrainWs {
    int B, Bp, D, H, TE, nb;
    bf16_t *xt_b, *xt_T, *e_b, *e_T, *u_b, *u_T, *temb_b, *temb_T;
    bf16_t *h_b[LDM_MAX_BLOCKS + 1], *h_T[LDM_MAX_BLOCKS + 1];
    bf16_t *g_b[LDM_MAX_BLOCKS], *g_T[LDM_MAX_BLOCKS];
    bf16_t *go_b, *go_T, *dtemb_b, *dtemb_T, *gt_T, *dh0_b, *dh0_T;
    float *a_t, *h_f[LDM_MAX_BLOCKS], *a_f[LDM_MAX_BLOCKS], *dh[2];
    float *p_bt1, *p_bt2, *p_bin, *p_bblk[LDM_MAX_BLOCKS], *p_bout, *loss_part;
    dag::Table* dag_table;      // the persistent step's job table (train_dag.h) and sync words
    unsigned* dag_sync;
    size_t bytes;
};

TrainWs layout(const ldm_denoiser_t* w, int B, void* base) {
    TrainWs L = {};
    L.B = B;
    L.Bp = (B + 63) / 64 * 64;
    L.D = w->D; L.H = w->H; L.TE = w->TE; L.nb = w->n_blocks;
    size_t off = 0;
    char* b = reinterpret_cast<char*>(base);
    auto take = [&](size_t bytes) -> void* {
        void* p = b ? b + off : nullptr;
        off = align256(off + bytes);
        return p;
    };
    const size_t Bp = L.Bp, D = L.D, H = L.H, TE = L.TE;
    auto bf = [&](size_t n) { return reinterpret_cast<bf16_t*>(take(n * 2)); };
    auto f32 = [&](size_t n) { return reinterpret_cast<float*>(take(n * 4)); };
    L.xt_b = bf(Bp * D); L.xt_T = bf(D * Bp);
    L.e_b = bf(Bp * TE); L.e_T = bf(TE * Bp);
    L.u_b = bf(Bp * H); L.u_T = bf(H * Bp);
    L.temb_b = bf(Bp * H); L.temb_T = bf(H * Bp);
    for (int k = 0; k <= L.nb; ++k) { L.h_b[k] = bf(Bp * H); L.h_T[k] = bf(H * Bp); }
    for (int k = 0; k < L.nb; ++k) { L.g_b[k] = bf(Bp * H); L.g_T[k] = bf(H * Bp); }
    L.go_b = bf(Bp * D); L.go_T = bf(D * Bp);
    L.dtemb_b = bf(Bp * H); L.dtemb_T = bf(H * Bp);
    L.gt_T = bf(H * Bp);
    L.dh0_b = bf(Bp * H); L.dh0_T = bf(H * Bp);
    L.a_t = f32(Bp * H);
    for (int k = 0; k < L.nb; ++k) { L.h_f[k] = f32(Bp * H); L.a_f[k] = f32(Bp * H); }
    L.dh[0] = f32(Bp * H); L.dh[1] = f32(Bp * H);
    const size_t R = Bp / 32;
    L.p_bt1 = f32(R * H); L.p_bt2 = f32(R * H); L.p_bin = f32(R * H);
    for (int k = 0; k < L.nb; ++k) L.p_bblk[k] = f32(R * H);
    L.p_bout = f32(R * D);
    L.loss_part = f32(R * (D / 32));
    L.dag_table = reinterpret_cast<dag::Table*>(take(dag::table_bytes()));
    L.dag_sync = reinterpret_cast<unsigned*>(take(dag::sync_bytes(dag::kMaxCounters)));
    L.bytes = off;
    return L;
}

// ---- elementwise kernels -------------------------------------------------------------------
// Training inputs as bf16 GEMM operands in both layouts, rows b >= B zero:
//   xt = sqrt(abar[t]) x0 + sqrt(1-abar[t]) eps (q_sample, QS) or the given x (!QS);
//   e  = emb[t].
// One thread per (b, column) of [Bp][D + TE].
template <bool QS>
__global__ __launch_bounds__(256) void prep_inputs_kernel(
    const float* __restrict__ x0, const float* __restrict__ eps, const int32_t* __restrict__ t,
    const float* __restrict__ sab, const float* __restrict__ s1mab,
    const float* __restrict__ emb, int B, int Bp, int D, int TE, bf16_t* xt_b, bf16_t* xt_T,
    bf16_t* e_b, bf16_t* e_T) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int W = D + TE;
    if (i >= (int64_t)Bp * W) return;
    const int b = (int)(i / W), c = (int)(i - (int64_t)b * W);
    const bool live = b < B;
    const int tb = live ? t[b] : 0;
    if (c < D) {
        float v = 0.f;
        if (live) {
            if constexpr (QS) {
                const float a = sab[tb] * x0[(int64_t)b * D + c];
                const float e = s1mab[tb] * eps[(int64_t)b * D + c];
                v = a + e;
            } else {
                v = x0[(int64_t)b * D + c];
            }
        }
        const bf16_t q = to_bf16(v);
        xt_b[(int64_t)b * D + c] = q;
        xt_T[(int64_t)c * Bp + b] = q;
    } else {
        const int cc = c - D;
        const bf16_t q = to_bf16(live ? emb[(int64_t)tb * TE + cc] : 0.f);
        e_b[(int64_t)b * TE + cc] = q;
        e_T[(int64_t)cc * Bp + b] = q;
    }
}

// deps fp32 [B][D] -> bf16 [Bp][D] and [D][Bp], rows b >= B zero (ldm_denoiser_bwd).
__global__ __launch_bounds__(256) void prep_grad_kernel(const float* __restrict__ g, int B,
                                                        int Bp, int D, bf16_t* gb, bf16_t* gT) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)Bp * D) return;
    const int b = (int)(i / D), c = (int)(i - (int64_t)b * D);
    const bf16_t q = to_bf16(b < B ? g[(int64_t)b * D + c] : 0.f);
    gb[i] = q;
    gT[(int64_t)c * Bp + b] = q;
}

// Fixed-order column sums: dst[c] = scale * sum_{r < rows} src[r * ld + c] for c < len, one
// job per blockIdx.y (bias gradients from the epilogues' 32-row partials, the loss).
struct SumJob { const float* src; float* dst; int rows, len, ld; float scale; };
constexpr int kMaxSumJobs = 2 * LDM_MAX_BLOCKS + 8;
struct SumJobs { SumJob j[kMaxSumJobs]; int n; };

__global__ __launch_bounds__(256) void colsum_jobs_kernel(SumJobs jobs) {
    typedef const __attribute__((address_space(4))) SumJobs KJ;
    KJ* kj = (KJ*)__builtin_amdgcn_kernarg_segment_ptr();
    const int jb = blockIdx.y;
    if (jb >= kj->n) return;
    const __attribute__((address_space(4))) SumJob& J = kj->j[jb];
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= J.len) return;
    // 8 loads in flight per round, summed in row order (deterministic)
    const float* src = J.src + c;
    const int64_t ld = J.ld;
    float s = 0.f;
    int r = 0;
    for (; r + 8 <= J.rows; r += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(r + u) * ld];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; r < J.rows; ++r) s += src[(int64_t)r * ld];
    J.dst[c] = J.scale * s;
}

int run_sums(const SumJobs& jobs, int max_len, hipStream_t s) {
    if (jobs.n == 0) return 0;
    hipLaunchKernelGGL(colsum_jobs_kernel, dim3((max_len + 255) / 256, jobs.n), dim3(256), 0, s,
                       jobs);
    return launch_status("denoiser finalize");
}

// ---- GEMM problem builders -----------------------------------------------------------------
ldm_gemm_prob_t prob(int M, int N, int M_valid) {
    ldm_gemm_prob_t p;
    memset(&p, 0, sizeof(p));
    p.M = M; p.N = N; p.M_valid = M_valid; p.mode = LDM_GEMM_STORE; p.scale = 1.f;
    return p;
}
void seg(ldm_gemm_prob_t& p, const void* A, int64_t lda, const void* B, int64_t ldb, int K) {
    ldm_gemm_seg_t& s = p.seg[p.n_seg++];
    s.A = A; s.B = B; s.lda = lda; s.ldb = ldb; s.K = K;
}
// With a recorder the launches are not made but recorded, one group per launch (build_dag).
struct Recorder {
    std::vector<ldm_gemm_args_t> launches;
};
int launch(std::initializer_list<ldm_gemm_prob_t> ps, hipStream_t s, Recorder* rec = nullptr) {
    ldm_gemm_args_t a;
    memset(&a, 0, sizeof(a));
    for (const auto& p : ps) a.prob[a.n_prob++] = p;
    if (rec) {
        rec->launches.push_back(a);
        return 0;
    }
    return gemm_bf16(a, s);
}

int check_desc(const ldm_denoiser_t* w, int B, bool bwd) {
    LDM_REQUIRE(w && w->abi_version == LDM_ABI_VERSION, LDM_EINVAL,
                "denoiser training: bad descriptor / ABI version");
    LDM_REQUIRE(w->dtype == LDM_BF16, LDM_ENOSYS,
                "denoiser training through the C ABI runs bf16 weights (got dtype %d); the exact "
                "fp32 path is ldm_linear", w->dtype);
    LDM_REQUIRE(B >= 1 && w->D % 64 == 0 && w->H % 64 == 0 && w->TE % 64 == 0 &&
                    w->n_blocks >= 1 && w->n_blocks <= LDM_MAX_BLOCKS,
                LDM_EINVAL, "denoiser training: D, H, TE must be multiples of 64 (D=%d H=%d "
                "TE=%d), 1..%d blocks, B >= 1", w->D, w->H, w->TE, LDM_MAX_BLOCKS);
    LDM_REQUIRE(w->w_in && w->w_t1 && w->w_t2 && w->w_out && w->emb_table && w->b_in &&
                    w->b_t1 && w->b_t2 && w->b_out,
                LDM_EINVAL, "denoiser training: weight pointer missing");
    for (int k = 0; k < w->n_blocks; ++k)
        LDM_REQUIRE(w->w_blk[k] && w->b_blk[k] && (!bwd || w->wt_blk[k]), LDM_EINVAL,
                    "denoiser training: block %d weights missing", k);
    LDM_REQUIRE(!bwd || (w->wt_t2 && w->wt_out), LDM_EINVAL,
                "denoiser backward: transposed bf16 weights (wt_t2, wt_blk, wt_out) missing");
    return 0;
}

// Forward GEMMs; out-projection: LOSS against `eps_target` (fused step) or STORE to eps_out.
int forward(const ldm_denoiser_t* w, const TrainWs& L, const float* eps_target,
            float* eps_out, float loss_scale, hipStream_t s, Recorder* rec = nullptr) {
    const int Bp = L.Bp, B = L.B, D = L.D, H = L.H, TE = L.TE;
    ldm_gemm_prob_t f1 = prob(Bp, H, B);                         // u = SiLU(Wt1 e + bt1)
    seg(f1, L.e_b, TE, w->w_t1, TE, TE);
    f1.mode = LDM_GEMM_SILU; f1.bias = w->b_t1;
    f1.P = L.a_t; f1.ldp = H; f1.Cb = L.u_b; f1.ldcb = H; f1.CbT = L.u_T; f1.ldct = Bp;
    ldm_gemm_prob_t f3 = prob(Bp, H, B);                         // h0 = Win xt + bin
    seg(f3, L.xt_b, D, w->w_in, D, D);
    f3.bias = w->b_in;
    f3.C = L.h_f[0]; f3.ldc = H; f3.Cb = L.h_b[0]; f3.ldcb = H; f3.CbT = L.h_T[0]; f3.ldct = Bp;
    LDM_TRY(launch({f1, f3}, s, rec));
    ldm_gemm_prob_t f2 = prob(Bp, H, B);                         // temb = Wt2 u + bt2
    seg(f2, L.u_b, H, w->w_t2, H, H);
    f2.bias = w->b_t2;
    f2.Cb = L.temb_b; f2.ldcb = H; f2.CbT = L.temb_T; f2.ldct = Bp;
    LDM_TRY(launch({f2}, s, rec));
    const bf16_t* const* Wb = reinterpret_cast<const bf16_t* const*>(w->w_blk);
    for (int k = 0; k < L.nb; ++k) {                              // h <- h + SiLU([h||temb] Wblk^T + b)
        ldm_gemm_prob_t fb = prob(Bp, H, B);
        seg(fb, L.h_b[k], H, Wb[k], 2 * H, H);
        seg(fb, L.temb_b, H, Wb[k] + H, 2 * H, H);
        fb.mode = LDM_GEMM_RESID_SILU; fb.bias = w->b_blk[k];
        fb.R = L.h_f[k]; fb.ldr = H; fb.P = L.a_f[k]; fb.ldp = H;
        if (k + 1 < L.nb) { fb.C = L.h_f[k + 1]; fb.ldc = H; }
        fb.Cb = L.h_b[k + 1]; fb.ldcb = H; fb.CbT = L.h_T[k + 1]; fb.ldct = Bp;
        LDM_TRY(launch({fb}, s, rec));
    }
    if (eps_target) {                                            // eps_hat -> eps-MSE gradient
        ldm_gemm_prob_t fo = prob(Bp, D, B);
        seg(fo, L.h_b[L.nb], H, w->w_out, H, H);
        fo.mode = LDM_GEMM_LOSS; fo.bias = w->b_out; fo.scale = loss_scale;
        fo.P_in = eps_target; fo.ldp_in = D;
        fo.Cb = L.go_b; fo.ldcb = D; fo.CbT = L.go_T; fo.ldct = Bp;
        fo.colsum = L.p_bout; fo.loss_part = L.loss_part;
        LDM_TRY(launch({fo}, s, rec));
    } else if (eps_out) {
        ldm_gemm_prob_t fo = prob(Bp, D, B);
        seg(fo, L.h_b[L.nb], H, w->w_out, H, H);
        fo.bias = w->b_out; fo.C = eps_out; fo.ldc = D;
        LDM_TRY(launch({fo}, s, rec));
    }
    return 0;
}

// Backward GEMMs from go_b / go_T (dL/d eps_hat in bf16) and the saved activations.
// `hook` (may be null) is called at point 0 once the gradients of the out-projection and block
// weights are final and no later launch of this backward reads those weights (after the dtemb
// launch, the last reader of the blocks' U_k), and at point 1 after the last GEMM (the time-MLP
// and in-projection weights: dWin and dx, which reads Win^T, are in the last launch), so
// their optimizer updates can start there.
struct StepHook {
    int (*fn)(void* ctx, int point, hipStream_t s);
    void* ctx;
};
int backward(const ldm_denoiser_t* w, const TrainWs& L, const ldm_denoiser_grads_t* gr,
             float* dx, hipStream_t s, const StepHook* hook = nullptr, Recorder* rec = nullptr) {
    const int Bp = L.Bp, B = L.B, D = L.D, H = L.H, TE = L.TE, nb = L.nb;
    const bf16_t* const* Wt = reinterpret_cast<const bf16_t* const*>(w->wt_blk);
    {
        ldm_gemm_prob_t dwo = prob(D, H, D);                     // dWout = go^T h_nb
        seg(dwo, L.go_T, Bp, L.h_T[nb], Bp, Bp);
        dwo.C = gr->w_out; dwo.ldc = H;
        ldm_gemm_prob_t dh = prob(Bp, H, B);                     // dh_nb = go Wout; g = dh SiLU'(a)
        seg(dh, L.go_b, D, w->wt_out, D, D);
        dh.mode = LDM_GEMM_DGRAD_SILU; dh.P_in = L.a_f[nb - 1]; dh.ldp_in = H;
        dh.C = L.dh[0]; dh.ldc = H;
        dh.Cb = L.g_b[nb - 1]; dh.ldcb = H; dh.CbT = L.g_T[nb - 1]; dh.ldct = Bp;
        dh.colsum = L.p_bblk[nb - 1];
        LDM_TRY(launch({dwo, dh}, s, rec));
    }
    int cur = 0;
    for (int k = nb - 1; k >= 0; --k) {
        ldm_gemm_prob_t dw = prob(H, H, H);                      // dW_k = g_k^T h_k
        seg(dw, L.g_T[k], Bp, L.h_T[k], Bp, Bp);
        dw.C = gr->w_blk[k]; dw.ldc = 2 * H;
        ldm_gemm_prob_t du = prob(H, H, H);                      // dU_k = g_k^T temb
        seg(du, L.g_T[k], Bp, L.temb_T, Bp, Bp);
        du.C = gr->w_blk[k] + H; du.ldc = 2 * H;
        ldm_gemm_prob_t dh = prob(Bp, H, B);                     // dh_k = dh_{k+1} + g_k W_k
        seg(dh, L.g_b[k], H, Wt[k], H, H);
        dh.R = L.dh[cur]; dh.ldr = H;
        if (k > 0) {                                             // ... and g_{k-1}
            dh.mode = LDM_GEMM_DGRAD_SILU; dh.P_in = L.a_f[k - 1]; dh.ldp_in = H;
            dh.C = L.dh[cur ^ 1]; dh.ldc = H;
            dh.Cb = L.g_b[k - 1]; dh.ldcb = H; dh.CbT = L.g_T[k - 1]; dh.ldct = Bp;
            dh.colsum = L.p_bblk[k - 1];
        } else {                                                 // dh_0 (the in-projection's)
            dh.mode = LDM_GEMM_ADD_R;
            dh.Cb = L.dh0_b; dh.ldcb = H; dh.CbT = L.dh0_T; dh.ldct = Bp;
            dh.colsum = L.p_bin;
        }
        LDM_TRY(launch({dw, du, dh}, s, rec));
        cur ^= 1;
    }
    {
        ldm_gemm_prob_t dt = prob(Bp, H, B);                     // dtemb = sum_k g_k U_k
        for (int k = 0; k < nb; ++k) seg(dt, L.g_b[k], H, Wt[k] + (size_t)H * H, H, H);
        dt.Cb = L.dtemb_b; dt.ldcb = H; dt.CbT = L.dtemb_T; dt.ldct = Bp;
        dt.colsum = L.p_bt2;
        // alone in its launch: 256 tiles, every K a multiple of 128 -> the 128-deep 2-group
        // tile (with dWin's 64 tiles beside it the launch fell to 64 x 64 tiles: 30.8 us)
        LDM_TRY(launch({dt}, s, rec));
        if (hook) LDM_TRY(hook->fn(hook->ctx, 0, s));
    }
    {
        ldm_gemm_prob_t dw2 = prob(H, H, H);                     // dWt2 = dtemb^T u
        seg(dw2, L.dtemb_T, Bp, L.u_T, Bp, Bp);
        dw2.C = gr->w_t2; dw2.ldc = H;
        ldm_gemm_prob_t gt = prob(Bp, H, B);                     // gt = (dtemb Wt2) SiLU'(a_t)
        seg(gt, L.dtemb_b, H, w->wt_t2, H, H);
        gt.mode = LDM_GEMM_DGRAD_SILU; gt.P_in = L.a_t; gt.ldp_in = H;
        gt.CbT = L.gt_T; gt.ldct = Bp; gt.colsum = L.p_bt1;
        LDM_TRY(launch({dw2, gt}, s, rec));
    }
    {
        ldm_gemm_prob_t dw1 = prob(H, TE, H);                    // dWt1 = gt^T e
        seg(dw1, L.gt_T, Bp, L.e_T, Bp, Bp);
        dw1.C = gr->w_t1; dw1.ldc = TE;
        // dWin rides in the step's last launch: its 64 tiles run beside dWt1's 32 on CUs that
        // launch leaves idle (beside dtemb it cost dtemb its 128-deep tile: 30.8 -> 22.7 us)
        ldm_gemm_prob_t dwi = prob(H, D, H);                     // dWin = dh0^T xt
        seg(dwi, L.dh0_T, Bp, L.xt_T, Bp, Bp);
        dwi.C = gr->w_in; dwi.ldc = D;
        if (dx) {
            ldm_gemm_prob_t px = prob(B, D, B);                  // dx = dh0 Win
            seg(px, L.dh0_b, H, w->wt_in, H, H);
            px.C = dx; px.ldc = D;
            LDM_TRY(launch({dw1, dwi, px}, s, rec));
        } else {
            LDM_TRY(launch({dw1, dwi}, s, rec));
        }
    }
    if (hook) LDM_TRY(hook->fn(hook->ctx, 1, s));
    return 0;
}

void add_job(SumJobs& J, const float* src, float* dst, int rows, int len, int ld, float scale,
             int* max_len) {
    J.j[J.n++] = {src, dst, rows, len, ld, scale};
    if (len > *max_len) *max_len = len;
}

// Bias gradients (and the loss) from the epilogue partials, one launch.
int finalize(const TrainWs& L, const ldm_denoiser_grads_t* gr, const float* deps,
             float* loss_out, float loss_scale, hipStream_t s) {
    SumJobs J;
    memset(&J, 0, sizeof(J));
    int ml = 1;
    const int R = L.Bp / 32;
    if (deps) add_job(J, deps, gr->b_out, L.B, L.D, L.D, 1.f, &ml);
    else add_job(J, L.p_bout, gr->b_out, R, L.D, L.D, 1.f, &ml);
    for (int k = 0; k < L.nb; ++k) add_job(J, L.p_bblk[k], gr->b_blk[k], R, L.H, L.H, 1.f, &ml);
    add_job(J, L.p_bin, gr->b_in, R, L.H, L.H, 1.f, &ml);
    add_job(J, L.p_bt2, gr->b_t2, R, L.H, L.H, 1.f, &ml);
    add_job(J, L.p_bt1, gr->b_t1, R, L.H, L.H, 1.f, &ml);
    if (loss_out) add_job(J, L.loss_part, loss_out, R * (L.D / 32), 1, 1, loss_scale, &ml);
    return run_sums(J, ml, s);
}

int check_grads(const ldm_denoiser_t* w, const ldm_denoiser_grads_t* g) {
    LDM_REQUIRE(g && g->w_in && g->b_in && g->w_t1 && g->b_t1 && g->w_t2 && g->b_t2 && g->w_out &&
                    g->b_out, LDM_EINVAL, "denoiser backward: gradient pointer missing");
    for (int k = 0; k < w->n_blocks; ++k)
        LDM_REQUIRE(g->w_blk[k] && g->b_blk[k], LDM_EINVAL,
                    "denoiser backward: block %d gradient missing", k);
    return 0;
}

int prep_inputs(const ldm_denoiser_t* w, const TrainWs& L, const float* x0, const float* eps,
                const int32_t* t, const ldm_sched_t* sc, hipStream_t s) {
    const int64_t n = (int64_t)L.Bp * (L.D + L.TE);
    const dim3 grid((unsigned)((n + 255) / 256));
    if (sc)
        hipLaunchKernelGGL(prep_inputs_kernel<true>, grid, dim3(256), 0, s, x0, eps, t,
                           sc->sqrt_ab, sc->sqrt_1mab, w->emb_table, L.B, L.Bp, L.D, L.TE,
                           L.xt_b, L.xt_T, L.e_b, L.e_T);
    else
        hipLaunchKernelGGL(prep_inputs_kernel<false>, grid, dim3(256), 0, s, x0, nullptr, t,
                           nullptr, nullptr, w->emb_table, L.B, L.Bp, L.D, L.TE, L.xt_b,
                           L.xt_T, L.e_b, L.e_T);
    return launch_status("denoiser prep");
}

}  // namespace
}  // namespace ldm

using namespace ldm;

extern "C" size_t ldm_denoiser_train_ws_bytes(const ldm_denoiser_t* w, int B) {
    if (!w || B < 1 || w->n_blocks < 1 || w->n_blocks > LDM_MAX_BLOCKS) return 0;
    return layout(w, B, nullptr).bytes;
}

extern "C" int ldm_denoiser_fwd(const ldm_denoiser_t* w, const float* x, const int32_t* t, int B,
                                float* eps_out, void* saved, ldm_stream_t s) {
    LDM_TRY(check_desc(w, B, false));
    LDM_REQUIRE(x && t && saved && LDM_ALIGNED(saved, 256), LDM_EINVAL,
                "ldm_denoiser_fwd: x, t and a 256-B aligned `saved` workspace are required");
    const TrainWs L = layout(w, B, saved);
    hipStream_t st = (hipStream_t)s;
    LDM_TRY(prep_inputs(w, L, x, nullptr, t, nullptr, st));
    return forward(w, L, nullptr, eps_out, 1.f, st);
}

extern "C" int ldm_denoiser_bwd(const ldm_denoiser_t* w, void* saved, const float* deps, int B,
                                const ldm_denoiser_grads_t* grads, float* dx, ldm_stream_t s) {
    LDM_TRY(check_desc(w, B, true));
    LDM_TRY(check_grads(w, grads));
    LDM_REQUIRE(deps && saved && LDM_ALIGNED(saved, 256), LDM_EINVAL,
                "ldm_denoiser_bwd: deps and the forward's `saved` workspace are required");
    LDM_REQUIRE(!dx || w->wt_in, LDM_EINVAL, "ldm_denoiser_bwd: dx needs wt_in");
    const TrainWs L = layout(w, B, saved);
    hipStream_t st = (hipStream_t)s;
    const int64_t n = (int64_t)L.Bp * L.D;
    hipLaunchKernelGGL(prep_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, deps,
                       B, L.Bp, L.D, L.go_b, L.go_T);
    LDM_TRY(launch_status("denoiser bwd prep"));
    LDM_TRY(backward(w, L, grads, dx, st));
    return finalize(L, grads, deps, nullptr, 1.f, st);
}

// ---- A9 head -------------------------------------------------------------------------------
extern "C" int ldm_q_sample_loss(const ldm_sched_t* sc, const float* x0, const float* eps,
                                 const int32_t* t, int B, int D, float* xt_out,
                                 const float* eps_hat, float* loss_out, float* grad_out,
                                 ldm_stream_t s) {
    LDM_REQUIRE(eps && B >= 1 && D >= 1, LDM_EINVAL, "ldm_q_sample_loss: bad arguments");
    if (xt_out) {
        LDM_REQUIRE(x0 && t, LDM_EINVAL, "ldm_q_sample_loss: x_t needs x0 and t");
        LDM_TRY(ldm_q_sample(sc, x0, eps, t, B, D, xt_out, s));
    }
    if (eps_hat) {
        LDM_REQUIRE(loss_out, LDM_EINVAL, "ldm_q_sample_loss: eps_hat given without loss_out");
        LDM_TRY(ldm_eps_mse_loss(eps_hat, eps, B * D, loss_out, grad_out, s));
    }
    return 0;
}

// ---- multi-tensor AdamW --------------------------------------------------------------------
// One launch over every tensor: 64 x 64 tiles (a 1-D tensor is one row), each thread 4 rows x
// 4 consecutive columns.  The update is ldm_adamw_step's, operation for operation (denoiser.hip
// adamw_kernel), so both give the same bits.  The transposed bf16 copy goes through an LDS tile
// so its stores are 32-byte row runs.
namespace ldm {
namespace {
struct AdamJobs {
    ldm_adamw_tensor_t t[LDM_ADAMW_MAX_TENSORS];
    int first[LDM_ADAMW_MAX_TENSORS + 1];
    int n;
    float decay, omb1, b2, omb2, eps, step_size, bc2_sqrt;
    const float* dh;    // non-null: the 7 scalars above are read from device memory instead
};

typedef const __attribute__((address_space(4))) AdamJobs KJobs;

__global__ __launch_bounds__(256) void adamw_multi_kernel(AdamJobs jobs) {
    typedef KJobs KJ;
    KJ* kj = (KJ*)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ unsigned short sT[64][64 + 8];
    // grid-stride over the tiles: a capped grid leaves wave slots free on every CU for work on
    // another stream (ldm_denoiser_train_step_adamw); uncapped, one tile per workgroup
    for (int tile = blockIdx.x; tile < kj->first[kj->n]; tile += gridDim.x) {
        __syncthreads();                   // the previous tile's transposed reads of sT are done
        int j = 0;
        for (int i = 1; i < kj->n; ++i)
            if (tile >= kj->first[i]) j = i;
        const float* dh = kj->dh;
        const AdamHyper hy = {dh ? dh[0] : kj->decay, dh ? dh[1] : kj->omb1,
                              dh ? dh[2] : kj->b2,    dh ? dh[3] : kj->omb2,
                              dh ? dh[4] : kj->eps,   dh ? dh[5] : kj->step_size,
                              dh ? dh[6] : kj->bc2_sqrt};
        adamw_tile(kj->t[j], hy, sT, tile - kj->first[j]);
    }
}
}  // namespace
}  // namespace ldm

namespace ldm {
namespace {
// One adamw_multi_kernel launch over the tensors list[0..n) (host descriptors).
// The update's scalars, derived in double and rounded once, as ldm_adamw_step (and torch) do:
// [decay, 1 - beta1, beta2, 1 - beta2, eps, lr / bc1, sqrt(bc2)].
void adamw_hyper(double lr, double beta1, double beta2, double eps, double weight_decay,
                 int step, float* o) {
    const double bc1 = 1.0 - pow(beta1, step), bc2 = 1.0 - pow(beta2, step);
    o[0] = (float)(1.0 - lr * weight_decay);
    o[1] = (float)(1.0 - beta1);
    o[2] = (float)beta2;
    o[3] = (float)(1.0 - beta2);
    o[4] = (float)eps;
    o[5] = (float)(lr / bc1);
    o[6] = (float)sqrt(bc2);
}

// One adamw_multi_kernel launch over the tensors list[0..n) (host descriptors); d_hyper
// (optional): device copy of adamw_hyper's 7 scalars, read by the kernel instead (a captured
// graph then replays with new step counts).
int adamw_launch(const ldm_adamw_tensor_t* const* list, int n, double lr, double beta1,
                 double beta2, double eps, double weight_decay, int step, hipStream_t s,
                 int grid_cap = 0, const float* d_hyper = nullptr) {
    if (n == 0) return 0;
    AdamJobs J;
    memset(&J, 0, sizeof(J));
    int tiles = 0;
    for (int i = 0; i < n; ++i) {
        const ldm_adamw_tensor_t& T = *list[i];
        LDM_REQUIRE(T.p && T.g && T.m && T.v && T.rows >= 1 && T.cols >= 1, LDM_EINVAL,
                    "ldm_adamw_multi: tensor %d incomplete", i);
        J.t[i] = T;
        J.first[i] = tiles;
        tiles += ((T.rows + 63) / 64) * ((T.cols + 63) / 64);
    }
    J.first[n] = tiles;
    J.n = n;
    float h[7];
    adamw_hyper(lr, beta1, beta2, eps, weight_decay, step, h);
    J.decay = h[0]; J.omb1 = h[1]; J.b2 = h[2]; J.omb2 = h[3]; J.eps = h[4];
    J.step_size = h[5]; J.bc2_sqrt = h[6];
    J.dh = d_hyper;
    const int grid = grid_cap > 0 && grid_cap < tiles ? grid_cap : tiles;
    hipLaunchKernelGGL(adamw_multi_kernel, dim3(grid), dim3(256), 0, s, J);
    return launch_status("ldm_adamw_multi");
}

// Fork / join events of ldm_denoiser_train_step_adamw, per device (created once): three forks
// (one per AdamW batch) and the join.
constexpr int kForks = 3;
int fork_events(hipEvent_t (&ev)[kForks + 1]) {
    static hipEvent_t pool[64][kForks + 1];
    int dev = 0;
    LDM_REQUIRE(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64, LDM_EINVAL,
                "train_step_adamw: no current device");
    for (int i = 0; i <= kForks; ++i) {
        if (!pool[dev][i]) {
            const hipError_t e = hipEventCreateWithFlags(&pool[dev][i], hipEventDisableTiming);
            LDM_REQUIRE(e == hipSuccess, (int)e, "train_step_adamw: hipEventCreate: %s",
                        hipGetErrorString(e));
        }
        ev[i] = pool[dev][i];
    }
    return 0;
}

// The step's AdamW in three batches, each started as soon as its gradients are final and no
// later launch of the step reads its weights: 0 = block and out-projection weights (after the
// dtemb launch), 1 = the time-MLP and in-projection weights (after the last GEMM), 2 = the
// biases (after the
// bias sums).  With a side stream every batch runs there behind a fork event, on a capped grid
// (2 workgroups per CU) so the main stream's GEMMs keep wave slots; the main stream waits for
// the side stream at the end.
struct AdamSplit {
    const ldm_adamw_tensor_t* batch[kForks][LDM_ADAMW_MAX_TENSORS];
    int nb[kForks];
    double lr, beta1, beta2, eps, wd;
    int step, grid_cap;
    const float* d_hyper;
    hipStream_t side;
    hipEvent_t ev[kForks + 1];
};

int adam_batch(AdamSplit& A, int i, hipStream_t s) {
    if (A.nb[i] == 0) return 0;
    hipStream_t q = s;
    if (A.side) {
        LDM_REQUIRE(hipEventRecord(A.ev[i], s) == hipSuccess &&
                        hipStreamWaitEvent(A.side, A.ev[i], 0) == hipSuccess,
                    LDM_EINVAL, "train_step_adamw: fork failed");
        q = A.side;
    }
    return adamw_launch(A.batch[i], A.nb[i], A.lr, A.beta1, A.beta2, A.eps, A.wd, A.step, q,
                        A.side ? A.grid_cap : 0, A.d_hyper);
}

int adam_hook(void* ctx, int point, hipStream_t s) {
    return adam_batch(*static_cast<AdamSplit*>(ctx), point, s);
}
}  // namespace
}  // namespace ldm

// ---- the persistent step (train_dag.hip) ----------------------------------------------------
// The DAG is derived from the launch path itself: forward() / backward() run with a Recorder,
// so the GEMM problems (operands, epilogues, layouts) are the launch path's, and each keeps the
// k-group split of the tile its launch would run (gemm_tile_choice): bit-identical results.
namespace ldm {
namespace {

struct TrainCfg {
    int form = LDM_TRAIN_AUTO;
    unsigned spin = 0;
    int last = 0;
    unsigned dbg = 0;           // ldm_dev_train_dag_flags (diagnostics only)
};
TrainCfg& train_cfg() {
    static TrainCfg cfg[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    return cfg[dev];
}

uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const unsigned char* c = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) {
        h ^= c[i];
        h *= 1099511628211ull;
    }
    return h;
}

// the LDS-transposed epilogue's vector conditions (gemm_bf16.hip epi(): `ok`), for every block
bool lds_epilogue_ok(const ldm_gemm_prob_t& P) {
    auto al = [](const void* p, int a) { return ((uintptr_t)p & (uintptr_t)(a - 1)) == 0; };
    return P.N % 64 == 0 && P.k_split <= 1 && (!P.C || (al(P.C, 16) && P.ldc % 4 == 0)) &&
           (!P.P || (al(P.P, 16) && P.ldp % 4 == 0)) &&
           (P.mode == LDM_GEMM_ACCUM || !P.R || (al(P.R, 16) && P.ldr % 4 == 0)) &&
           (!P.P_in || (al(P.P_in, 16) && P.ldp_in % 4 == 0)) &&
           (!P.Cb || (al(P.Cb, 8) && P.ldcb % 4 == 0)) &&
           (!P.Rb || (al(P.Rb, 8) && P.ldrb % 4 == 0)) && (!P.bias || al(P.bias, 16));
}

struct DagHost {
    uint64_t hash = 0;
    dag::Table tab;
    std::vector<uint32_t> entries;
};

// The uploaded tables, by device table address.  An entry's host copy is only read by its
// upload, which synchronises before dag_step returns, so entries may go at any time after that:
// ldm_denoiser_train_ws_init drops the one of its workspace, and the map is cleared when it
// reaches kMaxCached entries (a workload that keeps allocating workspaces of new sizes stays
// bounded; a dropped configuration re-uploads at its next step).  shared_ptr: a step in flight
// on another thread keeps its entry alive.
struct DagCache {
    static constexpr size_t kMaxCached = 32;
    std::mutex mu;
    std::unordered_map<const void*, std::shared_ptr<DagHost>> by_table;
};
DagCache& dag_cache() {
    static DagCache c;
    return c;
}

constexpr bool kSplitU = false;     // U_k's AdamW as an early update + late copies (measured: off)

// ---- operand extents vs the allocations (round 6, after the r05h illegal access) -----------
// Every byte range a job of the table may touch -- each GEMM operand over its problem's rows and
// leading dimension (ext_bytes, the same extents the kernel gives its buffer resources), the
// prep outputs, the sums' partials, each AdamW tensor -- must lie inside ONE allocation the
// caller handed over: the training workspace, a weight / bias / table of the descriptor, a
// gradient, an AdamW tensor, the schedule.  A table that fails is refused (LDM_EINVAL, named
// node and operand), so an indexing bug in the builder never reaches the GPU as a stray access.
struct Region {
    const char* p;
    int64_t bytes;
};
struct Regions {
    std::vector<Region> r;
    void add(const void* p, int64_t bytes) {
        if (p && bytes > 0) r.push_back({static_cast<const char*>(p), bytes});
    }
    bool holds(const void* p, int64_t bytes) const {
        const char* c = static_cast<const char*>(p);
        for (const Region& x : r)
            if (c >= x.p && c + bytes <= x.p + x.bytes) return true;
        return false;
    }
};

int check_dag_extents(const dag::Table& T, const ldm_denoiser_t* w, const ldm_sched_t* sc,
                      const TrainWs& L, const ldm_denoiser_grads_t* gr,
                      const ldm_adamw_tensor_t* tensors, int n, const void* eps_tag) {
    using namespace dag;
    const int64_t D = w->D, H = w->H, TE = w->TE, Tn = w->T;
    Regions R;
    R.add(L.xt_b, (int64_t)L.bytes);                        // the workspace (xt_b is its start)
    R.add(w->w_in, H * D * 2); R.add(w->w_t1, H * TE * 2); R.add(w->w_t2, H * H * 2);
    R.add(w->w_out, D * H * 2); R.add(w->wt_in, D * H * 2); R.add(w->wt_t2, H * H * 2);
    R.add(w->wt_out, H * D * 2);
    R.add(w->b_in, H * 4); R.add(w->b_t1, H * 4); R.add(w->b_t2, H * 4); R.add(w->b_out, D * 4);
    R.add(w->emb_table, Tn * TE * 4);
    for (int k = 0; k < w->n_blocks; ++k) {
        R.add(w->w_blk[k], H * 2 * H * 2); R.add(w->wt_blk[k], 2 * H * H * 2);
        R.add(w->b_blk[k], H * 4);
        R.add(gr->w_blk[k], H * 2 * H * 4); R.add(gr->b_blk[k], H * 4);
    }
    R.add(gr->w_in, H * D * 4); R.add(gr->b_in, H * 4); R.add(gr->w_t1, H * TE * 4);
    R.add(gr->b_t1, H * 4); R.add(gr->w_t2, H * H * 4); R.add(gr->b_t2, H * 4);
    R.add(gr->w_out, D * H * 4); R.add(gr->b_out, D * 4);
    R.add(sc->sqrt_ab, (int64_t)sc->T * 4); R.add(sc->sqrt_1mab, (int64_t)sc->T * 4);
    // (R so far: what the descriptors size.  An AdamW tensor's gradient and bf16 copies must
    // lie in it -- they are the step's own gradients and the descriptor's weights -- so a
    // tensor that claims more rows / columns than its gradient holds is refused below; its
    // fp32 master and moments are the caller's alone and join the regions here.)
    const Regions K = R;
    for (int i = 0; i < n; ++i) {
        const ldm_adamw_tensor_t& t = tensors[i];
        const int64_t e = (int64_t)t.rows * t.cols;
        R.add(t.p, e * 4); R.add(t.m, e * 4); R.add(t.v, e * 4);
    }
    const char* what = nullptr;
    int bad = -1;
    auto need = [&](int node, const char* name, const void* p, int64_t bytes) {
        if (!p || bytes <= 0 || bad >= 0 || p == eps_tag) return;   // eps: a launch argument
        if (bytes >= (int64_t)kMaxExtent || !R.holds(p, bytes)) {
            bad = node;
            what = name;
        }
    };
    for (int i = 0; i < T.n_nodes; ++i) {
        const Node& nd = T.node[i];
        if (nd.type == N_GEMM) {
            const ldm_gemm_prob_t& P = nd.P;
            const int64_t M = P.M, Nc = P.N, Mv = P.M_valid;
            // the job grid covers the problem and no more than one tile beyond it
            if ((int64_t)nd.tiles_m * tile_rows(nd.tile) < M ||
                (int64_t)(nd.tiles_m - 1) * tile_rows(nd.tile) >= M ||
                (int64_t)nd.tiles_n * tile_cols(nd.tile) < Nc ||
                (int64_t)(nd.tiles_n - 1) * tile_cols(nd.tile) >= Nc || Mv > M) {
                bad = i;
                what = "job grid vs problem";
            }
            int64_t ks = 0;
            for (int g = 0; g < P.n_seg; ++g) {
                const ldm_gemm_seg_t& S = P.seg[g];
                need(i, "A operand", S.A, ext_bytes(M, S.lda, S.K, 2));
                need(i, "B operand", S.B, ext_bytes(Nc, S.ldb, S.K, 2));
                if (S.K % 64 != 0) { bad = i; what = "segment K"; }
                ks += S.K / 64;
            }
            if (ks != nd.nk && bad < 0) { bad = i; what = "k-steps"; }
            need(i, "C", P.C, ext_bytes(Mv, P.ldc, Nc, 4));
            need(i, "P", P.P, ext_bytes(Mv, P.ldp, Nc, 4));
            if (P.mode != LDM_GEMM_ACCUM) need(i, "R", P.R, ext_bytes(Mv, P.ldr, Nc, 4));
            need(i, "P_in", P.P_in, ext_bytes(Mv, P.ldp_in, Nc, 4));
            need(i, "Rb", P.Rb, ext_bytes(Mv, P.ldrb, Nc, 2));
            need(i, "Cb", P.Cb, ext_bytes(M, P.ldcb, Nc, 2));
            need(i, "CbT", P.CbT, ext_bytes(Nc, P.ldct, M, 2));
            need(i, "colsum", P.colsum, ext_bytes((M - 1) / 32 + 1, Nc, Nc, 4));
            need(i, "loss_part", P.loss_part,
                 ext_bytes((M - 1) / 32 + 1, (Nc + 31) / 32, (Nc + 31) / 32, 4));
            need(i, "bias", P.bias, Nc * 4);
        } else if (nd.type == N_PREP) {
            need(i, "xt_b", nd.xt_b, ext_bytes(nd.Bp, nd.D, nd.D, 2));
            need(i, "xt_T", nd.xt_T, ext_bytes(nd.D, nd.Bp, nd.Bp, 2));
            need(i, "e_b", nd.e_b, ext_bytes(nd.Bp, nd.TE, nd.TE, 2));
            need(i, "e_T", nd.e_T, ext_bytes(nd.TE, nd.Bp, nd.Bp, 2));
            need(i, "emb", nd.emb, Tn * nd.TE * 4);
            if ((int64_t)nd.tiles_m * kBand < nd.Bp && bad < 0) { bad = i; what = "prep bands"; }
        } else if (nd.type == N_SUM) {
            need(i, "sum src", nd.src, ext_bytes(nd.rows, nd.ld, nd.len, 4));
            need(i, "sum dst", nd.dst, (int64_t)nd.len * 4);
        } else if (nd.type == N_ADAM) {
            if (nd.adam < 0 || nd.adam >= n) {
                if (bad < 0) { bad = i; what = "AdamW tensor index"; }
                continue;
            }
            const ldm_adamw_tensor_t& t = tensors[nd.adam];
            const int64_t e = (int64_t)t.rows * t.cols;
            for (const void* q : {static_cast<const void*>(t.g)})
                if (bad < 0 && q && !K.holds(q, e * 4)) { bad = i; what = "AdamW gradient"; }
            for (const void* q : {t.p_bf16, t.p_bf16_t})
                if (bad < 0 && q && !K.holds(q, e * 2)) { bad = i; what = "AdamW bf16 copy"; }
            if ((int64_t)nd.tiles_m * 64 < t.rows ||
                nd.col_off + nd.nk > (t.cols + 63) / 64) {
                if (bad < 0) { bad = i; what = "AdamW tiles vs tensor"; }
            }
        }
        if (nd.type == N_SUM && nd.adam >= 0 && nd.adam < n &&
            (int64_t)tensors[nd.adam].rows * tensors[nd.adam].cols != nd.len && bad < 0) {
            bad = i;
            what = "bias sum length vs its AdamW tensor";
        }
    }
    LDM_REQUIRE(bad < 0, LDM_EINVAL,
                "train dag: node %d: %s lies outside every allocation the step was given "
                "(or exceeds 2 GiB); table refused", bad, what ? what : "?");
    return 0;
}

// Builds the job table of one step; returns 1 (and builds nothing) when this configuration has
// no DAG form -- the caller then runs the launch path.
int build_dag(const ldm_denoiser_t* w, const ldm_sched_t* sc, const TrainWs& L,
              const ldm_denoiser_grads_t* gr, const ldm_adamw_tensor_t* tensors, int n,
              float nf, int grid, DagHost& H) {
    using namespace dag;
    const int nb = L.nb;
    Recorder rec;
    const float* kEps = reinterpret_cast<const float*>((uintptr_t)256);   // eps: a launch arg
    LDM_TRY(forward(w, L, kEps, nullptr, 2.f / nf, nullptr, &rec));
    LDM_TRY(backward(w, L, gr, nullptr, nullptr, nullptr, &rec));
    if ((int)rec.launches.size() != 2 * nb + 7) return 1;
    Table& T = H.tab;
    memset(&T, 0, sizeof(T));
    int nctr = 0;
    bool ok = true;
    auto add = [&](Node nd) -> int {
        if (T.n_nodes >= kMaxNodes) {          // (~50 nodes at 4 blocks; 8 blocks fit too)
            ok = false;
            return kMaxNodes - 1;
        }
        nd.out_band = -1;
        if (nd.type == N_GEMM || nd.type == N_PREP) {
            nd.out_band = nctr;
            nctr += nd.tiles_m;
        }
        nd.out_all = nctr++;
        T.node[T.n_nodes] = nd;
        return T.n_nodes++;
    };
    auto dep = [&](int c, int p, bool band) {
        Node& C = T.node[c];
        Node& Pn = T.node[p];
        Pn.signal = 1;
        // a band hand-off pairs the same 64-row bands: both nodes are row nodes
        if (band) ok = ok && (Pn.type == N_PREP || Pn.row) && (C.type == N_PREP || C.row);
        C.dep_ctr[C.ndep] = band ? Pn.out_band : Pn.out_all;
        C.dep_band[C.ndep] = band ? 1 : 0;
        C.dep_target[C.ndep] = band ? (unsigned)Pn.tiles_n : (unsigned)(Pn.tiles_m * Pn.tiles_n);
        ++C.ndep;
    };
    // row: the product's rows are the batch's (the forward / backward chain: band hand-offs,
    // 64 x 64 tiles); otherwise a weight-gradient product (rows = features, 128 x 128 tiles)
    auto gemm = [&](int li, int pi, bool row) -> int {
        const ldm_gemm_args_t& a = rec.launches[li];
        const ldm_gemm_prob_t& P = a.prob[pi];
        Node nd;
        memset(&nd, 0, sizeof(nd));
        nd.type = N_GEMM;
        nd.P = P;
        // row nodes: the batch's rows (the chain, band hand-offs); the tile kind: the launch
        // tile's two k-groups -> 64 x 64 in two groups, else 64 x 128 (row) or 128 x 128 (the
        // weight-gradient products) -- train_dag.hip TileCfg
        nd.row = row ? 1 : 0;
        ok = ok && (!row || P.M == L.Bp);
        for (int g = 0; g < P.n_seg; ++g) nd.nk += P.seg[g].K / 64;
        nd.kgp = gemm_tile_kgroup_period(gemm_tile_choice(a));
        bool k128 = true;                 // every segment's K a multiple of 128 (128-deep stages)
        for (int g = 0; g < P.n_seg; ++g) k128 = k128 && P.seg[g].K % 128 == 0;
        nd.tile = nd.kgp == 2 && k128 ? TILE_K2L : nd.kgp > 0 ? TILE_K2 : row ? TILE_ROW : TILE_W;
        nd.tiles_m = (P.M + tile_rows(nd.tile) - 1) / tile_rows(nd.tile);
        nd.tiles_n = (P.N + tile_cols(nd.tile) - 1) / tile_cols(nd.tile);
        nd.adam = -1;
        if (P.P_in == kEps) {
            nd.pin_eps = 1;
            nd.P.P_in = nullptr;
        }
        ok = ok && lds_epilogue_ok(nd.P) && P.ct_blk == 0 && nd.tiles_m * nd.tiles_n <= 65535;
        return add(nd);
    };
    // tensor of each gradient (AdamW), -1 if not in the table
    auto tens = [&](const float* g) {
        for (int i = 0; i < n; ++i)
            if (tensors[i].g == g) return i;
        return -1;
    };
    std::vector<bool> used(n, false);
    auto sum = [&](const float* src, float* dst, int rows, int len, int ld, float scale,
                   const float* g) -> int {
        Node nd;
        memset(&nd, 0, sizeof(nd));
        nd.type = N_SUM;
        nd.tiles_m = nd.tiles_n = 1;
        nd.src = src; nd.dst = dst; nd.rows = rows; nd.len = len; nd.ld = ld; nd.scale = scale;
        nd.adam = g ? tens(g) : -1;
        if (nd.adam >= 0) {
            const ldm_adamw_tensor_t& t = tensors[nd.adam];
            ok = ok && !t.p_bf16 && !t.p_bf16_t && (int64_t)t.rows * t.cols == len;
            used[nd.adam] = true;
        }
        return add(nd);
    };
    auto adam = [&](const float* g, int col_off, int col_tiles, int amode = 0) -> int {
        const int ti = tens(g);
        if (ti < 0) return -1;
        const ldm_adamw_tensor_t& t = tensors[ti];
        Node nd;
        memset(&nd, 0, sizeof(nd));
        nd.type = N_ADAM;
        nd.adam = ti;
        nd.amode = amode;
        nd.col_off = col_off;
        nd.tiles_m = (t.rows + 63) / 64;
        nd.nk = col_tiles ? col_tiles : (t.cols + 63) / 64;      // the node's 64-column tiles
        nd.tiles_n = (nd.nk + kAdamGroup - 1) / kAdamGroup;       // jobs: kAdamGroup of them
        used[ti] = true;
        return add(nd);
    };
    // ---- nodes in priority order (topological: every dependency is an earlier node) --------
    const int base = nb + 3, H_ = L.H;
    Node pr;
    memset(&pr, 0, sizeof(pr));
    pr.type = N_PREP;
    pr.tiles_m = (L.Bp + kBand - 1) / kBand;
    pr.row = 1;
    pr.tiles_n = (L.D + 63) / 64 + (L.TE + 63) / 64;     // 64-column chunks of [xt | e]
    pr.adam = -1;
    pr.sab = sc->sqrt_ab; pr.s1mab = sc->sqrt_1mab; pr.emb = w->emb_table;
    pr.B = L.B; pr.Bp = L.Bp; pr.D = L.D; pr.TE = L.TE;
    pr.xt_b = L.xt_b; pr.xt_T = L.xt_T; pr.e_b = L.e_b; pr.e_T = L.e_T;
    ok = ok && L.D % 4 == 0 && L.TE % 4 == 0;        // prep_job's 4-column stores
    const int prep = add(pr);
    const int f1 = gemm(0, 0, true), f3 = gemm(0, 1, true);
    dep(f1, prep, true);
    dep(f3, prep, true);
    const int f2 = gemm(1, 0, true);
    dep(f2, f1, true);
    std::vector<int> fb(nb);
    for (int k = 0; k < nb; ++k) {
        fb[k] = gemm(2 + k, 0, true);
        dep(fb[k], k == 0 ? f3 : fb[k - 1], true);
        dep(fb[k], f2, true);
    }
    const int fo = gemm(2 + nb, 0, true);
    dep(fo, fb[nb - 1], true);
    const int dhout = gemm(base, 1, true);
    dep(dhout, fo, true);
    dep(sum(L.p_bout, gr->b_out, L.Bp / 32, L.D, L.D, 1.f, gr->b_out), fo, false);
    dep(sum(L.loss_part, nullptr, (L.Bp / 32) * (L.D / 32), 1, 1, 1.f / nf, nullptr), fo,
        false);
    const int dwo = gemm(base, 0, false);
    dep(dwo, fo, false);
    std::vector<int> Dk(nb), dwk(nb), duk(nb), uupd(nb, -1);
    std::vector<bool> wdone(nb, false);
    bool wout_done = false;
    auto adam_w = [&](int k) {            // W_k's update: its gradient and dh_k (reads W_k^T)
        const int a = adam(gr->w_blk[k], 0, H_ / 64);
        if (a >= 0) {
            dep(a, dwk[k], false);
            dep(a, Dk[k], false);
        }
        wdone[k] = true;
    };
    auto adam_wout = [&]() {
        const int a = adam(gr->w_out, 0, 0);
        if (a >= 0) {
            dep(a, dwo, false);
            dep(a, dhout, false);
        }
        wout_done = true;
    };
    for (int i = 0; i < nb; ++i) {
        const int k = nb - 1 - i;
        const int gprod = k == nb - 1 ? dhout : Dk[k + 1];      // produced g_k and p_bblk[k]
        Dk[k] = gemm(base + 1 + i, 2, true);
        dep(Dk[k], gprod, true);
        dwk[k] = gemm(base + 1 + i, 0, false);
        dep(dwk[k], gprod, false);
        duk[k] = gemm(base + 1 + i, 1, false);
        dep(duk[k], gprod, false);
        dep(sum(L.p_bblk[k], gr->b_blk[k], L.Bp / 32, H_, H_, 1.f, gr->b_blk[k]), gprod, false);
        // (U_k's update waits for dtemb, which reads U_k^T: the tail below.  Split into an early
        // fp32 update here and late bf16 copies -- adamw_tile modes 1 / 2, kSplitU -- its
        // jobs took CUs from the backward chain: 321 -> 350 us per step, profiles/r05r.)
        if (kSplitU) {
            uupd[k] = adam(gr->w_blk[k], H_ / 64, H_ / 64, 1);
            if (uupd[k] >= 0) dep(uupd[k], duk[k], false);
        }
        if (k + 1 < nb) adam_w(k + 1);
        if (k == nb - 2) adam_wout();
    }
    if (!wout_done) adam_wout();
    dep(sum(L.p_bin, gr->b_in, L.Bp / 32, H_, H_, 1.f, gr->b_in), Dk[0], false);
    const int dt = gemm(base + 1 + nb, 0, true);
    dep(dt, nb >= 2 ? Dk[1] : dhout, true);      // the producer of g_0 (the chain covers g_k>0)
    adam_w(0);
    const int gt = gemm(base + 2 + nb, 1, true);
    dep(gt, dt, true);
    const int dwi = gemm(base + 3 + nb, 1, false);
    dep(dwi, Dk[0], false);
    const int dw2 = gemm(base + 2 + nb, 0, false);
    dep(dw2, dt, false);
    dep(sum(L.p_bt2, gr->b_t2, L.Bp / 32, H_, H_, 1.f, gr->b_t2), dt, false);
    // (Putting the critical tail -- dW_t1 and w_t1's update -- ahead of the U_k updates in node
    // order measured slower, 3070 -> 2972 steps/s, profiles/r05s: a queue hands out jobs in node
    // order, so a job placed before it is ready binds a workgroup to a wait.  Order by
    // readiness.)
    for (int k = nb - 1; k >= 0; --k) {      // U_k's update (or its bf16 copies): dtemb (WAR)
        const int u = adam(gr->w_blk[k], H_ / 64, H_ / 64, kSplitU ? 2 : 0);
        if (u >= 0) {
            dep(u, kSplitU ? uupd[k] : duk[k], false);
            dep(u, dt, false);
        }
    }
    const int dw1 = gemm(base + 3 + nb, 0, false);
    dep(dw1, gt, false);
    dep(sum(L.p_bt1, gr->b_t1, L.Bp / 32, H_, H_, 1.f, gr->b_t1), gt, false);
    int a = adam(gr->w_in, 0, 0);
    if (a >= 0) dep(a, dwi, false);
    a = adam(gr->w_t2, 0, 0);
    if (a >= 0) {
        dep(a, dw2, false);
        dep(a, gt, false);
    }
    a = adam(gr->w_t1, 0, 0);
    if (a >= 0) dep(a, dw1, false);
    for (int i = 0; i < n; ++i) ok = ok && used[i];         // every tensor is one of ours
    for (int i = 0; i < n; ++i) T.tensor[i] = tensors[i];
    if (!ok || nctr > kMaxCounters) return 1;
    // GEMM operands that are bf16 weight copies: a tensor's ADAM jobs rewrite its copies only
    // after every job reading them (the dependencies above), and the launch boundary before
    // the step made them visible, so those loads may go through the L2 (plain) instead of sc1
    // -- every band tile of a node re-reads the node's weights.  Measured ~1 % slower at config
    // 2 (profiles/r05v/train_ab_*.log), so only under ldm_dev_train_dag_flags kDbgWeightsL2.
    auto is_weight = [&](const void* p) {
        const char* c = static_cast<const char*>(p);
        for (int i = 0; i < n; ++i) {
            const int64_t bytes = (int64_t)tensors[i].rows * tensors[i].cols * 2;
            for (const void* w : {tensors[i].p_bf16, tensors[i].p_bf16_t}) {
                const char* w0 = static_cast<const char*>(w);
                if (w0 && c >= w0 && c < w0 + bytes) return true;
            }
        }
        return false;
    };
    for (int i = 0; i < T.n_nodes; ++i) {
        Node& nd = T.node[i];
        nd.stat = 0;
        if (nd.type != N_GEMM) continue;
        int sa = 1, sb = 2;
        for (int s = 0; s < nd.P.n_seg; ++s) {
            if (!is_weight(nd.P.seg[s].A)) sa = 0;
            if (!is_weight(nd.P.seg[s].B)) sb = 0;
        }
        nd.stat = sa | sb;
    }
    // every operand range inside an allocation the caller handed over (round 6)
    LDM_TRY(check_dag_extents(T, w, sc, L, gr, tensors, n, kEps));
    // every dependency points at an earlier node (the deadlock-freedom argument)
    for (int c = 0; c < T.n_nodes; ++c)
        for (int d = 0; d < T.node[c].ndep; ++d)
            LDM_REQUIRE(T.node[c].dep_ctr[d] < T.node[c].out_band ||
                            T.node[c].dep_ctr[d] < T.node[c].out_all,
                        LDM_EINVAL, "train dag: node %d depends on a later node", c);
    // ---- jobs -> queues: row bands of the batch stay on one queue (2 of the 16 bands each),
    // other nodes in contiguous chunks, single jobs round-robin
    std::vector<uint32_t> q[kQueues];
    int rr = 0;
    for (int i = 0; i < T.n_nodes; ++i) {
        const Node& nd = T.node[i];
        const int jobs = nd.tiles_m * nd.tiles_n;
        const bool rows = nd.type == N_PREP || (nd.type == N_GEMM && nd.row);
        for (int j = 0; j < jobs; ++j) {
            int qq;
            if (jobs == 1) qq = rr++ % kQueues;
            else if (rows) qq = (j / nd.tiles_n) * kQueues / nd.tiles_m;
            else qq = (int)((int64_t)j * kQueues / jobs);
            q[qq].push_back((uint32_t)i << 16 | (uint32_t)j);
        }
    }
    H.entries.clear();
    for (int qq = 0; qq < kQueues; ++qq) {
        T.qoff[qq] = (int)H.entries.size();
        T.qlen[qq] = (int)q[qq].size();
        H.entries.insert(H.entries.end(), q[qq].begin(), q[qq].end());
    }
    // the claim scheduler's lists: each queue split into its chain jobs and the rest
    for (int cls = 0; cls < 2; ++cls)
        for (int qq = 0; qq < kQueues; ++qq) {
            const int li = qq + cls * kQueues;
            T.qoff2[li] = (int)H.entries.size();
            for (uint32_t en : q[qq]) {
                const Node& nd = T.node[en >> 16];
                const bool chain = nd.type == N_PREP || (nd.type == N_GEMM && nd.row);
                if (chain == (cls == 0)) H.entries.push_back(en);
            }
            T.qlen2[li] = (int)H.entries.size() - T.qoff2[li];
        }
    if ((int)H.entries.size() > kMaxEntries) return 1;
    T.n_counters = nctr;
    T.n_entries = (int)H.entries.size();
    T.n_tensors = n;
    T.grid = grid;
    return 0;
}

// LDM_TRAIN_AUTO's choice: the one-launch step where it measured faster than the launch path
// (not yet at config 2's batch -- profiles/r05*/train_ab.log).
bool dag_auto(int B) {
    (void)B;
    return false;
}

// The step as one launch.  Returns 1 when the configuration has no DAG form (nothing done).
int dag_step(const ldm_denoiser_t* w, const ldm_sched_t* sc, const float* x0, const float* eps,
             const int32_t* t, int B, void* saved, const ldm_denoiser_grads_t* grads,
             float* loss_out, const ldm_adamw_tensor_t* tensors, int n, const float* hy7,
             const float* d_hyper, unsigned spin, unsigned dbg, hipStream_t s) {
    const TrainWs L = layout(w, B, saved);
    int grid = 0;
    LDM_TRY(dag::dag_grid(&grid));
    // the table depends on every pointer and size it names: hash them (the kernel refuses a
    // table built for other inputs: status 3)
    uint64_t h = 1469598103934665603ull;
    h = fnv(h, w, sizeof(*w));
    h = fnv(h, sc, sizeof(*sc));
    h = fnv(h, grads, sizeof(*grads));
    h = fnv(h, tensors, sizeof(*tensors) * (size_t)n);
    h = fnv(h, &B, sizeof(B));
    h = fnv(h, &grid, sizeof(grid));
    h = fnv(h, &L.dag_table, sizeof(L.dag_table));
    const size_t tb = sizeof(dag::Table);
    h = fnv(h, &tb, sizeof(tb));
    DagCache& dc = dag_cache();
    std::shared_ptr<DagHost> hc;
    {
        std::lock_guard<std::mutex> g(dc.mu);
        if (dc.by_table.size() >= DagCache::kMaxCached && !dc.by_table.count(L.dag_table))
            dc.by_table.clear();
        std::shared_ptr<DagHost>& slot = dc.by_table[L.dag_table];
        if (!slot) slot = std::make_shared<DagHost>();
        hc = slot;
    }
    if (hc->hash != h) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        LDM_REQUIRE(hipStreamIsCapturing(s, &cs) == hipSuccess &&
                        cs == hipStreamCaptureStatusNone,
                    LDM_EINVAL, "ldm_denoiser_train_step_adamw (dag): the first step of a "
                    "configuration uploads its job table; run it once before graph capture");
        const int r = build_dag(w, sc, L, grads, tensors, n, (float)B * (float)w->D, grid, *hc);
        if (r != 0) {
            hc->hash = 0;
            return r;
        }
        hc->tab.hash = h;
        hipError_t e = hipMemcpyAsync(L.dag_table, &hc->tab, sizeof(dag::Table),
                                      hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(L.dag_table + 1, hc->entries.data(),
                               hc->entries.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = hipMemsetAsync(L.dag_sync, 0, dag::sync_bytes(dag::kMaxCounters), s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);      // once per configuration
        LDM_REQUIRE(e == hipSuccess, (int)e, "train dag: table upload: %s",
                    hipGetErrorString(e));
        hc->hash = h;
    }
    dag::LaunchArgs a;
    memset(&a, 0, sizeof(a));
    a.tab = L.dag_table;
    a.sync = L.dag_sync;
    a.hash = h;
    a.x0 = x0; a.eps = eps; a.t = t; a.loss_out = loss_out;
    a.d_hyper = d_hyper;
    for (int i = 0; i < 7; ++i) a.hy[i] = hy7[i];
    a.spin_limit = spin ? spin : 2000000u;        // microseconds a wait may take: 2 s
    a.dbg = dbg;
    return dag::dag_launch(a, grid, s);
}

}  // namespace
}  // namespace ldm

// The forward + backward without the optimizer (the data-parallel step: the update waits for
// the gradient all-reduce).  The form follows ldm_train_step_config like the step with AdamW:
// the one-launch job DAG built WITHOUT AdamW nodes (no tensor table: the bias sums only store
// their gradients) or the launches.  Bit-identical either way (tests/test_gpu_train_dag.py).
extern "C" int ldm_denoiser_train_step(const ldm_denoiser_t* w, const ldm_sched_t* sc,
                                       const float* x0, const float* eps, const int32_t* t, int B,
                                       void* saved, const ldm_denoiser_grads_t* grads,
                                       float* loss_out, ldm_stream_t s) {
    LDM_TRY(check_desc(w, B, true));
    LDM_TRY(check_grads(w, grads));
    LDM_REQUIRE(sc && sc->abi_version == LDM_ABI_VERSION && sc->sqrt_ab && sc->sqrt_1mab,
                LDM_EINVAL, "ldm_denoiser_train_step: bad schedule");
    LDM_REQUIRE(x0 && eps && t && saved && LDM_ALIGNED(saved, 256), LDM_EINVAL,
                "ldm_denoiser_train_step: x0, eps, t and a 256-B aligned workspace are required");
    TrainCfg& cfg = train_cfg();
    if (cfg.form == LDM_TRAIN_DAG || (cfg.form == LDM_TRAIN_AUTO && dag_auto(B))) {
        const float h7[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const int r = dag_step(w, sc, x0, eps, t, B, saved, grads, loss_out, nullptr, 0, h7,
                               nullptr, cfg.spin, cfg.dbg, (hipStream_t)s);
        if (r == 0) {
            cfg.last = LDM_TRAIN_DAG;
            return 0;
        }
        if (r != 1) return r;
        LDM_REQUIRE(cfg.form != LDM_TRAIN_DAG, LDM_ENOSYS, "ldm_denoiser_train_step: no "
                    "one-launch form for this configuration (LDM_TRAIN_DAG was required)");
    }
    cfg.last = LDM_TRAIN_LAUNCHES;
    const TrainWs L = layout(w, B, saved);
    hipStream_t st = (hipStream_t)s;
    const float n = (float)B * (float)w->D;
    LDM_TRY(prep_inputs(w, L, x0, eps, t, sc, st));
    LDM_TRY(forward(w, L, eps, nullptr, 2.f / n, st));
    LDM_TRY(backward(w, L, grads, nullptr, st));
    return finalize(L, grads, nullptr, loss_out, 1.f / n, st);
}

extern "C" int ldm_adamw_multi(const ldm_adamw_tensor_t* tensors, int n, double lr,
                               double beta1, double beta2, double eps, double weight_decay,
                               int step, ldm_stream_t s) {
    LDM_REQUIRE(tensors && n >= 1 && n <= LDM_ADAMW_MAX_TENSORS && step >= 1, LDM_EINVAL,
                "ldm_adamw_multi: 1..%d tensors, step >= 1", LDM_ADAMW_MAX_TENSORS);
    const ldm_adamw_tensor_t* list[LDM_ADAMW_MAX_TENSORS];
    for (int i = 0; i < n; ++i) list[i] = &tensors[i];
    return adamw_launch(list, n, lr, beta1, beta2, eps, weight_decay, step, (hipStream_t)s);
}

extern "C" int ldm_denoiser_train_step_adamw(
    const ldm_denoiser_t* w, const ldm_sched_t* sc, const float* x0, const float* eps,
    const int32_t* t, int B, void* saved, const ldm_denoiser_grads_t* grads, float* loss_out,
    const ldm_adamw_tensor_t* tensors, int n, double lr, double beta1, double beta2,
    double eps_adam, double weight_decay, int step, const float* d_hyper, ldm_stream_t s,
    ldm_stream_t side) {
    LDM_TRY(check_desc(w, B, true));
    LDM_TRY(check_grads(w, grads));
    LDM_REQUIRE(sc && sc->abi_version == LDM_ABI_VERSION && sc->sqrt_ab && sc->sqrt_1mab,
                LDM_EINVAL, "ldm_denoiser_train_step_adamw: bad schedule");
    LDM_REQUIRE(x0 && eps && t && saved && LDM_ALIGNED(saved, 256), LDM_EINVAL,
                "ldm_denoiser_train_step_adamw: x0, eps, t and a 256-B aligned workspace are "
                "required");
    LDM_REQUIRE(tensors && n >= 1 && n <= LDM_ADAMW_MAX_TENSORS && step >= 1, LDM_EINVAL,
                "ldm_denoiser_train_step_adamw: 1..%d tensors, step >= 1",
                LDM_ADAMW_MAX_TENSORS);
    // the persistent step (one launch, train_dag.hip) unless configured off, a side stream was
    // asked for, or this configuration has no DAG form (then the launches below)
    TrainCfg& cfg = train_cfg();
    LDM_REQUIRE(cfg.form != LDM_TRAIN_DAG || side == nullptr || side == s, LDM_ENOSYS,
                "ldm_denoiser_train_step_adamw: the one-launch step (LDM_TRAIN_DAG, required) "
                "has no side-stream form");
    if ((side == nullptr || side == s) &&
        (cfg.form == LDM_TRAIN_DAG || (cfg.form == LDM_TRAIN_AUTO && dag_auto(B)))) {
        float h7[7];
        adamw_hyper(lr, beta1, beta2, eps_adam, weight_decay, step, h7);
        const int r = dag_step(w, sc, x0, eps, t, B, saved, grads, loss_out, tensors, n, h7,
                               d_hyper, cfg.spin, cfg.dbg, (hipStream_t)s);
        if (r == 0) {
            cfg.last = LDM_TRAIN_DAG;
            return 0;
        }
        if (r != 1) return r;
        LDM_REQUIRE(cfg.form != LDM_TRAIN_DAG, LDM_ENOSYS, "ldm_denoiser_train_step_adamw: no "
                    "one-launch form for this configuration (LDM_TRAIN_DAG was required)");
    }
    cfg.last = LDM_TRAIN_LAUNCHES;
    AdamSplit A;
    memset(&A, 0, sizeof(A));
    A.lr = lr; A.beta1 = beta1; A.beta2 = beta2; A.eps = eps_adam; A.wd = weight_decay;
    A.step = step;
    A.d_hyper = d_hyper;
    A.side = side == s ? nullptr : (hipStream_t)side;
    if (A.side) {
        LDM_TRY(fork_events(A.ev));
        int dev = 0, cus = 0;
        LDM_REQUIRE(hipGetDevice(&dev) == hipSuccess &&
                        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) ==
                            hipSuccess,
                    LDM_EINVAL, "train_step_adamw: device query failed");
        A.grid_cap = 2 * cus;
    }
    // batch of each tensor, matched by its gradient pointer
    for (int i = 0; i < n; ++i) {
        const float* g = tensors[i].g;
        bool b0 = g == grads->w_out;
        for (int k = 0; k < w->n_blocks; ++k) b0 = b0 || g == grads->w_blk[k];
        const bool b1 = g == grads->w_t1 || g == grads->w_t2 || g == grads->w_in;
        // without a side stream one launch after the bias sums (fewer launches, same bits)
        const int bi = !A.side ? 2 : b0 ? 0 : b1 ? 1 : 2;
        A.batch[bi][A.nb[bi]++] = &tensors[i];
    }
    const TrainWs L = layout(w, B, saved);
    hipStream_t st = (hipStream_t)s;
    const float nf = (float)B * (float)w->D;
    const StepHook hook = {adam_hook, &A};
    LDM_TRY(prep_inputs(w, L, x0, eps, t, sc, st));
    LDM_TRY(forward(w, L, eps, nullptr, 2.f / nf, st));
    LDM_TRY(backward(w, L, grads, nullptr, st, &hook));        // batches 0 and 1
    LDM_TRY(finalize(L, grads, nullptr, loss_out, 1.f / nf, st));
    LDM_TRY(adam_batch(A, 2, st));
    if (A.side)
        LDM_REQUIRE(hipEventRecord(A.ev[kForks], A.side) == hipSuccess &&
                        hipStreamWaitEvent(st, A.ev[kForks], 0) == hipSuccess,
                    LDM_EINVAL, "train_step_adamw: join failed");
    return 0;
}

extern "C" void ldm_adamw_hyper(double lr, double beta1, double beta2, double eps,
                                double weight_decay, int step, float* out7) {
    ldm::adamw_hyper(lr, beta1, beta2, eps, weight_decay, step, out7);
}

extern "C" int ldm_train_step_config(int form, unsigned spin_limit) {
    LDM_REQUIRE(form >= LDM_TRAIN_AUTO && form <= LDM_TRAIN_DAG, LDM_EINVAL,
                "ldm_train_step_config: form %d", form);
    TrainCfg& c = train_cfg();
    c.form = form;
    c.spin = spin_limit;
    return 0;
}

extern "C" int ldm_train_step_last_form(void) { return train_cfg().last; }

extern "C" int ldm_denoiser_train_status(const ldm_denoiser_t* w, int B, void* saved,
                                         unsigned* status_host, ldm_stream_t s) {
    LDM_REQUIRE(w && B >= 1 && saved && status_host && w->n_blocks >= 1 &&
                    w->n_blocks <= LDM_MAX_BLOCKS,
                LDM_EINVAL, "ldm_denoiser_train_status: bad arguments");
    const TrainWs L = layout(w, B, saved);
    unsigned* st = L.dag_sync + dag::kSyncStatus * dag::kCtrStride;
    hipStream_t hs = (hipStream_t)s;
    hipError_t e = hipMemcpyAsync(status_host, st, sizeof(unsigned), hipMemcpyDeviceToHost, hs);
    if (e == hipSuccess) e = hipStreamSynchronize(hs);
    if (e == hipSuccess && *status_host != 0)       // every word cleared for the next launch
        e = hipMemsetAsync(L.dag_sync, 0, dag::sync_bytes(dag::kMaxCounters), hs);
    if (e == hipSuccess) e = hipStreamSynchronize(hs);
    LDM_REQUIRE(e == hipSuccess, (int)e, "ldm_denoiser_train_status: %s", hipGetErrorString(e));
    return 0;
}

extern "C" int ldm_denoiser_train_ws_init(const ldm_denoiser_t* w, int B, void* saved,
                                          ldm_stream_t s) {
    LDM_REQUIRE(w && B >= 1 && saved && w->n_blocks >= 1 && w->n_blocks <= LDM_MAX_BLOCKS,
                LDM_EINVAL, "ldm_denoiser_train_ws_init: bad arguments");
    const TrainWs L = layout(w, B, saved);
    {
        DagCache& dc = dag_cache();
        std::lock_guard<std::mutex> g(dc.mu);
        auto it = dc.by_table.find(L.dag_table);
        if (it != dc.by_table.end()) dc.by_table.erase(it);     // re-built by the next step
    }
    const hipError_t e =
        hipMemsetAsync(L.dag_sync, 0, dag::sync_bytes(dag::kMaxCounters), (hipStream_t)s);
    LDM_REQUIRE(e == hipSuccess, (int)e, "ldm_denoiser_train_ws_init: %s", hipGetErrorString(e));
    return 0;
}

// Diagnostics: the job table a step of this configuration runs, as text (one line per node:
// type, jobs, k-steps, k-group period, counters, dependencies; then the queue lengths), built
// on the host exactly as the step builds it.  Returns 1 if the configuration has no DAG form.
extern "C" int ldm_denoiser_train_dag_describe(const ldm_denoiser_t* w, const ldm_sched_t* sc,
                                               int B, void* saved,
                                               const ldm_denoiser_grads_t* grads,
                                               const ldm_adamw_tensor_t* tensors, int n,
                                               char* buf, size_t len) {
    LDM_TRY(check_desc(w, B, true));
    LDM_TRY(check_grads(w, grads));
    LDM_REQUIRE(sc && saved && buf && len > 0 && tensors && n >= 1 &&
                    n <= LDM_ADAMW_MAX_TENSORS, LDM_EINVAL,
                "ldm_denoiser_train_dag_describe: bad arguments");
    const TrainWs L = layout(w, B, saved);
    int grid = 0;
    if (dag::dag_grid(&grid) != 0) grid = -1;        // (no device: the table alone)
    DagHost* h = new DagHost();
    const int r = build_dag(w, sc, L, grads, tensors, n, (float)B * (float)w->D, grid, *h);
    if (r != 0) {
        delete h;
        return r;
    }
    const dag::Table& T = h->tab;
    static const char* kType[] = {"gemm", "prep", "sum", "adam"};
    size_t o = 0;
#define put(...) (o < len ? (void)(o += (size_t)snprintf(buf + o, len - o, __VA_ARGS__)) : (void)0)
    put("grid %d nodes %d counters %d entries %d\n", T.grid, T.n_nodes, T.n_counters,
        T.n_entries);
    for (int i = 0; i < T.n_nodes; ++i) {
        const dag::Node& nd = T.node[i];
        put("%d %s %dx%d nk %d kgp %d band %d all %d sig %d wt %d deps", i, kType[nd.type],
            nd.tiles_m, nd.tiles_n, nd.nk, nd.kgp, nd.out_band, nd.out_all, nd.signal, nd.stat);
        for (int d = 0; d < nd.ndep; ++d)
            put(" [%d%s>=%u]", nd.dep_ctr[d], nd.dep_band[d] ? "+band" : "", nd.dep_target[d]);
        put("\n");
    }
    for (int q = 0; q < dag::kQueues; ++q) put("queue %d: %d jobs at %d\n", q, T.qlen[q], T.qoff[q]);
    for (int q = 0; q < 2 * dag::kQueues; ++q)
        put("claim list %d: %d jobs at %d\n", q, T.qlen2[q], T.qoff2[q]);
#undef put
    delete h;
    return 0;
}

#ifdef LDM_DEV_KNOBS
// Development build only (`make DEV=1`; not in include/ldm_sdf.h, not exported by the product
// library): skip the compute of DAG node types (bit t: type t of train_dag.h NodeType; the jobs
// still wait and signal), add the release / acquire fences to every hand-off (bit 7,
// dag::kDbgFences), the claim scheduler (kDbgClaim), weight operands through the L2
// (kDbgWeightsL2).
extern "C" int ldm_dev_train_dag_flags(unsigned flags) {
    train_cfg().dbg = flags;
    return 0;
}
#endif
