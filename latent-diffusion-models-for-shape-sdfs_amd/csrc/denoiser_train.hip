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

#include <math.h>
#include <string.h>

namespace ldm {

int gemm_bf16(const ldm_gemm_args_t& a, hipStream_t s);

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
int launch(std::initializer_list<ldm_gemm_prob_t> ps, hipStream_t s) {
    ldm_gemm_args_t a;
    memset(&a, 0, sizeof(a));
    for (const auto& p : ps) a.prob[a.n_prob++] = p;
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
            float* eps_out, float loss_scale, hipStream_t s) {
    const int Bp = L.Bp, B = L.B, D = L.D, H = L.H, TE = L.TE;
    ldm_gemm_prob_t f1 = prob(Bp, H, B);                         // u = SiLU(Wt1 e + bt1)
    seg(f1, L.e_b, TE, w->w_t1, TE, TE);
    f1.mode = LDM_GEMM_SILU; f1.bias = w->b_t1;
    f1.P = L.a_t; f1.ldp = H; f1.Cb = L.u_b; f1.ldcb = H; f1.CbT = L.u_T; f1.ldct = Bp;
    ldm_gemm_prob_t f3 = prob(Bp, H, B);                         // h0 = Win xt + bin
    seg(f3, L.xt_b, D, w->w_in, D, D);
    f3.bias = w->b_in;
    f3.C = L.h_f[0]; f3.ldc = H; f3.Cb = L.h_b[0]; f3.ldcb = H; f3.CbT = L.h_T[0]; f3.ldct = Bp;
    LDM_TRY(launch({f1, f3}, s));
    ldm_gemm_prob_t f2 = prob(Bp, H, B);                         // temb = Wt2 u + bt2
    seg(f2, L.u_b, H, w->w_t2, H, H);
    f2.bias = w->b_t2;
    f2.Cb = L.temb_b; f2.ldcb = H; f2.CbT = L.temb_T; f2.ldct = Bp;
    LDM_TRY(launch({f2}, s));
    const bf16_t* const* Wb = reinterpret_cast<const bf16_t* const*>(w->w_blk);
    for (int k = 0; k < L.nb; ++k) {                              // h <- h + SiLU([h||temb] Wblk^T + b)
        ldm_gemm_prob_t fb = prob(Bp, H, B);
        seg(fb, L.h_b[k], H, Wb[k], 2 * H, H);
        seg(fb, L.temb_b, H, Wb[k] + H, 2 * H, H);
        fb.mode = LDM_GEMM_RESID_SILU; fb.bias = w->b_blk[k];
        fb.R = L.h_f[k]; fb.ldr = H; fb.P = L.a_f[k]; fb.ldp = H;
        if (k + 1 < L.nb) { fb.C = L.h_f[k + 1]; fb.ldc = H; }
        fb.Cb = L.h_b[k + 1]; fb.ldcb = H; fb.CbT = L.h_T[k + 1]; fb.ldct = Bp;
        LDM_TRY(launch({fb}, s));
    }
    if (eps_target) {                                            // eps_hat -> eps-MSE gradient
        ldm_gemm_prob_t fo = prob(Bp, D, B);
        seg(fo, L.h_b[L.nb], H, w->w_out, H, H);
        fo.mode = LDM_GEMM_LOSS; fo.bias = w->b_out; fo.scale = loss_scale;
        fo.P_in = eps_target; fo.ldp_in = D;
        fo.Cb = L.go_b; fo.ldcb = D; fo.CbT = L.go_T; fo.ldct = Bp;
        fo.colsum = L.p_bout; fo.loss_part = L.loss_part;
        LDM_TRY(launch({fo}, s));
    } else if (eps_out) {
        ldm_gemm_prob_t fo = prob(Bp, D, B);
        seg(fo, L.h_b[L.nb], H, w->w_out, H, H);
        fo.bias = w->b_out; fo.C = eps_out; fo.ldc = D;
        LDM_TRY(launch({fo}, s));
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
             float* dx, hipStream_t s, const StepHook* hook = nullptr) {
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
        LDM_TRY(launch({dwo, dh}, s));
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
        LDM_TRY(launch({dw, du, dh}, s));
        cur ^= 1;
    }
    {
        ldm_gemm_prob_t dt = prob(Bp, H, B);                     // dtemb = sum_k g_k U_k
        for (int k = 0; k < nb; ++k) seg(dt, L.g_b[k], H, Wt[k] + (size_t)H * H, H, H);
        dt.Cb = L.dtemb_b; dt.ldcb = H; dt.CbT = L.dtemb_T; dt.ldct = Bp;
        dt.colsum = L.p_bt2;
        // alone in its launch: 256 tiles, every K a multiple of 128 -> the 128-deep 2-group
        // tile (with dWin's 64 tiles beside it the launch fell to 64 x 64 tiles: 30.8 us)
        LDM_TRY(launch({dt}, s));
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
        LDM_TRY(launch({dw2, gt}, s));
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
            LDM_TRY(launch({dw1, dwi, px}, s));
        } else {
            LDM_TRY(launch({dw1, dwi}, s));
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
    const TrainWs L = layout(w, B, saved);
    hipStream_t st = (hipStream_t)s;
    const float n = (float)B * (float)w->D;
    LDM_TRY(prep_inputs(w, L, x0, eps, t, sc, st));
    LDM_TRY(forward(w, L, eps, nullptr, 2.f / n, st));
    LDM_TRY(backward(w, L, grads, nullptr, st));
    return finalize(L, grads, nullptr, loss_out, 1.f / n, st);
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
template <typename KJ>
__device__ __forceinline__ void adamw_tile(KJ* kj, unsigned short (&sT)[64][64 + 8], int tile);

__global__ __launch_bounds__(256) void adamw_multi_kernel(AdamJobs jobs) {
    typedef KJobs KJ;
    KJ* kj = (KJ*)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ unsigned short sT[64][64 + 8];
    // grid-stride over the tiles: a capped grid leaves wave slots free on every CU for work on
    // another stream (ldm_denoiser_train_step_adamw); uncapped, one tile per workgroup
    for (int tile = blockIdx.x; tile < kj->first[kj->n]; tile += gridDim.x) {
        __syncthreads();                   // the previous tile's transposed reads of sT are done
        adamw_tile(kj, sT, tile);
    }
}

template <typename KJ>
__device__ __forceinline__ void adamw_tile(KJ* kj, unsigned short (&sT)[64][64 + 8], int tile) {
    int j = 0;
    for (int i = 1; i < kj->n; ++i)
        if (tile >= kj->first[i]) j = i;
    const __attribute__((address_space(4))) ldm_adamw_tensor_t& T = kj->t[j];
    const int rows = T.rows, cols = T.cols;
    const int tl = tile - kj->first[j], tcn = (cols + 63) / 64;
    const int r0 = (tl / tcn) * 64, c0 = (tl % tcn) * 64;
    const int tid = threadIdx.x;
    const int cq = (tid & 15) * 4;
    const float* dh = kj->dh;
    const float decay = dh ? dh[0] : kj->decay, omb1 = dh ? dh[1] : kj->omb1;
    const float b2 = dh ? dh[2] : kj->b2, omb2 = dh ? dh[3] : kj->omb2;
    const float eps = dh ? dh[4] : kj->eps, step_size = dh ? dh[5] : kj->step_size;
    const float bc2_sqrt = dh ? dh[6] : kj->bc2_sqrt;
    float* __restrict__ P = T.p;
    const float* __restrict__ Gp = T.g;
    float* __restrict__ M = T.m;
    float* __restrict__ V = T.v;
    // every load of the thread's 4 rows x 4 columns first (16-byte vectors when the row is
    // aligned and whole), then the updates, then the stores: one memory round trip
    const bool vec = (cols & 3) == 0 && c0 + cq + 4 <= cols;
    f32x4 p4[4], g4[4], m4[4], v4[4];
    int64_t off[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = min(r0 + (tid >> 4) + 16 * i, rows - 1);
        off[i] = (int64_t)r * cols + c0 + cq;
        if (vec) {
            p4[i] = *reinterpret_cast<const f32x4*>(P + off[i]);
            g4[i] = *reinterpret_cast<const f32x4*>(Gp + off[i]);
            m4[i] = *reinterpret_cast<const f32x4*>(M + off[i]);
            v4[i] = *reinterpret_cast<const f32x4*>(V + off[i]);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t x = c0 + cq + e < cols ? off[i] + e : off[i];
                p4[i][e] = P[x]; g4[i][e] = Gp[x]; m4[i][e] = M[x]; v4[i][e] = V[x];
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rl = (tid >> 4) + 16 * i;
        const bool rin = r0 + rl < rows;
        unsigned short q[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float pi = p4[i][e], mi = m4[i][e], vi = v4[i][e];
            adamw_update(pi, g4[i][e], mi, vi, decay, omb1, b2, omb2, eps, step_size, bc2_sqrt);
            p4[i][e] = pi; m4[i][e] = mi; v4[i][e] = vi;
            const unsigned u = __builtin_bit_cast(unsigned, pi);
            q[e] = (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
            sT[cq + e][rl] = rin ? q[e] : (unsigned short)0;
        }
        if (!rin) continue;
        if (vec) {
            *reinterpret_cast<f32x4*>(P + off[i]) = p4[i];
            *reinterpret_cast<f32x4*>(M + off[i]) = m4[i];
            *reinterpret_cast<f32x4*>(V + off[i]) = v4[i];
            if (T.p_bf16) {
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 w = {(unsigned)q[0] | ((unsigned)q[1] << 16),
                                 (unsigned)q[2] | ((unsigned)q[3] << 16)};
                *reinterpret_cast<u32x2*>(reinterpret_cast<unsigned short*>(T.p_bf16) + off[i]) = w;
            }
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (c0 + cq + e >= cols) continue;
                P[off[i] + e] = p4[i][e]; M[off[i] + e] = m4[i][e]; V[off[i] + e] = v4[i][e];
                if (T.p_bf16) reinterpret_cast<unsigned short*>(T.p_bf16)[off[i] + e] = q[e];
            }
        }
    }
    if (!T.p_bf16_t) return;
    __syncthreads();
    // transposed: [c][r], 16 consecutive rows per thread (4 threads per column)
    const int cl = tid >> 2, rb = (tid & 3) * 16;
    const int c = c0 + cl;
    if (c >= cols) return;
    unsigned short* dst = reinterpret_cast<unsigned short*>(T.p_bf16_t) + (int64_t)c * rows;
    if ((rows & 7) == 0 && r0 + rb + 16 <= rows) {
        u32x4 w0, w1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            w0[e] = (unsigned)sT[cl][rb + 2 * e] | ((unsigned)sT[cl][rb + 2 * e + 1] << 16);
            w1[e] = (unsigned)sT[cl][rb + 8 + 2 * e] | ((unsigned)sT[cl][rb + 9 + 2 * e] << 16);
        }
        *reinterpret_cast<u32x4*>(dst + r0 + rb) = w0;
        *reinterpret_cast<u32x4*>(dst + r0 + rb + 8) = w1;
    } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int r = r0 + rb + e;
            if (r < rows) dst[r] = sT[cl][rb + e];
        }
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
