/*
 * ldm_sdf.h -- C ABI of libldm_sdf.so, the MI355X (gfx950) hot path of latent diffusion
 * over DeepSDF shape codes.
 *
 * The reference project (SGI-2022/Latent-Diffusion-Models-for-Shape-SDFs) ships no code:
 * /root/reference/README.md:1 is its only line, so it has no FFI to mirror.  Every entry
 * point below is the build-defined boundary of SURVEY.md §8(b); each cites the §8(a) row it
 * implements (and, for the Python side, the ldm_sdf/api.py function that calls it).
 *
 * Conventions:
 *   - All buffers are caller-owned DEVICE pointers (torch tensors), contiguous, 16-byte aligned
 *     (the shim checks alignment).  The library never allocates or frees device memory.
 *   - Every launch is asynchronous on the caller's stream; no hidden synchronisation, no
 *     hipMalloc / hipMemcpy (so calls can be captured into a hipGraph).  Exceptions, each
 *     documented at its declaration: the *_status reads synchronise the stream.
 *   - Return 0 on success, a negative LDM_E* code for an argument error, or a positive
 *     hipError_t.  ldm_last_error() returns a thread-local message for the last failure.
 *   - One device per process (the current HIP device, as set by torch).
 */
#ifndef LDM_SDF_H
#define LDM_SDF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDM_ABI_VERSION 7

/* dtypes */
#define LDM_F32 0
#define LDM_BF16 1
#define LDM_F16 2

/* argument errors */
#define LDM_EINVAL (-22)
#define LDM_EALIGN (-14)
#define LDM_ENOSYS (-38)
#define LDM_ENOSPC (-28)

/* workspace ops for ldm_workspace_bytes() */
#define LDM_OP_DECODER_GRID 1
#define LDM_OP_DECODER_POINTS 2
/* ldm_workspace_bytes() returns the need of the (one) 16-bit layout, LDM_LAYOUT_SPLIT;
   ldm_workspace_bytes_layout() gives a layout's own size (0 for removed layouts) */

typedef void* ldm_stream_t; /* hipStream_t; NULL = the null stream */

/*
 * DeepSDF decoder weights, packed on the host by ldm_sdf/pack.py.
 * The hot kernels support hidden == 512 with 8 hidden layers and the latent re-injected at
 * layer 4 (DeepSDF); skip_width is the output width of layer 3: 253 (DeepSDF, L=256) or 512
 * (the "widen-skip" variant used for L >= H, config 5).  Layouts: DESIGN.md §3.
 */
typedef struct ldm_decoder {
    int32_t abi_version;  /* must equal LDM_ABI_VERSION */
    int32_t dtype;        /* LDM_F32 (parity kernel) / LDM_BF16 / LDM_F16 (MFMA kernel) */
    int32_t hidden;       /* H (512) */
    int32_t skip_width;   /* 253 or 512 */
    int32_t latent_dim;   /* L */
    int32_t n_stages;     /* bf16/f16: k-steps of one wave's weight stream (384 / 448 at skip
                             width 253 / 512); f32: 0 */
    const void* weights;  /* bf16/f16: per-wave stream blob (ldm_sdf/pack.py pack_split,
                             DESIGN.md §4); f32: fp32 blob */
    const float* wz;      /* fp32 [2][H][L]  latent columns of layer 0 and layer 4 */
    const float* bz;      /* fp32 [2][H]     biases of layer 0 and layer 4 */
    const float* wxyz;    /* fp32 [2][H][3]  xyz columns of layer 0 and layer 4 */
    const float* w_last;  /* fp32 [H] final 512->1 weights (bf16/f16: MFMA-row permuted) */
    float b_last;         /* final bias */
    int32_t layout;       /* bf16/f16 weight layout: LDM_LAYOUT_SPLIT */
} ldm_decoder_t;

/* Stage-blob layouts of the MFMA decoder. */
#define LDM_LAYOUT_PASS8 0   /* removed in ABI 5 (superseded by SPLIT): LDM_ENOSYS */
#define LDM_LAYOUT_QUARTER 1 /* removed in ABI 5 (superseded by SPLIT): LDM_ENOSYS */
#define LDM_LAYOUT_SPLIT 2   /* features split over the 4 waves, per-wave weight streams */
#define LDM_LAYOUT_SPLIT16 3 /* removed in ABI 7 (5.5 % slower than SPLIT): LDM_ENOSYS */

/* DDPM tables, fp32 device arrays of length T. */
typedef struct ldm_sched {
    int32_t abi_version;
    int32_t T;
    const float* sqrt_ab;   /* sqrt(abar_t) */
    const float* sqrt_1mab; /* sqrt(1 - abar_t) */
    const float* c1;        /* 1/sqrt(alpha_t) */
    const float* c2;        /* beta_t / sqrt(1 - abar_t) */
    const float* sigma;     /* sqrt(beta_t) */
} ldm_sched_t;

#define LDM_MAX_BLOCKS 8

/*
 * MLP denoiser (ldm_sdf/models.py MLPDenoiser).
 * Weights are [out][in] row-major in `dtype` (LDM_F32 or LDM_BF16); biases fp32.
 * w_blk[k] is [H][2H] = [W_k | U_k] acting on [h || temb].
 * e_tab[k] (inference only) is fp32 [T][H] = U_k temb(t) + b_k for every t.
 */
typedef struct ldm_denoiser {
    int32_t abi_version;
    int32_t dtype;
    int32_t D, H, n_blocks, TE, T;
    int32_t reserved;
    const void* w_in;   const float* b_in;    /* [H][D] */
    const void* w_t1;   const float* b_t1;    /* [H][TE] */
    const void* w_t2;   const float* b_t2;    /* [H][H] */
    const void* w_blk[LDM_MAX_BLOCKS];
    const float* b_blk[LDM_MAX_BLOCKS];       /* [H] */
    const float* e_tab[LDM_MAX_BLOCKS];       /* [T][H] */
    const void* w_out;  const float* b_out;   /* [D][H] */
    const float* emb_table;                   /* [T][TE] sinusoidal (A5) */
    /* bf16 training only (ldm_denoiser_fwd / _bwd / _train_step): TRANSPOSED bf16 copies the
     * backward's G W products read k-contiguous, kept current by ldm_adamw_multi. */
    const void* wt_in;                        /* [D][H]  = w_in^T  (only for dx)      */
    const void* wt_t2;                        /* [H][H]  = w_t2^T                     */
    const void* wt_blk[LDM_MAX_BLOCKS];       /* [2H][H] = w_blk[k]^T                 */
    const void* wt_out;                       /* [H][D]  = w_out^T                    */
} ldm_denoiser_t;

/* fp32 tensors with the denoiser's parameter shapes (gradients, masters, Adam moments). */
typedef struct ldm_denoiser_grads {
    float* w_in;  float* b_in;                /* [H][D], [H]   */
    float* w_t1;  float* b_t1;                /* [H][TE], [H]  */
    float* w_t2;  float* b_t2;                /* [H][H], [H]   */
    float* w_blk[LDM_MAX_BLOCKS];             /* [H][2H]       */
    float* b_blk[LDM_MAX_BLOCKS];             /* [H]           */
    float* w_out; float* b_out;               /* [D][H], [D]   */
} ldm_denoiser_grads_t;

/* ---- library -------------------------------------------------------------------------- */
int ldm_abi_version(void);
const char* ldm_last_error(void);
/* Device bytes of workspace an op needs (B shapes, n = N (grid) or P (points)). */
size_t ldm_workspace_bytes(int op, int B, int n, int dtype);
size_t ldm_workspace_bytes_layout(int op, int B, int n, int dtype, int layout);

/* ---- decoder: A1 grid coords, A2 latent fold, A3 fused MLP ----------------------------- */
/* A1 standalone: xyz_out fp32 [(k1-k0)*N*N][3], z slowest, x fastest, x = fl32(fl32(i*vs)+origin). */
int ldm_grid_coords(int N, int k0, int k1, float vs, float origin, float* xyz_out,
                    ldm_stream_t s);
/* A2: beta_out fp32 [B][2][H]; z fp32 [B][L]. */
int ldm_decoder_fold(const ldm_decoder_t* w, const float* z, int B, float* beta_out,
                     ldm_stream_t s);
/* out[0] (device) = max over shapes b of sqrt(mean_l z[b][l]^2), z fp32 [B][L]: the latent
 * scale the Python decode's dtype="auto" picks its 16-bit format by. */
int ldm_latent_rms_max(const float* z, int B, int L, float* out, ldm_stream_t s);
/* A1+A3 grid mode: out fp32 [B][(k1-k0)*N*N] (the z-slab [k0,k1) of each shape's N^3 grid). */
int ldm_decoder_grid_fwd(const ldm_decoder_t* w, const float* beta, int B, int N, int k0,
                         int k1, float vs, float origin, float* out, void* ws,
                         size_t ws_bytes, ldm_stream_t s);
/* A3 point-list mode: xyz fp32 [B][P][3] -> out fp32 [B][P]. */
int ldm_decoder_points_fwd(const ldm_decoder_t* w, const float* beta, const float* xyz,
                           int B, int P, float* out, void* ws, size_t ws_bytes,
                           ldm_stream_t s);

/* ---- DDPM: A8 reverse step, A9 q_sample + eps-MSE ------------------------------------ */
/* x_out[i] = c1[t]*(x[i] - c2[t]*eps[i]) + sigma[t]*z[i]  (z ignored at t == 0). n elements. */
int ldm_ddpm_step(const ldm_sched_t* sc, const float* x, const float* eps, const float* z,
                  int t, int n, float* x_out, ldm_stream_t s);
/* x_t[b][d] = sqrt_ab[t_b] x0 + sqrt_1mab[t_b] eps.  t int32 [B]. */
int ldm_q_sample(const ldm_sched_t* sc, const float* x0, const float* eps, const int32_t* t,
                 int B, int D, float* xt_out, ldm_stream_t s);
/* loss_out[0] = mean((eps_hat - eps)^2); grad_out = d loss / d eps_hat (may be NULL). */
int ldm_eps_mse_loss(const float* eps_hat, const float* eps, int n, float* loss_out,
                     float* grad_out, ldm_stream_t s);

/* ---- denoiser: A6 forward (sampling: uniform t) and the sampling step ------------------ */
/* eps_out fp32 [B][D] = net(x, t) for one timestep t shared by the batch (B <= 16), using
 * the tabulated e_tab.  ws: fp32 scratch of at least 2*B*H floats. */
int ldm_denoiser_fwd_uniform_t(const ldm_denoiser_t* w, const float* x, int t, int B,
                               float* eps_out, float* ws, ldm_stream_t s);
/* One DDPM reverse step fused with the denoiser (A6 + A8, the A10 loop body):
 * x_out = c1[t] (x - c2[t] net(x,t)) + sigma[t] z  (z ignored at t = 0).  x_out != x. */
int ldm_sample_step(const ldm_denoiser_t* w, const ldm_sched_t* sc, const float* x,
                    const float* z, int t, int B, float* x_out, float* ws, ldm_stream_t s);
/* The whole A10 loop as one persistent launch (whole grid resident): steps t_hi, t_hi-1, ...,
 * t_hi-steps+1 of ldm_sample_step, bit-identical to calling it per step.  x fp32 [2][B][D]
 * ping-pong with x[0] = x_T on entry; the result is x[steps & 1].  noise fp32 [T][B][D]
 * (noise[t] is the z of step t).  ws: ldm_sample_loop_ws_bytes(B, H) bytes, 256-byte aligned.
 * LDM_ENOSYS unless ldm_sample_loop_supported(w, B) (H = 1024, D in {256, 512}, 4 blocks,
 * B <= 16, and H/4 workgroups co-resident on the current device); callers then use
 * ldm_sample_step.  Every grid barrier is bounded: after the launch,
 * ldm_sample_loop_status() reads back 0 (completed) or 1 (abandoned on a timeout). */
int ldm_sample_loop_supported(const ldm_denoiser_t* w, int B);
size_t ldm_sample_loop_ws_bytes(int B, int H);
int ldm_sample_loop(const ldm_denoiser_t* w, const ldm_sched_t* sc, float* x, const float* noise,
                    int t_hi, int steps, int B, float* ws, size_t ws_bytes, ldm_stream_t s);
int ldm_sample_loop_status(const float* ws, int B, int H, unsigned* status_host, ldm_stream_t s);
/* Loop forms.  AUTO (default): the XCD-replica loop when the shape has it (bf16, status 2 on a
 * placement mismatch switches the device to XCD for good), else XCD. */
#define LDM_LOOP_AUTO 0
#define LDM_LOOP_REPLICA 1 /* one network copy per XCD, XCD-local tagged hand-offs */
#define LDM_LOOP_XCD 2     /* chip-wide loop, XCD-hierarchical grid barrier */
#define LDM_LOOP_DIRECT 3  /* chip-wide loop, hierarchical arrival, chip-wide polling */
#define LDM_LOOP_FLAT 4    /* chip-wide loop, one flat counter */
/* Explicit A/B and fault-injection control of ldm_sample_loop on the current device (the
 * library reads no environment variable): form LDM_LOOP_*, spin_limit (0 = default; a tiny
 * limit makes barriers give up, i.e. status 1), tagged (replica hand-offs: 1 = tagged
 * granules, default; 0 = XCD-local barriers).  Defaults: (LDM_LOOP_AUTO, 0, 1). */
int ldm_sample_loop_config(int form, unsigned spin_limit, int tagged);
/* The form the last ldm_sample_loop launch on the current device took (LDM_LOOP_REPLICA ..
 * LDM_LOOP_FLAT; 0 before any launch). */
int ldm_sample_loop_last_form(void);

/* ---- A6/A7/A9 training: denoiser forward with saved activations, backward, fused step ----
 * bf16 weights (w->dtype == LDM_BF16, the wt_* transposed copies set), matrix-core GEMMs
 * (ldm_gemm_bf16) with bf16 operands and fp32 accumulation, per-sample timesteps t int32 [B].
 * `saved` is a device workspace of ldm_denoiser_train_ws_bytes(w, B) bytes (256-B aligned):
 * the forward writes every activation the backward reads (bf16 GEMM operands in both layouts,
 * fp32 residual stream and pre-activations); its contents are opaque.  Gradients are fp32 in
 * the parameter shapes (ldm_denoiser_grads_t), overwritten (not accumulated).  Deterministic:
 * fixed reduction orders, no atomics.  D, H, TE multiples of 64; n_blocks 1..8. */
size_t ldm_denoiser_train_ws_bytes(const ldm_denoiser_t* w, int B);
/* eps_out fp32 [B][D] = net(x, t) (may be NULL when only the saved activations are wanted). */
int ldm_denoiser_fwd(const ldm_denoiser_t* w, const float* x, const int32_t* t, int B,
                     float* eps_out, void* saved, ldm_stream_t s);
/* Given deps = dL/d eps_hat fp32 [B][D] for the last ldm_denoiser_fwd on `saved`: every
 * parameter gradient, and dx = dL/dx fp32 [B][D] when dx != NULL. */
int ldm_denoiser_bwd(const ldm_denoiser_t* w, void* saved, const float* deps, int B,
                     const ldm_denoiser_grads_t* grads, float* dx, ldm_stream_t s);
/* A9 head.  xt_out (if not NULL) = sqrt(abar[t]) x0 + sqrt(1 - abar[t]) eps (bit-exact with the
 * fp32 oracle); eps_hat (if not NULL): loss_out[0] = mean((eps_hat - eps)^2) and grad_out (if
 * not NULL) = d loss / d eps_hat = 2 (eps_hat - eps) / (B D). */
int ldm_q_sample_loss(const ldm_sched_t* sc, const float* x0, const float* eps,
                      const int32_t* t, int B, int D, float* xt_out, const float* eps_hat,
                      float* loss_out, float* grad_out, ldm_stream_t s);
/* One whole DDPM training step's forward + backward (Alg. 1 without the optimizer):
 * q_sample -> net -> eps-MSE (loss_out[0]) -> every gradient, the loss gradient fused into
 * the out-projection's epilogue.  The data-parallel step (the update waits for the gradient
 * all-reduce).  Form per ldm_train_step_config: the launch path (17 launches, no host
 * synchronisation, graph-capturable) or the one-launch job DAG without AdamW nodes (its first
 * call per configuration uploads the table: one stream synchronisation, not inside a capture);
 * the same bits either way. */
int ldm_denoiser_train_step(const ldm_denoiser_t* w, const ldm_sched_t* sc, const float* x0,
                            const float* eps, const int32_t* t, int B, void* saved,
                            const ldm_denoiser_grads_t* grads, float* loss_out, ldm_stream_t s);

/* ---- optimizer (A7 training step) -------------------------------------------------------- */
/* Multi-tensor AdamW in ONE launch (torch.optim.AdamW's update order, as ldm_adamw_step):
 * per tensor fp32 p, g, m, v [rows][cols]; optional bf16 working copies p_bf16 [rows][cols]
 * and p_bf16_t [cols][rows] (transposed, for the backward's k-contiguous operands), rounded to
 * nearest even.  `tensors` is a HOST array of n <= LDM_ADAMW_MAX_TENSORS descriptors. */
#define LDM_ADAMW_MAX_TENSORS 40
typedef struct ldm_adamw_tensor {
    float* p; const float* g; float* m; float* v;
    void* p_bf16; void* p_bf16_t;
    int32_t rows, cols;
} ldm_adamw_tensor_t;
int ldm_adamw_multi(const ldm_adamw_tensor_t* tensors, int n, double lr, double beta1,
                    double beta2, double eps, double weight_decay, int step, ldm_stream_t s);
/* One whole single-rank training step: ldm_denoiser_train_step, then ldm_adamw_multi over
 * `tensors` (hyper-parameters as there; eps_adam is AdamW's eps).  The updates run in three
 * batches, each as soon as its gradients are final and no later launch of the step reads its
 * weights (matched by gradient pointer): grads->w_out / w_in / w_blk[k] after the backward's
 * dtemb launch, w_t1 / w_t2 after its last GEMM, everything else after the bias sums.  With a
 * `side` stream the batches run there behind fork events, on a grid capped at 2 workgroups per
 * CU, overlapping the backward's tail; s then waits for side.  side == NULL or == s: all in
 * order on s, one AdamW launch after the bias sums.  Results are those of the two calls in
 * sequence, bit for bit (each update reads only its own tensor's final gradient).  Measured
 * (DESIGN.md §5): the overlap does NOT pay at config 2 -- the HBM-bound AdamW slows the
 * latency-bound GEMMs beside it more than it hides -- so ldm_sdf.train passes side = NULL.  A data-parallel step needs the gradient all-reduce
 * in between: use the two calls there. */
int ldm_denoiser_train_step_adamw(const ldm_denoiser_t* w, const ldm_sched_t* sc,
                                  const float* x0, const float* eps, const int32_t* t, int B,
                                  void* saved, const ldm_denoiser_grads_t* grads,
                                  float* loss_out, const ldm_adamw_tensor_t* tensors, int n,
                                  double lr, double beta1, double beta2, double eps_adam,
                                  double weight_decay, int step, const float* d_hyper,
                                  ldm_stream_t s, ldm_stream_t side);
/* The whole step in ONE persistent launch (round 5, ABI 7; csrc/train_dag.hip):
 * with side == NULL (or == s), ldm_denoiser_train_step_adamw runs the step's job DAG -- input
 * preparation, every GEMM tile of the launch path with the same epilogues, the bias sums and every
 * AdamW tile -- in one launch whose workgroups take jobs as their inputs become ready (per 64-row
 * band for the residual chain, per problem for weight gradients and updates).  Results are those
 * of the launch path bit for bit.  The first call for a (descriptor, workspace, gradients, AdamW
 * table, B) configuration builds its job table on the host and uploads it into `saved` (one
 * stream synchronisation; not inside a graph capture); later calls launch at once.  Waits are
 * bounded: ldm_denoiser_train_status reads (and clears) the status word of `saved`: 0 ok, 1 a
 * wait timed out (the step's results are garbage), 3 the table in `saved` was built for other
 * inputs (nothing computed).  ldm_train_step_config selects the form per device:
 * LDM_TRAIN_AUTO (default: the form measured faster for the configuration, DESIGN.md §5 --
 * ldm_train_step_last_form tells which ran), LDM_TRAIN_LAUNCHES (the launch path), LDM_TRAIN_DAG
 * (required: LDM_ENOSYS otherwise); spin_limit: microseconds one dependency wait may take before
 * the launch gives up (0 = default, 2 s). */
#define LDM_TRAIN_AUTO 0
#define LDM_TRAIN_LAUNCHES 1
#define LDM_TRAIN_DAG 2
int ldm_train_step_config(int form, unsigned spin_limit);
int ldm_train_step_last_form(void);   /* the form the last step on this device ran (0: none) */
int ldm_denoiser_train_status(const ldm_denoiser_t* w, int B, void* saved, unsigned* status_host,
                              ldm_stream_t s);
/* Call once on a NEW `saved` workspace (fresh allocation) before its first one-launch step:
 * zeroes its sync words (on s) and drops the host's record of a job table uploaded to that
 * address.  The record is keyed by address and inputs, so a workspace allocated where a freed
 * one lay -- with the same descriptor, gradient and AdamW pointers, as a caching allocator
 * hands out -- would otherwise be taken as holding its predecessor's table and sync words,
 * which other allocations may have overwritten since (the kernel then reports status 3). */
int ldm_denoiser_train_ws_init(const ldm_denoiser_t* w, int B, void* saved, ldm_stream_t s);
/* Diagnostics (host only, no device work): the job table of this configuration as text into
 * buf[len] -- per node its type, jobs, k-steps, counters and dependencies, then the queues.
 * 1: the configuration has no one-launch form. */
int ldm_denoiser_train_dag_describe(const ldm_denoiser_t* w, const ldm_sched_t* sc, int B,
                                    void* saved, const ldm_denoiser_grads_t* grads,
                                    const ldm_adamw_tensor_t* tensors, int n, char* buf,
                                    size_t len);
/* d_hyper (may be NULL): a DEVICE array of the 7 AdamW scalars ldm_adamw_hyper computes for
 * (lr, beta1, beta2, eps_adam, weight_decay, step); the kernels read them from there instead
 * of the arguments, so a hipGraph captured once replays every step (the caller refills it).
 * ldm_adamw_hyper: host-only, the scalars exactly as the argument path derives them
 * (double, rounded once): [1 - lr wd, 1 - beta1, beta2, 1 - beta2, eps, lr / (1 - beta1^step),
 * sqrt(1 - beta2^step)]. */
void ldm_adamw_hyper(double lr, double beta1, double beta2, double eps, double weight_decay,
                     int step, float* out7);
/* AdamW on fp32 masters p [n] with grads g, moments m, v (torch.optim.AdamW's order; step is
 * 1-based).  p_bf16 (may be NULL): bf16 [n] working copy of the updated p, written in the same
 * pass (RNE). */
int ldm_adamw_step(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n,
                   double lr, double beta1, double beta2, double eps, double weight_decay,
                   int step, ldm_stream_t s);

/* ---- generic fused linear (A6/A7 building block, training) ---------------------------- */
/* acc[b][m] = sum_{k<K} X[b][k] W[m][k]  +  sum_{k<K2} X2[b][k] W2[m][k]   (K2 may be 0)
 * with arbitrary element strides, so the forward (X W^T), input-gradient (G W) and
 * weight-gradient (G^T X) products -- and the block's [h || temb] [W_k | U_k]^T -- are all
 * this one call.  Epilogues (pre = acc + bias, bias optional):
 *   LDM_EPI_BIAS        Y = pre
 *   LDM_EPI_SILU        Y = SiLU(pre);      A_out = pre (if A_out)
 *   LDM_EPI_RESID_SILU  Y = R + SiLU(pre);  A_out = pre (if A_out)      (A6 block)
 *   LDM_EPI_ACCUM       Y = Y + pre
 *   LDM_EPI_ADD_R       Y = R + pre                                     (A7 dh = dy + W^T g)
 *   LDM_EPI_RELU        Y = max(pre, 0)                    (C19 decoder hidden layers)
 *   LDM_EPI_MASK_R      Y = R > 0 ? pre : 0   (C19: ReLU backward through the post-activation
 *                                              R, fused into the G W product)
 * w_dtype: LDM_F32 or LDM_BF16 (elements of W and W2). */
#define LDM_EPI_BIAS 0
#define LDM_EPI_SILU 1
#define LDM_EPI_RESID_SILU 2
#define LDM_EPI_ACCUM 3
#define LDM_EPI_ADD_R 4
#define LDM_EPI_RELU 5
#define LDM_EPI_MASK_R 6
typedef struct ldm_linear_args {
    int32_t Bn, M, K, K2;
    int32_t epi;
    int32_t w_dtype;
    const float* X;  int64_t sxb, sxk;
    const void* W;   int64_t swm, swk;
    const float* X2; int64_t sx2b, sx2k;
    const void* W2;  int64_t sw2m, sw2k;
    const float* bias;               /* [M] or NULL */
    const float* R;  int64_t srb;    /* residual rows (col stride 1) */
    float* Y;        int64_t syb, sym;
    float* A_out;    int64_t sab;    /* pre-activation rows (col stride 1) */
    int32_t compute;                 /* LDM_COMPUTE_FP32 or LDM_COMPUTE_BF16 (below) */
    float* ws; int64_t ws_floats;    /* optional split-K workspace (LDM_COMPUTE_BF16), or NULL */
} ldm_linear_args_t;
/* LDM_COMPUTE_FP32: exact fp32 products (VALU register-tiled kernel).
 * LDM_COMPUTE_BF16: matrix cores -- X and W rounded to bf16 (RNE) as they are staged, fp32
 * products and accumulation (mixed-precision training; any w_dtype). */
#define LDM_COMPUTE_FP32 0
#define LDM_COMPUTE_BF16 1
int ldm_linear(const ldm_linear_args_t* a, ldm_stream_t s);
/* Split-K (LDM_COMPUTE_BF16, K2 == 0): when the output has too few 64x64 tiles to fill the
 * chip and K is long -- the weight gradients G^T X over ~1M samples of C19 -- the K range is
 * cut into slices that run as separate workgroups, each writing a partial [Bn][M] into ws,
 * and a second kernel sums the slices in fixed order (deterministic) and applies the
 * epilogue.  Returns the ws size (floats) that enables it for these args (0: not worth it);
 * ldm_linear uses it when a->ws has at least that many floats, else runs unsplit. */
int64_t ldm_linear_workspace_floats(const ldm_linear_args_t* a);

/* SiLU backward on the block pre-activation: g = dy * silu'(a)  (A7). n elements. */
int ldm_silu_bwd(const float* dy, const float* a, int n, float* g_out, ldm_stream_t s);
/* Column sums: out[m] (+)= sum_b G[b][m]  (bias gradients).  accumulate != 0 adds. */
int ldm_colsum(const float* G, int Bn, int M, float* out, int accumulate, ldm_stream_t s);
/* Row gather: out[b][:] = table[idx[b]][:] (timestep-embedding lookup, A5). */
int ldm_gather_rows(const float* table, const int32_t* idx, int Bn, int C, float* out,
                    ldm_stream_t s);

/* ---- C19 auto-decoder training (DeepSDF decoder backward + latent codes) --- */
/* The decoder forward/backward GEMMs are ldm_linear (LDM_EPI_RELU forward; G W and G^T X
 * backward) and the bias gradients ldm_colsum; these are the remaining pieces.
 * ReLU backward on the post-activation: g = dy * (y > 0).  n elements. */
int ldm_relu_bwd(const float* dy, const float* y, int n, float* g_out, ldm_stream_t s);
/* DeepSDF clamped L1 on the decoder's pre-tanh output (deep_sdf train loop, enforce_minmax):
 * pred = tanh(pre), loss_out[0] = scale * sum_i |clamp(pred_i) - clamp(gt_i)| with clamp to
 * [-delta, delta], and grad_out[i] = d loss / d pre_i
 *   = scale * sign(clamp(pred_i) - clamp(gt_i)) * [-delta <= pred_i <= delta] * (1 - pred_i^2)
 * (sign(0) = 0; the clamp passes the gradient on the closed interval).  One workgroup, fixed
 * summation order.  grad_out may be NULL. */
int ldm_sdf_l1_loss(const float* pre, const float* gt, int n, float delta, float scale,
                    float* loss_out, float* grad_out, ldm_stream_t s);
/* Segmented column sums: out[s][m] (+)= sum_{p<P} G[s*P + p][m] for s < S (per-shape latent
 * gradients: S shapes of P samples each, rows grouped by shape).  Deterministic. */
int ldm_colsum_segments(const float* G, int S, int P, int M, float* out, int accumulate,
                        ldm_stream_t s);
/* DeepSDF code regulariser, per-sample L2 norm: loss_io[0] += coef * sum_s |z_s| and
 * grad_io[s][:] += coef * z_s / |z_s| (0 where z_s = 0), z fp32 [S][L].  With S shapes of P
 * samples each out of N = S P, DeepSDF's lambda * min(1, epoch/100) * sum_samples |z| / N is
 * coef = lambda * min(1, epoch/100) / S.  One workgroup, fixed order. */
int ldm_latent_l2_reg(const float* z, int S, int L, float coef, float* loss_io, float* grad_io,
                      ldm_stream_t s);

/* ---- grouped bf16 GEMM with fused training epilogues (csrc/gemm_bf16.hip) ---
 * Per problem:  acc[m][n] = sum_seg sum_{k < K_seg} A_seg[m][k] B_seg[n][k]
 * A_seg / B_seg: bf16, k contiguous (row strides lda / ldb in elements, multiples of 8, 16-B
 * aligned), K_seg a multiple of 64.  A K-concatenation ([h || temb] [W | U]^T) is two segments.
 * Rows m >= M_valid are padding: R / P_in / C are not read there and the fp32 outputs (C, P) not
 * written (so caller buffers need only M_valid rows), the bf16 outputs Cb / CbT get zeros (so
 * operand buffers padded to M rows stay zero-padded), and they add nothing to colsum / loss.
 * Epilogue, with pre = acc + bias[n] (bias optional):
 *   LDM_GEMM_STORE       out = pre
 *   LDM_GEMM_SILU        out = SiLU(pre);        P = pre (if P)
 *   LDM_GEMM_RESID_SILU  out = R + SiLU(pre);    P = pre (if P)                 (A6 block)
 *   LDM_GEMM_RELU        out = max(pre, 0)
 *   LDM_GEMM_ACCUM       out = C + pre
 *   LDM_GEMM_DGRAD_SILU  dh = (R +) pre -> C;  out = dh * SiLU'(P_in)  (A7: the gradient at the
 *                        layer below's pre-activation, fused into the G W product)
 *   LDM_GEMM_LOSS        d = pre - P_in (targets); out = scale * d; loss_part += d^2 (A9)
 *   LDM_GEMM_ADD_R       out = R + pre
 *   LDM_GEMM_RELU_BWD    out = Rb[m][n] > 0 ? pre : 0   (Rb bf16: the ReLU backward through the
 *                        saved post-activation, fused into the G W product; C19)
 * Outputs (each optional): C fp32 [m][n] (ldc; in DGRAD_SILU C receives dh), Cb bf16 [m][n]
 * (ldcb), CbT bf16 TRANSPOSED [n][m] (ldct; M and ldct multiples of 4), colsum fp32
 * [ceil(M/32)][N]: per 32-row block column sums of out (bias gradients, summed in fixed order
 * by the caller), loss_part fp32 [ceil(M/32)][ceil(N/32)]: sums of d^2 (LOSS).
 * Split-K (k_split > 1; n_seg == 1, mode STORE or ACCUM, C the only output, K a multiple of
 * 128 * k_split): the K range is cut into k_split slices that run as separate tiles, each
 * writing its raw fp32 partial [M_valid][N] into ws (k_split * M * N floats); a second kernel
 * sums the slices in slice order (deterministic) and applies bias / ACCUM.  For the weight
 * gradients G^T X of C19, contracted over ~1M samples into a 512 x 512 output.
 * Up to LDM_GEMM_MAX_PROBS independent problems share one launch.  tile: 0 = auto, 1 = 64x64,
 * 2 = 128x64, 3 = 128x128, 4 = 64x64 with a 3-deep ring; 5 / 6 / 7 = 64x64 / 128x128 / 128x64
 * with 8 waves in two k-groups; 16 / 17 / 18 = persistent 128x128 (4-deep ring) / 128x128
 * (2-deep ring, 2 workgroups per CU) / 64x64 (3-deep ring): one workgroup per CU slot loops
 * over tiles and its LDS ring streams the next tile's k-steps under the current tile's last
 * MFMAs and epilogue (csrc/gemm_bf16.hip). */
#define LDM_GEMM_MAX_SEGS 8
#define LDM_GEMM_MAX_PROBS 4
#define LDM_GEMM_STORE 0
#define LDM_GEMM_SILU 1
#define LDM_GEMM_RESID_SILU 2
#define LDM_GEMM_RELU 3
#define LDM_GEMM_ACCUM 4
#define LDM_GEMM_DGRAD_SILU 5
#define LDM_GEMM_LOSS 6
#define LDM_GEMM_ADD_R 7
#define LDM_GEMM_RELU_BWD 8
typedef struct ldm_gemm_seg {
    const void* A; const void* B;    /* bf16 */
    int64_t lda, ldb;
    int32_t K, reserved;
} ldm_gemm_seg_t;
typedef struct ldm_gemm_prob {
    int32_t M, N, M_valid, n_seg;
    ldm_gemm_seg_t seg[LDM_GEMM_MAX_SEGS];
    int32_t mode; float scale;
    const float* bias;
    const float* R;    int64_t ldr;
    const float* P_in; int64_t ldp_in;
    float* C;          int64_t ldc;
    float* P;          int64_t ldp;
    void* Cb;          int64_t ldcb;
    void* CbT;         int64_t ldct;
    float* colsum;
    float* loss_part;
    int32_t k_split;   /* 0 or 1: whole K per tile; > 1: split-K into ws (see above) */
    int32_t ct_blk;    /* > 0: CbT written m-blocked, [ceil(M/ct_blk)][N][ct_blk] (ldct unused):
                        * the sample-axis operands of C19, whose 1M-long rows would otherwise put
                        * every row of a tile in its own memory page */
    float* ws;
    const void* Rb;    int64_t ldrb;   /* bf16 [m][n] (LDM_GEMM_RELU_BWD) */
    int64_t slice_a, slice_b;          /* split-K: slice s starts s * slice_a (A) / s * slice_b
                                        * (B) elements in (0: s * K / k_split, contiguous K);
                                        * with ct_blk-blocked operands each slice is one block */
} ldm_gemm_prob_t;
typedef struct ldm_gemm_args {
    int32_t n_prob, tile;
    ldm_gemm_prob_t prob[LDM_GEMM_MAX_PROBS];
} ldm_gemm_args_t;
int ldm_gemm_bf16(const ldm_gemm_args_t* a, ldm_stream_t s);

/* ---- C17 1D-UNet denoiser: fused conv1d (implicit GEMM) ------------------ */
/* Y[b][co][l] = epi( sum_s sum_{ci<C_s} sum_{k<ksize_s} W_s(co,ci,k) * act_s(Xsrc_s(b,ci,l,k))
 *                    + bias[co] + bias2[co] + cbias[b*scb + co]  (+ R[b][co][l]) )
 * act_s = SiLU if silu_in else identity (applied to the input before the taps).
 * Xsrc for LDM_CONV_DIRECT: X[b][ci][l*stride + k - pad];  LDM_CONV_UP2 (nearest 2x upsample,
 * then the conv, stride 1): p = l + k - pad, X[b][ci][p >> 1] for 0 <= p < 2 L_in.
 * Out-of-range positions read 0 (zero padding).  Weights are packed for the matrix cores
 * (ldm_sdf/ops.py pack_conv_weight): a torch [Cout][Cw][K] weight becomes
 * Wp[Cout16][K][Cw16] (Cout16, Cw16 = sizes rounded up to 16, zero-filled) with the input
 * channel stored at perm16(ci) = (ci & ~15) | ((ci & 3) << 2) | ((ci >> 2) & 3), so
 * W_s(co,ci,k) = W_s[co*ldw + k*kstride + perm16(ci)] with ldw = K*Cw16, kstride = Cw16.
 * A channel concat [u || s] is two segments whose W_s point at channel offsets (multiples
 * of 16) of one packed weight.
 * Epilogues: LDM_CONV_EPI_STORE  Y = pre
 *            LDM_CONV_EPI_DDPM   Y = c1[t] (xlat - c2[t] pre) + sigma[t] z   (A8 with
 *                                eps = pre; z ignored at t = 0; the UNet's output conv)   */
#define LDM_CONV_DIRECT 0
#define LDM_CONV_UP2 1
#define LDM_CONV_MAX_SEGS 4
#define LDM_CONV_EPI_STORE 0
#define LDM_CONV_EPI_DDPM 1
typedef struct ldm_conv1d_seg {
    const float* X;  /* fp32 [B][C][L_in] */
    const void* W;   /* w_dtype, packed (see above) */
    int32_t C, L_in, ksize, stride, pad, mode, silu_in, ldw, kstride;
} ldm_conv1d_seg_t;
typedef struct ldm_conv1d_args {
    int32_t B, Cout, L_out, n_seg, w_dtype, epi;
    ldm_conv1d_seg_t seg[LDM_CONV_MAX_SEGS];
    const float* bias;                /* [Cout] or NULL */
    const float* bias2;               /* [Cout] or NULL (shortcut bias) */
    const float* cbias; int64_t scb;  /* per-(b, co) bias or NULL; scb = 0: batch-uniform */
    const float* R;                   /* residual [B][Cout][L_out] or NULL */
    float* Y;                         /* [B][Cout][L_out] */
    const float* xlat; const float* z;           /* LDM_CONV_EPI_DDPM: x_t and noise [B][L] */
    const float* c1; const float* c2; const float* sigma; int32_t t;   /* A4 device tables */
} ldm_conv1d_args_t;
int ldm_conv1d(const ldm_conv1d_args_t* a, ldm_stream_t s);

/* (ABI 6: the round-3 one-launch UNet sampling loop, ldm_unet_loop*, was retired -- at 0.53x the
 * hipGraph of ldm_conv1d launches after the round-4 conv staging) */

/* ---- C18 marching cubes on a decoded volume ---------------------------- */
/* vol: fp32 [N][N][N] (z slowest, as decode writes it); a corner is inside when v < level.
 * Vertices are one per crossing grid edge, ordered by (owner point, axis), positions by the A1
 * grid rule and p0 + t (p1 - p0), t = (level - v0) / (v1 - v0), each op rounded to fp32;
 * faces are int32 vertex triples ordered by (cube, case-table order), wound so that
 * (b - a) x (c - a) points toward larger values.  Two passes, because the caller allocates
 * the outputs: ldm_mc_count writes device int32 counts_out[2] = {n_vertices, n_faces};
 * ldm_mc_emit (same vol / level / ws) then fills verts fp32 [V][3] and faces int32 [F][3]. */
size_t ldm_mc_workspace_bytes(int N);
int ldm_mc_count(const float* vol, int N, float level, void* ws, size_t ws_bytes,
                 int32_t* counts_out, ldm_stream_t s);
int ldm_mc_emit(const float* vol, int N, float level, float vs, float origin, void* ws,
                size_t ws_bytes, float* verts, int32_t* faces, ldm_stream_t s);
/* Host: the compile-time generated case table: tri [256][16] cube-edge ids (-1 padded),
 * ntri [256].  Edge e = 4a + m runs along axis a (x, y, z) from the corner whose other two
 * coordinate bits (lower axis first) are m; corner c sits at (c & 1, c >> 1 & 1, c >> 2 & 1). */
int ldm_mc_table(int8_t* tri, uint8_t* ntri);

#ifdef __cplusplus
}
#endif
#endif /* LDM_SDF_H */
