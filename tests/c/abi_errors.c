/* Host-side checks of libldm_sdf's C ABI under AddressSanitizer (csrc/Makefile `check-asan`):
 * every entry point of include/ldm_sdf.h called with invalid arguments must return an error
 * code and leave a message in ldm_last_error() -- never crash, read or write out of bounds --
 * and the host-only ones (ABI version, workspace sizes, AdamW scalars, the marching-cubes table,
 * the training step's job table built from descriptors) must work.  No GPU is needed: argument
 * checks run before any device work, and the device queries fail cleanly without one.
 * (Test infrastructure; SURVEY.md §5 "Sanitizers".) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ldm_sdf.h"

static int fails = 0, checks = 0;
#define EXPECT(cond)                                                               \
    do {                                                                           \
        ++checks;                                                                  \
        if (!(cond)) {                                                             \
            ++fails;                                                               \
            fprintf(stderr, "FAIL %s:%d: %s (last error: %s)\n", __FILE__, __LINE__, \
                    #cond, ldm_last_error());                                      \
        }                                                                          \
    } while (0)
#define EXPECT_ERR(expr)                                                          \
    do {                                                                          \
        const int rc_ = (expr);                                                   \
        EXPECT(rc_ != 0);                                                         \
        EXPECT(ldm_last_error() != NULL && ldm_last_error()[0] != 0);             \
    } while (0)

static uintptr_t fake_next = 0x7f0000000000ull;
static void* fake(void) { /* distinct, never dereferenced by host code */
    fake_next += 0x1000000;
    return (void*)fake_next;
}

int main(void) {
    float f[64];
    int32_t i32[64];
    unsigned st = 0;
    memset(f, 0, sizeof(f));
    memset(i32, 0, sizeof(i32));

    EXPECT(ldm_abi_version() == LDM_ABI_VERSION);
    EXPECT(ldm_last_error() != NULL);
    EXPECT(ldm_workspace_bytes(99, 1, 8, LDM_BF16) == 0);
    EXPECT(ldm_workspace_bytes(LDM_OP_DECODER_GRID, 0, 8, LDM_BF16) == 0);
    EXPECT(ldm_workspace_bytes(LDM_OP_DECODER_GRID, 2, 256, LDM_BF16) > 0);
    EXPECT(ldm_workspace_bytes_layout(LDM_OP_DECODER_GRID, 2, 256, LDM_BF16,
                                      LDM_LAYOUT_SPLIT16) == 0);

    /* decoder */
    EXPECT_ERR(ldm_grid_coords(0, 0, 1, 0.1f, -1.f, f, NULL));
    EXPECT_ERR(ldm_grid_coords(8, 4, 2, 0.1f, -1.f, f, NULL));
    EXPECT_ERR(ldm_decoder_fold(NULL, f, 1, f, NULL));
    ldm_decoder_t dec;
    memset(&dec, 0, sizeof(dec));
    dec.abi_version = LDM_ABI_VERSION - 1;     /* stale descriptor */
    EXPECT_ERR(ldm_decoder_grid_fwd(&dec, f, 1, 8, 0, 8, 0.1f, -1.f, f, NULL, 0, NULL));
    dec.abi_version = LDM_ABI_VERSION;
    dec.dtype = LDM_BF16;
    dec.hidden = 512;
    dec.skip_width = 253;
    dec.latent_dim = 256;
    dec.layout = LDM_LAYOUT_SPLIT16;           /* removed in ABI 7 */
    EXPECT_ERR(ldm_decoder_grid_fwd(&dec, f, 1, 8, 0, 8, 0.1f, -1.f, f, NULL, 0, NULL));
    EXPECT_ERR(ldm_decoder_points_fwd(NULL, f, f, 1, 10, f, NULL, 0, NULL));

    /* DDPM */
    EXPECT_ERR(ldm_ddpm_step(NULL, f, f, f, 0, 4, f, NULL));
    EXPECT_ERR(ldm_q_sample(NULL, f, f, i32, 1, 4, f, NULL));
    EXPECT_ERR(ldm_eps_mse_loss(NULL, f, 4, f, f, NULL));
    EXPECT_ERR(ldm_denoiser_fwd_uniform_t(NULL, f, 0, 1, f, f, NULL));
    EXPECT_ERR(ldm_sample_step(NULL, NULL, f, f, 0, 1, f, f, NULL));
    EXPECT(ldm_sample_loop_supported(NULL, 8) == 0);
    EXPECT(ldm_sample_loop_ws_bytes(8, 1024) > 0);
    EXPECT_ERR(ldm_sample_loop(NULL, NULL, f, f, 999, 10, 8, f, 0, NULL));
    EXPECT_ERR(ldm_sample_loop_status(NULL, 8, 1024, &st, NULL));
    EXPECT_ERR(ldm_sample_loop_config(99, 0, 1));
    (void)ldm_sample_loop_last_form();

    /* training */
    EXPECT(ldm_denoiser_train_ws_bytes(NULL, 1) == 0);
    EXPECT_ERR(ldm_denoiser_fwd(NULL, f, i32, 1, f, f, NULL));
    EXPECT_ERR(ldm_denoiser_bwd(NULL, f, f, 1, NULL, f, NULL));
    EXPECT_ERR(ldm_q_sample_loss(NULL, f, NULL, i32, 0, 4, f, f, f, f, NULL));
    EXPECT_ERR(ldm_denoiser_train_step(NULL, NULL, f, f, i32, 1, f, NULL, f, NULL));
    EXPECT_ERR(ldm_adamw_multi(NULL, 0, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1, NULL));
    EXPECT_ERR(ldm_denoiser_train_step_adamw(NULL, NULL, f, f, i32, 1, f, NULL, f, NULL, 0,
                                             1e-3, 0.9, 0.999, 1e-8, 0.0, 1, NULL, NULL, NULL));
    EXPECT_ERR(ldm_train_step_config(7, 0));
    EXPECT(ldm_train_step_config(LDM_TRAIN_AUTO, 0) == 0);
    (void)ldm_train_step_last_form();
    EXPECT_ERR(ldm_denoiser_train_status(NULL, 1, NULL, &st, NULL));
    float hy[7];
    ldm_adamw_hyper(1e-3, 0.9, 0.999, 1e-8, 0.01, 3, hy);
    EXPECT(hy[1] > 0.0999f && hy[1] < 0.1001f && hy[6] > 0.f);
    EXPECT_ERR(ldm_adamw_step(NULL, f, f, f, NULL, 4, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1, NULL));

    /* the one-launch step's job table, built on the host from descriptors (fake device
     * pointers: the builder only records them) -- the DAG builder under ASan */
    {
        ldm_denoiser_t w;
        memset(&w, 0, sizeof(w));
        w.abi_version = LDM_ABI_VERSION;
        w.dtype = LDM_BF16;
        w.D = 256; w.H = 1024; w.n_blocks = 4; w.TE = 128; w.T = 1000;
        w.w_in = fake(); w.b_in = fake(); w.w_t1 = fake(); w.b_t1 = fake();
        w.w_t2 = fake(); w.b_t2 = fake(); w.w_out = fake(); w.b_out = fake();
        w.emb_table = fake(); w.wt_in = fake(); w.wt_t2 = fake(); w.wt_out = fake();
        for (int k = 0; k < 4; ++k) {
            w.w_blk[k] = fake(); w.b_blk[k] = fake(); w.wt_blk[k] = fake();
        }
        ldm_sched_t sc;
        memset(&sc, 0, sizeof(sc));
        sc.abi_version = LDM_ABI_VERSION;
        sc.T = 1000;
        sc.sqrt_ab = fake(); sc.sqrt_1mab = fake();
        ldm_denoiser_grads_t g;
        memset(&g, 0, sizeof(g));
        g.w_in = fake(); g.b_in = fake(); g.w_t1 = fake(); g.b_t1 = fake();
        g.w_t2 = fake(); g.b_t2 = fake(); g.w_out = fake(); g.b_out = fake();
        for (int k = 0; k < 4; ++k) { g.w_blk[k] = fake(); g.b_blk[k] = fake(); }
        ldm_adamw_tensor_t t[16];
        memset(t, 0, sizeof(t));
        float* gs[16] = {g.w_in, g.b_in, g.w_t1, g.b_t1, g.w_t2, g.b_t2, g.w_out, g.b_out,
                         g.w_blk[0], g.w_blk[1], g.w_blk[2], g.w_blk[3],
                         g.b_blk[0], g.b_blk[1], g.b_blk[2], g.b_blk[3]};
        const int rows[16] = {1024, 1, 1024, 1, 1024, 1, 256, 1, 1024, 1024, 1024, 1024,
                              1, 1, 1, 1};
        const int cols[16] = {256, 1024, 128, 1024, 1024, 1024, 1024, 256, 2048, 2048, 2048,
                              2048, 1024, 1024, 1024, 1024};
        for (int i = 0; i < 16; ++i) {
            t[i].p = fake(); t[i].g = gs[i]; t[i].m = fake(); t[i].v = fake();
            t[i].rows = rows[i]; t[i].cols = cols[i];
        }
        /* the bf16 working copies ARE the descriptor's weights (as ldm_sdf.train builds it) */
        t[0].p_bf16 = (void*)w.w_in; t[0].p_bf16_t = (void*)w.wt_in; t[2].p_bf16 = (void*)w.w_t1;
        t[4].p_bf16 = (void*)w.w_t2; t[4].p_bf16_t = (void*)w.wt_t2; t[6].p_bf16 = (void*)w.w_out;
        t[6].p_bf16_t = (void*)w.wt_out;
        for (int k = 0; k < 4; ++k) { t[8 + k].p_bf16 = (void*)w.w_blk[k]; t[8 + k].p_bf16_t = (void*)w.wt_blk[k]; }
        static char buf[1 << 20];
        void* saved = fake();
        for (int B = 1; B <= 1000; B = B < 64 ? B * 4 : B + 312) {
            const int rc = ldm_denoiser_train_dag_describe(&w, &sc, B, saved, &g, t, 16, buf,
                                                           sizeof(buf));
            EXPECT(rc == 0);
            const char* nd = strstr(buf, "nodes ");
            EXPECT(nd != NULL && atoi(nd + 6) >= 45);   /* 4 blocks: ~50 nodes */
            /* weight operands marked for L2 loads, hand-offs (wt 0) not */
            EXPECT(strstr(buf, " wt 2 ") != NULL && strstr(buf, " wt 0 ") != NULL);
        }
        EXPECT(ldm_denoiser_train_dag_describe(&w, &sc, 1000, saved, &g, t, 16, buf, 64) == 0);
        /* the host extent check (check_dag_extents): an AdamW tensor that claims more rows than
         * its gradient (w_out: 256 x 1024) holds is refused before any upload */
        t[6].rows = 512;
        EXPECT_ERR(ldm_denoiser_train_dag_describe(&w, &sc, 1000, saved, &g, t, 16, buf, 64));
        EXPECT(strstr(ldm_last_error(), "outside every allocation") != NULL);
        t[6].rows = 256;
        EXPECT(ldm_denoiser_train_dag_describe(&w, &sc, 1000, saved, &g, t, 16, buf, 64) == 0);
        EXPECT_ERR(ldm_denoiser_train_dag_describe(&w, &sc, 0, saved, &g, t, 16, buf, 64));
        EXPECT_ERR(ldm_denoiser_train_dag_describe(NULL, &sc, 10, saved, &g, t, 16, buf, 64));
        EXPECT_ERR(ldm_denoiser_train_ws_init(NULL, 10, saved, NULL));
        EXPECT_ERR(ldm_denoiser_train_ws_init(&w, 0, saved, NULL));
        EXPECT_ERR(ldm_denoiser_train_ws_init(&w, 10, NULL, NULL));
    }

    /* generic linear / GEMM / conv / misc */
    ldm_linear_args_t la;
    memset(&la, 0, sizeof(la));
    EXPECT_ERR(ldm_linear(NULL, NULL));
    EXPECT_ERR(ldm_linear(&la, NULL));
    EXPECT_ERR(ldm_silu_bwd(NULL, NULL, 4, f, NULL));
    EXPECT_ERR(ldm_colsum(NULL, 4, 4, f, 0, NULL));
    EXPECT_ERR(ldm_gather_rows(NULL, i32, 2, 4, f, NULL));
    EXPECT_ERR(ldm_relu_bwd(NULL, f, 4, f, NULL));
    EXPECT_ERR(ldm_sdf_l1_loss(NULL, f, 4, 0.1f, 1.f, f, f, NULL));
    EXPECT_ERR(ldm_colsum_segments(NULL, 2, 2, 4, f, 0, NULL));
    EXPECT_ERR(ldm_latent_l2_reg(NULL, 2, 4, 1.f, f, f, NULL));
    ldm_gemm_args_t ga;
    memset(&ga, 0, sizeof(ga));
    EXPECT_ERR(ldm_gemm_bf16(NULL, NULL));
    EXPECT_ERR(ldm_gemm_bf16(&ga, NULL));
    ga.n_prob = LDM_GEMM_MAX_PROBS + 1;
    EXPECT_ERR(ldm_gemm_bf16(&ga, NULL));
    ldm_conv1d_args_t ca;
    memset(&ca, 0, sizeof(ca));
    EXPECT_ERR(ldm_conv1d(NULL, NULL));
    EXPECT_ERR(ldm_conv1d(&ca, NULL));

    /* marching cubes */
    EXPECT(ldm_mc_workspace_bytes(0) == 0 || ldm_mc_workspace_bytes(0) > 0);
    EXPECT_ERR(ldm_mc_count(NULL, 8, 0.f, NULL, 0, i32, NULL));
    EXPECT_ERR(ldm_mc_emit(NULL, 8, 0.f, 0.1f, -1.f, NULL, 0, f, i32, NULL));
    int8_t tri[256][16];
    uint8_t ntri[256];
    EXPECT(ldm_mc_table(&tri[0][0], ntri) == 0);
    EXPECT(ntri[0] == 0 && ntri[1] == 1 && tri[1][3] == -1);

    printf("abi_errors: %d checks, %d failures\n", checks, fails);
    return fails ? 1 : 0;
}
