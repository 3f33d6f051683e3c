// DeepSDF decoder on MI355X (gfx950): SURVEY.md §8(a) rows A1 (grid coords), A2 (latent
// fold) and A3 (fused 9-layer MLP), in grid mode and point-list mode.  This unit holds the
// ABI entry points and their dispatch; the 16-bit MFMA kernel lives in decoder_fs.hip (the
// "split" layout; the round-3 "split16" variant on 16x16x32 MFMAs measured 5.5 % slower and was
// deleted in ABI 7).
//
// The reference ships no implementation (/root/reference/README.md:1 is its only line); the
// math follows oracle/ref_cpu.py (decoder_forward_folded, grid_coords_np, latent_fold).
//
// Kernels here:
//   dec_f32_kernel_impl          exact-fp32 parity kernel (VALU, correctness first).
//   grid_coords_kernel           A1 on its own (bit-exactness test surface).
//   fold_kernel                  A2 per-shape biases.
// The round-1/2 layouts (LDM_LAYOUT_PASS8, LDM_LAYOUT_QUARTER) were removed in ABI 5: the split
// kernel superseded both; a descriptor naming them gets LDM_ENOSYS.
#include "decoder_common.h"

#include <math.h>
#include <stdlib.h>

namespace ldm {
namespace {
using namespace dec;

__global__ void grid_coords_kernel(int N, int k0, int npts, float vs, float origin,
                                   float* __restrict__ out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npts) return;
    float x, y, z;
    grid_point(p, N, k0, vs, origin, x, y, z);
    out[3 * (size_t)p + 0] = x;
    out[3 * (size_t)p + 1] = y;
    out[3 * (size_t)p + 2] = z;
}

// ------------------------------------------------------------------------------------------
// A2: beta[b][l][f] = sum_k wz[l][f][k] z[b][k] + bz[l][f]   (l = 0: layer 0, 1: layer 4)
// ------------------------------------------------------------------------------------------
__global__ void fold_kernel(const float* __restrict__ wz, const float* __restrict__ bz,
                            const float* __restrict__ z, int B, int L, int H,
                            float* __restrict__ beta) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= B * 2 * H) return;
    const int f = id % H;
    const int l = (id / H) % 2;
    const int b = id / (2 * H);
    const float* w = wz + ((size_t)l * H + f) * L;
    const float* zz = z + (size_t)b * L;
    float acc = 0.f;
    for (int k = 0; k < L; ++k) acc = fmaf(w[k], zz[k], acc);
    beta[id] = acc + bz[l * H + f];
}

// ------------------------------------------------------------------------------------------
// max over shapes b of sqrt(mean_l z[b][l]^2): the input of dtype="auto" (api.resolve_decode_dtype).
// One workgroup of 4 waves; wave w takes shapes w, w + 4, ...: per shape a lane sums its
// elements' squares in order, the wave sums the lanes (xor shuffles), and the largest RMS goes
// through LDS.  Here rather than as torch reductions: the process's first torch pow / mean /
// sqrt / max on the GPU loads their code objects (~0.25 s on a fresh process, DESIGN.md §7 round
// 6), while this kernel sits in the code object the decode itself loads.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rms_max_kernel(const float* __restrict__ z, int B, int L,
                                                      float* __restrict__ out) {
    __shared__ float wmax[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float m = 0.f;
    for (int b = wave; b < B; b += 4) {
        const float* zz = z + (size_t)b * L;
        float s = 0.f;
        for (int k = lane; k < L; k += 64) s = fmaf(zz[k], zz[k], s);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        m = fmaxf(m, sqrtf(s / (float)L));
    }
    if (lane == 0) wmax[wave] = m;
    __syncthreads();
    if (threadIdx.x == 0) out[0] = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
}

// ------------------------------------------------------------------------------------------
// fp32 parity kernel: 32 points per workgroup, activations in LDS [512][32], weights W^T
// streamed from L2 with coalesced loads, 8x8 register tile per thread, fmaf accumulation.
// Blob layout: for l = 1..7: WT_l [K_l][M_l] then b_l [M_l].
// ------------------------------------------------------------------------------------------
struct F32Args {
    const float* blob;
    const float* wxyz;     // [2][512][3]
    const float* beta;     // [B][2][512]
    const float* w_last;   // [512] natural order
    const float* xyz;      // points mode
    float* out;
    float b_last;
    int npts, tiles_per_shape, N, k0, sw;
    float vs, origin;
};

__global__ __launch_bounds__(256) void dec_f32_kernel_impl(F32Args a, int points) {
    __shared__ float hs[512 * 32];
    __shared__ float pxyz[32 * 3];
    const int t = threadIdx.x;
    const int shape = blockIdx.x / a.tiles_per_shape;
    const int local = blockIdx.x - shape * a.tiles_per_shape;
    const int p0 = local * 32;
    if (t < 32) {
        int pt = p0 + t;
        if (pt >= a.npts) pt = a.npts - 1;
        float x, y, z;
        if (points) {
            const float* q = a.xyz + ((size_t)shape * a.npts + pt) * 3;
            x = q[0]; y = q[1]; z = q[2];
        } else {
            grid_point(pt, a.N, a.k0, a.vs, a.origin, x, y, z);
        }
        pxyz[t * 3 + 0] = x;
        pxyz[t * 3 + 1] = y;
        pxyz[t * 3 + 2] = z;
    }
    __syncthreads();
    const float* beta0 = a.beta + (size_t)shape * 2 * 512;
    const float* beta4 = beta0 + 512;
    // layer 0: h = relu(Wxyz0 xyz + beta0)
    for (int e = t; e < 512 * 32; e += 256) {
        const int f = e >> 5, pp = e & 31;
        const float* w = a.wxyz + f * 3;
        float v = beta0[f];
        v = fmaf(w[0], pxyz[pp * 3 + 0], v);
        v = fmaf(w[1], pxyz[pp * 3 + 1], v);
        v = fmaf(w[2], pxyz[pp * 3 + 2], v);
        hs[e] = fmaxf(v, 0.f);
    }
    __syncthreads();
    const int tf = t & 63, tp = t >> 6;
    const float* blob = a.blob;
    for (int l = 1; l <= 7; ++l) {
        const int K = (l == 4) ? a.sw : 512;
        const int M = (l == 3) ? a.sw : 512;
        const float* WT = blob;
        const float* bias = blob + (size_t)K * M;
        blob = bias + M;
        float acc[8][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = tf + 64 * i;
            const float bv = (f < M) ? (l == 4 ? beta4[f] : bias[f]) : 0.f;
            float wx = 0.f, wy = 0.f, wzz = 0.f;
            if (l == 4 && f < M) {
                const float* w = a.wxyz + (512 + f) * 3;
                wx = w[0]; wy = w[1]; wzz = w[2];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float v = bv;
                if (l == 4) {
                    const int pp = tp * 8 + j;
                    v = fmaf(wx, pxyz[pp * 3 + 0], v);
                    v = fmaf(wy, pxyz[pp * 3 + 1], v);
                    v = fmaf(wzz, pxyz[pp * 3 + 2], v);
                }
                acc[i][j] = v;
            }
        }
        for (int k = 0; k < K; ++k) {
            float w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int f = tf + 64 * i;
                w[i] = (f < M) ? WT[(size_t)k * M + f] : 0.f;
            }
            const f32x4 h0 = *reinterpret_cast<const f32x4*>(hs + k * 32 + tp * 8);
            const f32x4 h1 = *reinterpret_cast<const f32x4*>(hs + k * 32 + tp * 8 + 4);
            const float hv[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(w[i], hv[j], acc[i][j]);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = tf + 64 * i;
            if (f < M) {
#pragma unroll
                for (int j = 0; j < 8; ++j) hs[f * 32 + tp * 8 + j] = fmaxf(acc[i][j], 0.f);
            }
        }
        __syncthreads();
    }
    if (t < 32) {
        float s = 0.f;
        for (int f = 0; f < 512; ++f) s = fmaf(a.w_last[f], hs[f * 32 + t], s);
        const int pt = p0 + t;
        if (pt < a.npts) a.out[(size_t)shape * a.npts + pt] = tanhf(s + a.b_last);
    }
}

int g_num_cus = 0;
int num_cus() {
    if (g_num_cus == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            n > 0)
            g_num_cus = n;
        else
            g_num_cus = 256;
    }
    return g_num_cus;
}

int check_decoder(const ldm_decoder_t* w) {
    LDM_REQUIRE(w != nullptr, LDM_EINVAL, "decoder descriptor is NULL");
    LDM_REQUIRE(w->abi_version == LDM_ABI_VERSION, LDM_EINVAL, "decoder abi_version %d != %d",
                w->abi_version, LDM_ABI_VERSION);
    LDM_REQUIRE(w->hidden == kHidden, LDM_ENOSYS, "GPU decoder supports hidden=512 (got %d)",
                w->hidden);
    LDM_REQUIRE(w->skip_width == 253 || w->skip_width == 512, LDM_ENOSYS,
                "skip_width must be 253 or 512 (got %d)", w->skip_width);
    LDM_REQUIRE(w->dtype == LDM_F32 || w->dtype == LDM_BF16 || w->dtype == LDM_F16, LDM_EINVAL,
                "bad decoder dtype %d", w->dtype);
    LDM_REQUIRE(w->weights && w->wxyz && w->w_last, LDM_EINVAL, "decoder weights are NULL");
    LDM_REQUIRE(LDM_ALIGNED(w->weights, 16) && LDM_ALIGNED(w->w_last, 16), LDM_EALIGN,
                "decoder weights must be 16-byte aligned");
    if (w->dtype != LDM_F32) {
        LDM_REQUIRE(w->layout != LDM_LAYOUT_PASS8 && w->layout != LDM_LAYOUT_QUARTER &&
                        w->layout != LDM_LAYOUT_SPLIT16,
                    LDM_ENOSYS, "decoder layout %d (pass8 / quarter: removed in ABI 5; split16: "
                    "removed in ABI 7) -- pack the weights in LDM_LAYOUT_SPLIT", w->layout);
        LDM_REQUIRE(w->layout == LDM_LAYOUT_SPLIT, LDM_EINVAL, "bad decoder layout %d",
                    w->layout);
        const int want = decoder_fs_n_stages(w->skip_width);
        LDM_REQUIRE(w->n_stages == want, LDM_EINVAL, "n_stages %d != %d for skip width %d",
                    w->n_stages, want, w->skip_width);
    }
    return 0;
}

int decoder_fwd(const ldm_decoder_t* w, const float* beta, const float* xyz, int B, int npts,
                int N, int k0, float vs, float origin, float* out, void* ws, size_t ws_bytes,
                hipStream_t s) {
    if (int e = check_decoder(w)) return e;
    LDM_REQUIRE(B >= 1 && npts >= 1, LDM_EINVAL, "empty decode (B=%d, npts=%d)", B, npts);
    LDM_REQUIRE((long long)B * npts < (1ll << 31), LDM_EINVAL, "B*npts too large");
    LDM_REQUIRE(beta && out, LDM_EINVAL, "beta/out NULL");
    LDM_REQUIRE(LDM_ALIGNED(beta, 16) && LDM_ALIGNED(out, 4), LDM_EALIGN, "misaligned buffers");
    const bool points = xyz != nullptr;
    if (w->dtype == LDM_F32) {
        F32Args a;
        a.blob = (const float*)w->weights;
        a.wxyz = w->wxyz;
        a.beta = beta;
        a.w_last = w->w_last;
        a.xyz = xyz;
        a.out = out;
        a.b_last = w->b_last;
        a.npts = npts;
        a.tiles_per_shape = (npts + 31) / 32;
        a.N = N;
        a.k0 = k0;
        a.sw = w->skip_width;
        a.vs = vs;
        a.origin = origin;
        hipLaunchKernelGGL(dec_f32_kernel_impl, dim3(B * a.tiles_per_shape), dim3(256), 0, s, a,
                           points ? 1 : 0);
        return launch_status("ldm_decoder_fwd(f32)");
    }
    return decoder_fs_fwd(w, beta, xyz, B, npts, N, k0, vs, origin, out, ws, ws_bytes, s,
                          num_cus());
}

}  // namespace

size_t decoder_workspace_bytes(int B, int dtype, int layout) {
    if (dtype == LDM_F32 || layout != LDM_LAYOUT_SPLIT) return 0;
    return decoder_fs_aux_bytes(B);
}

}  // namespace ldm

using namespace ldm;

extern "C" int ldm_grid_coords(int N, int k0, int k1, float vs, float origin, float* xyz_out,
                               ldm_stream_t s) {
    LDM_REQUIRE(N >= 1 && k0 >= 0 && k1 > k0 && k1 <= N, LDM_EINVAL,
                "bad grid slab N=%d [%d,%d)", N, k0, k1);
    LDM_REQUIRE(xyz_out != nullptr && LDM_ALIGNED(xyz_out, 4), LDM_EINVAL, "xyz_out NULL");
    const long long npts = (long long)(k1 - k0) * N * N;
    LDM_REQUIRE(npts < (1ll << 31), LDM_EINVAL, "grid too large");
    hipLaunchKernelGGL(grid_coords_kernel, dim3((unsigned)((npts + 255) / 256)), dim3(256), 0,
                       (hipStream_t)s, N, k0, (int)npts, vs, origin, xyz_out);
    return launch_status("ldm_grid_coords");
}

extern "C" int ldm_decoder_fold(const ldm_decoder_t* w, const float* z, int B, float* beta_out,
                                ldm_stream_t s) {
    LDM_REQUIRE(w && w->abi_version == LDM_ABI_VERSION, LDM_EINVAL, "bad decoder descriptor");
    LDM_REQUIRE(w->wz && w->bz && z && beta_out && B >= 1 && w->latent_dim >= 1, LDM_EINVAL,
                "bad fold arguments");
    const int n = B * 2 * w->hidden;
    hipLaunchKernelGGL(fold_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, w->wz,
                       w->bz, z, B, w->latent_dim, w->hidden, beta_out);
    return launch_status("ldm_decoder_fold");
}

extern "C" int ldm_latent_rms_max(const float* z, int B, int L, float* out, ldm_stream_t s) {
    LDM_REQUIRE(z && out && B >= 1 && L >= 1, LDM_EINVAL, "ldm_latent_rms_max: bad arguments");
    hipLaunchKernelGGL(rms_max_kernel, dim3(1), dim3(256), 0, (hipStream_t)s, z, B, L, out);
    return launch_status("ldm_latent_rms_max");
}

extern "C" int ldm_decoder_grid_fwd(const ldm_decoder_t* w, const float* beta, int B, int N,
                                    int k0, int k1, float vs, float origin, float* out, void* ws,
                                    size_t ws_bytes, ldm_stream_t s) {
    LDM_REQUIRE(N >= 2 && k0 >= 0 && k1 > k0 && k1 <= N, LDM_EINVAL,
                "bad grid slab N=%d [%d,%d)", N, k0, k1);
    const long long npts = (long long)(k1 - k0) * N * N;
    LDM_REQUIRE(npts < (1ll << 31), LDM_EINVAL, "grid slab too large");
    return decoder_fwd(w, beta, nullptr, B, (int)npts, N, k0, vs, origin, out, ws, ws_bytes,
                       (hipStream_t)s);
}

extern "C" int ldm_decoder_points_fwd(const ldm_decoder_t* w, const float* beta, const float* xyz,
                                      int B, int P, float* out, void* ws, size_t ws_bytes,
                                      ldm_stream_t s) {
    LDM_REQUIRE(xyz != nullptr && LDM_ALIGNED(xyz, 4), LDM_EINVAL, "xyz NULL");
    return decoder_fwd(w, beta, xyz, B, P, 0, 0, 0.f, 0.f, out, ws, ws_bytes, (hipStream_t)s);
}
