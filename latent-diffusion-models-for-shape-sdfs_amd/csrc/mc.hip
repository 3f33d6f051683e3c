// C18: marching cubes on a decoded SDF volume, MI355X (gfx950).  DESIGN.md §10.
//
// The consumer of decode's output.  Conventions -- corner / edge
// numbering, the face-local ambiguity rule, vertex and face order, fp32 interpolation -- are
// those of oracle/ref_mc.py, which the GPU output matches bit for bit.
//
// The case table is GENERATED at compile time (constexpr) from the rule, independently of the
// oracle's Python generator; tests compare the two tables (ldm_mc_table exports this one).
//
// Passes (HBM-bound integer/byte work; no MFMA):
//   1. classify   one thread per grid point: 3-bit mask of its owned crossing edges (+x, +y,
//                 +z), and for the cube it anchors the 8-corner case and its triangle count,
//                 packed in one u16 (mask | ntri << 3 | case << 8) -> 2 B/point written
//   2. block sums per 4096-point chunk: (#vertices, #triangles)
//   3. chunk scan  one workgroup: exclusive offsets of the chunks + the totals
//   4. vertices   per chunk: in-chunk exclusive scan, vertex positions, per-point first
//                 vertex index (vofs)
//   5. faces      per chunk: in-chunk scan of triangle counts, 3 vertex ids per triangle
//                 through vofs + the owner's mask
// Vertex order = (owner point, axis); face order = (cube, table order): a pure function of
// the volume, so the output is deterministic and equal to the oracle's.
#include "ldm_internal.h"

#include <string.h>

namespace ldm {
namespace {

// ------------------------------------------------------------------------------ case table
// 16-byte aligned: the kernels stage the tables into LDS as u32x4 / unsigned words
struct alignas(16) McTables {
    signed char tri[256][16];
    unsigned char ntri[256];
};
static_assert(alignof(McTables) >= 16 && offsetof(McTables, ntri) % 16 == 0,
              "McTables: the LDS staging reads tri / ntri as 16-byte vectors");

// corner c: offset (c & 1, c >> 1 & 1, c >> 2 & 1); edge e = 4a + m along axis a from the
// corner whose other two bits (lower axis first) are m.
constexpr int mc_edge_id(int c0, int c1) {
    const int d = c0 ^ c1;
    const int a = d == 1 ? 0 : (d == 2 ? 1 : 2);
    const int o0 = a == 0 ? 1 : 0, o1 = a == 2 ? 1 : 2;
    const int lo = c0 & c1;
    return 4 * a + (((lo >> o0) & 1) | (((lo >> o1) & 1) << 1));
}
constexpr int mc_edge_start(int e) {
    const int a = e / 4, m = e % 4;
    const int o0 = a == 0 ? 1 : 0, o1 = a == 2 ? 1 : 2;
    return ((m & 1) << o0) | (((m >> 1) & 1) << o1);
}

struct McFaces {
    int c[6][4];
};
// faces as corner rings, counter-clockwise seen from outside the cube
constexpr McFaces mc_faces() {
    McFaces f{};
    int n = 0;
    for (int a = 0; a < 3; ++a) {
        const int u = (a + 1) % 3, w = (a + 2) % 3;
        for (int s = 0; s < 2; ++s) {
            const int ub[4] = {0, 1, 1, 0}, wb[4] = {0, 0, 1, 1};
            for (int q = 0; q < 4; ++q) {
                const int r = s ? q : 3 - q;          // outward normal -e_a: reversed ring
                f.c[n][q] = (s << a) | (ub[r] << u) | (wb[r] << w);
            }
            ++n;
        }
    }
    return f;
}

// bitmask of the (two) faces containing edge e
constexpr int mc_edge_face_mask(int e, const McFaces& F) {
    const int c0 = mc_edge_start(e), c1 = c0 | (1 << (e / 4));
    int m = 0;
    for (int f = 0; f < 6; ++f) {
        bool h0 = false, h1 = false;
        for (int q = 0; q < 4; ++q) {
            h0 = h0 || F.c[f][q] == c0;
            h1 = h1 || F.c[f][q] == c1;
        }
        if (h0 && h1) m |= 1 << f;
    }
    return m;
}

constexpr McTables make_mc_tables() {
    McTables T{};
    const McFaces F = mc_faces();
    int efm[12] = {};
    for (int e = 0; e < 12; ++e) efm[e] = mc_edge_face_mask(e, F);
    for (int cfg = 0; cfg < 256; ++cfg) {
        for (int i = 0; i < 16; ++i) T.tri[cfg][i] = -1;
        int nxt[12] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
        for (int f = 0; f < 6; ++f) {
            int ce[4] = {}, ck[4] = {}, nc = 0;      // crossings: edge, kind (1 = leaves inside)
            for (int q = 0; q < 4; ++q) {
                const int A = F.c[f][q], B = F.c[f][(q + 1) % 4];
                const int ia = (cfg >> A) & 1, ib = (cfg >> B) & 1;
                if (ia != ib) {
                    ce[nc] = mc_edge_id(A, B);
                    ck[nc] = ia;
                    ++nc;
                }
            }
            for (int q = 0; q < nc; ++q) {
                if (!ck[q]) continue;
                int r = (q + nc - 1) % nc;
                while (ck[r]) r = (r + nc - 1) % nc;  // closest earlier "enters inside"
                nxt[ce[q]] = ce[r];
            }
        }
        bool seen[12] = {};
        int nt = 0;
        for (int s0 = 0; s0 < 12; ++s0) {
            if (nxt[s0] < 0 || seen[s0]) continue;
            int cyc[12] = {}, n = 0;
            int e = s0;
            do {
                cyc[n++] = e;
                seen[e] = true;
                e = nxt[e];
            } while (e != s0);
            // first rotation whose fan diagonals avoid the cube faces
            int r0 = -1;
            for (int r = 0; r < n && r0 < 0; ++r) {
                bool ok = true;
                for (int i = 2; i < n - 1; ++i)
                    if (efm[cyc[r]] & efm[cyc[(r + i) % n]]) ok = false;
                if (ok) r0 = r;
            }
            if (r0 < 0) r0 = 0;                       // never taken (checked by the tests)
            for (int i = 1; i < n - 1; ++i) {
                T.tri[cfg][3 * nt + 0] = (signed char)cyc[r0];
                T.tri[cfg][3 * nt + 1] = (signed char)cyc[(r0 + i + 1) % n];
                T.tri[cfg][3 * nt + 2] = (signed char)cyc[(r0 + i) % n];
                ++nt;
            }
        }
        T.ntri[cfg] = (unsigned char)nt;
    }
    return T;
}

constexpr McTables kMcHost = make_mc_tables();
__constant__ McTables kMc = make_mc_tables();

// ------------------------------------------------------------------------------ kernels
// points per thread of the scan-chunk passes (a multiple of 8; MC_PER A/B builds), a chunk =
// 256 threads x kPer points
#ifndef MC_PER
#define MC_PER 16
#endif
constexpr int kPer = MC_PER;
constexpr int kChunk = 256 * kPer;
static_assert(kPer % 8 == 0 && kPer <= 32, "whole 16-byte code vectors; a 32-bit cube mask");

__device__ __forceinline__ float grid_c(int i, float vs, float origin) {
#pragma clang fp contract(off)
    return i * vs + origin;             // A1: two roundings
}

// Every volume load below is UNCONDITIONAL, at a clamped (in-bounds) index, with the value
// selected after: a load under a divergent branch makes the compiler wait for it before the
// branch rejoins (one memory round trip per load), which is what the first
// kernels of this file paid.

// table of triangle counts, staged per workgroup into LDS (a divergent __constant__ lookup is a
// vector memory round trip)
__device__ __forceinline__ void stage_ntri(unsigned char* s_ntri) {
    if (threadIdx.x < 64)
        reinterpret_cast<unsigned*>(s_ntri)[threadIdx.x] =
            reinterpret_cast<const unsigned*>(kMc.ntri)[threadIdx.x];
}

// 1. classify: one thread per "quad" = 4 consecutive points of a row (Q = ceil(N/4) quads per
// row, rows in (k, j) order), flat over the Q * N * N quads.  Per quad it loads the 5 values
// i0 .. i0+4 of the rows (j, k), (j+1, k), (j, k+1), (j+1, k+1) (clamped to the volume), as
// 16-byte vectors when rows are 16-byte aligned (N % 4 == 0), and writes 4 codes.
template <bool VEC>
__global__ __launch_bounds__(256) void mc_classify_kernel(const float* __restrict__ vol, int N,
                                                          float iso,
                                                          unsigned short* __restrict__ code) {
    __shared__ unsigned char s_ntri[256];
    stage_ntri(s_ntri);
    const int Q = (N + 3) >> 2;
    const int64_t NN = (int64_t)N * N;
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t gc = min(g, (int64_t)Q * NN - 1);      // past the end: a clamped quad
    const int64_t row = gc / Q;
    const int i0 = (int)(gc - row * Q) * 4, j = (int)(row % N), k = (int)(row / N);
    const int j1 = min(j + 1, N - 1), k1 = min(k + 1, N - 1);
    const int64_t r[4] = {k * NN + (int64_t)j * N, k * NN + (int64_t)j1 * N,
                          k1 * NN + (int64_t)j * N, k1 * NN + (int64_t)j1 * N};
    float v[4][5];
    const int ic = min(i0, N - 1);
    if (VEC && i0 + 4 <= N) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(vol + r[q] + i0);
            v[q][0] = a[0]; v[q][1] = a[1]; v[q][2] = a[2]; v[q][3] = a[3];
            v[q][4] = vol[r[q] + min(i0 + 4, N - 1)];
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int u = 0; u < 5; ++u) v[q][u] = vol[r[q] + min(ic + u, N - 1)];
    }
    __syncthreads();                                   // s_ntri
    if (g != gc) return;
    const bool jy = j + 1 < N, kz = k + 1 < N;
    unsigned short cd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const bool ix = i0 + u + 1 < N;
        const bool in0 = v[0][u] < iso;
        unsigned m = 0;
        if (ix && ((v[0][u + 1] < iso) != in0)) m |= 1;
        if (jy && ((v[1][u] < iso) != in0)) m |= 2;
        if (kz && ((v[2][u] < iso) != in0)) m |= 4;
        // corner c = (c & 1, c >> 1 & 1, c >> 2 & 1): rows 0..3 = (dy, dz) = 00, 10, 01, 11
        unsigned cfg = (unsigned)in0 | (unsigned)(v[0][u + 1] < iso) << 1 |
                       (unsigned)(v[1][u] < iso) << 2 | (unsigned)(v[1][u + 1] < iso) << 3 |
                       (unsigned)(v[2][u] < iso) << 4 | (unsigned)(v[2][u + 1] < iso) << 5 |
                       (unsigned)(v[3][u] < iso) << 6 | (unsigned)(v[3][u + 1] < iso) << 7;
        const bool cube = ix && jy && kz;
        cfg = cube ? cfg : 0u;
        const unsigned nt = cube ? s_ntri[cfg] : 0u;
        cd[u] = (unsigned short)(m | (nt << 3) | (cfg << 8));
    }
    unsigned short* dst = code + r[0] + i0;
    if (VEC && i0 + 4 <= N) {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 w = {(unsigned)cd[0] | (unsigned)cd[1] << 16,
                         (unsigned)cd[2] | (unsigned)cd[3] << 16};
        *reinterpret_cast<u32x2*>(dst) = w;
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + u < N) dst[u] = cd[u];
    }
}

__device__ __forceinline__ int nvert_of(unsigned c) { return __popc(c & 7u); }
__device__ __forceinline__ int ntri_of(unsigned c) { return (c >> 3) & 7u; }

// block-wide exclusive scan of one int per thread (256 threads); returns the block total
__device__ __forceinline__ int block_excl_scan(int v, int* lds /*[4]*/, int* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wv] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        if (w < wv) base += lds[w];
        tot += lds[w];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// load the kPer codes of this thread's slice of chunk `blk` (zeros past n)
__device__ __forceinline__ void load_codes(const unsigned short* __restrict__ code, int64_t n,
                                           int blk, unsigned (&c)[kPer]) {
    const int64_t p0 = (int64_t)blk * kChunk + threadIdx.x * kPer;
    if (p0 + kPer <= n) {
        const u32x4* src = reinterpret_cast<const u32x4*>(code + p0);
        u32x4 a[kPer / 8];
#pragma unroll
        for (int h = 0; h < kPer / 8; ++h) a[h] = src[h];
#pragma unroll
        for (int h = 0; h < kPer / 8; ++h)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c[8 * h + 2 * q] = a[h][q] & 0xffffu;
                c[8 * h + 2 * q + 1] = a[h][q] >> 16;
            }
    } else {
#pragma unroll
        for (int q = 0; q < kPer; ++q) c[q] = p0 + q < n ? code[p0 + q] : 0u;
    }
}

// 2. per-chunk (#vertices, #triangles)
__global__ __launch_bounds__(256) void mc_block_sums_kernel(const unsigned short* __restrict__ code,
                                                            int64_t n, int2* __restrict__ bsum) {
    __shared__ int lds[8];
    unsigned c[kPer];
    load_codes(code, n, blockIdx.x, c);
    int nv = 0, nt = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        nv += nvert_of(c[q]);
        nt += ntri_of(c[q]);
    }
    int tv, tt;
    block_excl_scan(nv, lds, &tv);
    block_excl_scan(nt, lds + 4, &tt);
    if (threadIdx.x == 0) bsum[blockIdx.x] = make_int2(tv, tt);
}

// 3. exclusive scan of the chunk sums (one workgroup) + totals: thread t owns the chunks
// [t * per, (t + 1) * per), summed serially, then ONE block scan of the 256 thread sums and a
// second serial pass writes the offsets (the previous form ran nb / 256 block scans, each with
// its barriers: 16 us at 256^3)
// The serial passes read their chunk sums kScanBatch at a time, every load of a batch issued
// before any use (clamped index, value selected): a plain loop waited out one round trip per
// chunk, 2 x 16 of them at 256^3 (9.4 us, profiles/r04a/mc_kernel_stats.csv).
constexpr int kScanBatch = 8;
__global__ __launch_bounds__(256) void mc_chunk_scan_kernel(const int2* __restrict__ bsum, int nb,
                                                            int2* __restrict__ boff,
                                                            int32_t* __restrict__ totals) {
    __shared__ int lds[8];
    const int per = (nb + 255) / 256;
    const int b0 = threadIdx.x * per, b1 = min(b0 + per, nb);
    auto batch = [&](int b, int2 (&x)[kScanBatch]) {
#pragma unroll
        for (int u = 0; u < kScanBatch; ++u) x[u] = bsum[min(b + u, b1 - 1)];
#pragma unroll
        for (int u = 0; u < kScanBatch; ++u)
            if (b + u >= b1) x[u] = make_int2(0, 0);
    };
    int sv = 0, st = 0;
    for (int b = b0; b < b1; b += kScanBatch) {
        int2 x[kScanBatch];
        batch(b, x);
#pragma unroll
        for (int u = 0; u < kScanBatch; ++u) {
            sv += x[u].x;
            st += x[u].y;
        }
    }
    int tv, tt;
    int cv = block_excl_scan(sv, lds, &tv);
    int ct = block_excl_scan(st, lds + 4, &tt);
    for (int b = b0; b < b1; b += kScanBatch) {
        int2 x[kScanBatch];
        batch(b, x);
#pragma unroll
        for (int u = 0; u < kScanBatch; ++u) {
            if (b + u < b1) boff[b + u] = make_int2(cv, ct);
            cv += x[u].x;
            ct += x[u].y;
        }
    }
    if (threadIdx.x == 0) {
        totals[0] = tv;
        totals[1] = tt;
    }
}

// The 16 volume values v[q] = vol[p0 + q + st] of this thread's points, shifted by `st`
// (0, 1, N or N*N), clamped to the volume: four 16-byte loads when the run is aligned and
// in bounds, else 16 scalar loads (all issued before any use).
__device__ __forceinline__ void load_run(const float* __restrict__ vol, int64_t n, int64_t p0,
                                         int64_t st, bool vec, float (&v)[kPer]) {
    const int64_t b = p0 + st;
    if (vec && b + kPer <= n) {
#pragma unroll
        for (int q = 0; q < kPer / 4; ++q) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(vol + b + 4 * q);
            v[4 * q] = a[0]; v[4 * q + 1] = a[1]; v[4 * q + 2] = a[2]; v[4 * q + 3] = a[3];
        }
    } else {
#pragma unroll
        for (int q = 0; q < kPer; ++q) v[q] = vol[min(b + q, n - 1)];
    }
}

// 4. vertices + per-point first vertex index.  A thread that owns vertices loads its 16
// points' values and their +x, +y, +z neighbours up front (clamped, unconditional), then emits
// the vertices from registers.
__global__ __launch_bounds__(256) void mc_vertices_kernel(const float* __restrict__ vol, int N,
                                                          float iso, float vs, float origin,
                                                          const unsigned short* __restrict__ code,
                                                          const int2* __restrict__ boff,
                                                          int32_t* __restrict__ vofs,
                                                          float* __restrict__ verts) {
#pragma clang fp contract(off)
    __shared__ int lds[4];
    const int64_t NN = (int64_t)N * N, n = NN * N;
    unsigned c[kPer];
    load_codes(code, n, blockIdx.x, c);
    int nv = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) nv += nvert_of(c[q]);
    int tot;
    int off = boff[blockIdx.x].x + block_excl_scan(nv, lds, &tot);
    if (nv == 0) return;
    const int64_t p0 = (int64_t)blockIdx.x * kChunk + threadIdx.x * kPer;
    const bool vec = (N & 3) == 0;
    float v0[kPer], vy[kPer], vz[kPer];
    load_run(vol, n, p0, 0, vec, v0);
    load_run(vol, n, p0, N, vec, vy);
    load_run(vol, n, p0, NN, vec, vz);
    const float v16 = vol[min(p0 + kPer, n - 1)];
    // (i, j, k) of p0, then stepped point by point
    int i = (int)(p0 % N), j = (int)((p0 / N) % N), k = (int)(p0 / NN);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const unsigned m = c[q] & 7u;
        if (m) {
            const int64_t p = p0 + q;
            vofs[p] = off;
            const float x = grid_c(i, vs, origin), y = grid_c(j, vs, origin);
            const float z = grid_c(k, vs, origin);
            const float v1s[3] = {q + 1 < kPer ? v0[q + 1] : v16, vy[q], vz[q]};
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                if (!(m & (1u << a))) continue;
                const float t = (iso - v0[q]) / (v1s[a] - v0[q]);
                float o[3] = {x, y, z};
                const int ia = a == 0 ? i : (a == 1 ? j : k);
                const float c0 = o[a], c1 = grid_c(ia + 1, vs, origin);
                const float d = c1 - c0;
                const float td = t * d;
                o[a] = c0 + td;
                float* dst = verts + (int64_t)off * 3;
                dst[0] = o[0];
                dst[1] = o[1];
                dst[2] = o[2];
                ++off;
            }
        }
        if (++i == N) {
            i = 0;
            if (++j == N) {
                j = 0;
                ++k;
            }
        }
    }
}

// 5. triangles.  The case table is staged into LDS; per cube with triangles every vertex id it
// can reference (its 12 edges, owned by corners 0..6) is formed from ONE round of 14
// independent gathers (code and vofs of the 7 owner corners), kept in LDS per thread, and the
// triangles are read off the table.
// MC_FACES_PAIR (round 6): a thread takes its cubes with triangles two at a time, from a bit
// mask, with both cubes' 28 gathers issued before either is used.  The earlier form walked the
// thread's 16 points in order and gathered inside the walk: a wave paid one serial round trip
// for every point index at which ANY of its lanes had a cube, up to 16 per wave.
#ifndef MC_FACES_PAIR
#define MC_FACES_PAIR 1
#endif
__device__ __forceinline__ void mc_gather_owners(const unsigned short* __restrict__ code,
                                                 const int32_t* __restrict__ vofs, int64_t p,
                                                 int64_t N, int64_t NN, unsigned (&oc)[7],
                                                 int (&ov)[7]) {
#pragma unroll
    for (int s = 0; s < 7; ++s) {
        const int64_t o = p + (s & 1) + ((s >> 1) & 1) * N + ((s >> 2) & 1) * NN;
        oc[s] = code[o];
        ov[s] = vofs[o];
    }
}

// one cube's triangles: vertex ids through the thread's LDS slots, faces at `off` (the cube's
// first triangle); oc[0] is the cube's own code
__device__ __forceinline__ void mc_emit_cube(const unsigned (&oc)[7], const int (&ov)[7], int* ev,
                                             const signed char* s_tri, int off,
                                             int32_t* __restrict__ faces) {
#pragma unroll
    for (int e = 0; e < 12; ++e) {
        const int s = mc_edge_start(e), a = e >> 2;
        ev[e * 256] = ov[s] + __popc(oc[s] & 7u & ((1u << a) - 1u));
    }
    const int ntq = ntri_of(oc[0]);
    const signed char* tr = s_tri + (oc[0] >> 8) * 16;
    for (int t = 0; t < ntq; ++t) {
        int32_t* dst = faces + (int64_t)(off + t) * 3;
#pragma unroll
        for (int r = 0; r < 3; ++r) dst[r] = ev[tr[3 * t + r] * 256];
    }
}

__global__ __launch_bounds__(256) void mc_faces_kernel(int N, const unsigned short* __restrict__ code,
                                                       const int2* __restrict__ boff,
                                                       const int32_t* __restrict__ vofs,
                                                       int32_t* __restrict__ faces) {
    __shared__ int lds[4];
    __shared__ __attribute__((aligned(16))) signed char s_tri[256 * 16];
    __shared__ int s_ev[12][256];
    reinterpret_cast<u32x4*>(s_tri)[threadIdx.x] = reinterpret_cast<const u32x4*>(kMc.tri)[threadIdx.x];
    const int64_t NN = (int64_t)N * N, n = NN * N;
    unsigned c[kPer];
    load_codes(code, n, blockIdx.x, c);
    int nt = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) nt += ntri_of(c[q]);
    int tot;
    int off = boff[blockIdx.x].y + block_excl_scan(nt, lds, &tot);   // (its barriers: s_tri)
    if (nt == 0) return;
    const int64_t p0 = (int64_t)blockIdx.x * kChunk + threadIdx.x * kPer;
    int* ev = &s_ev[0][threadIdx.x];
    if (MC_FACES_PAIR) {
        unsigned am = 0;
#pragma unroll
        for (int q = 0; q < kPer; ++q) am |= (ntri_of(c[q]) ? 1u : 0u) << q;
        // the first triangle of the cube at point q: the thread's offset + the counts before q
        auto first = [&](int q) {
            int f = off;
#pragma unroll
            for (int u = 0; u < kPer; ++u) f += u < q ? ntri_of(c[u]) : 0;
            return f;
        };
        while (am) {
            const int qa = __builtin_ctz(am);
            am &= am - 1u;
            const bool hb = am != 0u;
            const int qb = hb ? __builtin_ctz(am) : qa;
            if (hb) am &= am - 1u;
            unsigned oa[7], ob[7];
            int va[7], vb[7];
            mc_gather_owners(code, vofs, p0 + qa, N, NN, oa, va);   // a cube with triangles:
            mc_gather_owners(code, vofs, p0 + qb, N, NN, ob, vb);   // every owner in bounds
            mc_emit_cube(oa, va, ev, s_tri, first(qa), faces);
            if (hb) mc_emit_cube(ob, vb, ev, s_tri, first(qb), faces);
        }
        return;
    }
    for (int q = 0; q < kPer; ++q) {
        const int ntq = ntri_of(c[q]);
        if (!ntq) continue;
        const int64_t p = p0 + q;            // a cube with triangles: every owner is in bounds
        unsigned oc[7];
        int ov[7];
        mc_gather_owners(code, vofs, p, N, NN, oc, ov);
        mc_emit_cube(oc, ov, ev, s_tri, off, faces);
        off += ntq;
    }
}

struct McWs {
    unsigned short* code;
    int2* bsum;
    int2* boff;
    int32_t* vofs;
    size_t bytes;
};

McWs mc_ws_layout(int N, void* base) {
    const int64_t n = (int64_t)N * N * N;
    const int64_t nb = (n + kChunk - 1) / kChunk;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    McWs w{};
    char* b = reinterpret_cast<char*>(base);
    size_t o = 0;
    w.code = reinterpret_cast<unsigned short*>(b + o);
    o += up((size_t)nb * kChunk * 2);           // padded to whole chunks (vector loads)
    w.bsum = reinterpret_cast<int2*>(b + o);
    o += up((size_t)nb * sizeof(int2));
    w.boff = reinterpret_cast<int2*>(b + o);
    o += up((size_t)nb * sizeof(int2));
    w.vofs = reinterpret_cast<int32_t*>(b + o);
    o += up((size_t)n * 4);
    w.bytes = o;
    return w;
}

int check_mc(const float* vol, int N, const void* ws, size_t ws_bytes) {
    LDM_REQUIRE(vol && ws, LDM_EINVAL, "marching cubes: NULL volume/workspace");
    LDM_REQUIRE(N >= 2 && N <= 1290, LDM_EINVAL, "marching cubes: N = %d out of [2, 1290]", N);
    LDM_REQUIRE(LDM_ALIGNED(ws, 256) && LDM_ALIGNED(vol, 16), LDM_EALIGN,
                "marching cubes: workspace must be 256-B aligned");
    const McWs w = mc_ws_layout(N, nullptr);
    LDM_REQUIRE(ws_bytes >= w.bytes, LDM_ENOSPC, "marching cubes: workspace %zu < %zu B",
                ws_bytes, w.bytes);
    return 0;
}

}  // namespace
}  // namespace ldm

extern "C" size_t ldm_mc_workspace_bytes(int N) {
    if (N < 2) return 0;
    return ldm::mc_ws_layout(N, nullptr).bytes;
}

extern "C" int ldm_mc_table(int8_t* tri, uint8_t* ntri) {
    LDM_REQUIRE(tri && ntri, LDM_EINVAL, "ldm_mc_table: NULL output");
    memcpy(tri, ldm::kMcHost.tri, sizeof(ldm::kMcHost.tri));
    memcpy(ntri, ldm::kMcHost.ntri, sizeof(ldm::kMcHost.ntri));
    return 0;
}

extern "C" int ldm_mc_count(const float* vol, int N, float level, void* ws, size_t ws_bytes,
                            int32_t* counts_out, ldm_stream_t s) {
    using namespace ldm;
    if (int e = check_mc(vol, N, ws, ws_bytes)) return e;
    LDM_REQUIRE(counts_out, LDM_EINVAL, "ldm_mc_count: NULL counts_out");
    const McWs w = mc_ws_layout(N, ws);
    const int64_t n = (int64_t)N * N * N;
    const int nb = (int)((n + kChunk - 1) / kChunk);
    hipStream_t st = (hipStream_t)s;
    // the chunk padding past n must read as zero codes
    if ((int64_t)nb * kChunk > n) {
        const hipError_t e = hipMemsetAsync(w.code + n, 0, ((int64_t)nb * kChunk - n) * 2, st);
        LDM_REQUIRE(e == hipSuccess, (int)e, "ldm_mc_count: memset: %s", hipGetErrorString(e));
    }
    const int64_t quads = (int64_t)((N + 3) / 4) * N * N;
    const dim3 cgrid((unsigned)((quads + 255) / 256));
    if ((N & 3) == 0)
        hipLaunchKernelGGL(mc_classify_kernel<true>, cgrid, dim3(256), 0, st, vol, N, level,
                           w.code);
    else
        hipLaunchKernelGGL(mc_classify_kernel<false>, cgrid, dim3(256), 0, st, vol, N, level,
                           w.code);
    hipLaunchKernelGGL(mc_block_sums_kernel, dim3(nb), dim3(256), 0, st, w.code, n, w.bsum);
    hipLaunchKernelGGL(mc_chunk_scan_kernel, dim3(1), dim3(256), 0, st, w.bsum, nb, w.boff,
                       counts_out);
    return launch_status("ldm_mc_count");
}

extern "C" int ldm_mc_emit(const float* vol, int N, float level, float vs, float origin,
                           void* ws, size_t ws_bytes, float* verts, int32_t* faces,
                           ldm_stream_t s) {
    using namespace ldm;
    if (int e = check_mc(vol, N, ws, ws_bytes)) return e;
    const McWs w = mc_ws_layout(N, ws);
    const int64_t n = (int64_t)N * N * N;
    const int nb = (int)((n + kChunk - 1) / kChunk);
    hipStream_t st = (hipStream_t)s;
    if (verts)
        hipLaunchKernelGGL(mc_vertices_kernel, dim3(nb), dim3(256), 0, st, vol, N, level, vs,
                           origin, w.code, w.boff, w.vofs, verts);
    if (faces) {
        LDM_REQUIRE(verts, LDM_EINVAL, "ldm_mc_emit: faces need the vertex pass");
        hipLaunchKernelGGL(mc_faces_kernel, dim3(nb), dim3(256), 0, st, N, w.code, w.boff,
                           w.vofs, faces);
    }
    return launch_status("ldm_mc_emit");
}
