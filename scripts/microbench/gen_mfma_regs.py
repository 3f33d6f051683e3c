"""Generates mfma_regs.hip: does a 32x32x16 bf16 MFMA k-step's speed depend on WHICH registers
hold its operands?  (the split decoder's part-0 plain loops -- B fragments
in v[0:35] -- run ~40 cycles per k-step slower than its part-1 loops -- B fragments in
v[128:187] -- with the same instructions; A in v[136:175] in both, accumulators a[128:255] vs
a[0:127].)  Each kernel runs the decoder's rolling k-step in inline asm on FIXED registers: per
step 8 MFMAs (2 A fragments x 4 B fragments, 8 accumulators of 16), each B fragment re-read
from LDS (ds_read_b128) right behind its MFMA pair; optionally the 2 A fragments of the step
reloaded from L2 4 steps ahead (buffer_load_dwordx4, the decoder's weight ring).  One
workgroup of 4 waves per CU (one per SIMD), every CU; wave 0 times 64 steps with s_memtime (after a register init).
Pass 0: constant operands; pass 1: pseudo-random bf16 (ReLU'd activations in LDS, signed weights).
python gen_mfma_regs.py > mfma_regs.hip && hipcc --offload-arch=gfx950 -O3 mfma_regs.hip -o mfma_regs"""

VARIANTS = [
    # name, A base (8 regs; "v" or "a"), B base (16 regs), C base (128 regs), ring (A reloads)
    ("dec_p0", "v136", "v0", "a128", 0),
    ("dec_p1", "v136", "v168", "a0", 0),
    ("A136_B0_C0", "v136", "v0", "a0", 0),
    ("A136_B168_C128", "v136", "v168", "a128", 0),
    ("A0_B16_C0", "v0", "v16", "a0", 0),
    ("A0_B16_C128", "v0", "v16", "a128", 0),
    ("A136_B200_C128", "v136", "v200", "a128", 0),
    ("A16_B0_C128", "v16", "v0", "a128", 0),
    ("A136_B64_C128", "v136", "v64", "a128", 0),
    ("ring_dec_p0", "v136", "v0", "a128", 1),
    ("ring_dec_p1", "v136", "v168", "a0", 1),
    ("ring_A136_B168_C128", "v136", "v168", "a128", 1),
    ("ring_A136_B0_C0", "v136", "v0", "a0", 1),
]


def reg(base, off, n):
    k, i = base[0], int(base[1:])
    return f"{k}[{i + off}:{i + off + n - 1}]"


def step(A, B, C, ring, slot, ldsoff):
    """One k-step: A fragments of ring slot `slot` (ring: 4 slots x 8 regs), B re-read from
    LDS at byte offset ldsoff."""
    s = []
    a0 = reg(A, 8 * slot if ring else 0, 4)
    a1 = reg(A, 8 * slot + 4 if ring else 4, 4)
    for n in range(4):
        s.append("s_waitcnt lgkmcnt(3)")
        s.append(f"v_mfma_f32_32x32x16_bf16 {reg(C, 32 * n, 16)}, {a0}, {reg(B, 4 * n, 4)}, {reg(C, 32 * n, 16)}")
        s.append(f"v_mfma_f32_32x32x16_bf16 {reg(C, 32 * n + 16, 16)}, {a1}, {reg(B, 4 * n, 4)}, {reg(C, 32 * n + 16, 16)}")
        s.append(f"ds_read_b128 {reg(B, 4 * n, 4)}, v250 offset:{ldsoff + 1024 * n}")
    if ring:
        # reload this slot's A fragments (consumed 4 steps later), as the decoder's issue()
        s.append(f"s_waitcnt vmcnt(6)")
        s.append(f"buffer_load_dwordx4 {a0}, v251, %4, 0 offen")
        s.append(f"buffer_load_dwordx4 {a1}, v251, %4, 0 offen offset:1024")
    return s


def clob(base, n):
    k, i = base[0], int(base[1:])
    return [f'"{k}{j}"' for j in range(i, i + n)]


def kernel(name, A, B, C, ring):
    init = []
    for n in range(4):
        init.append(f"ds_read_b128 {reg(B, 4 * n, 4)}, v250 offset:{1024 * n}")
    for q in range(8 if ring else 2):
        init.append(f"buffer_load_dwordx4 {reg(A, 4 * q, 4)}, v251, %4, 0 offen")
    for q in range(128):
        init.append(f"v_accvgpr_write_b32 {C[0]}{int(C[1:]) + q}, 0")
    init.append("s_waitcnt vmcnt(0) lgkmcnt(0)")
    init.append("s_memtime %0")
    init.append("s_waitcnt lgkmcnt(0)")
    body = []
    for rep in range(4):
        for j in range(16):
            body += step(A, B, C, ring, j % 4, (j % 16) * 4096)
    body += ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_memtime %1", "s_waitcnt lgkmcnt(0)"]
    asm = "\\n\\t".join(init + body)
    cl = clob(A, 32 if ring else 8) + clob(B, 16) + clob(C, 128) + ['"v250"', '"v251"', '"memory"']
    init = []
    # zero accumulators, load A/B once
    return f'''
__global__ __launch_bounds__(256, 1) void k_{name}(int reps, const void* wts, unsigned long long* out, int rnd) {{
    __shared__ __attribute__((aligned(16))) char smem[64 * 1024 + 4096];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < (64 * 1024 + 4096) / 4; i += 256) {{
        unsigned v;
        if (rnd) {{      // two ReLU'd bf16 of N(0, 1)-like magnitude: random sign / exponent / mantissa
            unsigned h = (unsigned)i * 2654435761u;
            h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
            unsigned lo = (h & 0x8000u) ? 0u : (0x3e00u + (h & 0x1ffu) * 0x4u + (h >> 20 & 0x7fu));
            unsigned hi = (h & 0x80000000u) ? 0u : (0x3e00u + (h >> 16 & 0x1ffu) * 0x4u + (h >> 9 & 0x7fu));
            v = lo | hi << 16;
        }} else {{
            const unsigned c[4] = {{0x3f803f80u ^ (unsigned)((i >> 2) & 7), 0x3c003f80u, 0xbf80u, 0x3f800000u}};
            v = c[i & 3];
        }}
        reinterpret_cast<unsigned*>(smem)[i] = v;
    }}
    __syncthreads();
    const unsigned lds = (unsigned)(uintptr_t)smem + lane * 16;
    const unsigned wof = (unsigned)(wave * 64 + lane) * 16;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(wts), (short)0, 0x7ffffff0, 0x00020000);
    unsigned long long t0 = 0, t1 = 0;
    for (int r = 0; r < reps; ++r) {{
        asm volatile("v_mov_b32 v250, %2\\n\\tv_mov_b32 v251, %3\\n\\t{asm}"
                     : "=s"(t0), "=s"(t1) : "v"(lds), "v"(wof), "s"(rs)
                     : {", ".join(cl)});
    }}
    if (lane == 0 && wave == 0) out[blockIdx.x] = t1 - t0;
}}
'''


def main():
    print('''// GENERATED by gen_mfma_regs.py -- see its docstring.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <vector>
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
''')
    for v in VARIANTS:
        print(kernel(*v))
    print('''
typedef void (*KFn)(int, const void*, unsigned long long*, int);
int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned long long* d;
    void* w;
    CHECK(hipMalloc(&d, (size_t)cus * 8));
    CHECK(hipMalloc(&w, 1 << 20));
    void* wr;
    CHECK(hipMalloc(&wr, 1 << 20));
    CHECK(hipMemset(w, 0x3c, 1 << 20));
    {   // random bf16 weights, He-like magnitudes (sign, exponent 2^-5..2^-3, mantissa)
        std::vector<unsigned short> hw(1 << 19);
        unsigned x = 12345u;
        for (auto& e : hw) {
            x = x * 1664525u + 1013904223u;
            e = (unsigned short)(((x >> 31) << 15) | ((0x3c + (x >> 28 & 3)) << 7 & 0x7f80) | (x >> 9 & 0x7f));
        }
        CHECK(hipMemcpy(wr, hw.data(), 1 << 20, hipMemcpyHostToDevice));
    }
    struct { const char* n; KFn f; } ks[] = {''')
    for v in VARIANTS:
        print(f'        {{"{v[0]}", k_{v[0]}}},')
    print('''    };
    for (int pass = 0; pass < 2; ++pass)
        for (auto& k : ks) {
            for (int it = 0; it < 3; ++it) {
                hipLaunchKernelGGL(k.f, dim3(cus), dim3(256), 0, 0, 8, (const void*)(pass ? wr : w), d, pass);
                CHECK(hipDeviceSynchronize());
            }
            std::vector<unsigned long long> h(cus);
            CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
            std::sort(h.begin(), h.end());
            printf("{\\"variant\\": \\"%s\\", \\"data\\": %d, \\"cycles_per_step\\": %.1f, \\"mfma_floor\\": 256}\\n",
                   k.n, pass, h[h.size() / 2] / 64.0);
        }
    return 0;
}''')


if __name__ == "__main__":
    main()
