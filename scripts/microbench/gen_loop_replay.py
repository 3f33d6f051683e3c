"""Generates loop_replay.hip: the split decoder's compiled plain k-step loops, replayed
VERBATIM in inline asm.  scripts/microbench/mfma_regs showed that the
registers and the data of a k-step do not change its speed (257 cycles per step, the MFMA
floor); this asks whether the decoder's OWN loop bodies -- a part-0 one (~320 cycles per step
inside the decoder) and a part-1 one (~278) -- are slow by themselves or only in the kernel.
The bodies are read from the disassembly of dec_fs_kernel<bf16, 256, grid> (llvm-objdump of the
gfx950 code object; the listing is an argument), the loop branch replaced by a 64-iteration
count and the LDS base wrapped at 64 KiB.  One workgroup of 4 waves per CU, every CU, wave 0
times the 256 steps with s_memtime.
python gen_loop_replay.py <dfs.dis> > loop_replay.hip && hipcc --offload-arch=gfx950 -O3 loop_replay.hip -o loop_replay"""
import re
import sys

KERN = "dec_fs_kernelIDF16bLi256ELb0ELi2E"


def loops(dis):
    txt = open(dis).read().split("\n")
    start = [i for i, l in enumerate(txt) if KERN in l and l.endswith(">:")][0]
    end = [i for i, l in enumerate(txt) if i > start and l.endswith(">:")]
    end = end[0] if end else len(txt)
    ins = []
    for l in txt[start:end]:
        m = re.match(r"\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):", l)
        if m:
            ins.append((int(m.group(2), 16), m.group(1).strip()))
    out = []
    for a, t in ins:
        m = re.match(r"s_cbranch_scc1 (\d+)", t)
        if m and int(m.group(1)) > 65000:
            s0 = a + 4 + (int(m.group(1)) - 65536) * 4
            out.append([x[1] for x in ins if s0 <= x[0] <= a])
    return out


def _late_vm(body):
    """every vmcnt wait removed from the MFMA side; `s_waitcnt vmcnt(6)` before each pair of
    ring loads instead (the slot reloaded must be consumed; the one consumed next has arrived)"""
    out = []
    for t in body:
        if t.startswith("s_waitcnt"):
            parts = [p for p in t.split()[1:] if not p.startswith("vmcnt")]
            if parts:
                out.append("s_waitcnt " + " ".join(parts))
            continue
        if t.startswith("buffer_load") and (not out or not out[-1].startswith("buffer_load")):
            out.append("s_waitcnt vmcnt(6)")
        out.append(t)
    return out


def _no_vm(body):
    """no vmcnt waits at all (the ring's data is never waited for: timing only)"""
    out = []
    for t in body:
        if t.startswith("s_waitcnt"):
            parts = [p for p in t.split()[1:] if not p.startswith("vmcnt")]
            if parts:
                out.append("s_waitcnt " + " ".join(parts))
            continue
        out.append(t)
    return out


def _no_loads(body):
    """no ring loads (and no vmcnt waits)"""
    return [t for t in _no_vm(body) if not t.startswith("buffer_load")]


def _bar(every):
    """a workgroup barrier (the decoder's fs_bar: lgkmcnt(0) + s_barrier) at the top of every
    `every`-th 4-step group: the body repeated every // 4 times, the barrier before the first
    copy -- the waves restart in lock step, as after the decoder's in-step barriers"""
    def f(body):
        core, tail = body[:-2], body[-2:]
        return ["s_waitcnt lgkmcnt(0)", "s_barrier"] + core * (every // 4 - 1) + core + tail
    return f


VARIANTS = [("L1p1_late_vm", _late_vm), ("L1p1_no_vm", _no_vm), ("L1p1_no_loads", _no_loads),
            ("L1p1_bar4", _bar(4)), ("L1p1_bar16", _bar(16)), ("L7p0_bar16", None)]


def kernel(name, body):
    # the loop counter compare / branch -> our own; the LDS group base (s2 or s13 / s0 ...)
    # wrapped: every s_addk_i32 sX, 0x4000 gets an s_and to 64 KiB
    b = []
    for t in body[:-2]:
        b.append(t)
        m = re.match(r"s_addk_i32 (s\d+), 0x4000", t)
        if m:
            b.append(f"s_and_b32 {m.group(1)}, {m.group(1)}, 0xffff")
    cmpreg = re.match(r"s_cmp_lt_u32 (s\d+), \d+", body[-2]).group(1)
    lab = f"L_{name}_%="
    loop = [f"{lab}:"] + b + [f"s_cmp_lt_u32 {cmpreg}, 256", f"s_cbranch_scc1 {lab}"]
    # registers the body names
    regs = set()
    for t in body:
        for k, lo, hi in re.findall(r"([vas])\[(\d+):(\d+)\]", t):
            regs |= {f"{k}{j}" for j in range(int(lo), int(hi) + 1)}
        for k, j in re.findall(r"\b([vas])(\d+)\b", t):
            regs.add(f"{k}{j}")
    sregs = sorted((r for r in regs if r[0] == "s"), key=lambda r: int(r[1:]))
    pro = ["s_mov_b32 s16, %2", "s_mov_b32 s17, %3", "s_mov_b32 s18, %4", "s_mov_b32 s19, %5"]
    for r in sregs:
        if r not in ("s16", "s17", "s18", "s19"):
            pro.append(f"s_mov_b32 {r}, 0")
    pro += ["s_mov_b32 s40, 0x40000", "s_mov_b32 s39, 0"]
    for j, off in zip((248, 249, 250, 251), (0, 1024, 2048, 3072)):
        pro.append(f"v_add_u32 v{j}, {off}, %6")
    asm = pro + ["s_waitcnt lgkmcnt(0)", "s_memtime %0", "s_waitcnt lgkmcnt(0)"] + loop + \
        ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_memtime %1", "s_waitcnt lgkmcnt(0)"]
    clob = sorted(regs | {"v248", "v249", "v250", "v251", "s16", "s17", "s18", "s19", "s39", "s40"})
    clob = [f'"{r}"' for r in clob] + ['"scc"', '"memory"']
    txt = "\\n\\t".join(asm)
    return f'''
__global__ __launch_bounds__(256, 1) void k_{name}(const void* wts, unsigned long long* out) {{
    __shared__ __attribute__((aligned(16))) char smem[128 * 1024];
    for (int i = threadIdx.x; i < 128 * 1024 / 4; i += 256)
        reinterpret_cast<unsigned*>(smem)[i] = 0x3e803f00u ^ (unsigned)(i * 2654435761u >> 7 & 0x007f007fu);
    __syncthreads();
    const unsigned voff = (threadIdx.x & 63) * 16 + (unsigned)(uintptr_t)smem * 0;
    // raw buffer resource words: base (48 bits, stride 0), num_records, the raw dword flags
    const unsigned long long base = (unsigned long long)(uintptr_t)wts;
    const unsigned w[4] = {{(unsigned)base, (unsigned)(base >> 32) & 0xffffu, 0x7ffffff0u, 0x00020000u}};
    unsigned long long t0, t1;
    asm volatile("{txt}"
                 : "=s"(t0), "=s"(t1) : "s"(w[0]), "s"(w[1]), "s"(w[2]), "s"(w[3]), "v"(voff)
                 : {", ".join(clob)});
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}}
'''


def main():
    ls = loops(sys.argv[1])
    names = ["L1p0", "L1p1", "L2p0", "L2p1", "L3p0", "L4p0", "L56p0", "L56p1", "L7p0", "L7p1"]
    assert len(ls) == len(names), len(ls)
    print('''// GENERATED by gen_loop_replay.py from the decoder's disassembly -- see its docstring.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <vector>
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
''')
    for n, b in zip(names, ls):
        print(kernel(n, b))
    # variants of L1p1's body: where the ring's vmcnt waits sit
    base = ls[1]
    for vn, f in VARIANTS:
        print(kernel(vn, _bar(16)(ls[8]) if f is None else f(base)))
    names += [vn for vn, _ in VARIANTS]
    print('''typedef void (*KFn)(const void*, unsigned long long*);
int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned long long* d;
    void* w;
    CHECK(hipMalloc(&d, (size_t)cus * 8));
    CHECK(hipMalloc(&w, 1 << 20));
    CHECK(hipMemset(w, 0x3c, 1 << 20));
    struct { const char* n; KFn f; } ks[] = {''')
    for n in names:
        print(f'        {{"{n}", k_{n}}},')
    print('''    };
    for (int pass = 0; pass < 2; ++pass)
        for (auto& k : ks) {
            for (int it = 0; it < 3; ++it) {
                hipLaunchKernelGGL(k.f, dim3(cus), dim3(256), 0, 0, (const void*)w, d);
                CHECK(hipDeviceSynchronize());
            }
            std::vector<unsigned long long> h(cus);
            CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
            std::sort(h.begin(), h.end());
            printf("{\\"loop\\": \\"%s\\", \\"pass\\": %d, \\"cycles_per_step\\": %.1f, \\"mfma_floor\\": 256}\\n",
                   k.n, pass, h[h.size() / 2] / 256.0);
        }
    return 0;
}''')


if __name__ == "__main__":
    main()
