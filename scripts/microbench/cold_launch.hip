// Microbenchmark: what the first loads of a kernel in a dependent launch chain pay, by who
// wrote the line -- the 1D-UNet graph path runs 18 such launches per step and its stamps show
// ~1-2 us per staging / epilogue-operand round trip.  Each node of a captured
// chain (grid 512 x 256 threads, the convs' shape; workgroup i runs on XCD i mod 8) writes one
// line per workgroup; thread 0 of workgroup 0 of each node stamps s_memtime around dependent
// loads of a line written by the PREVIOUS node:
//   same_xcd:     by workgroup 8 (same XCD as workgroup 0),
//   other_xcd:    by workgroup 1 (XCD 1),
//   other_xcd_2:  by workgroup 3 two nodes back,
//   untouched:    a line no node writes (read by every node),
//   same_again:   the same_xcd line again (now in this CU's path).
// An earlier version of this file timed straight-line s_nop code, cold vs warm: identical
// (profiles/r04f/cold_launch_code.json) -- instruction fetch is not a launch-start cost.
// Median over the chain's last 1000 nodes, s_memtime ticks.
// Build (here): hipcc --offload-arch=gfx950 -O3 cold_launch.hip -o cold_launch
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

constexpr int kSteps = 2000;
constexpr int kGrid = 512;
constexpr int kLine = 32;   // floats per 128-B line

__device__ __forceinline__ long long now() {
    long long t;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__device__ __forceinline__ float vload(const float* p) {
    float x = *(const volatile float*)p;
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(x) : "memory");
    return x;
}

// buffers b0, b1, b2 rotate: node n writes b[n % 3], reads b[(n - 1) % 3] and b[(n - 2) % 3]
__global__ __launch_bounds__(256) void probe(float* w, const float* p1, const float* p2,
                                             const float* cold, long long* st, int node) {
    long long t[6];
    float acc = 0.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t[0] = now();
        acc += vload(p1 + 8 * kLine);
        t[1] = now();
        acc += vload(p1 + 1 * kLine);
        t[2] = now();
        acc += vload(p2 + 3 * kLine);
        t[3] = now();
        acc += vload(cold + 5 * kLine);
        t[4] = now();
        acc += vload(p1 + 8 * kLine + 1);
        t[5] = now();
        long long* o = st + (size_t)node * 6;
        for (int i = 0; i < 5; ++i) o[i] = t[i + 1] - t[i];
        o[5] = (long long)acc;
    }
    if (threadIdx.x < kLine) w[blockIdx.x * kLine + threadIdx.x] = (float)(node + threadIdx.x);
}

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,            \
                    hipGetErrorString(e_));                                      \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *b[3], *cold;
    for (int i = 0; i < 3; ++i) {
        CK(hipMalloc(&b[i], kGrid * kLine * sizeof(float)));
        CK(hipMemset(b[i], 0, kGrid * kLine * sizeof(float)));
    }
    CK(hipMalloc(&cold, 64 * kLine * sizeof(float)));
    CK(hipMemset(cold, 0, 64 * kLine * sizeof(float)));
    long long* st;
    CK(hipMalloc(&st, (size_t)kSteps * 6 * sizeof(long long)));
    const char* names[5] = {"same_xcd", "other_xcd", "other_xcd_2", "untouched", "same_again"};
    for (int mode = 0; mode < 2; ++mode) {
        auto issue = [&]() {
            for (int i = 0; i < kSteps; ++i)
                hipLaunchKernelGGL(probe, dim3(kGrid), dim3(256), 0, s, b[i % 3],
                                   b[(i + 2) % 3], b[(i + 1) % 3], (const float*)cold, st, i);
        };
        hipGraphExec_t ge = nullptr;
        hipGraph_t g = nullptr;
        if (mode == 0) {
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            issue();
            CK(hipGetLastError());
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge, s));
            CK(hipGraphLaunch(ge, s));
        } else {
            issue();
            issue();
        }
        CK(hipStreamSynchronize(s));
        std::vector<long long> h((size_t)kSteps * 6);
        CK(hipMemcpy(h.data(), st, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
        printf("{\"mode\": \"%s\", \"grid\": %d, \"unit\": \"s_memtime ticks\"",
               mode == 0 ? "graph" : "stream", kGrid);
        for (int k = 0; k < 5; ++k) {
            std::vector<long long> v;
            for (int n = kSteps - 1000; n < kSteps; ++n) v.push_back(h[(size_t)n * 6 + k]);
            std::sort(v.begin(), v.end());
            printf(", \"%s\": %lld, \"%s_p90\": %lld", names[k], v[v.size() / 2], names[k],
                   v[v.size() * 9 / 10]);
        }
        printf("}\n");
        fflush(stdout);
        if (ge) {
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    }
    CK(hipStreamDestroy(s));
    return 0;
}
