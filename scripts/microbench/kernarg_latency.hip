// Microbenchmark: the latency of a kernel's first scalar reads of its OWN ARGUMENTS (the
// kernarg segment) inside a dependent launch chain -- ldm_conv1d passes a ~1 KiB argument
// block (the call + its LDS plan) and reads its fields through scalar loads as it goes, and
// its stamps show ~2 us of staging for a conv with one input channel.
// A 1 KiB by-value struct; thread 0 of workgroup 0 of each node stamps s_memtime around
// dependent volatile scalar reads of: line 0 (first touch), line 4 (first touch of another
// line), line 0 again (warm), a 1 KiB device buffer's line 0 through a constant-address-space
// pointer (the same read from device memory written once at setup), and line 8 + line 12
// issued together (two misses in one round trip).
// Both a captured graph chain and plain stream launches; median over the last 1000 nodes.
// Build (here): hipcc --offload-arch=gfx950 -O3 kernarg_latency.hip -o kernarg_latency
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

constexpr int kSteps = 2000;
constexpr int kGrid = 512;

struct Big {
    int v[256];   // 1 KiB: 16 lines of 64 B
    long long* st;
    int node;
};

#define AS4 __attribute__((address_space(4)))

__device__ __forceinline__ long long now() {
    long long t;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__device__ __forceinline__ int sread(const AS4 int* p) {
    int x;
    asm volatile("s_load_dword %0, %1, 0x0\n s_waitcnt lgkmcnt(0)" : "=s"(x) : "s"(p) : "memory");
    return x;
}

__device__ __forceinline__ int sread2(const AS4 int* p, const AS4 int* q) {
    int x, y;
    asm volatile("s_load_dword %0, %2, 0x0\n s_load_dword %1, %3, 0x0\n s_waitcnt lgkmcnt(0)"
                 : "=&s"(x), "=&s"(y)
                 : "s"(p), "s"(q)
                 : "memory");
    return x + y;
}

__global__ __launch_bounds__(256) void probe(Big k, const AS4 int* dev) {
    const AS4 int* kp = (const AS4 int*)__builtin_amdgcn_kernarg_segment_ptr();
    long long t[6];
    int acc = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::"s"(dev) : "memory");   // the pointer itself: loaded first
    t[0] = now();
    acc += sread(kp + 0);
    t[1] = now();
    acc += sread(kp + 64);
    t[2] = now();
    acc += sread(kp + 1);
    t[3] = now();
    acc += sread(dev);
    t[4] = now();
    acc += sread2(kp + 128, kp + 192);
    t[5] = now();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        long long* o = k.st + (size_t)k.node * 6;
        for (int i = 0; i < 5; ++i) o[i] = t[i + 1] - t[i];
        o[5] = acc;
    }
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

int report(const char* mode, long long* st) {
    std::vector<long long> h((size_t)kSteps * 6);
    CK(hipMemcpy(h.data(), st, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
    const char* names[5] = {"kernarg_line0_first", "kernarg_line4_first", "kernarg_line0_again",
                            "device_buffer_line0", "kernarg_lines8_12_together"};
    printf("{\"mode\": \"%s\", \"grid\": %d, \"unit\": \"s_memtime ticks (x ~0.41 ns)\"", mode,
           kGrid);
    for (int k = 0; k < 5; ++k) {
        std::vector<long long> v;
        for (int n = kSteps - 1000; n < kSteps; ++n) v.push_back(h[(size_t)n * 6 + k]);
        std::sort(v.begin(), v.end());
        printf(", \"%s\": %lld", names[k], v[v.size() / 2]);
    }
    printf("}\n");
    fflush(stdout);
    return 0;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    long long* st;
    int* dev;
    CK(hipMalloc(&st, (size_t)kSteps * 6 * sizeof(long long)));
    CK(hipMalloc(&dev, 1024));
    CK(hipMemset(dev, 0, 1024));
    Big k = {};
    k.st = st;
    // graph chain
    hipGraph_t g;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < kSteps; ++i) {
        k.node = i;
        hipLaunchKernelGGL(probe, dim3(kGrid), dim3(256), 0, s, k, (const AS4 int*)dev);
    }
    CK(hipGetLastError());
    CK(hipStreamEndCapture(s, &g));
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    if (report("graph", st)) return 1;
    // plain stream launches
    for (int rep = 0; rep < 2; ++rep)
        for (int i = 0; i < kSteps; ++i) {
            k.node = i;
            hipLaunchKernelGGL(probe, dim3(kGrid), dim3(256), 0, s, k, (const AS4 int*)dev);
        }
    CK(hipStreamSynchronize(s));
    if (report("stream", st)) return 1;
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(s));
    return 0;
}
