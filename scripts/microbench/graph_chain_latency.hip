// Microbenchmark: the latency of one dependent node in a hipGraph chain of kernel launches --
// the floor of the 1D-UNet sampler's graph path (1000 steps x 18 dependent ldm_conv1d launches,
// DESIGN.md §9), priced WITHOUT the convs' work: each node is an empty kernel of the given grid
// (256 threads per workgroup, the conv launches' shape), so a replay's time / its node count is
// what one dependent launch costs (launch, first wave, drain) on this box.
//
// For each grid in {64, 128, 256, 512, 1024, 2048}: capture STEPS x 18 launches on one stream into a
// graph, instantiate, replay once untimed, then REPS timed replays between hipEvents.  Prints one
// JSON line per grid: {"grid", "nodes", "node_ns_median", "node_ns_min"}.
//
// Build (here): hipcc --offload-arch=gfx950 -O3 graph_chain_latency.hip -o graph_chain_latency
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

constexpr int kSteps = 1000;
constexpr int kPerStep = 18;
constexpr int kReps = 7;

__global__ __launch_bounds__(256) void empty_node(int* sink, int tag) {
    if (tag < 0 && sink) sink[threadIdx.x] = tag;   // never taken: keeps the argument live
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
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grids[] = {64, 128, 256, 512, 1024, 2048};
    for (int grid : grids) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < kSteps * kPerStep; ++i)
            hipLaunchKernelGGL(empty_node, dim3(grid), dim3(256), 0, s, (int*)nullptr, i);
        CK(hipGetLastError());
        CK(hipStreamEndCapture(s, &g));
        hipGraphExec_t ge;
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        std::vector<float> ns;
        for (int r = 0; r < kReps; ++r) {
            CK(hipEventRecord(e0, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ns.push_back(ms * 1e6f / (kSteps * kPerStep));
        }
        std::sort(ns.begin(), ns.end());
        printf("{\"grid\": %d, \"threads\": 256, \"nodes\": %d, \"node_ns_median\": %.1f, "
               "\"node_ns_min\": %.1f, \"reps\": %d}\n",
               grid, kSteps * kPerStep, ns[ns.size() / 2], ns[0], kReps);
        fflush(stdout);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CK(hipStreamDestroy(s));
    return 0;
}
