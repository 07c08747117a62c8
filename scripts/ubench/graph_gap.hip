// Launch-boundary cost of a chain of dependent kernels on one stream: plain stream launches
// vs the same chain captured once into a hipGraph and replayed (developer tool).
//
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench/graph_gap.hip -o scripts/ubench/graph_gap
//   ./scripts/ubench/graph_gap [kernels_per_chain] [spin_cycles]
//
// Each kernel is one wave that spins for `spin` cycles (s_memtime) and bumps a counter, so the
// chain's wall time minus kernels x spin is the per-boundary overhead the SQP loop pays between
// its QP launches and packing sorts.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

__global__ void spin_kernel(long long cycles, int* counter) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) counter[0] += 1;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 100;
    const long long spin = argc > 2 ? std::atoll(argv[2]) : 1000;
    int* counter;
    CK(hipMalloc(&counter, sizeof(int)));
    CK(hipMemset(counter, 0, sizeof(int)));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto chain = [&]() {
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, st, spin, counter);
    };
    // one kernel alone: its own duration (spin + dispatch)
    float one = 0.f;
    for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0, st));
        hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, st, spin, counter);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&one, e0, e1));
    }
    // plain stream launches
    float ms_stream = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0, st));
        chain();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < ms_stream) ms_stream = ms;
    }
    // captured graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    chain();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    float ms_graph = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < ms_graph) ms_graph = ms;
    }
    int cnt = 0;
    CK(hipMemcpy(&cnt, counter, sizeof(int), hipMemcpyDeviceToHost));
    std::printf("kernels %d spin %lld cycles: one kernel %.2f us; chain: stream %.2f us/kernel, graph %.2f us/kernel "
                "(counter %d)\n",
                n, spin, one * 1e3, ms_stream * 1e3 / n, ms_graph * 1e3 / n, cnt);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(st));
    CK(hipFree(counter));
    return 0;
}
