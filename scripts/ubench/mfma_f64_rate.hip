// Throughput and dependent latency of v_mfma_f64_4x4x4_4b_f64 and v_mfma_f64_16x16x4_f64 on one
// wave (developer tool): cycles per instruction from s_memtime over a long unrolled loop.
// Measured (profiles/r02/mfma_f64_rate.txt): 4x4x4_4b dependent latency 48 cycles, 18 cycles per
// instruction with 8 independent accumulators (256 FMA: 14 FMA/cycle/SIMD); 16x16x4 64 cycles
// either way (16 FMA/cycle, the FP64 peak).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int CHAINS>
__global__ void rate4(double* out, long* cyc, int iters) {
    double acc[CHAINS];
    const double a = 1.0 + threadIdx.x * 1e-3, b = 0.5 - threadIdx.x * 1e-4;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = c;
    const long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[c], 0, 0, 0);
    }
    const long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CHAINS>
__global__ void rate16(double* out, long* cyc, int iters) {
    d4 acc[CHAINS];
    const double a = 1.0 + threadIdx.x * 1e-3, b = 0.5 - threadIdx.x * 1e-4;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = (d4){(double)c, 0, 0, 0};
    const long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
    const long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += acc[c][0] + acc[c][3];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run(K k, const char* name, int chains, int blocks) {
    double* o; long* c;
    if (hipMalloc(&o, blocks * 64 * 8) != hipSuccess) return;
    if (hipMalloc(&c, blocks * 8) != hipSuccess) return;
    const int iters = 2000;
    for (int p = 0; p < 2; ++p) hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, o, c, iters);
    long h[2048];
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, c, blocks * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    double m = 0;
    for (int i = 0; i < blocks; ++i) m += h[i];
    m /= blocks;
    printf("%-28s chains %2d, %5d waves: %.1f cycles per MFMA (per chain step %.1f)\n", name, chains, blocks,
           m / (iters * (double)chains), m / iters);
    (void)hipFree(o);
    (void)hipFree(c);
}

int main() {
    // one wave per SIMD (1 024 waves) and two (2 048)
    for (int w : {1024, 2048}) {
        run(rate4<1>, "mfma_f64_4x4x4_4b", 1, w);
        run(rate4<4>, "mfma_f64_4x4x4_4b", 4, w);
        run(rate4<8>, "mfma_f64_4x4x4_4b", 8, w);
        run(rate16<1>, "mfma_f64_16x16x4", 1, w);
        run(rate16<4>, "mfma_f64_16x16x4", 4, w);
    }
    return 0;
}
