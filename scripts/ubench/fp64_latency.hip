// Microbenchmark (developer tool): dependent-issue latency of FP64 FMA and of a DPP move on
// gfx950, one wave on one SIMD, cycles from s_memtime.  Informs how much ILP a walk step
// needs.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CHAINS>
__global__ void fma_chain(double* out, long long* cyc, int n) {
    double v[CHAINS];
    for (int c = 0; c < CHAINS; ++c) v[c] = out[threadIdx.x & 63] + c;
    const double a = out[64 + (threadIdx.x & 63)], b = out[128 + (threadIdx.x & 63)];
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) v[c] = fma(v[c], a, b);
    }
    const long long t1 = clock64();
    double s = 0;
    for (int c = 0; c < CHAINS; ++c) s += v[c];
    out[256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void dpp_chain(double* out, long long* cyc, int n) {
    int x = __double2loint(out[threadIdx.x]);
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
        x = __builtin_amdgcn_update_dpp(x, x, 0x130, 0xf, 0xf, false);
        x = x + 1;
    }
    const long long t1 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error line %d\n", __LINE__); return 1; } } while (0)

template <int CHAINS>
static int run(double* d, long long* c, int n, int threads) {
    long long h = 0;
    hipLaunchKernelGGL(fma_chain<CHAINS>, 1, threads, 0, 0, d, c, n);
    CK(hipGetLastError());
    CK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
    const int wps = threads / 256;   // waves per SIMD (4 SIMDs per CU)
    printf("%2d chain(s), %d wave(s)/SIMD: %6.2f cycles per FMA of one wave, %5.2f cycles per FMA per SIMD\n",
           CHAINS, wps, (double)h / ((double)CHAINS * n), (double)h / ((double)CHAINS * n * wps));
    return 0;
}

int main() {
    double* d; long long* c;
    CK(hipMalloc(&d, 4096 * 8)); CK(hipMemset(d, 0, 4096 * 8)); CK(hipMalloc(&c, 8));
    const int n = 4096;
    for (int threads : {256, 256, 512}) {
        if (run<1>(d, c, n, threads) || run<2>(d, c, n, threads) || run<4>(d, c, n, threads) ||
            run<8>(d, c, n, threads) || run<16>(d, c, n, threads))
            return 1;
    }
    long long h = 0;
    hipLaunchKernelGGL(dpp_chain, 1, 64, 0, 0, d, c, n);
    CK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
    printf("dpp+add : %.2f cycles per dependent (v_mov_dpp wave_shl:1, v_add_u32) pair\n", (double)h / n);
    return 0;
}
