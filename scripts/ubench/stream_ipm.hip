// Feasibility micro-benchmark (developer tool): the memory traffic of an
// "instance per lane" interior point — every lane owns one NMPC instance and walks its
// 21 stages four times per IPM iteration, with all per-stage data in HBM (SoA across
// instances, coalesced).  Arithmetic is a token dependent chain; only the bytes are real.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int NS = 21;   // stages
// field blocks (doubles per stage)
constexpr int F_LIN = 24, F_ST = 15, F_PEND = 8, F_FAC = 17, F_DA = 3, F_DN = 3, F_KK = 2;
constexpr int F_TOT = F_LIN + F_ST + F_PEND + F_FAC + F_DA + F_DN + F_KK;

__device__ __forceinline__ size_t at(int f, int k, int i, int B) { return ((size_t)f * NS + k) * B + i; }

__global__ void __launch_bounds__(256) ipm_stream(double* w, int B, int iters) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    double acc = 0.0;
    for (int it = 0; it < iters; ++it) {
        // P1 backward: lin + state + pending -> factors, state
        for (int k = NS - 1; k >= 0; --k) {
            double s = acc;
            for (int f = 0; f < F_LIN + F_ST + F_PEND; ++f) s += w[at(f, k, i, B)];
            for (int f = 0; f < F_FAC; ++f) w[at(F_LIN + F_ST + F_PEND + f, k, i, B)] = s * 1e-30 + f;
            for (int f = 0; f < 14; ++f) w[at(F_LIN + f, k, i, B)] = s * 1e-30;
            acc = s * 1e-30;
        }
        // P2 forward: factors + lin(18) + state -> dv_aff
        for (int k = 0; k < NS; ++k) {
            double s = acc;
            for (int f = 0; f < 10; ++f) s += w[at(F_LIN + F_ST + F_PEND + f, k, i, B)];
            for (int f = 0; f < 18; ++f) s += w[at(f, k, i, B)];
            for (int f = 0; f < F_ST; ++f) s += w[at(F_LIN + f, k, i, B)];
            for (int f = 0; f < F_DA; ++f) w[at(F_LIN + F_ST + F_PEND + F_FAC + f, k, i, B)] = s * 1e-30;
            acc = s * 1e-30;
        }
        // P3 backward vector: 53 reads, kk
        for (int k = NS - 1; k >= 0; --k) {
            double s = acc;
            for (int f = 0; f < 20; ++f) s += w[at(f, k, i, B)];
            for (int f = 0; f < 15; ++f) s += w[at(F_LIN + F_ST + F_PEND + f, k, i, B)];
            for (int f = 0; f < F_ST; ++f) s += w[at(F_LIN + f, k, i, B)];
            for (int f = 0; f < F_DA; ++f) s += w[at(F_LIN + F_ST + F_PEND + F_FAC + f, k, i, B)];
            for (int f = 0; f < F_KK; ++f) w[at(F_TOT - F_KK + f, k, i, B)] = s * 1e-30;
            acc = s * 1e-30;
        }
        // P4 forward corrector: 46 reads, dv
        for (int k = 0; k < NS; ++k) {
            double s = acc;
            for (int f = 0; f < 8; ++f) s += w[at(F_LIN + F_ST + F_PEND + f, k, i, B)];
            for (int f = 0; f < F_KK; ++f) s += w[at(F_TOT - F_KK + f, k, i, B)];
            for (int f = 0; f < 18; ++f) s += w[at(f, k, i, B)];
            for (int f = 0; f < F_ST; ++f) s += w[at(F_LIN + f, k, i, B)];
            for (int f = 0; f < F_DA; ++f) s += w[at(F_LIN + F_ST + F_PEND + F_FAC + f, k, i, B)];
            for (int f = 0; f < F_DN; ++f) w[at(F_LIN + F_ST + F_PEND + F_FAC + F_DA + f, k, i, B)] = s * 1e-30;
            acc = s * 1e-30;
        }
    }
    if (acc == 12345.0) w[i] = acc;
}

int main() {
    const int iters = 9;
    for (int B : {16384, 32768, 65536}) {
        const size_t n = (size_t)F_TOT * NS * B;
        double* w;
        CHK(hipMalloc(&w, n * 8));
        CHK(hipMemset(w, 0, n * 8));
        hipEvent_t a, b;
        CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
        for (int bs : {64, 128, 256}) {
            const int grid = (B + bs - 1) / bs;
            hipLaunchKernelGGL(ipm_stream, dim3(grid), dim3(bs), 0, 0, w, B, iters);
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(a));
            for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(ipm_stream, dim3(grid), dim3(bs), 0, 0, w, B, iters);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms;
            CHK(hipEventElapsedTime(&ms, a, b));
            ms /= 3;
            const double bytes = (double)B * NS * iters * (47 + 31 + 43 + 3 + 53 + 2 + 46 + 3) * 8.0;
            printf("B=%6d block=%3d  %.3f ms per launch  (%.2f GB moved, %.2f TB/s)\n", B, bs, ms, bytes / 1e9,
                   bytes / (ms * 1e-3) / 1e12);
        }
        CHK(hipFree(w));
    }
    return 0;
}
