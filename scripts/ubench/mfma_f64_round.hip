// Rounding probe (developer tool) for v_mfma_f64_4x4x4_4b_f64: which sequence of roundings does
// one output element D[i][j] = C[i][j] + sum_k A[k][i] B[k][j] go through?  (Layout as
// mfma_f64_probe.hip: lane l <-> block (l >> 2) & 3, element (l >> 4, l & 3); A read transposed.)
// Random operands over a wide exponent range plus cancellation-heavy cases; the host compares every
// element with candidate evaluation orders and prints how many elements each one reproduces.
// The oracle twin restates the matrix-core factor walk with the order that matches all of them.
// Usage: mfma_f64_round [trials]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void run(const double* A, const double* B, const double* C, double* D, int T) {
    const int t = blockIdx.x, l = threadIdx.x;
    if (t >= T) return;
    const size_t o = (size_t)t * 64 + l;
    D[o] = __builtin_amdgcn_mfma_f64_4x4x4f64(A[o], B[o], C[o], 0, 0, 0);
}

static double rnd_val(int mode) {
    const double m = 1.0 + (double)rand() / RAND_MAX;
    const int e = mode == 0 ? rand() % 41 - 20 : rand() % 7 - 3;
    const double s = (rand() & 1) ? -1.0 : 1.0;
    return s * ldexp(m, e);
}

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 20000;
    std::vector<double> A((size_t)T * 64), B((size_t)T * 64), C((size_t)T * 64), D((size_t)T * 64);
    srand(11);
    for (int t = 0; t < T; ++t) {
        const int mode = t % 3;   // 0 wide exponents, 1 narrow, 2 near-cancelling C
        for (int l = 0; l < 64; ++l) {
            const size_t o = (size_t)t * 64 + l;
            A[o] = rnd_val(mode);
            B[o] = rnd_val(mode);
            C[o] = rnd_val(mode);
        }
        if (mode == 2) {   // C close to minus the product sum: heavy cancellation
            for (int l = 0; l < 64; ++l) {
                const int blk = (l >> 2) & 3, i = l >> 4, j = l & 3;
                long double s = 0;
                for (int k = 0; k < 4; ++k) s += (long double)A[(size_t)t * 64 + k * 16 + blk * 4 + i] * B[(size_t)t * 64 + k * 16 + blk * 4 + j];
                C[(size_t)t * 64 + l] = -(double)s * (1.0 + ldexp((double)(rand() % 64), -52));
            }
        }
    }
    double *dA, *dB, *dC, *dD;
    const size_t bytes = (size_t)T * 64 * 8;
    if (hipMalloc(&dA, bytes) || hipMalloc(&dB, bytes) || hipMalloc(&dC, bytes) || hipMalloc(&dD, bytes)) return 1;
    hipMemcpy(dA, A.data(), bytes, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), bytes, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), bytes, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(run, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD, T);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    hipMemcpy(D.data(), dD, bytes, hipMemcpyDeviceToHost);
    const char* names[] = {"fma chain k=0..3 from C", "fma chain k=3..0 from C", "fma chain k=0..3, C added last",
                           "exact sum, one rounding (binary128)", "pairwise (a0b0+a1b1)+(a2b2+a3b3)+C, fma", "products rounded, summed k=0..3 from C"};
    const int NC = 6;
    long match[NC] = {0}, total = 0;
    long by_mode[3][NC] = {{0}}, tot_mode[3] = {0};
    for (int t = 0; t < T; ++t)
        for (int l = 0; l < 64; ++l) {
            const int blk = (l >> 2) & 3, i = l >> 4, j = l & 3;
            double a[4], b[4];
            for (int k = 0; k < 4; ++k) {
                a[k] = A[(size_t)t * 64 + k * 16 + blk * 4 + i];
                b[k] = B[(size_t)t * 64 + k * 16 + blk * 4 + j];
            }
            const double c = C[(size_t)t * 64 + l], d = D[(size_t)t * 64 + l];
            double cand[NC];
            double x = c;
            for (int k = 0; k < 4; ++k) x = fma(a[k], b[k], x);
            cand[0] = x;
            x = c;
            for (int k = 3; k >= 0; --k) x = fma(a[k], b[k], x);
            cand[1] = x;
            x = a[0] * b[0];
            for (int k = 1; k < 4; ++k) x = fma(a[k], b[k], x);
            cand[2] = x + c;
            __float128 q = c;
            for (int k = 0; k < 4; ++k) q += (__float128)a[k] * (__float128)b[k];
            cand[3] = (double)q;
            cand[4] = fma(a[3], b[3], a[2] * b[2]) + fma(a[1], b[1], a[0] * b[0]) + c;
            x = c;
            for (int k = 0; k < 4; ++k) x = x + a[k] * b[k];
            cand[5] = x;
            const int mode = t % 3;
            ++total;
            ++tot_mode[mode];
            for (int n = 0; n < NC; ++n)
                if (memcmp(&cand[n], &d, 8) == 0) { ++match[n]; ++by_mode[mode][n]; }
        }
    printf("v_mfma_f64_4x4x4_4b_f64 rounding probe: %ld elements (%d trials)\n", total, T);
    for (int n = 0; n < NC; ++n)
        printf("  %-44s %ld / %ld   (wide %ld/%ld, narrow %ld/%ld, cancelling %ld/%ld)\n", names[n], match[n], total,
               by_mode[0][n], tot_mode[0], by_mode[1][n], tot_mode[1], by_mode[2][n], tot_mode[2]);
    return 0;
}
