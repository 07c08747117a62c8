// Layout check (developer tool): block-diagonal use of v_mfma_f64_16x16x4_f64 for the
// Riccati quadratic forms of four independent 4x4 problems held one element per lane.
// Lane l <-> (instance i = (l >> 2) & 3, row a = l >> 4, column b = l & 3).
//   MFMA1: M_i = P_i G_i         (A = own P[a][b] (P symmetric), B = own G[a][b])
//   MFMA2: Z_i = G_i' M_i        (A = own G[a][b], B = own M[a][b])
//   MFMA3: z_i = G_i' pp_i       (A = pp[a] replicated over b, B = own G[a][b]) -> lane holds z[b]
// The useful result of each product is register i of the lane (the diagonal block).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double diag(d4 c, int i) {
    const double r01 = (i & 1) ? c[1] : c[0];
    const double r23 = (i & 1) ? c[3] : c[2];
    return (i & 2) ? r23 : r01;
}

__global__ void check(const double* P, const double* G, const double* pp, double* M, double* Z, double* z) {
    const int l = threadIdx.x;
    const int i = (l >> 2) & 3, a = l >> 4, b = l & 3;
    const double p = P[i * 16 + a * 4 + b];
    const double g = G[i * 16 + a * 4 + b];
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    const d4 c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(p, g, zero, 0, 0, 0);
    const double m = diag(c1, i);
    const d4 c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(g, m, zero, 0, 0, 0);
    const double zz = diag(c2, i);
    const d4 c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(pp[i * 4 + a], g, zero, 0, 0, 0);
    M[i * 16 + a * 4 + b] = m;
    Z[i * 16 + a * 4 + b] = zz;
    z[i * 16 + a * 4 + b] = diag(c3, i);
}

int main() {
    std::vector<double> P(64), G(64), pp(16);
    for (int i = 0; i < 4; ++i)
        for (int a = 0; a < 4; ++a) {
            pp[i * 4 + a] = 0.5 + i - 0.25 * a;
            for (int b = 0; b < 4; ++b) {
                G[i * 16 + a * 4 + b] = 1.0 + i * 16 + a * 4 + b * b * 0.5;        // asymmetric
                const int lo = a < b ? a : b, hi = a < b ? b : a;
                P[i * 16 + a * 4 + b] = 2.0 + i + lo * 3 + hi * 7 + (a == b ? 10.0 : 0.0);  // symmetric
            }
        }
    double *dP, *dG, *dpp, *dM, *dZ, *dz;
    CHK(hipMalloc(&dP, 512)); CHK(hipMalloc(&dG, 512)); CHK(hipMalloc(&dpp, 128));
    CHK(hipMalloc(&dM, 512)); CHK(hipMalloc(&dZ, 512)); CHK(hipMalloc(&dz, 512));
    CHK(hipMemcpy(dP, P.data(), 512, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dG, G.data(), 512, hipMemcpyHostToDevice));
    CHK(hipMemcpy(dpp, pp.data(), 128, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, dP, dG, dpp, dM, dZ, dz);
    CHK(hipDeviceSynchronize());
    std::vector<double> M(64), Z(64), z(64);
    CHK(hipMemcpy(M.data(), dM, 512, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(Z.data(), dZ, 512, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(z.data(), dz, 512, hipMemcpyDeviceToHost));
    double eM = 0, eZ = 0, ez = 0;
    for (int i = 0; i < 4; ++i) {
        double Mr[4][4], Zr[4][4], zr[4];
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) {
                double s = 0;
                for (int k = 0; k < 4; ++k) s += P[i * 16 + a * 4 + k] * G[i * 16 + k * 4 + b];
                Mr[a][b] = s;
            }
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) {
                double s = 0;
                for (int k = 0; k < 4; ++k) s += G[i * 16 + k * 4 + a] * Mr[k][b];
                Zr[a][b] = s;
            }
        for (int b = 0; b < 4; ++b) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += G[i * 16 + k * 4 + b] * pp[i * 4 + k];
            zr[b] = s;
        }
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) {
                eM = fmax(eM, fabs(M[i * 16 + a * 4 + b] - Mr[a][b]) / fabs(Mr[a][b]));
                eZ = fmax(eZ, fabs(Z[i * 16 + a * 4 + b] - Zr[a][b]) / fabs(Zr[a][b]));
                ez = fmax(ez, fabs(z[i * 16 + a * 4 + b] - zr[b]) / fabs(zr[b]));
            }
    }
    printf("mfma_f64 block-diagonal: rel err M %.3g  Z %.3g  z %.3g  -> %s\n", eM, eZ, ez,
           (eM < 1e-14 && eZ < 1e-14 && ez < 1e-14) ? "OK" : "MISMATCH");
    return (eM < 1e-14 && eZ < 1e-14 && ez < 1e-14) ? 0 : 2;
}
