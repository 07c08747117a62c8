// Where the matrix-core factor step's time goes (developer tool, one MI355X): the production step's
// dependence structure on register-resident operands, timed per wave with s_memtime at one and two
// waves per SIMD, against reduced forms of it.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o factor_step_lat scripts/ubench/factor_step_lat.hip
// Variants (cycles per step per wave):
//   0  the step as qsp_solver.hip factor_walk_mfma runs it (11 products, the R~ gather, 2x2 inverse)
//   1  the same products, R~ gather and inverse replaced by Xa = Z, idet = 1 (no VALU between products)
//   2  the critical chain alone: T2 -> Z -> Ka -> Pu (four dependent products)
//   3  one product chained through its B operand (x = mfma(c, x, 0))
//   4  one product chained through its C operand (x = mfma(a, b, x))
//   5  the R~ gather and inverse alone (permlane16_swap, DPP broadcasts, det, rcp: VALU chain)
//   6  four independent product chains (x_i = mfma(a, b, x_i)): the matrix-core pipe's issue rate
//   7  eight independent product chains
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double mfma4(double a, double b, double c) { return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0); }
template <int CTRL>
__device__ __forceinline__ double qb(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

template <int V>
__global__ void __launch_bounds__(64) steps(const double* in, double* out, long long* cyc, int n) {
    const int l = threadIdx.x;
    const int r = l >> 4, cc = l & 3;
    double P = in[l], pv = cc == 2 ? in[64 + l] : 0.0;
    const double Am = in[128 + l], G2 = in[192 + l], CH = in[256 + l], CZ = in[320 + l], gq = cc == 2 ? in[384 + l] : 0.0;
    double acc = 0.0, gqv = gq, e0 = 0.1, e1 = 0.2, e2 = 0.3, e3 = 0.4;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < n; ++k) {
        if constexpr (V == 0 || V == 1) {
            const double T1 = mfma4(P, Am, 0.0);
            const double T2 = mfma4(P, G2, pv);
            const double Y = mfma4(G2, T1, 0.0);
            const double Z = mfma4(G2, T2, CZ);
            const double Q = mfma4(Am, T1, CH);
            const double Qt = mfma4(T1, Am, CH);
            const double pp = cc == 2 ? T2 : 0.0;
            const double qv = mfma4(Am, pp, gq);
            double Xa, idet;
            if constexpr (V == 0) {
                const auto slo = __builtin_amdgcn_permlane16_swap(__double2loint(Z), __double2loint(Z), false, false);
                const auto shi = __builtin_amdgcn_permlane16_swap(__double2hiint(Z), __double2hiint(Z), false, false);
                const double w0 = __hiloint2double(shi[0], slo[0]), w1 = __hiloint2double(shi[1], slo[1]);
                const double R00 = qb<0x00>(w0), R01 = qb<0x55>(w0), R11 = qb<0x55>(w1);
                const double det = fma(R00, R11, -(R01 * R01));
                Xa = (r < 2 && cc < 2) ? (r != cc ? R01 : (r == 0 ? -R11 : -R00)) : 0.0;
                idet = rcp(det);
            } else {
                Xa = Z * 1e-3;
                idet = 1.0;
            }
            const double Ka = mfma4(Xa, Y, 0.0);
            const double Kf = Ka * (r < 2 ? idet : 0.0);
            acc += Z;
            const double RT = r < 2 && cc == 2 ? Z : 0.0;
            const double Pu = mfma4(Y, Kf, Q);
            const double Pl = mfma4(Kf, Y, Qt);
            P = (r <= cc ? Pu : Pl) * 0.5;
            pv = mfma4(Kf, RT, qv) * 0.5;
        } else if constexpr (V == 2) {
            const double T2 = mfma4(P, G2, pv);
            const double Z = mfma4(G2, T2, CZ);
            const double Ka = mfma4(Z, G2, 0.0);
            P = mfma4(G2, Ka, CH) * 0.5;
        } else if constexpr (V == 3) {
            P = mfma4(G2, P, 0.0);
        } else if constexpr (V == 4) {
            P = mfma4(G2, Am, P);
        } else if constexpr (V == 6) {
            P = mfma4(G2, Am, P);
            pv = mfma4(G2, Am, pv);
            acc = mfma4(CH, Am, acc);
            gqv = mfma4(CZ, Am, gqv);
        } else if constexpr (V == 7) {
            P = mfma4(G2, Am, P);
            pv = mfma4(G2, Am, pv);
            acc = mfma4(CH, Am, acc);
            gqv = mfma4(CZ, Am, gqv);
            e0 = mfma4(G2, CH, e0);
            e1 = mfma4(G2, CZ, e1);
            e2 = mfma4(CH, CZ, e2);
            e3 = mfma4(CZ, CH, e3);
        } else {
            const auto slo = __builtin_amdgcn_permlane16_swap(__double2loint(P), __double2loint(P), false, false);
            const auto shi = __builtin_amdgcn_permlane16_swap(__double2hiint(P), __double2hiint(P), false, false);
            const double w0 = __hiloint2double(shi[0], slo[0]), w1 = __hiloint2double(shi[1], slo[1]);
            const double R00 = qb<0x00>(w0), R01 = qb<0x55>(w0), R11 = qb<0x55>(w1);
            const double det = fma(R00, R11, -(R01 * R01)) + 2.0;
            P = rcp(det) + P * 0.5;
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + l] = P + pv + acc + gqv + e0 + e1 + e2 + e3;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(const char* name, const double* din, double* dout, long long* dcyc, int blocks) {
    const int n = 1000;
    for (int p = 0; p < 2; ++p) hipLaunchKernelGGL(steps<V>, dim3(blocks), dim3(64), 0, 0, din, dout, dcyc, n);
    static long long h[4096];
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, dcyc, blocks * 8, hipMemcpyDeviceToHost) != hipSuccess) {
        printf("%s: HIP error\n", name);
        return;
    }
    double m = 0;
    for (int i = 0; i < blocks; ++i) m += h[i];
    m /= blocks;
    printf("variant %d %-48s %4d waves (%d per SIMD): %7.1f cycles per step per wave\n", V, name, blocks, blocks / 1024,
           m / n);
}

int main() {
    double hin[448];
    for (int i = 0; i < 448; ++i) hin[i] = 0.25 + 0.001 * (i % 37) - 0.0005 * (i % 11);
    double *din, *dout;
    long long* dcyc;
    if (hipMalloc(&din, sizeof hin) != hipSuccess || hipMalloc(&dout, 4096 * 64 * 8) != hipSuccess ||
        hipMalloc(&dcyc, 4096 * 8) != hipSuccess)
        return 1;
    if (hipMemcpy(din, hin, sizeof hin, hipMemcpyHostToDevice) != hipSuccess) return 1;
    for (int blocks : {1024, 2048}) {
        run<0>("production step", din, dout, dcyc, blocks);
        run<1>("products only (no gather, no inverse)", din, dout, dcyc, blocks);
        run<2>("critical chain: 4 dependent products", din, dout, dcyc, blocks);
        run<3>("one product chained through B", din, dout, dcyc, blocks);
        run<4>("one product chained through C", din, dout, dcyc, blocks);
        run<5>("R~ gather + 2x2 inverse alone", din, dout, dcyc, blocks);
        run<6>("4 independent product chains (4 products)", din, dout, dcyc, blocks);
        run<7>("8 independent product chains (8 products)", din, dout, dcyc, blocks);
    }
    return 0;
}
