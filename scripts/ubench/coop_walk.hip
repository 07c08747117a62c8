// Microbenchmark (developer tool): the QP kernel's factor walk (qsp_solver.hip riccati_solve<1, true>)
// as the production DPP lane walk against a cooperative walk across the waves of a workgroup.
//
// Both kernels run R "IPM iterations" on the production lane layout (N = 20: an instance = 21 lanes, 3
// instances per wave, lane k holds stage k) and hold 17.9 KB of LDS per wave like the QP kernel, i.e.
// two waves per SIMD.  An iteration is X FP64 FMAs per lane standing in for the stage-parallel phases
// (4 independent chains), then the factorisation of every instance (ric_factor_step, the production
// step, copied below).
//   dpp:  one-wave workgroups; the value function (P, p) is handed from lane k+1 to lane k by DPP, one
//         stage per step; every step is issued by the whole wave for its 3 instances.
//   coop: four-wave workgroups (12 instances); ONE wave (rotating with the iteration) walks all 12
//         instances, one lane per instance, the value function in its registers.  The owners of stage
//         k-1 put its inputs into a 2-slot LDS ring while the walker factors stage k; the walker puts
//         K, Rn, kk into a 2-slot output ring; one workgroup barrier per step.  The walk's VALU
//         instructions are issued once per workgroup instead of once per wave.
// The factors (K, Rn, kk) of both kernels must be bit-identical: the same step on the same values.
// Usage: coop_walk [X] [reps] [instances]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../uclv_qs_pushing_matlab_amd/csrc/qsp_fp.hpp"
using qsp::qfma;
using qsp::rcp;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int N = 20, L = N + 1, G = 3;
constexpr int NIN = 30;                      // a 6, B 8, bb 4, Hx 4, Hu 2, gx 4, gu 2
constexpr int NOUT = 14;                     // K 8, Rn 3, kk 2, pad
constexpr int LDS_WAVE = 35 * 64 * 8;        // the QP kernel's per-wave LDS block (S = 1)
constexpr int WAVES = 4;                     // coop: waves per workgroup
constexpr int WI = WAVES * G;                // coop: instances per workgroup

__device__ __forceinline__ int sidx(int i, int j) {
    if (i > j) { int t = i; i = j; j = t; }
    return i == 0 ? j : (i == 1 ? 3 + j : (i == 2 ? 5 + j : 9));
}
__device__ __forceinline__ double from_next(double old, double v) {   // lane i <- lane i+1
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// ---- the production step (qsp_solver.hip)
__device__ __forceinline__ void ric_factor_step(const double a[6], const double B[8], const double bb[4],
                                                const double Hx[4], const double Hu[2],
                                                const double gx[4], const double gu[2],
                                                double P[10], double pv[4],
                                                double K[8], double Rn[3], double kk[2], bool upd = true) {
    // full symmetric P
    double Pm[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) Pm[i][j] = P[sidx(i, j)];
    // PA (columns 0, 1 of A are e0, e1)
    double PA[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        PA[i][0] = Pm[i][0];
        PA[i][1] = Pm[i][1];
        PA[i][2] = qfma(Pm[i][1], a[2], qfma(Pm[i][0], a[0], Pm[i][2]));
        PA[i][3] = qfma(Pm[i][3], a[5], qfma(Pm[i][2], a[4], qfma(Pm[i][1], a[3], Pm[i][0] * a[1])));
    }
    // PB
    double PB[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            PB[i][j] = qfma(Pm[i][3], B[6 + j], qfma(Pm[i][2], B[4 + j], qfma(Pm[i][1], B[2 + j], Pm[i][0] * B[j])));
    // pp = p + P b
    double pp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        pp[i] = qfma(Pm[i][3], bb[3], qfma(Pm[i][2], bb[2], qfma(Pm[i][1], bb[1], qfma(Pm[i][0], bb[0], pv[i]))));
    // R~ = Hu + B'PB (sym), S~ = B'PA (2x4), r~ = gu + B'pp
    const double R00 = qfma(B[6], PB[3][0], qfma(B[4], PB[2][0], qfma(B[2], PB[1][0], qfma(B[0], PB[0][0], Hu[0]))));
    const double R01 = qfma(B[6], PB[3][1], qfma(B[4], PB[2][1], qfma(B[2], PB[1][1], B[0] * PB[0][1])));
    const double R11 = qfma(B[7], PB[3][1], qfma(B[5], PB[2][1], qfma(B[3], PB[1][1], qfma(B[1], PB[0][1], Hu[1]))));
    // S~ = B'PA = (PB)'A with the structure of A
    double St[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        St[i][0] = PB[0][i];
        St[i][1] = PB[1][i];
        St[i][2] = qfma(PB[1][i], a[2], qfma(PB[0][i], a[0], PB[2][i]));
        St[i][3] = qfma(PB[3][i], a[5], qfma(PB[2][i], a[4], qfma(PB[1][i], a[3], PB[0][i] * a[1])));
    }
    double rt[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
        rt[i] = qfma(B[6 + i], pp[3], qfma(B[4 + i], pp[2], qfma(B[2 + i], pp[1], qfma(B[i], pp[0], gu[i]))));
    // Q~ = Hx + A'PA  (upper triangle), q~ = gx + A'pp
    double Qt[10];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const double c0 = PA[0][j], c1 = PA[1][j], c2 = PA[2][j], c3 = PA[3][j];
        if (j >= 0) Qt[sidx(0, j)] = c0;
        if (j >= 1) Qt[sidx(1, j)] = c1;
        if (j >= 2) Qt[sidx(2, j)] = qfma(a[2], c1, qfma(a[0], c0, j == 2 ? Hx[2] + c2 : c2));
        if (j >= 3) Qt[sidx(3, j)] = qfma(a[5], c3, qfma(a[4], c2, qfma(a[3], c1, qfma(a[1], c0, Hx[3]))));
    }
    Qt[0] += Hx[0]; Qt[4] += Hx[1];
    double qt[4];
    qt[0] = gx[0] + pp[0];
    qt[1] = gx[1] + pp[1];
    qt[2] = qfma(a[2], pp[1], qfma(a[0], pp[0], gx[2] + pp[2]));
    qt[3] = qfma(a[5], pp[3], qfma(a[4], pp[2], qfma(a[3], pp[1], qfma(a[1], pp[0], gx[3]))));
    // Rn = -R~^-1 (kept negated: the sign folds into the multiplies)
    const double idet = rcp(qfma(R00, R11, -(R01 * R01)));
    Rn[0] = (-R11) * idet; Rn[1] = R01 * idet; Rn[2] = (-R00) * idet;
    // K = -R~^-1 S~ ; kk = -R~^-1 r~
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        K[j] = qfma(Rn[1], St[1][j], Rn[0] * St[0][j]);
        K[4 + j] = qfma(Rn[2], St[1][j], Rn[1] * St[0][j]);
    }
    kk[0] = qfma(Rn[1], rt[1], Rn[0] * rt[0]);
    kk[1] = qfma(Rn[2], rt[1], Rn[1] * rt[0]);
    // P = Q~ + S~'K ; p = q~ + K'r~ (not at stage 0: nothing reads P_0, p_0; upd is uniform)
    if (!upd) return;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) P[sidx(i, j)] = qfma(St[1][i], K[4 + j], qfma(St[0][i], K[j], Qt[sidx(i, j)]));
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = qfma(K[4 + i], rt[1], qfma(K[i], rt[0], qt[i]));
}


struct In { double a[6], B[8], bb[4], Hx[4], Hu[2], gx[4], gu[2]; };

__device__ __forceinline__ void load_in(const double* p, In& s) {
    double* d = &s.a[0];
#pragma unroll
    for (int q = 0; q < 30; ++q) d[q] = p[q];
}
// stand-in for the stage-parallel phases: X FMAs in 4 independent chains, folded into gx[0] at 1e-300
__device__ __forceinline__ void parallel_work(In& s, int X) {
    double c0 = s.a[0], c1 = s.a[1], c2 = s.a[2], c3 = s.a[3];
    const double m = 0.999999, b = s.B[0];
    for (int q = 0; q < X; q += 4) {
        c0 = qfma(c0, m, b); c1 = qfma(c1, m, b); c2 = qfma(c2, m, b); c3 = qfma(c3, m, b);
    }
    s.gx[0] = qfma(1e-300, (c0 + c1) + (c2 + c3), s.gx[0]);
}
__device__ __forceinline__ void store_out(double* o, const double K[8], const double Rn[3], const double kk[2]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = K[q];
#pragma unroll
    for (int q = 0; q < 3; ++q) o[8 + q] = Rn[q];
    o[11] = kk[0]; o[12] = kk[1];
}

__global__ void __launch_bounds__(64) dpp_kernel(const double* in, double* out, int nI, int X, int reps) {
    extern __shared__ double lds[];
    const int lane = threadIdx.x, grp = lane / L, lig = lane - grp * L;
    const int inst = blockIdx.x * G + grp;
    const bool real = grp < G && inst < nI;
    In s;
    load_in(in + ((size_t)(real ? inst : 0) * L + lig) * 30, s);
    double K[8] = {}, Rn[3] = {}, kk[2] = {};
    lds[lane] = 0.0;
    for (int r = 0; r < reps; ++r) {
        parallel_work(s, X);
        double P[10], pv[4];
#pragma unroll
        for (int q = 0; q < 10; ++q) P[q] = 0.0;
        P[0] = s.Hx[0]; P[4] = s.Hx[1]; P[7] = s.Hx[2]; P[9] = s.Hx[3];   // terminal (lane N's Hx, gx)
#pragma unroll
        for (int q = 0; q < 4; ++q) pv[q] = s.gx[q];
        for (int j = L - 1; j >= 0; --j) {
            if (lig <= j) {
                double Pc[10], pvc[4];
#pragma unroll
                for (int q = 0; q < 10; ++q) Pc[q] = P[q];
#pragma unroll
                for (int q = 0; q < 4; ++q) pvc[q] = pv[q];
                if (j < L - 1)
                    ric_factor_step(s.a, s.B, s.bb, s.Hx, s.Hu, s.gx, s.gu, Pc, pvc, K, Rn, kk, j > 0);
                if (j > 0) {
#pragma unroll
                    for (int q = 0; q < 10; ++q) P[q] = from_next(P[q], Pc[q]);
#pragma unroll
                    for (int q = 0; q < 4; ++q) pv[q] = from_next(pv[q], pvc[q]);
                }
            }
        }
        s.gu[0] = qfma(1e-300, kk[0], s.gu[0]);   // keep the iterations dependent
    }
    if (real && lig < N) store_out(out + ((size_t)inst * N + lig) * NOUT, K, Rn, kk);
}

__global__ void __launch_bounds__(64 * WAVES) coop_kernel(const double* in, double* out, int nI, int X, int reps) {
    extern __shared__ double lds[];
    double* rin = lds + WAVES * LDS_WAVE / 8;        // [2][WI][NIN]
    double* rout = rin + 2 * WI * NIN;               // [2][WI][NOUT]
    double* rterm = rout + 2 * WI * NOUT;            // [WI][14]: terminal P diag (Hx) and p (gx)
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, grp = lane / L, lig = lane - grp * L;
    const int wi = wv * G + grp;                     // instance within the workgroup
    const int inst = blockIdx.x * WI + wi;
    const bool real = grp < G && inst < nI;
    In s;
    load_in(in + ((size_t)(real ? inst : 0) * L + lig) * 30, s);
    double K[8] = {}, Rn[3] = {}, kk[2] = {};
    lds[threadIdx.x] = 0.0;
    for (int r = 0; r < reps; ++r) {
        parallel_work(s, X);
        const bool walker = wv == (r & (WAVES - 1));
        const int wl = lane;                          // walker lane = instance within the workgroup
        // prologue: terminal data and stage N-1's inputs
        if (grp < G && lig == N) {
#pragma unroll
            for (int q = 0; q < 4; ++q) { rterm[wi * 14 + q] = s.Hx[q]; rterm[wi * 14 + 4 + q] = s.gx[q]; }
        }
        if (grp < G && lig == N - 1) {
            const double* d = &s.a[0];
#pragma unroll
            for (int q = 0; q < NIN; ++q) rin[(((N - 1) & 1) * WI + wi) * NIN + q] = d[q];
        }
        __syncthreads();
        double P[10], pv[4];
        if (walker && wl < WI) {
#pragma unroll
            for (int q = 0; q < 10; ++q) P[q] = 0.0;
            P[0] = rterm[wl * 14 + 0]; P[4] = rterm[wl * 14 + 1]; P[7] = rterm[wl * 14 + 2]; P[9] = rterm[wl * 14 + 3];
#pragma unroll
            for (int q = 0; q < 4; ++q) pv[q] = rterm[wl * 14 + 4 + q];
        }
        for (int k = N - 1; k >= 0; --k) {
            if (k >= 1 && grp < G && lig == k - 1) {
                const double* d = &s.a[0];
#pragma unroll
                for (int q = 0; q < NIN; ++q) rin[(((k - 1) & 1) * WI + wi) * NIN + q] = d[q];
            }
            if (walker && wl < WI) {
                In t;
                const double* src = rin + ((k & 1) * WI + wl) * NIN;
                double* d = &t.a[0];
#pragma unroll
                for (int q = 0; q < NIN; ++q) d[q] = src[q];
                double Kw[8], Rw[3], kw[2];
                ric_factor_step(t.a, t.B, t.bb, t.Hx, t.Hu, t.gx, t.gu, P, pv, Kw, Rw, kw, k > 0);
                store_out(rout + ((k & 1) * WI + wl) * NOUT, Kw, Rw, kw);
            }
            __syncthreads();
            if (grp < G && lig == k) {
                const double* o = rout + ((k & 1) * WI + wi) * NOUT;
#pragma unroll
                for (int q = 0; q < 8; ++q) K[q] = o[q];
#pragma unroll
                for (int q = 0; q < 3; ++q) Rn[q] = o[8 + q];
                kk[0] = o[11]; kk[1] = o[12];
            }
        }
        s.gu[0] = qfma(1e-300, kk[0], s.gu[0]);
    }
    if (real && lig < N) store_out(out + ((size_t)inst * N + lig) * NOUT, K, Rn, kk);
}

int main(int argc, char** argv) {
    const int X = argc > 1 ? atoi(argv[1]) : 3000;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int nI = argc > 3 ? atoi(argv[3]) : 65520;
    std::vector<double> h((size_t)nI * L * 30);
    srand(7);
    auto U = [](double lo, double hi) { return lo + (hi - lo) * (rand() / (double)RAND_MAX); };
    for (int i = 0; i < nI; ++i)
        for (int k = 0; k < L; ++k) {
            double* d = &h[((size_t)i * L + k) * 30];
            for (int q = 0; q < 6; ++q) d[q] = U(-0.05, 0.05);
            d[5] = U(0.9, 1.0);
            for (int q = 6; q < 14; ++q) d[q] = U(-0.05, 0.05);
            for (int q = 14; q < 18; ++q) d[q] = U(-0.01, 0.01);
            for (int q = 18; q < 22; ++q) d[q] = U(0.5, 2.0);
            for (int q = 22; q < 24; ++q) d[q] = U(0.1, 1.0);
            for (int q = 24; q < 30; ++q) d[q] = U(-1.0, 1.0);
        }
    double *din, *dA, *dB;
    const size_t nout = (size_t)nI * N * NOUT;
    CK(hipMalloc(&din, h.size() * 8));
    CK(hipMalloc(&dA, nout * 8));
    CK(hipMalloc(&dB, nout * 8));
    CK(hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemset(dA, 0, nout * 8));
    CK(hipMemset(dB, 0, nout * 8));
    const int ldsA = LDS_WAVE, ldsB = WAVES * LDS_WAVE + (2 * WI * NIN + 2 * WI * NOUT + WI * 14) * 8;
    CK(hipFuncSetAttribute((const void*)dpp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, ldsA));
    CK(hipFuncSetAttribute((const void*)coop_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, ldsB));
    const int gA = (nI + G - 1) / G, gB = (nI + WI - 1) / WI;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tA = 1e30f, tB = 1e30f;
    for (int t = 0; t < 4; ++t) {
        float ms;
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(dpp_kernel, dim3(gA), dim3(64), ldsA, 0, din, dA, nI, X, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (t) tA = fminf(tA, ms);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(coop_kernel, dim3(gB), dim3(64 * WAVES), ldsB, 0, din, dB, nI, X, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (t) tB = fminf(tB, ms);
    }
    CK(hipGetLastError());
    std::vector<double> a(nout), b(nout);
    CK(hipMemcpy(a.data(), dA, nout * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), dB, nout * 8, hipMemcpyDeviceToHost));
    size_t diff = 0, nz = 0;
    for (size_t q = 0; q < nout; ++q) { diff += a[q] != b[q]; nz += a[q] != 0.0; }
    printf("N=%d instances=%d X=%d reps=%d lds/wave=%d B: dpp %.3f ms, coop (%d waves) %.3f ms (coop/dpp %.2f); "
           "factors differing %zu of %zu (nonzero %zu)\n",
           N, nI, X, reps, LDS_WAVE, tA, WAVES, tB, tB / tA, diff, nout, nz);
    return 0;
}
