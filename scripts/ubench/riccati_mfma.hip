// Microbenchmark (developer tool): the Riccati factorisation walk on the FP64 matrix cores with
// the value function kept in MFMA operand layout, against the production lane walk.
//
// Walk (production, qsp_solver.hip riccati_solve<1, true>): one instance = N+1 consecutive lanes
//   (lane k: stage k), the value function (P, p) handed lane to lane by DPP; at each of the N
//   steps one lane per instance does useful work (three instances per wave at N = 20).
// Block: one instance = the 16 lanes of one block of v_mfma_f64_4x4x4_4b_f64 (four independent
//   4x4x4 products per instruction: lane l <-> block (l >> 2) & 3, element (l >> 4, l & 3); the A
//   operand is read transposed, so X passed as A gives X' B + C).  Four instances per wave; every
//   stage's matrices are held one element per lane, the whole horizon in registers, and a step is
//   nine dependent-in-part 4x4x4 products:
//     T1 = P A,  T2 = P [B | b | 0] + [0 | 0 | p | 0]   (column 2: pp = p + P b)
//     Q  = A' T1 + Hx,  Y = [B | b | 0]' T1  (rows 0, 1: S = B' P A),
//     Z  = [B | b | 0]' T2 + [Hu | gu]       (R = B' P B + Hu, column 2: r = gu + B' pp)
//     q  = A' pp + gx,  K = -R^-1 S,  P+ = Q + S' K,  p+ = q + K' r
//   with R^-1 formed on the VALU from the 2x2 gathered within the instance (one ds_bpermute row
//   swap and quad broadcasts).
// Both produce P_k, p_k for every stage; the check compares them (and both against a long-double
// reference on the first 64 instances; RM_DEBUG=1 prints instance 0 per stage).
// Measured on one MI355X (profiles/r02/riccati_mfma.txt): N = 20, 65 536 instances, the block
// walk 0.080 ms against 0.234 ms for the lane walk per factorisation of the batch (0.34x), at
// 256 VGPRs + 207 AGPRs (one wave per SIMD: the whole horizon's operands are held one element per
// lane); N = 10 0.42x.  Every lane must form -R^-1 from the same R01: taking R01 and R10 from
// their own rows gave each lane a slightly different determinant, and on ill-conditioned R the
// factors drifted 1e-8 relative from the long-double reference (8.9e-11 with one R01, as the
// lane walk's 9.5e-11).  Variants: -DRM_BPERMUTE=1 (row swap by ds_bpermute: 0.085 ms),
// -DRM_ADJ=1 (K from adj R, the reciprocal off the product chain: 0.084 ms).
// Hybrid (N = 20): the block walk inside the QP kernel's layout and occupancy (three instances per
// wave, two waves per SIMD, 19.5 KB of LDS per wave) with its inputs resident in LDS: 0.133 ms,
// 0.56x the lane walk here (RM_PREFETCH=1, the next step's operands read one step ahead: 0.143 ms);
// the production walk (10-entry P, 209 VALU per step) is itself ~0.7x this lane walk, so the
// hybrid's best case is ~1.2x on the factorisation.
// Usage: riccati_mfma [instances] [reps]   (N = 20 and N = 10 are compiled in)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef RM_BPERMUTE
#define RM_BPERMUTE 0
#endif
#ifndef RM_ADJ
#define RM_ADJ 0
#endif
#ifndef RM_PREFETCH
#define RM_PREFETCH 0
#endif

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct StageIn {   // as riccati_scan.hip
    double a[6], B[8], c[4], hx[4], hu[2], gx[4], gu[2];
};
constexpr int NIN = 30;

__device__ __forceinline__ double from_next(double old, double v) {   // lane i <- lane i+1 (DPP wave shift)
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ double quad(double v) {   // DPP quad_perm broadcast inside each group of 4 lanes
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double mfma(double a, double b, double c) {
    return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ double rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// ------------------------------------------------------------------ walk (production form)
__device__ __forceinline__ void walk_step(const StageIn& s, double P[16], double p[4]) {
    double PA[4][4], PB[4][2], pp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        PA[i][0] = P[4 * i];
        PA[i][1] = P[4 * i + 1];
        PA[i][2] = P[4 * i + 2] + P[4 * i] * s.a[0] + P[4 * i + 1] * s.a[2];
        PA[i][3] = P[4 * i] * s.a[1] + P[4 * i + 1] * s.a[3] + P[4 * i + 2] * s.a[4] + P[4 * i + 3] * s.a[5];
#pragma unroll
        for (int j = 0; j < 2; ++j)
            PB[i][j] = P[4 * i] * s.B[j] + P[4 * i + 1] * s.B[2 + j] + P[4 * i + 2] * s.B[4 + j] + P[4 * i + 3] * s.B[6 + j];
        pp[i] = p[i] + P[4 * i] * s.c[0] + P[4 * i + 1] * s.c[1] + P[4 * i + 2] * s.c[2] + P[4 * i + 3] * s.c[3];
    }
    const double R00 = s.hu[0] + s.B[0] * PB[0][0] + s.B[2] * PB[1][0] + s.B[4] * PB[2][0] + s.B[6] * PB[3][0];
    const double R01 = s.B[0] * PB[0][1] + s.B[2] * PB[1][1] + s.B[4] * PB[2][1] + s.B[6] * PB[3][1];
    const double R11 = s.hu[1] + s.B[1] * PB[0][1] + s.B[3] * PB[1][1] + s.B[5] * PB[2][1] + s.B[7] * PB[3][1];
    double St[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        St[i][0] = PB[0][i];
        St[i][1] = PB[1][i];
        St[i][2] = PB[2][i] + PB[0][i] * s.a[0] + PB[1][i] * s.a[2];
        St[i][3] = PB[0][i] * s.a[1] + PB[1][i] * s.a[3] + PB[2][i] * s.a[4] + PB[3][i] * s.a[5];
    }
    double rt[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) rt[i] = s.gu[i] + s.B[i] * pp[0] + s.B[2 + i] * pp[1] + s.B[4 + i] * pp[2] + s.B[6 + i] * pp[3];
    double Qt[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        Qt[0][j] = PA[0][j];
        Qt[1][j] = PA[1][j];
        Qt[2][j] = PA[2][j] + s.a[0] * PA[0][j] + s.a[2] * PA[1][j];
        Qt[3][j] = s.a[1] * PA[0][j] + s.a[3] * PA[1][j] + s.a[4] * PA[2][j] + s.a[5] * PA[3][j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) Qt[i][i] += s.hx[i];
    double qt[4];
    qt[0] = s.gx[0] + pp[0];
    qt[1] = s.gx[1] + pp[1];
    qt[2] = s.gx[2] + pp[2] + s.a[0] * pp[0] + s.a[2] * pp[1];
    qt[3] = s.gx[3] + s.a[1] * pp[0] + s.a[3] * pp[1] + s.a[4] * pp[2] + s.a[5] * pp[3];
    const double id = 1.0 / (R00 * R11 - R01 * R01);
    const double Rn0 = -R11 * id, Rn1 = R01 * id, Rn2 = -R00 * id;
    double K[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        K[0][j] = Rn0 * St[0][j] + Rn1 * St[1][j];
        K[1][j] = Rn1 * St[0][j] + Rn2 * St[1][j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) P[4 * i + j] = Qt[i][j] + St[0][i] * K[0][j] + St[1][i] * K[1][j];
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = qt[i] + K[0][i] * rt[0] + K[1][i] * rt[1];
}

__global__ void __launch_bounds__(64) walk_kernel(const double* in, double* out, int N, int nI, int reps) {
    const int lane = threadIdx.x & 63, L = N + 1, G = 64 / L;
    const int grp = lane / L, lig = lane - grp * L;
    const int inst = blockIdx.x * G + grp;
    const bool real = grp < G && inst < nI;
    StageIn s;
    const double* src = in + ((size_t)(real ? inst : 0) * L + lig) * NIN;
    double* d = &s.a[0];
#pragma unroll
    for (int q = 0; q < NIN; ++q) d[q] = src[q];
    double P[16], p[4];
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int q = 0; q < 16; ++q) P[q] = (q % 5 == 0) ? s.hx[q / 5] : 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = s.gx[q];
        for (int j = L - 1; j >= 0; --j) {
            if (lig <= j) {
                double Pc[16], pc[4];
#pragma unroll
                for (int q = 0; q < 16; ++q) Pc[q] = P[q];
#pragma unroll
                for (int q = 0; q < 4; ++q) pc[q] = p[q];
                if (j < L - 1) walk_step(s, Pc, pc);
#pragma unroll
                for (int q = 0; q < 16; ++q) P[q] = from_next(P[q], Pc[q]);
#pragma unroll
                for (int q = 0; q < 4; ++q) p[q] = from_next(p[q], pc[q]);
            }
        }
        s.gx[0] += 1e-300 * P[0];
    }
    if (real) {
        double* o = out + ((size_t)inst * L + lig) * 20;   // lane k < N: P_{k+1}
        for (int q = 0; q < 16; ++q) o[q] = P[q];
        for (int q = 0; q < 4; ++q) o[16 + q] = p[q];
    }
}

// ------------------------------------------------------------------ block (matrix cores)
template <int N>
__global__ void __launch_bounds__(64) block_kernel(const double* in, double* out, double* kout, int nI, int reps) {
    const int l = threadIdx.x & 63;
    const int blk = (l >> 2) & 3, r = l >> 4, c = l & 3;
    const int inst = blockIdx.x * 4 + blk;
    const bool real = inst < nI;
    const size_t ib = (size_t)(real ? inst : 0) * (N + 1);
    // the horizon, one element per lane: A, G2 = [B | b | 0], C operands of Q (Hx diagonal),
    // of Z (Hu diagonal, gu in column 2) and of q (gx, replicated over columns)
    double Am[N], G2[N], CHx[N], CZ[N], Cgx[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const double* s = in + (ib + k) * NIN;
        const double* a = s;
        const double Af[16] = {1.0, 0.0, a[0], a[1], 0.0, 1.0, a[2], a[3], 0.0, 0.0, 1.0, a[4], 0.0, 0.0, 0.0, a[5]};
        Am[k] = Af[4 * r + c];
        G2[k] = c < 2 ? s[6 + 2 * r + c] : (c == 2 ? s[14 + r] : 0.0);
        CHx[k] = r == c ? s[18 + r] : 0.0;
        CZ[k] = r < 2 ? (r == c ? s[22 + r] : (c == 2 ? s[28 + r] : 0.0)) : 0.0;
        Cgx[k] = s[24 + r];
    }
    const double* sN = in + (ib + N) * NIN;
    double hxN = r == c ? sN[18 + r] : 0.0, gxN = sN[24 + r];
    double Kst[N];
    double P = 0.0, p = 0.0;
    for (int rep = 0; rep < reps; ++rep) {
        P = hxN;
        p = gxN;
        const bool last = rep == reps - 1;
#pragma unroll
        for (int k = N - 1; k >= 0; --k) {
            if (last && real) {
                double* o = out + ((ib + k + 1) * 20);
                o[4 * r + c] = P;
                if (c == 0) o[16 + r] = p;
            }
            const double T1 = mfma(P, Am[k], 0.0);
            const double T2 = mfma(P, G2[k], c == 2 ? p : 0.0);
            const double pp = quad<0xAA>(T2);                 // (p + P b)[r] on every lane of the row
            const double Q = mfma(Am[k], T1, CHx[k]);
            const double Y = mfma(G2[k], T1, 0.0);
            const double Z = mfma(G2[k], T2, CZ[k]);
            const double q = mfma(Am[k], pp, Cgx[k]);
            // the 2x2 R and r = Z[0..1][0..2] on every lane of the instance: v_permlane16_swap puts
            // row 0 of Z (Z[0][*]) into rows 0 and 1 of one result and row 1 into the other (rows
            // 2, 3 get rows 2, 3, unused), then quad broadcasts pick the columns
#if RM_BPERMUTE
            const double Zx = __shfl_xor(Z, 16);
            const bool odd = r & 1;
            const double w0 = odd ? Zx : Z, w1 = odd ? Z : Zx;
#else
            const auto slo = __builtin_amdgcn_permlane16_swap(__double2loint(Z), __double2loint(Z), false, false);
            const auto shi = __builtin_amdgcn_permlane16_swap(__double2hiint(Z), __double2hiint(Z), false, false);
            const double w0 = __hiloint2double(shi[0], slo[0]), w1 = __hiloint2double(shi[1], slo[1]);
#endif
            const double R00 = quad<0x00>(w0), R01 = quad<0x55>(w0), r0 = quad<0xAA>(w0);
            const double R11 = quad<0x55>(w1), r1 = quad<0xAA>(w1);
            const bool in2 = r < 2 && c < 2;
#if RM_ADJ
            // K = -R^-1 S = -(adj R) S / det: the product with adj R does not wait for the reciprocal
            const double idet = rcp(R00 * R11 - R01 * R01);
            const double Xadj = in2 ? (r == c ? (r == 0 ? R11 : R00) : -R01) : 0.0;
            const double Kf = -idet * mfma(Xadj, Y, 0.0);       // rows 0, 1: K
#else
            const double idet = rcp(R00 * R11 - R01 * R01);
            const double n00 = -R11 * idet, n01 = R01 * idet, n11 = -R00 * idet;   // -R^-1
            const double Xop = in2 ? (r == c ? (r == 0 ? n00 : n11) : n01) : 0.0;
            const double Kf = mfma(Xop, Y, 0.0);              // rows 0, 1: K = -R^-1 S
#endif
            P = mfma(Y, Kf, Q);                                // Q + S' K
            const double RT = r == 0 ? r0 : (r == 1 ? r1 : 0.0);
            p = mfma(Kf, RT, q);                               // q + K' r
            Kst[k] = Kf;
        }
        Cgx[0] += 1e-300 * P;   // keep the repetitions dependent
    }
    if (real) {
        double* o = out + (ib * 20);
        o[4 * r + c] = P;
        if (c == 0) o[16 + r] = p;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) acc += Kst[k];
        kout[inst * 64 + l] = acc;
    }
}

// ------------------------------------------------------------------ hybrid (stage lanes + block walk)
// The QP kernel's lane layout (one instance = N+1 lanes, three per wave at N = 20) with the walk
// inputs resident in LDS (one SoA column per lane, as the stage lanes would keep them), the
// block-MFMA walk reading its operand elements straight from the stage lanes' columns (no
// per-step publish) and handing K, -R^-1, kk back through a two-slot ring.  LDS per one-wave
// workgroup: 27 columns + ring + filler up to the QP kernel's 19.5 KB, so that 8 workgroups fit
// a CU (two waves per SIMD) as in the kernel.
constexpr int HF = 27;   // a 6, B 8, b 4, gx 4, hx 4 (hx[3] varies), hu 2 -> 28 slots, gu 2 in the tail
constexpr int H_A = 0, H_B = 6, H_BB = 14, H_GX = 18, H_HX = 22, H_HU = 26, H_GU = 28, H_COLS = 30;
constexpr int HRING_OUT = 16, HG = 3;
constexpr int HYB_LDS_BYTES = 19968;   // H_COLS x 64 x 8 = 15 360 + ring 768 + filler

template <int N>
__global__ void __launch_bounds__(64) hybrid_kernel(const double* in, double* out, int nI, int reps) {
    extern __shared__ double sm[];
    constexpr int L = N + 1, G = 64 / L;
    static_assert(G <= HG, "at most three instances per wave");
    const int lane = threadIdx.x & 63, grp = lane / L, lig = lane - grp * L;
    const bool stage_lane = grp < G;
    const int inst = blockIdx.x * G + (stage_lane ? grp : 0);
    const bool real = stage_lane && inst < nI;
    {
        const double* s = in + ((size_t)(real ? inst : 0) * L + lig) * NIN;
        // columns: a, B, b, gx, hx, hu, gu
        for (int q = 0; q < 6; ++q) sm[(H_A + q) * 64 + lane] = s[q];
        for (int q = 0; q < 8; ++q) sm[(H_B + q) * 64 + lane] = s[6 + q];
        for (int q = 0; q < 4; ++q) sm[(H_BB + q) * 64 + lane] = s[14 + q];
        for (int q = 0; q < 4; ++q) sm[(H_GX + q) * 64 + lane] = s[24 + q];
        for (int q = 0; q < 4; ++q) sm[(H_HX + q) * 64 + lane] = s[18 + q];
        for (int q = 0; q < 2; ++q) sm[(H_HU + q) * 64 + lane] = s[22 + q];
        for (int q = 0; q < 2; ++q) sm[(H_GU + q) * 64 + lane] = s[28 + q];
    }
    double* rout = sm + H_COLS * 64;   // [parity][instance][HRING_OUT]
    double K[8] = {0}, Rn[3] = {0}, kk[2] = {0};
    int l2 = lane;
    asm volatile("" : "+v"(l2));
    const int blk = (l2 >> 2) & 3, r = l2 >> 4, cc = l2 & 3;
    const int bg = blk < G ? blk : G - 1;
    const bool bout = blk < G;
    int ao = -1;
    if (cc >= 2 && r < 2) ao = H_A + 2 * r + (cc - 2);
    else if (cc == 3 && r >= 2) ao = H_A + 2 + r;
    const double aconst = r == cc ? 1.0 : 0.0;
    const int go = cc < 2 ? H_B + 2 * r + cc : (cc == 2 ? H_BB + r : -1);
    const int ho = r == cc ? H_HX + r : -1;
    const int zo = r < 2 ? (r == cc ? H_HU + r : (cc == 2 ? H_GU + r : -1)) : -1;
    const int ao_ = ao < 0 ? 0 : ao, go_ = go < 0 ? 0 : go, ho_ = ho < 0 ? 0 : ho, zo_ = zo < 0 ? 0 : zo;
    double Pout = 0.0, pout = 0.0;
    for (int rep = 0; rep < reps; ++rep) {
        const int colN = bg * L + N;
        double P = r == cc ? sm[(H_HX + r) * 64 + colN] : 0.0;
        double pv = sm[(H_GX + r) * 64 + colN];
#if RM_PREFETCH
        // operand elements of the next step read one step ahead: the LDS latency overlaps the chain
        int col = bg * L + N - 1;
        double na = sm[ao_ * 64 + col], ng = sm[go_ * 64 + col], nh = sm[ho_ * 64 + col];
        double nz = sm[zo_ * 64 + col], nq = sm[(H_GX + r) * 64 + col];
#endif
        for (int j = N - 1; j >= 0; --j) {
#if RM_PREFETCH
            const double va = na, vg = ng, vh = nh, vz = nz, vq = nq;
            col = bg * L + (j > 0 ? j - 1 : 0);
            na = sm[ao_ * 64 + col]; ng = sm[go_ * 64 + col]; nh = sm[ho_ * 64 + col];
            nz = sm[zo_ * 64 + col]; nq = sm[(H_GX + r) * 64 + col];
#else
            const int col = bg * L + j;
            const double va = sm[ao_ * 64 + col], vg = sm[go_ * 64 + col], vh = sm[ho_ * 64 + col];
            const double vz = sm[zo_ * 64 + col], vq = sm[(H_GX + r) * 64 + col];
#endif
            const double Am = ao >= 0 ? va : aconst;
            const double G2 = go >= 0 ? vg : 0.0;
            const double CH = ho >= 0 ? vh : 0.0;
            const double CZ = zo >= 0 ? vz : 0.0;
            const double T1 = mfma(P, Am, 0.0);
            const double T2 = mfma(P, G2, cc == 2 ? pv : 0.0);
            const double pp = quad<0xAA>(T2);
            const double Q = mfma(Am, T1, CH);
            const double Y = mfma(G2, T1, 0.0);
            const double Z = mfma(G2, T2, CZ);
            const double q = mfma(Am, pp, vq);
            const auto slo = __builtin_amdgcn_permlane16_swap(__double2loint(Z), __double2loint(Z), false, false);
            const auto shi = __builtin_amdgcn_permlane16_swap(__double2hiint(Z), __double2hiint(Z), false, false);
            const double w0 = __hiloint2double(shi[0], slo[0]), w1 = __hiloint2double(shi[1], slo[1]);
            const double R00 = quad<0x00>(w0), R01 = quad<0x55>(w0), rt0 = quad<0xAA>(w0);
            const double R11 = quad<0x55>(w1), rt1 = quad<0xAA>(w1);
            const double idet = rcp(R00 * R11 - R01 * R01);
            const double n0 = -R11 * idet, n1 = R01 * idet, n2 = -R00 * idet;
            const double Xn = (r < 2 && cc < 2) ? (r != cc ? n1 : (r == 0 ? n0 : n2)) : 0.0;
            const double Kf = mfma(Xn, Y, 0.0);
            P = mfma(Y, Kf, Q);
            pv = mfma(Kf, r == 0 ? rt0 : (r == 1 ? rt1 : 0.0), q);
            double* o = rout + ((j & 1) * HG + bg) * HRING_OUT;
            if (bout && r < 2) o[4 * r + cc] = Kf;
            if (bout && r == 0 && cc == 0) {
                o[8] = n0; o[9] = n1; o[10] = n2;
                o[11] = n0 * rt0 + n1 * rt1;
                o[12] = n1 * rt0 + n2 * rt1;
            }
            if (stage_lane && lig == j + 1 && j + 1 < N) {
                const double* oi = rout + (((j + 1) & 1) * HG + grp) * HRING_OUT;
                for (int t = 0; t < 8; ++t) K[t] = oi[t];
                for (int t = 0; t < 3; ++t) Rn[t] = oi[8 + t];
                kk[0] = oi[11]; kk[1] = oi[12];
            }
        }
        if (stage_lane && lig == 0) {
            const double* oi = rout + grp * HRING_OUT;
            for (int t = 0; t < 8; ++t) K[t] = oi[t];
            for (int t = 0; t < 3; ++t) Rn[t] = oi[8 + t];
            kk[0] = oi[11]; kk[1] = oi[12];
        }
        // keep the repetitions dependent (as the walk's gx[0] nudge)
        sm[(H_GX) * 64 + lane] += 1e-300 * (K[0] + kk[0] + Rn[0]);
        Pout = P;
        pout = pv;
    }
    if (bout && inst < nI) {
        const int ib = blockIdx.x * G + blk;
        if (ib < nI) {
            out[(size_t)ib * L * 20 + 4 * r + cc] = Pout;   // slot 0: P_0
            if (cc == 0) out[(size_t)ib * L * 20 + 16 + r] = pout;
        }
    }
}

template <int N>
static int run(int nI, int reps) {
    const int L = N + 1, G = 64 / L;
    std::vector<double> h((size_t)nI * L * NIN);
    srand(7);
    auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
    for (size_t i = 0; i < (size_t)nI * L; ++i) {
        double* d = &h[i * NIN];
        for (int q = 0; q < 6; ++q) d[q] = 0.05 * rnd();
        d[5] += 1.0;
        for (int q = 0; q < 8; ++q) d[6 + q] = 0.05 * rnd();
        for (int q = 0; q < 4; ++q) d[14 + q] = 1e-3 * rnd();
        const double hx[4] = {0.05, 0.05, 5e-5, 1e-3}, hu[2] = {5e-5, 5e-5};
        for (int q = 0; q < 4; ++q) d[18 + q] = hx[q] * (1.0 + 100.0 * (rnd() + 0.5));
        for (int q = 0; q < 2; ++q) d[22 + q] = hu[q] * (1.0 + 1e3 * (rnd() + 0.5));
        for (int q = 0; q < 4; ++q) d[24 + q] = 1e-2 * rnd();
        for (int q = 0; q < 2; ++q) d[28 + q] = 1e-4 * rnd();
        if (i % L == (size_t)N) {
            d[18] = d[19] = 2e5; d[20] = 20.0; d[21] = 1.0;
        }
    }
    double *din, *dw, *db, *dk;
    CK(hipMalloc(&din, h.size() * 8));
    CK(hipMalloc(&dw, (size_t)nI * L * 20 * 8));
    CK(hipMalloc(&db, (size_t)nI * L * 20 * 8));
    CK(hipMalloc(&dk, (size_t)nI * 64 * 8));
    CK(hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemset(db, 0, (size_t)nI * L * 20 * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tw = 0, tb = 0;
    for (int pass = 0; pass < 2; ++pass) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(walk_kernel, dim3((nI + G - 1) / G), dim3(64), 0, 0, din, dw, N, nI, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&tw, e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((block_kernel<N>), dim3((nI + 3) / 4), dim3(64), 0, 0, din, db, dk, nI, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&tb, e0, e1));
    }
    float th = -1.0f;
    if constexpr (64 / (N + 1) <= HG) {
        double* dh;
        CK(hipMalloc(&dh, (size_t)nI * L * 20 * 8));
        CK(hipFuncSetAttribute((const void*)hybrid_kernel<N>, hipFuncAttributeMaxDynamicSharedMemorySize, HYB_LDS_BYTES));
        for (int pass = 0; pass < 2; ++pass) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL((hybrid_kernel<N>), dim3((nI + G - 1) / G), dim3(64), HYB_LDS_BYTES, 0, din, dh, nI, reps);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&th, e0, e1));
        }
        CK(hipGetLastError());
        std::vector<double> oh((size_t)nI * L * 20);
        CK(hipMemcpy(oh.data(), dh, oh.size() * 8, hipMemcpyDeviceToHost));
        double mh = 0.0;
        for (int i = 0; i < nI; ++i) {
            // hybrid slot 0 holds P_0 (reps perturb gx[0] by 1e-300 only)
            double nrm = 0.0, diff = 0.0;
            std::vector<double> ref(20);
            CK(hipMemcpy(ref.data(), db + (size_t)i * L * 20, 20 * 8, hipMemcpyDeviceToHost));
            for (int q = 0; q < 20; ++q) { nrm = fmax(nrm, fabs(ref[q])); diff = fmax(diff, fabs(oh[(size_t)i * L * 20 + q] - ref[q])); }
            mh = fmax(mh, diff / (nrm + 1e-300));
            if (i > 256) break;
        }
        printf("  hybrid (stage lanes, LDS-resident walk inputs, %d B LDS per wave): %.3f ms per factorisation (hybrid/walk %.3f); P_0 vs block %.2e\n",
               HYB_LDS_BYTES, th / reps, th / tw, mh);
        CK(hipFree(dh));
    }
    CK(hipGetLastError());
    std::vector<double> ow((size_t)nI * L * 20), ob((size_t)nI * L * 20);
    CK(hipMemcpy(ow.data(), dw, ow.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ob.data(), db, ob.size() * 8, hipMemcpyDeviceToHost));
    double maxrel = 0.0;
    for (int i = 0; i < nI; ++i)
        for (int k = 0; k < N; ++k) {   // walk: lane k holds P_{k+1}; block: slot k+1 holds P_{k+1}
            const double* a = &ow[((size_t)i * L + k) * 20];
            const double* b = &ob[((size_t)i * L + k + 1) * 20];
            double nrm = 0.0, diff = 0.0;
            for (int q = 0; q < 20; ++q) { nrm = fmax(nrm, fabs(a[q])); diff = fmax(diff, fabs(a[q] - b[q])); }
            maxrel = fmax(maxrel, diff / (nrm + 1e-300));
        }
    // CPU reference for the first instances (plain dense Riccati in long double)
    double ew = 0.0, eb = 0.0;
    int worst_k = -1, worst_q = -1;
    for (int i = 0; i < 64 && i < nI; ++i) {
        long double P[16] = {0}, p[4];
        const double* sN = &h[((size_t)i * L + N) * NIN];
        for (int q = 0; q < 4; ++q) { P[5 * q] = sN[18 + q]; p[q] = sN[24 + q]; }
        for (int k = N - 1; k >= 0; --k) {
            const double* d = &h[((size_t)i * L + k) * NIN];
            const double* a = d;
            const long double A[16] = {1, 0, a[0], a[1], 0, 1, a[2], a[3], 0, 0, 1, a[4], 0, 0, 0, a[5]};
            long double Bm[8], bb[4];
            for (int q = 0; q < 8; ++q) Bm[q] = d[6 + q];
            for (int q = 0; q < 4; ++q) bb[q] = d[14 + q];
            long double pp[4], PA[16], PB[8];
            for (int x = 0; x < 4; ++x) {
                pp[x] = p[x];
                for (int y = 0; y < 4; ++y) pp[x] += P[4 * x + y] * bb[y];
                for (int y = 0; y < 4; ++y) { PA[4 * x + y] = 0; for (int z = 0; z < 4; ++z) PA[4 * x + y] += P[4 * x + z] * A[4 * z + y]; }
                for (int y = 0; y < 2; ++y) { PB[2 * x + y] = 0; for (int z = 0; z < 4; ++z) PB[2 * x + y] += P[4 * x + z] * Bm[2 * z + y]; }
            }
            long double R[4], S[8], rt[2], Q[16], qt[4];
            for (int x = 0; x < 2; ++x) {
                for (int y = 0; y < 2; ++y) { R[2 * x + y] = x == y ? d[22 + x] : 0; for (int z = 0; z < 4; ++z) R[2 * x + y] += Bm[2 * z + x] * PB[2 * z + y]; }
                for (int y = 0; y < 4; ++y) { S[4 * x + y] = 0; for (int z = 0; z < 4; ++z) S[4 * x + y] += Bm[2 * z + x] * PA[4 * z + y]; }
                rt[x] = d[28 + x]; for (int z = 0; z < 4; ++z) rt[x] += Bm[2 * z + x] * pp[z];
            }
            for (int x = 0; x < 4; ++x) {
                for (int y = 0; y < 4; ++y) { Q[4 * x + y] = x == y ? d[18 + x] : 0; for (int z = 0; z < 4; ++z) Q[4 * x + y] += A[4 * z + x] * PA[4 * z + y]; }
                qt[x] = d[24 + x]; for (int z = 0; z < 4; ++z) qt[x] += A[4 * z + x] * pp[z];
            }
            const long double det = R[0] * R[3] - R[1] * R[2];
            const long double Ri[4] = {R[3] / det, -R[1] / det, -R[2] / det, R[0] / det};
            long double K[8];
            for (int x = 0; x < 2; ++x) for (int y = 0; y < 4; ++y) K[4 * x + y] = -(Ri[2 * x] * S[y] + Ri[2 * x + 1] * S[4 + y]);
            for (int x = 0; x < 4; ++x) {
                for (int y = 0; y < 4; ++y) P[4 * x + y] = Q[4 * x + y] + S[x] * K[y] + S[4 + x] * K[4 + y];
                p[x] = qt[x] + K[x] * rt[0] + K[4 + x] * rt[1];
            }
            const double* w = &ow[((size_t)i * L + k - 1 + 1 - 1 + (k > 0 ? 0 : 0)) * 20];
            (void)w;
            // P_k: walk lane k-1 (k >= 1), block slot k
            double nrm = 0.0;
            for (int q = 0; q < 16; ++q) nrm = fmax(nrm, fabs((double)P[q]));
            for (int q = 0; q < 4; ++q) nrm = fmax(nrm, fabs((double)p[q]));
            const double* bo = &ob[((size_t)i * L + k) * 20];
            if (i == 0 && getenv("RM_DEBUG")) {
                double ebk = 0.0, ewk = 0.0; int qb = -1;
                for (int q = 0; q < 20; ++q) {
                    const double ref = q < 16 ? (double)P[q] : (double)p[q - 16];
                    const double e1 = fabs(bo[q] - ref) / nrm;
                    if (e1 > ebk) { ebk = e1; qb = q; }
                    if (k >= 1) ewk = fmax(ewk, fabs(ow[((size_t)i * L + k - 1) * 20 + q] - ref) / nrm);
                }
                printf("    k=%d nrm %.3e walk %.2e block %.2e (entry %d: block %.17g ref %.17g)\n", k, nrm, ewk, ebk, qb,
                       bo[qb], qb < 16 ? (double)P[qb] : (double)p[qb - 16]);
            }
            for (int q = 0; q < 20; ++q) {
                const double ref = q < 16 ? (double)P[q] : (double)p[q - 16];
                const double e = fabs(bo[q] - ref) / nrm;
                if (e > eb) { eb = e; worst_k = k; worst_q = q; }
                if (k >= 1) ew = fmax(ew, fabs(ow[((size_t)i * L + k - 1) * 20 + q] - ref) / nrm);
            }
        }
    }
    printf("  vs long-double reference (64 instances): walk %.2e, block %.2e (worst at k=%d entry %d)\n", ew, eb, worst_k, worst_q);
    printf("N=%d instances=%d reps=%d: walk %.3f ms, block-mfma %.3f ms (block/walk %.3f) per factorisation "
           "of the batch; max rel |P_walk - P_block| = %.2e\n", N, nI, reps, tw / reps, tb / reps, tb / tw, maxrel);
    CK(hipFree(din)); CK(hipFree(dw)); CK(hipFree(db)); CK(hipFree(dk));
    return 0;
}

int main(int argc, char** argv) {
    const int nI = argc > 1 ? atoi(argv[1]) : 65536;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    if (run<20>(nI, reps)) return 1;
    if (run<10>(nI, reps)) return 1;
    return 0;
}
