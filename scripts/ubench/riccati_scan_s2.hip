// Microbenchmark (developer tool): riccati_scan.hip's comparison at TWO stages per lane, the QP
// kernel's layout at N = 50 (configs[4]): an instance = a group of L = ceil((N+1)/2) lanes, lane j
// holding stages 2j and 2j+1 (the terminal stage N in the last lane), 64 / L instances per wave,
// one-wave workgroups padded with dynamic LDS to the kernel's occupancy (one wave per SIMD).
// Walk: per lane step the lane factors its two stages (2j+1, then 2j) and hands (P, p) to lane j-1.
// Scan: every lane builds the elements of its two stages and combines them locally (e_2j (x) e_2j+1),
// a Hillis-Steele suffix scan over the lanes gives E_{2j:N}, and one more combine with the next
// lane's result gives E_{2j+1:N}: (P, p) of both slots.  Same element and combine as riccati_scan.hip.
//
// Walk: the value function (P, p) is handed from lane k+1 to lane k by a DPP shift, one stage per
//   step, L - 1 steps; at step j only lane j of each group keeps its result (the structured step of
//   ric_factor_step: A = [[1,0,a0,a1],[0,1,a2,a3],[0,0,1,a4],[0,0,0,a5]], diagonal H).
// Scan: every lane builds the conditional value-function element of its stage,
//   e_k = (A, b, C, eta, J) = (F, c - L Hu^-1 gu, L Hu^-1 L', -gx, diag Hx), e_N = (0, 0, 0, -p_N, P_N)
//   (Sarkka & Garcia-Fernandez, "Temporal parallelization of dynamic programming and linear
//   quadratic control", IEEE TAC 2023), and a Hillis-Steele suffix scan over the group combines
//     M = (I + C_ij J_jk)^-1, A_ik = A_jk M A_ij, b_ik = A_jk M (b_ij + C_ij eta_jk) + b_jk,
//     C_ik = A_jk M C_ij A_jk' + C_jk, eta_ik = A_ij' M' (eta_jk - J_jk b_ij) + eta_ij,
//     J_ik = A_ij' M' J_jk A_ij + J_ij
//   in ceil(log2 L) levels (partner lane k + 2^d through ds_bpermute); lane k ends with
//   e_{k:N}: P_k = J, p_k = -eta.  Both produce P_k, p_k for every lane; the check compares them.
// Usage: riccati_scan [N] [instances] [reps]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct StageIn {   // SoA over (instance, stage) would be the kernel's; AoS per lane here (read once)
    double a[6], B[8], c[4], hx[4], hu[2], gx[4], gu[2];
};
constexpr int NIN = 30;

__device__ __forceinline__ double shfl_d(double v, int src) {
    const int lo = __shfl(__double2loint(v), src), hi = __shfl(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double from_next(double old, double v) {   // lane i <- lane i+1 (DPP wave shift)
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void load_stage(const double* in, StageIn& s) {
    double* d = &s.a[0];
#pragma unroll
    for (int q = 0; q < NIN; ++q) d[q] = in[q];
}

// ------------------------------------------------------------------ walk
// the production structured factor step (qsp_solver.hip ric_factor_step), value function only
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

// ------------------------------------------------------------------ scan
struct Elem {
    double A[16], b[4], C[10], eta[4], J[10];   // C, J symmetric (upper triangle, row-major)
};
__device__ __forceinline__ int si(int i, int j) {
    if (i > j) { int t = i; i = j; j = t; }
    return i == 0 ? j : (i == 1 ? 3 + j : (i == 2 ? 5 + j : 9));
}

// e_ij (*this lane) combined with e_jk (partner): result in e
__device__ __forceinline__ void combine(Elem& e, const Elem& f) {
    // M = (I + C_ij J_jk)^-1 by Gauss-Jordan without pivoting (I + C J has eigenvalues >= 1 for
    // C, J symmetric positive semidefinite)
    double T[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double v = (i == j) ? 1.0 : 0.0;
#pragma unroll
            for (int m = 0; m < 4; ++m) v += e.C[si(i, m)] * f.J[si(m, j)];
            T[i][j] = v;
            T[i][4 + j] = (i == j) ? 1.0 : 0.0;
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const double piv = 1.0 / T[c][c];
#pragma unroll
        for (int j = 0; j < 8; ++j) T[c][j] *= piv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            const double fct = T[r][c];
#pragma unroll
            for (int j = 0; j < 8; ++j) T[r][j] -= fct * T[c][j];
        }
    }
    // TA = A_jk M
    double TA[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double v = 0.0;
#pragma unroll
            for (int m = 0; m < 4; ++m) v += f.A[4 * i + m] * T[m][4 + j];
            TA[i][j] = v;
        }
    // U = A_ij' M'  (= A_ij' (I + J_jk C_ij)^-1)
    double U[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double v = 0.0;
#pragma unroll
            for (int m = 0; m < 4; ++m) v += e.A[4 * m + i] * T[j][4 + m];
            U[i][j] = v;
        }
    Elem r;
    // b: A_jk M (b_ij + C_ij eta_jk) + b_jk ; eta: U (eta_jk - J_jk b_ij) + eta_ij
    double w[4], z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double v = e.b[i], y = f.eta[i];
#pragma unroll
        for (int m = 0; m < 4; ++m) { v += e.C[si(i, m)] * f.eta[m]; y -= f.J[si(i, m)] * e.b[m]; }
        w[i] = v;
        z[i] = y;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double v = f.b[i], y = e.eta[i];
#pragma unroll
        for (int m = 0; m < 4; ++m) { v += TA[i][m] * w[m]; y += U[i][m] * z[m]; }
        r.b[i] = v;
        r.eta[i] = y;
    }
    // A = TA A_ij
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double v = 0.0;
#pragma unroll
            for (int m = 0; m < 4; ++m) v += TA[i][m] * e.A[4 * m + j];
            r.A[4 * i + j] = v;
        }
    // C = (TA C_ij) A_jk' + C_jk ; J = (U J_jk) A_ij + J_ij  (upper triangles)
    double X[4][4], Y[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double v = 0.0, y = 0.0;
#pragma unroll
            for (int m = 0; m < 4; ++m) { v += TA[i][m] * e.C[si(m, j)]; y += U[i][m] * f.J[si(m, j)]; }
            X[i][j] = v;
            Y[i][j] = y;
        }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) {
            double v = f.C[si(i, j)], y = e.J[si(i, j)];
#pragma unroll
            for (int m = 0; m < 4; ++m) { v += X[i][m] * f.A[4 * j + m]; y += Y[i][m] * e.A[4 * m + j]; }
            r.C[si(i, j)] = v;
            r.J[si(i, j)] = y;
        }
    e = r;
}


__device__ __forceinline__ bool stage_ok(int k, int N) { return k <= N; }

__global__ void __launch_bounds__(64) walk2_kernel(const double* in, double* out, int N, int nI, int reps) {
    extern __shared__ double pad[];
    const int lane = threadIdx.x & 63, L = (N + 2) / 2, G = 64 / L;
    const int grp = lane / L, lig = lane - grp * L;
    const int inst = blockIdx.x * G + grp;
    const bool real = grp < G && inst < nI;
    StageIn s[2];
#pragma unroll
    for (int ls = 0; ls < 2; ++ls) {
        const int k = 2 * lig + ls;
        load_stage(in + ((size_t)(real ? inst : 0) * (N + 1) + (k <= N ? k : N)) * NIN, s[ls]);
    }
    if (threadIdx.x == 1000) pad[0] = 0.0;
    double P[16], p[4];
    const int lsN = N - 2 * (L - 1);   // slot of the terminal stage in the last lane
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int q = 0; q < 16; ++q) P[q] = (q % 5 == 0) ? (lsN == 0 ? s[0].hx[q / 5] : s[1].hx[q / 5]) : 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = lsN == 0 ? s[0].gx[q] : s[1].gx[q];
        for (int j = L - 1; j >= 0; --j) {
            if (lig <= j) {
                double Pc[16], pc[4];
#pragma unroll
                for (int q = 0; q < 16; ++q) Pc[q] = P[q];
#pragma unroll
                for (int q = 0; q < 4; ++q) pc[q] = p[q];
#pragma unroll
                for (int ls = 1; ls >= 0; --ls) {
                    if (j == L - 1 && ls >= lsN) continue;
                    walk_step(s[ls], Pc, pc);
                }
#pragma unroll
                for (int q = 0; q < 16; ++q) P[q] = from_next(P[q], Pc[q]);
#pragma unroll
                for (int q = 0; q < 4; ++q) p[q] = from_next(p[q], pc[q]);
            }
        }
        s[0].gx[0] += 1e-300 * P[0];
    }
    if (real && 2 * lig + 1 < N) {
        // lane j ends holding the value function handed to it, P_{2j+2}: row 2j+1
        double* o = out + ((size_t)inst * (N + 1) + 2 * lig + 1) * 20;
        for (int q = 0; q < 16; ++q) o[q] = P[q];
        for (int q = 0; q < 4; ++q) o[16 + q] = p[q];
    }
}

__device__ __forceinline__ void make_elem(const StageIn& s, bool terminal, Elem& e) {
    if (terminal) {
#pragma unroll
        for (int q = 0; q < 16; ++q) e.A[q] = 0.0;
#pragma unroll
        for (int q = 0; q < 10; ++q) { e.C[q] = 0.0; e.J[q] = 0.0; }
#pragma unroll
        for (int q = 0; q < 4; ++q) { e.b[q] = 0.0; e.eta[q] = -s.gx[q]; e.J[si(q, q)] = s.hx[q]; }
        return;
    }
    const double F[16] = {1.0, 0.0, s.a[0], s.a[1], 0.0, 1.0, s.a[2], s.a[3], 0.0, 0.0, 1.0, s.a[4], 0.0, 0.0, 0.0, s.a[5]};
#pragma unroll
    for (int q = 0; q < 16; ++q) e.A[q] = F[q];
    const double ih0 = 1.0 / s.hu[0], ih1 = 1.0 / s.hu[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        e.b[i] = s.c[i] - s.B[2 * i] * ih0 * s.gu[0] - s.B[2 * i + 1] * ih1 * s.gu[1];
        e.eta[i] = -s.gx[i];
#pragma unroll
        for (int j = i; j < 4; ++j) {
            e.C[si(i, j)] = s.B[2 * i] * ih0 * s.B[2 * j] + s.B[2 * i + 1] * ih1 * s.B[2 * j + 1];
            e.J[si(i, j)] = (i == j) ? s.hx[i] : 0.0;
        }
    }
}

__global__ void __launch_bounds__(64) scan2_kernel(const double* in, double* out, int N, int nI, int reps) {
    extern __shared__ double pad[];
    const int lane = threadIdx.x & 63, L = (N + 2) / 2, G = 64 / L;
    const int grp = lane / L, lig = lane - grp * L;
    const int inst = blockIdx.x * G + grp;
    const bool real = grp < G && inst < nI;
    StageIn s[2];
#pragma unroll
    for (int ls = 0; ls < 2; ++ls) {
        const int k = 2 * lig + ls;
        load_stage(in + ((size_t)(real ? inst : 0) * (N + 1) + (k <= N ? k : N)) * NIN, s[ls]);
    }
    if (threadIdx.x == 1000) pad[0] = 0.0;
    const int k0 = 2 * lig, k1 = k0 + 1;
    Elem e, e1;
    for (int r = 0; r < reps; ++r) {
        make_elem(s[0], k0 == N, e);
        make_elem(s[1], k1 == N, e1);
        if (k1 <= N) combine(e, e1);   // e_{2j} (x) e_{2j+1}
        // suffix scan over the lanes of the group: lane j <- E_j (x) E_{j+off} while j + off < L
        for (int off = 1; off < L; off <<= 1) {
            const bool take = lig + off < L;
            const int src = take ? lane + off : lane;
            Elem f;
            double* fd = &f.A[0];
            const double* ed = &e.A[0];
#pragma unroll
            for (int q = 0; q < 44; ++q) fd[q] = shfl_d(ed[q], src);
            if (take) combine(e, f);
        }
        // slot 1: E_{2j+1:N} = e_{2j+1} (x) E_{2j+2:N} (the next lane's result)
        {
            Elem f;
            double* fd = &f.A[0];
            const double* ed = &e.A[0];
            const int src = lig + 1 < L ? lane + 1 : lane;
#pragma unroll
            for (int q = 0; q < 44; ++q) fd[q] = shfl_d(ed[q], src);
            if (k1 < N) combine(e1, f);
            // the factors of both slots from their successor's value function (the walk forms them in
            // its steps; here one structured step per slot, in parallel): slot 1 from P_{2j+2} (the
            // next lane's E), slot 0 from P_{2j+1} (this lane's slot-1 E)
#pragma unroll
            for (int ls = 1; ls >= 0; --ls) {
                const Elem& v = ls == 1 ? f : e1;
                double Pn[16], pn[4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) Pn[4 * i + jj] = v.J[si(i, jj)];
#pragma unroll
                for (int q = 0; q < 4; ++q) pn[q] = -v.eta[q];
                if (2 * lig + ls < N) walk_step(s[ls], Pn, pn);
                s[ls].gx[1] += 1e-300 * Pn[0];
            }
        }
        s[0].gx[0] += 1e-300 * e.J[0] + 1e-300 * e1.J[0];
    }
    if (real) {
        // P_k of both slots; the walk's output convention: row k holds P_{k+1}, so slot 0's value goes
        // to row k0 - 1 and slot 1's to row k0
        for (int ls = 0; ls < 2; ++ls) {
            const int k = 2 * lig + ls;
            if (k < 1 || k > N) continue;
            const Elem& v = ls == 0 ? e : e1;
            double* o = out + ((size_t)inst * (N + 1) + k - 1) * 20;
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) o[4 * i + j] = v.J[si(i, j)];
            for (int q = 0; q < 4; ++q) o[16 + q] = -v.eta[q];
        }
    }
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 50;
    const int nI = argc > 2 ? atoi(argv[2]) : 16384;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const int ldsKB = argc > 4 ? atoi(argv[4]) : 36;   // the QP kernel's LDS per wave at S = 2 (35.8 KB)
    const int L = (N + 2) / 2, G = 64 / L;
    if (L > 64) { printf("N + 1 must be <= 128\n"); return 1; }
    std::vector<double> h((size_t)nI * (N + 1) * NIN);
    srand(7);
    auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
    for (size_t i = 0; i < (size_t)nI * (N + 1); ++i) {
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
        if (i % (N + 1) == (size_t)N) { d[18] = d[19] = 2e5; d[20] = 20.0; d[21] = 1.0; }
    }
    double *din, *dw, *ds;
    const size_t nout = (size_t)nI * (N + 1) * 20;
    CK(hipMalloc(&din, h.size() * 8));
    CK(hipMalloc(&dw, nout * 8));
    CK(hipMalloc(&ds, nout * 8));
    CK(hipMemset(dw, 0, nout * 8));
    CK(hipMemset(ds, 0, nout * 8));
    CK(hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    const int blocks = (nI + G - 1) / G;
    const size_t lds = (size_t)ldsKB * 1024;
    CK(hipFuncSetAttribute((const void*)walk2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)scan2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tw = 0, ts = 0;
    for (int pass = 0; pass < 2; ++pass) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(walk2_kernel, dim3(blocks), dim3(64), lds, 0, din, dw, N, nI, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&tw, e0, e1));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(scan2_kernel, dim3(blocks), dim3(64), lds, 0, din, ds, N, nI, reps);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ts, e0, e1));
    }
    CK(hipGetLastError());
    std::vector<double> ow(nout), os(nout);
    CK(hipMemcpy(ow.data(), dw, nout * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(os.data(), ds, nout * 8, hipMemcpyDeviceToHost));
    double maxrel = 0.0;
    for (int i = 0; i < nI; ++i)
        for (int k = 1; k < N; k += 2) {   // rows the walk writes: P_{2j+2} at row 2j+1
            const double* a = &ow[((size_t)i * (N + 1) + k) * 20];
            const double* b = &os[((size_t)i * (N + 1) + k) * 20];
            double nrm = 0.0, diff = 0.0;
            for (int q = 0; q < 20; ++q) { nrm = fmax(nrm, fabs(a[q])); diff = fmax(diff, fabs(a[q] - b[q])); }
            maxrel = fmax(maxrel, diff / (nrm + 1e-300));
        }
    printf("S=2 N=%d L=%d instances=%d reps=%d lds=%dKB: walk %.3f ms, scan %.3f ms (scan/walk %.2f) per "
           "factorisation of the batch; max rel |P_walk - P_scan| = %.2e\n", N, L, nI, reps, ldsKB, tw / reps, ts / reps,
           ts / tw, maxrel);
    return 0;
}
