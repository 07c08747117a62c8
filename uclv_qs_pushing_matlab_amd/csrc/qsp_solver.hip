// qsp_solver.hip — batched pusher–slider NMPC solve on gfx950 (FP64).
//
// Lane layout: one NMPC instance owns a group of L = ceil((N+1)/S)
// consecutive lanes of a wavefront; lane `lig` of the group owns the S horizon
// stages k = lig*S .. lig*S+S-1 (stage N is the terminal stage).  Every per-stage
// quantity (iterate, RK4 linearisation, IPM slacks/multipliers, Riccati factors)
// lives in that lane's VGPRs for the whole solve; nothing spills to HBM between
// SQP or IPM iterations.  Stage-parallel work (RK4 + sensitivities, barrier terms,
// step lengths) runs on all lanes at once; the two horizon recursions (Riccati
// backward, state forward) walk the group lane by lane, handing the 4x4 value
// function / state step to the neighbour lane with one DPP/bpermute shuffle.
//
// Algorithm (restating the reference OCP, NMPC_controller.m:174-300):
//   SQP  : fixed-K full Gauss-Newton steps (BASELINE "SQP-RTI, K iterations")
//   QP   : box-constrained LQ-OCP, Mehrotra predictor-corrector interior point,
//          Riccati factorisation reused by the corrector (stands in for HPIPM)
//   model: RK4 (1 step, h = Ts) + forward sensitivities of f (qsp_math.hpp)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qsp_math.hpp"
#include "qsp_kernels.h"

namespace qsp {

// ------------------------------------------------------------- group helpers
__device__ __forceinline__ double group_sum(double v, int base, int L) {
    double s = 0.0;
    for (int d = 0; d < L; ++d) s += __shfl(v, base + d);   // fixed order: identical in every lane
    return s;
}
__device__ __forceinline__ double group_min(double v, int base, int L) {
    double s = v;
    for (int d = 0; d < L; ++d) s = fmin(s, __shfl(v, base + d));
    return s;
}

// symmetric 4x4 stored as 10 entries: (0,0)(0,1)(0,2)(0,3)(1,1)(1,2)(1,3)(2,2)(2,3)(3,3)
__device__ __forceinline__ int sidx(int i, int j) {
    if (i > j) { int t = i; i = j; j = t; }
    return i == 0 ? j : (i == 1 ? 3 + j : (i == 2 ? 5 + j : 9));
}

// ------------------------------------------------------------- per-lane state
template <int S>
struct Stage {
    // SQP iterate and stage data of the current linearisation
    double x[S][4], u[S][2];
    double g[S][6];          // cost gradient (stage: tau W (y - y_ref); terminal: We (x - y_ref_e))
    double a[S][6];          // free entries of A_k (qsp_math.hpp rk4)
    double B[S][8];
    double bb[S][4];         // defect phi(x_k,u_k) - x_{k+1}
    // interior point
    double t[S][6], lm[S][6];   // slacks / multipliers: s_lo s_hi un_lo un_hi ut_lo ut_hi
    double hg[S][6];            // barrier Hessian (0..2) and gradient (3..5) additions
    double K[S][8], Ri[S][3], Pb[S][4], kk[S][2];
    double du[S][2];            // damped QP control step
    double vn[S][3];            // last QP solution of the bounded components (ds, dun, dut)
    double va[S][3];            // affine-predictor solution of the bounded components
    double dx[S][4];            // final QP state step
};

struct Ctx {
    int lane, L, grp, lig, base, N;
    bool real;
    int inst;
};

template <int S>
__device__ __forceinline__ int kof(const Ctx& c, int ls) { return c.lig * S + ls; }

// bounded component value of the QP step in slot ls
template <int S>
__device__ __forceinline__ void bnd_lohi(const SolveParams& p, const Stage<S>& st, int ls, double lo[3], double hi[3]) {
    const double v0 = st.x[ls][3], v1 = st.u[ls][0], v2 = st.u[ls][1];
    lo[0] = p.lh[0] - v0; hi[0] = p.uh[0] - v0;
    lo[1] = p.lh[1] - v1; hi[1] = p.uh[1] - v1;
    lo[2] = p.lh[2] - v2; hi[2] = p.uh[2] - v2;
}

// --------------------------------------------------------- Riccati primitives
// Terminal value function: P = diag(We), p = g_N
__device__ __forceinline__ void ric_terminal(const SolveParams& p, const double g[6], double P[10], double pv[4]) {
#pragma unroll
    for (int i = 0; i < 10; ++i) P[i] = 0.0;
    P[0] = p.We[0]; P[4] = p.We[1]; P[7] = p.We[2]; P[9] = p.We[3];
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = g[i];
}

// One backward factorisation step exploiting A = [[1,0,a0,a1],[0,1,a2,a3],[0,0,1,a4],[0,0,0,a5]].
// Hx, Hu: diagonal stage Hessian (incl. barrier); gx, gu: gradient (incl. barrier).
__device__ __forceinline__ void ric_factor_step(const double a[6], const double B[8], const double bb[4],
                                                const double Hx[4], const double Hu[2],
                                                const double gx[4], const double gu[2],
                                                double P[10], double pv[4],
                                                double K[8], double Ri[3], double Pb[4], double kk[2]) {
    // full symmetric P
    double Pm[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) Pm[i][j] = P[sidx(i, j)];
    // PA
    double PA[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        PA[i][0] = Pm[i][0];
        PA[i][1] = Pm[i][1];
        PA[i][2] = Pm[i][0] * a[0] + Pm[i][1] * a[2] + Pm[i][2];
        PA[i][3] = Pm[i][0] * a[1] + Pm[i][1] * a[3] + Pm[i][2] * a[4] + Pm[i][3] * a[5];
    }
    // PB
    double PB[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            PB[i][j] = Pm[i][0] * B[j] + Pm[i][1] * B[2 + j] + Pm[i][2] * B[4 + j] + Pm[i][3] * B[6 + j];
    // Pb, pp = p + P b
    double pp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        Pb[i] = Pm[i][0] * bb[0] + Pm[i][1] * bb[1] + Pm[i][2] * bb[2] + Pm[i][3] * bb[3];
        pp[i] = pv[i] + Pb[i];
    }
    // R~ = Hu + B'PB (sym), S~ = B'PA (2x4), r~ = gu + B'pp
    double R00 = Hu[0] + (B[0] * PB[0][0] + B[2] * PB[1][0] + B[4] * PB[2][0] + B[6] * PB[3][0]);
    double R01 = B[0] * PB[0][1] + B[2] * PB[1][1] + B[4] * PB[2][1] + B[6] * PB[3][1];
    double R11 = Hu[1] + (B[1] * PB[0][1] + B[3] * PB[1][1] + B[5] * PB[2][1] + B[7] * PB[3][1]);
    double St[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            St[i][j] = B[i] * PA[0][j] + B[2 + i] * PA[1][j] + B[4 + i] * PA[2][j] + B[6 + i] * PA[3][j];
    double rt[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) rt[i] = gu[i] + (B[i] * pp[0] + B[2 + i] * pp[1] + B[4 + i] * pp[2] + B[6 + i] * pp[3]);
    // Q~ = Hx + A'PA  (upper triangle), q~ = gx + A'pp
    double Qt[10];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const double c0 = PA[0][j], c1 = PA[1][j], c2 = PA[2][j], c3 = PA[3][j];
        const double r2 = a[0] * c0 + a[2] * c1 + c2;
        const double r3 = a[1] * c0 + a[3] * c1 + a[4] * c2 + a[5] * c3;
        if (j >= 0) Qt[sidx(0, j)] = c0;
        if (j >= 1) Qt[sidx(1, j)] = c1;
        if (j >= 2) Qt[sidx(2, j)] = r2;
        if (j >= 3) Qt[sidx(3, j)] = r3;
    }
    Qt[0] += Hx[0]; Qt[4] += Hx[1]; Qt[7] += Hx[2]; Qt[9] += Hx[3];
    double qt[4];
    qt[0] = gx[0] + pp[0];
    qt[1] = gx[1] + pp[1];
    qt[2] = gx[2] + (a[0] * pp[0] + a[2] * pp[1] + pp[2]);
    qt[3] = gx[3] + (a[1] * pp[0] + a[3] * pp[1] + a[4] * pp[2] + a[5] * pp[3]);
    // R~^-1
    const double idet = 1.0 / (R00 * R11 - R01 * R01);
    Ri[0] = R11 * idet; Ri[1] = -R01 * idet; Ri[2] = R00 * idet;
    // K = -R~^-1 S~ ; kk = -R~^-1 r~
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        K[j] = -(Ri[0] * St[0][j] + Ri[1] * St[1][j]);
        K[4 + j] = -(Ri[1] * St[0][j] + Ri[2] * St[1][j]);
    }
    kk[0] = -(Ri[0] * rt[0] + Ri[1] * rt[1]);
    kk[1] = -(Ri[1] * rt[0] + Ri[2] * rt[1]);
    // P = Q~ + S~'K ; p = q~ + K'r~
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) P[sidx(i, j)] = Qt[sidx(i, j)] + (St[0][i] * K[j] + St[1][i] * K[4 + j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = qt[i] + (K[i] * rt[0] + K[4 + i] * rt[1]);
}

// Vector-only backward step reusing the factorisation (Mehrotra corrector).
__device__ __forceinline__ void ric_vector_step(const double a[6], const double B[8], const double gx[4], const double gu[2],
                                                const double K[8], const double Ri[3], const double Pb[4],
                                                double pv[4], double kk[2]) {
    double pp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) pp[i] = pv[i] + Pb[i];
    double rt[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) rt[i] = gu[i] + (B[i] * pp[0] + B[2 + i] * pp[1] + B[4 + i] * pp[2] + B[6 + i] * pp[3]);
    double qt[4];
    qt[0] = gx[0] + pp[0];
    qt[1] = gx[1] + pp[1];
    qt[2] = gx[2] + (a[0] * pp[0] + a[2] * pp[1] + pp[2]);
    qt[3] = gx[3] + (a[1] * pp[0] + a[3] * pp[1] + a[4] * pp[2] + a[5] * pp[3]);
    kk[0] = -(Ri[0] * rt[0] + Ri[1] * rt[1]);
    kk[1] = -(Ri[1] * rt[0] + Ri[2] * rt[1]);
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = qt[i] + (K[i] * rt[0] + K[4 + i] * rt[1]);
}

// dx_{k+1} = A dx + B du + b
__device__ __forceinline__ void dyn_step(const double a[6], const double B[8], const double bb[4],
                                         const double du[2], double dx[4]) {
    const double n0 = bb[0] + ((dx[0] + a[0] * dx[2] + a[1] * dx[3]) + (B[0] * du[0] + B[1] * du[1]));
    const double n1 = bb[1] + ((dx[1] + a[2] * dx[2] + a[3] * dx[3]) + (B[2] * du[0] + B[3] * du[1]));
    const double n2 = bb[2] + ((dx[2] + a[4] * dx[3]) + (B[4] * du[0] + B[5] * du[1]));
    const double n3 = bb[3] + ((a[5] * dx[3]) + (B[6] * du[0] + B[7] * du[1]));
    dx[0] = n0; dx[1] = n1; dx[2] = n2; dx[3] = n3;
}

// ------------------------------------------------------------------ QP core
// Barrier terms of slot ls: hg[0..2] Hessian additions, hg[3..5] gradient additions.
// corrector: c_j = sigma_mu - dt_aff dl_aff  (0 for the predictor)
template <int S>
__device__ __forceinline__ void barrier_terms(const Ctx& c, const SolveParams& p, Stage<S>& st, int ls,
                                              bool corrector, double smu) {
    const int k = kof<S>(c, ls);
    double lo[3], hi[3];
    bnd_lohi<S>(p, st, ls, lo, hi);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool act = (k < c.N) && (j > 0 || k >= 1);
        const double tl = st.t[ls][2 * j], th = st.t[ls][2 * j + 1];
        const double ll = st.lm[ls][2 * j], lh = st.lm[ls][2 * j + 1];
        const double sl = ll / tl, sh = lh / th;
        double cl = 0.0, ch = 0.0;
        if (corrector) {
            const double v = st.va[ls][j];
            const double dtl = v - lo[j] - tl, dth = hi[j] - v - th;
            const double dll = -ll - sl * dtl, dlh = -lh - sh * dth;
            cl = smu - dtl * dll;
            ch = smu - dth * dlh;
        }
        const double hadd = sl + sh;
        const double gadd = ((-sl * lo[j] - sh * hi[j]) + (lh - ll)) + (ch / th - cl / tl);
        st.hg[ls][j] = act ? hadd : 0.0;
        st.hg[ls][3 + j] = act ? gadd : 0.0;
    }
}

// slack/multiplier directions of slot ls from the bounded components v of a QP solution
template <int S>
__device__ __forceinline__ void directions(const Ctx& c, const SolveParams& p, const Stage<S>& st, int ls,
                                           const double v[3], bool corrector, double smu,
                                           double dt[6], double dl[6]) {
    const int k = kof<S>(c, ls);
    double lo[3], hi[3];
    bnd_lohi<S>(p, st, ls, lo, hi);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool act = (k < c.N) && (j > 0 || k >= 1);
        const double tl = st.t[ls][2 * j], th = st.t[ls][2 * j + 1];
        const double ll = st.lm[ls][2 * j], lh = st.lm[ls][2 * j + 1];
        const double sl = ll / tl, sh = lh / th;
        double cl = 0.0, ch = 0.0;
        if (corrector) {
            const double va = st.va[ls][j];
            const double atl = va - lo[j] - tl, ath = hi[j] - va - th;
            const double all = -ll - sl * atl, alh = -lh - sh * ath;
            cl = smu - atl * all;
            ch = smu - ath * alh;
        }
        const double dtl = v[j] - lo[j] - tl, dth = hi[j] - v[j] - th;
        dt[2 * j] = act ? dtl : 0.0;
        dt[2 * j + 1] = act ? dth : 0.0;
        dl[2 * j] = act ? (cl / tl - ll - sl * dtl) : 0.0;
        dl[2 * j + 1] = act ? (ch / th - lh - sh * dth) : 0.0;
    }
}

__device__ __forceinline__ double max_step(double t, double dt, double l, double dl, double amax) {
    if (dt < 0.0) amax = fmin(amax, -t / dt);
    if (dl < 0.0) amax = fmin(amax, -l / dl);
    return amax;
}

// Backward pass over the group (factorisation or vector only), then forward pass
// writing the bounded components of the solution into `out` (va or vn).
template <int S, bool FACTOR>
__device__ __forceinline__ void riccati_solve(const Ctx& c, const SolveParams& p, Stage<S>& st, const double dx0[4],
                                              double (*out)[3]) {
    double P[10], pv[4];
#pragma unroll
    for (int i = 0; i < 10; ++i) P[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = 0.0;
    for (int j = c.L - 1; j >= 0; --j) {
        if (c.lig == j) {
#pragma unroll
            for (int ls = S - 1; ls >= 0; --ls) {
                const int k = j * S + ls;
                if (k == c.N) {
                    if (FACTOR) ric_terminal(p, st.g[ls], P, pv);
                    else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) pv[i] = st.g[ls][i];
                    }
                } else if (k < c.N) {
                    const double gx[4] = {st.g[ls][0], st.g[ls][1], st.g[ls][2], st.g[ls][3] + st.hg[ls][3]};
                    const double gu[2] = {st.g[ls][4] + st.hg[ls][4], st.g[ls][5] + st.hg[ls][5]};
                    if (FACTOR) {
                        const double Hx[4] = {p.tau * p.W[0], p.tau * p.W[1], p.tau * p.W[2], p.tau * p.W[3] + st.hg[ls][0]};
                        const double Hu[2] = {p.tau * p.W[4] + st.hg[ls][1], p.tau * p.W[5] + st.hg[ls][2]};
                        ric_factor_step(st.a[ls], st.B[ls], st.bb[ls], Hx, Hu, gx, gu, P, pv,
                                        st.K[ls], st.Ri[ls], st.Pb[ls], st.kk[ls]);
                    } else {
                        ric_vector_step(st.a[ls], st.B[ls], gx, gu, st.K[ls], st.Ri[ls], st.Pb[ls], pv, st.kk[ls]);
                    }
                }
            }
        }
        if (FACTOR) {
#pragma unroll
            for (int i = 0; i < 10; ++i) P[i] = __shfl_down(P[i], 1);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) pv[i] = __shfl_down(pv[i], 1);
    }
    // forward
    double dx[4] = {dx0[0], dx0[1], dx0[2], dx0[3]};
    for (int j = 0; j < c.L; ++j) {
        if (c.lig == j) {
#pragma unroll
            for (int ls = 0; ls < S; ++ls) {
                const int k = j * S + ls;
                if (k < c.N) {
                    double du[2];
                    du[0] = st.kk[ls][0] + (st.K[ls][0] * dx[0] + st.K[ls][1] * dx[1] + st.K[ls][2] * dx[2] + st.K[ls][3] * dx[3]);
                    du[1] = st.kk[ls][1] + (st.K[ls][4] * dx[0] + st.K[ls][5] * dx[1] + st.K[ls][6] * dx[2] + st.K[ls][7] * dx[3]);
                    out[ls][0] = dx[3];
                    out[ls][1] = du[0];
                    out[ls][2] = du[1];
                    dyn_step(st.a[ls], st.B[ls], st.bb[ls], du, dx);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) dx[i] = __shfl_up(dx[i], 1);
    }
}

// Mehrotra predictor-corrector IPM on the current linearisation.  Leaves the
// damped control step in st.du and the slacks/multipliers in st.t / st.lm.
// Returns the number of iterations taken by this lane's instance.
template <int S>
__device__ int qp_ipm(const Ctx& c, const SolveParams& p, Stage<S>& st, const double dx0[4]) {
    const double m = 2.0 * (3.0 * c.N - 1.0);
    // initial point
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        double lo[3], hi[3];
        bnd_lohi<S>(p, st, ls, lo, hi);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const bool act = (k < c.N) && (j > 0 || k >= 1);
            const double tl = fmax(-lo[j], p.t_min), th = fmax(hi[j], p.t_min);
            st.t[ls][2 * j] = act ? tl : 1.0;
            st.t[ls][2 * j + 1] = act ? th : 1.0;
            st.lm[ls][2 * j] = act ? p.mu0 / tl : 0.0;
            st.lm[ls][2 * j + 1] = act ? p.mu0 / th : 0.0;
        }
        st.du[ls][0] = 0.0;
        st.du[ls][1] = 0.0;
    }
    int nit = 0;
    for (int it = 0; it < p.qp_iters; ++it) {
        double tl_sum = 0.0;
#pragma unroll
        for (int ls = 0; ls < S; ++ls)
#pragma unroll
            for (int q = 0; q < 6; ++q) tl_sum += st.t[ls][q] * st.lm[ls][q];
        const double mu = group_sum(tl_sum, c.base, c.L) / m;
        const bool done = !(mu >= p.mu_stop);
        if (__ballot(!done) == 0ull) break;
        nit += done ? 0 : 1;
        // ---- predictor
#pragma unroll
        for (int ls = 0; ls < S; ++ls) barrier_terms<S>(c, p, st, ls, false, 0.0);
        riccati_solve<S, true>(c, p, st, dx0, st.va);
        double amax = 1.0;
        double dts[S][6], dls[S][6];
#pragma unroll
        for (int ls = 0; ls < S; ++ls) {
            directions<S>(c, p, st, ls, st.va[ls], false, 0.0, dts[ls], dls[ls]);
#pragma unroll
            for (int q = 0; q < 6; ++q) amax = max_step(st.t[ls][q], dts[ls][q], st.lm[ls][q], dls[ls][q], amax);
        }
        const double aa = group_min(amax, c.base, c.L);
        double ma = 0.0;
#pragma unroll
        for (int ls = 0; ls < S; ++ls)
#pragma unroll
            for (int q = 0; q < 6; ++q) ma += (st.t[ls][q] + aa * dts[ls][q]) * (st.lm[ls][q] + aa * dls[ls][q]);
        const double mua = group_sum(ma, c.base, c.L) / m;
        const double r = mua / mu;
        const double sg = fmax(r * r * r, p.sigma_min);
        const double smu = sg * mu;
        // ---- corrector
#pragma unroll
        for (int ls = 0; ls < S; ++ls) barrier_terms<S>(c, p, st, ls, true, smu);
        riccati_solve<S, false>(c, p, st, dx0, st.vn);
        double amx = 1.0 / p.frac;
#pragma unroll
        for (int ls = 0; ls < S; ++ls) {
            directions<S>(c, p, st, ls, st.vn[ls], true, smu, dts[ls], dls[ls]);
#pragma unroll
            for (int q = 0; q < 6; ++q) amx = max_step(st.t[ls][q], dts[ls][q], st.lm[ls][q], dls[ls][q], amx);
        }
        double alpha = p.frac * group_min(amx, c.base, c.L);
        alpha = fmin(alpha, 1.0);
        if (done) alpha = 0.0;
#pragma unroll
        for (int ls = 0; ls < S; ++ls) {
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                st.t[ls][q] += alpha * dts[ls][q];
                st.lm[ls][q] += alpha * dls[ls][q];
            }
            st.du[ls][0] += alpha * (st.vn[ls][1] - st.du[ls][0]);
            st.du[ls][1] += alpha * (st.vn[ls][2] - st.du[ls][1]);
        }
    }
    return nit;
}

// State step of the damped QP solution (rollout of the affine dynamics), into st.dx.
template <int S>
__device__ __forceinline__ void qp_rollout(const Ctx& c, Stage<S>& st, const double dx0[4]) {
    double dx[4] = {dx0[0], dx0[1], dx0[2], dx0[3]};
    for (int j = 0; j < c.L; ++j) {
        if (c.lig == j) {
#pragma unroll
            for (int ls = 0; ls < S; ++ls) {
                const int k = j * S + ls;
                if (k <= c.N) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) st.dx[ls][i] = dx[i];
                }
                if (k < c.N) dyn_step(st.a[ls], st.B[ls], st.bb[ls], st.du[ls], dx);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) dx[i] = __shfl_up(dx[i], 1);
    }
}

// Dynamics multipliers by the adjoint recursion; writes PI (B x N x 4).
//   pi_{N-1} = We dx_N + g_N ; pi_{k-1} = Hx dx_k + gx_k + A_k' pi_k + (lam_hi - lam_lo)_s
template <int S>
__device__ __forceinline__ void qp_adjoint_store(const Ctx& c, const SolveParams& p, const Stage<S>& st,
                                                 double* PI, bool write, bool shift) {
    double pi[4] = {0, 0, 0, 0};
    for (int j = c.L - 1; j >= 0; --j) {
        if (c.lig == j) {
#pragma unroll
            for (int ls = S - 1; ls >= 0; --ls) {
                const int k = j * S + ls;
                if (k == c.N) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) pi[i] = p.We[i] * st.dx[ls][i] + st.g[ls][i];
                } else if (k < c.N) {
                    if (write && (!shift || k >= 1)) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) PI[(size_t)(shift ? k - 1 : k) * 4 + i] = pi[i];
                    }
                    if (write && shift && k == c.N - 1) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) PI[(size_t)k * 4 + i] = pi[i];
                    }
                    if (k >= 1) {
                        const double* a = st.a[ls];
                        double np[4];
                        np[0] = p.tau * p.W[0] * st.dx[ls][0] + st.g[ls][0] + pi[0];
                        np[1] = p.tau * p.W[1] * st.dx[ls][1] + st.g[ls][1] + pi[1];
                        np[2] = p.tau * p.W[2] * st.dx[ls][2] + st.g[ls][2] + (a[0] * pi[0] + a[2] * pi[1] + pi[2]);
                        np[3] = p.tau * p.W[3] * st.dx[ls][3] + st.g[ls][3] +
                                (a[1] * pi[0] + a[3] * pi[1] + a[4] * pi[2] + a[5] * pi[3]);
                        np[3] += st.lm[ls][1] - st.lm[ls][0];
#pragma unroll
                        for (int i = 0; i < 4; ++i) pi[i] = np[i];
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) pi[i] = __shfl_down(pi[i], 1);
    }
}

// ------------------------------------------------------------- linearisation
template <int S>
__device__ __forceinline__ void linearize(const Ctx& c, const SolveParams& p, const ShapeDev& sh, Stage<S>& st,
                                          const double* yref, const double* yref_e) {
    // x_{k+1} of the last slot lives in slot 0 of the next lane
    double xnext[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xnext[i] = __shfl_down(st.x[0][i], 1);
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        double xn1[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) xn1[i] = (ls + 1 < S) ? st.x[(ls + 1 < S) ? ls + 1 : 0][i] : xnext[i];
        if (k < c.N) {
            Lin L;
            rk4<true>(sh, p.Ts, st.x[ls], st.u[ls], L);
#pragma unroll
            for (int i = 0; i < 4; ++i) st.bb[ls][i] = L.xn[i] - xn1[i];
#pragma unroll
            for (int i = 0; i < 6; ++i) st.a[ls][i] = L.a[i];
#pragma unroll
            for (int i = 0; i < 8; ++i) st.B[ls][i] = L.B[i];
            const double* yr = yref + (size_t)k * 6;
#pragma unroll
            for (int i = 0; i < 4; ++i) st.g[ls][i] = p.tau * p.W[i] * (st.x[ls][i] - yr[i]);
#pragma unroll
            for (int i = 0; i < 2; ++i) st.g[ls][4 + i] = p.tau * p.W[4 + i] * (st.u[ls][i] - yr[4 + i]);
        } else if (k == c.N) {
#pragma unroll
            for (int i = 0; i < 4; ++i) st.g[ls][i] = p.We[i] * (st.x[ls][i] - yref_e[i]);
            st.g[ls][4] = st.g[ls][5] = 0.0;
        }
    }
}

template <int S>
__device__ __forceinline__ double stage_cost(const Ctx& c, const SolveParams& p, const Stage<S>& st,
                                             const double* yref, const double* yref_e) {
    double cost = 0.0;
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        if (k < c.N) {
            const double* yr = yref + (size_t)k * 6;
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) { const double r = st.x[ls][i] - yr[i]; s += p.W[i] * r * r; }
#pragma unroll
            for (int i = 0; i < 2; ++i) { const double r = st.u[ls][i] - yr[4 + i]; s += p.W[4 + i] * r * r; }
            cost += 0.5 * p.tau * s;
        } else if (k == c.N) {
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) { const double r = st.x[ls][i] - yref_e[i]; s += p.We[i] * r * r; }
            cost += 0.5 * s;
        }
    }
    return cost;
}

// ------------------------------------------------------------------ kernels
template <int S>
__global__ void __launch_bounds__(256) sqp_kernel(SolveArgs A) {
    const SolveParams& p = A.p;
    Ctx c;
    c.lane = threadIdx.x & 63;
    c.N = p.N;
    c.L = (p.N + S) / S;                 // ceil((N+1)/S)
    const int G = 64 / c.L;
    c.grp = c.lane / c.L;
    c.lig = c.lane - c.grp * c.L;
    c.base = c.grp * c.L;
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    c.inst = wave * G + c.grp;
    c.real = (c.grp < G) && (c.inst < A.B);
    const int iv = c.real ? c.inst : A.B - 1;
    const int N = p.N;

    const ShapeDev& sh = A.shapes[A.shape_id ? A.shape_id[iv] : 0];
    Stage<S> st;

    // ---------------- inputs: x0, references, initial guess
    double x0[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x0[i] = A.x0[(size_t)iv * 4 + i];
    const bool ctrl = (A.flags & QSP_FLAG_CONTROLLER) != 0;
    if (ctrl) x0[3] = mat_mod(x0[3], sh.b) - sh.b * ((x0[3] < 0.0) ? 1.0 : 0.0);   // NMPC_controller.m:332
    const double* yref = A.yref + (size_t)iv * N * 6;
    const double* yref_e = A.yref_e + (size_t)iv * 4;
    const bool cold = ctrl && (A.warm_valid == nullptr || A.warm_valid[iv] == 0);
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        const int kc = k <= N ? k : N;
        const int ku = k < N ? k : N - 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) st.x[ls][i] = cold ? 0.0 : A.X_in[((size_t)iv * (N + 1) + kc) * 4 + i];
        st.u[ls][0] = cold ? p.cp.u_n_lb : A.U_in[((size_t)iv * N + ku) * 2 + 0];   // :351-355
        st.u[ls][1] = cold ? 0.0 : A.U_in[((size_t)iv * N + ku) * 2 + 1];
    }
    if (ctrl) {
        // :357-380  clip + Euler warm-start rollout, serial along the horizon
        double xc[4] = {x0[0], x0[1], x0[2], x0[3]};
        for (int j = 0; j < c.L; ++j) {
            if (c.lig == j) {
#pragma unroll
                for (int ls = 0; ls < S; ++ls) {
                    const int k = j * S + ls;
                    if (k <= N) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) st.x[ls][i] = xc[i];
                    }
                    if (k < N) {
                        const double vb = v_bound(sh, p.cp, xc[3]);
                        const double ut_old = st.u[ls][1];
                        if (fabs(ut_old) > vb) {
                            const double sgn = ut_old > 0.0 ? 1.0 : -1.0;
                            st.u[ls][1] = sgn * vb;
                            st.u[ls][0] = st.u[ls][1] * st.u[ls][0] / ut_old;
                        }
                        DynOut d;
                        dynamics<false>(sh, xc[2], xc[3], st.u[ls][0], st.u[ls][1], d);
#pragma unroll
                        for (int i = 0; i < 4; ++i) xc[i] = xc[i] + p.Ts * d.f[i];
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) xc[i] = __shfl_up(xc[i], 1);
        }
    }

    // ---------------- SQP
    int status = 0;
    int qp_total = 0;
    for (int it = 0; it < p.sqp_iters; ++it) {
        linearize<S>(c, p, sh, st, yref, yref_e);
        double dx0[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) dx0[i] = x0[i] - st.x[0][i];   // valid in lane lig == 0
        qp_total += qp_ipm<S>(c, p, st, dx0);
        qp_rollout<S>(c, st, dx0);
        const bool last = (it + 1 == p.sqp_iters);
        if (last) qp_adjoint_store<S>(c, p, st, A.PI_out + (size_t)iv * N * 4, c.real, (A.flags & QSP_FLAG_SHIFT) != 0);
#pragma unroll
        for (int ls = 0; ls < S; ++ls) {
            const int k = kof<S>(c, ls);
            if (k <= N) {
#pragma unroll
                for (int i = 0; i < 4; ++i) st.x[ls][i] += st.dx[ls][i];
            }
            if (k < N) {
                st.u[ls][0] += st.du[ls][0];
                st.u[ls][1] += st.du[ls][1];
            }
        }
    }
    // ---------------- outputs
    bool bad = false;
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        if (k <= N) for (int i = 0; i < 4; ++i) bad |= !isfinite(st.x[ls][i]);
        if (k < N) for (int i = 0; i < 2; ++i) bad |= !isfinite(st.u[ls][i]);
    }
    const double nbad = group_sum(bad ? 1.0 : 0.0, c.base, c.L);
    status = nbad > 0.0 ? 1 : 0;
    const double cost = group_sum(stage_cost<S>(c, p, st, yref, yref_e), c.base, c.L);
    if (!c.real) return;
    const bool shift = (A.flags & QSP_FLAG_SHIFT) != 0;
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        if (k == 0) {
            A.u0[(size_t)iv * 2 + 0] = st.u[ls][0];
            A.u0[(size_t)iv * 2 + 1] = st.u[ls][1];
            A.status[iv] = status;
            A.sqp_iter[iv] = p.sqp_iters;
            A.qp_iter[iv] = qp_total;
            A.cost[iv] = cost;
        }
        if (k <= N) {
            // shifted: X(:,k-1) = X(:,k) for k>=1, and X(:,N) = X(:,N)  (NMPC_controller.m:397-399)
            if (!shift || k >= 1)
                for (int i = 0; i < 4; ++i) A.X_out[((size_t)iv * (N + 1) + (shift ? k - 1 : k)) * 4 + i] = st.x[ls][i];
            if (shift && k == N)
                for (int i = 0; i < 4; ++i) A.X_out[((size_t)iv * (N + 1) + N) * 4 + i] = st.x[ls][i];
        }
        if (k < N) {
            if (!shift || k >= 1)
                for (int i = 0; i < 2; ++i) A.U_out[((size_t)iv * N + (shift ? k - 1 : k)) * 2 + i] = st.u[ls][i];
            if (shift && k == N - 1)
                for (int i = 0; i < 2; ++i) A.U_out[((size_t)iv * N + N - 1) * 2 + i] = st.u[ls][i];
        }
    }
    if (A.warm_valid && ctrl) A.warm_valid[iv] = 1;
}

// ----------------------------------------------------- building-block kernels
__global__ void spline_kernel(const ShapeDev* shapes, const int32_t* sid, int n, const double* s,
                              double* C, double* D, double* Dd, double* kappa) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ShapeDev& sh = shapes[sid[i]];
    SplineEval e;
    spline_eval(sh, s[i], e);
    for (int c = 0; c < 2; ++c) { C[2 * i + c] = e.C[c]; D[2 * i + c] = e.D[c]; Dd[2 * i + c] = e.Dd[c]; }
    kappa[i] = (e.D[0] * e.Dd[1] - e.D[1] * e.Dd[0]) / (e.D[0] * e.D[0] + e.D[1] * e.D[1]);
}

__global__ void dynamics_kernel(const ShapeDev* shapes, const int32_t* sid, int n, const double* x, const double* u,
                                double* f, double* J) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ShapeDev& sh = shapes[sid[i]];
    DynOut d;
    dynamics<true>(sh, x[4 * i + 2], x[4 * i + 3], u[2 * i], u[2 * i + 1], d);
    for (int r = 0; r < 4; ++r) {
        f[4 * i + r] = d.f[r];
        double* Jr = J + (size_t)24 * i + 6 * r;
        Jr[0] = 0.0; Jr[1] = 0.0;
        Jr[2] = r < 2 ? d.Jth[r] : 0.0;
        Jr[3] = d.Js[r]; Jr[4] = d.Jun[r]; Jr[5] = d.Jut[r];
    }
}

__global__ void rk4_kernel(const ShapeDev* shapes, const int32_t* sid, int n, double h, const double* x, const double* u,
                           double* xn, double* Aout, double* Bout) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ShapeDev& sh = shapes[sid[i]];
    double xi[4] = {x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]};
    double ui[2] = {u[2 * i], u[2 * i + 1]};
    Lin L;
    rk4<true>(sh, h, xi, ui, L);
    double* Ai = Aout + (size_t)16 * i;
    const double Afull[16] = {1.0, 0.0, L.a[0], L.a[1], 0.0, 1.0, L.a[2], L.a[3],
                              0.0, 0.0, 1.0, L.a[4], 0.0, 0.0, 0.0, L.a[5]};
    for (int q = 0; q < 16; ++q) Ai[q] = Afull[q];
    for (int q = 0; q < 8; ++q) Bout[(size_t)8 * i + q] = L.B[q];
    for (int q = 0; q < 4; ++q) xn[4 * i + q] = L.xn[q];
}

__global__ void vbound_kernel(const ShapeDev* shapes, const int32_t* sid, int n, CtrlParams cp, const double* s,
                              double* vb) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    vb[i] = v_bound(shapes[sid[i]], cp, s[i]);
}

// Batched LQ-QP solve with given stage data (QP-level parity).  Uses the same
// register-resident lane layout and IPM as the SQP kernel.  A must have the
// pusher-slider structure (only its six free entries are read).
template <int S>
__global__ void __launch_bounds__(256) qp_kernel(QPArgs A) {
    const SolveParams& p = A.p;
    Ctx c;
    c.lane = threadIdx.x & 63;
    c.N = p.N;
    c.L = (p.N + S) / S;
    const int G = 64 / c.L;
    c.grp = c.lane / c.L;
    c.lig = c.lane - c.grp * c.L;
    c.base = c.grp * c.L;
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    c.inst = wave * G + c.grp;
    c.real = (c.grp < G) && (c.inst < A.nb);
    const int iv = c.real ? c.inst : A.nb - 1;
    const int N = p.N;
    Stage<S> st;
    // bounds in step space: lo = lh - v, hi = uh - v  =>  v = lh - lo  (QPArgs uses lh = 0)
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        const int ku = k < N ? k : N - 1;
        const double* Ak = A.A + ((size_t)iv * N + ku) * 16;
        st.a[ls][0] = Ak[2]; st.a[ls][1] = Ak[3]; st.a[ls][2] = Ak[6];
        st.a[ls][3] = Ak[7]; st.a[ls][4] = Ak[11]; st.a[ls][5] = Ak[15];
        for (int q = 0; q < 8; ++q) st.B[ls][q] = A.B[((size_t)iv * N + ku) * 8 + q];
        for (int q = 0; q < 4; ++q) st.bb[ls][q] = A.b[((size_t)iv * N + ku) * 4 + q];
        const double* gk = A.g + (size_t)iv * (6 * N + 4) + (k < N ? 6 * k : 6 * N);
        for (int q = 0; q < 6; ++q) st.g[ls][q] = (k < N || q < 4) ? gk[q] : 0.0;
        // encode the bounds through x/u so that bnd_lohi() reproduces lo/hi with lh = 0
        const double* lo = A.lo + ((size_t)iv * N + ku) * 3;
        st.x[ls][3] = -lo[0]; st.u[ls][0] = -lo[1]; st.u[ls][1] = -lo[2];
    }
    // lo = lh - v with lh = 0 and hi = uh - v with uh = bound width (equal on every stage, as in the OCP);
    // Hessian: tau = 1, W = stage diag, We = terminal diag (equal on every stage, as in the OCP).
    SolveParams pq = p;
    for (int j = 0; j < 3; ++j) { pq.lh[j] = 0.0; pq.uh[j] = A.width[j]; }
    double dx0[4];
    for (int i = 0; i < 4; ++i) dx0[i] = A.dx0[(size_t)iv * 4 + i];
    const int nit = qp_ipm<S>(c, pq, st, dx0);
    qp_rollout<S>(c, st, dx0);
    qp_adjoint_store<S>(c, pq, st, A.pi + (size_t)iv * N * 4, c.real, false);
    if (!c.real) return;
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        if (k <= N) for (int i = 0; i < 4; ++i) A.dx[((size_t)iv * (N + 1) + k) * 4 + i] = st.dx[ls][i];
        if (k < N) {
            for (int i = 0; i < 2; ++i) A.du[((size_t)iv * N + k) * 2 + i] = st.du[ls][i];
            for (int q = 0; q < 6; ++q) A.lam[((size_t)iv * N + k) * 6 + q] = st.lm[ls][q];
        }
        if (k == 0) A.iters[iv] = nit;
    }
}

// ------------------------------------------------------------------ launchers
template <int S>
static hipError_t launch_sqp_S(const SolveArgs& a, hipStream_t stream) {
    const int L = (a.p.N + S) / S;
    const int G = 64 / L;
    const int waves = (a.B + G - 1) / G;
    const int threads = 256;
    const int blocks = (waves * 64 + threads - 1) / threads;
    hipLaunchKernelGGL(sqp_kernel<S>, dim3(blocks), dim3(threads), 0, stream, a);
    return hipGetLastError();
}

template <int S>
static hipError_t launch_qp_S(const QPArgs& a, hipStream_t stream) {
    const int L = (a.p.N + S) / S;
    const int G = 64 / L;
    const int waves = (a.nb + G - 1) / G;
    const int threads = 256;
    const int blocks = (waves * 64 + threads - 1) / threads;
    hipLaunchKernelGGL(qp_kernel<S>, dim3(blocks), dim3(threads), 0, stream, a);
    return hipGetLastError();
}

int lanes_per_instance(int N, int S) { return (N + S) / S; }

hipError_t launch_sqp(const SolveArgs& a, int S, hipStream_t stream) {
    switch (S) {
        case 1: return launch_sqp_S<1>(a, stream);
        case 2: return launch_sqp_S<2>(a, stream);
        case 3: return launch_sqp_S<3>(a, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_qp(const QPArgs& a, int S, hipStream_t stream) {
    switch (S) {
        case 1: return launch_qp_S<1>(a, stream);
        case 2: return launch_qp_S<2>(a, stream);
        case 3: return launch_qp_S<3>(a, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_spline(const ShapeDev* shapes, const int32_t* sid, int n, const double* s, double* C, double* D,
                         double* Dd, double* kappa, hipStream_t stream) {
    hipLaunchKernelGGL(spline_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, shapes, sid, n, s, C, D, Dd, kappa);
    return hipGetLastError();
}
hipError_t launch_dynamics(const ShapeDev* shapes, const int32_t* sid, int n, const double* x, const double* u,
                           double* f, double* J, hipStream_t stream) {
    hipLaunchKernelGGL(dynamics_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, shapes, sid, n, x, u, f, J);
    return hipGetLastError();
}
hipError_t launch_rk4(const ShapeDev* shapes, const int32_t* sid, int n, double h, const double* x, const double* u,
                      double* xn, double* A, double* B, hipStream_t stream) {
    hipLaunchKernelGGL(rk4_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, shapes, sid, n, h, x, u, xn, A, B);
    return hipGetLastError();
}
hipError_t launch_vbound(const ShapeDev* shapes, const int32_t* sid, int n, CtrlParams cp, const double* s, double* vb,
                         hipStream_t stream) {
    hipLaunchKernelGGL(vbound_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, shapes, sid, n, cp, s, vb);
    return hipGetLastError();
}

}  // namespace qsp
