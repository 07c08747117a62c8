/*
 * qsp_oracle.c — CPU restatement of the reference NMPC hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker.  The product
 * path (uclv_qs_pushing_matlab_amd/) never links or calls it.
 *
 * PARITY STATUS: UNPINNED against acados/CasADi/HPIPM.  The reference solves the
 * OCP inside acados v0.2.1 (un-vendored, not runnable here: no MATLAB, no CasADi,
 * no acados).  This file restates, from the reference sources:
 *   - the clamped cubic B-spline contour, as a FULL basis sum with the half-open
 *     degree-0 indicator and the zero-denominator guards
 *       (acados_nmpc/bspline_shape.m:40-72 eval_bspline_sym, :74-83 getSymbolicSpline,
 *        :85-104 getSymboliSplineDot, :106-116 getNormalTangentialVersors,
 *        :137-152 getSymbolicAngleCurvatures / getAngleCurvatures)
 *   - the variable-shape motion-cone dynamics f(x,u)
 *       (acados_nmpc/PusherSliderModel.m:503-603 symbolic_model_variable_shape)
 *     differentiated by forward-mode AD (dual numbers), as CasADi's VDE would
 *   - ERK/RK4 with forward sensitivities (acados sim_method "erk", NMPC_controller.m:272)
 *   - the linear-LS Gauss-Newton OCP (NMPC_controller.m:174-268) with bgh bounds
 *     h = [s; u_n; u_t] (:237,:251-252) and x0 equality (:265,:334)
 *   - a box-constrained LQ-QP primal-dual interior point (Mehrotra) solved by a
 *     dense Riccati recursion (stands in for HPIPM, NMPC_controller.m:272-276)
 *   - fixed-K full-step SQP (the BASELINE "SQP-RTI, K iterations" metric)
 *   - the NMPC_controller.solve() wrapper semantics (NMPC_controller.m:329-423):
 *     s pre-wrap, y_ref staging, cold start, tangential-velocity clip, Euler
 *     warm-start rollout, shift of the warm start, u0, cost.
 * The GPU kernel is an independent implementation (span-based de Boor, hand
 * derived Jacobian, structure-exploiting Riccati); agreement between the two is
 * what the parity tests check.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* The scalar type of the restatement.  Default: real = double (the or_* API).  Built a second
 * time with OR_EXT = 1 (long double, 64-bit significand) or OR_EXT = 2 (__float128, 113-bit,
 * libquadmath) it is the extended-precision oracle: the same formulas evaluated 2^11 / 2^60 times
 * more finely, exported as orx_controller_solve (double in/out, converted at the boundary) to
 * adjudicate the lanes where the kernel-order twin and the double restatement disagree
 * (tests/test_extended_oracle.py). */
#if defined(OR_EXT) && OR_EXT == 2
#include <quadmath.h>
typedef __float128 real;
#undef isfinite
#define isfinite(x) finiteq(x)
#define sin(x) sinq(x)
#define cos(x) cosq(x)
#define sqrt(x) sqrtq(x)
#define fabs(x) fabsq(x)
#define fmod(x, y) fmodq(x, y)
#define floor(x) floorq(x)
#elif defined(OR_EXT) && OR_EXT == 1
#include <tgmath.h>
typedef long double real;
#else
typedef double real;
#endif
#ifdef OR_EXT
#define OR_EXPORT static   /* the extended build exports orx_controller_solve only */
#else
#define OR_EXPORT
#endif

#define NX 4
#define NU 2
#define NDIR 6 /* AD directions: x, y, theta, s, u_n, u_t */
#define OR_MAX_N 128
#define OR_MAX_CTRL 256
#define OR_KKT_DIAG 22   /* doubles per lane of or_set_kkt_diag */

/* ------------------------------------------------------------------ shapes */
typedef struct {
    int n;              /* number of control points (after closing the loop) */
    const real *P;    /* n x 2, row-major */
    const real *S;    /* n + 4 knots */
    real b;           /* contour length (bspline_shape.m:37) */
    real c;           /* c_ellipse = tau_max / (mu_sg m g)  (PusherSliderModel.m:53,55) */
    real mu;          /* mu_sp */
} or_shape;

#include "or_opts.h"

/* ================================================================ dual numbers */
typedef struct { real v, d[NDIR]; } dual;

static inline dual dc(real v) { dual r; r.v = v; for (int i = 0; i < NDIR; ++i) r.d[i] = 0.0; return r; }
static inline dual dadd(dual a, dual b) { dual r; r.v = a.v + b.v; for (int i = 0; i < NDIR; ++i) r.d[i] = a.d[i] + b.d[i]; return r; }
static inline dual dsub(dual a, dual b) { dual r; r.v = a.v - b.v; for (int i = 0; i < NDIR; ++i) r.d[i] = a.d[i] - b.d[i]; return r; }
static inline dual dneg(dual a) { dual r; r.v = -a.v; for (int i = 0; i < NDIR; ++i) r.d[i] = -a.d[i]; return r; }
static inline dual dmul(dual a, dual b) { dual r; r.v = a.v * b.v; for (int i = 0; i < NDIR; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i]; return r; }
static inline dual dscale(dual a, real s) { dual r; r.v = a.v * s; for (int i = 0; i < NDIR; ++i) r.d[i] = a.d[i] * s; return r; }
static inline dual ddiv(dual a, dual b) {
    dual r; r.v = a.v / b.v;
    for (int i = 0; i < NDIR; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) / b.v;
    return r;
}
static inline dual dsqrt(dual a) {
    dual r; r.v = sqrt(a.v);
    for (int i = 0; i < NDIR; ++i) r.d[i] = a.d[i] / (2.0 * r.v);
    return r;
}
static inline dual dsin(dual a) { dual r; r.v = sin(a.v); real c = cos(a.v); for (int i = 0; i < NDIR; ++i) r.d[i] = c * a.d[i]; return r; }
static inline dual dcos(dual a) { dual r; r.v = cos(a.v); real s = -sin(a.v); for (int i = 0; i < NDIR; ++i) r.d[i] = s * a.d[i]; return r; }
/* indicator: derivative is zero (CasADi comparison operators) */
static inline dual dind(int cond) { return dc(cond ? 1.0 : 0.0); }

/* ================================================================ B-spline */
/* Cox–de Boor recursion with value and d/ds, 1-based knot index i, as
 * bspline_shape.m:40-72: zero-support guard :46, half-open indicator :52,
 * zero-denominator guards :59-68. */
static void basis(const real *S1 /* 1-based */, real s, int i, int ord, real *N, real *dN)
{
    if (S1[i + ord + 1] == S1[i]) { *N = 0.0; *dN = 0.0; return; }
    if (ord == 0) { *N = ((s < S1[i + 1]) && (s >= S1[i])) ? 1.0 : 0.0; *dN = 0.0; return; }
    real N1, dN1, N2, dN2;
    basis(S1, s, i, ord - 1, &N1, &dN1);
    basis(S1, s, i + 1, ord - 1, &N2, &dN2);
    real m1 = 0.0, dm1 = 0.0, m2 = 0.0, dm2 = 0.0;
    if (S1[i + ord] != S1[i]) { real den = S1[i + ord] - S1[i]; m1 = (s - S1[i]) / den; dm1 = 1.0 / den; }
    if (S1[i + ord + 1] != S1[i + 1]) { real den = S1[i + ord + 1] - S1[i + 1]; m2 = (S1[i + ord + 1] - s) / den; dm2 = -1.0 / den; }
    *N = m1 * N1 + m2 * N2;
    *dN = (dm1 * N1 + m1 * dN1) + (dm2 * N2 + m2 * dN2);
}

/* FC(s) = sum_i N_{i,3}(s) P_i  (getSymbolicSpline, bspline_shape.m:74-83) */
static void spline_C(const or_shape *sh, real s, real C[2], real dC[2])
{
    const real *S1 = sh->S - 1;
    C[0] = C[1] = dC[0] = dC[1] = 0.0;
    for (int i = 1; i <= sh->n; ++i) {
        real N, dN;
        basis(S1, s, i, 3, &N, &dN);
        C[0] += N * sh->P[2 * (i - 1) + 0];
        C[1] += N * sh->P[2 * (i - 1) + 1];
        dC[0] += dN * sh->P[2 * (i - 1) + 0];
        dC[1] += dN * sh->P[2 * (i - 1) + 1];
    }
}

/* FC_dot(s) = sum_{i>=2} cj_1(i) N_{i,2}(s), cj_1 = p (P_i - P_{i-1})/(S_{i+p} - S_i)
 * (getSymboliSplineDot, bspline_shape.m:85-104) */
static void spline_Cdot(const or_shape *sh, real s, real D[2], real dD[2])
{
    const real *S1 = sh->S - 1;
    D[0] = D[1] = dD[0] = dD[1] = 0.0;
    for (int i = 2; i <= sh->n; ++i) {
        real cx = 0.0, cy = 0.0;
        if (S1[i + 3] != S1[i]) {
            real den = S1[i + 3] - S1[i];
            cx = 3.0 * ((sh->P[2 * (i - 1) + 0] - sh->P[2 * (i - 2) + 0]) / den);
            cy = 3.0 * ((sh->P[2 * (i - 1) + 1] - sh->P[2 * (i - 2) + 1]) / den);
        }
        real N, dN;
        basis(S1, s, i, 2, &N, &dN);
        D[0] += cx * N; D[1] += cy * N;
        dD[0] += cx * dN; dD[1] += cy * dN;
    }
}

/* s_mod inside the OCP model: fmod(s,b) + (s<0) b  (PusherSliderModel.m:526) */
static real smod_model(real s, real b) { return fmod(s, b) + ((s < 0.0) ? b : 0.0); }

/* MATLAB floor-mod  mod(a,b) = a - floor(a/b) b   (NMPC_controller.m:320,332) */
static real mat_mod(real a, real b)
{
    if (b == 0.0) return a;
    real r = a - floor(a / b) * b;
    if (r == b) r = 0.0;
    return r;
}

/* ================================================================ dynamics */
/* f(x,u) and J = d f / d(x,u) (4 x 6, row-major) — PusherSliderModel.m:503-603 */
/* motion-cone modes of the dynamics evaluations since the last reset, base 4 (diagnostics only;
 * unsigned: evaluations outside the SQP's reset points keep shifting it, which wraps, never UB) */
static __thread uint32_t g_mode_code = 0;

static void dynamics(const or_shape *sh, const real x[4], const real u[2], real f[4], real *J)
{
    dual X[4], U[2];
    for (int i = 0; i < 4; ++i) { X[i] = dc(x[i]); X[i].d[i] = 1.0; }
    for (int i = 0; i < 2; ++i) { U[i] = dc(u[i]); U[i].d[4 + i] = 1.0; }

    /* s_mod (:526); d/ds fmod(s,b) = 1 */
    dual sig = X[3];
    sig.v = smod_model(x[3], sh->b);

    real C[2], dC[2], D[2], dD[2];
    spline_C(sh, sig.v, C, dC);
    spline_Cdot(sh, sig.v, D, dD);
    dual Px = dc(C[0]), Py = dc(C[1]), Dx = dc(D[0]), Dy = dc(D[1]);
    for (int i = 0; i < NDIR; ++i) {
        Px.d[i] = dC[0] * sig.d[i]; Py.d[i] = dC[1] * sig.d[i];
        Dx.d[i] = dD[0] * sig.d[i]; Dy.d[i] = dD[1] * sig.d[i];
    }
    /* t = C'/|C'|, n = -[-t_y, t_x]  (bspline_shape.m:108-111) */
    dual nrm = dsqrt(dadd(dmul(Dx, Dx), dmul(Dy, Dy)));
    dual tx = ddiv(Dx, nrm), ty = ddiv(Dy, nrm);
    dual nx = ty, ny = dneg(tx);
    /* NT_p = R_NT' S_p'  (:532-534) */
    dual px = dadd(dmul(nx, Px), dmul(ny, Py));
    dual py = dadd(dmul(tx, Px), dmul(ty, Py));

    dual sn = dsin(X[2]), cs = dcos(X[2]);
    real c = sh->c, mu = sh->mu;
    real c2 = c * c;
    dual px2 = dmul(px, px), py2 = dmul(py, py), pxpy = dmul(px, py);
    dual fac = ddiv(dc(1.0), dadd(dadd(dc(c2), px2), py2));                              /* :544 */
    dual gl = ddiv(dadd(dsub(dc(mu * c2), pxpy), dscale(px2, mu)),
                   dsub(dadd(dc(c2), py2), dscale(pxpy, mu)));                            /* :547 */
    dual gr = ddiv(dsub(dsub(dc(-mu * c2), pxpy), dscale(px2, mu)),
                   dadd(dadd(dc(c2), py2), dscale(pxpy, mu)));                            /* :548 */
    dual rho = ddiv(U[1], U[0]);                                                         /* :551 */

    /* W_R_S S_R_NT fac Q  (:554-559) */
    dual R[2][2] = {{cs, dneg(sn)}, {sn, cs}};
    dual RNT[2][2] = {{nx, tx}, {ny, ty}};
    dual Q[2][2] = {{dadd(dc(c2), px2), pxpy}, {pxpy, dadd(dc(c2), py2)}};
    dual M1[2][2], M3[2][2];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            M1[i][j] = dadd(dmul(R[i][0], RNT[0][j]), dmul(R[i][1], RNT[1][j]));
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) {
            dual a = dmul(M1[i][0], fac), b = dmul(M1[i][1], fac);
            M3[i][j] = dadd(dmul(a, Q[0][j]), dmul(b, Q[1][j]));
        }
    /* sticking (:557-560) */
    dual st[4];
    st[0] = dadd(dmul(M3[0][0], U[0]), dmul(M3[0][1], U[1]));
    st[1] = dadd(dmul(M3[1][0], U[0]), dmul(M3[1][1], U[1]));
    st[2] = dadd(dmul(dmul(fac, dneg(py)), U[0]), dmul(dmul(fac, px), U[1]));
    st[3] = dc(0.0);
    /* sliding left (:563-573) and right (:575-585) */
    dual sl[4], sr[4];
    for (int side = 0; side < 2; ++side) {
        dual g = side == 0 ? gl : gr;
        dual *o = side == 0 ? sl : sr;
        dual v0 = dadd(M3[0][0], dmul(M3[0][1], g));
        dual v1 = dadd(M3[1][0], dmul(M3[1][1], g));
        o[0] = dmul(v0, U[0]);
        o[1] = dmul(v1, U[0]);
        o[2] = dmul(dmul(fac, dadd(dneg(py), dmul(g, px))), U[0]);
        o[3] = dsub(U[1], dmul(U[0], g));
    }
    /* indicator blend (:587-589); comparisons with NaN are false */
    dual ist = dmul(dind(rho.v >= gr.v), dind(rho.v <= gl.v));
    dual isl = dind(rho.v > gl.v), isr = dind(rho.v < gr.v);
    g_mode_code = g_mode_code * 4u + (uint32_t)(ist.v != 0.0 ? 0 : (isl.v != 0.0 ? 1 : (isr.v != 0.0 ? 2 : 3)));
    for (int r = 0; r < 4; ++r) {
        dual v = dadd(dadd(dmul(ist, st[r]), dmul(isl, sl[r])), dmul(isr, sr[r]));
        f[r] = v.v;
        if (J) for (int q = 0; q < NDIR; ++q) J[r * NDIR + q] = v.d[q];
    }
}

/* tangent-angle rate kappa(s) = d/ds atan2(C'_y, C'_x) (bspline_shape.m:137-152) */
static real angle_rate(const or_shape *sh, real s)
{
    real D[2], dD[2];
    spline_Cdot(sh, s, D, dD);
    return (D[0] * dD[1] - D[1] * dD[0]) / (D[0] * D[0] + D[1] * D[1]);
}

/* v_bound(s)  (NMPC_controller.m:319-327) */
static real v_bound(const or_shape *sh, const or_opts *o, real s)
{
    real sm = mat_mod(s, sh->b);
    real ta = fabs(angle_rate(sh, sm));
    real v = o->v_alpha / (fabs(ta - o->t_angle0) + 0.0001) + o->d_v;
    return v < o->u_t_ub ? v : o->u_t_ub;
}

/* ================================================================ RK4 + VDE */
static const real RK_A[4] = {0.0, 0.5, 0.5, 1.0};
static const real RK_B[4] = {(real)1 / 6, (real)1 / 3, (real)1 / 3, (real)1 / 6};

/* The model probe (or_opts.model_probe): set by the solve entry points before their parallel
 * region, read-only inside it. */
static real g_probe_eps = 0.0;
static uint64_t g_probe_seed = 0;

static inline uint64_t mix64(uint64_t z)
{
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static void probe_outputs(const real x[4], const real u[2], real xn[4], real A[16], real B[8])
{
    uint64_t h = mix64(g_probe_seed);
    for (int i = 0; i < 4; ++i) { uint64_t b; memcpy(&b, &x[i], 8); h = mix64(h ^ b); }
    for (int i = 0; i < 2; ++i) { uint64_t b; memcpy(&b, &u[i], 8); h = mix64(h ^ b); }
    real *out[3] = {xn, A, B};
    const int len[3] = {4, 16, 8};
    int e = 0;
    for (int a = 0; a < 3; ++a) {
        real scale = 0.0;   /* the array's largest entry: differences between formulations are
                                 absolute at that scale, not relative to each (possibly tiny) entry */
        for (int i = 0; i < len[a]; ++i) scale = fmax(scale, fabs(out[a][i]));
        for (int i = 0; i < len[a]; ++i, ++e) {
            const uint64_t r = mix64(h + (uint64_t)e);
            out[a][i] += ((r & 1) ? g_probe_eps : -g_probe_eps) * scale;
        }
    }
}

/* x+ = phi(x,u) and A = dphi/dx (4x4), B = dphi/du (4x2), row-major */
static void rk4_sens(const or_shape *sh, real h, const real x[4], const real u[2],
                     real xn[4], real A[16], real B[8])
{
    real Sx[4][6];   /* sensitivity of current stage state wrt (x0,u) */
    real K[4][4], SK[4][4][6];
    for (int st = 0; st < 4; ++st) {
        real xs[4];
        for (int i = 0; i < 4; ++i) {
            xs[i] = x[i];
            for (int j = 0; j < 6; ++j) Sx[i][j] = (i == j) ? 1.0 : 0.0;
        }
        if (st > 0) {
            real a = h * RK_A[st];
            for (int i = 0; i < 4; ++i) {
                xs[i] += a * K[st - 1][i];
                for (int j = 0; j < 6; ++j) Sx[i][j] += a * SK[st - 1][i][j];
            }
        }
        real J[24];
        dynamics(sh, xs, u, K[st], J);
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 6; ++j) {
                real acc = (j >= 4) ? J[i * 6 + j] : 0.0;
                for (int m = 0; m < 4; ++m) acc += J[i * 6 + m] * Sx[m][j];
                SK[st][i][j] = acc;
            }
    }
    for (int i = 0; i < 4; ++i) {
        real acc = x[i];
        real S[6];
        for (int j = 0; j < 6; ++j) S[j] = (i == j) ? 1.0 : 0.0;
        for (int st = 0; st < 4; ++st) {
            real w = h * RK_B[st];
            acc += w * K[st][i];
            for (int j = 0; j < 6; ++j) S[j] += w * SK[st][i][j];
        }
        xn[i] = acc;
        for (int j = 0; j < 4; ++j) A[i * 4 + j] = S[j];
        for (int j = 0; j < 2; ++j) B[i * 2 + j] = S[4 + j];
    }
    if (g_probe_eps != 0.0) probe_outputs(x, u, xn, A, B);
}

/* ================================================================ QP (IPM) */
/* Bounded components per stage: 0 = s (x[3]), 1 = u_n (u[0]), 2 = u_t (u[1]) */
typedef struct {
    int N;
    const real *A, *B, *b;     /* N x 16, N x 8, N x 4 */
    const real *H;             /* N x 6 stage diag Hessian, + 4 terminal (at H + 6N) */
    const real *g;             /* N x 6 stage gradient, + 4 terminal */
    const real *lo, *hi;       /* N x 3 bounds in step space */
    const uint8_t *act;          /* N x 3 active flags */
    real dx0[4];
} or_qp;

typedef struct {
    real *dx;   /* (N+1) x 4 */
    real *du;   /* N x 2 */
    real *pi;   /* N x 4 */
    real *lam;  /* N x 3 x 2 (lo, hi) */
    real *t;    /* N x 3 x 2 */
} or_qp_sol;

/* Experiments on the merit SQP (tests/tools/kkt_breakdown.py; 0 = the reference's algorithm):
 *   1 full-step multipliers (PI, LAM = the QP's; acados full_step_dual),
 *   2 the QP's u-bound multipliers recovered from its u-stationarity (exact QP duals),
 *   4 no minimum step: backtrack down to 1e-12 instead of accepting the step at ls_alpha_min. */
static int g_exp = 0;
OR_EXPORT void or_set_experiment(int flags) { g_exp = flags; }

static void inv2(const real R[4], real Ri[4])
{
    real det = R[0] * R[3] - R[1] * R[2];
    real id = 1.0 / det;
    Ri[0] = R[3] * id; Ri[1] = -R[1] * id; Ri[2] = -R[2] * id; Ri[3] = R[0] * id;
}

/* Riccati factor + solve of the barrier-modified LQ problem.
 * Hd: N x 6 diag Hessian incl. barrier; gd: N x 6 gradient; terminal from qp.
 * If factor != 0 computes and stores K, Ri, Pb; otherwise reuses them. */
typedef struct { real K[OR_MAX_N][8], kk[OR_MAX_N][2], Ri[OR_MAX_N][4], Pb[OR_MAX_N][4]; } or_fact;

static void riccati(const or_qp *qp, const real *Hd, const real *gd, or_fact *F, int factor,
                    real *dx /* (N+1)x4 */, real *du /* N x 2 */)
{
    int N = qp->N;
    real P[16] = {0}, p[4];
    for (int i = 0; i < 4; ++i) { P[i * 4 + i] = qp->H[6 * N + i]; p[i] = qp->g[6 * N + i]; }
    for (int k = N - 1; k >= 0; --k) {
        const real *A = qp->A + 16 * k, *B = qp->B + 8 * k, *bb = qp->b + 4 * k;
        const real *Hk = Hd + 6 * k, *gk = gd + 6 * k;
        real pp[4], rt[2], qt[4];
        if (factor) {
            real Pb[4];
            for (int i = 0; i < 4; ++i) { real a = 0; for (int j = 0; j < 4; ++j) a += P[i * 4 + j] * bb[j]; Pb[i] = a; }
            memcpy(F->Pb[k], Pb, sizeof Pb);
        }
        for (int i = 0; i < 4; ++i) pp[i] = p[i] + F->Pb[k][i];
        for (int i = 0; i < 2; ++i) { real a = gk[4 + i]; for (int j = 0; j < 4; ++j) a += B[j * 2 + i] * pp[j]; rt[i] = a; }
        for (int i = 0; i < 4; ++i) { real a = gk[i]; for (int j = 0; j < 4; ++j) a += A[j * 4 + i] * pp[j]; qt[i] = a; }
        if (factor) {
            real PA[16], PB[8], Rt[4], St[8], Qt[16];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) { real a = 0; for (int m = 0; m < 4; ++m) a += P[i * 4 + m] * A[m * 4 + j]; PA[i * 4 + j] = a; }
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 2; ++j) { real a = 0; for (int m = 0; m < 4; ++m) a += P[i * 4 + m] * B[m * 2 + j]; PB[i * 2 + j] = a; }
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) { real a = (i == j) ? Hk[4 + i] : 0.0; for (int m = 0; m < 4; ++m) a += B[m * 2 + i] * PB[m * 2 + j]; Rt[i * 2 + j] = a; }
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 4; ++j) { real a = 0; for (int m = 0; m < 4; ++m) a += B[m * 2 + i] * PA[m * 4 + j]; St[i * 4 + j] = a; }
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) { real a = (i == j) ? Hk[i] : 0.0; for (int m = 0; m < 4; ++m) a += A[m * 4 + i] * PA[m * 4 + j]; Qt[i * 4 + j] = a; }
            /* symmetrise the 2x2 before inversion */
            real rs = 0.5 * (Rt[1] + Rt[2]); Rt[1] = Rt[2] = rs;
            inv2(Rt, F->Ri[k]);
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 4; ++j) F->K[k][i * 4 + j] = -(F->Ri[k][i * 2 + 0] * St[0 * 4 + j] + F->Ri[k][i * 2 + 1] * St[1 * 4 + j]);
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) P[i * 4 + j] = Qt[i * 4 + j] + St[0 * 4 + i] * F->K[k][0 * 4 + j] + St[1 * 4 + i] * F->K[k][1 * 4 + j];
            for (int i = 0; i < 4; ++i)
                for (int j = i + 1; j < 4; ++j) { real s = 0.5 * (P[i * 4 + j] + P[j * 4 + i]); P[i * 4 + j] = P[j * 4 + i] = s; }
        }
        for (int i = 0; i < 2; ++i) F->kk[k][i] = -(F->Ri[k][i * 2 + 0] * rt[0] + F->Ri[k][i * 2 + 1] * rt[1]);
        for (int i = 0; i < 4; ++i) p[i] = qt[i] + F->K[k][0 * 4 + i] * rt[0] + F->K[k][1 * 4 + i] * rt[1];
    }
    /* forward */
    real x[4];
    memcpy(x, qp->dx0, sizeof x);
    memcpy(dx, x, sizeof x);
    for (int k = 0; k < N; ++k) {
        const real *A = qp->A + 16 * k, *B = qp->B + 8 * k, *bb = qp->b + 4 * k;
        real u[2];
        for (int i = 0; i < 2; ++i) { real a = F->kk[k][i]; for (int j = 0; j < 4; ++j) a += F->K[k][i * 4 + j] * x[j]; u[i] = a; }
        real xn[4];
        for (int i = 0; i < 4; ++i) {
            real a = bb[i];
            for (int j = 0; j < 4; ++j) a += A[i * 4 + j] * x[j];
            for (int j = 0; j < 2; ++j) a += B[i * 2 + j] * u[j];
            xn[i] = a;
        }
        du[2 * k] = u[0]; du[2 * k + 1] = u[1];
        memcpy(x, xn, sizeof x);
        memcpy(dx + 4 * (k + 1), x, sizeof x);
    }
}

static inline real bnd_val(const real *dx, const real *du, int k, int j)
{
    return j == 0 ? dx[4 * k + 3] : du[2 * k + (j - 1)];
}

/* Mehrotra predictor-corrector IPM.  Returns 0 (stop test met), 1 (non-finite solution),
 * 2 (iteration cap reached first: the last iterate is returned, as HPIPM at iter_max),
 * 3 (infeasible: a fixed bounded component, the stage-0 s = x0's s, lies outside its bounds),
 * 4 (stall exit: the last iterate is returned as at the cap), 5 (diverged: mu reached
 * qp_mu_max or turned non-finite -- a QP failure, acados ACADOS_QP_FAILURE). */
static int qp_solve(const or_qp *qp, const or_opts *o, or_qp_sol *sol, or_fact *F, real *work, int *nit_out)
{
    int N = qp->N;
    real *Hd = work, *gd = work + 6 * N, *dxn = work + 12 * N, *dun = dxn + 4 * (N + 1);
    real *dta = dun + 2 * N, *dla = dta + 6 * N;
    real *t = sol->t, *lam = sol->lam;
    int m = 0;
    /* Bound residual r = v - lo - t (resp. hi - v - t) of the infeasible start: nonzero where
     * the linearisation point is within t_min of a bound or beyond it.  Every update scales
     * all residuals by (1 - alpha), so max|r| = r0 * prod(1 - alpha) exactly. */
    real r0 = 0.0, rscale = 1.0;
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < 3; ++j) {
            for (int sd = 0; sd < 2; ++sd) {
                int q = (k * 3 + j) * 2 + sd;
                if (qp->act[k * 3 + j]) {
                    real d = sd == 0 ? -qp->lo[k * 3 + j] : qp->hi[k * 3 + j];
                    t[q] = d > o->t_min ? d : o->t_min;
                    lam[q] = o->mu0 / t[q];
                    if (t[q] - d > r0) r0 = t[q] - d;
                    m++;
                } else { t[q] = 1.0; lam[q] = 0.0; }
            }
        }
    for (int k = 0; k < N; ++k) { sol->du[2 * k] = 0.0; sol->du[2 * k + 1] = 0.0; }
    static const int comp[3] = {3, 4, 5};
    /* the stage-0 s is fixed (dx_0 = dx0): its bound is a feasibility check, not a variable */
    int infeasible = 0;
    if (qp->act[0]) {
        real v = qp->dx0[3];
        if (v < qp->lo[0] || v > qp->hi[0]) infeasible = 1;
    }
    /* start-point residuals of the stop test (z = 0, pi = 0): stationarity g + C' lam,
     * equality dx0 and the defects b */
    real rg0 = 0.0, rb0 = 0.0;
    for (int k = 0; k < N; ++k) {
        for (int i = 0; i < 6; ++i) {
            real r = qp->g[6 * k + i];
            int j = i == 3 ? 0 : (i >= 4 ? i - 3 : -1);
            if (j >= 0 && qp->act[k * 3 + j]) r += lam[(k * 3 + j) * 2 + 1] - lam[(k * 3 + j) * 2 + 0];
            if (fabs(r) > rg0) rg0 = fabs(r);
        }
        for (int i = 0; i < 4; ++i) if (fabs(qp->b[4 * k + i]) > rb0) rb0 = fabs(qp->b[4 * k + i]);
    }
    for (int i = 0; i < 4; ++i) {
        if (fabs(qp->g[6 * N + i]) > rg0) rg0 = fabs(qp->g[6 * N + i]);
        if (fabs(qp->dx0[i]) > rb0) rb0 = fabs(qp->dx0[i]);
    }

    real rs_stop = o->res_stop / r0;
    if (o->qp_tol_stat / rg0 < rs_stop) rs_stop = o->qp_tol_stat / rg0;
    if (o->qp_tol_eq / rb0 < rs_stop) rs_stop = o->qp_tol_eq / rb0;
    int nit = 0, converged = 0, stall = 0, stalled = 0, diverged = 0;
    for (int it = 0; it <= o->qp_iters && !infeasible; ++it) {
        real mu = 0.0;
        for (int q = 0; q < 6 * N; ++q) mu += t[q] * lam[q];
        mu /= (real)m;
        /* divergence (multipliers growing without bound; a NaN mu would pass the stop test) */
        if (!(mu < o->qp_mu_max)) { diverged = 1; break; }
        /* HPIPM's four exit residuals: complementarity, and the bound, stationarity and equality
         * residuals r0, rg0, rb0 times their common scale prod(1 - alpha) -- tested as
         * prod < min(tol / r) (x / 0 = inf: a residual that starts at zero never binds) */
        if (!(mu >= o->mu_stop) && !(rscale >= rs_stop)) { converged = 1; break; }
        /* the stall exit is tested before the cap, as the kernel's qp_ipm does, so that a QP stalled at
         * the cap counts as stalled in both */
        if (o->qp_stall_iters > 0 && stall >= o->qp_stall_iters) { stalled = 1; break; }   /* as at the cap */
        if (it == o->qp_iters) break;   /* cap reached: tested once more above, no further step */
        nit++;
        for (int pass = 0; pass < 2; ++pass) {
            real sigma_mu = 0.0;
            if (pass == 1) {
                /* affine step length and centering parameter */
                real amax = 1.0;
                for (int q = 0; q < 6 * N; ++q) {
                    if (dta[q] < 0.0) { real a = -t[q] / dta[q]; if (a < amax) amax = a; }
                    if (dla[q] < 0.0) { real a = -lam[q] / dla[q]; if (a < amax) amax = a; }
                }
                real mua = 0.0;
                for (int q = 0; q < 6 * N; ++q) mua += (t[q] + amax * dta[q]) * (lam[q] + amax * dla[q]);
                mua /= (real)m;
                real r = mua / mu;
                real sg = r * r * r;
                if (sg < o->sigma_min) sg = o->sigma_min;
                sigma_mu = sg * mu;
            }
            for (int k = 0; k < N; ++k) {
                for (int i = 0; i < 6; ++i) { Hd[6 * k + i] = qp->H[6 * k + i]; gd[6 * k + i] = qp->g[6 * k + i]; }
                for (int j = 0; j < 3; ++j) {
                    if (!qp->act[k * 3 + j]) continue;
                    int ql = (k * 3 + j) * 2, qh = ql + 1;
                    real sl = lam[ql] / t[ql], sh = lam[qh] / t[qh];
                    real cl = 0.0, ch = 0.0;
                    if (pass == 1) { cl = sigma_mu - dta[ql] * dla[ql]; ch = sigma_mu - dta[qh] * dla[qh]; }
                    Hd[6 * k + comp[j]] += sl + sh;
                    gd[6 * k + comp[j]] += -sl * qp->lo[k * 3 + j] - sh * qp->hi[k * 3 + j]
                                           - lam[ql] + lam[qh] - cl / t[ql] + ch / t[qh];
                }
            }
            riccati(qp, Hd, gd, F, pass == 0, dxn, dun);
            /* slack / multiplier directions */
            for (int k = 0; k < N; ++k)
                for (int j = 0; j < 3; ++j) {
                    int ql = (k * 3 + j) * 2, qh = ql + 1;
                    if (!qp->act[k * 3 + j]) { dta[ql] = dta[qh] = dla[ql] = dla[qh] = 0.0; continue; }
                    real v = bnd_val(dxn, dun, k, j);
                    real sl = lam[ql] / t[ql], sh = lam[qh] / t[qh];
                    real cl = 0.0, ch = 0.0;
                    if (pass == 1) { cl = sigma_mu - dta[ql] * dla[ql]; ch = sigma_mu - dta[qh] * dla[qh]; }
                    real dtl = v - qp->lo[k * 3 + j] - t[ql];
                    real dth = qp->hi[k * 3 + j] - v - t[qh];
                    dta[ql] = dtl; dta[qh] = dth;
                    dla[ql] = cl / t[ql] - lam[ql] - sl * dtl;
                    dla[qh] = ch / t[qh] - lam[qh] - sh * dth;
                }
        }
        /* step length with fraction to boundary */
        real amax = 1.0 / o->frac;
        for (int q = 0; q < 6 * N; ++q) {
            if (dta[q] < 0.0) { real a = -t[q] / dta[q]; if (a < amax) amax = a; }
            if (dla[q] < 0.0) { real a = -lam[q] / dla[q]; if (a < amax) amax = a; }
        }
        real alpha = o->frac * amax;
        if (alpha > 1.0) alpha = 1.0;
        stall = alpha < o->qp_stall_alpha ? stall + 1 : 0;
        rscale *= 1.0 - alpha;
        for (int q = 0; q < 6 * N; ++q) { t[q] += alpha * dta[q]; lam[q] += alpha * dla[q]; }
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < 2; ++i) sol->du[2 * k + i] += alpha * (dun[2 * k + i] - sol->du[2 * k + i]);
    }
    if (nit_out) *nit_out = nit;
    /* final state rollout from the damped controls */
    real x[4];
    memcpy(x, qp->dx0, sizeof x);
    memcpy(sol->dx, x, sizeof x);
    for (int k = 0; k < N; ++k) {
        const real *A = qp->A + 16 * k, *B = qp->B + 8 * k, *bb = qp->b + 4 * k;
        real xn[4];
        for (int i = 0; i < 4; ++i) {
            real a = bb[i];
            for (int j = 0; j < 4; ++j) a += A[i * 4 + j] * x[j];
            for (int j = 0; j < 2; ++j) a += B[i * 2 + j] * sol->du[2 * k + j];
            xn[i] = a;
        }
        memcpy(x, xn, sizeof x);
        memcpy(sol->dx + 4 * (k + 1), x, sizeof x);
    }
    /* dynamics multipliers by the adjoint recursion:
     * pi_{N-1} = We dx_N + g_N ; pi_{k-1} = Hx dx_k + gx_k + A_k' pi_k + (lam_hi - lam_lo)_s */
    real pi[4];
    for (int i = 0; i < 4; ++i) pi[i] = qp->H[6 * N + i] * sol->dx[4 * N + i] + qp->g[6 * N + i];
    memcpy(sol->pi + 4 * (N - 1), pi, sizeof pi);
    for (int k = N - 1; k >= 1; --k) {
        const real *A = qp->A + 16 * k;
        real np[4];
        for (int i = 0; i < 4; ++i) {
            real a = qp->H[6 * k + i] * sol->dx[4 * k + i] + qp->g[6 * k + i];
            for (int j = 0; j < 4; ++j) a += A[j * 4 + i] * pi[j];
            np[i] = a;
        }
        if (qp->act[k * 3 + 0]) np[3] += lam[(k * 3 + 0) * 2 + 1] - lam[(k * 3 + 0) * 2 + 0];
        memcpy(pi, np, sizeof pi);
        memcpy(sol->pi + 4 * (k - 1), pi, sizeof pi);
    }
    if (g_exp & 2) {
        for (int k = 0; k < N; ++k) {
            const real *B = qp->B + 8 * k, *pk = sol->pi + 4 * k;
            for (int i = 0; i < 2; ++i) {
                real r = qp->H[6 * k + 4 + i] * sol->du[2 * k + i] + qp->g[6 * k + 4 + i];
                for (int j = 0; j < 4; ++j) r += B[j * 2 + i] * pk[j];
                const int q = (k * 3 + 1 + i) * 2;
                lam[q + 1] = -r > 0.0 ? -r : 0.0;
                lam[q] = r > 0.0 ? r : 0.0;
            }
        }
    }
    /* a QP whose mu turned non-finite diverged (5, as the kernel's QP_EXIT_DIVERGED, which it tests
     * first): its solution is non-finite too, but it is a QP failure, not a status-1 breakdown */
    if (infeasible) return 3;
    if (diverged) return 5;
    for (int q = 0; q < 4 * (N + 1); ++q) if (!isfinite(sol->dx[q])) return 1;
    for (int q = 0; q < 2 * N; ++q) if (!isfinite(sol->du[q])) return 1;
    return converged ? 0 : (stalled ? 4 : 2);
}

/* ================================================================ SQP */
typedef struct {
    real A[OR_MAX_N * 16], B[OR_MAX_N * 8], b[OR_MAX_N * 4];
    real H[OR_MAX_N * 6 + 4], g[OR_MAX_N * 6 + 4];
    real lo[OR_MAX_N * 3], hi[OR_MAX_N * 3];
    uint8_t act[OR_MAX_N * 3];
    real dx[(OR_MAX_N + 1) * 4], du[OR_MAX_N * 2], pi[OR_MAX_N * 4];
    real lam[OR_MAX_N * 6], t[OR_MAX_N * 6];
    real work[OR_MAX_N * 40 + 64];
    or_fact F;
    int qp_total;
    int qp_capped;   /* QPs of this solve stopped by the iteration cap */
    int qp_stalled;  /* ... by the stall exit */
    uint32_t mode[OR_MAX_N];  /* motion-cone modes of the stages' RK4 evaluations (diagnostics) */
    real kkt[OR_KKT_DIAG];  /* diagnostics of the NLP KKT tests (nlp_mode 1): see or_set_kkt_diag */
} or_ws;

/* KKT diagnostics (nlp_mode 1), per lane OR_KKT_DIAG = 22 doubles: the residuals of the last KKT test the SQP
 * evaluated -- u-stationarity, x-stationarity (stages 1..N-1), terminal stationarity, equality,
 * inequality, complementarity -- then the SQP iteration of that test, the last line-search
 * step length, that line search's directional derivative, merit at alpha = 0 and at the last step
 * tried, the number of line searches that ended at ls_alpha_min; for the last QP its exit code,
 * the term sum r_u' du of its u-stationarity residual r_u, -d'Hd, and sum pi'b - nu|b|; the number
 * of stages whose motion-cone modes (at the four RK4 evaluations) changed between the last two
 * linearisations, and over all linearisations from SQP iteration 10 on; the tolerance margin of
 * the solve's decisions: over every KKT test it evaluated, the smallest |log10 q| with q = max of
 * res_stat/tol_stat, res_eq/tol_eq, res_ineq/tol_ineq, res_comp/tol_comp (q < 1 passes), and the q
 * of that closest test.  A solve whose margin exceeds 1 never had a residual within a factor 10 of
 * its tolerance at any decision; the line searches' margin: over every Armijo test of the solve,
 * the smallest |phi(alpha) - phi0 - eps alpha dphi| / |phi0|, and the SQP iteration of that test (a
 * test whose two sides agree to rounding is decided by rounding).  NULL: off. */
static real *g_kkt_diag = NULL;
OR_EXPORT void or_set_kkt_diag(real *buf) { g_kkt_diag = buf; }


static real ocp_cost(const or_opts *o, int N, const real *X, const real *U, const real *yref, const real *yref_e)
{
    real c = 0.0;
    for (int k = 0; k < N; ++k) {
        real s = 0.0;
        for (int i = 0; i < 4; ++i) { real r = X[4 * k + i] - yref[6 * k + i]; s += o->W[i] * r * r; }
        for (int i = 0; i < 2; ++i) { real r = U[2 * k + i] - yref[6 * k + 4 + i]; s += o->W[4 + i] * r * r; }
        c += 0.5 * o->tau * s;
    }
    real s = 0.0;
    for (int i = 0; i < 4; ++i) { real r = X[4 * N + i] - yref_e[i]; s += o->We[i] * r * r; }
    return c + 0.5 * s;
}

/* Merit function for the line search (l1 exact penalty, Nocedal & Wright 18.2):
 * phi = J + sum_k nu_k' |phi(x_k,u_k) - x_{k+1}| + sum_bounds eta * violation */
static real merit_eval(const or_shape *sh, const or_opts *o, const real *X, const real *U,
                         const real *yref, const real *yref_e, const real *nu, const real *eta)
{
    int N = o->N;
    real phi = ocp_cost(o, N, X, U, yref, yref_e);
    for (int k = 0; k < N; ++k) {
        real xn[4], A[16], B[8];
        rk4_sens(sh, o->Ts, X + 4 * k, U + 2 * k, xn, A, B);
        for (int i = 0; i < 4; ++i) phi += nu[4 * k + i] * fabs(xn[i] - X[4 * (k + 1) + i]);
        real v[3] = {X[4 * k + 3], U[2 * k], U[2 * k + 1]};
        for (int j = (k == 0 && !o->stage0_s_bound ? 1 : 0); j < 3; ++j) {
            real vl = o->lh[j] - v[j], vh = v[j] - o->uh[j];
            if (vl > 0) phi += eta[(3 * k + j) * 2 + 0] * vl;
            if (vh > 0) phi += eta[(3 * k + j) * 2 + 1] * vh;
        }
    }
    return phi;
}

/* SQP from the initial guess (X,U,PI) in place.
 *   nlp_mode 0: K full Gauss-Newton steps (the BASELINE "SQP-RTI, K iterations" metric).
 *   nlp_mode 1: acados-style SQP: KKT residual check against tol_* before each QP,
 *               merit backtracking with sufficient descent (alpha *= ls_alpha_red down
 *               to ls_alpha_min), damped multiplier update, at most sqp_iters QPs.
 * Returns status: 0 ok/converged, 1 NaN/Inf, 2 max iterations (mode 1). */
static int sqp_solve(const or_shape *sh, const or_opts *o, const real x0[4],
                     const real *yref, const real *yref_e,
                     real *X, real *U, real *PI, real *lam_out, int32_t *iters, or_ws *ws)
{
    int N = o->N;
    int status = 0;
    or_qp qp;
    qp.N = N; qp.A = ws->A; qp.B = ws->B; qp.b = ws->b; qp.H = ws->H; qp.g = ws->g;
    qp.lo = ws->lo; qp.hi = ws->hi; qp.act = ws->act;
    or_qp_sol sol = {ws->dx, ws->du, ws->pi, ws->lam, ws->t};
    real LAM[OR_MAX_N * 6];
    real nu[OR_MAX_N * 4], eta[OR_MAX_N * 6];
    real Xt[(OR_MAX_N + 1) * 4], Ut[OR_MAX_N * 2];
    memset(LAM, 0, sizeof(real) * 6 * N);
    memset(nu, 0, sizeof(real) * 4 * N);
    memset(eta, 0, sizeof(real) * 6 * N);
    int it;
    memset(ws->kkt, 0, sizeof ws->kkt);
    ws->kkt[18] = 1e300;
    ws->kkt[20] = 1e300;
    if (o->nlp_mode == 1) status = 2;
    /* stage-0 s bound: s_0 = x0's s is fixed in every QP; outside [lh_s, uh_s] all of them are
     * infeasible and the solve stops before its first iteration (status 4, ACADOS_QP_FAILURE) */
    if (o->stage0_s_bound && !(x0[3] >= o->lh[0] && x0[3] <= o->uh[0])) {
        if (iters) *iters = 0;
        if (lam_out) memset(lam_out, 0, sizeof(real) * 6 * N);
        return 4;
    }
    for (it = 0; it < o->sqp_iters; ++it) {
        ws->kkt[16] = 0.0;
        for (int k = 0; k < N; ++k) {
            real xn[4];
            g_mode_code = 0;
            rk4_sens(sh, o->Ts, X + 4 * k, U + 2 * k, xn, ws->A + 16 * k, ws->B + 8 * k);
            if (it > 0 && g_mode_code != ws->mode[k]) {
                if (it >= 10) ws->kkt[17] += 1.0;
                ws->kkt[16] += 1.0;
            }
            ws->mode[k] = g_mode_code;
            for (int i = 0; i < 4; ++i) ws->b[4 * k + i] = xn[i] - X[4 * (k + 1) + i];
            for (int i = 0; i < 4; ++i) {
                ws->H[6 * k + i] = o->tau * o->W[i];
                ws->g[6 * k + i] = o->tau * o->W[i] * (X[4 * k + i] - yref[6 * k + i]);
            }
            for (int i = 0; i < 2; ++i) {
                ws->H[6 * k + 4 + i] = o->tau * o->W[4 + i];
                ws->g[6 * k + 4 + i] = o->tau * o->W[4 + i] * (U[2 * k + i] - yref[6 * k + 4 + i]);
            }
            real v[3] = {X[4 * k + 3], U[2 * k], U[2 * k + 1]};
            for (int j = 0; j < 3; ++j) {
                ws->lo[3 * k + j] = o->lh[j] - v[j];
                ws->hi[3 * k + j] = o->uh[j] - v[j];
                ws->act[3 * k + j] = (j == 0 && k == 0) ? (uint8_t)(o->stage0_s_bound != 0) : 1;
            }
        }
        for (int i = 0; i < 4; ++i) {
            ws->H[6 * N + i] = o->We[i];
            ws->g[6 * N + i] = o->We[i] * (X[4 * N + i] - yref_e[i]);
            qp.dx0[i] = x0[i] - X[i];
        }
        if (o->nlp_mode == 1) {
            /* KKT residuals of the NLP at the current iterate */
            ws->kkt[2] = 0.0;
            real r_stat = 0.0, r_eq = 0.0, r_ineq = 0.0, r_comp = 0.0, r_u = 0.0, r_x = 0.0;
            for (int k = 0; k < N; ++k) {
                const real *A = ws->A + 16 * k, *B = ws->B + 8 * k, *pk = PI + 4 * k;
                for (int i = 0; i < 2; ++i) {
                    real r = ws->g[6 * k + 4 + i];
                    for (int j = 0; j < 4; ++j) r += B[j * 2 + i] * pk[j];
                    r += LAM[(3 * k + 1 + i) * 2 + 1] - LAM[(3 * k + 1 + i) * 2 + 0];
                    if (fabs(r) > r_stat) r_stat = fabs(r);
                    if (fabs(r) > r_u) r_u = fabs(r);
                }
                if (k >= 1) {
                    for (int i = 0; i < 4; ++i) {
                        real r = ws->g[6 * k + i] - PI[4 * (k - 1) + i];
                        for (int j = 0; j < 4; ++j) r += A[j * 4 + i] * pk[j];
                        if (i == 3) r += LAM[(3 * k) * 2 + 1] - LAM[(3 * k) * 2 + 0];
                        if (fabs(r) > r_stat) r_stat = fabs(r);
                        if (fabs(r) > r_x) r_x = fabs(r);
                    }
                }
                for (int i = 0; i < 4; ++i) if (fabs(ws->b[4 * k + i]) > r_eq) r_eq = fabs(ws->b[4 * k + i]);
                for (int j = (k == 0 && !o->stage0_s_bound ? 1 : 0); j < 3; ++j) {
                    real sl = -ws->lo[3 * k + j], sh_ = ws->hi[3 * k + j];
                    if (-sl > r_ineq) r_ineq = -sl;
                    if (-sh_ > r_ineq) r_ineq = -sh_;
                    real cl = fabs(LAM[(3 * k + j) * 2 + 0] * sl), ch = fabs(LAM[(3 * k + j) * 2 + 1] * sh_);
                    if (cl > r_comp) r_comp = cl;
                    if (ch > r_comp) r_comp = ch;
                }
            }
            for (int i = 0; i < 4; ++i) {
                real r = ws->g[6 * N + i] - PI[4 * (N - 1) + i];
                if (fabs(r) > r_stat) r_stat = fabs(r);
                if (fabs(r) > ws->kkt[2]) ws->kkt[2] = fabs(r);
            }
            ws->kkt[0] = r_u; ws->kkt[1] = r_x; ws->kkt[3] = r_eq; ws->kkt[4] = r_ineq; ws->kkt[5] = r_comp;
            ws->kkt[6] = it;
            {
                real q = r_stat / o->tol_stat;
                if (r_eq / o->tol_eq > q) q = r_eq / o->tol_eq;
                if (r_ineq / o->tol_ineq > q) q = r_ineq / o->tol_ineq;
                if (r_comp / o->tol_comp > q) q = r_comp / o->tol_comp;
                const double qd = (double)q, mg = qd > 0.0 ? (qd >= 1.0 ? log10(qd) : -log10(qd)) : 1e300;
                if (mg < (double)ws->kkt[18]) { ws->kkt[18] = mg; ws->kkt[19] = q; }
            }
            if (r_stat < o->tol_stat && r_eq < o->tol_eq && r_ineq < o->tol_ineq && r_comp < o->tol_comp) {
                status = 0;
                break;
            }
        }
        int nit = 0;
        const int qst = qp_solve(&qp, o, &sol, &ws->F, ws->work, &nit);
        ws->qp_total += nit;
        if (qst == 2) ws->qp_capped++;
        if (qst == 4) ws->qp_stalled++;
        /* non-finite QP solution: status 1; infeasible or diverged QP: status 4 (acados
         * ACADOS_QP_FAILURE); either way the SQP stops with its last finite iterate */
        if (qst == 1 || qst == 3 || qst == 5) { status = qst == 1 ? 1 : 4; break; }
        real alpha = 1.0;
        if (o->nlp_mode == 1) {
            /* merit weights (acados: max(|mult|, (weight + |mult|)/2)) */
            for (int q = 0; q < 4 * N; ++q) {
                real a = fabs(ws->pi[q]);
                real w = 0.5 * (nu[q] + a);
                nu[q] = a > w ? a : w;
            }
            for (int q = 0; q < 6 * N; ++q) {
                real a = fabs(ws->lam[q]);
                real w = 0.5 * (eta[q] + a);
                eta[q] = a > w ? a : w;
            }
            real phi0 = merit_eval(sh, o, X, U, yref, yref_e, nu, eta);
            /* directional derivative  grad J' dw - sum nu|d| - sum eta viol (N&W 18.29) */
            real dphi = 0.0;
            for (int k = 0; k < N; ++k) {
                for (int i = 0; i < 4; ++i) dphi += ws->g[6 * k + i] * ws->dx[4 * k + i];
                for (int i = 0; i < 2; ++i) dphi += ws->g[6 * k + 4 + i] * ws->du[2 * k + i];
                for (int i = 0; i < 4; ++i) dphi -= nu[4 * k + i] * fabs(ws->b[4 * k + i]);
                for (int j = (k == 0 && !o->stage0_s_bound ? 1 : 0); j < 3; ++j) {
                    if (ws->lo[3 * k + j] > 0) dphi -= eta[(3 * k + j) * 2 + 0] * ws->lo[3 * k + j];
                    if (ws->hi[3 * k + j] < 0) dphi -= eta[(3 * k + j) * 2 + 1] * (-ws->hi[3 * k + j]);
                }
            }
            for (int i = 0; i < 4; ++i) dphi += ws->g[6 * N + i] * ws->dx[4 * N + i];
            ws->kkt[8] = dphi;
            ws->kkt[9] = phi0;
            {
                real ru = 0.0, dhd = 0.0, pb = 0.0;
                for (int k = 0; k < N; ++k) {
                    const real *Bk = ws->B + 8 * k, *pk = ws->pi + 4 * k;
                    for (int i = 0; i < 2; ++i) {
                        real r = ws->H[6 * k + 4 + i] * ws->du[2 * k + i] + ws->g[6 * k + 4 + i];
                        for (int j = 0; j < 4; ++j) r += Bk[j * 2 + i] * pk[j];
                        r += ws->lam[(k * 3 + 1 + i) * 2 + 1] - ws->lam[(k * 3 + 1 + i) * 2 + 0];
                        ru += r * ws->du[2 * k + i];
                        dhd -= ws->H[6 * k + 4 + i] * ws->du[2 * k + i] * ws->du[2 * k + i];
                    }
                    for (int i = 0; i < 4; ++i) {
                        dhd -= ws->H[6 * k + i] * ws->dx[4 * k + i] * ws->dx[4 * k + i];
                        pb += pk[i] * ws->b[4 * k + i] - nu[4 * k + i] * fabs(ws->b[4 * k + i]);
                    }
                }
                for (int i = 0; i < 4; ++i) dhd -= ws->H[6 * N + i] * ws->dx[4 * N + i] * ws->dx[4 * N + i];
                ws->kkt[12] = qst; ws->kkt[13] = ru; ws->kkt[14] = dhd; ws->kkt[15] = pb;
            }
            for (;;) {
                for (int q = 0; q < 4 * (N + 1); ++q) Xt[q] = X[q] + alpha * ws->dx[q];
                for (int q = 0; q < 2 * N; ++q) Ut[q] = U[q] + alpha * ws->du[q];
                real phi = merit_eval(sh, o, Xt, Ut, yref, yref_e, nu, eta);
                ws->kkt[10] = phi;
                {
                    const real gap = phi - (phi0 + o->ls_eps * alpha * dphi);
                    const double rel = (double)(fabs(gap) / (fabs(phi0) > 1e-300 ? fabs(phi0) : 1e-300));
                    if (rel < (double)ws->kkt[20]) { ws->kkt[20] = rel; ws->kkt[21] = it; }
                }
                if (phi <= phi0 + o->ls_eps * alpha * dphi) break;
                real an = alpha * o->ls_alpha_red;
                if (an < ((g_exp & 4) ? 1e-12 : o->ls_alpha_min)) { ws->kkt[11] += 1.0; break; }   /* accept the last step tried */
                alpha = an;
            }
            ws->kkt[7] = alpha;
        }
        for (int q = 0; q < 4 * (N + 1); ++q) X[q] += alpha * ws->dx[q];
        for (int q = 0; q < 2 * N; ++q) U[q] += alpha * ws->du[q];
        const real ad = (g_exp & 1) ? 1.0 : alpha;
        for (int q = 0; q < 4 * N; ++q) PI[q] += ad * (ws->pi[q] - PI[q]);
        for (int q = 0; q < 6 * N; ++q) LAM[q] += ad * (ws->lam[q] - LAM[q]);
    }
    if (iters) *iters = it;
    if (lam_out) memcpy(lam_out, LAM, sizeof(real) * 6 * N);
    for (int q = 0; q < 4 * (N + 1); ++q) if (!isfinite(X[q])) status = 1;
    for (int q = 0; q < 2 * N; ++q) if (!isfinite(U[q])) status = 1;
    return status;
}

/* ================================================================ exported API */
static void make_shape(or_shape *sh, const int32_t *n_ctrl, const real *ctrl, const real *knots,
                       const real *params /* [b, c, mu] per shape */, int id, int max_ctrl)
{
    sh->n = n_ctrl[id];
    sh->P = ctrl + (size_t)id * max_ctrl * 2;
    sh->S = knots + (size_t)id * (max_ctrl + 4);
    sh->b = params[3 * id + 0];
    sh->c = params[3 * id + 1];
    sh->mu = params[3 * id + 2];
}

/* shape table layout shared by every entry point:
 *   n_ctrl[n_shapes], ctrl[n_shapes][max_ctrl][2], knots[n_shapes][max_ctrl+4],
 *   params[n_shapes][3] = {b, c_ellipse, mu_sp} */

OR_EXPORT int or_spline_eval(const int32_t *n_ctrl, const real *ctrl, const real *knots, const real *params,
                   int max_ctrl, int32_t n, const int32_t *shape_id, const real *s,
                   real *C, real *dC, real *D, real *dD, real *kappa)
{
    for (int32_t i = 0; i < n; ++i) {
        or_shape sh; make_shape(&sh, n_ctrl, ctrl, knots, params, shape_id[i], max_ctrl);
        spline_C(&sh, s[i], C + 2 * i, dC + 2 * i);
        spline_Cdot(&sh, s[i], D + 2 * i, dD + 2 * i);
        kappa[i] = angle_rate(&sh, s[i]);
    }
    return 0;
}

OR_EXPORT int or_dynamics(const int32_t *n_ctrl, const real *ctrl, const real *knots, const real *params,
                int max_ctrl, int32_t n, const int32_t *shape_id, const real *x, const real *u,
                real *f, real *J)
{
    #pragma omp parallel for schedule(static)
    for (int32_t i = 0; i < n; ++i) {
        or_shape sh; make_shape(&sh, n_ctrl, ctrl, knots, params, shape_id[i], max_ctrl);
        dynamics(&sh, x + 4 * i, u + 2 * i, f + 4 * i, J ? J + 24 * i : NULL);
    }
    return 0;
}

OR_EXPORT int or_rk4(const int32_t *n_ctrl, const real *ctrl, const real *knots, const real *params,
           int max_ctrl, int32_t n, const int32_t *shape_id, real h, const real *x, const real *u,
           real *xn, real *A, real *B)
{
    g_probe_eps = 0.0;
    #pragma omp parallel for schedule(static)
    for (int32_t i = 0; i < n; ++i) {
        or_shape sh; make_shape(&sh, n_ctrl, ctrl, knots, params, shape_id[i], max_ctrl);
        rk4_sens(&sh, h, x + 4 * i, u + 2 * i, xn + 4 * i, A + 16 * i, B + 8 * i);
    }
    return 0;
}

OR_EXPORT int or_vbound(const int32_t *n_ctrl, const real *ctrl, const real *knots, const real *params,
              int max_ctrl, const or_opts *o, int32_t n, const int32_t *shape_id, const real *s, real *vb)
{
    for (int32_t i = 0; i < n; ++i) {
        or_shape sh; make_shape(&sh, n_ctrl, ctrl, knots, params, shape_id[i], max_ctrl);
        vb[i] = v_bound(&sh, o, s[i]);
    }
    return 0;
}

/* Batched QP solve (for QP-level parity).  Per lane: A (N x16), B (N x 8), b (N x 4),
 * H (6N+4), g (6N+4), lo/hi (N x 3), act (N x 3), dx0 (4).
 * Outputs dx ((N+1)x4), du (N x 2), pi (N x 4), lam (N x 6). */
OR_EXPORT int or_qp_batch(const or_opts *o, int32_t nb, const real *A, const real *B, const real *b,
                const real *H, const real *g, const real *lo, const real *hi, const uint8_t *act,
                const real *dx0, real *dx, real *du, real *pi, real *lam, int32_t *iters,
                int32_t *qp_status /* optional: 0 converged, 1 non-finite, 2 capped, 3 infeasible */)
{
    int N = o->N;
    if (N > OR_MAX_N) return -1;
    int fail = 0;
    #pragma omp parallel
    {
        or_ws *ws = (or_ws *)malloc(sizeof(or_ws));
        #pragma omp for schedule(dynamic, 4)
        for (int32_t i = 0; i < nb; ++i) {
            or_qp qp;
            qp.N = N;
            qp.A = A + (size_t)i * 16 * N; qp.B = B + (size_t)i * 8 * N; qp.b = b + (size_t)i * 4 * N;
            qp.H = H + (size_t)i * (6 * N + 4); qp.g = g + (size_t)i * (6 * N + 4);
            qp.lo = lo + (size_t)i * 3 * N; qp.hi = hi + (size_t)i * 3 * N; qp.act = act + (size_t)i * 3 * N;
            memcpy(qp.dx0, dx0 + 4 * i, sizeof qp.dx0);
            or_qp_sol sol = {dx + (size_t)i * 4 * (N + 1), du + (size_t)i * 2 * N, pi + (size_t)i * 4 * N,
                             lam + (size_t)i * 6 * N, ws->t};
            const int st = qp_solve(&qp, o, &sol, &ws->F, ws->work, iters ? iters + i : NULL);
            if (qp_status) qp_status[i] = st;
            if (st == 1) {
                #pragma omp atomic write
                fail = 1;
            }
        }
        free(ws);
    }
    return fail;
}

/* Batched OCP solve (acados ocp.solve() level): initial guess X,U,PI in/out.
 * x0: B x 4, yref: B x N x 6, yref_e: B x 4, X: B x (N+1) x 4, U: B x N x 2, PI: B x N x 4.
 * status, cost: B. */
OR_EXPORT int or_ocp_solve(const int32_t *n_ctrl, const real *ctrl, const real *knots, const real *params,
                 int max_ctrl, const or_opts *o, int32_t nb, const int32_t *shape_id,
                 const real *x0, const real *yref, const real *yref_e,
                 real *X, real *U, real *PI, real *lam, int32_t *status, int32_t *iters, int32_t *qp_iter,
                 real *cost, int nthreads, int32_t *qp_capped, int32_t *qp_stalled)
{
    g_probe_eps = o->model_probe;
    g_probe_seed = (uint64_t)(uint32_t)o->probe_seed;
    int N = o->N;
    if (N > OR_MAX_N) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    #pragma omp parallel
    {
        or_ws *ws = (or_ws *)malloc(sizeof(or_ws));
        #pragma omp for schedule(dynamic, 1)
        for (int32_t i = 0; i < nb; ++i) {
            or_shape sh; make_shape(&sh, n_ctrl, ctrl, knots, params, shape_id[i], max_ctrl);
            real *Xi = X + (size_t)i * 4 * (N + 1), *Ui = U + (size_t)i * 2 * N, *Pi = PI + (size_t)i * 4 * N;
            const real *yr = yref + (size_t)i * 6 * N, *ye = yref_e + (size_t)i * 4;
            ws->qp_total = 0;
            ws->qp_capped = 0;
            ws->qp_stalled = 0;
            status[i] = sqp_solve(&sh, o, x0 + 4 * i, yr, ye, Xi, Ui, Pi, lam ? lam + (size_t)i * 6 * N : NULL, iters ? iters + i : NULL, ws);
            if (qp_iter) qp_iter[i] = ws->qp_total;
            if (qp_capped) qp_capped[i] = ws->qp_capped;
            if (qp_stalled) qp_stalled[i] = ws->qp_stalled;
            if (g_kkt_diag) memcpy(g_kkt_diag + (size_t)OR_KKT_DIAG * i, ws->kkt, sizeof ws->kkt);
            cost[i] = ocp_cost(o, N, Xi, Ui, yr, ye);
        }
        free(ws);
    }
    return 0;
}

/* Column c (1-based) of the controller's reference table as set_reference_trajectory builds it
 * (NMPC_controller.m:425-431): D = delay_buff_comp zero columns prepended to the T columns of
 * traj, whose u_t-reference row (6) copies the first real column; get_y_ref (:307-313) clamps
 * an index past the end to the last column. */
static void ref_column(const real *traj, int32_t T, int32_t D, int c, real out[6])
{
    if (c > T + D) c = T + D;
    if (c < 1) c = 1;
    if (c <= D) {
        for (int q = 0; q < 5; ++q) out[q] = 0.0;
        out[5] = traj[5];
    } else {
        for (int q = 0; q < 6; ++q) out[q] = traj[(size_t)(c - D - 1) * 6 + q];
    }
}

/* One NMPC_controller.solve(x0, index_time) (NMPC_controller.m:329-423) on one lane.  Warm start
 * X/U/PI + warm_valid in/out (shifted on return, :397-399); returns the status; u0 = U(:,1) of the
 * unshifted solution (:403). */
static int ctrl_solve_lane(const or_shape *sh, const or_opts *o, const real x0_in[4], const real *traj,
                           int32_t T, int32_t D, int32_t index_time, real *X, real *U, real *PI,
                           uint8_t *warm_valid, real u0[2], int32_t *iters, int32_t *qp_iter, int32_t *qp_capped,
                           real *cost, or_ws *ws, int32_t *qp_stalled)
{
    int N = o->N;
    if (N < 1 || N > OR_MAX_N) return 1;
    real yref[OR_MAX_N * 6], ye[4];
    real x0[4];
    memcpy(x0, x0_in, sizeof x0);
    /* :332 pre-wrap of s into [-b, b) */
    x0[3] = mat_mod(x0[3], sh->b) - sh->b * (x0[3] < 0.0 ? 1.0 : 0.0);
    /* :343-348 reference staging with clamp (get_y_ref :307-313) */
    for (int k = 0; k < N; ++k) ref_column(traj, T, D, index_time + k, yref + 6 * k);
    for (int c = 0; c < 4; ++c) ye[c] = yref[6 * (N - 1) + c];
    /* :351-355 cold start */
    if (!*warm_valid) {
        for (int q = 0; q < 4 * (N + 1); ++q) X[q] = 0.0;
        for (int k = 0; k < N; ++k) { U[2 * k] = o->u_n_lb; U[2 * k + 1] = 0.0; }
        for (int q = 0; q < 4 * N; ++q) PI[q] = 0.0;
    }
    /* :357-364 clip first control */
    real vb = v_bound(sh, o, x0[3]);
    if (fabs(U[1]) > vb) {
        real ut_old = U[1];
        U[1] = (ut_old > 0 ? 1.0 : (ut_old < 0 ? -1.0 : 0.0)) * vb;
        U[0] = U[1] * U[0] / ut_old;
    }
    /* :366-380 Euler warm-start rollout with per-stage clip */
    memcpy(X, x0, sizeof x0);
    for (int j = 1; j <= N; ++j) {
        real f[4];
        dynamics(sh, X + 4 * (j - 1), U + 2 * (j - 1), f, NULL);
        for (int c = 0; c < 4; ++c) X[4 * j + c] = X[4 * (j - 1) + c] + o->Ts * f[c];
        vb = v_bound(sh, o, X[4 * j + 3]);
        if (j == N) break;
        if (fabs(U[2 * j + 1]) > vb) {
            real ut_old = U[2 * j + 1];
            U[2 * j + 1] = (ut_old > 0 ? 1.0 : (ut_old < 0 ? -1.0 : 0.0)) * vb;
            U[2 * j] = U[2 * j + 1] * U[2 * j] / ut_old;
        }
    }
    /* :389 solve */
    ws->qp_total = 0;
    ws->qp_capped = 0;
    ws->qp_stalled = 0;
    int status = sqp_solve(sh, o, x0, yref, ye, X, U, PI, NULL, iters, ws);
    if (qp_iter) *qp_iter = ws->qp_total;
    if (qp_capped) *qp_capped = ws->qp_capped;
    if (qp_stalled) *qp_stalled = ws->qp_stalled;
    if (cost) *cost = ocp_cost(o, N, X, U, yref, ye);
    u0[0] = U[0]; u0[1] = U[1];
    /* :397-399 shift (duplicate last column) */
    memmove(U, U + 2, sizeof(real) * 2 * (N - 1));
    memmove(X, X + 4, sizeof(real) * 4 * N);
    memmove(PI, PI + 4, sizeof(real) * 4 * (N - 1));
    *warm_valid = 1;
    return status;
}

/* Batched NMPC_controller.solve(x0, index_time) (NMPC_controller.m:329-423).
 * traj: T x 6 reference table (column k = y_ref(:,k+1)), shared by all lanes; delay_cols = the
 * controller's delay_buff_comp (the table as set_reference_trajectory prepends it).
 * index_time: B (1-based, as in MATLAB).  Warm start Xw/Uw/PIw: B x ... in/out,
 * warm_valid: B flags (0 = cold start, :351-355); on return they hold the SHIFTED
 * solution (:397-399) and warm_valid = 1.  u0: B x 2 (the unshifted U(:,1), :403). */
OR_EXPORT int or_controller_solve(const int32_t *n_ctrl, const real *ctrl, const real *knots, const real *params,
                        int max_ctrl, const or_opts *o, int32_t nb, const int32_t *shape_id,
                        const real *x0_in, const real *traj, int32_t T, const int32_t *index_time,
                        real *Xw, real *Uw, real *PIw, uint8_t *warm_valid,
                        real *u0, int32_t *status, int32_t *iters, int32_t *qp_iter, real *cost, int nthreads,
                        int32_t *qp_capped, int32_t delay_cols, int32_t *qp_stalled)
{
    g_probe_eps = o->model_probe;
    g_probe_seed = (uint64_t)(uint32_t)o->probe_seed;
    int N = o->N;
    if (N > OR_MAX_N) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    #pragma omp parallel
    {
        or_ws *ws = (or_ws *)malloc(sizeof(or_ws));
        #pragma omp for schedule(dynamic, 1)
        for (int32_t i = 0; i < nb; ++i) {
            or_shape sh; make_shape(&sh, n_ctrl, ctrl, knots, params, shape_id[i], max_ctrl);
            status[i] = ctrl_solve_lane(&sh, o, x0_in + 4 * i, traj, T, delay_cols, index_time[i],
                                        Xw + (size_t)i * 4 * (N + 1), Uw + (size_t)i * 2 * N, PIw + (size_t)i * 4 * N,
                                        warm_valid + i, u0 + 2 * i, iters ? iters + i : NULL, qp_iter ? qp_iter + i : NULL,
                                        qp_capped ? qp_capped + i : NULL, cost + i, ws, qp_stalled ? qp_stalled + i : NULL);
            if (g_kkt_diag) memcpy(g_kkt_diag + (size_t)OR_KKT_DIAG * i, ws->kkt, sizeof ws->kkt);
        }
        free(ws);
    }
    return 0;
}

/* Contact re-projection after a lateral disturbance (helper.m:221-236): s minimising
 * |C(s) - p|^2, p = (-xwidth/2, C_y(s_x) - amplitude), started from s0 (fminunc in the
 * reference, whose iterates cannot be reproduced: restated as a damped Newton iteration on the
 * periodic spline, C evaluated at the floor-mod of s as evalSpline does, bspline_shape.m:192-199;
 * it converges to the local minimum of the start point's basin). */
static real phi_contact(const or_shape *sh, real s, real px, real py)
{
    real C[2], dC[2];
    spline_C(sh, mat_mod(s, sh->b), C, dC);
    return (C[0] - px) * (C[0] - px) + (C[1] - py) * (C[1] - py);
}

static real reproject_contact(const or_shape *sh, real px, real py, real s0)
{
    real s = s0, phi = phi_contact(sh, s, px, py);
    for (int it = 0; it < 60; ++it) {
        real C[2], dC[2], D[2], dD[2];
        const real sw = mat_mod(s, sh->b);
        spline_C(sh, sw, C, dC);
        spline_Cdot(sh, sw, D, dD);
        const real ex = C[0] - px, ey = C[1] - py;
        const real g = 2.0 * (ex * dC[0] + ey * dC[1]);
        const real h = 2.0 * (dC[0] * dC[0] + dC[1] * dC[1] + ex * dD[0] + ey * dD[1]);
        if (fabs(g) < 1e-14) break;
        real step = h > 0.0 ? -g / h : (g > 0.0 ? -0.05 : 0.05) * sh->b;
        const real smax = 0.25 * sh->b;
        if (step > smax) step = smax;
        if (step < -smax) step = -smax;
        int ok = 0;
        real sn = s, phin = phi;
        for (int k = 0; k < 60; ++k) {
            sn = s + step;
            phin = phi_contact(sh, sn, px, py);
            if (phin < phi) { ok = 1; break; }
            step *= 0.5;
        }
        if (!ok) break;
        s = sn;
        phi = phin;
        if (fabs(step) < 1e-13 * sh->b) break;
    }
    return s;
}

/* Batched closed loop of helper.m:195-322 (closed_loop_matlab) with NMPC_controller.solve:
 * per step i = 1..n_steps: (disturbance at i == dist_step: y += amplitude, contact re-projected),
 * sim_noise, the controller's delay prediction (delay_buffer_sim, NMPC_controller.m:112-120:
 * delay_cols Euler steps with the buffered inputs, oldest first), u = solve(x_sim, index0 + i - 1 +
 * delay_cols), the controller buffer push, then the plant x += Ts f(x, u) -- with plant_delay_cols
 * > 0 the plant applies its buffered input (helper.m:289-296).  Cold start; both buffers start at
 * zero.  Outputs: Xtraj nb x (n+1) x 4 (states after disturbance and noise), Xsim nb x n x 4 (the
 * predicted states handed to the solver; optional), Utraj nb x n x 2, Straj nb x n (status). */
OR_EXPORT int or_closed_loop(const int32_t *n_ctrl, const real *ctrl, const real *knots, const real *params,
                   int max_ctrl, const or_opts *o, int32_t nb, const int32_t *shape_id, const real *x0_in,
                   const real *traj, int32_t T, const int32_t *index0, int32_t n_steps, const real *noise,
                   int32_t delay_cols, int32_t plant_delay_cols, int32_t dist_step, const real *dist_amp,
                   const real *xwidth, real *Xtraj, real *Xsim, real *Utraj, int32_t *Straj, int nthreads)
{
    g_probe_eps = o->model_probe;
    g_probe_seed = (uint64_t)(uint32_t)o->probe_seed;
    int N = o->N;
    if (N > OR_MAX_N || delay_cols < 0 || plant_delay_cols < 0 || delay_cols > 1024 || plant_delay_cols > 1024) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    #pragma omp parallel
    {
        or_ws *ws = (or_ws *)malloc(sizeof(or_ws));
        real *X = (real *)malloc(sizeof(real) * 4 * (N + 1)), *U = (real *)malloc(sizeof(real) * 2 * N);
        real *PI = (real *)malloc(sizeof(real) * 4 * N);
        real *ubc = (real *)calloc(2 * (size_t)(delay_cols + 1), sizeof(real));
        real *ubp = (real *)calloc(2 * (size_t)(plant_delay_cols + 1), sizeof(real));
        #pragma omp for schedule(dynamic, 1)
        for (int32_t i = 0; i < nb; ++i) {
            or_shape sh; make_shape(&sh, n_ctrl, ctrl, knots, params, shape_id[i], max_ctrl);
            uint8_t valid = 0;
            memset(ubc, 0, sizeof(real) * 2 * (size_t)(delay_cols + 1));
            memset(ubp, 0, sizeof(real) * 2 * (size_t)(plant_delay_cols + 1));
            real x[4];
            memcpy(x, x0_in + 4 * i, sizeof x);
            real s0_spline = 0.0;
            for (int32_t t = 0; t < n_steps; ++t) {
                if (dist_step > 0 && t + 1 == dist_step) {
                    x[1] += dist_amp[i];
                    real C[2], dC[2];
                    spline_C(&sh, mat_mod(x[3], sh.b), C, dC);
                    const real s = reproject_contact(&sh, -0.5 * xwidth[shape_id[i]], C[1] - dist_amp[i], s0_spline);
                    s0_spline = mat_mod(s, sh.b) - sh.b * (s < 0.0 ? 1.0 : 0.0);
                    x[3] = s0_spline;
                }
                if (noise)
                    for (int c = 0; c < 4; ++c) x[c] += noise[((size_t)t * nb + i) * 4 + c];
                memcpy(Xtraj + ((size_t)i * (n_steps + 1) + t) * 4, x, sizeof x);
                real xs[4];
                memcpy(xs, x, sizeof xs);
                for (int k = 1; k <= delay_cols; ++k) {       /* u_buff_contr(:, end-k+1): oldest first */
                    real f[4];
                    dynamics(&sh, xs, ubc + 2 * (delay_cols - k), f, NULL);
                    for (int c = 0; c < 4; ++c) xs[c] += o->Ts * f[c];
                }
                if (Xsim) memcpy(Xsim + ((size_t)i * n_steps + t) * 4, xs, sizeof xs);
                real u[2];
                const int st = ctrl_solve_lane(&sh, o, xs, traj, T, delay_cols, index0[i] + t + delay_cols, X, U, PI,
                                               &valid, u, NULL, NULL, NULL, NULL, ws, NULL);
                if (delay_cols > 0) {                         /* u_buff_contr = [u, u_buff_contr(:, 1:end-1)] */
                    memmove(ubc + 2, ubc, sizeof(real) * 2 * (size_t)(delay_cols - 1));
                    ubc[0] = u[0]; ubc[1] = u[1];
                }
                memcpy(Utraj + ((size_t)i * n_steps + t) * 2, u, sizeof u);
                if (Straj) Straj[(size_t)i * n_steps + t] = st;
                real f[4];
                if (plant_delay_cols == 0) {
                    dynamics(&sh, x, u, f, NULL);
                } else {                                      /* u_buff_plant(:, end), then push */
                    dynamics(&sh, x, ubp + 2 * (plant_delay_cols - 1), f, NULL);
                    memmove(ubp + 2, ubp, sizeof(real) * 2 * (size_t)(plant_delay_cols - 1));
                    ubp[0] = u[0]; ubp[1] = u[1];
                }
                for (int c = 0; c < 4; ++c) x[c] += o->Ts * f[c];
            }
            memcpy(Xtraj + ((size_t)i * (n_steps + 1) + n_steps) * 4, x, sizeof x);
        }
        free(ws); free(X); free(U); free(PI); free(ubc); free(ubp);
    }
    return 0;
}

/* contact re-projection alone (building block for the tests) */
OR_EXPORT int or_reproject_contact(const int32_t *n_ctrl, const real *ctrl, const real *knots, const real *params,
                         int max_ctrl, int32_t n, const int32_t *shape_id, const real *px, const real *py,
                         const real *s0, real *s)
{
    for (int32_t i = 0; i < n; ++i) {
        or_shape sh; make_shape(&sh, n_ctrl, ctrl, knots, params, shape_id[i], max_ctrl);
        s[i] = reproject_contact(&sh, px[i], py[i], s0[i]);
    }
    return 0;
}

OR_EXPORT int or_max_n(void) { return OR_MAX_N; }

#ifdef OR_EXT
/* orx_controller_solve: or_controller_solve in the extended scalar type, double in/out (inputs
 * converted exactly; outputs rounded once).  Shapes: n_shapes entries of the usual table layout.
 * No model probe, no diagnostics. */
#if OR_EXT == 2
#define ORX_NAME orx_controller_solve_q
#else
#define ORX_NAME orx_controller_solve_l
#endif
static real *to_real(const double *a, size_t n)
{
    real *r = (real *)malloc(sizeof(real) * (n ? n : 1));
    for (size_t i = 0; i < n; ++i) r[i] = a[i];
    return r;
}
static void from_real(double *a, const real *r, size_t n) { for (size_t i = 0; i < n; ++i) a[i] = (double)r[i]; }

int ORX_NAME(const int32_t *n_ctrl, const double *ctrl, const double *knots, const double *params, int max_ctrl,
             int32_t n_shapes, const or_opts *o, int32_t nb, const int32_t *shape_id, const double *x0_in,
             const double *traj, int32_t T, const int32_t *index_time, double *Xw, double *Uw, double *PIw,
             uint8_t *warm_valid, double *u0, int32_t *status, int32_t *iters, int32_t *qp_iter, double *cost,
             int nthreads, int32_t delay_cols)
{
    if (o->model_probe != 0.0) return -1;
    const int N = o->N;
    const size_t ns = (size_t)n_shapes, nbs = (size_t)nb;
    real *c = to_real(ctrl, ns * max_ctrl * 2), *k = to_real(knots, ns * (max_ctrl + 4)), *pr = to_real(params, ns * 3);
    real *x0 = to_real(x0_in, nbs * 4), *tr = to_real(traj, (size_t)T * 6);
    real *X = to_real(Xw, nbs * 4 * (N + 1)), *U = to_real(Uw, nbs * 2 * N), *P = to_real(PIw, nbs * 4 * N);
    real *u = (real *)calloc(nbs * 2 + 1, sizeof(real)), *cs = (real *)calloc(nbs + 1, sizeof(real));
    const int r = or_controller_solve(n_ctrl, c, k, pr, max_ctrl, o, nb, shape_id, x0, tr, T, index_time, X, U, P,
                                      warm_valid, u, status, iters, qp_iter, cs, nthreads, NULL, delay_cols, NULL);
    from_real(Xw, X, nbs * 4 * (N + 1));
    from_real(Uw, U, nbs * 2 * N);
    from_real(PIw, P, nbs * 4 * N);
    from_real(u0, u, nbs * 2);
    from_real(cost, cs, nbs);
    free(c); free(k); free(pr); free(x0); free(tr); free(X); free(U); free(P); free(u); free(cs);
    return r;
}
#endif
