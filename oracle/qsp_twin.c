/*
 * qsp_twin.c — the CPU oracle's kernel-order twin.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker; the product (uclv_qs_pushing_matlab_amd/) never
 * links or calls it.
 *
 * PARITY STATUS: UNPINNED against acados/CasADi/HPIPM (not runnable here), as
 * qsp_oracle.c.  This file restates the same reference path as qsp_oracle.c -- the B-spline contour
 * (acados_nmpc/bspline_shape.m:40-116, 137-152), the motion-cone dynamics
 * (PusherSliderModel.m:503-603), ERK/RK4 with sensitivities (NMPC_controller.m:272), the linear-LS
 * OCP with bgh bounds (NMPC_controller.m:174-268), the Mehrotra interior point standing in for
 * HPIPM (:272-276), fixed-K and merit-backtracking SQP (:271-276), the NMPC_controller.solve
 * wrapper (:329-423) and helper.closed_loop_matlab (helper.m:195-322) -- but evaluates it in the
 * device library's formulation and operation order: span-based de Boor and the hand-derived
 * Jacobian, the structured Riccati step with its closed-loop walks, the lane-group reductions'
 * summation tree, every fused multiply-add as an explicit fma() (the library is built with
 * -ffp-contract=off, this file too).  The operations are IEEE-exact on both sides (checked on the
 * device by scripts/ubench/fp_exact.hip), so this twin reproduces the library's results BIT FOR
 * BIT, lane by lane, including lanes where the fixed-K SQP is chaotic.  qsp_oracle.c's literal
 * restatement (full basis sum, AD) pins this formulation's building blocks to rounding level
 * (tests/test_oracle.py); the twin pins the device's execution of it exactly.
 * Kernel counterparts are cited as qsp_math.hpp / qsp_solver.hip function names.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "or_opts.h"

#define TW_MAX_N 128
#define TW_MAX_SLOTS (TW_MAX_N + 2)
#define TW_MAX_CTRL 64

static inline double qfma(double a, double b, double c) { return fma(a, b, c); }

/* rcp (qsp_fp.hpp): the device refines its hardware reciprocal by two Newton steps, which lands on
 * the correctly rounded 1/x; the same two steps from 1.0 / x give the same bits (also for 0, inf) */
static inline double rcp(double x)
{
    double r = 1.0 / x;
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

/* sin_cos (qsp_fp.hpp): fdlibm reduction + kernels, the library's own sequence */
static void sin_cos(double x, double *sp, double *cp)
{
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_2 = 6.07710050630396597660e-11;
    const double pio2_2t = 2.02226624879595063154e-21;
    const double fn = rint(x * invpio2);
    double r = x - fn * pio2_1;
    double w = fn * pio2_2;
    const double t = r;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    const double y = r - w;
    const double yy = (r - y) - w;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = y * y, zz = z * z;
    const double rs = S2 + z * (S3 + z * S4) + z * zz * (S5 + z * S6);
    const double v = z * y;
    const double ks = y - ((z * (0.5 * yy - v * rs) - yy) - v * S1);
    const double rc = z * (C1 + z * (C2 + z * C3)) + zz * zz * (C4 + z * (C5 + z * C6));
    const double hz = 0.5 * z, wc = 1.0 - hz;
    const double kc = wc + (((1.0 - wc) - hz) + (z * rc - y * yy));
    const double q = fn - 4.0 * floor(fn * 0.25);
    const int q1 = q == 1.0, q2 = q == 2.0, q3 = q == 3.0;
    *sp = q1 ? kc : (q2 ? -ks : (q3 ? -kc : ks));
    *cp = q1 ? -ks : (q2 ? -kc : (q3 ? ks : kc));
}

/* ------------------------------------------------------------------ shapes (qsp_set_shapes) */
typedef struct {
    int n;
    double b, c, mu, inv_h, xwidth;
    double knots[TW_MAX_CTRL + 4], ctrl[2 * TW_MAX_CTRL], dctrl[2 * TW_MAX_CTRL], ddctrl[2 * TW_MAX_CTRL];
} tw_shape;

static void make_shape(tw_shape *d, const int32_t *n_ctrl, const double *ctrl, const double *knots,
                       const double *params, int max_ctrl, int id, double xwidth)
{
    memset(d, 0, sizeof *d);
    const int nc = n_ctrl[id];
    const double *S = knots + (size_t)id * (max_ctrl + 4), *P = ctrl + (size_t)id * max_ctrl * 2;
    d->n = nc;
    d->b = params[3 * id];
    d->c = params[3 * id + 1];
    d->mu = params[3 * id + 2];
    d->xwidth = xwidth;
    for (int i = 0; i < nc + 4; ++i) d->knots[i] = S[i];
    for (int i = 0; i < 2 * nc; ++i) d->ctrl[i] = P[i];
    const double h0 = S[4] - S[3];
    d->inv_h = h0 > 0.0 ? 1.0 / h0 : 0.0;
    for (int i = 1; i < nc; ++i) {
        const double den = d->knots[i + 3] - d->knots[i];
        for (int c = 0; c < 2; ++c)
            d->dctrl[2 * i + c] = den != 0.0 ? 3.0 * ((d->ctrl[2 * i + c] - d->ctrl[2 * (i - 1) + c]) / den) : 0.0;
    }
    for (int i = 2; i < nc; ++i) {
        const double den = d->knots[i + 2] - d->knots[i];
        for (int c = 0; c < 2; ++c)
            d->ddctrl[2 * i + c] = den != 0.0 ? 2.0 * ((d->dctrl[2 * i + c] - d->dctrl[2 * (i - 1) + c]) / den) : 0.0;
    }
}

/* ------------------------------------------------------------------ spline (spline_eval) */
typedef struct { double C[2], D[2], Dd[2]; } spl;

static void spline_eval(const tw_shape *sh, double sig, spl *o)
{
    const int n = sh->n;
    const double *S = sh->knots;
    const int inside = (sig >= S[3]) && (sig < S[n]);
    /* the span guess; outside [S3, Sn) every output is masked to zero, so the guess only matters
     * inside, where sig * inv_h is a small non-negative number (truncated as the device does) */
    const double qg = sig * sh->inv_h;
    int j = 3 + ((qg > -1e9 && qg < 1e9) ? (int)qg : 0);
    j = j < 3 ? 3 : (j > n - 1 ? n - 1 : j);
    if (sig < S[j]) j = (j > 3) ? j - 1 : j;
    if (sig < S[j]) j = (j > 3) ? j - 1 : j;
    if (sig >= S[j + 1]) j = (j < n - 1) ? j + 1 : j;
    if (sig >= S[j + 1]) j = (j < n - 1) ? j + 1 : j;
    const double l1 = sig - S[j], l2 = sig - S[j - 1], l3 = sig - S[j - 2];
    const double r1 = S[j + 1] - sig, r2 = S[j + 2] - sig, r3 = S[j + 3] - sig;
    double N1_0, N1_1, N2_0, N2_1, N2_2, N3_0, N3_1, N3_2, N3_3;
    {
        const double t = 1.0 / (r1 + l1);
        N1_0 = r1 * t;
        N1_1 = l1 * t;
    }
    {
        const double t0 = N1_0 / (r1 + l2);
        const double t1 = N1_1 / (r2 + l1);
        N2_0 = r1 * t0;
        N2_1 = qfma(r2, t1, l2 * t0);
        N2_2 = l1 * t1;
    }
    {
        const double t0 = N2_0 / (r1 + l3);
        const double t1 = N2_1 / (r2 + l2);
        const double t2 = N2_2 / (r3 + l1);
        N3_0 = r1 * t0;
        N3_1 = qfma(r2, t1, l3 * t0);
        N3_2 = qfma(r3, t2, l2 * t1);
        N3_3 = l1 * t2;
    }
    const double *P = sh->ctrl + 2 * (j - 3);
    const double *cd = sh->dctrl + 2 * (j - 2);
    const double *dd = sh->ddctrl + 2 * (j - 1);
    for (int c = 0; c < 2; ++c) {
        double Cv = N3_0 * P[c];
        Cv = qfma(N3_1, P[2 + c], Cv);
        Cv = qfma(N3_2, P[4 + c], Cv);
        Cv = qfma(N3_3, P[6 + c], Cv);
        double Dv = N2_0 * cd[c];
        Dv = qfma(N2_1, cd[2 + c], Dv);
        Dv = qfma(N2_2, cd[4 + c], Dv);
        const double Ddv = qfma(N1_1, dd[2 + c], N1_0 * dd[c]);
        o->C[c] = inside ? Cv : 0.0;
        o->D[c] = inside ? Dv : 0.0;
        o->Dd[c] = inside ? Ddv : 0.0;
    }
}

static double smod_model(double s, double b) { return fmod(s, b) + ((s < 0.0) ? b : 0.0); }

static double mat_mod(double a, double b)
{
    const double r = qfma(-floor(a / b), b, a);
    return (r == b) ? 0.0 : r;
}

static double angle_rate_of(const spl *e)
{
    return qfma(e->D[0], e->Dd[1], -(e->D[1] * e->Dd[0])) / qfma(e->D[0], e->D[0], e->D[1] * e->D[1]);
}

static double v_bound(const tw_shape *sh, const or_opts *o, double s)
{
    const double sm = mat_mod(s, sh->b);
    spl e;
    spline_eval(sh, sm, &e);
    const double ta = fabs(angle_rate_of(&e));
    const double v = o->v_alpha / (fabs(ta - o->t_angle0) + 0.0001) + o->d_v;
    return v < o->u_t_ub ? v : o->u_t_ub;
}

/* ------------------------------------------------------------------ dynamics */
typedef struct { double f[4], Jth[2], Js[4], Jun[4], Jut[4]; } dyn;

static inline double blend3(double ist, double a, double isl, double b, double isr, double c)
{
    return qfma(isr, c, qfma(isl, b, ist * a));
}

static void dynamics(const tw_shape *sh, double th, double s, double un, double ut, dyn *o, int with_jac)
{
    const double sig = smod_model(s, sh->b);
    spl e;
    spline_eval(sh, sig, &e);
    const double l2 = qfma(e.D[0], e.D[0], e.D[1] * e.D[1]);
    const double l = sqrt(l2);
    const double il = 1.0 / l;
    const double tx = e.D[0] * il, ty = e.D[1] * il;
    const double nx = ty, ny = -tx;
    const double Px = e.C[0], Py = e.C[1];
    const double px = qfma(nx, Px, ny * Py);
    const double py = qfma(tx, Px, ty * Py);
    const double c2 = sh->c * sh->c, mu = sh->mu;
    const double pxpy = px * py, px2 = px * px;
    const double q00 = qfma(px, px, c2), q11 = qfma(py, py, c2);
    const double fac = 1.0 / qfma(py, py, q00);
    const double nl = qfma(mu, px2, qfma(mu, c2, -pxpy));
    const double dl = qfma(-mu, pxpy, q11);
    const double nr = qfma(-mu, px2, qfma(-mu, c2, -pxpy));
    const double dr = qfma(mu, pxpy, q11);
    const double gl = nl / dl, gr = nr / dr;
    const double rho = ut / un;
    double sn, cs;
    sin_cos(th, &sn, &cs);
    const double H00 = qfma(tx, pxpy, nx * q00), H01 = qfma(tx, q11, nx * pxpy);
    const double H10 = qfma(ty, pxpy, ny * q00), H11 = qfma(ty, q11, ny * pxpy);
    const double G00 = fac * H00, G01 = fac * H01, G10 = fac * H10, G11 = fac * H11;
    const double M00 = qfma(-sn, G10, cs * G00), M01 = qfma(-sn, G11, cs * G01);
    const double M10 = qfma(cs, G10, sn * G00), M11 = qfma(cs, G11, sn * G01);
    const double ist = ((rho >= gr) && (rho <= gl)) ? 1.0 : 0.0;
    const double isl = (rho > gl) ? 1.0 : 0.0;
    const double isr = (rho < gr) ? 1.0 : 0.0;
    const double st0 = qfma(M01, ut, M00 * un);
    const double st1 = qfma(M11, ut, M10 * un);
    const double st2 = fac * qfma(px, ut, -(py * un));
    const double vl0 = qfma(M01, gl, M00), vl1 = qfma(M11, gl, M10);
    const double vr0 = qfma(M01, gr, M00), vr1 = qfma(M11, gr, M10);
    const double wl = fac * qfma(gl, px, -py), wr = fac * qfma(gr, px, -py);
    o->f[0] = blend3(ist, st0, isl, vl0 * un, isr, vr0 * un);
    o->f[1] = blend3(ist, st1, isl, vl1 * un, isr, vr1 * un);
    o->f[2] = blend3(ist, st2, isl, wl * un, isr, wr * un);
    o->f[3] = qfma(isr, qfma(-gr, un, ut), isl * qfma(-gl, un, ut));
    if (!with_jac) return;
    const double tDd = qfma(ty, e.Dd[1], tx * e.Dd[0]);
    const double txs = qfma(-tx, tDd, e.Dd[0]) * il, tys = qfma(-ty, tDd, e.Dd[1]) * il;
    const double nxs = tys, nys = -txs;
    const double pxs = qfma(nxs, Px, nys * Py);
    const double pys = qfma(txs, Px, tys * Py) + l;
    const double pxpys = qfma(px, pys, pxs * py);
    const double q00s = 2.0 * px * pxs, q11s = 2.0 * py * pys;
    const double facs = -fac * fac * (q00s + q11s);
    const double gls = qfma(-gl, qfma(-mu, pxpys, q11s), qfma(mu, q00s, -pxpys)) / dl;
    const double grs = qfma(-gr, qfma(mu, pxpys, q11s), qfma(-mu, q00s, -pxpys)) / dr;
    const double G00s = qfma(facs, H00, fac * qfma(tx, pxpys, qfma(txs, pxpy, qfma(nx, q00s, nxs * q00))));
    const double G01s = qfma(facs, H01, fac * qfma(tx, q11s, qfma(txs, q11, qfma(nx, pxpys, nxs * pxpy))));
    const double G10s = qfma(facs, H10, fac * qfma(ty, pxpys, qfma(tys, pxpy, qfma(ny, q00s, nys * q00))));
    const double G11s = qfma(facs, H11, fac * qfma(ty, q11s, qfma(tys, q11, qfma(ny, pxpys, nys * pxpy))));
    const double M00s = qfma(-sn, G10s, cs * G00s), M01s = qfma(-sn, G11s, cs * G01s);
    const double M10s = qfma(cs, G10s, sn * G00s), M11s = qfma(cs, G11s, sn * G01s);
    const double M00t = qfma(-cs, G10, -sn * G00), M01t = qfma(-cs, G11, -sn * G01);
    const double M10t = qfma(-sn, G10, cs * G00), M11t = qfma(-sn, G11, cs * G01);
    const double st0t = qfma(M01t, ut, M00t * un), st1t = qfma(M11t, ut, M10t * un);
    const double st0s = qfma(M01s, ut, M00s * un), st1s = qfma(M11s, ut, M10s * un);
    const double st2s = qfma(facs, qfma(px, ut, -(py * un)), fac * qfma(pxs, ut, -(pys * un)));
    const double vl0s = qfma(M01, gls, qfma(M01s, gl, M00s)), vl1s = qfma(M11, gls, qfma(M11s, gl, M10s));
    const double vr0s = qfma(M01, grs, qfma(M01s, gr, M00s)), vr1s = qfma(M11, grs, qfma(M11s, gr, M10s));
    const double vl0t = qfma(M01t, gl, M00t), vl1t = qfma(M11t, gl, M10t);
    const double vr0t = qfma(M01t, gr, M00t), vr1t = qfma(M11t, gr, M10t);
    const double wls = qfma(facs, qfma(gl, px, -py), fac * (qfma(gl, pxs, gls * px) - pys));
    const double wrs = qfma(facs, qfma(gr, px, -py), fac * (qfma(gr, pxs, grs * px) - pys));
    o->Jth[0] = blend3(ist, st0t, isl, vl0t * un, isr, vr0t * un);
    o->Jth[1] = blend3(ist, st1t, isl, vl1t * un, isr, vr1t * un);
    o->Js[0] = blend3(ist, st0s, isl, vl0s * un, isr, vr0s * un);
    o->Js[1] = blend3(ist, st1s, isl, vl1s * un, isr, vr1s * un);
    o->Js[2] = blend3(ist, st2s, isl, wls * un, isr, wrs * un);
    o->Js[3] = -qfma(isr, grs * un, isl * (gls * un));
    o->Jun[0] = blend3(ist, M00, isl, vl0, isr, vr0);
    o->Jun[1] = blend3(ist, M10, isl, vl1, isr, vr1);
    o->Jun[2] = blend3(-ist, fac * py, isl, wl, isr, wr);
    o->Jun[3] = -qfma(isr, gr, isl * gl);
    o->Jut[0] = ist * M01;
    o->Jut[1] = ist * M11;
    o->Jut[2] = ist * (fac * px);
    o->Jut[3] = isl + isr;
}

/* ------------------------------------------------------------------ RK4 + VDE (rk4) */
typedef struct { double xn[4], a[6], B[8]; } lin;

static void rk4(const tw_shape *sh, double h, const double x[4], const double u[2], lin *o, int with_sens)
{
    static const double ca[4] = {0.0, 0.5, 0.5, 1.0};
    const double cb[4] = {1.0 / 6.0, 1.0 / 3.0, 1.0 / 3.0, 1.0 / 6.0};
    double acc[4] = {x[0], x[1], x[2], x[3]};
    double Sa[4][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {1, 0, 0, 0}, {0, 1, 0, 0}};
    double K[4] = {0, 0, 0, 0};
    double SK[4][4] = {{0}};
    for (int st = 0; st < 4; ++st) {
        const double aa = h * ca[st];
        double xs[4], Ss[2][4];
        for (int i = 0; i < 4; ++i) xs[i] = (st == 0) ? x[i] : qfma(aa, K[i], x[i]);
        for (int c = 0; c < 4; ++c) {
            const double e2 = (c == 0) ? 1.0 : 0.0, e3 = (c == 1) ? 1.0 : 0.0;
            Ss[0][c] = (st == 0) ? e2 : qfma(aa, SK[2][c], e2);
            Ss[1][c] = (st == 0) ? e3 : qfma(aa, SK[3][c], e3);
        }
        dyn d;
        dynamics(sh, xs[2], xs[3], u[0], u[1], &d, with_sens);
        for (int i = 0; i < 4; ++i) K[i] = d.f[i];
        if (with_sens) {
            for (int c = 0; c < 4; ++c) {
                const double jt = Ss[0][c], js = Ss[1][c];
                SK[0][c] = qfma(d.Js[0], js, d.Jth[0] * jt);
                SK[1][c] = qfma(d.Js[1], js, d.Jth[1] * jt);
                SK[2][c] = d.Js[2] * js;
                SK[3][c] = d.Js[3] * js;
            }
            for (int i = 0; i < 4; ++i) {
                SK[i][2] += d.Jun[i];
                SK[i][3] += d.Jut[i];
            }
        }
        const double w = h * cb[st];
        for (int i = 0; i < 4; ++i) acc[i] = qfma(w, K[i], acc[i]);
        if (with_sens)
            for (int i = 0; i < 4; ++i)
                for (int c = 0; c < 4; ++c) Sa[i][c] = qfma(w, SK[i][c], Sa[i][c]);
    }
    for (int i = 0; i < 4; ++i) o->xn[i] = acc[i];
    if (with_sens) {
        o->a[0] = Sa[0][0]; o->a[1] = Sa[0][1];
        o->a[2] = Sa[1][0]; o->a[3] = Sa[1][1];
        o->a[4] = Sa[2][1]; o->a[5] = Sa[3][1];
        for (int i = 0; i < 4; ++i) { o->B[2 * i] = Sa[i][2]; o->B[2 * i + 1] = Sa[i][3]; }
    }
}

/* ================================================================== the QP (qp_ipm) */
typedef struct {
    double a[6], B[8], bb[4], g[6], v[3];
    double K[8], Rn[3], kk[2], M[16];
    double t[6], lm[6], rt[6], hg[6];
    double VA[3], VN[3], du[2], dxs[4];
    double at[6], al[6], dt[6], dl[6];
} tw_stage;

/* the solve parameters the kernels read (SolveParams): the options plus the QP-level overrides */
typedef struct {
    int N, S, L, nlp_mode, sqp_iters, qp_iters, qp_stall_iters, s0_bound, factor_scan, mfma_walk;
    double Ts, tau, W[6], We[4], lh[3], uh[3];
    double mu0, t_min, frac, sigma_min, mu_stop, res_stop, qp_tol_stat, qp_tol_eq, qp_stall_alpha, qp_mu_max;
    double tol_stat, tol_eq, tol_ineq, tol_comp, ls_alpha_min, ls_alpha_red, ls_eps;
    double v_alpha, d_v, t_angle0, u_n_lb, u_t_ub;
} tw_par;

static int auto_S(const or_opts *o)
{
    if (o->stages_per_lane > 0) return o->stages_per_lane;
    if (o->nlp_mode == 1) return 1;
    return o->N + 1 <= 32 ? 1 : 2;
}

static void make_par(tw_par *p, const or_opts *o)
{
    memset(p, 0, sizeof *p);
    p->N = o->N;
    p->S = auto_S(o);
    p->L = (p->N + p->S) / p->S;
    p->nlp_mode = o->nlp_mode;
    p->sqp_iters = o->sqp_iters;
    p->qp_iters = o->qp_iters;
    p->qp_stall_iters = o->qp_stall_iters;
    p->s0_bound = o->stage0_s_bound ? 1 : 0;
    p->factor_scan = o->factor_scan ? 1 : 0;
    /* the kernels factorise on the matrix cores where one instance per 16-lane block and a phase's
     * stage records fit (mfw_fits: one stage per lane at 12 <= N <= 31, two stages per lane from four
     * instances per wave down), unless the library's developer switch QSP_MFMA_WALK=0 selects the lane
     * walk there too */
    const char *mw = getenv("QSP_MFMA_WALK");
    {
        const int G = 64 / p->L, H = (p->N + 1) / 2, CM = p->N + 1 - H;
        const int cap = (p->S == 1 ? 12 + 2 : 24 + 4) * 64;   /* F_VA .. F_HG per slot + mfw_extra, x 64 lanes */
        const int fits = G <= 4 && G * CM * 27 + 5 <= cap && (p->S == 2 || p->N <= 31);   /* + 5 constants */
        p->mfma_walk = fits && !(mw && mw[0] == '0') && !o->lane_walk;
    }
    p->Ts = o->Ts;
    p->tau = o->tau;
    memcpy(p->W, o->W, sizeof p->W);
    memcpy(p->We, o->We, sizeof p->We);
    memcpy(p->lh, o->lh, sizeof p->lh);
    memcpy(p->uh, o->uh, sizeof p->uh);
    p->mu0 = o->mu0; p->t_min = o->t_min; p->frac = o->frac; p->sigma_min = o->sigma_min; p->mu_stop = o->mu_stop;
    p->res_stop = o->res_stop; p->qp_tol_stat = o->qp_tol_stat; p->qp_tol_eq = o->qp_tol_eq;
    p->qp_stall_alpha = o->qp_stall_alpha; p->qp_mu_max = o->qp_mu_max;
    p->tol_stat = o->tol_stat; p->tol_eq = o->tol_eq; p->tol_ineq = o->tol_ineq; p->tol_comp = o->tol_comp;
    p->ls_alpha_min = o->ls_alpha_min; p->ls_alpha_red = o->ls_alpha_red; p->ls_eps = o->ls_eps;
    p->v_alpha = o->v_alpha; p->d_v = o->d_v; p->t_angle0 = o->t_angle0; p->u_n_lb = o->u_n_lb; p->u_t_ub = o->u_t_ub;
}

/* group_sum: the kernel's log-step shuffle tree towards the group's first lane */
static double group_sum(double *v, int L)
{
    double tmp[64];
    for (int off = 1; off < L; off <<= 1) {
        for (int i = 0; i < L; ++i) tmp[i] = v[i] + ((i + off < L) ? v[i + off] : 0.0);
        memcpy(v, tmp, sizeof(double) * (size_t)L);
    }
    return v[0];
}
/* group_min / group_max of non-NaN values (exact in any order) */
static double group_min(const double *v, int L)
{
    double r = v[L - 1];
    for (int i = L - 2; i >= 0; --i) r = (v[i] < r) ? v[i] : r;
    return r;
}
static double group_max(const double *v, int L)
{
    double r = v[L - 1];
    for (int i = L - 2; i >= 0; --i) r = (v[i] > r) ? v[i] : r;
    return r;
}

static inline int bnd_act(const tw_par *p, int k, int j) { return (k < p->N) && (j > 0 || k >= 1 || p->s0_bound != 0); }

static inline void bnd_lohi(const tw_par *p, const tw_stage *s, double lo[3], double hi[3])
{
    for (int j = 0; j < 3; ++j) { lo[j] = p->lh[j] - s->v[j]; hi[j] = p->uh[j] - s->v[j]; }
}

static inline int sidx(int i, int j)
{
    if (i > j) { int t = i; i = j; j = t; }
    return i == 0 ? j : (i == 1 ? 3 + j : (i == 2 ? 5 + j : 9));
}

/* ric_factor_step */
static void ric_factor_step(const double a[6], const double B[8], const double bb[4], const double Hx[4],
                            const double Hu[2], const double gx[4], const double gu[2], double P[10], double pv[4],
                            double K[8], double Rn[3], double kk[2], int upd)
{
    double Pm[4][4], PA[4][4], PB[4][2], pp[4], St[2][4], rt[2], Qt[10], qt[4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) Pm[i][j] = P[sidx(i, j)];
    for (int i = 0; i < 4; ++i) {
        PA[i][0] = Pm[i][0];
        PA[i][1] = Pm[i][1];
        PA[i][2] = qfma(Pm[i][1], a[2], qfma(Pm[i][0], a[0], Pm[i][2]));
        PA[i][3] = qfma(Pm[i][3], a[5], qfma(Pm[i][2], a[4], qfma(Pm[i][1], a[3], Pm[i][0] * a[1])));
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 2; ++j)
            PB[i][j] = qfma(Pm[i][3], B[6 + j], qfma(Pm[i][2], B[4 + j], qfma(Pm[i][1], B[2 + j], Pm[i][0] * B[j])));
    for (int i = 0; i < 4; ++i)
        pp[i] = qfma(Pm[i][3], bb[3], qfma(Pm[i][2], bb[2], qfma(Pm[i][1], bb[1], qfma(Pm[i][0], bb[0], pv[i]))));
    const double R00 = qfma(B[6], PB[3][0], qfma(B[4], PB[2][0], qfma(B[2], PB[1][0], qfma(B[0], PB[0][0], Hu[0]))));
    const double R01 = qfma(B[6], PB[3][1], qfma(B[4], PB[2][1], qfma(B[2], PB[1][1], B[0] * PB[0][1])));
    const double R11 = qfma(B[7], PB[3][1], qfma(B[5], PB[2][1], qfma(B[3], PB[1][1], qfma(B[1], PB[0][1], Hu[1]))));
    for (int i = 0; i < 2; ++i) {
        St[i][0] = PB[0][i];
        St[i][1] = PB[1][i];
        St[i][2] = qfma(PB[1][i], a[2], qfma(PB[0][i], a[0], PB[2][i]));
        St[i][3] = qfma(PB[3][i], a[5], qfma(PB[2][i], a[4], qfma(PB[1][i], a[3], PB[0][i] * a[1])));
    }
    for (int i = 0; i < 2; ++i)
        rt[i] = qfma(B[6 + i], pp[3], qfma(B[4 + i], pp[2], qfma(B[2 + i], pp[1], qfma(B[i], pp[0], gu[i]))));
    for (int j = 0; j < 4; ++j) {
        const double c0 = PA[0][j], c1 = PA[1][j], c2 = PA[2][j], c3 = PA[3][j];
        Qt[sidx(0, j)] = c0;
        if (j >= 1) Qt[sidx(1, j)] = c1;
        if (j >= 2) Qt[sidx(2, j)] = qfma(a[2], c1, qfma(a[0], c0, j == 2 ? Hx[2] + c2 : c2));
        if (j >= 3) Qt[sidx(3, j)] = qfma(a[5], c3, qfma(a[4], c2, qfma(a[3], c1, qfma(a[1], c0, Hx[3]))));
    }
    Qt[0] += Hx[0];
    Qt[4] += Hx[1];
    qt[0] = gx[0] + pp[0];
    qt[1] = gx[1] + pp[1];
    qt[2] = qfma(a[2], pp[1], qfma(a[0], pp[0], gx[2] + pp[2]));
    qt[3] = qfma(a[5], pp[3], qfma(a[4], pp[2], qfma(a[3], pp[1], qfma(a[1], pp[0], gx[3]))));
    const double idet = rcp(qfma(R00, R11, -(R01 * R01)));
    Rn[0] = (-R11) * idet; Rn[1] = R01 * idet; Rn[2] = (-R00) * idet;
    for (int j = 0; j < 4; ++j) {
        K[j] = qfma(Rn[1], St[1][j], Rn[0] * St[0][j]);
        K[4 + j] = qfma(Rn[2], St[1][j], Rn[1] * St[0][j]);
    }
    kk[0] = qfma(Rn[1], rt[1], Rn[0] * rt[0]);
    kk[1] = qfma(Rn[2], rt[1], Rn[1] * rt[0]);
    if (!upd) return;
    for (int i = 0; i < 4; ++i)
        for (int j = i; j < 4; ++j) P[sidx(i, j)] = qfma(St[1][i], K[4 + j], qfma(St[0][i], K[j], Qt[sidx(i, j)]));
    for (int i = 0; i < 4; ++i) pv[i] = qfma(K[4 + i], rt[1], qfma(K[i], rt[0], qt[i]));
}

/* ric_delta_step */
static void ric_delta_step(const double a[6], const double B[8], double dgx3, const double dgu[2], const double K[8],
                           const double Rn[3], double pv[4], double dkk[2])
{
    double rt[2], qt[4];
    for (int i = 0; i < 2; ++i)
        rt[i] = qfma(B[6 + i], pv[3], qfma(B[4 + i], pv[2], qfma(B[2 + i], pv[1], qfma(B[i], pv[0], dgu[i]))));
    qt[0] = pv[0];
    qt[1] = pv[1];
    qt[2] = qfma(a[2], pv[1], qfma(a[0], pv[0], pv[2]));
    qt[3] = qfma(a[5], pv[3], qfma(a[4], pv[2], qfma(a[3], pv[1], qfma(a[1], pv[0], dgx3))));
    dkk[0] = qfma(Rn[1], rt[1], Rn[0] * rt[0]);
    dkk[1] = qfma(Rn[2], rt[1], Rn[1] * rt[0]);
    for (int i = 0; i < 4; ++i) pv[i] = qfma(K[4 + i], rt[1], qfma(K[i], rt[0], qt[i]));
}

/* dyn_step */
static void dyn_step(const double a[6], const double B[8], const double bb[4], const double du[2], double dx[4])
{
    const double n0 = qfma(B[1], du[1], qfma(B[0], du[0], qfma(a[1], dx[3], qfma(a[0], dx[2], bb[0] + dx[0]))));
    const double n1 = qfma(B[3], du[1], qfma(B[2], du[0], qfma(a[3], dx[3], qfma(a[2], dx[2], bb[1] + dx[1]))));
    const double n2 = qfma(B[5], du[1], qfma(B[4], du[0], qfma(a[4], dx[3], bb[2] + dx[2])));
    const double n3 = qfma(B[7], du[1], qfma(B[6], du[0], qfma(a[5], dx[3], bb[3])));
    dx[0] = n0; dx[1] = n1; dx[2] = n2; dx[3] = n3;
}

/* barrier_terms */
static void barrier_terms(const tw_par *p, tw_stage *s, int k)
{
    double lo[3], hi[3];
    bnd_lohi(p, s, lo, hi);
    for (int j = 0; j < 3; ++j) {
        const int act = bnd_act(p, k, j);
        const double ll = s->lm[2 * j], lh = s->lm[2 * j + 1];
        const double sl = ll * s->rt[2 * j], sh = lh * s->rt[2 * j + 1];
        const double gadd = qfma(-sh, hi[j], -sl * lo[j]) + (lh - ll);
        s->hg[j] = act ? sl + sh : 0.0;
        s->hg[3 + j] = act ? gadd : 0.0;
    }
}

#define RATIO(tv, dv) do { if ((dv) < 0.0 && (tv) * den < num * -(dv)) { num = (tv); den = -(dv); } } while (0)

/* affine_dirs: directions kept in at / al, ratio folded into num/den of the lane */
static void affine_dirs(const tw_par *p, tw_stage *s, int k, double *pnum, double *pden)
{
    double num = *pnum, den = *pden;
    double lo[3], hi[3];
    bnd_lohi(p, s, lo, hi);
    for (int j = 0; j < 3; ++j) {
        const int act = bnd_act(p, k, j);
        const double tl = s->t[2 * j], th = s->t[2 * j + 1];
        const double ll = s->lm[2 * j], lh = s->lm[2 * j + 1];
        const double sl = ll * s->rt[2 * j], sh = lh * s->rt[2 * j + 1];
        const double v = s->VA[j];
        s->at[2 * j] = v - lo[j] - tl;
        s->at[2 * j + 1] = hi[j] - v - th;
        s->al[2 * j] = qfma(-sl, s->at[2 * j], -ll);
        s->al[2 * j + 1] = qfma(-sh, s->at[2 * j + 1], -lh);
        const double dtl = act ? s->at[2 * j] : 0.0, dth = act ? s->at[2 * j + 1] : 0.0;
        const double dll = act ? s->al[2 * j] : 0.0, dlh = act ? s->al[2 * j + 1] : 0.0;
        RATIO(tl, dtl);
        RATIO(th, dth);
        RATIO(ll, dll);
        RATIO(lh, dlh);
    }
    *pnum = num;
    *pden = den;
}

static double affine_mu_part(const tw_par *p, const tw_stage *s, int k, double aa, double part)
{
    for (int j = 0; j < 3; ++j) {
        const int act = bnd_act(p, k, j);
        const double tl = s->t[2 * j], th = s->t[2 * j + 1];
        const double ll = s->lm[2 * j], lh = s->lm[2 * j + 1];
        const double dtl = act ? s->at[2 * j] : 0.0, dth = act ? s->at[2 * j + 1] : 0.0;
        const double dll = act ? s->al[2 * j] : 0.0, dlh = act ? s->al[2 * j + 1] : 0.0;
        part = qfma(qfma(aa, dtl, tl), qfma(aa, dll, ll), part);
        part = qfma(qfma(aa, dth, th), qfma(aa, dlh, lh), part);
    }
    return part;
}

static void corrector_terms(const tw_par *p, tw_stage *s, int k, double smu)
{
    for (int j = 0; j < 3; ++j) {
        const int act = bnd_act(p, k, j);
        const double cl = qfma(-s->at[2 * j], s->al[2 * j], smu), ch = qfma(-s->at[2 * j + 1], s->al[2 * j + 1], smu);
        s->hg[3 + j] = act ? qfma(ch, s->rt[2 * j + 1], -(cl * s->rt[2 * j])) : 0.0;
    }
}

static void corrector_dirs(const tw_par *p, tw_stage *s, int k, double smu, double *pnum, double *pden)
{
    double num = *pnum, den = *pden;
    double lo[3], hi[3];
    bnd_lohi(p, s, lo, hi);
    for (int j = 0; j < 3; ++j) {
        const int act = bnd_act(p, k, j);
        const double tl = s->t[2 * j], th = s->t[2 * j + 1];
        const double ll = s->lm[2 * j], lh = s->lm[2 * j + 1];
        const double rtl = s->rt[2 * j], rth = s->rt[2 * j + 1];
        const double sl = ll * rtl, sh = lh * rth;
        const double v = s->VN[j];
        double dtl = v - lo[j] - tl, dth = hi[j] - v - th;
        double dll = qfma(-sl, dtl, -ll), dlh = qfma(-sh, dth, -lh);
        dll = qfma(qfma(-s->at[2 * j], s->al[2 * j], smu), rtl, dll);
        dlh = qfma(qfma(-s->at[2 * j + 1], s->al[2 * j + 1], smu), rth, dlh);
        dtl = act ? dtl : 0.0; dth = act ? dth : 0.0;
        dll = act ? dll : 0.0; dlh = act ? dlh : 0.0;
        RATIO(tl, dtl);
        RATIO(th, dth);
        RATIO(ll, dll);
        RATIO(lh, dlh);
        s->dt[2 * j] = dtl; s->dt[2 * j + 1] = dth;
        s->dl[2 * j] = dll; s->dl[2 * j + 1] = dlh;
    }
    *pnum = num;
    *pden = den;
}

static void apply_step(tw_stage *s, double alpha)
{
    for (int q = 0; q < 6; ++q) {
        const double tn = qfma(alpha, s->dt[q], s->t[q]);
        s->t[q] = tn;
        s->rt[q] = rcp(tn);
        s->lm[q] = qfma(alpha, s->dl[q], s->lm[q]);
    }
}

/* ---- S = 2: the affine passes as scans (qsp_solver.hip Aff, aff_*; riccati_solve<2, ...>) */
typedef struct { double F[16], c[4]; } tw_aff;   /* x -> F x + c */

/* g <- g o f, in place row by row (aff_compose) */
static void aff_compose(tw_aff *g, const tw_aff *f)
{
    for (int i = 0; i < 4; ++i) {
        double r[5];
        for (int j = 0; j < 4; ++j)
            r[j] = qfma(g->F[4 * i + 3], f->F[12 + j], qfma(g->F[4 * i + 2], f->F[8 + j],
                        qfma(g->F[4 * i + 1], f->F[4 + j], g->F[4 * i] * f->F[j])));
        r[4] = qfma(g->F[4 * i + 3], f->c[3], qfma(g->F[4 * i + 2], f->c[2], qfma(g->F[4 * i + 1], f->c[1],
                    qfma(g->F[4 * i], f->c[0], g->c[i]))));
        for (int j = 0; j < 4; ++j) g->F[4 * i + j] = r[j];
        g->c[i] = r[4];
    }
}
static void aff_apply(const tw_aff *m, const double x[4], double y[4])
{
    for (int i = 0; i < 4; ++i)
        y[i] = qfma(m->F[4 * i + 3], x[3], qfma(m->F[4 * i + 2], x[2], qfma(m->F[4 * i + 1], x[1], qfma(m->F[4 * i], x[0], m->c[i]))));
}
static void aff_identity(tw_aff *m)
{
    for (int q = 0; q < 16; ++q) m->F[q] = (q % 5 == 0) ? 1.0 : 0.0;
    for (int q = 0; q < 4; ++q) m->c[q] = 0.0;
}
static void aff_forward(const tw_stage *s, tw_aff *m)
{
    const double *a = s->a, *B = s->B, *K = s->K;
    const double Am[4][4] = {{1.0, 0.0, a[0], a[1]}, {0.0, 1.0, a[2], a[3]}, {0.0, 0.0, 1.0, a[4]}, {0.0, 0.0, 0.0, a[5]}};
    for (int i = 0; i < 4; ++i) {
        for (int q = 0; q < 4; ++q) m->F[4 * i + q] = qfma(B[2 * i + 1], K[4 + q], qfma(B[2 * i], K[q], Am[i][q]));
        m->c[i] = qfma(B[2 * i + 1], s->kk[1], qfma(B[2 * i], s->kk[0], s->bb[i]));
    }
}
static void aff_delta(const tw_stage *s, double dgx3, const double dgu[2], tw_aff *m)
{
    const double *a = s->a, *B = s->B, *K = s->K;
    const double Am[4][4] = {{1.0, 0.0, a[0], a[1]}, {0.0, 1.0, a[2], a[3]}, {0.0, 0.0, 1.0, a[4]}, {0.0, 0.0, 0.0, a[5]}};
    for (int i = 0; i < 4; ++i) {
        for (int q = 0; q < 4; ++q) m->F[4 * q + i] = qfma(B[2 * i + 1], K[4 + q], qfma(B[2 * i], K[q], Am[i][q]));
        m->c[i] = qfma(K[4 + i], dgu[1], qfma(K[i], dgu[0], i == 3 ? dgx3 : 0.0));
    }
}

/* the S = 2 difference pass: suffix scan of the lanes' backward maps (slot 1's, then slot 0's;
 * identity past the horizon), dp_N = 0; each slot's dkk from the dp reaching it */
static void delta_scan_s2(const tw_par *p, tw_stage *st, const double *gx3, double (*gu)[2])
{
    const int N = p->N, L = p->L;
    tw_aff d[64], nd[64];
    for (int l = 0; l < L; ++l) {
        const int k0 = 2 * l;
        if (k0 + 1 < N) {
            tw_aff m1;
            aff_delta(st + k0, gx3[k0], gu[k0], d + l);
            aff_delta(st + k0 + 1, gx3[k0 + 1], gu[k0 + 1], &m1);
            aff_compose(d + l, &m1);
        } else if (k0 < N) {
            aff_delta(st + k0, gx3[k0], gu[k0], d + l);
        } else {
            aff_identity(d + l);
        }
    }
    for (int off = 1; off < L; off <<= 1) {
        for (int l = 0; l < L; ++l) {
            nd[l] = d[l];
            if (l + off < L) aff_compose(nd + l, d + l + off);
        }
        memcpy(d, nd, sizeof(tw_aff) * (size_t)L);
    }
    for (int l = 0; l < L; ++l) {
        double pv[4];
        for (int i = 0; i < 4; ++i) pv[i] = (l + 1 < L) ? d[l + 1].c[i] : 0.0;
        for (int ls = 1; ls >= 0; --ls) {
            const int k = 2 * l + ls;
            if (k < N) {
                tw_stage *s = st + k;
                double dkk[2];
                ric_delta_step(s->a, s->B, gx3[k], gu[k], s->K, s->Rn, pv, dkk);
                s->kk[0] += dkk[0];
                s->kk[1] += dkk[1];
            }
        }
    }
}

/* the S = 2 forward pass: prefix scan of the lanes' closed-loop maps (slot 0's, then slot 1's); the
 * state entering lane l is T_{l-1}(dx0); slot 0 forms du and steps the dynamics, slot 1 forms du */
static void forward_scan_s2(const tw_par *p, tw_stage *st, const double dx0[4], int factor)
{
    const int N = p->N, L = p->L;
    tw_aff e[64], ne[64];
    for (int l = 0; l < L; ++l) {
        const int k0 = 2 * l;
        if (k0 + 1 < N) {   /* the last lane's map is consumed by no lane (values there are unused) */
            tw_aff m1;
            aff_forward(st + k0, e + l);
            aff_forward(st + k0 + 1, &m1);
            aff_compose(&m1, e + l);
            e[l] = m1;
        } else {
            aff_identity(e + l);
        }
    }
    for (int off = 1; off < L; off <<= 1) {
        for (int l = 0; l < L; ++l) {
            ne[l] = e[l];
            if (l >= off) aff_compose(ne + l, e + l - off);
        }
        memcpy(e, ne, sizeof(tw_aff) * (size_t)L);
    }
    for (int l = 0; l < L; ++l) {
        double dx[4];
        if (l == 0) memcpy(dx, dx0, sizeof dx);
        else aff_apply(e + l - 1, dx0, dx);
        for (int ls = 0; ls < 2; ++ls) {
            const int k = 2 * l + ls;
            if (k >= N) break;
            tw_stage *s = st + k;
            double du[2];
            du[0] = qfma(s->K[3], dx[3], qfma(s->K[2], dx[2], qfma(s->K[1], dx[1], qfma(s->K[0], dx[0], s->kk[0]))));
            du[1] = qfma(s->K[7], dx[3], qfma(s->K[6], dx[2], qfma(s->K[5], dx[1], qfma(s->K[4], dx[0], s->kk[1]))));
            double *out = factor ? s->VA : s->VN;
            out[0] = dx[3];
            out[1] = du[0];
            out[2] = du[1];
            if (ls == 0) dyn_step(s->a, s->B, s->bb, du, dx);
        }
    }
}

/* ---- S = 2: the factorisation as an associative scan (qsp_solver.hip VElem, velem_*; riccati_solve<2, true>):
 * the conditional value-function elements of Sarkka & Garcia-Fernandez (IEEE TAC 2023),
 * e_k = (A_k, c_k - B Hu^-1 gu, B Hu^-1 B', -gx, diag Hx), e_N = (0, 0, 0, -g_N, We), combined in
 * the kernel's association order; P_k = J, p_k = -eta of the suffix product over k..N */
typedef struct { double A[16], b[4], C[10], eta[4], J[10]; } tw_velem;

static void velem_stage(const double a[6], const double B[8], const double bb[4], const double Hx[4], const double Hu[2],
                        const double gx[4], const double gu[2], tw_velem *e)
{
    const double F[16] = {1.0, 0.0, a[0], a[1], 0.0, 1.0, a[2], a[3], 0.0, 0.0, 1.0, a[4], 0.0, 0.0, 0.0, a[5]};
    memcpy(e->A, F, sizeof F);
    const double ih0 = rcp(Hu[0]), ih1 = rcp(Hu[1]);
    const double v0 = ih0 * gu[0], v1 = ih1 * gu[1];
    for (int i = 0; i < 4; ++i) {
        e->b[i] = qfma(-B[2 * i + 1], v1, qfma(-B[2 * i], v0, bb[i]));
        e->eta[i] = -gx[i];
        const double w0 = B[2 * i] * ih0, w1 = B[2 * i + 1] * ih1;
        for (int j = i; j < 4; ++j) {
            e->C[sidx(i, j)] = qfma(w1, B[2 * j + 1], w0 * B[2 * j]);
            e->J[sidx(i, j)] = (i == j) ? Hx[i] : 0.0;
        }
    }
}
static void velem_terminal(const double We[4], const double g[6], tw_velem *e)
{
    memset(e, 0, sizeof *e);
    for (int q = 0; q < 4; ++q) { e->eta[q] = -g[q]; e->J[sidx(q, q)] = We[q]; }
}
/* e <- e (x) f in place (velem_combine) */
static void velem_combine(tw_velem *e, const tw_velem *f)
{
    double T[4][4], TA[4][4], Um[4][4], w[4], z[4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            T[i][j] = qfma(e->C[sidx(i, 3)], f->J[sidx(3, j)], qfma(e->C[sidx(i, 2)], f->J[sidx(2, j)],
                      qfma(e->C[sidx(i, 1)], f->J[sidx(1, j)], qfma(e->C[sidx(i, 0)], f->J[sidx(0, j)], i == j ? 1.0 : 0.0))));
    for (int c = 0; c < 4; ++c) {
        const double piv = rcp(T[c][c]);
        T[c][c] = 1.0;
        for (int j = 0; j < 4; ++j) T[c][j] *= piv;
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            const double fct = T[r][c];
            T[r][c] = 0.0;
            for (int j = 0; j < 4; ++j) T[r][j] = qfma(-fct, T[c][j], T[r][j]);
        }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            TA[i][j] = qfma(f->A[4 * i + 3], T[3][j], qfma(f->A[4 * i + 2], T[2][j], qfma(f->A[4 * i + 1], T[1][j], f->A[4 * i] * T[0][j])));
            Um[i][j] = qfma(e->A[12 + i], T[j][3], qfma(e->A[8 + i], T[j][2], qfma(e->A[4 + i], T[j][1], e->A[i] * T[j][0])));
        }
    for (int i = 0; i < 4; ++i) {
        w[i] = qfma(e->C[sidx(i, 3)], f->eta[3], qfma(e->C[sidx(i, 2)], f->eta[2], qfma(e->C[sidx(i, 1)], f->eta[1], qfma(e->C[sidx(i, 0)], f->eta[0], e->b[i]))));
        z[i] = qfma(-f->J[sidx(i, 3)], e->b[3], qfma(-f->J[sidx(i, 2)], e->b[2], qfma(-f->J[sidx(i, 1)], e->b[1], qfma(-f->J[sidx(i, 0)], e->b[0], f->eta[i]))));
    }
    for (int i = 0; i < 4; ++i) {
        e->b[i] = qfma(TA[i][3], w[3], qfma(TA[i][2], w[2], qfma(TA[i][1], w[1], qfma(TA[i][0], w[0], f->b[i]))));
        e->eta[i] = qfma(Um[i][3], z[3], qfma(Um[i][2], z[2], qfma(Um[i][1], z[1], qfma(Um[i][0], z[0], e->eta[i]))));
    }
    {
        double Y[4][4];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                Y[i][j] = qfma(Um[i][3], f->J[sidx(3, j)], qfma(Um[i][2], f->J[sidx(2, j)], qfma(Um[i][1], f->J[sidx(1, j)], Um[i][0] * f->J[sidx(0, j)])));
        for (int i = 0; i < 4; ++i)
            for (int j = i; j < 4; ++j)
                e->J[sidx(i, j)] = qfma(Y[i][3], e->A[12 + j], qfma(Y[i][2], e->A[8 + j], qfma(Y[i][1], e->A[4 + j], qfma(Y[i][0], e->A[j], e->J[sidx(i, j)]))));
    }
    {
        double X[4][4];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                X[i][j] = qfma(TA[i][3], e->C[sidx(3, j)], qfma(TA[i][2], e->C[sidx(2, j)], qfma(TA[i][1], e->C[sidx(1, j)], TA[i][0] * e->C[sidx(0, j)])));
        for (int i = 0; i < 4; ++i)
            for (int j = i; j < 4; ++j)
                e->C[sidx(i, j)] = qfma(X[i][3], f->A[4 * j + 3], qfma(X[i][2], f->A[4 * j + 2], qfma(X[i][1], f->A[4 * j + 1], qfma(X[i][0], f->A[4 * j], f->C[sidx(i, j)]))));
    }
    for (int j = 0; j < 4; ++j) {
        const double c0 = e->A[j], c1 = e->A[4 + j], c2 = e->A[8 + j], c3 = e->A[12 + j];
        for (int i = 0; i < 4; ++i) e->A[4 * i + j] = qfma(TA[i][3], c3, qfma(TA[i][2], c2, qfma(TA[i][1], c1, TA[i][0] * c0)));
    }
}

/* developer check of the element arithmetic (scripts/ubench/velem_check.hip runs the same on the
 * device): per case two stages (a, B, bb, Hx, Hu, gx, gu: 30 doubles each) and a terminal (We, g: 8);
 * out = e0 (x) e1, then (x) the terminal element (We[0] > 0) or (x) e1 (x) e0 (We[0] <= 0): 2 x 44 doubles */
void tw_velem_check(int32_t n, const double *in, double *out)
{
    for (int i = 0; i < n; ++i) {
        const double *c = in + (size_t)i * 68;
        tw_velem e, e1, t;
        velem_stage(c, c + 6, c + 14, c + 18, c + 22, c + 24, c + 28, &e);
        velem_stage(c + 30, c + 36, c + 44, c + 48, c + 52, c + 54, c + 58, &e1);
        velem_combine(&e, &e1);
        memcpy(out + (size_t)i * 88, &e, sizeof e);
        const double g6[6] = {c[64], c[65], c[66], c[67], 0.0, 0.0};
        if (c[60] > 0.0) {
            velem_terminal(c + 60, g6, &t);
        } else {   /* a general element on the right: the case's two stages combined in the other order */
            tw_velem u;
            velem_stage(c + 30, c + 36, c + 44, c + 48, c + 52, c + 54, c + 58, &t);
            velem_stage(c, c + 6, c + 14, c + 18, c + 22, c + 24, c + 28, &u);
            velem_combine(&t, &u);
        }
        velem_combine(&e, &t);
        memcpy(out + (size_t)i * 88 + 44, &e, sizeof e);
    }
}

/* the S = 2 factorisation: lane l combines its slots' elements, Hillis-Steele suffix levels over the
 * lanes, slot 1's suffix from the next lane's result; each slot then forms K, Rn, kk from its
 * successor's value function (ric_factor_step without the P update) */
static void factor_scan_s2(const tw_par *p, tw_stage *st, const double *hx3, double (*hu)[2], const double *gx3,
                           double (*gu)[2])
{
    const int N = p->N, L = p->L;
    tw_velem e[64], ne[64], e1[64];
    for (int l = 0; l < L; ++l) {
        const int k0 = 2 * l, k1 = k0 + 1;
        for (int ls = 0; ls < 2; ++ls) {
            const int k = k0 + ls;
            tw_velem *d = ls == 0 ? e + l : e1 + l;
            if (k < N) {
                const tw_stage *s = st + k;
                const double Hx[4] = {p->tau * p->W[0], p->tau * p->W[1], p->tau * p->W[2], hx3[k]};
                const double gx[4] = {s->g[0], s->g[1], s->g[2], gx3[k]};
                velem_stage(s->a, s->B, s->bb, Hx, hu[k], gx, gu[k], d);
            } else if (k == N) {
                velem_terminal(p->We, st[N].g, d);
            }
        }
        if (k1 <= N) velem_combine(e + l, e1 + l);
    }
    for (int off = 1; off < L; off <<= 1) {
        for (int l = 0; l < L; ++l) {
            ne[l] = e[l];
            if (l + off < L) velem_combine(ne + l, e + l + off);
        }
        memcpy(e, ne, sizeof(tw_velem) * (size_t)L);
    }
    for (int l = 0; l < L; ++l) {
        const int k0 = 2 * l, k1 = k0 + 1;
        if (k1 < N) {
            const tw_velem *f = e + l + 1;
            velem_combine(e1 + l, f);
            double Pn[10], pn[4];
            for (int q = 0; q < 10; ++q) Pn[q] = f->J[q];
            for (int q = 0; q < 4; ++q) pn[q] = -f->eta[q];
            tw_stage *s = st + k1;
            const double gx[4] = {s->g[0], s->g[1], s->g[2], gx3[k1]};
            const double Hx[4] = {p->tau * p->W[0], p->tau * p->W[1], p->tau * p->W[2], hx3[k1]};
            ric_factor_step(s->a, s->B, s->bb, Hx, hu[k1], gx, gu[k1], Pn, pn, s->K, s->Rn, s->kk, 0);
        }
        if (k0 < N) {
            double Pn[10], pn[4];
            for (int q = 0; q < 10; ++q) Pn[q] = e1[l].J[q];
            for (int q = 0; q < 4; ++q) pn[q] = -e1[l].eta[q];
            tw_stage *s = st + k0;
            const double gx[4] = {s->g[0], s->g[1], s->g[2], gx3[k0]};
            const double Hx[4] = {p->tau * p->W[0], p->tau * p->W[1], p->tau * p->W[2], hx3[k0]};
            ric_factor_step(s->a, s->B, s->bb, Hx, hu[k0], gx, gu[k0], Pn, pn, s->K, s->Rn, s->kk, 0);
        }
    }
}

/* riccati_solve: factor (predictor) or the corrector's difference recursion, then the forward pass
 * writing the bounded solution components into VA (factor) / VN (corrector) */
/* mfma4: D = X'Y + C for 4x4 blocks held row-major (X read transposed, as the kernel's A operand);
 * every element is one fused multiply-add chain over k = 0..3 starting from C, the order of
 * v_mfma_f64_4x4x4_4b_f64 (scripts/ubench/mfma_f64_round.hip: 1 920 000 of 1 920 000 elements) */
static void mfma4(const double X[16], const double Y[16], const double C[16], double D[16])
{
    double T[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double d = C[4 * i + j];
            for (int k = 0; k < 4; ++k) d = fma(X[4 * k + i], Y[4 * k + j], d);
            T[4 * i + j] = d;
        }
    memcpy(D, T, sizeof T);
}

/* factor_walk_mfma (qsp_solver.hip): the factorisation of one stage per lane on the matrix cores.
 * The value function is a full symmetric 4x4 P and p replicated across the columns; a step is
 * T1 = P'A, T2 = P'[B | b | 0] + [0 | 0 | p | 0], Q = A'T1 + Hx, Y = G'T1, Z = G'T2 + [Hu | gu],
 * q = A'pp + gx, K = (-adj R~)'S~ / det, P = Y'K + Q (upper triangle; lower = K'Y + Q' elementwise,
 * its exact transpose), p = K'[r~] + q; the stage keeps K and forms -R~^-1 and kk from Z's R~, r~. */
static void factor_walk_mfma(const tw_par *p, tw_stage *st, const double *hx3, double (*hu)[2], const double *gx3,
                             double (*gu)[2])
{
    const int N = p->N;
    static const double zero[16] = {0};
    double P[16] = {0}, pv[16];
    for (int i = 0; i < 4; ++i) P[5 * i] = p->We[i];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) pv[4 * r + c] = st[N].g[r];
    for (int k = N - 1; k >= 0; --k) {
        tw_stage *s = st + k;
        const double *a = s->a;
        const double Am[16] = {1.0, 0.0, a[0], a[1], 0.0, 1.0, a[2], a[3], 0.0, 0.0, 1.0, a[4], 0.0, 0.0, 0.0, a[5]};
        const double gx[4] = {s->g[0], s->g[1], s->g[2], gx3[k]};
        double G2[16], CH[16] = {0}, CZ[16] = {0}, GQ[16], C2[16] = {0}, PP[16];
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) {
                G2[4 * r + c] = c < 2 ? s->B[2 * r + c] : (c == 2 ? s->bb[r] : 0.0);
                GQ[4 * r + c] = gx[r];
            }
        CH[0] = p->tau * p->W[0];
        CH[5] = p->tau * p->W[1];
        CH[10] = p->tau * p->W[2];
        CH[15] = hx3[k];
        CZ[0] = hu[k][0];
        CZ[5] = hu[k][1];
        CZ[2] = gu[k][0];
        CZ[6] = gu[k][1];
        for (int r = 0; r < 4; ++r) C2[4 * r + 2] = pv[4 * r + 2];
        double T1[16], T2[16], Q[16], Y[16], Z[16], QV[16], KA[16], Kf[16];
        mfma4(P, Am, zero, T1);
        mfma4(P, G2, C2, T2);
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) PP[4 * r + c] = T2[4 * r + 2];
        mfma4(Am, T1, CH, Q);
        mfma4(G2, T1, zero, Y);
        mfma4(G2, T2, CZ, Z);
        mfma4(Am, PP, GQ, QV);
        const double R00 = Z[0], R01 = Z[1], rt0 = Z[2], R11 = Z[5], rt1 = Z[6];
        const double idet = rcp(qfma(R00, R11, -(R01 * R01)));
        double Xa[16] = {0};
        Xa[0] = -R11; Xa[1] = R01; Xa[4] = R01; Xa[5] = -R00;
        mfma4(Xa, Y, zero, KA);
        for (int q = 0; q < 16; ++q) Kf[q] = KA[q] * (q < 8 ? idet : 0.0);
        for (int q = 0; q < 8; ++q) s->K[q] = Kf[q];
        s->Rn[0] = (-R11) * idet;
        s->Rn[1] = R01 * idet;
        s->Rn[2] = (-R00) * idet;
        s->kk[0] = qfma(s->Rn[1], rt1, s->Rn[0] * rt0);
        s->kk[1] = qfma(s->Rn[2], rt1, s->Rn[1] * rt0);
        if (k > 0) {
            /* P = Q~ + S~'K keeps its upper triangle; the lower one is the same products transposed
             * (K'S~ + Q~', with Q~' = T1'A + Hx: bit for bit the transposes), so P stays symmetric as the
             * lane walk's */
            double RT[16] = {0}, QT[16], PT[16];
            for (int c = 0; c < 4; ++c) { RT[c] = rt0; RT[4 + c] = rt1; }
            mfma4(T1, Am, CH, QT);
            mfma4(Y, Kf, Q, P);
            mfma4(Kf, Y, QT, PT);
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < r; ++c) P[4 * r + c] = PT[4 * r + c];
            mfma4(Kf, RT, QV, pv);
        }
    }
}

static void riccati_solve(const tw_par *p, tw_stage *st, const double dx0[4], int factor)
{
    const int N = p->N, S = p->S;
    double P[10], pv[4];
    double hx3[TW_MAX_SLOTS], hu[TW_MAX_SLOTS][2], gx3[TW_MAX_SLOTS], gu[TW_MAX_SLOTS][2];
    for (int k = 0; k < N; ++k) {
        const tw_stage *s = st + k;
        if (factor) {
            hx3[k] = qfma(p->tau, p->W[3], s->hg[0]);
            hu[k][0] = qfma(p->tau, p->W[4], s->hg[1]);
            hu[k][1] = qfma(p->tau, p->W[5], s->hg[2]);
            gx3[k] = s->g[3] + s->hg[3];
            gu[k][0] = s->g[4] + s->hg[4];
            gu[k][1] = s->g[5] + s->hg[5];
        } else {
            gx3[k] = s->hg[3];
            gu[k][0] = s->hg[4];
            gu[k][1] = s->hg[5];
        }
    }
    if (S == 1 && !factor) {
        /* closed-loop difference walk: dp_k = e_k + (A + B K)' dp_{k+1}, dp_N = 0; each stage k
         * forms kk += Rn (dg_u + B' dp_{k+1}) from the dp that reaches it */
        double dp[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k = N - 1; k >= 0; --k) {
            tw_stage *s = st + k;
            double rt[2];
            for (int i = 0; i < 2; ++i)
                rt[i] = qfma(s->B[6 + i], dp[3], qfma(s->B[4 + i], dp[2], qfma(s->B[2 + i], dp[1], qfma(s->B[i], dp[0], gu[k][i]))));
            s->kk[0] = qfma(s->Rn[1], rt[1], qfma(s->Rn[0], rt[0], s->kk[0]));
            s->kk[1] = qfma(s->Rn[2], rt[1], qfma(s->Rn[1], rt[0], s->kk[1]));
            if (k >= 1) {
                double e[4], n[4];
                for (int i = 0; i < 4; ++i) e[i] = qfma(s->K[4 + i], gu[k][1], qfma(s->K[i], gu[k][0], i == 3 ? gx3[k] : 0.0));
                for (int i = 0; i < 4; ++i)
                    n[i] = qfma(s->M[12 + i], dp[3], qfma(s->M[8 + i], dp[2], qfma(s->M[4 + i], dp[1], qfma(s->M[i], dp[0], e[i]))));
                memcpy(dp, n, sizeof dp);
            }
        }
    } else if (S == 2 && !factor) {
        delta_scan_s2(p, st, gx3, gu);
    } else if (S == 2 && factor && p->factor_scan) {
        factor_scan_s2(p, st, hx3, hu, gx3, gu);
    } else if (factor && p->mfma_walk) {
        factor_walk_mfma(p, st, hx3, hu, gx3, gu);
    } else {
        if (factor) {
            for (int i = 0; i < 10; ++i) P[i] = 0.0;
            P[0] = p->We[0]; P[4] = p->We[1]; P[7] = p->We[2]; P[9] = p->We[3];
            for (int i = 0; i < 4; ++i) pv[i] = st[N].g[i];
        } else {
            for (int i = 0; i < 4; ++i) pv[i] = 0.0;
        }
        for (int k = N - 1; k >= 0; --k) {
            tw_stage *s = st + k;
            if (factor) {
                const double gx[4] = {s->g[0], s->g[1], s->g[2], gx3[k]};
                const double Hx[4] = {p->tau * p->W[0], p->tau * p->W[1], p->tau * p->W[2], hx3[k]};
                ric_factor_step(s->a, s->B, s->bb, Hx, hu[k], gx, gu[k], P, pv, s->K, s->Rn, s->kk, k > 0);
            } else {
                double dkk[2];
                ric_delta_step(s->a, s->B, gx3[k], gu[k], s->K, s->Rn, pv, dkk);
                s->kk[0] += dkk[0];
                s->kk[1] += dkk[1];
            }
        }
    }
    double dx[4] = {dx0[0], dx0[1], dx0[2], dx0[3]};
    if (S == 1) {
        if (factor) {
            for (int k = 0; k < N; ++k) {
                tw_stage *s = st + k;
                const double *a = s->a, *B = s->B, *K = s->K;
                const double Am[4][4] = {{1.0, 0.0, a[0], a[1]}, {0.0, 1.0, a[2], a[3]}, {0.0, 0.0, 1.0, a[4]},
                                         {0.0, 0.0, 0.0, a[5]}};
                for (int i = 0; i < 4; ++i)
                    for (int q = 0; q < 4; ++q) s->M[4 * i + q] = qfma(B[2 * i + 1], K[4 + q], qfma(B[2 * i], K[q], Am[i][q]));
            }
        }
        for (int k = 0; k < N; ++k) {
            tw_stage *s = st + k;
            const double *K = s->K;
            double *out = factor ? s->VA : s->VN;
            out[0] = dx[3];
            out[1] = qfma(K[3], dx[3], qfma(K[2], dx[2], qfma(K[1], dx[1], qfma(K[0], dx[0], s->kk[0]))));
            out[2] = qfma(K[7], dx[3], qfma(K[6], dx[2], qfma(K[5], dx[1], qfma(K[4], dx[0], s->kk[1]))));
            double cv[4], n[4];
            for (int i = 0; i < 4; ++i) cv[i] = qfma(s->B[2 * i + 1], s->kk[1], qfma(s->B[2 * i], s->kk[0], s->bb[i]));
            for (int i = 0; i < 4; ++i)
                n[i] = qfma(s->M[4 * i + 3], dx[3], qfma(s->M[4 * i + 2], dx[2], qfma(s->M[4 * i + 1], dx[1], qfma(s->M[4 * i], dx[0], cv[i]))));
            memcpy(dx, n, sizeof dx);
        }
        return;
    }
    if (S == 2) {
        forward_scan_s2(p, st, dx0, factor);
        return;
    }
    for (int k = 0; k < N; ++k) {
        tw_stage *s = st + k;
        double du[2];
        du[0] = qfma(s->K[3], dx[3], qfma(s->K[2], dx[2], qfma(s->K[1], dx[1], qfma(s->K[0], dx[0], s->kk[0]))));
        du[1] = qfma(s->K[7], dx[3], qfma(s->K[6], dx[2], qfma(s->K[5], dx[1], qfma(s->K[4], dx[0], s->kk[1]))));
        double *out = factor ? s->VA : s->VN;
        out[0] = dx[3];
        out[1] = du[0];
        out[2] = du[1];
        dyn_step(s->a, s->B, s->bb, du, dx);
    }
}

enum { QP_EXIT_CONV = 0, QP_EXIT_CAP = 1, QP_EXIT_STALL = 2, QP_EXIT_DIVERGED = 3 };

/* qp_ipm: slots 0 .. L*S-1 of st are filled (a, B, bb, g, v; padding slots past N hold the terminal
 * stage's data as the kernel loads them).  Returns the iterations taken; *exit why it stopped. */
static int qp_ipm(const tw_par *p, tw_stage *st, const double dx0[4], int *exit, int skip)
{
    const int N = p->N, S = p->S, L = p->L;
    const double m = 2.0 * (3.0 * N - (p->s0_bound ? 0.0 : 1.0));
    double r0 = 0.0, rg0 = 0.0, rb0 = 0.0;
    for (int k = 0; k < L * S; ++k) {
        tw_stage *s = st + k;
        double lo[3], hi[3], gl[3];
        bnd_lohi(p, s, lo, hi);
        for (int j = 0; j < 3; ++j) {
            const int act = bnd_act(p, k, j);
            const double tl = fmax(-lo[j], p->t_min), th = fmax(hi[j], p->t_min);
            if (act) r0 = fmax(r0, fmax(tl + lo[j], th - hi[j]));
            const double rl = rcp(tl), rh = rcp(th);
            s->t[2 * j] = act ? tl : 1.0;
            s->t[2 * j + 1] = act ? th : 1.0;
            s->rt[2 * j] = act ? rl : 1.0;
            s->rt[2 * j + 1] = act ? rh : 1.0;
            s->lm[2 * j] = act ? p->mu0 * rl : 0.0;
            s->lm[2 * j + 1] = act ? p->mu0 * rh : 0.0;
            gl[j] = act ? qfma(p->mu0, rh, -(p->mu0 * rl)) : 0.0;
        }
        if (k <= N) {
            rg0 = fmax(rg0, fmax(fmax(fabs(s->g[0]), fabs(s->g[1])), fmax(fabs(s->g[2]), fabs(s->g[3] + gl[0]))));
            rg0 = fmax(rg0, fmax(fabs(s->g[4] + gl[1]), fabs(s->g[5] + gl[2])));
            rb0 = fmax(rb0, fmax(fmax(fabs(s->bb[0]), fabs(s->bb[1])), fmax(fabs(s->bb[2]), fabs(s->bb[3]))));
            if (k == 0) rb0 = fmax(rb0, fmax(fmax(fabs(dx0[0]), fabs(dx0[1])), fmax(fabs(dx0[2]), fabs(dx0[3]))));
        }
        s->du[0] = s->du[1] = 0.0;
        for (int q = 0; q < 3; ++q) s->VA[q] = s->VN[q] = 0.0;
    }
    double rs_stop = p->res_stop / r0;
    const double rs_g = p->qp_tol_stat / rg0, rs_b = p->qp_tol_eq / rb0;
    rs_stop = rs_g < rs_stop ? rs_g : rs_stop;
    rs_stop = rs_b < rs_stop ? rs_b : rs_stop;
    double rscale = 1.0;
    int nit = 0, stall = 0, conv = 0, stalled = 0, div = 0;
    double lane[64], num[64], den[64];
    for (int it = 0;; ++it) {
        for (int l = 0; l < L; ++l) {
            double acc = 0.0;
            for (int ls = 0; ls < S; ++ls)
                for (int q = 0; q < 6; ++q) acc = qfma(st[l * S + ls].t[q], st[l * S + ls].lm[q], acc);
            lane[l] = acc;
        }
        const double mu = group_sum(lane, L) / m;
        div = !skip && !(mu < p->qp_mu_max);
        conv = !div && (skip || (!(mu >= p->mu_stop) && !(rscale >= rs_stop)));
        stalled = !conv && !div && p->qp_stall_iters > 0 && stall >= p->qp_stall_iters;
        const int done = conv || div || stalled;
        if (it == p->qp_iters || done) break;
        nit++;
        /* predictor */
        for (int k = 0; k < L * S; ++k) barrier_terms(p, st + k, k);
        riccati_solve(p, st, dx0, 1);
        for (int l = 0; l < L; ++l) {
            num[l] = 1.0;
            den[l] = 1.0;
            for (int ls = 0; ls < S; ++ls) affine_dirs(p, st + l * S + ls, l * S + ls, num + l, den + l);
            lane[l] = num[l] / den[l];
        }
        const double aa = group_min(lane, L);
        for (int l = 0; l < L; ++l) {
            double ma = 0.0;
            for (int ls = 0; ls < S; ++ls) ma = affine_mu_part(p, st + l * S + ls, l * S + ls, aa, ma);
            lane[l] = ma;
        }
        const double mua = group_sum(lane, L) / m;
        const double r = mua / mu;
        const double sg = fmax(r * r * r, p->sigma_min);
        const double smu = sg * mu;
        /* corrector */
        for (int k = 0; k < L * S; ++k) corrector_terms(p, st + k, k, smu);
        riccati_solve(p, st, dx0, 0);
        for (int l = 0; l < L; ++l) {
            num[l] = 1.0;
            den[l] = p->frac;
            for (int ls = 0; ls < S; ++ls) corrector_dirs(p, st + l * S + ls, l * S + ls, smu, num + l, den + l);
            lane[l] = num[l] / den[l];
        }
        double alpha = p->frac * group_min(lane, L);
        alpha = fmin(alpha, 1.0);
        stall = alpha < p->qp_stall_alpha ? stall + 1 : 0;
        rscale *= 1.0 - alpha;
        for (int k = 0; k < L * S; ++k) {
            tw_stage *s = st + k;
            apply_step(s, alpha);
            s->du[0] = qfma(alpha, s->VN[1] - s->du[0], s->du[0]);
            s->du[1] = qfma(alpha, s->VN[2] - s->du[1], s->du[1]);
        }
    }
    *exit = conv ? QP_EXIT_CONV : (div ? QP_EXIT_DIVERGED : (stalled ? QP_EXIT_STALL : QP_EXIT_CAP));
    return nit;
}

/* qp_rollout: state step of the damped QP solution */
static void qp_rollout(const tw_par *p, tw_stage *st, const double dx0[4])
{
    double dx[4] = {dx0[0], dx0[1], dx0[2], dx0[3]};
    for (int k = 0; k <= p->N; ++k) {
        memcpy(st[k].dxs, dx, sizeof dx);
        if (k < p->N) dyn_step(st[k].a, st[k].B, st[k].bb, st[k].du, dx);
    }
}

/* adjoint_step */
static void adjoint_step(const tw_par *p, const double a[6], const double dx[4], const double g[6], double dlam_s,
                         double pi[4])
{
    double np[4];
    np[0] = qfma(p->tau * p->W[0], dx[0], g[0]) + pi[0];
    np[1] = qfma(p->tau * p->W[1], dx[1], g[1]) + pi[1];
    np[2] = qfma(p->tau * p->W[2], dx[2], g[2]) + (qfma(a[2], pi[1], a[0] * pi[0]) + pi[2]);
    np[3] = qfma(p->tau * p->W[3], dx[3], g[3]) + qfma(a[5], pi[3], qfma(a[4], pi[2], qfma(a[3], pi[1], a[1] * pi[0])));
    np[3] += dlam_s;
    memcpy(pi, np, sizeof np);
}

/* the QP's dynamics multipliers pi_k (k = 0..N-1) by the adjoint recursion (qp_adjoint_store) */
static void qp_adjoint(const tw_par *p, const tw_stage *st, double *PI /* N x 4 */)
{
    const int N = p->N;
    double pi[4];
    for (int i = 0; i < 4; ++i) pi[i] = qfma(p->We[i], st[N].dxs[i], st[N].g[i]);
    for (int k = N - 1; k >= 0; --k) {
        memcpy(PI + 4 * k, pi, sizeof pi);
        if (k >= 1) adjoint_step(p, st[k].a, st[k].dxs, st[k].g, st[k].lm[1] - st[k].lm[0], pi);
    }
}

/* ================================================================== one instance's SQP */
typedef struct {
    tw_stage st[TW_MAX_SLOTS];
    double nlpPI[TW_MAX_N * 4], LAM[TW_MAX_N * 6], NU[TW_MAX_N * 4], ETA[TW_MAX_N * 6];
    double qPI[TW_MAX_N * 4];
    double kkt[8];   /* diagnostics of the last NLP KKT test (nlp_mode 1): see tw_set_kkt_diag */
} tw_ws;

/* KKT diagnostics (nlp_mode 1), per lane 8 doubles, as or_set_kkt_diag: u-, x- and terminal
 * stationarity, equality, inequality, complementarity residuals of the last KKT test, its SQP
 * iteration, the last line-search step length.  NULL: off. */
static double *g_kkt_diag = NULL;
void tw_set_kkt_diag(double *buf) { g_kkt_diag = buf; }

/* stage data of slot k from the SQP iterate (qp_step_kernel's LIN block) */
static void load_stage(const tw_par *p, const tw_shape *sh, tw_stage *s, int k, const double *X, const double *U,
                       const double *yref, const double *ye, int lin_live)
{
    const int N = p->N;
    const int kc = k <= N ? k : N, ku = k < N ? k : N - 1;
    if (kc < N && lin_live) {
        const double *xk = X + 4 * kc, *uk = U + 2 * kc;
        lin Ln;
        rk4(sh, p->Ts, xk, uk, &Ln, 1);
        const double *yr = yref + 6 * kc;
        memcpy(s->a, Ln.a, sizeof s->a);
        memcpy(s->B, Ln.B, sizeof s->B);
        for (int q = 0; q < 4; ++q) s->bb[q] = Ln.xn[q] - X[4 * (kc + 1) + q];
        for (int q = 0; q < 4; ++q) s->g[q] = p->tau * p->W[q] * (xk[q] - yr[q]);
        for (int q = 0; q < 2; ++q) s->g[4 + q] = p->tau * p->W[4 + q] * (uk[q] - yr[4 + q]);
    } else {
        memset(s->a, 0, sizeof s->a);
        memset(s->B, 0, sizeof s->B);
        memset(s->bb, 0, sizeof s->bb);
        for (int q = 0; q < 4; ++q) s->g[q] = p->We[q] * (X[4 * N + q] - ye[q]);
        s->g[4] = s->g[5] = 0.0;
    }
    s->v[0] = X[4 * kc + 3];
    s->v[1] = U[2 * ku];
    s->v[2] = U[2 * ku + 1];
}

/* nlp_converged: KKT residuals of the NLP iterate against tol_* (nlp_mode 1) */
static int nlp_converged(const tw_par *p, const tw_stage *st, const double *PI, const double *LAM, double *kkt)
{
    const int N = p->N;
    double rs = 0.0, re = 0.0, ri = 0.0, rc = 0.0, ru = 0.0, rx = 0.0, rt = 0.0;
    for (int k = 0; k <= N; ++k) {
        const tw_stage *s = st + k;
        const double zero[6] = {0, 0, 0, 0, 0, 0};
        const double *PIk = k < N ? PI + 4 * k : zero, *LAMk = k < N ? LAM + 6 * k : zero;
        const double *PIp = k >= 1 ? PI + 4 * (k - 1) : zero;
        if (k < N) {
            const double *B = s->B, *a = s->a;
            for (int i = 0; i < 2; ++i) {
                const double r = (s->g[4 + i] + qfma(B[6 + i], PIk[3], qfma(B[4 + i], PIk[2], qfma(B[2 + i], PIk[1], B[i] * PIk[0])))) +
                                 (LAMk[2 * (1 + i) + 1] - LAMk[2 * (1 + i)]);
                rs = fmax(rs, fabs(r));
                ru = fmax(ru, fabs(r));
            }
            if (k >= 1) {
                const double at[4] = {PIk[0], PIk[1], qfma(a[2], PIk[1], a[0] * PIk[0]) + PIk[2],
                                      qfma(a[5], PIk[3], qfma(a[4], PIk[2], qfma(a[3], PIk[1], a[1] * PIk[0])))};
                for (int i = 0; i < 4; ++i) {
                    double r = s->g[i] - PIp[i] + at[i];
                    if (i == 3) r += LAMk[1] - LAMk[0];
                    rs = fmax(rs, fabs(r));
                    rx = fmax(rx, fabs(r));
                }
            }
            for (int i = 0; i < 4; ++i) re = fmax(re, fabs(s->bb[i]));
            for (int j = 0; j < 3; ++j) {
                if (j == 0 && k == 0 && !p->s0_bound) continue;
                const double sl = s->v[j] - p->lh[j], sh_ = p->uh[j] - s->v[j];
                ri = fmax(ri, fmax(-sl, -sh_));
                rc = fmax(rc, fmax(fabs(LAMk[2 * j] * sl), fabs(LAMk[2 * j + 1] * sh_)));
            }
        } else {
            for (int i = 0; i < 4; ++i) rs = fmax(rs, fabs(s->g[i] - PIp[i]));
            for (int i = 0; i < 4; ++i) rt = fmax(rt, fabs(s->g[i] - PIp[i]));
        }
    }
    kkt[0] = ru; kkt[1] = rx; kkt[2] = rt; kkt[3] = re; kkt[4] = ri; kkt[5] = rc;
    return rs < p->tol_stat && re < p->tol_eq && ri < p->tol_ineq && rc < p->tol_comp;
}

/* merit_stage */
static double merit_stage(const tw_par *p, int k, const double x[4], const double u[2], const double *yr,
                          const double *ye, const double def[4], const double nu[4], const double eta[6])
{
    if (k == p->N) {
        double s = 0.0;
        for (int i = 0; i < 4; ++i) { const double r = x[i] - ye[i]; s = qfma(p->We[i] * r, r, s); }
        return 0.5 * s;
    }
    double s = 0.0;
    for (int i = 0; i < 4; ++i) { const double r = x[i] - yr[i]; s = qfma(p->W[i] * r, r, s); }
    for (int i = 0; i < 2; ++i) { const double r = u[i] - yr[4 + i]; s = qfma(p->W[4 + i] * r, r, s); }
    double ph = 0.5 * p->tau * s;
    for (int i = 0; i < 4; ++i) ph = qfma(nu[i], fabs(def[i]), ph);
    const double v[3] = {x[3], u[0], u[1]};
    for (int j = 0; j < 3; ++j) {
        if (j == 0 && k == 0 && !p->s0_bound) continue;
        const double vl = p->lh[j] - v[j], vh = v[j] - p->uh[j];
        if (vl > 0.0) ph = qfma(eta[2 * j], vl, ph);
        if (vh > 0.0) ph = qfma(eta[2 * j + 1], vh, ph);
    }
    return ph;
}

/* merit_ls_kernel for one instance (stages = lanes 0..N of its group) */
static void merit_ls(const tw_par *p, const tw_shape *sh, tw_ws *w, double *X, double *U, const double *yref,
                     const double *ye)
{
    const int N = p->N, L = N + 1;
    const tw_stage *st = w->st;
    double NUk[TW_MAX_N + 1][4], ETAk[TW_MAX_N + 1][6], dph[TW_MAX_N + 1], lane[64] = {0};
    double xk[TW_MAX_N + 1][4], uk[TW_MAX_N + 1][2], dxk[TW_MAX_N + 1][4], duk[TW_MAX_N + 1][2];
    for (int k = 0; k <= N; ++k) {
        const int stg = k < N, ku = stg ? k : N - 1;
        for (int q = 0; q < 4; ++q) { xk[k][q] = X[4 * k + q]; dxk[k][q] = st[k].dxs[q]; }
        uk[k][0] = U[2 * ku];
        uk[k][1] = U[2 * ku + 1];
        duk[k][0] = stg ? st[k].du[0] : 0.0;
        duk[k][1] = stg ? st[k].du[1] : 0.0;
        for (int q = 0; q < 4; ++q) NUk[k][q] = stg ? w->NU[4 * k + q] : 0.0;
        for (int q = 0; q < 6; ++q) ETAk[k][q] = stg ? w->ETA[6 * k + q] : 0.0;
        if (stg) {
            for (int q = 0; q < 4; ++q) {
                const double a = fabs(w->qPI[4 * k + q]), wq = 0.5 * (NUk[k][q] + a);
                NUk[k][q] = a > wq ? a : wq;
            }
            for (int q = 0; q < 6; ++q) {
                const double a = fabs(st[k].lm[q]), wq = 0.5 * (ETAk[k][q] + a);
                ETAk[k][q] = a > wq ? a : wq;
            }
        }
        double d = 0.0;
        for (int i = 0; i < 4; ++i) d = qfma(st[k].g[i], dxk[k][i], d);
        if (stg) {
            d = qfma(st[k].g[5], duk[k][1], qfma(st[k].g[4], duk[k][0], d));
            for (int i = 0; i < 4; ++i) d = qfma(-NUk[k][i], fabs(st[k].bb[i]), d);
            const double v[3] = {xk[k][3], uk[k][0], uk[k][1]};
            for (int j = 0; j < 3; ++j) {
                if (j == 0 && k == 0 && !p->s0_bound) continue;
                const double lo = p->lh[j] - v[j], hi = p->uh[j] - v[j];
                if (lo > 0.0) d = qfma(-ETAk[k][2 * j], lo, d);
                if (hi < 0.0) d = qfma(ETAk[k][2 * j + 1], hi, d);
            }
        }
        dph[k] = d;
    }
    for (int k = 0; k <= N; ++k) {
        const int ku = k < N ? k : N - 1;
        lane[k] = merit_stage(p, k, xk[k], uk[k], yref + 6 * ku, ye, st[k].bb, NUk[k], ETAk[k]);
    }
    const double phi0 = group_sum(lane, L);
    for (int k = 0; k <= N; ++k) lane[k] = dph[k];
    const double dphi = group_sum(lane, L);
    double alpha = 1.0;
    for (;;) {
        double xt[TW_MAX_N + 1][4], ut[TW_MAX_N + 1][2];
        for (int k = 0; k <= N; ++k) {
            for (int q = 0; q < 4; ++q) xt[k][q] = qfma(alpha, dxk[k][q], xk[k][q]);
            ut[k][0] = qfma(alpha, duk[k][0], uk[k][0]);
            ut[k][1] = qfma(alpha, duk[k][1], uk[k][1]);
        }
        for (int k = 0; k <= N; ++k) {
            double def[4] = {0.0, 0.0, 0.0, 0.0};
            if (k < N) {
                lin Lt;
                rk4(sh, p->Ts, xt[k], ut[k], &Lt, 0);
                for (int q = 0; q < 4; ++q) def[q] = Lt.xn[q] - xt[k + 1][q];
            }
            const int ku = k < N ? k : N - 1;
            lane[k] = merit_stage(p, k, xt[k], ut[k], yref + 6 * ku, ye, def, NUk[k], ETAk[k]);
        }
        const double phi = group_sum(lane, L);
        if (phi <= qfma(p->ls_eps * alpha, dphi, phi0)) break;
        const double an = alpha * p->ls_alpha_red;
        if (an < p->ls_alpha_min) break;
        alpha = an;
    }
    w->kkt[7] = alpha;
    for (int k = 0; k <= N; ++k) {
        for (int q = 0; q < 4; ++q) X[4 * k + q] = qfma(alpha, dxk[k][q], xk[k][q]);
        if (k < N) {
            U[2 * k] = qfma(alpha, duk[k][0], uk[k][0]);
            U[2 * k + 1] = qfma(alpha, duk[k][1], uk[k][1]);
            for (int q = 0; q < 4; ++q) {
                const double pk = w->nlpPI[4 * k + q];
                w->nlpPI[4 * k + q] = qfma(alpha, w->qPI[4 * k + q] - pk, pk);
            }
            for (int q = 0; q < 6; ++q) {
                const double lk = w->LAM[6 * k + q];
                w->LAM[6 * k + q] = qfma(alpha, st[k].lm[q] - lk, lk);
            }
            memcpy(w->NU + 4 * k, NUk[k], sizeof(double) * 4);
            memcpy(w->ETA + 6 * k, ETAk[k], sizeof(double) * 6);
        }
    }
}

typedef struct {
    int status, sqp_iter, qp_iter, qp_capped, qp_stalled;
    int pi_written;
} tw_out;

/* launch_sqp for one instance between prologue and epilogue: X, U (the iterate), x0 (wx0), the
 * staged y_ref; PI_out (N x 4) receives the multipliers (nlp_mode 0: the last successful QP's,
 * shifted when `shift`; nlp_mode 1: the NLP iterate's, written by the epilogue).  PI_in: the
 * initial dynamics multipliers (nlp_mode 1; NULL: zeros). */
static void sqp_solve(const tw_par *p, const tw_shape *sh, tw_ws *w, const double x0[4], const double *yref,
                      const double *ye, double *X, double *U, const double *PI_in, double *PI_out, int shift,
                      int wdone0, tw_out *o)
{
    const int N = p->N, S = p->S, L = p->L;
    int wdone = wdone0;   /* 0 running, 1 converged (nlp 1), 2 non-finite QP, 3 infeasible s0, 4 diverged QP */
    o->sqp_iter = 0;
    o->qp_iter = 0;
    o->qp_capped = 0;
    o->qp_stalled = 0;
    o->pi_written = 0;
    memset(w->kkt, 0, sizeof w->kkt);
    if (p->nlp_mode == 1) {
        for (int k = 0; k < N; ++k)
            for (int q = 0; q < 4; ++q) w->nlpPI[4 * k + q] = PI_in ? PI_in[4 * k + q] : 0.0;
        memset(w->LAM, 0, sizeof(double) * 6 * N);
        memset(w->NU, 0, sizeof(double) * 4 * N);
        memset(w->ETA, 0, sizeof(double) * 6 * N);
    }
    if (wdone0 == 3) o->sqp_iter = 0;
    for (int it = 0; it < p->sqp_iters; ++it) {
        const int was_done = wdone != 0;
        const int lin_live = !was_done;
        for (int k = 0; k < L * S; ++k) load_stage(p, sh, w->st + k, k, X, U, yref, ye, lin_live);
        double dx0[4];
        for (int q = 0; q < 4; ++q) dx0[q] = x0[q] - X[q];
        int skip = was_done;
        if (p->nlp_mode == 1) {
            const int conv = !was_done && nlp_converged(p, w->st, w->nlpPI, w->LAM, w->kkt);
            if (!was_done) w->kkt[6] = it;
            skip = was_done || conv;
            if (conv) {
                wdone = 1;
                o->sqp_iter = it;
            }
        }
        if (skip && p->nlp_mode == 0) continue;   /* a stopped instance does nothing in nlp_mode 0 */
        int exit;
        const int nit = qp_ipm(p, w->st, dx0, &exit, skip);
        qp_rollout(p, w->st, dx0);
        int failed = 0;
        if (!skip) {
            if (exit == QP_EXIT_CAP) o->qp_capped++;
            if (exit == QP_EXIT_STALL) o->qp_stalled++;
            int bad = 0;
            for (int k = 0; k <= N; ++k)
                for (int q = 0; q < 4; ++q) bad |= !isfinite(w->st[k].dxs[q]);
            for (int k = 0; k < N; ++k) bad |= !(isfinite(w->st[k].du[0]) && isfinite(w->st[k].du[1]));
            const int dv = exit == QP_EXIT_DIVERGED;
            failed = dv || bad;
            if (failed) {
                wdone = dv ? 4 : 2;
                o->sqp_iter = it;
            }
        }
        if (p->nlp_mode == 1) {
            o->qp_iter += nit;
            if (skip || failed) continue;
            qp_adjoint(p, w->st, w->qPI);
            merit_ls(p, sh, w, X, U, yref, ye);
            continue;
        }
        if (failed) continue;
        double pik[TW_MAX_N * 4];
        qp_adjoint(p, w->st, pik);
        for (int k = 0; k < N; ++k) {
            const int dst = shift ? (k >= 1 ? k - 1 : -1) : k;
            if (dst >= 0) memcpy(PI_out + 4 * dst, pik + 4 * k, sizeof(double) * 4);
        }
        if (shift) memcpy(PI_out + 4 * (N - 1), pik + 4 * (N - 1), sizeof(double) * 4);
        o->pi_written = 1;
        for (int k = 0; k <= N; ++k)
            for (int q = 0; q < 4; ++q) X[4 * k + q] += w->st[k].dxs[q];
        for (int k = 0; k < N; ++k) {
            U[2 * k] += w->st[k].du[0];
            U[2 * k + 1] += w->st[k].du[1];
        }
        o->qp_iter += nit;
    }
    /* epilogue_kernel (status; cost and outputs by the callers) */
    int bad = 0;
    for (int q = 0; q < 4 * (N + 1); ++q) bad |= !isfinite(X[q]);
    for (int q = 0; q < 2 * N; ++q) bad |= !isfinite(U[q]);
    if (wdone == 3 || wdone == 4) o->status = 4;
    else if (p->nlp_mode == 1) o->status = (bad || wdone == 2) ? 1 : (wdone == 1 ? 0 : 2);
    else o->status = (bad || wdone == 2) ? 1 : 0;
    if (wdone == 0) o->sqp_iter = p->sqp_iters;
    if (p->nlp_mode == 1) {
        for (int k = 0; k < N; ++k) {
            const int src = shift ? (k + 1 < N ? k + 1 : N - 1) : k;
            memcpy(PI_out + 4 * k, w->nlpPI + 4 * src, sizeof(double) * 4);
        }
        o->pi_written = 1;
    }
}

static double epilogue_cost(const tw_par *p, const double *X, const double *U, const double *yref, const double *ye)
{
    const int N = p->N;
    double cost = 0.0;
    for (int k = 0; k < N; ++k) {
        double s = 0.0;
        for (int q = 0; q < 4; ++q) { const double r = X[4 * k + q] - yref[6 * k + q]; s = qfma(p->W[q] * r, r, s); }
        for (int q = 0; q < 2; ++q) { const double r = U[2 * k + q] - yref[6 * k + 4 + q]; s = qfma(p->W[4 + q] * r, r, s); }
        cost = qfma(0.5 * p->tau, s, cost);
    }
    double s = 0.0;
    for (int q = 0; q < 4; ++q) { const double r = X[4 * N + q] - ye[q]; s = qfma(p->We[q] * r, r, s); }
    return qfma(0.5, s, cost);
}

static int s0_infeasible(const tw_par *p, double s0) { return p->s0_bound && !(s0 >= p->lh[0] && s0 <= p->uh[0]); }

/* ================================================================== exported API (as qsp_oracle.c) */
int tw_spline_eval(const int32_t *n_ctrl, const double *ctrl, const double *knots, const double *params,
                   int max_ctrl, int32_t n, const int32_t *shape_id, const double *s,
                   double *C, double *D, double *Dd, double *kappa)
{
    for (int32_t i = 0; i < n; ++i) {
        tw_shape sh;
        make_shape(&sh, n_ctrl, ctrl, knots, params, max_ctrl, shape_id[i], 0.0);
        spl e;
        spline_eval(&sh, s[i], &e);
        for (int c = 0; c < 2; ++c) { C[2 * i + c] = e.C[c]; D[2 * i + c] = e.D[c]; Dd[2 * i + c] = e.Dd[c]; }
        kappa[i] = angle_rate_of(&e);
    }
    return 0;
}

int tw_dynamics(const int32_t *n_ctrl, const double *ctrl, const double *knots, const double *params,
                int max_ctrl, int32_t n, const int32_t *shape_id, const double *x, const double *u, double *f, double *J)
{
    #pragma omp parallel for schedule(static)
    for (int32_t i = 0; i < n; ++i) {
        tw_shape sh;
        make_shape(&sh, n_ctrl, ctrl, knots, params, max_ctrl, shape_id[i], 0.0);
        dyn d;
        dynamics(&sh, x[4 * i + 2], x[4 * i + 3], u[2 * i], u[2 * i + 1], &d, 1);
        for (int r = 0; r < 4; ++r) {
            f[4 * i + r] = d.f[r];
            if (J) {
                double *Jr = J + (size_t)24 * i + 6 * r;
                Jr[0] = 0.0; Jr[1] = 0.0;
                Jr[2] = r < 2 ? d.Jth[r] : 0.0;
                Jr[3] = d.Js[r]; Jr[4] = d.Jun[r]; Jr[5] = d.Jut[r];
            }
        }
    }
    return 0;
}

int tw_rk4(const int32_t *n_ctrl, const double *ctrl, const double *knots, const double *params,
           int max_ctrl, int32_t n, const int32_t *shape_id, double h, const double *x, const double *u,
           double *xn, double *A, double *B)
{
    #pragma omp parallel for schedule(static)
    for (int32_t i = 0; i < n; ++i) {
        tw_shape sh;
        make_shape(&sh, n_ctrl, ctrl, knots, params, max_ctrl, shape_id[i], 0.0);
        lin L;
        rk4(&sh, h, x + 4 * i, u + 2 * i, &L, 1);
        const double Af[16] = {1.0, 0.0, L.a[0], L.a[1], 0.0, 1.0, L.a[2], L.a[3], 0.0, 0.0, 1.0, L.a[4], 0.0, 0.0, 0.0, L.a[5]};
        memcpy(A + (size_t)16 * i, Af, sizeof Af);
        memcpy(B + (size_t)8 * i, L.B, sizeof L.B);
        memcpy(xn + 4 * i, L.xn, sizeof L.xn);
    }
    return 0;
}

int tw_vbound(const int32_t *n_ctrl, const double *ctrl, const double *knots, const double *params,
              int max_ctrl, const or_opts *o, int32_t n, const int32_t *shape_id, const double *s, double *vb)
{
    for (int32_t i = 0; i < n; ++i) {
        tw_shape sh;
        make_shape(&sh, n_ctrl, ctrl, knots, params, max_ctrl, shape_id[i], 0.0);
        vb[i] = v_bound(&sh, o, s[i]);
    }
    return 0;
}

/* QP level (qsp_qp_solve): the same mapping onto the kernel's parameters -- tau = 1, W = the stage
 * Hessian, We = the terminal one, lh = 0, uh = hi - lo of the first lane's first stage, the bounded
 * components v = -lo through X/U, x0 = dx0 + X_0.  qp_status: 0 stop test met, 1 non-finite,
 * 2 cap, 3 infeasible stage-0 s, 4 stall, 5 diverged. */
int tw_qp_batch(const or_opts *o, int32_t nb, const double *A, const double *B, const double *b,
                const double *H, const double *g, const double *lo, const double *hi, const uint8_t *act,
                const double *dx0, double *dx, double *du, double *pi, double *lam, int32_t *iters, int32_t *qp_status)
{
    (void)act;
    const int N = o->N;
    if (N > TW_MAX_N) return -1;
    tw_par p;
    make_par(&p, o);
    p.tau = 1.0;
    for (int i = 0; i < 6; ++i) p.W[i] = H[i];
    for (int i = 0; i < 4; ++i) p.We[i] = H[6 * N + i];
    for (int j = 0; j < 3; ++j) { p.lh[j] = 0.0; p.uh[j] = hi[j] - lo[j]; }
    int fail = 0;
    #pragma omp parallel
    {
        tw_ws *w = (tw_ws *)malloc(sizeof(tw_ws));
        #pragma omp for schedule(dynamic, 4)
        for (int32_t l = 0; l < nb; ++l) {
            const int L = p.L, S = p.S;
            for (int k = 0; k < L * S; ++k) {
                tw_stage *s = w->st + k;
                const int kc = k <= N ? k : N, ku = k < N ? k : N - 1;
                memset(s, 0, sizeof *s);
                if (kc < N) {
                    const double *Ak = A + ((size_t)l * N + kc) * 16;
                    const double av[6] = {Ak[2], Ak[3], Ak[6], Ak[7], Ak[11], Ak[15]};
                    memcpy(s->a, av, sizeof av);
                    memcpy(s->B, B + ((size_t)l * N + kc) * 8, sizeof s->B);
                    memcpy(s->bb, b + ((size_t)l * N + kc) * 4, sizeof s->bb);
                    memcpy(s->g, g + (size_t)l * (6 * N + 4) + 6 * kc, sizeof s->g);
                } else {
                    memcpy(s->g, g + (size_t)l * (6 * N + 4) + 6 * N, sizeof(double) * 4);
                }
                /* v through the workspace X (s of stage kc; X_N's s is 0) and U (stage ku) */
                s->v[0] = kc < N ? -lo[((size_t)l * N + kc) * 3] : 0.0;
                s->v[1] = -lo[((size_t)l * N + ku) * 3 + 1];
                s->v[2] = -lo[((size_t)l * N + ku) * 3 + 2];
            }
            double x0w[4], d0[4];
            memcpy(x0w, dx0 + 4 * l, sizeof x0w);
            const double X0s = -lo[(size_t)l * N * 3];
            x0w[3] += X0s;
            for (int q = 0; q < 4; ++q) d0[q] = x0w[q] - (q == 3 ? X0s : 0.0);
            int exit;
            const int nit = qp_ipm(&p, w->st, d0, &exit, 0);
            qp_rollout(&p, w->st, d0);
            for (int k = 0; k <= N; ++k) memcpy(dx + ((size_t)l * (N + 1) + k) * 4, w->st[k].dxs, sizeof(double) * 4);
            for (int k = 0; k < N; ++k) {
                memcpy(du + ((size_t)l * N + k) * 2, w->st[k].du, sizeof(double) * 2);
                memcpy(lam + ((size_t)l * N + k) * 6, w->st[k].lm, sizeof(double) * 6);
            }
            qp_adjoint(&p, w->st, pi + (size_t)l * N * 4);
            if (iters) iters[l] = nit;
            int fin = 1;
            for (int q = 0; q < (N + 1) * 4; ++q) fin = fin && isfinite(dx[(size_t)l * (N + 1) * 4 + q]);
            for (int q = 0; q < N * 2; ++q) fin = fin && isfinite(du[(size_t)l * N * 2 + q]);
            const int infeas = p.s0_bound && (dx0[4 * l + 3] < lo[(size_t)l * N * 3] || dx0[4 * l + 3] > hi[(size_t)l * N * 3]);
            const int kst = exit == QP_EXIT_CONV ? 0 : (exit == QP_EXIT_CAP ? 2 : (exit == QP_EXIT_STALL ? 4 : 5));
            if (qp_status) qp_status[l] = !fin ? 1 : (infeas ? 3 : kst);
            if (!fin) {
                #pragma omp atomic write
                fail = 1;
            }
        }
        free(w);
    }
    return fail;
}

/* acados-level solve (qsp_solve): X, U = the initial guess in, the solution out; PI: init_pi in
 * (nlp_mode 1), the multipliers out (see sqp_solve); lam: the NLP's bound multipliers (nlp_mode 1). */
int tw_ocp_solve(const int32_t *n_ctrl, const double *ctrl, const double *knots, const double *params,
                 int max_ctrl, const or_opts *o, int32_t nb, const int32_t *shape_id,
                 const double *x0, const double *yref, const double *yref_e,
                 double *X, double *U, double *PI, double *lam, int32_t *status, int32_t *iters, int32_t *qp_iter,
                 double *cost, int nthreads, int32_t *qp_capped, int32_t *qp_stalled)
{
    const int N = o->N;
    if (N > TW_MAX_N) return -1;
    tw_par p;
    make_par(&p, o);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    #pragma omp parallel
    {
        tw_ws *w = (tw_ws *)malloc(sizeof(tw_ws));
        #pragma omp for schedule(dynamic, 1)
        for (int32_t i = 0; i < nb; ++i) {
            tw_shape sh;
            make_shape(&sh, n_ctrl, ctrl, knots, params, max_ctrl, shape_id[i], 0.0);
            double *Xi = X + (size_t)i * 4 * (N + 1), *Ui = U + (size_t)i * 2 * N, *Pi = PI + (size_t)i * 4 * N;
            const double *yr = yref + (size_t)i * 6 * N, *ye = yref_e + (size_t)i * 4;
            double PIin[TW_MAX_N * 4];
            memcpy(PIin, Pi, sizeof(double) * 4 * N);
            tw_out out;
            const int w0 = s0_infeasible(&p, x0[4 * i + 3]) ? 3 : 0;
            sqp_solve(&p, &sh, w, x0 + 4 * i, yr, ye, Xi, Ui, PIin, Pi, 0, w0, &out);
            status[i] = out.status;
            if (iters) iters[i] = out.sqp_iter;
            if (qp_iter) qp_iter[i] = out.qp_iter;
            if (qp_capped) qp_capped[i] = out.qp_capped;
            if (qp_stalled) qp_stalled[i] = out.qp_stalled;
            if (g_kkt_diag) memcpy(g_kkt_diag + (size_t)8 * i, w->kkt, sizeof w->kkt);
            if (lam) {
                if (p.nlp_mode == 1) memcpy(lam + (size_t)i * 6 * N, w->LAM, sizeof(double) * 6 * N);
                else memset(lam + (size_t)i * 6 * N, 0, sizeof(double) * 6 * N);
            }
            cost[i] = epilogue_cost(&p, Xi, Ui, yr, ye);
        }
        free(w);
    }
    return 0;
}

/* stage_yref_kernel: column index_time + k (1-based) of the table as set_reference_trajectory
 * builds it (D zero columns prepended, their u_t row copied from the first real column), clamped */
static void stage_yref(const double *traj, int32_t T, int32_t D, int32_t index_time, int N, double *yref, double *ye)
{
    for (int k = 0; k < N; ++k) {
        int idx = index_time + k;
        if (idx > T + D) idx = T + D;
        if (idx < 1) idx = 1;
        double *out = yref + 6 * k;
        if (idx <= D) {
            for (int c = 0; c < 5; ++c) out[c] = 0.0;
            out[5] = traj[5];
        } else {
            for (int c = 0; c < 6; ++c) out[c] = traj[(size_t)(idx - D - 1) * 6 + c];
        }
    }
    for (int c = 0; c < 4; ++c) ye[c] = yref[6 * (N - 1) + c];
}

/* NMPC_controller.solve on one lane (prologue_kernel in controller mode, the SQP, the epilogue's
 * shifted warm start).  Warm X/U/PI + valid in/out; returns the status. */
static int ctrl_lane(const tw_par *p, const tw_shape *sh, tw_ws *w, const double x0_in[4], const double *traj,
                     int32_t T, int32_t D, int32_t index_time, double *Xw, double *Uw, double *PIw, uint8_t *valid,
                     double u0[2], tw_out *out, double *cost)
{
    const int N = p->N;
    double yref[TW_MAX_N * 6], ye[4], X[(TW_MAX_N + 1) * 4], U[TW_MAX_N * 2];
    stage_yref(traj, T, D, index_time, N, yref, ye);
    double x0[4] = {x0_in[0], x0_in[1], x0_in[2], x0_in[3]};
    x0[3] = qfma(-sh->b, (x0[3] < 0.0) ? 1.0 : 0.0, mat_mod(x0[3], sh->b));
    const int cold = !*valid;
    for (int k = 0; k < N; ++k) {
        U[2 * k] = cold ? p->u_n_lb : Uw[2 * k];
        U[2 * k + 1] = cold ? 0.0 : Uw[2 * k + 1];
    }
    double xc[4] = {x0[0], x0[1], x0[2], x0[3]};
    const or_opts *oo = NULL;
    (void)oo;
    for (int k = 0; k <= N; ++k) {
        for (int c = 0; c < 4; ++c) X[4 * k + c] = xc[c];
        if (k == N) break;
        /* v_bound with the handle's controller parameters */
        const double sm = mat_mod(xc[3], sh->b);
        spl e;
        spline_eval(sh, sm, &e);
        const double ta = fabs(angle_rate_of(&e));
        double vb = p->v_alpha / (fabs(ta - p->t_angle0) + 0.0001) + p->d_v;
        vb = vb < p->u_t_ub ? vb : p->u_t_ub;
        const double ut_old = U[2 * k + 1];
        if (fabs(ut_old) > vb) {
            const double sgn = ut_old > 0.0 ? 1.0 : -1.0;
            U[2 * k + 1] = sgn * vb;
            U[2 * k] = U[2 * k + 1] * U[2 * k] / ut_old;
        }
        dyn d;
        dynamics(sh, xc[2], xc[3], U[2 * k], U[2 * k + 1], &d, 0);
        for (int c = 0; c < 4; ++c) xc[c] = qfma(p->Ts, d.f[c], xc[c]);
    }
    double PIin[TW_MAX_N * 4];
    memcpy(PIin, PIw, sizeof(double) * 4 * N);
    const int w0 = s0_infeasible(p, x0[3]) ? 3 : 0;
    sqp_solve(p, sh, w, x0, yref, ye, X, U, cold ? NULL : PIin, PIw, 1, w0, out);
    if (cost) *cost = epilogue_cost(p, X, U, yref, ye);
    u0[0] = U[0];
    u0[1] = U[1];
    for (int k = 0; k <= N; ++k) {
        const int src = (k + 1 <= N) ? k + 1 : N;
        memcpy(Xw + 4 * k, X + 4 * src, sizeof(double) * 4);
    }
    for (int k = 0; k < N; ++k) {
        const int src = (k + 1 < N) ? k + 1 : N - 1;
        memcpy(Uw + 2 * k, U + 2 * src, sizeof(double) * 2);
    }
    *valid = 1;
    return out->status;
}

int tw_controller_solve(const int32_t *n_ctrl, const double *ctrl, const double *knots, const double *params,
                        int max_ctrl, const or_opts *o, int32_t nb, const int32_t *shape_id,
                        const double *x0_in, const double *traj, int32_t T, const int32_t *index_time,
                        double *Xw, double *Uw, double *PIw, uint8_t *warm_valid,
                        double *u0, int32_t *status, int32_t *iters, int32_t *qp_iter, double *cost, int nthreads,
                        int32_t *qp_capped, int32_t delay_cols, int32_t traj_per_lane, int32_t *qp_stalled)
{
    const int N = o->N;
    if (N > TW_MAX_N) return -1;
    tw_par p;
    make_par(&p, o);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    #pragma omp parallel
    {
        tw_ws *w = (tw_ws *)malloc(sizeof(tw_ws));
        #pragma omp for schedule(dynamic, 1)
        for (int32_t i = 0; i < nb; ++i) {
            tw_shape sh;
            make_shape(&sh, n_ctrl, ctrl, knots, params, max_ctrl, shape_id[i], 0.0);
            tw_out out;
            status[i] = ctrl_lane(&p, &sh, w, x0_in + 4 * i, traj + (traj_per_lane ? (size_t)i * T * 6 : 0), T,
                                  delay_cols, index_time[i], Xw + (size_t)i * 4 * (N + 1), Uw + (size_t)i * 2 * N,
                                  PIw + (size_t)i * 4 * N, warm_valid + i, u0 + 2 * i, &out, cost + i);
            if (iters) iters[i] = out.sqp_iter;
            if (qp_iter) qp_iter[i] = out.qp_iter;
            if (qp_capped) qp_capped[i] = out.qp_capped;
            if (qp_stalled) qp_stalled[i] = out.qp_stalled;
            if (g_kkt_diag) memcpy(g_kkt_diag + (size_t)8 * i, w->kkt, sizeof w->kkt);
        }
        free(w);
    }
    return 0;
}

/* contact re-projection (reproject_contact / contact_phi) */
static double contact_phi(const tw_shape *sh, double s, double px, double py)
{
    spl e;
    spline_eval(sh, mat_mod(s, sh->b), &e);
    const double ex = e.C[0] - px, ey = e.C[1] - py;
    return qfma(ey, ey, ex * ex);
}

static double reproject_contact(const tw_shape *sh, double px, double py, double s0)
{
    double s = s0, phi = contact_phi(sh, s, px, py);
    for (int it = 0; it < 60; ++it) {
        spl e;
        spline_eval(sh, mat_mod(s, sh->b), &e);
        const double ex = e.C[0] - px, ey = e.C[1] - py;
        const double g = 2.0 * qfma(ey, e.D[1], ex * e.D[0]);
        const double h = 2.0 * qfma(ey, e.Dd[1], qfma(ex, e.Dd[0], qfma(e.D[1], e.D[1], e.D[0] * e.D[0])));
        if (fabs(g) < 1e-14) break;
        double step = h > 0.0 ? -g / h : (g > 0.0 ? -0.05 : 0.05) * sh->b;
        const double smax = 0.25 * sh->b;
        step = fmin(fmax(step, -smax), smax);
        int ok = 0;
        double sn = s, phin = phi;
        for (int k = 0; k < 60; ++k) {
            sn = s + step;
            phin = contact_phi(sh, sn, px, py);
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

int tw_reproject_contact(const int32_t *n_ctrl, const double *ctrl, const double *knots, const double *params,
                         int max_ctrl, int32_t n, const int32_t *shape_id, const double *px, const double *py,
                         const double *s0, double *s)
{
    for (int32_t i = 0; i < n; ++i) {
        tw_shape sh;
        make_shape(&sh, n_ctrl, ctrl, knots, params, max_ctrl, shape_id[i], 0.0);
        s[i] = reproject_contact(&sh, px[i], py[i], s0[i]);
    }
    return 0;
}

/* helper.closed_loop_matlab on the device (qsp_closed_loop_ex: closed_loop_pre_kernel, the controller
 * solve, plant_kernel), per lane: cold start; the plant's input buffer starts at zero, the
 * controller's u_buff_contr at ubc0 (B x delay_cols x 2, NULL: zero -- as set_delay_comp leaves it). */
int tw_closed_loop(const int32_t *n_ctrl, const double *ctrl, const double *knots, const double *params,
                   int max_ctrl, const or_opts *o, int32_t nb, const int32_t *shape_id, const double *x0_in,
                   const double *traj, int32_t T, const int32_t *index0, int32_t n_steps, const double *noise,
                   int32_t delay_cols, int32_t plant_delay_cols, int32_t dist_step, const double *dist_amp,
                   const double *xwidth, double *Xtraj, double *Xsim, double *Utraj, int32_t *Straj, int nthreads,
                   const double *ubc0)
{
    const int N = o->N;
    if (N > TW_MAX_N || delay_cols < 0 || plant_delay_cols < 0 || delay_cols > 1024 || plant_delay_cols > 1024) return -1;
    tw_par p;
    make_par(&p, o);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    if (g_kkt_diag) memset(g_kkt_diag, 0, sizeof(double) * 8 * (size_t)nb);
    #pragma omp parallel
    {
        tw_ws *w = (tw_ws *)malloc(sizeof(tw_ws));
        double *Xw = (double *)malloc(sizeof(double) * 4 * (N + 1)), *Uw = (double *)malloc(sizeof(double) * 2 * N);
        double *PIw = (double *)malloc(sizeof(double) * 4 * N);
        double *ubc = (double *)calloc(2 * (size_t)(delay_cols + 1), sizeof(double));
        double *ubp = (double *)calloc(2 * (size_t)(plant_delay_cols + 1), sizeof(double));
        #pragma omp for schedule(dynamic, 1)
        for (int32_t i = 0; i < nb; ++i) {
            tw_shape sh;
            make_shape(&sh, n_ctrl, ctrl, knots, params, max_ctrl, shape_id[i], xwidth ? xwidth[shape_id[i]] : 0.0);
            uint8_t valid = 0;
            memset(Xw, 0, sizeof(double) * 4 * (N + 1));
            memset(Uw, 0, sizeof(double) * 2 * N);
            memset(PIw, 0, sizeof(double) * 4 * N);
            memset(ubc, 0, sizeof(double) * 2 * (size_t)(delay_cols + 1));
            if (ubc0 && delay_cols > 0) memcpy(ubc, ubc0 + (size_t)i * delay_cols * 2, sizeof(double) * 2 * (size_t)delay_cols);
            memset(ubp, 0, sizeof(double) * 2 * (size_t)(plant_delay_cols + 1));
            double x[4];
            memcpy(x, x0_in + 4 * i, sizeof x);
            for (int32_t t = 0; t < n_steps; ++t) {
                /* closed_loop_pre_kernel */
                if (dist_step > 0 && t + 1 == dist_step) {
                    const double amp = dist_amp ? dist_amp[i] : 0.0;
                    x[1] += amp;
                    spl e;
                    spline_eval(&sh, mat_mod(x[3], sh.b), &e);
                    const double sn = reproject_contact(&sh, -0.5 * sh.xwidth, e.C[1] - amp, 0.0);
                    x[3] = qfma(-sh.b, sn < 0.0 ? 1.0 : 0.0, mat_mod(sn, sh.b));
                }
                if (noise)
                    for (int c = 0; c < 4; ++c) x[c] += noise[((size_t)t * nb + i) * 4 + c];
                memcpy(Xtraj + ((size_t)i * (n_steps + 1) + t) * 4, x, sizeof x);
                double xs[4];
                memcpy(xs, x, sizeof xs);
                for (int k = 1; k <= delay_cols; ++k) {
                    const double *u = ubc + 2 * (delay_cols - k);
                    dyn d;
                    dynamics(&sh, xs[2], xs[3], u[0], u[1], &d, 0);
                    for (int c = 0; c < 4; ++c) xs[c] = qfma(p.Ts, d.f[c], xs[c]);
                }
                if (Xsim) memcpy(Xsim + ((size_t)i * n_steps + t) * 4, xs, sizeof xs);
                double u[2];
                tw_out out;
                const int st = ctrl_lane(&p, &sh, w, xs, traj, T, delay_cols, index0[i] + t + delay_cols, Xw, Uw, PIw,
                                         &valid, u, &out, NULL);
                /* plant_kernel */
                if (delay_cols > 0) {
                    for (int k = delay_cols - 1; k >= 1; --k) { ubc[2 * k] = ubc[2 * (k - 1)]; ubc[2 * k + 1] = ubc[2 * (k - 1) + 1]; }
                    ubc[0] = u[0];
                    ubc[1] = u[1];
                }
                double ua[2] = {u[0], u[1]};
                if (plant_delay_cols > 0) {
                    ua[0] = ubp[2 * (plant_delay_cols - 1)];
                    ua[1] = ubp[2 * (plant_delay_cols - 1) + 1];
                    for (int k = plant_delay_cols - 1; k >= 1; --k) { ubp[2 * k] = ubp[2 * (k - 1)]; ubp[2 * k + 1] = ubp[2 * (k - 1) + 1]; }
                    ubp[0] = u[0];
                    ubp[1] = u[1];
                }
                dyn d;
                dynamics(&sh, x[2], x[3], ua[0], ua[1], &d, 0);
                for (int c = 0; c < 4; ++c) x[c] = qfma(p.Ts, d.f[c], x[c]);
                memcpy(Utraj + ((size_t)i * n_steps + t) * 2, u, sizeof u);
                if (Straj) Straj[(size_t)i * n_steps + t] = st;
                if (g_kkt_diag && st == 2) {
                    /* closed loop: per lane, over its status-2 steps, how often each KKT residual
                     * failed (stat, eq, ineq, comp), the steps, those failing stationarity alone,
                     * and those whose stationarity residual is below 1e-3 (near misses) */
                    double *dg = g_kkt_diag + (size_t)8 * i;
                    const double rs = fmax(fmax(w->kkt[0], w->kkt[1]), w->kkt[2]);
                    const int f0 = rs >= p.tol_stat, f1 = w->kkt[3] >= p.tol_eq, f2 = w->kkt[4] >= p.tol_ineq,
                              f3 = w->kkt[5] >= p.tol_comp;
                    dg[0] += f0; dg[1] += f1; dg[2] += f2; dg[3] += f3;
                    dg[4] += 1.0;
                    dg[5] += (f0 && !f1 && !f2 && !f3);
                    dg[6] += rs < 1e-3;
                }
            }
            memcpy(Xtraj + ((size_t)i * (n_steps + 1) + n_steps) * 4, x, sizeof x);
        }
        free(w); free(Xw); free(Uw); free(PIw); free(ubc); free(ubp);
    }
    return 0;
}
