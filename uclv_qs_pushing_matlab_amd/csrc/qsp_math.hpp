// qsp_math.hpp — device math for the pusher–slider OCP (gfx950, FP64).
//
// Span-based clamped cubic B-spline, motion-cone dynamics with a hand-derived
// Jacobian, and RK4 with forward sensitivities.  Restates, without the CasADi
// graph, what the reference builds symbolically:
//   spline / frame / tangent-angle rate : acados_nmpc/bspline_shape.m:40-116, 137-152
//   dynamics f(x,u)                     : acados_nmpc/PusherSliderModel.m:503-603
//   ERK integrator (RK4, 1 step)        : acados sim_method "erk" (NMPC_controller.m:272)
// Every fused multiply-add is written out (qfma; the library is built with
// -ffp-contract=off): the oracle's kernel-order twin (oracle/qsp_twin.c) evaluates the same
// operations in the same order and reproduces these results bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qsp_fp.hpp"
#include "qsp_types.h"


namespace qsp {

// ---------------------------------------------------------------- B-spline
// Evaluation at sigma on the unique span S[j] <= sigma < S[j+1] (3 <= j <= n-1).
// The reference sums ALL n basis functions with the half-open indicator
// (s<S(i+1))*(s>=S(i)) (bspline_shape.m:52); outside [S[3], S[n]) every term is
// zero, so C = C' = 0 there (in particular at sigma == b).
struct SplineEval {
    double C[2];    // FC(sigma)                         (getSymbolicSpline :74-83)
    double D[2];    // FC_dot(sigma)                     (getSymboliSplineDot :85-104)
    double Dd[2];   // d FC_dot / d sigma
};

__device__ __forceinline__ void spline_eval(const ShapeDev& sh, double sig, SplineEval& o) {
    const int n = sh.n;
    const double* S = sh.knots;
    const bool inside = (sig >= S[3]) && (sig < S[n]);
    int j = 3 + (int)(sig * sh.inv_h);
    j = j < 3 ? 3 : (j > n - 1 ? n - 1 : j);
    // exact half-open span by comparison against the stored knots
    if (sig < S[j]) j = (j > 3) ? j - 1 : j;
    if (sig < S[j]) j = (j > 3) ? j - 1 : j;
    if (sig >= S[j + 1]) j = (j < n - 1) ? j + 1 : j;
    if (sig >= S[j + 1]) j = (j < n - 1) ? j + 1 : j;

    // Cox–de Boor triangle on span j: N1[0..1] (deg 1), N2[0..2] (deg 2), N3[0..3] (deg 3)
    const double l1 = sig - S[j], l2 = sig - S[j - 1], l3 = sig - S[j - 2];
    const double r1 = S[j + 1] - sig, r2 = S[j + 2] - sig, r3 = S[j + 3] - sig;
    double N1_0, N1_1;
    {
        const double t = 1.0 / (r1 + l1);
        N1_0 = r1 * t;
        N1_1 = l1 * t;
    }
    double N2_0, N2_1, N2_2;
    {
        const double t0 = N1_0 / (r1 + l2);
        const double t1 = N1_1 / (r2 + l1);
        N2_0 = r1 * t0;
        N2_1 = qfma(r2, t1, l2 * t0);
        N2_2 = l1 * t1;
    }
    double N3_0, N3_1, N3_2, N3_3;
    {
        const double t0 = N2_0 / (r1 + l3);
        const double t1 = N2_1 / (r2 + l2);
        const double t2 = N2_2 / (r3 + l1);
        N3_0 = r1 * t0;
        N3_1 = qfma(r2, t1, l3 * t0);
        N3_2 = qfma(r3, t2, l2 * t1);
        N3_3 = l1 * t2;
    }
    const double* P = sh.ctrl + 2 * (j - 3);     // P_{j-3..j}
    const double* cd = sh.dctrl + 2 * (j - 2);   // derivative coefficients of N_{j-2..j,2}
    const double* dd = sh.ddctrl + 2 * (j - 1);  // second-derivative coefficients of N_{j-1..j,1}
    for (int c = 0; c < 2; ++c) {
        double Cv = N3_0 * P[c];
        Cv = qfma(N3_1, P[2 + c], Cv);
        Cv = qfma(N3_2, P[4 + c], Cv);
        Cv = qfma(N3_3, P[6 + c], Cv);
        double Dv = N2_0 * cd[c];
        Dv = qfma(N2_1, cd[2 + c], Dv);
        Dv = qfma(N2_2, cd[4 + c], Dv);
        const double Ddv = qfma(N1_1, dd[2 + c], N1_0 * dd[c]);
        o.C[c] = inside ? Cv : 0.0;
        o.D[c] = inside ? Dv : 0.0;
        o.Dd[c] = inside ? Ddv : 0.0;
    }
}

// s_mod inside the OCP model: fmod(s,b) + (s<0)*b   (PusherSliderModel.m:526)
__device__ __forceinline__ double smod_model(double s, double b) {
    return fmod(s, b) + ((s < 0.0) ? b : 0.0);
}

// MATLAB floor-mod  mod(a,b) = a - floor(a/b)*b   (NMPC_controller.m:320,332)
__device__ __forceinline__ double mat_mod(double a, double b) {
    const double r = qfma(-floor(a / b), b, a);
    return (r == b) ? 0.0 : r;
}

// tangent-angle rate kappa = d/ds atan2(C'_y, C'_x)  (bspline_shape.m:137-144)
__device__ __forceinline__ double angle_rate_of(const SplineEval& e) {
    return qfma(e.D[0], e.Dd[1], -(e.D[1] * e.Dd[0])) / qfma(e.D[0], e.D[0], e.D[1] * e.D[1]);
}
__device__ __forceinline__ double angle_rate(const ShapeDev& sh, double sig) {
    SplineEval e;
    spline_eval(sh, sig, e);
    return angle_rate_of(e);
}

// tangential velocity bound v_bound(s)  (NMPC_controller.m:319-327)
__device__ __forceinline__ double v_bound(const ShapeDev& sh, const CtrlParams& cp, double s) {
    const double sm = mat_mod(s, sh.b);
    const double ta = fabs(angle_rate(sh, sm));
    const double v = cp.v_alpha / (fabs(ta - cp.t_angle0) + 0.0001) + cp.d_v;
    return v < cp.u_t_ub ? v : cp.u_t_ub;
}

// ---------------------------------------------------------------- dynamics
// f(x,u) and its Jacobian.  f does not depend on (x, y); d f/d theta only has
// rows 0,1.  Jacobian columns: Jth[2], Js[4], Jun[4], Jut[4].
struct DynOut {
    double f[4];
    double Jth[2];
    double Js[4];
    double Jun[4];
    double Jut[4];
};

// indicator blend i_st * a + i_sl * b + i_sr * c (PusherSliderModel.m:587-589)
__device__ __forceinline__ double blend3(double ist, double a, double isl, double b, double isr, double c) {
    return qfma(isr, c, qfma(isl, b, ist * a));
}

template <bool WITH_JAC>
__device__ __forceinline__ void dynamics(const ShapeDev& sh, double th, double s, double un, double ut, DynOut& o) {
    const double sig = smod_model(s, sh.b);
    SplineEval e;
    spline_eval(sh, sig, e);
    // frame (bspline_shape.m:108-111): t = C'/|C'|, n = (t_y, -t_x)
    const double l2 = qfma(e.D[0], e.D[0], e.D[1] * e.D[1]);
    const double l = sqrt(l2);
    const double il = 1.0 / l;
    const double tx = e.D[0] * il, ty = e.D[1] * il;
    const double nx = ty, ny = -tx;
    const double Px = e.C[0], Py = e.C[1];
    // contact point in the N-T frame (PusherSliderModel.m:532-534)
    const double px = qfma(nx, Px, ny * Py);
    const double py = qfma(tx, Px, ty * Py);

    const double c2 = sh.c * sh.c, mu = sh.mu;
    const double pxpy = px * py, px2 = px * px;
    const double q00 = qfma(px, px, c2), q11 = qfma(py, py, c2);
    const double fac = 1.0 / qfma(py, py, q00);                        // :544
    const double nl = qfma(mu, px2, qfma(mu, c2, -pxpy));              // :547
    const double dl = qfma(-mu, pxpy, q11);
    const double nr = qfma(-mu, px2, qfma(-mu, c2, -pxpy));            // :548
    const double dr = qfma(mu, pxpy, q11);
    const double gl = nl / dl, gr = nr / dr;
    const double rho = ut / un;                                        // :551

    double sn, cs;
    sin_cos(th, &sn, &cs);
    // G = R_NT * fac * Q  (body frame), M = R(theta) G   (:554-559)
    const double H00 = qfma(tx, pxpy, nx * q00), H01 = qfma(tx, q11, nx * pxpy);
    const double H10 = qfma(ty, pxpy, ny * q00), H11 = qfma(ty, q11, ny * pxpy);
    const double G00 = fac * H00, G01 = fac * H01, G10 = fac * H10, G11 = fac * H11;
    const double M00 = qfma(-sn, G10, cs * G00), M01 = qfma(-sn, G11, cs * G01);
    const double M10 = qfma(cs, G10, sn * G00), M11 = qfma(cs, G11, sn * G01);

    // indicator blend (:587-589); every comparison with NaN is false
    const double ist = ((rho >= gr) && (rho <= gl)) ? 1.0 : 0.0;
    const double isl = (rho > gl) ? 1.0 : 0.0;
    const double isr = (rho < gr) ? 1.0 : 0.0;

    // sticking (:557-560)
    const double st0 = qfma(M01, ut, M00 * un);
    const double st1 = qfma(M11, ut, M10 * un);
    const double st2 = fac * qfma(px, ut, -(py * un));
    // sliding left / right (:563-585)
    const double vl0 = qfma(M01, gl, M00), vl1 = qfma(M11, gl, M10);
    const double vr0 = qfma(M01, gr, M00), vr1 = qfma(M11, gr, M10);
    const double wl = fac * qfma(gl, px, -py), wr = fac * qfma(gr, px, -py);
    o.f[0] = blend3(ist, st0, isl, vl0 * un, isr, vr0 * un);
    o.f[1] = blend3(ist, st1, isl, vl1 * un, isr, vr1 * un);
    o.f[2] = blend3(ist, st2, isl, wl * un, isr, wr * un);
    o.f[3] = qfma(isr, qfma(-gr, un, ut), isl * qfma(-gl, un, ut));
    if (!WITH_JAC) return;

    // ---- d/d sigma of the frame, contact point, Q, fac, gammas (chain rule by hand)
    const double tDd = qfma(ty, e.Dd[1], tx * e.Dd[0]);
    const double txs = qfma(-tx, tDd, e.Dd[0]) * il, tys = qfma(-ty, tDd, e.Dd[1]) * il;
    const double nxs = tys, nys = -txs;
    // dP/dsigma = C'(sigma) = D ; n.D = 0, t.D = l
    const double pxs = qfma(nxs, Px, nys * Py);
    const double pys = qfma(txs, Px, tys * Py) + l;
    const double pxpys = qfma(px, pys, pxs * py);
    const double q00s = 2.0 * px * pxs, q11s = 2.0 * py * pys;
    const double facs = -fac * fac * (q00s + q11s);
    const double gls = qfma(-gl, qfma(-mu, pxpys, q11s), qfma(mu, q00s, -pxpys)) / dl;
    const double grs = qfma(-gr, qfma(mu, pxpys, q11s), qfma(-mu, q00s, -pxpys)) / dr;
    // G_s = d/dsigma [R_NT fac Q]
    const double G00s = qfma(facs, H00, fac * qfma(tx, pxpys, qfma(txs, pxpy, qfma(nx, q00s, nxs * q00))));
    const double G01s = qfma(facs, H01, fac * qfma(tx, q11s, qfma(txs, q11, qfma(nx, pxpys, nxs * pxpy))));
    const double G10s = qfma(facs, H10, fac * qfma(ty, pxpys, qfma(tys, pxpy, qfma(ny, q00s, nys * q00))));
    const double G11s = qfma(facs, H11, fac * qfma(ty, q11s, qfma(tys, q11, qfma(ny, pxpys, nys * pxpy))));
    const double M00s = qfma(-sn, G10s, cs * G00s), M01s = qfma(-sn, G11s, cs * G01s);
    const double M10s = qfma(cs, G10s, sn * G00s), M11s = qfma(cs, G11s, sn * G01s);
    // d/dtheta of M: R'(theta) G
    const double M00t = qfma(-cs, G10, -sn * G00), M01t = qfma(-cs, G11, -sn * G01);
    const double M10t = qfma(-sn, G10, cs * G00), M11t = qfma(-sn, G11, cs * G01);

    // sticking derivatives
    const double st0t = qfma(M01t, ut, M00t * un), st1t = qfma(M11t, ut, M10t * un);
    const double st0s = qfma(M01s, ut, M00s * un), st1s = qfma(M11s, ut, M10s * un);
    const double st2s = qfma(facs, qfma(px, ut, -(py * un)), fac * qfma(pxs, ut, -(pys * un)));
    // sliding derivatives
    const double vl0s = qfma(M01, gls, qfma(M01s, gl, M00s)), vl1s = qfma(M11, gls, qfma(M11s, gl, M10s));
    const double vr0s = qfma(M01, grs, qfma(M01s, gr, M00s)), vr1s = qfma(M11, grs, qfma(M11s, gr, M10s));
    const double vl0t = qfma(M01t, gl, M00t), vl1t = qfma(M11t, gl, M10t);
    const double vr0t = qfma(M01t, gr, M00t), vr1t = qfma(M11t, gr, M10t);
    const double wls = qfma(facs, qfma(gl, px, -py), fac * (qfma(gl, pxs, gls * px) - pys));
    const double wrs = qfma(facs, qfma(gr, px, -py), fac * (qfma(gr, pxs, grs * px) - pys));

    o.Jth[0] = blend3(ist, st0t, isl, vl0t * un, isr, vr0t * un);
    o.Jth[1] = blend3(ist, st1t, isl, vl1t * un, isr, vr1t * un);
    o.Js[0] = blend3(ist, st0s, isl, vl0s * un, isr, vr0s * un);
    o.Js[1] = blend3(ist, st1s, isl, vl1s * un, isr, vr1s * un);
    o.Js[2] = blend3(ist, st2s, isl, wls * un, isr, wrs * un);
    o.Js[3] = -qfma(isr, grs * un, isl * (gls * un));
    o.Jun[0] = blend3(ist, M00, isl, vl0, isr, vr0);
    o.Jun[1] = blend3(ist, M10, isl, vl1, isr, vr1);
    o.Jun[2] = blend3(-ist, fac * py, isl, wl, isr, wr);
    o.Jun[3] = -qfma(isr, gr, isl * gl);
    o.Jut[0] = ist * M01;
    o.Jut[1] = ist * M11;
    o.Jut[2] = ist * (fac * px);
    o.Jut[3] = isl + isr;
}

// ---------------------------------------------------------------- RK4 + VDE
// x+ = phi(x,u) over h with one RK4 step (acados ERK default: 4 stages, 1 step);
// sensitivities w.r.t. (theta0, s0, u_n, u_t).  Columns x0, y0 of dphi/dx are
// exactly e0, e1 and d(theta+, s+)/d theta0 = (1, 0): A is stored by its six
// free entries  a = {a02, a03, a12, a13, a23, a33}.
struct Lin {
    double xn[4];
    double a[6];
    double B[8];   // row-major 4x2
};

template <bool WITH_SENS>
__device__ __forceinline__ void rk4(const ShapeDev& sh, double h, const double x[4], const double u[2], Lin& o) {
    const double ca[4] = {0.0, 0.5, 0.5, 1.0};
    const double cb[4] = {1.0 / 6.0, 1.0 / 3.0, 1.0 / 3.0, 1.0 / 6.0};
    double acc[4] = {x[0], x[1], x[2], x[3]};
    // accumulated sensitivity S+ (rows 0..3) for columns th, s, un, ut
    double Sa[4][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {1, 0, 0, 0}, {0, 1, 0, 0}};
    double K[4] = {0, 0, 0, 0};
    double SK[4][4] = {{0}};
#pragma unroll 1   // sequential RK stages keep the register footprint of the VDE small
    for (int st = 0; st < 4; ++st) {
        const double aa = h * ca[st];
        double xs[4];
        double Ss[2][4];   // rows theta, s of the stage-state sensitivity
#pragma unroll
        for (int i = 0; i < 4; ++i) xs[i] = (st == 0) ? x[i] : qfma(aa, K[i], x[i]);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double e2 = (c == 0) ? 1.0 : 0.0, e3 = (c == 1) ? 1.0 : 0.0;
            Ss[0][c] = (st == 0) ? e2 : qfma(aa, SK[2][c], e2);
            Ss[1][c] = (st == 0) ? e3 : qfma(aa, SK[3][c], e3);
        }
        DynOut d;
        dynamics<WITH_SENS>(sh, xs[2], xs[3], u[0], u[1], d);
#pragma unroll
        for (int i = 0; i < 4; ++i) K[i] = d.f[i];
        if (WITH_SENS) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const double jt = Ss[0][c], js = Ss[1][c];
                SK[0][c] = qfma(d.Js[0], js, d.Jth[0] * jt);
                SK[1][c] = qfma(d.Js[1], js, d.Jth[1] * jt);
                SK[2][c] = d.Js[2] * js;
                SK[3][c] = d.Js[3] * js;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                SK[i][2] += d.Jun[i];
                SK[i][3] += d.Jut[i];
            }
        }
        const double w = h * cb[st];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = qfma(w, K[i], acc[i]);
        if (WITH_SENS) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int c = 0; c < 4; ++c) Sa[i][c] = qfma(w, SK[i][c], Sa[i][c]);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) o.xn[i] = acc[i];
    if (WITH_SENS) {
        o.a[0] = Sa[0][0]; o.a[1] = Sa[0][1];
        o.a[2] = Sa[1][0]; o.a[3] = Sa[1][1];
        o.a[4] = Sa[2][1]; o.a[5] = Sa[3][1];
#pragma unroll
        for (int i = 0; i < 4; ++i) { o.B[2 * i] = Sa[i][2]; o.B[2 * i + 1] = Sa[i][3]; }
    }
}

}  // namespace qsp
