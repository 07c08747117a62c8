// qsp_fp.hpp — FP64 primitives whose bits the CPU oracle reproduces.
//
// The library is compiled with -ffp-contract=off: every fused multiply-add in the solve is an
// explicit fma() (qfma below), so the oracle's kernel-order restatement performs the same IEEE
// operations in the same order and reproduces the device results bit for bit.  The operations
// used are those gfx950 rounds exactly as the host does (+ - * / sqrt fma, fmod, floor, rint;
// scripts/ubench/fp_exact.hip checks them), plus the two below:
//   rcp     1/x from the hardware reciprocal refined by two Newton steps.  From any start
//           within 2^-27 the second step lands on the correctly rounded 1/x (barring a
//           2^-90-close tie), so the oracle writes it as the same two steps from 1.0 / x.
//   sin_cos sin and cos by fdlibm's Cody–Waite reduction (two stages, 118 bits of pi/2) and
//           the fdlibm/musl kernel polynomials, written out here so that both sides evaluate
//           the same sequence (ocml's and glibc's sin differ in the last bit).  Accurate to
//           about one ulp for |x| < 2^20 pi/2; beyond that the reduction degrades (the model's
//           theta stays within a few radians).
#pragma once
#include <hip/hip_runtime.h>

namespace qsp {

// explicit fused multiply-add: a * b + c with one rounding
__host__ __device__ __forceinline__ double qfma(double a, double b, double c) { return __builtin_fma(a, b, c); }

__device__ __forceinline__ double rcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
#else
    double r = 1.0 / x;   // host pass of device code (never run)
#endif
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
}
// the host counterpart (developer tools; the oracle restates it in C)
inline double rcp_host(double x) {
    double r = 1.0 / x;
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
}

__host__ __device__ __forceinline__ void sin_cos(double x, double* sp, double* cp) {
    // x = n pi/2 + (y + yy), |y| <= pi/4 (fdlibm __ieee754_rem_pio2, medium case, two stages)
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;    // first 33 bits of pi/2
    const double pio2_2 = 6.07710050630396597660e-11;    // next 33 bits
    const double pio2_2t = 2.02226624879595063154e-21;   // pi/2 - pio2_1 - pio2_2
    const double fn = rint(x * invpio2);
    double r = x - fn * pio2_1;                           // exact: fn * pio2_1 has <= 53 bits
    double w = fn * pio2_2;
    const double t = r;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    const double y = r - w;
    const double yy = (r - y) - w;
    // kernels on [-pi/4, pi/4] with the tail yy (musl __sin, __cos)
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
    // quadrant n mod 4 without an integer conversion (NaN / Inf fall through to quadrant 0: NaN)
    const double q = fn - 4.0 * floor(fn * 0.25);
    const bool q1 = q == 1.0, q2 = q == 2.0, q3 = q == 3.0;
    const double s = q1 ? kc : (q2 ? -ks : (q3 ? -kc : ks));
    const double c = q1 ? -ks : (q2 ? -kc : (q3 ? ks : kc));
    *sp = s;
    *cp = c;
}

}  // namespace qsp
