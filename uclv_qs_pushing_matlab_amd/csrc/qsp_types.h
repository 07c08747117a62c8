// qsp_types.h — plain-old-data tables shared by the host C-ABI and the kernels.
#pragma once
#include <stdint.h>

#define QSP_MAX_CTRL 64  // control points per shape (pulirapid: 56)

namespace qsp {

// One slider shape: clamped cubic B-spline (bspline_shape.m, PusherSliderModel.m:113-132)
// plus the physical constants that enter f (PusherSliderModel.m:53,55; object_selection.m).
struct ShapeDev {
    int32_t n;                             // control points (closed contour, first point repeated)
    int32_t pad_;
    double b;                              // contour length = last knot
    double c;                              // c_ellipse = tau_max / (mu_sg m g)
    double mu;                             // mu_sp
    double inv_h;                          // 1 / interior knot spacing (span guess only)
    double xwidth;                         // slider width along x (object_selection.m; disturbance re-projection)
    double knots[QSP_MAX_CTRL + 4];        // S, n + 4 entries
    double ctrl[2 * QSP_MAX_CTRL];         // P_i (x, y)
    double dctrl[2 * QSP_MAX_CTRL];        // cd_i = 3 (P_i - P_{i-1}) / (S_{i+3} - S_i), cd_0 = 0
    double ddctrl[2 * QSP_MAX_CTRL];       // dd_i = 2 (cd_i - cd_{i-1}) / (S_{i+2} - S_i)
};

// warm-start clip parameters (NMPC_controller.m:98-100, 23-26)
struct CtrlParams {
    double v_alpha, d_v, t_angle0, u_n_lb, u_t_ub;
};

// everything a solve needs besides per-lane data
struct SolveParams {
    int32_t N;            // horizon
    int32_t nlp_mode;     // 0: fixed-K full-step SQP (RTI metric); 1: SQP + merit backtracking + KKT tolerances
    int32_t sqp_iters;    // K
    int32_t qp_iters;     // max Mehrotra iterations per QP
    double Ts;            // integrator step h = T / N
    double tau;           // stage-cost scaling (acados: Ts)
    double W[6];          // diag of blkdiag(W_x, W_u)
    double We[4];         // diag of W_x_e
    double lh[3], uh[3];  // bounds of h = [s; u_n; u_t]
    double mu0, t_min, frac, sigma_min, mu_stop;  // interior-point parameters
    double res_stop;                              // IPM stop also needs the bound residual < res_stop
    double qp_tol_stat, qp_tol_eq;                // IPM stop also needs the stationarity / equality residuals below these
    double qp_stall_alpha;                        // stall exit: step length below this ...
    int32_t qp_stall_iters;                       // ... for this many consecutive iterations (0: off)
    double qp_mu_max;                             // divergence exit: mu >= this (or NaN) is a QP failure
    int32_t s0_bound;                             // 1: the s bound of h also applies at stage 0
    int32_t factor_scan;                          // 1: S = 2 factorisation as an associative scan (qsp_options)
    int32_t mfma_walk;                            // 1: factorisation on the FP64 matrix cores where it fits (mfw_fits:
                                                  // S = 1 at 12 <= N <= 31, S = 2 from N = 24)
    int32_t mfw_on[2];                            // per stages-per-lane S = 1, 2: mfma_walk and the records fit
    int32_t mfw_is[2];                            // ... and the doubles between instances' record regions
                                                  // (mfw_prepare, host-side: the kernels only read them)
    double tol_stat, tol_eq, tol_ineq, tol_comp;  // nlp_mode 1 termination
    double ls_alpha_min, ls_alpha_red, ls_eps;    // nlp_mode 1 line search
    CtrlParams cp;
};

}  // namespace qsp
