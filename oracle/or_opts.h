/*
 * or_opts.h — solver options shared by the CPU oracle's two restatements (TEST INFRASTRUCTURE
 * ONLY): qsp_oracle.c (literal) and qsp_twin.c (kernel order).  Layout mirrored by oracle.py Opts.
 */
#ifndef OR_OPTS_H
#define OR_OPTS_H
#include <stdint.h>

/* -------------------------------------------------------------- options */
typedef struct {
    int32_t N;          /* horizon (param_scheme_N) */
    int32_t sqp_iters;  /* K full Gauss-Newton steps */
    int32_t qp_iters;   /* Mehrotra iterations per QP */
    int32_t stage0_s_bound; /* 1: the s bound of h also applies at stage 0 (acados-recall: bgh at
                               stage 0, NMPC_controller.m:237,251-252); s_0 is fixed by x0, so an
                               x0 with s outside [lh_s, uh_s] makes every QP infeasible */
    double Ts;          /* h = T/N */
    double tau;         /* stage-cost scaling (acados: Ts) */
    double W[6];        /* diag(blkdiag(W_x, W_u))   (NMPC_controller.m:157, main.m:82-86) */
    double We[4];       /* diag(W_x_e)               (NMPC_controller.m:154) */
    double lh[3], uh[3];/* bounds on h = [s; u_n; u_t] (NMPC_controller.m:251-252) */
    double mu0;         /* IPM initial complementarity */
    double t_min;       /* IPM slack floor at initialisation */
    double frac;        /* fraction to boundary */
    double sigma_min;   /* lower clamp of the Mehrotra centering parameter */
    double mu_stop;     /* per-QP early exit once mu < mu_stop */
    double v_alpha, d_v, t_angle0; /* NMPC_controller.m:98-100 */
    double u_n_lb, u_t_ub;         /* NMPC_controller.m:23-26 */
    /* globalised SQP (nlp_mode == 1): acados "sqp" + "merit_backtracking",
     * tolerances nlp_solver_tol_* (NMPC_controller.m:271-276) */
    int32_t nlp_mode;   /* 0: fixed-K full-step (RTI metric), 1: SQP + merit line search + tolerances */
    int32_t pad_;
    double tol_stat, tol_eq, tol_ineq, tol_comp;
    double ls_alpha_min, ls_alpha_red, ls_eps;
    double res_stop;    /* per-QP early exit also needs the bound residual below res_stop */
    /* HPIPM-style QP termination (ocp_qp_ipm: res_g, res_b next to res_d = res_stop and
     * res_m = mu_stop): the stationarity and equality residuals of the IPM iterate.  Both are
     * linear in the iterate and every Newton step solves them exactly, so each update scales
     * them by (1 - alpha): tracked as r_0 * prod(1 - alpha) from the start point (z = 0, pi = 0,
     * lam = mu0 / t), like the bound residual. */
    double qp_tol_stat, qp_tol_eq;
    /* stall exit: a QP whose step length stays below qp_stall_alpha for qp_stall_iters
     * consecutive iterations is locally infeasible (e.g. the linearised s dynamics cannot meet
     * the s bound): mu grows without bound and alpha ~1e-5 to the cap.  It stops there, with
     * the capped QPs' status (its last iterate is used, as at the cap).  0 iterations: off. */
    double qp_stall_alpha;
    int32_t qp_stall_iters;
    int32_t stages_per_lane; /* twin only: the device layout S whose arithmetic order it follows (0: the
                                library's choice, 1 for N + 1 <= 32 or nlp_mode 1, else 2) */
    double qp_mu_max;   /* divergence exit: mu >= qp_mu_max (or non-finite) is a QP failure (status 4) */
    /* literal restatement only (the twin ignores it): the model probe.  Every entry of each output
     * of the linearisation (x+, A, B of rk4_sens) moves by +- model_probe x that array's largest
     * entry, the sign hashed from probe_seed, the stage's inputs and the entry -- a perturbation of
     * the model of the size by which the two formulations differ (measured: up to 1.6e-13 of the
     * scale in A, 5.5e-14 in B, 1e-14 in x+), to tell lanes whose u0 depends on those last digits
     * of the model from the others.  0: off. */
    double model_probe;
    int32_t probe_seed;
    int32_t factor_scan; /* twin only: at S = 2 the factorisation as the device's associative scan
                            (qsp_options.factor_scan) instead of the walk */
    int32_t lane_walk;   /* twin only: 1 = factorise by the lane walk's order even where the device uses the
                            matrix cores (the fastest CPU formulation of the same algorithm: bench.py's
                            cpu_baseline; the matrix-core order, emulated, is the bit-exact checker) */
} or_opts;

#endif
