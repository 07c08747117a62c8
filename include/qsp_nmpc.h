/*
 * qsp_nmpc.h — C ABI of the MI355X batched pusher–slider NMPC solver.
 *
 * Drop-in boundary for the reference's solver backend: the acados MATLAB object
 * `ocp_solver = acados_ocp(ocp_model, ocp_opts)` created in
 * acados_nmpc/NMPC_controller.m:302-305 and driven through `.set/.solve/.get`
 * (NMPC_controller.m:154-157, 170, 334-348, 382-394, 403, 420; helper.m:253, 264-269).
 * One handle replaces B independent acados solver objects: every per-lane array is
 * batched along a leading dimension B.  MATLAB column-major per-lane arrays
 * (4 x (N+1), 2 x N, 4 x N) are exactly the row-major (N+1) x 4 / N x 2 / N x 4 blocks
 * used here, so they pass through unchanged.
 *
 * Conventions
 *   ownership : the caller owns host buffers; the handle owns device memory.
 *   errors    : every entry point returns QSP_OK (0) or a negative QSP_ERR_*;
 *               qsp_last_error() gives the message (thread-local).  Numerical
 *               failure is NOT an error: it is the per-lane status (as acados 'status').
 *   threading : one handle per host thread; a handle owns one HIP stream on one device.
 *   precision : FP64 throughout.
 *   versions  : qsp_version() is QSP_ABI_VERSION of the library.  Callers compiled against
 *               this header check it before anything else; qsp_options and qsp_shape carry
 *               their own size in struct_size (set by qsp_default_options / qsp_shape_from_ply,
 *               or by the caller), which qsp_create and qsp_set_shapes reject when it differs
 *               from the library's sizeof, so a stale layout fails loudly instead of being
 *               read at the wrong offsets.
 */
#ifndef QSP_NMPC_H
#define QSP_NMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QSP_NX 4          /* x = [x, y, theta, s]   (PusherSliderModel.m:519) */
#define QSP_NU 2          /* u = [u_n, u_t]         (PusherSliderModel.m:520) */
#define QSP_NY 6
#define QSP_NY_E 4
#define QSP_NH 3          /* h = [s; u_n; u_t]      (NMPC_controller.m:237) */
#define QSP_MAX_CTRL 64   /* spline control points per shape */
#define QSP_ABI_VERSION 4 /* 2: struct_size fields, qp_mu_max, qsp_get_qp_stalled, QP-failure exits;
                             3: qsp_options.factor_scan; 4: qsp_get_factor_walk */

#define QSP_OK 0
#define QSP_ERR_ARG (-1)
#define QSP_ERR_HIP (-2)
#define QSP_ERR_STATE (-3)
#define QSP_ERR_IO (-4)

/* per-lane solver status (acados meaning where one exists) */
#define QSP_STATUS_SUCCESS 0
#define QSP_STATUS_NAN 1
#define QSP_STATUS_MAXITER 2      /* QSP_NLP_SQP_MERIT: tolerances not met within sqp_iters */
#define QSP_STATUS_QP_FAIL 4      /* acados ACADOS_QP_FAILURE: an infeasible QP (stage0_s_bound with x0's s
                                     outside [lh_s, uh_s]: the instance does not iterate) or a QP whose
                                     interior point diverged (mu >= qp_mu_max or non-finite): the SQP
                                     stops there with its last iterate */

#define QSP_NLP_SQP_RTI_FIXED 0   /* K full Gauss-Newton steps: the BASELINE metric */
#define QSP_NLP_SQP_MERIT 1       /* acados 'SQP' + 'merit_backtracking' with KKT tolerances
                                     (NMPC_controller.m:271-276); sqp_iters = max_iter */

typedef struct qsp_solver qsp_solver;

/* Solver options: NMPC_controller.m:270-300 (create_ocp_opts) + dims. */
typedef struct {
    int32_t struct_size;      /* sizeof(qsp_options) (qsp_default_options sets it)      */
    int32_t N;                /* horizon, param_scheme_N (NMPC_controller.m:281)        */
    int32_t batch;            /* number of lanes B                                      */
    int32_t nlp_mode;         /* QSP_NLP_*                                              */
    int32_t sqp_iters;        /* K (fixed-K mode)                                       */
    int32_t qp_iters;         /* max interior-point iterations per QP                   */
    int32_t stages_per_lane;  /* S in the kernel's lane layout (0 = auto)               */
    int32_t device;           /* HIP device ordinal                                     */
    int32_t cost_scale_Ts;    /* 1: stage cost scaled by Ts as acados does             */
    double Ts;                /* sample time, T = N * Ts (NMPC_controller.m:89,221)     */
    double mu0, t_min, frac, sigma_min, mu_stop;  /* interior-point parameters         */
    /* QSP_NLP_SQP_MERIT only: tol_stat/eq/ineq/comp (NMPC_controller.m:275-276) and the
     * backtracking line search (alpha *= ls_alpha_red while alpha >= ls_alpha_min,
     * Armijo constant ls_eps on the l1 merit function) */
    double tol_stat, tol_eq, tol_ineq, tol_comp;
    double ls_alpha_min, ls_alpha_red, ls_eps;
    double res_stop;          /* interior point stops when mu < mu_stop AND the bound residual < res_stop */
    /* ... AND (HPIPM's other two exit residuals, ocp_qp_ipm res_g / res_b) the stationarity and
     * equality residuals of the IPM iterate are below these (tracked exactly: each Newton step
     * scales them by 1 - alpha); qp_iters caps it (default 20: acados' qp_solver_iter_max 50 is
     * selectable; measured no change in the SQP's rounding sensitivity, 2.3x slower at B = 4 096) */
    double qp_tol_stat, qp_tol_eq;
    int32_t stage0_s_bound;   /* 1 (default): the s bound of h also applies at stage 0 (acados bgh on
                                 stages 0..N-1, NMPC_controller.m:237,251-252); 0: stages 1..N-1 */
    int32_t qp_stall_iters;   /* stall exit (generalises HPIPM's alpha_min exit): a QP whose step length
                                 stays below qp_stall_alpha for qp_stall_iters consecutive iterations is
                                 locally infeasible and stops there; its last iterate is used as at the
                                 cap (qsp_get_qp_stalled counts them); default 3 x 1e-3, 0 = off */
    double qp_stall_alpha;
    double qp_mu_max;         /* divergence exit: a QP whose complementarity mu reaches qp_mu_max (or
                                 turns non-finite) is a QP failure (status 4, the SQP stops with its last
                                 iterate) instead of overflowing to NaN; default 1e100 (mu starts at mu0 = 1:
                                 an overflow guard -- QPs whose mu grows large but finite end at the stall
                                 exit, from which the SQP recovers; measured on the bench workload) */
    int32_t factor_scan;      /* two stages per lane (S = 2: N + 1 > 32, e.g. N = 50) only.  0 (default): the
                                 Riccati factorisation walks the horizon stage by stage, as at S = 1 and in
                                 HPIPM.  1: it runs as an associative (parallel-in-time) scan of the stages'
                                 value-function elements -- configs[4] 110k -> 115k solves/s on one MI355X, but
                                 about two digits less accurate (u0 vs the extended-precision oracle: median
                                 8e-11 instead of 2e-12 after 5 SQP iterations), which the fixed-K SQP's
                                 rounding sensitivity turns into more lanes off the reference */
} qsp_options;

/* One slider shape: object_selection.m:3-42 + PusherSliderModel.m:84-132. */
typedef struct {
    int32_t n_ctrl;                     /* control points, first point repeated last   */
    int32_t struct_size;                /* sizeof(qsp_shape) (qsp_shape_from_ply sets it) */
    double ctrl[QSP_MAX_CTRL][2];       /* contour points [m]                            */
    double knots[QSP_MAX_CTRL + 4];     /* clamped cubic knot vector S (n_ctrl + 4)      */
    double b;                           /* contour length (bspline_shape.m:37)           */
    double c_ellipse;                   /* tau_max / (mu_sg m g)  (PusherSliderModel.m:55) */
    double mu_sp;                       /* pusher-slider friction                        */
    double xwidth;                      /* slider width along x (object_selection.m; the
                                           disturbance re-projection, helper.m:229)       */
} qsp_shape;

/* Device-resident I/O for qsp_solve_device (all pointers on the handle's device). */
typedef struct {
    const double* x0;        /* B x 4              'constr_x0'                 */
    const double* yref;      /* B x N x 6          'cost_y_ref' stages 0..N-1   */
    const double* yref_e;    /* B x 4              'cost_y_ref_e'               */
    const double* X_in;      /* B x (N+1) x 4      'init_x'                     */
    const double* U_in;      /* B x N x 2          'init_u'                     */
    const int32_t* shape_id; /* B (NULL: shape 0)                              */
    double* u0;              /* B x 2              get('u', 0)                  */
    double* X_out;           /* B x (N+1) x 4      get('x')                     */
    double* U_out;           /* B x N x 2          get('u')                     */
    double* PI_out;          /* B x N x 4          get('pi')                    */
    int32_t* status;         /* B                  get('status')                */
    double* cost;            /* B                  get_cost()                   */
    int32_t controller;      /* 1: NMPC_controller.solve semantics (s pre-wrap, cold/warm start,
                                tangential clip, Euler warm-start rollout, shifted X/U/PI out)    */
    int32_t pad_;
    uint8_t* warm_valid;     /* B, controller mode: 0 = cold start (set to 1 on exit); NULL = always cold */
    const double* PI_in;     /* B x N x 4  'init_pi' (NULL: zeros); read by QSP_NLP_SQP_MERIT only */
} qsp_device_io;

/* ---------------------------------------------------------------- lifecycle */
void qsp_default_options(qsp_options* opts);          /* N=20, B=1, K=50, Ts=0.05 ... */
int qsp_create(const qsp_options* opts, qsp_solver** out);   /* acados_ocp(model, opts), :304 */
int qsp_destroy(qsp_solver* s);
const char* qsp_last_error(void);
int qsp_version(void);                                 /* QSP_ABI_VERSION */
int qsp_get_layout(const qsp_solver* s, int32_t* stages_per_lane, int32_t* lanes_per_instance);
/* How the handle's QPs walk the horizon (the solver reports its own options, as acados' print does for
 * ocp_opts, NMPC_controller.m:270-300).  The choice follows N, the layout and factor_scan, and it fixes
 * the rounding order of every result: */
#define QSP_WALK_LANE 0   /* the Riccati recursion as 4x4 algebra on one lane per stage, handed lane to lane */
#define QSP_WALK_MFMA 1   /* the factorisation on the FP64 matrix cores (v_mfma_f64_4x4x4_4b_f64, one
                             instance per 16-lane block): at one stage per lane for 12 <= N <= 31, at two
                             stages per lane from N = 24 (four instances per wave or fewer).  The closed-loop forward and difference passes
                             stay lane walks (at two stages per lane: scans) */
#define QSP_WALK_SCAN 2   /* factor_scan = 1 at two stages per lane: the associative scan */
int qsp_get_factor_walk(const qsp_solver* s, int32_t* walk);

/* ------------------------------------------------------------- model / OCP */
/* PLY contour -> ordered control points, knots, c_ellipse (PusherSliderModel.m:84-132, :53-55). */
int qsp_shape_from_ply(const char* ply_path, int32_t flip, double mu_sg, double mu_sp, double mass,
                       double tau_max, qsp_shape* out);
int qsp_set_shapes(qsp_solver* s, const qsp_shape* shapes, int32_t n_shapes);
int qsp_set_shape_ids(qsp_solver* s, const int32_t* shape_id /* B */);
/* 'cost_W' (stages 0..N-1, diag of blkdiag(W_x, W_u)) and 'cost_W' at stage N (W_x_e)
 * (NMPC_controller.m:153-164).  Only diagonal weights are supported. */
int qsp_set_cost_W(qsp_solver* s, const double W_diag[6], const double W_e_diag[4]);
/* 'constr_lh' / 'constr_uh' for h = [s; u_n; u_t] (NMPC_controller.m:251-252). */
int qsp_set_constr_h(qsp_solver* s, const double lh[3], const double uh[3]);
/* warm-start clip (update_tangential_velocity_bounds, NMPC_controller.m:98-100, 319-327) */
int qsp_set_ctrl_params(qsp_solver* s, double v_alpha, double d_v_bound, double t_angle0, double u_n_lb,
                        double u_t_ub);

/* ------------------------------------------------- acados-level set/solve/get */
int qsp_set_x0(qsp_solver* s, const double* x0 /* B x 4 */);                          /* 'constr_x0' */
int qsp_set_yref(qsp_solver* s, const double* yref /* B x N x 6 */, const double* yref_e /* B x 4 */);
int qsp_set_init(qsp_solver* s, const double* X /* B x (N+1) x 4 */, const double* U /* B x N x 2 */,
                 const double* PI /* B x N x 4 or NULL */);                              /* 'init_*' */
int qsp_solve(qsp_solver* s);                                                           /* .solve() */
int qsp_get_u0(qsp_solver* s, double* u0 /* B x 2 */);                                  /* get('u',0) */
/* get_x/u/pi return the last solve's trajectories; after qsp_controller_solve they are the
 * shifted warm start the controller keeps (xtraj/utraj/ptraj, NMPC_controller.m:392-399). */
int qsp_get_x(qsp_solver* s, double* X);
int qsp_get_u(qsp_solver* s, double* U);
int qsp_get_pi(qsp_solver* s, double* PI);
int qsp_get_cost(qsp_solver* s, double* cost /* B */);
int qsp_get_status(qsp_solver* s, int32_t* status /* B */);
int qsp_get_sqp_iter(qsp_solver* s, int32_t* sqp_iter /* B */);
int qsp_get_qp_iter(qsp_solver* s, int32_t* qp_iter /* B, summed over the SQP iterations */);
/* QPs of the last solve that stopped at the iteration cap qp_iters instead of meeting the stop
 * test (their last iterate is used, as HPIPM's at iter_max): B counts */
int qsp_get_qp_capped(qsp_solver* s, int32_t* capped /* B */);
/* QPs of the last solve stopped by the stall exit (qp_stall_iters steps below qp_stall_alpha;
 * their last iterate is used as at the cap): B counts */
int qsp_get_qp_stalled(qsp_solver* s, int32_t* stalled /* B */);
/* nlp_mode 1 only (else QSP_ERR_STATE): the NLP's KKT residuals of the last test each instance
 * evaluated -- acados' statistics res_stat, res_eq, res_ineq, res_comp (max norms; ocp_nlp_res of
 * the SQP with nlp_solver_tol_* at NMPC_controller.m:275-276).  For status 0 that is the test that
 * passed; for status 2 the test before the last QP (the final iterate after the max_iter-th step is
 * not re-tested); zeros for an instance that never iterated, and before the first solve.
 * Parity unpinned: the reference was run with acados v0.2.1; later acados releases re-linearise and
 * test the final iterate at max_iter, which moves both these residuals and the status 0/2 boundary
 * for an instance that converges on its last step.  No reference fixture fixes either behaviour. */
int qsp_get_residuals(qsp_solver* s, double* res /* B x 4 */);
int qsp_get_time_tot(qsp_solver* s, double* ms);                                        /* 'time_tot' */
/* dims of the handle (outputs of a MEX/FFI layer are sized from these, never from caller input) */
int qsp_get_dims(const qsp_solver* s, int32_t* N, int32_t* B);
/* the acados field-by-field setters: set('cost_y_ref', y, k) for one stage k in 0..N-1 (B x 6),
 * set('cost_y_ref_e', y_e, N) (B x 4), set('init_x'/'init_u'/'init_pi') one at a time */
int qsp_set_yref_stage(qsp_solver* s, int32_t stage, const double* y /* B x 6 */);
int qsp_set_yref_e(qsp_solver* s, const double* y_e /* B x 4 */);
int qsp_set_init_x(qsp_solver* s, const double* X /* B x (N+1) x 4 */);
int qsp_set_init_u(qsp_solver* s, const double* U /* B x N x 2 */);
int qsp_set_init_pi(qsp_solver* s, const double* PI /* B x N x 4 */);
/* acados get('time_tot'/'time_lin'/'time_qp_sol') in seconds (helper.m:264-269): with qsp_set_timing(s, 1)
 * every solve records HIP events at its kernel boundaries and qsp_get_timings reports the last solve
 * (time_lin = the separate linearisation / packing-sort kernels, time_qp_sol = the QP kernels, which in
 * nlp_mode 0 include the fused linearisation); without it time_lin / time_qp_sol are NaN. */
int qsp_set_timing(qsp_solver* s, int32_t on);
int qsp_get_timings(qsp_solver* s, double* time_tot, double* time_lin, double* time_qp_sol);

/* --------------------------------------- NMPC_controller.solve(x0, index_time) */
/* reference table y_ref (6 x T, MATLAB column-major == T x 6 row-major), shared by all lanes
 * (set_reference_trajectory, NMPC_controller.m:425-431 with delay_buff_comp = 0) */
int qsp_set_reference_trajectory(qsp_solver* s, const double* traj /* T x 6 */, int32_t T);
/* one reference table per lane: traj B x T x 6 (scenario sweeps; same staging rule) */
int qsp_set_reference_trajectories(qsp_solver* s, const double* traj /* B x T x 6 */, int32_t T);
/* per-lane TrajectoryGenerator.straight_line generated on the device (TrajectoryGenerator.m:39-79):
 * x0, xf: B x 3 (x, y, theta); samples t0:Ts:tf; rows [x y theta 0 0 0] (main.m:165-178).
 * Installs the tables as with qsp_set_reference_trajectories; T_out (optional) = samples. */
int qsp_gen_straight_lines(qsp_solver* s, const double* x0, const double* xf, double t0, double tf,
                           int32_t auto_angle, int32_t* T_out);
/* copy of the installed table(s): T x 6 (shared) or B x T x 6 (per lane) */
int qsp_get_reference_trajectories(qsp_solver* s, double* traj);
/* x0: B x 4, index_time: B (1-based, as MATLAB).  Warm start lives on the device and is
 * shifted after every call; u0 is available through qsp_get_u0. */
int qsp_controller_solve(qsp_solver* s, const double* x0, const int32_t* index_time);
int qsp_controller_reset(qsp_solver* s);                                                 /* clear_variables */
/* Closed-loop simulation on the device (helper.m:195-322, closed_loop_matlab): cold start of the
 * solver's warm start (X, U, PI), then for t = 0..n_steps-1: x += noise[t] (sim_noise, optional), u = solve(x, index0 + t),
 * x += Ts * f(x, u) (evalModelVariableShape + Euler, :292-307).  x0: B x 4; index0: B (1-based);
 * noise: n_steps x B x 4 or NULL; X_traj: B x (n_steps+1) x 4; U_traj: B x n_steps x 2;
 * status_traj: B x n_steps (found_sol = status == 0) or NULL. */
int qsp_closed_loop(qsp_solver* s, const double* x0, const int32_t* index0, int32_t n_steps, const double* noise,
                    double* X_traj, double* U_traj, int32_t* status_traj);
/* closed_loop_matlab's other branches (helper.m:195-322) */
typedef struct {
    double plant_delay;        /* plant.time_delay [s]: the plant applies u delayed by ceil(delay/Ts) steps
                                  (u_buff_plant, helper.m:211-212, 289-296) */
    int32_t disturbance;       /* disturbance_: at step t_dist (1-based) y += amplitude and the contact
                                  point is re-projected onto the contour (helper.m:221-236) */
    int32_t t_dist;
    const double* amplitude;   /* B amplitude_dist per lane (NULL: 0) */
} qsp_closed_loop_opts;
/* Per step i: disturbance (i == t_dist), noise, the controller's delay prediction (delay_buffer_sim
 * with the handle's delay compensation), u = solve(x_sim, index0 + i - 1 + delay_buff_comp), the
 * controller buffer push, the (delayed) plant step.  X_traj: the plant states after disturbance and
 * noise (B x (n+1) x 4); X_sim (optional): the states handed to the solver (B x n x 4).
 * State carried between calls: the controller's input buffer u_buff_contr is the controller
 * object's (NMPC_controller.m:109), as in helper.m, where it persists across closed_loop_matlab
 * calls: it is NOT reset here (a second closed loop on the same handle starts from the buffer the
 * first one left); only qsp_set_delay_comp zeroes it.  The plant's buffer u_buff_plant is local
 * to one call (helper.m:211-212) and starts at zero.  Both closed-loop entry points behave so. */
int qsp_closed_loop_ex(qsp_solver* s, const qsp_closed_loop_opts* opts, const double* x0, const int32_t* index0,
                       int32_t n_steps, const double* noise, double* X_traj, double* X_sim, double* U_traj,
                       int32_t* status_traj);
/* set_delay_comp (NMPC_controller.m:106-110): delay_buff_comp = ceil(delay / Ts) columns; the
 * reference table is read as set_reference_trajectory prepends it (:425-431) and the per-lane input
 * buffer u_buff_contr is zeroed (the only call that zeroes it).  get: the column count. */
int qsp_set_delay_comp(qsp_solver* s, double delay);
int qsp_get_delay_comp(qsp_solver* s, int32_t* cols);
/* delay_buffer_sim (NMPC_controller.m:112-120): x (B x 4) advanced by delay_buff_comp Euler steps with
 * the buffered inputs, oldest first -> x_sim (B x 4); and the buffer update the caller does after a
 * solve, u_buff_contr = [u, u_buff_contr(:, 1:end-1)] (helper.m:255), u: B x 2. */
int qsp_delay_buffer_sim(qsp_solver* s, const double* x, double* x_sim);
int qsp_delay_buffer_push(qsp_solver* s, const double* u);
/* the disturbance branch's contact re-projection alone: s = argmin |C(s) - (px, py)|^2 from s0 (per
 * lane shape ids; fminunc in helper.m:230, restated as a damped Newton iteration) */
int qsp_reproject_contact(qsp_solver* s, int32_t n, const int32_t* shape_id, const double* px, const double* py,
                          const double* s0, double* s_out);

/* ------------------------------------------------ device-resident fast path */
int qsp_solve_device(qsp_solver* s, const qsp_device_io* io, void* hip_stream);
int qsp_synchronize(qsp_solver* s);
/* The SQP loop of a solve can run in two parts, each half of the lanes iterating on its own
 * HIP stream (forked from and joined back into the solve's stream), so that the tail of one
 * half's QP launch overlaps the other half's work.  Results are bit-identical either way.
 * parts: 0 = auto (two once the batch fills the GPU's wave slots), 1, or 2.  No acados
 * counterpart (an execution choice of the batched engine).  get: the count the next solve uses.
 * Batches whose waves fit the GPU's SIMDs once (nlp_mode 0) run the whole SQP loop in one launch
 * instead (one part; environment QSP_FUSED_LOOP=0/1 at qsp_create overrides the automatic choice).
 * The Riccati factorisation runs on the FP64 matrix cores at one stage per lane for 12 <= N <= 31 and at
 * two stages per lane from N = 24 (qsp_get_factor_walk reports it); environment
 * QSP_MFMA_WALK=0 at qsp_create selects the lane walk instead, a developer A/B that rounds differently
 * (the oracle twin follows the same variable). */
int qsp_set_stream_parts(qsp_solver* s, int32_t parts);
int qsp_get_stream_parts(qsp_solver* s, int32_t* parts);
/* Per-kernel timing (acados' time_lin / time_qp split).  qsp_set_kernel_timing(s, n) pre-creates
 * HIP events for the next n solves (0 disables): every kernel boundary of each solve is then
 * recorded on the solve's stream.  qsp_get_kernel_times synchronises the recorded events and
 * returns the summed milliseconds and launch counts per kernel family in the order
 * {prologue, linearize, qp_step, epilogue}, then re-arms the pool.  With nlp_mode 0 the SQP
 * iteration's linearisation runs inside the qp_step kernel, so "linearize" is only the
 * wave-packing sort before it; with nlp_mode 1 it is the separate linearisation kernel. */
int qsp_set_kernel_timing(qsp_solver* s, int32_t max_solves);
int qsp_get_kernel_times(qsp_solver* s, double* ms /* 4 */, int32_t* launches /* 4 */);

/* ------------------------------------------- building blocks (host arrays) */
int qsp_eval_spline(qsp_solver* s, int32_t n, const int32_t* shape_id, const double* sigma,
                    double* C /* n x 2 */, double* D /* n x 2 */, double* Dd /* n x 2 */, double* kappa /* n */);
int qsp_eval_dynamics(qsp_solver* s, int32_t n, const int32_t* shape_id, const double* x, const double* u,
                      double* f /* n x 4 */, double* J /* n x 4 x 6 */);
int qsp_eval_rk4(qsp_solver* s, int32_t n, const int32_t* shape_id, double h, const double* x, const double* u,
                 double* xn /* n x 4 */, double* A /* n x 4 x 4 */, double* B /* n x 4 x 2 */);
int qsp_eval_vbound(qsp_solver* s, int32_t n, const int32_t* shape_id, const double* sval, double* vb);
/* Batched LQ-QP (interior point) with per-stage data; H and bound widths must be equal on
 * every stage (as in the OCP).  H: nb x (6N+4) diag, g: nb x (6N+4), lo/hi: nb x N x 3,
 * stage-0 s bound as the handle's stage0_s_bound.  qp_status (optional, nb): 0 the stop test
 * was met, 1 non-finite solution, 2 stopped at the iteration cap, 3 infeasible (the fixed
 * stage-0 s = dx0's outside its bounds), 4 stall exit, 5 diverged (mu >= qp_mu_max). */
int qsp_qp_solve(qsp_solver* s, int32_t nb, const double* A, const double* B, const double* b, const double* H,
                 const double* g, const double* lo, const double* hi, const double* dx0, double* dx, double* du,
                 double* pi, double* lam, int32_t* iters, int32_t* qp_status);

#ifdef __cplusplus
}
#endif
#endif /* QSP_NMPC_H */
