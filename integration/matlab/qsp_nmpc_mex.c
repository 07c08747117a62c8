/*
 * qsp_nmpc_mex.c — MATLAB MEX gateway over the C ABI (include/qsp_nmpc.h).
 *
 * Replaces the acados MEX layer behind `ocp_solver = acados_ocp(ocp_model, ocp_opts)`
 * (acados_nmpc/NMPC_controller.m:302-305) for NMPC_controller_hip.m.  One command string per
 * call; the handle is a uint64 scalar owned by the MATLAB object.  Every output is sized from the
 * handle's own dims (qsp_get_dims) and every input's element count is checked against them before
 * the library reads it.
 *
 *   h = qsp_nmpc_mex('create', N, B, Ts [, opts])      % opts: struct, fields as acados_ocp_opts
 *        nlp_solver_type 'SQP' (default, + merit_backtracking) | 'SQP_RTI' (fixed K full steps)
 *        nlp_solver_max_iter (30 for SQP, 1 for SQP_RTI), nlp_solver_tol_stat/eq/ineq/comp (1e-6),
 *        qp_solver_iter_max (50 for SQP, 20 for SQP_RTI), globalization_alpha_min (0.05), globalization_alpha_reduction
 *        (0.7), eps_sufficient_descent (1e-4), stage0_s_bound (1), stages_per_lane (0 = auto),
 *        factor_scan (0; 1 = the S = 2 factorisation as an associative scan: faster, less accurate),
 *        device (0), qp_solver_cond_N (1..N; validated only, see below)  -- NMPC_controller.m:270-300
 *   d = qsp_nmpc_mex('dims', h)                          % [N B]
 *   qsp_nmpc_mex('shape_ply', h, {ply, flip, mu_sg, mu_sp, m, tau_max, xwidth; ...}, shape_id)
 *   qsp_nmpc_mex('set', h, field, value [, stage])
 *        constr_x0 (4 x B) | cost_y_ref (6 x B at stage k, or 6 x N x B) | cost_y_ref_e (4 x B)
 *        | init_x (4 x (N+1) x B) | init_u (2 x N x B) | init_pi (4 x N x B)
 *   qsp_nmpc_mex('cost_W', h, W6, We4)  /  qsp_nmpc_mex('constr_h', h, lh3, uh3)
 *   qsp_nmpc_mex('ctrl_params', h, v_alpha, d_v, t_angle0, u_n_lb, u_t_ub)
 *   qsp_nmpc_mex('solve', h)                             % acados .solve()
 *   v = qsp_nmpc_mex('get', h, field [, stage])          % u (stage 0: 2 x B) | x | pi | cost |
 *        status | sqp_iter | qp_iter | qp_capped | qp_stalled | time_tot | time_lin | time_qp_sol
 *        | residuals (4 x B: res_stat/eq/ineq/comp of the last KKT test, SQP only)   (helper.m:253,264-269)
 *   qsp_nmpc_mex('reference', h, y_ref)                  % 6 x T, set_reference_trajectory (:425-431)
 *   u0 = qsp_nmpc_mex('controller_solve', h, x0, index_time)   % NMPC_controller.solve (:329-423)
 *   qsp_nmpc_mex('delay_comp', h, delay)                 % set_delay_comp (:106-110)
 *   xs = qsp_nmpc_mex('delay_sim', h, x)                 % delay_buffer_sim (:112-120)
 *   qsp_nmpc_mex('push_u', h, u)                         % u_buff_contr update (helper.m:255)
 *   [X, U, st] = qsp_nmpc_mex('closed_loop', h, x0, n_steps [, opts])   % helper.m:195-322 on the GPU
 *        opts: struct with plant_delay, disturbance, t_dist, amplitude (1 x B)
 *   qsp_nmpc_mex('reset', h) / qsp_nmpc_mex('destroy', h)
 *
 * MATLAB column-major per-lane arrays (4 x B, 4 x (N+1) x B, ...) are the row-major B x ... blocks
 * of the C ABI, so data passes through without transposes.
 * Build:  mex -R2018a -I../../include qsp_nmpc_mex.c -L../../uclv_qs_pushing_matlab_amd -lqsp_nmpc
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "mex.h"
#include "qsp_nmpc.h"

static qsp_solver* handle_of(const mxArray* a) {
    if (!mxIsUint64(a) || mxGetNumberOfElements(a) != 1) mexErrMsgIdAndTxt("qsp:handle", "invalid solver handle");
    return (qsp_solver*)(uintptr_t)(*(uint64_t*)mxGetData(a));
}

static void check(int rc, const char* what) {
    if (rc != QSP_OK) mexErrMsgIdAndTxt("qsp:call", "%s failed (%d): %s", what, rc, qsp_last_error());
}

static const double* dbl(const mxArray* a, size_t n, const char* what) {
    if (!mxIsDouble(a) || mxIsComplex(a) || mxGetNumberOfElements(a) != n)
        mexErrMsgIdAndTxt("qsp:dims", "%s: expected %zu real doubles", what, n);
    return mxGetPr(a);
}

static double scalar(const mxArray* a, const char* what) {
    return *dbl(a, 1, what);
}

static void need(int nrhs, int n, const char* usage) {
    if (nrhs < n) mexErrMsgIdAndTxt("qsp:args", "usage: %s", usage);
}

/* optional struct field: value or the default */
static double opt_num(const mxArray* s, const char* f, double dflt) {
    const mxArray* v = s ? mxGetField(s, 0, f) : NULL;
    return v ? scalar(v, f) : dflt;
}

static void dims_of(qsp_solver* h, size_t* N, size_t* B) {
    int32_t n, b;
    check(qsp_get_dims(h, &n, &b), "qsp_get_dims");
    *N = (size_t)n;
    *B = (size_t)b;
}

static mxArray* new_dbl3(size_t a, size_t b, size_t c) {
    const size_t d[3] = {a, b, c};
    return mxCreateNumericArray(3, d, mxDOUBLE_CLASS, mxREAL);
}

static void cmd_create(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    need(nrhs, 4, "h = create(N, B, Ts [, opts])");
    (void)nlhs;
    const mxArray* op = nrhs > 4 ? prhs[4] : NULL;
    if (op && !mxIsStruct(op)) mexErrMsgIdAndTxt("qsp:args", "create: opts must be a struct");
    qsp_options o;
    qsp_default_options(&o);
    o.N = (int32_t)scalar(prhs[1], "N");
    o.batch = (int32_t)scalar(prhs[2], "B");
    o.Ts = scalar(prhs[3], "Ts");
    /* create_ocp_opts (NMPC_controller.m:270-300): 'sqp' + 'merit_backtracking', max_iter 30, tol 1e-6 */
    o.nlp_mode = QSP_NLP_SQP_MERIT;
    const mxArray* t = op ? mxGetField(op, 0, "nlp_solver_type") : NULL;
    if (t) {
        char buf[16];
        if (mxGetString(t, buf, sizeof buf)) mexErrMsgIdAndTxt("qsp:args", "nlp_solver_type: 'SQP' or 'SQP_RTI'");
        if (!strcmp(buf, "SQP") || !strcmp(buf, "sqp")) o.nlp_mode = QSP_NLP_SQP_MERIT;
        else if (!strcmp(buf, "SQP_RTI") || !strcmp(buf, "sqp_rti")) o.nlp_mode = QSP_NLP_SQP_RTI_FIXED;
        else mexErrMsgIdAndTxt("qsp:args", "nlp_solver_type: 'SQP' or 'SQP_RTI'");
    }
    o.sqp_iters = (int32_t)opt_num(op, "nlp_solver_max_iter", o.nlp_mode == QSP_NLP_SQP_MERIT ? 30 : 1);
    o.tol_stat = opt_num(op, "nlp_solver_tol_stat", 1e-6);
    o.tol_eq = opt_num(op, "nlp_solver_tol_eq", 1e-6);
    o.tol_ineq = opt_num(op, "nlp_solver_tol_ineq", 1e-6);
    o.tol_comp = opt_num(op, "nlp_solver_tol_comp", 1e-6);
    /* acados' qp_solver_iter_max default is 50 (the reference never sets it); the library's own default
     * of 20 serves the fixed-K throughput path */
    o.qp_iters = (int32_t)opt_num(op, "qp_solver_iter_max", o.nlp_mode == QSP_NLP_SQP_MERIT ? 50 : o.qp_iters);
    o.ls_alpha_min = opt_num(op, "globalization_alpha_min", o.ls_alpha_min);
    o.ls_alpha_red = opt_num(op, "globalization_alpha_reduction", o.ls_alpha_red);
    o.ls_eps = opt_num(op, "eps_sufficient_descent", o.ls_eps);
    o.stage0_s_bound = (int32_t)opt_num(op, "stage0_s_bound", o.stage0_s_bound);
    o.factor_scan = (int32_t)opt_num(op, "factor_scan", o.factor_scan);
    o.stages_per_lane = (int32_t)opt_num(op, "stages_per_lane", 0);
    o.device = (int32_t)opt_num(op, "device", 0);
    /* qp_solver_cond_N (NMPC_controller.m:276, 5 there) picks HPIPM's partial condensing: a different
     * factorisation of the same QP, so the solution does not depend on it.  The library always
     * factorises stage-wise, which measured 1.16-3.1x faster than condensed blocks at N = 20 and 50
     * (profiles/r03/cond_block.txt); the field is accepted for drop-in option structs and checked. */
    const double cn = opt_num(op, "qp_solver_cond_N", o.N);
    if (cn != floor(cn) || cn < 1 || cn > o.N) mexErrMsgIdAndTxt("qsp:args", "qp_solver_cond_N: an integer in 1..N");
    qsp_solver* h = NULL;
    check(qsp_create(&o, &h), "qsp_create");
    if (qsp_set_timing(h, 1) != QSP_OK) {   /* acados reports time_lin / time_qp_sol for every solve */
        qsp_destroy(h);
        mexErrMsgIdAndTxt("qsp:call", "qsp_set_timing failed: %s", qsp_last_error());
    }
    plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
    *(uint64_t*)mxGetData(plhs[0]) = (uint64_t)(uintptr_t)h;
}

static void cmd_shape_ply(qsp_solver* h, int nrhs, const mxArray* prhs[]) {
    /* prhs[2]: n x 7 cell {path, flip, mu_sg, mu_sp, m, tau_max, xwidth}; prhs[3]: shape_id (1 x B, 0-based) */
    need(nrhs, 3, "shape_ply(h, {ply, flip, mu_sg, mu_sp, m, tau_max, xwidth; ...} [, shape_id])");
    size_t N, B;
    dims_of(h, &N, &B);
    const mxArray* c = prhs[2];
    if (!mxIsCell(c) || mxGetN(c) < 6 || mxGetM(c) < 1) mexErrMsgIdAndTxt("qsp:args", "shape_ply: n x 7 cell expected");
    const size_t n = mxGetM(c), ncol = mxGetN(c);
    qsp_shape* sh = (qsp_shape*)mxCalloc(n, sizeof(qsp_shape));
    for (size_t i = 0; i < n; ++i) {
        char path[1024];
        if (mxGetString(mxGetCell(c, i), path, sizeof path)) mexErrMsgIdAndTxt("qsp:args", "shape_ply: path");
        double v[5];
        for (int q = 0; q < 5; ++q) v[q] = scalar(mxGetCell(c, i + (q + 1) * n), "shape parameter");
        check(qsp_shape_from_ply(path, (int32_t)v[0], v[1], v[2], v[3], v[4], &sh[i]), "qsp_shape_from_ply");
        if (ncol >= 7) sh[i].xwidth = scalar(mxGetCell(c, i + 6 * n), "xwidth");
    }
    check(qsp_set_shapes(h, sh, (int32_t)n), "qsp_set_shapes");
    mxFree(sh);
    if (nrhs > 3) {
        const double* d = dbl(prhs[3], B, "shape_id (1 x B)");
        int32_t* id = (int32_t*)mxMalloc(B * sizeof(int32_t));
        for (size_t i = 0; i < B; ++i) id[i] = (int32_t)d[i];
        check(qsp_set_shape_ids(h, id), "qsp_set_shape_ids");
        mxFree(id);
    }
}

static void cmd_set(qsp_solver* h, int nrhs, const mxArray* prhs[]) {
    need(nrhs, 4, "set(h, field, value [, stage])");
    size_t N, B;
    dims_of(h, &N, &B);
    char f[32];
    if (mxGetString(prhs[2], f, sizeof f)) mexErrMsgIdAndTxt("qsp:field", "set: field name");
    const mxArray* v = prhs[3];
    const int staged = nrhs > 4;
    if (!strcmp(f, "constr_x0")) {
        check(qsp_set_x0(h, dbl(v, 4 * B, "constr_x0 (4 x B)")), "qsp_set_x0");
    } else if (!strcmp(f, "cost_y_ref")) {
        if (staged) {
            const double k = scalar(prhs[4], "stage");
            if (k < 0 || k >= (double)N || k != floor(k)) mexErrMsgIdAndTxt("qsp:dims", "cost_y_ref: stage 0..N-1");
            check(qsp_set_yref_stage(h, (int32_t)k, dbl(v, 6 * B, "cost_y_ref (6 x B)")), "qsp_set_yref_stage");
        } else {
            const double* y = dbl(v, 6 * N * B, "cost_y_ref (6 x N x B)");
            for (size_t k = 0; k < N; ++k) {   /* lane-major blocks: stage k of lane i at (i N + k) 6 */
                double* col = (double*)mxMalloc(6 * B * sizeof(double));
                for (size_t i = 0; i < B; ++i) memcpy(col + 6 * i, y + (i * N + k) * 6, 6 * sizeof(double));
                check(qsp_set_yref_stage(h, (int32_t)k, col), "qsp_set_yref_stage");
                mxFree(col);
            }
        }
    } else if (!strcmp(f, "cost_y_ref_e")) {
        if (staged && scalar(prhs[4], "stage") != (double)N) mexErrMsgIdAndTxt("qsp:dims", "cost_y_ref_e: stage N only");
        check(qsp_set_yref_e(h, dbl(v, 4 * B, "cost_y_ref_e (4 x B)")), "qsp_set_yref_e");
    } else if (!strcmp(f, "init_x")) {
        check(qsp_set_init_x(h, dbl(v, 4 * (N + 1) * B, "init_x (4 x (N+1) x B)")), "qsp_set_init_x");
    } else if (!strcmp(f, "init_u")) {
        check(qsp_set_init_u(h, dbl(v, 2 * N * B, "init_u (2 x N x B)")), "qsp_set_init_u");
    } else if (!strcmp(f, "init_pi")) {
        check(qsp_set_init_pi(h, dbl(v, 4 * N * B, "init_pi (4 x N x B)")), "qsp_set_init_pi");
    } else {
        mexErrMsgIdAndTxt("qsp:field", "set: unknown field %s", f);
    }
}

static void cmd_get(qsp_solver* h, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    need(nrhs, 3, "v = get(h, field [, stage])");
    size_t N, B;
    dims_of(h, &N, &B);
    char f[32];
    if (mxGetString(prhs[2], f, sizeof f)) mexErrMsgIdAndTxt("qsp:field", "get: field name");
    const int staged = nrhs > 3;
    if (!strcmp(f, "status") || !strcmp(f, "sqp_iter") || !strcmp(f, "qp_iter") || !strcmp(f, "qp_capped") ||
        !strcmp(f, "qp_stalled")) {
        plhs[0] = mxCreateNumericMatrix(1, B, mxINT32_CLASS, mxREAL);
        int32_t* d = (int32_t*)mxGetData(plhs[0]);
        if (!strcmp(f, "status")) check(qsp_get_status(h, d), "qsp_get_status");
        else if (!strcmp(f, "sqp_iter")) check(qsp_get_sqp_iter(h, d), "qsp_get_sqp_iter");
        else if (!strcmp(f, "qp_iter")) check(qsp_get_qp_iter(h, d), "qsp_get_qp_iter");
        else if (!strcmp(f, "qp_stalled")) check(qsp_get_qp_stalled(h, d), "qsp_get_qp_stalled");
        else check(qsp_get_qp_capped(h, d), "qsp_get_qp_capped");
        return;
    }
    if (!strcmp(f, "residuals")) {
        /* res_stat, res_eq, res_ineq, res_comp of each lane's last KKT test ('sqp' only): the
         * residual columns of acados' get('stat') at the lane's last iteration; 4 x B */
        plhs[0] = mxCreateDoubleMatrix(4, B, mxREAL);
        check(qsp_get_residuals(h, mxGetPr(plhs[0])), "qsp_get_residuals");
        return;
    }
    if (!strcmp(f, "time_tot") || !strcmp(f, "time_lin") || !strcmp(f, "time_qp_sol")) {
        double tt, tl, tq;
        check(qsp_get_timings(h, &tt, &tl, &tq), "qsp_get_timings");
        plhs[0] = mxCreateDoubleMatrix(1, 1, mxREAL);
        *mxGetPr(plhs[0]) = !strcmp(f, "time_tot") ? tt : (!strcmp(f, "time_lin") ? tl : tq);
        return;
    }
    if (!strcmp(f, "u") && staged) {
        if (scalar(prhs[3], "stage") != 0.0) mexErrMsgIdAndTxt("qsp:dims", "get('u', k): only stage 0 (u0)");
        plhs[0] = mxCreateDoubleMatrix(2, B, mxREAL);
        check(qsp_get_u0(h, mxGetPr(plhs[0])), "qsp_get_u0");
        return;
    }
    if (!strcmp(f, "u0")) {
        plhs[0] = mxCreateDoubleMatrix(2, B, mxREAL);
        check(qsp_get_u0(h, mxGetPr(plhs[0])), "qsp_get_u0");
    } else if (!strcmp(f, "x")) {
        plhs[0] = new_dbl3(4, N + 1, B);
        check(qsp_get_x(h, mxGetPr(plhs[0])), "qsp_get_x");
    } else if (!strcmp(f, "u")) {
        plhs[0] = new_dbl3(2, N, B);
        check(qsp_get_u(h, mxGetPr(plhs[0])), "qsp_get_u");
    } else if (!strcmp(f, "pi")) {
        plhs[0] = new_dbl3(4, N, B);
        check(qsp_get_pi(h, mxGetPr(plhs[0])), "qsp_get_pi");
    } else if (!strcmp(f, "cost")) {
        plhs[0] = mxCreateDoubleMatrix(1, B, mxREAL);
        check(qsp_get_cost(h, mxGetPr(plhs[0])), "qsp_get_cost");
    } else {
        mexErrMsgIdAndTxt("qsp:field", "get: unknown field %s", f);
    }
}

static void cmd_controller_solve(qsp_solver* h, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    need(nrhs, 4, "u0 = controller_solve(h, x0 (4 x B), index_time (scalar or 1 x B))");
    size_t N, B;
    dims_of(h, &N, &B);
    const double* x0 = dbl(prhs[2], 4 * B, "x0 (4 x B)");
    const size_t ni = mxGetNumberOfElements(prhs[3]);
    if (ni != 1 && ni != B) mexErrMsgIdAndTxt("qsp:dims", "index_time: scalar or 1 x B");
    const double* it = dbl(prhs[3], ni, "index_time");
    int32_t* idx = (int32_t*)mxMalloc(B * sizeof(int32_t));
    for (size_t i = 0; i < B; ++i) idx[i] = (int32_t)it[ni == 1 ? 0 : i];
    check(qsp_controller_solve(h, x0, idx), "qsp_controller_solve");
    mxFree(idx);
    plhs[0] = mxCreateDoubleMatrix(2, B, mxREAL);
    check(qsp_get_u0(h, mxGetPr(plhs[0])), "qsp_get_u0");
}

static void cmd_closed_loop(qsp_solver* h, int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    need(nrhs, 4, "[X, U, status] = closed_loop(h, x0 (4 x B), n_steps [, opts])");
    size_t N, B;
    dims_of(h, &N, &B);
    const double* x0 = dbl(prhs[2], 4 * B, "x0 (4 x B)");
    const double ns = scalar(prhs[3], "n_steps");
    if (!(ns >= 1.0) || ns != floor(ns) || ns > 1e6) mexErrMsgIdAndTxt("qsp:args", "n_steps must be a positive integer");
    const size_t n = (size_t)ns;
    const mxArray* op = nrhs > 4 ? prhs[4] : NULL;
    if (op && !mxIsStruct(op)) mexErrMsgIdAndTxt("qsp:args", "closed_loop: opts must be a struct");
    qsp_closed_loop_opts o;
    memset(&o, 0, sizeof o);
    o.plant_delay = opt_num(op, "plant_delay", 0.0);
    o.disturbance = (int32_t)opt_num(op, "disturbance", 0.0);
    o.t_dist = (int32_t)opt_num(op, "t_dist", 0.0);
    const mxArray* am = op ? mxGetField(op, 0, "amplitude") : NULL;
    o.amplitude = am ? dbl(am, B, "amplitude (1 x B)") : NULL;
    int32_t* idx = (int32_t*)mxMalloc(B * sizeof(int32_t));
    for (size_t i = 0; i < B; ++i) idx[i] = 1;
    mxArray* X = new_dbl3(4, n + 1, B);
    mxArray* U = new_dbl3(2, n, B);
    mxArray* S = mxCreateNumericMatrix(n, B, mxINT32_CLASS, mxREAL);
    check(qsp_closed_loop_ex(h, &o, x0, idx, (int32_t)n, NULL, mxGetPr(X), NULL, mxGetPr(U), (int32_t*)mxGetData(S)),
          "qsp_closed_loop_ex");
    mxFree(idx);
    plhs[0] = X;
    if (nlhs > 1) plhs[1] = U; else mxDestroyArray(U);
    if (nlhs > 2) plhs[2] = S; else mxDestroyArray(S);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char cmd[32];
    if (nrhs < 1 || mxGetString(prhs[0], cmd, sizeof cmd)) mexErrMsgIdAndTxt("qsp:cmd", "first argument: command");
    if (!strcmp(cmd, "create")) { cmd_create(nlhs, plhs, nrhs, prhs); return; }
    need(nrhs, 2, "command(h, ...)");
    qsp_solver* h = handle_of(prhs[1]);
    if (!strcmp(cmd, "destroy")) { check(qsp_destroy(h), "qsp_destroy"); return; }
    if (!strcmp(cmd, "reset")) { check(qsp_controller_reset(h), "qsp_controller_reset"); return; }
    if (!strcmp(cmd, "solve")) { check(qsp_solve(h), "qsp_solve"); return; }
    if (!strcmp(cmd, "dims")) {
        size_t N, B;
        dims_of(h, &N, &B);
        plhs[0] = mxCreateDoubleMatrix(1, 2, mxREAL);
        mxGetPr(plhs[0])[0] = (double)N;
        mxGetPr(plhs[0])[1] = (double)B;
        return;
    }
    if (!strcmp(cmd, "shape_ply")) { cmd_shape_ply(h, nrhs, prhs); return; }
    if (!strcmp(cmd, "set")) { cmd_set(h, nrhs, prhs); return; }
    if (!strcmp(cmd, "get")) { cmd_get(h, plhs, nrhs, prhs); return; }
    if (!strcmp(cmd, "controller_solve")) { cmd_controller_solve(h, plhs, nrhs, prhs); return; }
    if (!strcmp(cmd, "closed_loop")) { cmd_closed_loop(h, nlhs, plhs, nrhs, prhs); return; }
    if (!strcmp(cmd, "cost_W")) {
        need(nrhs, 4, "cost_W(h, W6, We4)");
        check(qsp_set_cost_W(h, dbl(prhs[2], 6, "W (6)"), dbl(prhs[3], 4, "We (4)")), "qsp_set_cost_W");
        return;
    }
    if (!strcmp(cmd, "constr_h")) {
        need(nrhs, 4, "constr_h(h, lh3, uh3)");
        check(qsp_set_constr_h(h, dbl(prhs[2], 3, "lh (3)"), dbl(prhs[3], 3, "uh (3)")), "qsp_set_constr_h");
        return;
    }
    if (!strcmp(cmd, "ctrl_params")) {
        need(nrhs, 7, "ctrl_params(h, v_alpha, d_v, t_angle0, u_n_lb, u_t_ub)");
        check(qsp_set_ctrl_params(h, scalar(prhs[2], "v_alpha"), scalar(prhs[3], "d_v"), scalar(prhs[4], "t_angle0"),
                                  scalar(prhs[5], "u_n_lb"), scalar(prhs[6], "u_t_ub")), "qsp_set_ctrl_params");
        return;
    }
    if (!strcmp(cmd, "reference")) {
        need(nrhs, 3, "reference(h, y_ref (6 x T))");
        const mxArray* y = prhs[2];
        if (!mxIsDouble(y) || mxIsComplex(y) || mxGetM(y) != 6 || mxGetN(y) < 1)
            mexErrMsgIdAndTxt("qsp:dims", "y_ref must be 6 x T real doubles");
        check(qsp_set_reference_trajectory(h, mxGetPr(y), (int32_t)mxGetN(y)), "qsp_set_reference_trajectory");
        return;
    }
    if (!strcmp(cmd, "delay_comp")) {
        need(nrhs, 3, "delay_comp(h, delay)");
        check(qsp_set_delay_comp(h, scalar(prhs[2], "delay")), "qsp_set_delay_comp");
        return;
    }
    if (!strcmp(cmd, "delay_sim") || !strcmp(cmd, "push_u")) {
        need(nrhs, 3, "delay_sim(h, x (4 x B)) / push_u(h, u (2 x B))");
        size_t N, B;
        dims_of(h, &N, &B);
        if (!strcmp(cmd, "push_u")) {
            check(qsp_delay_buffer_push(h, dbl(prhs[2], 2 * B, "u (2 x B)")), "qsp_delay_buffer_push");
            return;
        }
        plhs[0] = mxCreateDoubleMatrix(4, B, mxREAL);
        check(qsp_delay_buffer_sim(h, dbl(prhs[2], 4 * B, "x (4 x B)"), mxGetPr(plhs[0])), "qsp_delay_buffer_sim");
        return;
    }
    mexErrMsgIdAndTxt("qsp:cmd", "unknown command %s", cmd);
}
