/*
 * qsp_nmpc_mex.c — MATLAB MEX gateway over the C ABI (include/qsp_nmpc.h).
 *
 * Replaces the acados MEX layer behind `ocp_solver = acados_ocp(...)`
 * (acados_nmpc/NMPC_controller.m:302-305) for NMPC_controller_hip.m.  One command
 * string per call; the handle is a uint64 scalar owned by the MATLAB object.
 *
 *   h = qsp_nmpc_mex('create', N, B, Ts, sqp_iters)
 *   qsp_nmpc_mex('shape_ply', h, {ply, flip, mu_sg, mu_sp, m, tau_max; ...}, shape_id)
 *   qsp_nmpc_mex('set', h, field, value)         % constr_x0 | cost_y_ref | cost_y_ref_e | init_x | init_u | init_pi
 *   qsp_nmpc_mex('cost_W', h, W6, We4)  /  qsp_nmpc_mex('constr_h', h, lh3, uh3)
 *   qsp_nmpc_mex('ctrl_params', h, v_alpha, d_v, t_angle0, u_n_lb, u_t_ub)
 *   qsp_nmpc_mex('solve', h)                     % acados .solve()
 *   v = qsp_nmpc_mex('get', h, field)            % u0 | x | u | pi | cost | status | sqp_iter | time_tot
 *   qsp_nmpc_mex('reference', h, y_ref)          % 6 x T, set_reference_trajectory (:425-431)
 *   u0 = qsp_nmpc_mex('controller_solve', h, x0, index_time)   % NMPC_controller.solve (:329-423)
 *   qsp_nmpc_mex('reset', h) / qsp_nmpc_mex('destroy', h)
 *
 * MATLAB column-major per-lane arrays (4 x B, 4 x (N+1) x B, ...) are the row-major
 * B x ... blocks of the C ABI, so data passes through without transposes.
 * Build:  mex -R2018a -I../../include qsp_nmpc_mex.c -L../../uclv_qs_pushing_matlab_amd -lqsp_nmpc
 */
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

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char cmd[32];
    if (nrhs < 1 || mxGetString(prhs[0], cmd, sizeof cmd)) mexErrMsgIdAndTxt("qsp:cmd", "first argument: command");
    if (!strcmp(cmd, "create")) {
        if (nrhs != 5) mexErrMsgIdAndTxt("qsp:args", "create(N, B, Ts, sqp_iters)");
        qsp_options o;
        qsp_default_options(&o);
        o.N = (int32_t)mxGetScalar(prhs[1]);
        o.batch = (int32_t)mxGetScalar(prhs[2]);
        o.Ts = mxGetScalar(prhs[3]);
        o.sqp_iters = (int32_t)mxGetScalar(prhs[4]);
        qsp_solver* h = NULL;
        check(qsp_create(&o, &h), "qsp_create");
        plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
        *(uint64_t*)mxGetData(plhs[0]) = (uint64_t)(uintptr_t)h;
        return;
    }
    if (nrhs < 2) mexErrMsgIdAndTxt("qsp:args", "missing handle");
    qsp_solver* h = handle_of(prhs[1]);
    if (!strcmp(cmd, "destroy")) { check(qsp_destroy(h), "qsp_destroy"); return; }
    if (!strcmp(cmd, "reset")) { check(qsp_controller_reset(h), "qsp_controller_reset"); return; }
    if (!strcmp(cmd, "solve")) { check(qsp_solve(h), "qsp_solve"); return; }
    if (!strcmp(cmd, "shape_ply")) {
        /* prhs[2]: n x 6 cell {path, flip, mu_sg, mu_sp, m, tau_max}; prhs[3]: shape_id (B, 0-based) */
        const mxArray* c = prhs[2];
        const size_t n = mxGetM(c);
        qsp_shape* sh = (qsp_shape*)mxCalloc(n, sizeof(qsp_shape));
        for (size_t i = 0; i < n; ++i) {
            char path[1024];
            if (mxGetString(mxGetCell(c, i), path, sizeof path)) mexErrMsgIdAndTxt("qsp:args", "shape path");
            double v[5];
            for (int q = 0; q < 5; ++q) v[q] = mxGetScalar(mxGetCell(c, i + (q + 1) * n));
            check(qsp_shape_from_ply(path, (int32_t)v[0], v[1], v[2], v[3], v[4], &sh[i]), "qsp_shape_from_ply");
        }
        check(qsp_set_shapes(h, sh, (int32_t)n), "qsp_set_shapes");
        mxFree(sh);
        if (nrhs > 3) {
            const size_t B = mxGetNumberOfElements(prhs[3]);
            int32_t* id = (int32_t*)mxMalloc(B * sizeof(int32_t));
            const double* d = mxGetPr(prhs[3]);
            for (size_t i = 0; i < B; ++i) id[i] = (int32_t)d[i];
            check(qsp_set_shape_ids(h, id), "qsp_set_shape_ids");
            mxFree(id);
        }
        return;
    }
    if (!strcmp(cmd, "cost_W")) { check(qsp_set_cost_W(h, dbl(prhs[2], 6, "W"), dbl(prhs[3], 4, "We")), "qsp_set_cost_W"); return; }
    if (!strcmp(cmd, "constr_h")) { check(qsp_set_constr_h(h, dbl(prhs[2], 3, "lh"), dbl(prhs[3], 3, "uh")), "qsp_set_constr_h"); return; }
    if (!strcmp(cmd, "ctrl_params")) {
        check(qsp_set_ctrl_params(h, mxGetScalar(prhs[2]), mxGetScalar(prhs[3]), mxGetScalar(prhs[4]),
                                  mxGetScalar(prhs[5]), mxGetScalar(prhs[6])), "qsp_set_ctrl_params");
        return;
    }
    if (!strcmp(cmd, "reference")) {
        const mxArray* y = prhs[2];
        if (mxGetM(y) != 6) mexErrMsgIdAndTxt("qsp:dims", "y_ref must be 6 x T");
        check(qsp_set_reference_trajectory(h, mxGetPr(y), (int32_t)mxGetN(y)), "qsp_set_reference_trajectory");
        return;
    }
    if (!strcmp(cmd, "controller_solve")) {
        /* x0: 4 x B, index_time: scalar or 1 x B (1-based) */
        const size_t B = mxGetN(prhs[2]);
        if (mxGetM(prhs[2]) != 4) mexErrMsgIdAndTxt("qsp:dims", "x0 must be 4 x B");
        int32_t* idx = (int32_t*)mxMalloc(B * sizeof(int32_t));
        const size_t ni = mxGetNumberOfElements(prhs[3]);
        for (size_t i = 0; i < B; ++i) idx[i] = (int32_t)mxGetPr(prhs[3])[ni == 1 ? 0 : i];
        check(qsp_controller_solve(h, mxGetPr(prhs[2]), idx), "qsp_controller_solve");
        mxFree(idx);
        plhs[0] = mxCreateDoubleMatrix(2, B, mxREAL);
        check(qsp_get_u0(h, mxGetPr(plhs[0])), "qsp_get_u0");
        return;
    }
    if (!strcmp(cmd, "set")) {
        char f[32];
        mxGetString(prhs[2], f, sizeof f);
        const double* v = mxGetPr(prhs[3]);
        if (!strcmp(f, "constr_x0")) check(qsp_set_x0(h, v), "qsp_set_x0");
        else if (!strcmp(f, "cost_y_ref")) check(qsp_set_yref(h, v, mxGetPr(prhs[4])), "qsp_set_yref");
        else if (!strcmp(f, "init")) check(qsp_set_init(h, v, mxGetPr(prhs[4]), nrhs > 5 ? mxGetPr(prhs[5]) : NULL), "qsp_set_init");
        else mexErrMsgIdAndTxt("qsp:field", "unknown field %s", f);
        return;
    }
    if (!strcmp(cmd, "get")) {
        /* prhs[3..4]: sizes (rows, cols) the MATLAB object knows from its dims */
        char f[32];
        mxGetString(prhs[2], f, sizeof f);
        const size_t m = (size_t)mxGetScalar(prhs[3]), n = (size_t)mxGetScalar(prhs[4]);
        if (!strcmp(f, "status") || !strcmp(f, "sqp_iter") || !strcmp(f, "qp_iter")) {
            plhs[0] = mxCreateNumericMatrix(m, n, mxINT32_CLASS, mxREAL);
            int32_t* d = (int32_t*)mxGetData(plhs[0]);
            if (!strcmp(f, "status")) check(qsp_get_status(h, d), "qsp_get_status");
            else if (!strcmp(f, "sqp_iter")) check(qsp_get_sqp_iter(h, d), "qsp_get_sqp_iter");
            else check(qsp_get_qp_iter(h, d), "qsp_get_qp_iter");
            return;
        }
        plhs[0] = mxCreateDoubleMatrix(m, n, mxREAL);
        double* d = mxGetPr(plhs[0]);
        if (!strcmp(f, "u0")) check(qsp_get_u0(h, d), "qsp_get_u0");
        else if (!strcmp(f, "x")) check(qsp_get_x(h, d), "qsp_get_x");
        else if (!strcmp(f, "u")) check(qsp_get_u(h, d), "qsp_get_u");
        else if (!strcmp(f, "pi")) check(qsp_get_pi(h, d), "qsp_get_pi");
        else if (!strcmp(f, "cost")) check(qsp_get_cost(h, d), "qsp_get_cost");
        else if (!strcmp(f, "time_tot")) check(qsp_get_time_tot(h, d), "qsp_get_time_tot");
        else mexErrMsgIdAndTxt("qsp:field", "unknown field %s", f);
        return;
    }
    mexErrMsgIdAndTxt("qsp:cmd", "unknown command %s", cmd);
}
