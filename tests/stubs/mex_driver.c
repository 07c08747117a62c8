/* Drives integration/matlab/qsp_nmpc_mex.c the way NMPC_controller_hip.m + main.m would
 * (test infrastructure): create with the reference's create_ocp_opts defaults (sqp + merit
 * backtracking, max_iter 30, tol 1e-6), santal from its PLY, Hp = 10, the straight-line
 * reference, then main.m's 201-step closed loop (helper.m:195-322) with the Euler plant through
 * qsp_eval_dynamics.  Also exercises the argument checks (each must raise a MEX error).
 * Usage: mex_driver <santal.ply> <out.bin>; writes U (201x2), X (202x4), status, sqp_iter (int32),
 * then the error count and the summed time_lin / time_qp_sol / time_tot (doubles). */
#include <setjmp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"
#include "qsp_nmpc.h"

extern jmp_buf stub_err_jmp;
extern char stub_err_msg[512];

static mxArray* row(const double* v, size_t n) {
    mxArray* a = mxCreateDoubleMatrix(1, n, mxREAL);
    memcpy(mxGetPr(a), v, n * sizeof(double));
    return a;
}

static int call(int nlhs, mxArray** plhs, int nrhs, mxArray** prhs) {
    if (setjmp(stub_err_jmp)) return 1;
    mexFunction(nlhs, plhs, nrhs, (const mxArray**)prhs);
    return 0;
}

#define CALL(nl, pl, ...)                                                              \
    do {                                                                               \
        mxArray* a_[] = {__VA_ARGS__};                                                 \
        if (call(nl, pl, (int)(sizeof a_ / sizeof a_[0]), a_)) {                       \
            fprintf(stderr, "unexpected MEX error: %s\n", stub_err_msg);                \
            return 1;                                                                  \
        }                                                                              \
    } while (0)
#define EXPECT_ERR(...)                                                                \
    do {                                                                               \
        mxArray* a_[] = {__VA_ARGS__};                                                 \
        mxArray* o_[3] = {0};                                                          \
        if (call(1, o_, (int)(sizeof a_ / sizeof a_[0]), a_)) { ++errors; fprintf(stderr, "expected error: %s\n", stub_err_msg); } \
        else { fprintf(stderr, "missing MEX error\n"); return 1; }                     \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <santal.ply> <out.bin>\n", argv[0]);
        return 2;
    }
    enum { STEPS = 201, T = 201, HP = 10 };
    int errors = 0;
    mxArray* out[3] = {0};
    /* h = qsp_nmpc_mex('create', Hp, 1, Ts, opts) -- opts empty: create_ocp_opts defaults */
    CALL(1, out, stub_string("create"), stub_scalar(HP), stub_scalar(1), stub_scalar(0.05), stub_struct());
    mxArray* h = out[0];
    qsp_solver* s = (qsp_solver*)(uintptr_t)(*(uint64_t*)mxGetData(h));
    /* shape_ply: {path, flip, mu_sg, mu_sp, m, tau_max, xwidth} (object_selection.m santal) */
    mxArray* cell = stub_cell(1, 7);
    stub_cell_set(cell, 0, stub_string(argv[1]));
    const double sp[6] = {0, 0.32, 0.19, 0.2875, 0.0251, 0.068};
    for (int q = 0; q < 6; ++q) stub_cell_set(cell, q + 1, stub_scalar(sp[q]));
    CALL(0, out, stub_string("shape_ply"), h, cell, stub_scalar(0));
    const double W[6] = {1, 1, 1e-3, 0, 1e-3, 1e-3}, We[4] = {2e5, 2e5, 20, 0};
    CALL(0, out, stub_string("cost_W"), h, row(W, 6), row(We, 4));
    const double lh[3] = {-0.06, 0, -0.05}, uh[3] = {0.011, 0.03, 0.05};
    CALL(0, out, stub_string("constr_h"), h, row(lh, 3), row(uh, 3));
    CALL(0, out, stub_string("ctrl_params"), h, stub_scalar(1.0), stub_scalar(0.0), stub_scalar(3.0), stub_scalar(0.0),
         stub_scalar(0.05));
    mxArray* dims = NULL;
    CALL(1, &dims, stub_string("dims"), h);
    if (mxGetPr(dims)[0] != HP || mxGetPr(dims)[1] != 1) { fprintf(stderr, "dims\n"); return 1; }
    /* main.m:150-178: y_ref 6 x T, x = 0.01 t */
    mxArray* yref = mxCreateDoubleMatrix(6, T, mxREAL);
    for (int k = 0; k < T; ++k) mxGetPr(yref)[6 * k] = 0.01 * 0.05 * k;
    CALL(0, out, stub_string("reference"), h, yref);
    CALL(0, out, stub_string("reset"), h);
    /* argument checks: wrong element counts, unknown fields, bad stage */
    const double three[3] = {0, 0, 0}, eight[8] = {0};
    EXPECT_ERR(stub_string("set"), h, stub_string("constr_x0"), row(three, 3));
    EXPECT_ERR(stub_string("set"), h, stub_string("cost_y_ref"), row(three, 3), stub_scalar(0));
    EXPECT_ERR(stub_string("set"), h, stub_string("cost_y_ref"), row(eight, 6), stub_scalar(HP));
    EXPECT_ERR(stub_string("set"), h, stub_string("init_u"), row(eight, 8));
    EXPECT_ERR(stub_string("get"), h, stub_string("no_such_field"));
    EXPECT_ERR(stub_string("controller_solve"), h, row(eight, 8), stub_scalar(1));
    EXPECT_ERR(stub_string("no_such_command"), h);
    /* closed loop: u = solve(x, i); plant x += Ts f(x, u) (helper.m:292-307) */
    double U[STEPS][2], X[STEPS + 1][4] = {{0}};
    int32_t ST[STEPS], IT[STEPS];
    double RES[STEPS][4];
    double tl = 0, tq = 0, tt = 0;
    for (int i = 0; i < STEPS; ++i) {
        mxArray* u = NULL;
        CALL(1, &u, stub_string("controller_solve"), h, row(X[i], 4), stub_scalar(i + 1));
        U[i][0] = mxGetPr(u)[0];
        U[i][1] = mxGetPr(u)[1];
        mxArray* st = NULL;
        CALL(1, &st, stub_string("get"), h, stub_string("status"));
        ST[i] = ((int32_t*)mxGetData(st))[0];
        CALL(1, &st, stub_string("get"), h, stub_string("sqp_iter"));
        IT[i] = ((int32_t*)mxGetData(st))[0];
        mxArray* rs = NULL;
        CALL(1, &rs, stub_string("get"), h, stub_string("residuals"));   /* 4 x 1 */
        for (int c = 0; c < 4; ++c) RES[i][c] = mxGetPr(rs)[c];
        mxArray* tv = NULL;
        CALL(1, &tv, stub_string("get"), h, stub_string("time_lin"));
        tl += mxGetScalar(tv);
        CALL(1, &tv, stub_string("get"), h, stub_string("time_qp_sol"));
        tq += mxGetScalar(tv);
        CALL(1, &tv, stub_string("get"), h, stub_string("time_tot"));
        tt += mxGetScalar(tv);
        double f[4], J[24];
        const int32_t sid = 0;
        if (qsp_eval_dynamics(s, 1, &sid, X[i], U[i], f, J) != QSP_OK) { fprintf(stderr, "%s\n", qsp_last_error()); return 1; }
        for (int c = 0; c < 4; ++c) X[i + 1][c] = X[i][c] + 0.05 * f[c];
    }
    mxArray* xg = NULL;
    CALL(1, &xg, stub_string("get"), h, stub_string("x"));   /* sized from the handle: 4 x (Hp+1) x 1 */
    if (mxGetNumberOfElements(xg) != 4 * (HP + 1)) { fprintf(stderr, "get x size\n"); return 1; }
    CALL(0, out, stub_string("destroy"), h);
    FILE* fo = fopen(argv[2], "wb");
    if (!fo) return 1;
    fwrite(U, sizeof U, 1, fo);
    fwrite(X, sizeof X, 1, fo);
    fwrite(ST, sizeof ST, 1, fo);
    fwrite(IT, sizeof IT, 1, fo);
    const double tail[4] = {(double)errors, tl, tq, tt};
    fwrite(tail, sizeof tail, 1, fo);
    fwrite(RES, sizeof RES, 1, fo);
    fclose(fo);
    return 0;
}
