/*
 * qsp_demo.c — the reference's main.m closed loop (BASELINE configs[0]: santal, N = 20,
 * one SQP-RTI iteration per control step, 201 steps at Ts = 0.05) driven from plain C
 * through the C ABI alone (include/qsp_nmpc.h), as a non-Python host would bind it.
 *
 *   main.m:44-86     controller = NMPC_controller(...); create_ocp_solver; weights/bounds
 *   main.m:150-178   straight-line reference x_ref(t) = [0.01 t, 0, 0], t = 0:Ts:10
 *   helper.m:195-322 closed_loop_matlab: u = controller.solve(x, index); x += Ts f(x, u)
 *
 * Usage: qsp_demo <santal.ply> <out.txt>   (writes the 201 x 2 control trajectory)
 * Exit status 0 when every step returned status 0.
 */
#include <stdio.h>
#include <stdlib.h>

#include "qsp_nmpc.h"

#define CHECK(call)                                                              \
    do {                                                                         \
        int rc_ = (call);                                                        \
        if (rc_ != QSP_OK) {                                                     \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, qsp_last_error()); \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <santal.ply> <out.txt>\n", argv[0]);
        return 2;
    }
    enum { STEPS = 201, T = 201 };
    qsp_options o;
    qsp_default_options(&o);
    o.N = 20;
    o.batch = 1;
    o.sqp_iters = 1;                 /* SQP-RTI: one iteration per control step */
    qsp_solver* s = NULL;
    CHECK(qsp_create(&o, &s));

    /* object_selection('santal') (object_selection.m:3-9): mu_sg, mu_sp, m, tau_max */
    qsp_shape santal;
    CHECK(qsp_shape_from_ply(argv[1], 0, 0.32, 0.19, 0.2875, 0.0251, &santal));
    CHECK(qsp_set_shapes(s, &santal, 1));

    static double traj[T][6];        /* 6 x T in MATLAB, T x 6 row-major here */
    for (int t = 0; t < T; ++t) traj[t][0] = 0.01 * (0.05 * t);
    CHECK(qsp_set_reference_trajectory(s, &traj[0][0], T));

    static double X[STEPS + 1][4], U[STEPS][2];
    int32_t status[STEPS];
    const double x0[4] = {0.0, 0.0, 0.0, 0.0};
    const int32_t index0 = 1;
    CHECK(qsp_closed_loop(s, x0, &index0, STEPS, NULL, &X[0][0], &U[0][0], status));
    CHECK(qsp_destroy(s));

    FILE* f = fopen(argv[2], "w");
    if (!f) {
        perror(argv[2]);
        return 1;
    }
    int bad = 0;
    for (int k = 0; k < STEPS; ++k) {
        fprintf(f, "%.17g %.17g\n", U[k][0], U[k][1]);
        bad += status[k] != 0;
    }
    fclose(f);
    printf("qsp_demo: %d steps, final x = (%.6f, %.6f, %.6f, %.6f), %d non-zero statuses\n", STEPS, X[STEPS][0],
           X[STEPS][1], X[STEPS][2], X[STEPS][3], bad);
    return bad ? 1 : 0;
}
