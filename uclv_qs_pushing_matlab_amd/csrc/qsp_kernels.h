// qsp_kernels.h — kernel argument blocks and launchers (internal to the .so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qsp_types.h"

#define QSP_FLAG_CONTROLLER 1u  // NMPC_controller.solve prologue: s pre-wrap, cold/warm start, clip, Euler rollout
#define QSP_FLAG_SHIFT 2u       // write the warm start shifted by one stage (NMPC_controller.m:397-399)

namespace qsp {

struct SolveArgs {
    SolveParams p;
    int32_t B;
    uint32_t flags;
    const ShapeDev* shapes;
    const int32_t* shape_id;   // B (nullptr: shape 0)
    const double* x0;          // B x 4
    const double* yref;        // B x N x 6
    const double* yref_e;      // B x 4
    const double* X_in;        // B x (N+1) x 4   initial guess / warm start
    const double* U_in;        // B x N x 2
    uint8_t* warm_valid;       // B (controller mode; nullptr: always cold)
    double* u0;                // B x 2
    double* X_out;             // B x (N+1) x 4
    double* U_out;             // B x N x 2
    double* PI_out;            // B x N x 4
    int32_t* status;           // B
    int32_t* sqp_iter;         // B
    int32_t* qp_iter;          // B (sum of IPM iterations)
    double* cost;              // B
};

struct QPArgs {
    SolveParams p;             // tau = 1, W = stage Hessian diag, We = terminal Hessian diag
    int32_t nb;
    double width[3];           // hi - lo per bounded component (equal on every stage)
    const double* A;           // nb x N x 16 (pusher-slider structure)
    const double* B;           // nb x N x 8
    const double* b;           // nb x N x 4
    const double* g;           // nb x (6N + 4)
    const double* lo;          // nb x N x 3
    const double* dx0;         // nb x 4
    double* dx;                // nb x (N+1) x 4
    double* du;                // nb x N x 2
    double* pi;                // nb x N x 4
    double* lam;               // nb x N x 6
    int32_t* iters;            // nb
};

int lanes_per_instance(int N, int S);
hipError_t launch_sqp(const SolveArgs& a, int S, hipStream_t stream);
hipError_t launch_qp(const QPArgs& a, int S, hipStream_t stream);
hipError_t launch_spline(const ShapeDev* shapes, const int32_t* sid, int n, const double* s, double* C, double* D,
                         double* Dd, double* kappa, hipStream_t stream);
hipError_t launch_dynamics(const ShapeDev* shapes, const int32_t* sid, int n, const double* x, const double* u,
                           double* f, double* J, hipStream_t stream);
hipError_t launch_rk4(const ShapeDev* shapes, const int32_t* sid, int n, double h, const double* x, const double* u,
                      double* xn, double* A, double* B, hipStream_t stream);
hipError_t launch_vbound(const ShapeDev* shapes, const int32_t* sid, int n, CtrlParams cp, const double* s, double* vb,
                         hipStream_t stream);

}  // namespace qsp
