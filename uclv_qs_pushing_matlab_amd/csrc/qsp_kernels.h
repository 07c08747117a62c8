// qsp_kernels.h — kernel argument blocks and launchers (internal to the .so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qsp_types.h"

#define QSP_FLAG_CONTROLLER 1u  // NMPC_controller.solve prologue: s pre-wrap, cold/warm start, clip, Euler rollout
#define QSP_FLAG_SHIFT 2u       // write the warm start shifted by one stage (NMPC_controller.m:397-399)
#define QSP_FLAG_POISON 4u      // debug (QSP_DEBUG_POISON=1): QP kernels fill their LDS with NaN first

namespace qsp {

struct SolveArgs {
    SolveParams p;
    int32_t B;
    // instance range [i0, i0 + nI) of one QP / line-search launch: launch_sqp may split the
    // batch into parts iterated on their own HIP streams (whist then points at the part's own
    // histogram); strides of the SoA workspace stay B(N+1)
    int32_t i0, nI;
    uint32_t flags;
    const ShapeDev* shapes;
    int32_t n_shapes;
    const int32_t* shape_id;   // B (nullptr: shape 0); clamped into [0, n_shapes)
    const double* x0;          // B x 4
    const double* yref;        // B x N x 6
    const double* yref_e;      // B x 4
    const double* X_in;        // B x (N+1) x 4   initial guess / warm start
    const double* U_in;        // B x N x 2
    uint8_t* warm_valid;       // B (controller mode; nullptr: always cold)
    const double* PI_in;       // B x N x 4   initial dynamics multipliers (nlp_mode 1; nullptr: zeros)
    double* u0;                // B x 2
    double* X_out;             // B x (N+1) x 4
    double* U_out;             // B x N x 2
    double* PI_out;            // B x N x 4
    int32_t* status;           // B
    int32_t* sqp_iter;         // B
    int32_t* qp_iter;          // B (sum of IPM iterations)
    int32_t* qp_capped;        // B (QPs stopped by the iteration cap; nullptr: not counted)
    int32_t* qp_stalled;       // B (QPs stopped by the stall exit; nullptr: not counted)
    double* cost;              // B
    // workspace (device, owned by the handle)
    double* wX;                // B x (N+1) x 4   SQP iterate
    double* wU;                // B x N x 2
    double* wx0;               // B x 4           x0 after the controller's s pre-wrap
    double* wlin;              // 24 x B(N+1)     stage data (A, B, defect, gradient), SoA
    double* wnlp;              // 20 x B(N+1)     nlp_mode 1: PI(4), LAM(6), merit weights NU(4), ETA(6), SoA
    int32_t* wdone;            // B               nlp_mode 1: converged (KKT tolerances met)
    double* wres;              // B x 4           nlp_mode 1: the last KKT test's residuals (stat, eq, ineq, comp;
                               //                 nullptr: not recorded).  At max_iter (status 2) that is the test
                               //                 before the last QP: the final iterate is not re-tested (acados
                               //                 v0.2.1 semantics as restated; unpinned, qsp_nmpc.h)
    double* wqp;               // 16 x B(N+1)     nlp_mode 1: QP step dx(4), du(2), multipliers pi(4), lam(6), SoA
    int32_t* wperm;            // B               wave packing order of the QP kernel (nullptr: identity)
    int32_t* wnit;             // B               IPM iterations of each instance's last four QPs (8 bits each, last lowest)
    int32_t* whist;            // 4 x 1024        per parity of the SQP iteration: histogram of the wave-packing
                               //                 keys (accumulated by the QP kernel) and running scatter offsets
    // QP-level interface only (qsp_qp_solve): when qp_dx != nullptr the QP kernel
    // reports the QP solution instead of updating the iterate
    double* qp_dx;             // B x (N+1) x 4
    double* qp_du;             // B x N x 2
    double* qp_lam;            // B x N x 6
};


int lanes_per_instance(int N, int S);
// QSP_WALK_* of a handle's QP kernels (the same rule the launchers apply: mfw_use, factor_scan)
int factor_walk_kind(const SolveParams& p, int S);
void mfw_prepare(SolveParams& p);   // SolveParams::mfw_on / mfw_is from N and mfma_walk
// Multi-stream split of the SQP loop (SqpStreams::parts = P > 1): the instances are cut into
// P parts and each part runs its own (sort, qp_step) sequence on its own stream (part 0 on
// the solve's stream, part p on aux[p-1]), so the launch tail of one part's QP overlaps the
// other parts' work.  Results are bit-identical to the single-stream loop (instances are
// independent).  Streams and events owned by the handle.
// Two parts at most: measured (scripts/parts_sweep.sh) three or four parts run slower than one
// at every batch size (down to half the rate at B = 4 096) -- with GPU_MAX_HW_QUEUES = 4 the
// extra streams share hardware queues, whose kernels then serialise across parts.
constexpr int SQP_MAX_PARTS = 2;
struct SqpStreams {
    hipStream_t aux[SQP_MAX_PARTS - 1] = {};
    hipEvent_t fork = nullptr, join[SQP_MAX_PARTS - 1] = {};
    int parts = 1;   // 1 .. SQP_MAX_PARTS
    int fused = 0;   // 1: the whole SQP loop in one launch (sqp_loop_kernel; small batches, nlp_mode 0)
};
// ev (optional): 2*sqp_iters + 3 events recorded on `stream` at every kernel boundary
// (prologue | sort, qp_step x sqp_iters | epilogue), for per-kernel timing.  With several
// parts only ev[0], ev[1] (fork), ev[2K+1] (join) and ev[2K+2] are recorded: the SQP loop is
// timed as a whole (qsp_get_kernel_times then reports K qp_step "launches" = SQP iterations).
hipError_t launch_sqp(const SolveArgs& a, int S, hipStream_t stream, hipEvent_t* ev = nullptr,
                      const SqpStreams* split = nullptr);
// cus: compute units of the handle's device (hipDeviceProp multiProcessorCount; 256 on a whole
// MI355X, fewer on a partitioned one)
int sqp_parts_auto(int B, int N, int S, int cus);
int sqp_fused_auto(int B, int N, int S, int nlp_mode, int cus);
hipError_t launch_qp(const SolveArgs& a, int S, hipStream_t stream);   // one QP step on prepared workspace
// Device closed loop (helper.m:195-322): buffers and logs of qsp_closed_loop, one thread per lane.
struct ClosedLoopArgs {
    const ShapeDev* shapes;
    int32_t n_shapes;
    const int32_t* sid;        // B (nullptr: shape 0)
    int32_t B, n_steps;
    double Ts;
    double* x;                 // B x 4   plant state
    double* xs;                // B x 4   state handed to the solver (after the delay prediction)
    const double* noise;       // n_steps x B x 4 (sim_noise) or nullptr
    int32_t dist_step;         // 1-based step of the disturbance (0: none)
    const double* dist_amp;    // B amplitude_dist (nullptr: 0)
    int32_t D, Dp;             // controller delay_buff_comp, plant delay_buff_plant
    double* ubc;               // B x D x 2  u_buff_contr (column 0 = newest)
    double* ubp;               // B x Dp x 2 u_buff_plant
    const double* u0;          // B x 2   the solve's u0
    const int32_t* status;     // B
    double* Xtraj;             // B x (n_steps + 1) x 4
    double* Xsim;              // B x n_steps x 4 or nullptr
    double* Utraj;             // B x n_steps x 2
    int32_t* Straj;            // B x n_steps or nullptr
};
hipError_t launch_closed_loop_pre(const ClosedLoopArgs& a, int t, hipStream_t stream);
hipError_t launch_plant(const ClosedLoopArgs& a, int t, hipStream_t stream);
hipError_t launch_delay_sim(const ClosedLoopArgs& a, hipStream_t stream);   // x -> xs (delay_buffer_sim)
hipError_t launch_reproject(const ShapeDev* shapes, int n_shapes, const int32_t* sid, int n, const double* px,
                            const double* py, const double* s0, double* s, hipStream_t stream);
hipError_t launch_straight_lines(int B, int T, const double* x0, const double* xf, double t0, double tf, double Ts,
                                 int auto_angle, double* traj, hipStream_t stream);
hipError_t launch_spline(const ShapeDev* shapes, const int32_t* sid, int n, const double* s, double* C, double* D,
                         double* Dd, double* kappa, hipStream_t stream);
hipError_t launch_dynamics(const ShapeDev* shapes, const int32_t* sid, int n, const double* x, const double* u,
                           double* f, double* J, hipStream_t stream);
hipError_t launch_rk4(const ShapeDev* shapes, const int32_t* sid, int n, double h, const double* x, const double* u,
                      double* xn, double* A, double* B, hipStream_t stream);
hipError_t launch_vbound(const ShapeDev* shapes, const int32_t* sid, int n, CtrlParams cp, const double* s, double* vb,
                         hipStream_t stream);

}  // namespace qsp
