// qsp_capi.hip — C ABI (include/qsp_nmpc.h): handle, device buffers, set/solve/get.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/qsp_nmpc.h"
#include "qsp_kernels.h"

using namespace qsp;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) return fail(QSP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) n = bytes;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct qsp_solver {
    qsp_options o;
    SolveParams p;
    int S = 1;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int n_shapes = 0;
    DevBuf shapes, shape_id, x0, yref, yref_e, X, U, PI, Xo, Uo, PIo, u0, status, sqp_iter, qp_iter, qp_capped, qp_stalled, cost;
    DevBuf warm_valid, traj, index_time;
    // delay compensation (set_delay_comp, NMPC_controller.m:106-110): delay_buff_comp columns and the
    // per-lane controller input buffer u_buff_contr (B x D x 2, column 0 newest); closed-loop state
    int32_t D = 0;
    DevBuf ubc, ubp, cl_x, cl_xsim, cl_amp;
    DevBuf wX, wU, wx0, wlin, wnlp, wdone, wres, wqp, wperm, wnit, whist;
    DevBuf scratch[12];
    int32_t T = 0;
    bool have_traj = false;
    bool traj_per_lane = false;     // reference table per lane (B x T x 6) instead of shared (T x 6)
    float last_ms = 0.0f;
    bool last_controller = false;
    bool poison = false;            // QSP_DEBUG_POISON=1: NaN-filled workspace and QP-kernel LDS   // get_x/u/pi: controller mode returns the shifted warm start (utraj/xtraj/ptraj)
    std::vector<hipEvent_t> kev;   // kernel-timing pool (qsp_set_kernel_timing)
    int kev_used = 0;
    std::vector<int> kev_solves;   // event offset of each timed solve
    std::vector<int> kev_split;    // ... and whether its SQP loop ran in two parts
    bool auto_timing = false;      // qsp_set_timing: every solve times its kernels (acados time_lin / time_qp_sol)
    // two-stream SQP loop (launch_sqp): second stream, fork/join events, requested parts (0 = auto)
    SqpStreams split;
    int parts_req = 0;
    int fused_req = -1;            // QSP_FUSED_LOOP (-1: auto)
    bool nopack = false;           // QSP_PACKING=0: instances in lane order (developer A/B of the wave packing)
    bool mfw = true;               // QSP_MFMA_WALK=0: the lane walk wherever the matrix cores would factorise
                                   // (developer A/B; rounds differently: the oracle twin reads the same variable)
    int cus = 256;                 // compute units of the device (hipDeviceProp multiProcessorCount)
};

// --------------------------------------------------------------- helpers
static const SqpStreams* sqp_split(qsp_solver* s) {
    s->split.parts = s->parts_req > 0 ? s->parts_req : sqp_parts_auto(s->o.batch, s->o.N, s->S, s->cus);
    // the whole SQP loop in one launch: auto for batches below one fill of the wave slots
    // when one part is in use; QSP_FUSED_LOOP=0/1 overrides (experiments, parity tests) where
    // the fused kernel exists (nlp_mode 0, S = 1 or 2)
    const bool can_fuse = s->o.nlp_mode == QSP_NLP_SQP_RTI_FIXED && (s->S == 1 || s->S == 2);
    s->split.fused = !can_fuse ? 0
                   : s->fused_req >= 0 ? s->fused_req
                   : (s->split.parts == 1 && sqp_fused_auto(s->o.batch, s->o.N, s->S, s->o.nlp_mode, s->cus));
    if (s->split.fused) s->split.parts = 1;
    return &s->split;
}

// events for one timed solve (nullptr when timing is off or the pool is used up); with
// qsp_set_timing the one-solve pool is reused by every solve (the last one is reported)
static hipEvent_t* take_kernel_events(qsp_solver* s) {
    const int per = 2 * s->o.sqp_iters + 3;
    if (s->auto_timing) {
        s->kev_used = 0;
        s->kev_solves.clear();
        s->kev_split.clear();
    }
    if (s->kev.empty() || s->kev_used + per > (int)s->kev.size()) return nullptr;
    s->kev_solves.push_back(s->kev_used);
    s->kev_split.push_back((sqp_split(s)->parts > 1 || s->split.fused) ? 1 : 0);
    hipEvent_t* e = s->kev.data() + s->kev_used;
    s->kev_used += per;
    return e;
}

static int kernel_times_of(qsp_solver* s, double* ms, int32_t* launches);

static void fill_params(qsp_solver* s) {
    SolveParams& p = s->p;
    p.N = s->o.N;
    p.nlp_mode = s->o.nlp_mode;
    p.sqp_iters = s->o.sqp_iters;
    p.qp_iters = s->o.qp_iters;
    p.Ts = s->o.Ts;
    p.tau = s->o.cost_scale_Ts ? s->o.Ts : 1.0;
    p.mu0 = s->o.mu0;
    p.t_min = s->o.t_min;
    p.frac = s->o.frac;
    p.sigma_min = s->o.sigma_min;
    p.mu_stop = s->o.mu_stop;
    p.res_stop = s->o.res_stop;
    p.qp_tol_stat = s->o.qp_tol_stat;
    p.qp_tol_eq = s->o.qp_tol_eq;
    p.s0_bound = s->o.stage0_s_bound ? 1 : 0;
    p.factor_scan = s->o.factor_scan ? 1 : 0;
    p.mfma_walk = s->mfw ? 1 : 0;
    mfw_prepare(p);
    p.qp_stall_iters = s->o.qp_stall_iters;
    p.qp_stall_alpha = s->o.qp_stall_alpha;
    p.qp_mu_max = s->o.qp_mu_max;
    p.tol_stat = s->o.tol_stat;
    p.tol_eq = s->o.tol_eq;
    p.tol_ineq = s->o.tol_ineq;
    p.tol_comp = s->o.tol_comp;
    p.ls_alpha_min = s->o.ls_alpha_min;
    p.ls_alpha_red = s->o.ls_alpha_red;
    p.ls_eps = s->o.ls_eps;
}

static int auto_S(int N) {
    // One stage per lane keeps the QP kernel at 2 waves/SIMD with its closed-loop walks and
    // wins while a wavefront still holds two or more instances; once one stage per lane leaves
    // a single instance per wave (N + 1 > 32), two stages per lane (1 wave/SIMD, 2-3 instances
    // per wave) win.  scripts/layout_sweep.sh, round 1 (one-wave workgroups): N = 10 1.32M vs
    // 1.17M, N = 20 493k vs 422k, N = 50 (B = 16 384) 62.6k vs 70.0k solves/s for S = 1 vs 2.
    return N + 1 <= 32 ? 1 : 2;
}

// Binary little-endian PLY with float32 vertex properties (the reference's cad_models/*.ply).
static int read_ply_xy(const char* path, std::vector<float>& xy) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(QSP_ERR_IO, std::string("cannot open ") + path);
    std::string hdr;
    char line[512];
    int nv = -1, nprop = 0;
    bool binle = false;
    while (std::fgets(line, sizeof line, f)) {
        std::string l(line);
        if (l.rfind("format binary_little_endian", 0) == 0) binle = true;
        if (l.rfind("element vertex", 0) == 0) nv = std::atoi(l.c_str() + 14);
        if (l.rfind("property float", 0) == 0) ++nprop;
        if (l.rfind("property list", 0) == 0 && nv < 0) { std::fclose(f); return fail(QSP_ERR_IO, "unsupported PLY"); }
        if (l.rfind("end_header", 0) == 0) break;
    }
    if (!binle || nv <= 0 || nprop < 2) { std::fclose(f); return fail(QSP_ERR_IO, std::string("unsupported PLY ") + path); }
    std::vector<float> v((size_t)nv * nprop);
    if (std::fread(v.data(), sizeof(float), v.size(), f) != v.size()) { std::fclose(f); return fail(QSP_ERR_IO, "short PLY"); }
    std::fclose(f);
    xy.resize((size_t)nv * 2);
    for (int i = 0; i < nv; ++i) { xy[2 * i] = v[(size_t)i * nprop]; xy[2 * i + 1] = v[(size_t)i * nprop + 1]; }
    return QSP_OK;
}

static int h2d(qsp_solver* s, DevBuf& b, const void* src, size_t bytes) {
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}
static int d2h(qsp_solver* s, void* dst, const DevBuf& b, size_t bytes) {
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(hipMemcpyAsync(dst, b.p, bytes, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

static SolveArgs make_args(qsp_solver* s) {
    SolveArgs a;
    std::memset(&a, 0, sizeof a);
    a.p = s->p;
    a.B = s->o.batch;
    a.shapes = s->shapes.as<ShapeDev>();
    a.n_shapes = s->n_shapes;
    a.shape_id = s->shape_id.as<int32_t>();
    a.x0 = s->x0.as<double>();
    a.yref = s->yref.as<double>();
    a.yref_e = s->yref_e.as<double>();
    a.X_in = s->X.as<double>();
    a.U_in = s->U.as<double>();
    a.u0 = s->u0.as<double>();
    a.X_out = s->Xo.as<double>();
    a.U_out = s->Uo.as<double>();
    a.PI_out = s->PIo.as<double>();
    s->last_controller = false;
    a.status = s->status.as<int32_t>();
    a.sqp_iter = s->sqp_iter.as<int32_t>();
    a.qp_iter = s->qp_iter.as<int32_t>();
    a.qp_capped = s->qp_capped.as<int32_t>();
    a.qp_stalled = s->qp_stalled.as<int32_t>();
    a.cost = s->cost.as<double>();
    a.wX = s->wX.as<double>();
    a.wU = s->wU.as<double>();
    a.wx0 = s->wx0.as<double>();
    a.wlin = s->wlin.as<double>();
    a.wnlp = s->wnlp.as<double>();
    a.wdone = s->wdone.as<int32_t>();
    a.wres = s->wres.as<double>();
    a.wqp = s->wqp.as<double>();
    a.wperm = s->nopack ? nullptr : s->wperm.as<int32_t>();
    if (s->poison) a.flags |= QSP_FLAG_POISON;
    a.wnit = s->wnit.as<int32_t>();
    a.whist = s->whist.as<int32_t>();
    a.PI_in = s->PI.as<double>();   // 'init_pi' (solve) / shifted warm start (controller)
    return a;
}

static int run_timed(qsp_solver* s, const SolveArgs& a) {
    HIPCHK(hipEventRecord(s->ev0, s->stream));
    HIPCHK(launch_sqp(a, s->S, s->stream, take_kernel_events(s), sqp_split(s)));
    HIPCHK(hipEventRecord(s->ev1, s->stream));
    HIPCHK(hipEventSynchronize(s->ev1));
    HIPCHK(hipEventElapsedTime(&s->last_ms, s->ev0, s->ev1));
    return QSP_OK;
}

template <class T>
static int stage_in(qsp_solver* s, DevBuf& b, const T* src, size_t count) {
    HIPCHK(b.ensure(count * sizeof(T)));
    HIPCHK(hipMemcpyAsync(b.p, src, count * sizeof(T), hipMemcpyHostToDevice, s->stream));
    return QSP_OK;
}
template <class T>
static int stage_out(qsp_solver* s, T* dst, DevBuf& b, size_t count) {
    HIPCHK(hipMemcpyAsync(dst, b.p, count * sizeof(T), hipMemcpyDeviceToHost, s->stream));
    return QSP_OK;
}

static int check_ids(qsp_solver* s, int32_t n, const int32_t* ids) {
    if (s->n_shapes < 1) return fail(QSP_ERR_STATE, "no shapes set");
    for (int i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= s->n_shapes) return fail(QSP_ERR_ARG, "shape id out of range");
    return QSP_OK;
}

__global__ void stage_yref_kernel(const double* traj, int T, int per_lane, const int32_t* index_time, int offset,
                                  int D, int B, int N, double* yref, double* yref_e) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    if (per_lane) traj += (size_t)i * T * 6;
    // get_y_ref (NMPC_controller.m:307-313): column index_time+k (1-based) of the table as
    // set_reference_trajectory (:425-431) builds it -- D = delay_buff_comp zero columns prepended,
    // their u_t-reference row copied from the first real column -- clamped to the last column
    for (int k = 0; k < N; ++k) {
        int idx = index_time[i] + offset + k;
        if (idx > T + D) idx = T + D;
        if (idx < 1) idx = 1;
        double* out = yref + ((size_t)i * N + k) * 6;
        if (idx <= D) {
            for (int c = 0; c < 5; ++c) out[c] = 0.0;
            out[5] = traj[5];
        } else {
            for (int c = 0; c < 6; ++c) out[c] = traj[(size_t)(idx - D - 1) * 6 + c];
        }
    }
    // terminal reference = last stage reference (:348)
    for (int c = 0; c < 4; ++c) yref_e[(size_t)i * 4 + c] = yref[((size_t)i * N + N - 1) * 6 + c];
}

// y_ref staging for the controller step at index_time + offset
static hipError_t launch_controller_step(qsp_solver* s, int offset) {
    const size_t B = s->o.batch;
    hipLaunchKernelGGL(stage_yref_kernel, dim3((unsigned)((B + 127) / 128)), dim3(128), 0, s->stream,
                       s->traj.as<double>(), s->T, s->traj_per_lane ? 1 : 0, s->index_time.as<int32_t>(), offset,
                       s->D, (int)B, s->o.N,
                       s->yref.as<double>(), s->yref_e.as<double>());
    return hipGetLastError();
}

// NMPC_controller.solve arguments: warm buffers updated in place (each instance reads its
// own stages before writing), shifted outputs
static SolveArgs controller_args(qsp_solver* s) {
    SolveArgs a = make_args(s);
    a.flags |= QSP_FLAG_CONTROLLER | QSP_FLAG_SHIFT;
    a.warm_valid = s->warm_valid.as<uint8_t>();
    a.X_out = s->X.as<double>();
    a.U_out = s->U.as<double>();
    a.PI_out = s->PI.as<double>();
    s->last_controller = true;
    return a;
}

extern "C" {

void qsp_default_options(qsp_options* o) {
    std::memset(o, 0, sizeof(*o));
    o->N = 20;
    o->batch = 1;
    o->nlp_mode = QSP_NLP_SQP_RTI_FIXED;
    o->sqp_iters = 50;
    o->qp_iters = 20;               // acados qp_solver_iter_max is 50: measured no effect on chaos, 2.3x slower at B = 4 096
    o->stages_per_lane = 0;
    o->device = 0;
    o->cost_scale_Ts = 1;
    o->Ts = 0.05;
    o->mu0 = 1.0;
    o->t_min = 1e-2;
    o->frac = 0.995;
    o->sigma_min = 1e-2;
    o->mu_stop = 1e-10;
    o->res_stop = 1e-10;
    o->qp_tol_stat = 1e-10;
    o->qp_tol_eq = 1e-10;
    o->stage0_s_bound = 1;          // acados: bgh constraints on stages 0..N-1
    o->qp_stall_iters = 3;          // stall exit: alpha < 1e-3 three times in a row
    o->qp_stall_alpha = 1e-3;
    o->qp_mu_max = 1e100;           // divergence exit: overflow guard
    o->factor_scan = 0;             // S = 2 factorisation: the walk (the scan is faster, less accurate: DESIGN.md 4)
    o->struct_size = (int32_t)sizeof(qsp_options);
    // nlp_mode 1: NMPC_controller.m:275-276 tolerances; acados merit_backtracking defaults
    o->tol_stat = o->tol_eq = o->tol_ineq = o->tol_comp = 1e-6;
    o->ls_alpha_min = 0.05;
    o->ls_alpha_red = 0.7;
    o->ls_eps = 1e-4;
}

int qsp_version(void) { return QSP_ABI_VERSION; }

const char* qsp_last_error(void) { return g_err.c_str(); }

int qsp_create(const qsp_options* o, qsp_solver** out) {
    if (!o || !out) return fail(QSP_ERR_ARG, "qsp_create: null argument");
    if (o->struct_size != (int32_t)sizeof(qsp_options))
        return fail(QSP_ERR_ARG, "qsp_create: qsp_options.struct_size != sizeof(qsp_options) (caller built "
                                 "against another qsp_nmpc.h? check qsp_version() == QSP_ABI_VERSION)");
    if (!(o->qp_mu_max > 0.0)) return fail(QSP_ERR_ARG, "qsp_create: qp_mu_max must be > 0");
    if (o->N < 1 || o->batch < 1) return fail(QSP_ERR_ARG, "qsp_create: N and batch must be >= 1");
    if (o->nlp_mode != QSP_NLP_SQP_RTI_FIXED && o->nlp_mode != QSP_NLP_SQP_MERIT)
        return fail(QSP_ERR_ARG, "qsp_create: unsupported nlp_mode");
    if (o->nlp_mode == QSP_NLP_SQP_MERIT &&
        (o->N + 1 > 64 || o->stages_per_lane > 1 || !(o->ls_alpha_red > 0.0 && o->ls_alpha_red < 1.0) ||
         !(o->ls_alpha_min > 0.0 && o->ls_alpha_min <= 1.0)))
        return fail(QSP_ERR_ARG, "qsp_create: nlp_mode 1 needs N+1 <= 64 (one stage per lane), "
                                 "0 < ls_alpha_red < 1 and 0 < ls_alpha_min <= 1");
    if (o->sqp_iters < 1 || o->qp_iters < 1) return fail(QSP_ERR_ARG, "qsp_create: iteration counts must be >= 1");
    if (o->qp_iters > 255) return fail(QSP_ERR_ARG, "qsp_create: qp_iters must be <= 255");
    if (o->qp_stall_iters < 0) return fail(QSP_ERR_ARG, "qsp_create: qp_stall_iters must be >= 0");
    if (o->factor_scan != 0 && o->factor_scan != 1) return fail(QSP_ERR_ARG, "qsp_create: factor_scan must be 0 or 1");
    if (!(o->qp_tol_stat > 0.0) || !(o->qp_tol_eq > 0.0) || !(o->mu_stop > 0.0) || !(o->res_stop > 0.0))
        return fail(QSP_ERR_ARG, "qsp_create: QP stop tolerances must be > 0");
    if (!(o->Ts > 0.0)) return fail(QSP_ERR_ARG, "qsp_create: Ts must be > 0");
    int S = o->stages_per_lane > 0 ? o->stages_per_lane : (o->nlp_mode == QSP_NLP_SQP_MERIT ? 1 : auto_S(o->N));
    if (S < 1 || S > 2) return fail(QSP_ERR_ARG, "qsp_create: stages_per_lane must be 1 or 2");
    if (lanes_per_instance(o->N, S) > 64)
        return fail(QSP_ERR_ARG, "qsp_create: N+1 > 64*stages_per_lane (one instance must fit in a wavefront)");
    HIPCHK(hipSetDevice(o->device));
    qsp_solver* s = new qsp_solver();
    s->o = *o;
    s->S = S;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, o->device) == hipSuccess && prop.multiProcessorCount > 0)
            s->cus = prop.multiProcessorCount;
    }
    fill_params(s);
    // reference defaults (main.m:82-90, NMPC_controller.m:16-26, 98-100, 251-252)
    const double W[6] = {1.0, 1.0, 1e-3, 0.0, 1e-3, 1e-3};
    const double We[4] = {2e5, 2e5, 20.0, 0.0};
    const double lh[3] = {-0.06, 0.0, -0.05}, uh[3] = {0.011, 0.03, 0.05};
    std::memcpy(s->p.W, W, sizeof W);
    std::memcpy(s->p.We, We, sizeof We);
    std::memcpy(s->p.lh, lh, sizeof lh);
    std::memcpy(s->p.uh, uh, sizeof uh);
    s->p.cp = CtrlParams{1.0, 0.0, 3.0, 0.0, 0.05};
    hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&s->ev0);
    if (e == hipSuccess) e = hipEventCreate(&s->ev1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s->split.fork, hipEventDisableTiming);
    for (int q = 0; q < SQP_MAX_PARTS - 1; ++q) {
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->split.aux[q], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s->split.join[q], hipEventDisableTiming);
    }
    const size_t B = o->batch, N = o->N;
    auto al = [&](DevBuf& b, size_t bytes) { if (e == hipSuccess) e = b.ensure(bytes); };
    al(s->shape_id, B * 4);
    al(s->x0, B * 4 * 8);
    al(s->yref, B * N * 6 * 8);
    al(s->yref_e, B * 4 * 8);
    al(s->X, B * (N + 1) * 4 * 8);
    al(s->U, B * N * 2 * 8);
    al(s->PI, B * N * 4 * 8);
    al(s->Xo, B * (N + 1) * 4 * 8);
    al(s->Uo, B * N * 2 * 8);
    al(s->PIo, B * N * 4 * 8);
    al(s->u0, B * 2 * 8);
    al(s->status, B * 4);
    al(s->sqp_iter, B * 4);
    al(s->qp_iter, B * 4);
    al(s->qp_capped, B * 4);
    al(s->qp_stalled, B * 4);
    al(s->cost, B * 8);
    al(s->warm_valid, B);
    al(s->wX, B * (N + 1) * 4 * 8);
    al(s->wU, B * N * 2 * 8);
    al(s->wx0, B * 4 * 8);
    al(s->wperm, B * 4);
    al(s->wnit, B * 4);
    al(s->whist, SQP_MAX_PARTS * 4 * 1024 * 4);   // per part of the SQP loop; qsp_solver.hip PACK_KEYS_MAX
    al(s->wdone, B * 4);
    if (o->nlp_mode == QSP_NLP_SQP_MERIT) {
        // stage data in HBM only for the line search (defect and gradient at the iterate); the
        // fixed-K path linearises inside the QP kernel, and qsp_qp_solve stages its own
        al(s->wlin, B * (N + 1) * 24 * 8);
        al(s->wnlp, B * (N + 1) * 20 * 8);
        al(s->wqp, B * (N + 1) * 16 * 8);
        al(s->wres, B * 4 * 8);
    }
    if (e == hipSuccess) e = hipMemsetAsync(s->shape_id.p, 0, B * 4, s->stream);
    if (e == hipSuccess) e = hipMemsetAsync(s->warm_valid.p, 0, B, s->stream);
    if (e == hipSuccess) e = hipMemsetAsync(s->X.p, 0, B * (N + 1) * 4 * 8, s->stream);
    if (e == hipSuccess) e = hipMemsetAsync(s->U.p, 0, B * N * 2 * 8, s->stream);
    if (e == hipSuccess) e = hipMemsetAsync(s->PI.p, 0, B * N * 4 * 8, s->stream);
    // debug: every workspace byte starts as a NaN pattern, so a kernel that reads a word it
    // never wrote shows up as NaN (tests/test_gpu_errors.py)
    if (const char* fl = std::getenv("QSP_FUSED_LOOP")) s->fused_req = (fl[0] == '1') ? 1 : (fl[0] == '0' ? 0 : -1);
    if (const char* pk = std::getenv("QSP_PACKING")) s->nopack = pk[0] == '0';
    if (const char* mw = std::getenv("QSP_MFMA_WALK")) s->mfw = mw[0] != '0';
    s->p.mfma_walk = s->mfw ? 1 : 0;
    mfw_prepare(s->p);
    const char* pz = std::getenv("QSP_DEBUG_POISON");
    s->poison = pz && pz[0] == '1';
    if (s->poison) {
        DevBuf* ws[] = {&s->wX, &s->wU, &s->wx0, &s->wlin, &s->wnlp, &s->wdone, &s->wres, &s->wqp, &s->wperm, &s->wnit,
                        &s->X, &s->U, &s->PI, &s->Xo, &s->Uo, &s->PIo, &s->u0, &s->cost, &s->yref, &s->yref_e};
        for (DevBuf* b : ws)
            if (e == hipSuccess && b->p) e = hipMemsetAsync(b->p, 0xff, b->n, s->stream);
        // ... except what a caller legitimately relies on being zero: the initial guess and warm state
        if (e == hipSuccess) e = hipMemsetAsync(s->X.p, 0, B * (N + 1) * 4 * 8, s->stream);
        if (e == hipSuccess) e = hipMemsetAsync(s->U.p, 0, B * N * 2 * 8, s->stream);
        if (e == hipSuccess) e = hipMemsetAsync(s->PI.p, 0, B * N * 4 * 8, s->stream);
    }
    // qsp_get_residuals before the first solve returns zeros (header contract)
    if (e == hipSuccess && s->wres.p) e = hipMemsetAsync(s->wres.p, 0, B * 4 * 8, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) {
        std::string m = std::string("qsp_create: ") + hipGetErrorString(e);
        qsp_destroy(s);
        return fail(QSP_ERR_HIP, m);
    }
    *out = s;
    return QSP_OK;
}

int qsp_destroy(qsp_solver* s) {
    if (!s) return QSP_OK;
    (void)hipSetDevice(s->o.device);
    DevBuf* bufs[] = {&s->ubc, &s->ubp, &s->cl_x, &s->cl_xsim, &s->cl_amp,
                      &s->shapes, &s->shape_id, &s->x0, &s->yref, &s->yref_e, &s->X, &s->U, &s->PI, &s->Xo,
                      &s->Uo, &s->PIo, &s->u0, &s->status, &s->sqp_iter, &s->qp_iter, &s->qp_capped, &s->qp_stalled, &s->cost,
                      &s->warm_valid,
                      &s->traj, &s->index_time, &s->wX, &s->wU, &s->wx0, &s->wlin, &s->wnlp, &s->wdone, &s->wres, &s->wqp, &s->wperm, &s->wnit,
                      &s->whist};
    for (DevBuf* b : bufs) b->release();
    for (auto& b : s->scratch) b.release();
    for (hipEvent_t e : s->kev) (void)hipEventDestroy(e);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->split.fork) (void)hipEventDestroy(s->split.fork);
    for (int q = 0; q < SQP_MAX_PARTS - 1; ++q) {
        if (s->split.join[q]) (void)hipEventDestroy(s->split.join[q]);
        if (s->split.aux[q]) (void)hipStreamDestroy(s->split.aux[q]);
    }
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return QSP_OK;
}

int qsp_get_layout(const qsp_solver* s, int32_t* S, int32_t* L) {
    if (!s) return fail(QSP_ERR_ARG, "qsp_get_layout: null handle");
    if (S) *S = s->S;
    if (L) *L = lanes_per_instance(s->o.N, s->S);
    return QSP_OK;
}

int qsp_get_factor_walk(const qsp_solver* s, int32_t* walk) {
    if (!s || !walk) return fail(QSP_ERR_ARG, "qsp_get_factor_walk: null argument");
    *walk = factor_walk_kind(s->p, s->S);
    return QSP_OK;
}

// ------------------------------------------------------------------ shapes
int qsp_shape_from_ply(const char* path, int32_t flip, double mu_sg, double mu_sp, double mass, double tau_max,
                       qsp_shape* out) {
    if (!path || !out) return fail(QSP_ERR_ARG, "qsp_shape_from_ply: null argument");
    std::vector<float> P;
    int r = read_ply_xy(path, P);
    if (r != QSP_OK) return r;
    const int n0 = (int)(P.size() / 2);
    if (n0 + 1 > QSP_MAX_CTRL) return fail(QSP_ERR_ARG, "qsp_shape_from_ply: too many points");
    // sortCadPoints (PusherSliderModel.m:84-111): start at the first min-x point, then
    // greedy nearest neighbour in float32 with first-index ties; consumed points -> Inf.
    std::vector<float> xs(P);
    const float inf = INFINITY;
    int ind = 0;
    for (int i = 1; i < n0; ++i) if (xs[2 * i] < xs[2 * ind]) ind = i;
    float tx = xs[2 * ind], ty = xs[2 * ind + 1];
    xs[2 * ind] = xs[2 * ind + 1] = inf;
    std::vector<double> srt((size_t)(n0 + 1) * 2);
    srt[0] = tx; srt[1] = ty;
    for (int i = 1; i < n0; ++i) {
        int best = -1;
        float bd = 0.0f;
        for (int q = 0; q < n0; ++q) {
            const float dx = xs[2 * q] - tx, dy = xs[2 * q + 1] - ty;
            const float d = std::sqrt(dx * dx + dy * dy);
            if (best < 0 || d < bd) { best = q; bd = d; }
        }
        tx = xs[2 * best]; ty = xs[2 * best + 1];
        srt[2 * i] = tx; srt[2 * i + 1] = ty;
        xs[2 * best] = xs[2 * best + 1] = inf;
    }
    const double sc = 1.0 / 1000.0;   // scale_factor (PusherSliderModel.m:72,105)
    for (int i = 0; i < n0; ++i) { srt[2 * i] *= sc; srt[2 * i + 1] *= sc; }
    srt[2 * n0] = srt[0]; srt[2 * n0 + 1] = srt[1];   // close the loop (:106)
    const int n = n0 + 1;
    if (flip) {   // flipud for montana / pulirapid (:107-109)
        for (int i = 0; i < n / 2; ++i)
            for (int c = 0; c < 2; ++c) std::swap(srt[2 * i + c], srt[2 * (n - 1 - i) + c]);
    }
    std::memset(out, 0, sizeof(*out));
    out->n_ctrl = n;
    out->struct_size = (int32_t)sizeof(qsp_shape);
    for (int i = 0; i < n; ++i) { out->ctrl[i][0] = srt[2 * i]; out->ctrl[i][1] = srt[2 * i + 1]; }
    // knots (getSpline :117-123): p = 3, m = n - 2, S = [0 0 0 linspace(0,b,m) b b b]
    double b = 0.0;
    for (int i = 0; i + 1 < n; ++i) {
        const double dx = out->ctrl[i + 1][0] - out->ctrl[i][0], dy = out->ctrl[i + 1][1] - out->ctrl[i][1];
        b += std::sqrt(dx * dx + dy * dy);
    }
    const int m = n - 2;
    for (int i = 0; i < 3; ++i) out->knots[i] = 0.0;
    const double step = b / (double)(m - 1);
    for (int i = 0; i < m; ++i) out->knots[3 + i] = (i == m - 1) ? b : (double)i * step;
    for (int i = 0; i < 3; ++i) out->knots[3 + m + i] = b;
    out->b = b;
    out->c_ellipse = tau_max / (mu_sg * mass * 9.81);   // :53,55 with helper.g = 9.81
    out->mu_sp = mu_sp;
    return QSP_OK;
}

int qsp_set_shapes(qsp_solver* s, const qsp_shape* shapes, int32_t n) {
    if (!s || !shapes || n < 1) return fail(QSP_ERR_ARG, "qsp_set_shapes: bad argument");
    std::vector<ShapeDev> h((size_t)n);
    for (int q = 0; q < n; ++q) {
        const qsp_shape& in = shapes[q];
        if (in.struct_size != (int32_t)sizeof(qsp_shape))
            return fail(QSP_ERR_ARG, "qsp_set_shapes: qsp_shape.struct_size != sizeof(qsp_shape) (stale layout?)");
        ShapeDev& d = h[q];
        std::memset(&d, 0, sizeof d);
        const int nc = in.n_ctrl;
        if (nc < 5 || nc > QSP_MAX_CTRL) return fail(QSP_ERR_ARG, "qsp_set_shapes: n_ctrl out of range");
        d.n = nc;
        d.b = in.b;
        d.c = in.c_ellipse;
        d.mu = in.mu_sp;
        for (int i = 0; i < nc + 4; ++i) d.knots[i] = in.knots[i];
        for (int i = 0; i < nc; ++i) { d.ctrl[2 * i] = in.ctrl[i][0]; d.ctrl[2 * i + 1] = in.ctrl[i][1]; }
        const double h0 = in.knots[4] - in.knots[3];
        d.inv_h = h0 > 0.0 ? 1.0 / h0 : 0.0;
        d.xwidth = in.xwidth;
        // derivative-spline coefficients (bspline_shape.m:92-99 with zero-denominator guard :93)
        for (int i = 1; i < nc; ++i) {
            const double den = d.knots[i + 3] - d.knots[i];
            for (int c = 0; c < 2; ++c)
                d.dctrl[2 * i + c] = den != 0.0 ? 3.0 * ((d.ctrl[2 * i + c] - d.ctrl[2 * (i - 1) + c]) / den) : 0.0;
        }
        for (int i = 2; i < nc; ++i) {
            const double den = d.knots[i + 2] - d.knots[i];
            for (int c = 0; c < 2; ++c)
                d.ddctrl[2 * i + c] = den != 0.0 ? 2.0 * ((d.dctrl[2 * i + c] - d.dctrl[2 * (i - 1) + c]) / den) : 0.0;
        }
    }
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(s->shapes.ensure(sizeof(ShapeDev) * n));
    HIPCHK(hipMemcpyAsync(s->shapes.p, h.data(), sizeof(ShapeDev) * n, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    s->n_shapes = n;
    return QSP_OK;
}

int qsp_set_shape_ids(qsp_solver* s, const int32_t* ids) {
    if (!s || !ids) return fail(QSP_ERR_ARG, "qsp_set_shape_ids: null argument");
    for (int i = 0; i < s->o.batch; ++i)
        if (ids[i] < 0 || ids[i] >= s->n_shapes) return fail(QSP_ERR_ARG, "qsp_set_shape_ids: id out of range");
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(hipMemcpy(s->shape_id.p, ids, (size_t)s->o.batch * 4, hipMemcpyHostToDevice));
    return QSP_OK;
}

int qsp_set_cost_W(qsp_solver* s, const double W[6], const double We[4]) {
    if (!s || !W || !We) return fail(QSP_ERR_ARG, "qsp_set_cost_W: null argument");
    for (int i = 0; i < 6; ++i) if (!(W[i] >= 0.0)) return fail(QSP_ERR_ARG, "qsp_set_cost_W: W must be >= 0");
    for (int i = 0; i < 4; ++i) if (!(We[i] >= 0.0)) return fail(QSP_ERR_ARG, "qsp_set_cost_W: W_e must be >= 0");
    if (!(W[4] > 0.0 && W[5] > 0.0)) return fail(QSP_ERR_ARG, "qsp_set_cost_W: control weights must be > 0");
    std::memcpy(s->p.W, W, sizeof(double) * 6);
    std::memcpy(s->p.We, We, sizeof(double) * 4);
    return QSP_OK;
}

int qsp_set_constr_h(qsp_solver* s, const double lh[3], const double uh[3]) {
    if (!s || !lh || !uh) return fail(QSP_ERR_ARG, "qsp_set_constr_h: null argument");
    for (int i = 0; i < 3; ++i) if (!(lh[i] < uh[i])) return fail(QSP_ERR_ARG, "qsp_set_constr_h: need lh < uh");
    std::memcpy(s->p.lh, lh, sizeof(double) * 3);
    std::memcpy(s->p.uh, uh, sizeof(double) * 3);
    return QSP_OK;
}

int qsp_set_ctrl_params(qsp_solver* s, double v_alpha, double d_v, double t_angle0, double u_n_lb, double u_t_ub) {
    if (!s) return fail(QSP_ERR_ARG, "qsp_set_ctrl_params: null handle");
    s->p.cp = CtrlParams{v_alpha, d_v, t_angle0, u_n_lb, u_t_ub};
    return QSP_OK;
}

// --------------------------------------------------------- acados level
int qsp_set_x0(qsp_solver* s, const double* x0) {
    if (!s || !x0) return fail(QSP_ERR_ARG, "qsp_set_x0: null argument");
    return h2d(s, s->x0, x0, (size_t)s->o.batch * 4 * 8);
}

int qsp_set_yref(qsp_solver* s, const double* yref, const double* yref_e) {
    if (!s || !yref || !yref_e) return fail(QSP_ERR_ARG, "qsp_set_yref: null argument");
    int r = h2d(s, s->yref, yref, (size_t)s->o.batch * s->o.N * 6 * 8);
    if (r) return r;
    return h2d(s, s->yref_e, yref_e, (size_t)s->o.batch * 4 * 8);
}

int qsp_set_init(qsp_solver* s, const double* X, const double* U, const double* PI) {
    if (!s || !X || !U) return fail(QSP_ERR_ARG, "qsp_set_init: null argument");
    const size_t B = s->o.batch, N = s->o.N;
    int r = h2d(s, s->X, X, B * (N + 1) * 4 * 8);
    if (!r) r = h2d(s, s->U, U, B * N * 2 * 8);
    if (!r && PI) r = h2d(s, s->PI, PI, B * N * 4 * 8);
    return r;
}

int qsp_solve(qsp_solver* s) {
    if (!s) return fail(QSP_ERR_ARG, "qsp_solve: null handle");
    if (s->n_shapes < 1) return fail(QSP_ERR_STATE, "qsp_solve: no shapes set");
    HIPCHK(hipSetDevice(s->o.device));
    SolveArgs a = make_args(s);
    return run_timed(s, a);
}

int qsp_get_u0(qsp_solver* s, double* u0) {
    if (!s || !u0) return fail(QSP_ERR_ARG, "qsp_get_u0: null argument");
    return d2h(s, u0, s->u0, (size_t)s->o.batch * 2 * 8);
}
int qsp_get_x(qsp_solver* s, double* X) {
    if (!s || !X) return fail(QSP_ERR_ARG, "qsp_get_x: null argument");
    return d2h(s, X, s->last_controller ? s->X : s->Xo, (size_t)s->o.batch * (s->o.N + 1) * 4 * 8);
}
int qsp_get_u(qsp_solver* s, double* U) {
    if (!s || !U) return fail(QSP_ERR_ARG, "qsp_get_u: null argument");
    return d2h(s, U, s->last_controller ? s->U : s->Uo, (size_t)s->o.batch * s->o.N * 2 * 8);
}
int qsp_get_pi(qsp_solver* s, double* PI) {
    if (!s || !PI) return fail(QSP_ERR_ARG, "qsp_get_pi: null argument");
    return d2h(s, PI, s->last_controller ? s->PI : s->PIo, (size_t)s->o.batch * s->o.N * 4 * 8);
}
int qsp_get_cost(qsp_solver* s, double* c) {
    if (!s || !c) return fail(QSP_ERR_ARG, "qsp_get_cost: null argument");
    return d2h(s, c, s->cost, (size_t)s->o.batch * 8);
}
int qsp_get_status(qsp_solver* s, int32_t* st) {
    if (!s || !st) return fail(QSP_ERR_ARG, "qsp_get_status: null argument");
    return d2h(s, st, s->status, (size_t)s->o.batch * 4);
}
int qsp_get_sqp_iter(qsp_solver* s, int32_t* it) {
    if (!s || !it) return fail(QSP_ERR_ARG, "qsp_get_sqp_iter: null argument");
    return d2h(s, it, s->sqp_iter, (size_t)s->o.batch * 4);
}
int qsp_get_qp_iter(qsp_solver* s, int32_t* it) {
    if (!s || !it) return fail(QSP_ERR_ARG, "qsp_get_qp_iter: null argument");
    return d2h(s, it, s->qp_iter, (size_t)s->o.batch * 4);
}
int qsp_get_qp_capped(qsp_solver* s, int32_t* c) {
    if (!s || !c) return fail(QSP_ERR_ARG, "qsp_get_qp_capped: null argument");
    return d2h(s, c, s->qp_capped, (size_t)s->o.batch * 4);
}

int qsp_get_qp_stalled(qsp_solver* s, int32_t* c) {
    if (!s || !c) return fail(QSP_ERR_ARG, "qsp_get_qp_stalled: null argument");
    return d2h(s, c, s->qp_stalled, (size_t)s->o.batch * 4);
}
int qsp_get_residuals(qsp_solver* s, double* res) {
    if (!s || !res) return fail(QSP_ERR_ARG, "qsp_get_residuals: null argument");
    if (s->o.nlp_mode != QSP_NLP_SQP_MERIT || !s->wres.p) return fail(QSP_ERR_STATE, "qsp_get_residuals: nlp_mode 1 (SQP) only");
    return d2h(s, res, s->wres, (size_t)s->o.batch * 4 * 8);
}
int qsp_get_time_tot(qsp_solver* s, double* ms) {
    if (!s || !ms) return fail(QSP_ERR_ARG, "qsp_get_time_tot: null argument");
    *ms = (double)s->last_ms;
    return QSP_OK;
}

int qsp_get_dims(const qsp_solver* s, int32_t* N, int32_t* B) {
    if (!s) return fail(QSP_ERR_ARG, "qsp_get_dims: null handle");
    if (N) *N = s->o.N;
    if (B) *B = s->o.batch;
    return QSP_OK;
}

int qsp_set_yref_stage(qsp_solver* s, int32_t k, const double* y) {
    if (!s || !y) return fail(QSP_ERR_ARG, "qsp_set_yref_stage: null argument");
    if (k < 0 || k >= s->o.N) return fail(QSP_ERR_ARG, "qsp_set_yref_stage: stage out of range 0..N-1");
    HIPCHK(hipSetDevice(s->o.device));
    // column k of every lane's N x 6 block: a strided copy (B rows of 6 doubles)
    HIPCHK(hipMemcpy2DAsync(s->yref.as<double>() + (size_t)k * 6, (size_t)s->o.N * 6 * 8, y, 6 * 8, 6 * 8,
                            (size_t)s->o.batch, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

int qsp_set_yref_e(qsp_solver* s, const double* y_e) {
    if (!s || !y_e) return fail(QSP_ERR_ARG, "qsp_set_yref_e: null argument");
    return h2d(s, s->yref_e, y_e, (size_t)s->o.batch * 4 * 8);
}

int qsp_set_init_x(qsp_solver* s, const double* X) {
    if (!s || !X) return fail(QSP_ERR_ARG, "qsp_set_init_x: null argument");
    return h2d(s, s->X, X, (size_t)s->o.batch * (s->o.N + 1) * 4 * 8);
}
int qsp_set_init_u(qsp_solver* s, const double* U) {
    if (!s || !U) return fail(QSP_ERR_ARG, "qsp_set_init_u: null argument");
    return h2d(s, s->U, U, (size_t)s->o.batch * s->o.N * 2 * 8);
}
int qsp_set_init_pi(qsp_solver* s, const double* PI) {
    if (!s || !PI) return fail(QSP_ERR_ARG, "qsp_set_init_pi: null argument");
    return h2d(s, s->PI, PI, (size_t)s->o.batch * s->o.N * 4 * 8);
}

int qsp_set_timing(qsp_solver* s, int32_t on) {
    if (!s) return fail(QSP_ERR_ARG, "qsp_set_timing: null handle");
    int r = qsp_set_kernel_timing(s, on ? 1 : 0);
    if (r) return r;
    s->auto_timing = on != 0;
    return QSP_OK;
}

int qsp_get_timings(qsp_solver* s, double* time_tot, double* time_lin, double* time_qp_sol) {
    if (!s) return fail(QSP_ERR_ARG, "qsp_get_timings: null handle");
    if (time_tot) *time_tot = s->last_ms * 1e-3;
    double lin = NAN, qp = NAN;
    if (s->auto_timing && !s->kev_solves.empty()) {
        double ms[4];
        int32_t n[4];
        HIPCHK(hipSetDevice(s->o.device));
        const int r = kernel_times_of(s, ms, n);   // the last solve's events stay readable
        if (r) return r;
        lin = ms[1] * 1e-3;
        qp = ms[2] * 1e-3;
    }
    if (time_lin) *time_lin = lin;
    if (time_qp_sol) *time_qp_sol = qp;
    return QSP_OK;
}

// ------------------------------------------------------ controller level
int qsp_set_reference_trajectory(qsp_solver* s, const double* traj, int32_t T) {
    if (!s || !traj || T < 1) return fail(QSP_ERR_ARG, "qsp_set_reference_trajectory: bad argument");
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(s->traj.ensure((size_t)T * 6 * 8));
    HIPCHK(hipMemcpyAsync(s->traj.p, traj, (size_t)T * 6 * 8, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    s->T = T;
    s->have_traj = true;
    s->traj_per_lane = false;
    return QSP_OK;
}

int qsp_set_reference_trajectories(qsp_solver* s, const double* traj, int32_t T) {
    if (!s || !traj || T < 1) return fail(QSP_ERR_ARG, "qsp_set_reference_trajectories: bad argument");
    const size_t bytes = (size_t)s->o.batch * T * 6 * 8;
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(s->traj.ensure(bytes));
    HIPCHK(hipMemcpyAsync(s->traj.p, traj, bytes, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    s->T = T;
    s->have_traj = true;
    s->traj_per_lane = true;
    return QSP_OK;
}

int qsp_gen_straight_lines(qsp_solver* s, const double* x0, const double* xf, double t0, double tf,
                           int32_t auto_angle, int32_t* T_out) {
    if (!s || !x0 || !xf || !(tf > t0) || t0 < 0.0) return fail(QSP_ERR_ARG, "qsp_gen_straight_lines: bad argument");
    const size_t B = s->o.batch;
    // MATLAB t0:Ts:tf
    const int32_t T = (int32_t)std::floor((tf - t0) / s->o.Ts + 1e-9) + 1;
    HIPCHK(hipSetDevice(s->o.device));
    DevBuf& d0 = s->scratch[0];
    DevBuf& d1 = s->scratch[1];
    HIPCHK(d0.ensure(B * 3 * 8));
    HIPCHK(d1.ensure(B * 3 * 8));
    HIPCHK(hipMemcpyAsync(d0.p, x0, B * 3 * 8, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipMemcpyAsync(d1.p, xf, B * 3 * 8, hipMemcpyHostToDevice, s->stream));
    HIPCHK(s->traj.ensure(B * (size_t)T * 6 * 8));
    HIPCHK(launch_straight_lines((int)B, T, d0.as<double>(), d1.as<double>(), t0, tf, s->o.Ts, auto_angle,
                                 s->traj.as<double>(), s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    s->T = T;
    s->have_traj = true;
    s->traj_per_lane = true;
    if (T_out) *T_out = T;
    return QSP_OK;
}

int qsp_get_reference_trajectories(qsp_solver* s, double* traj) {
    if (!s || !traj) return fail(QSP_ERR_ARG, "qsp_get_reference_trajectories: null argument");
    if (!s->have_traj) return fail(QSP_ERR_STATE, "qsp_get_reference_trajectories: no reference trajectory");
    const size_t n = (s->traj_per_lane ? (size_t)s->o.batch : 1) * s->T * 6 * 8;
    return d2h(s, traj, s->traj, n);
}

int qsp_controller_reset(qsp_solver* s) {
    if (!s) return fail(QSP_ERR_ARG, "qsp_controller_reset: null handle");
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(hipMemsetAsync(s->warm_valid.p, 0, (size_t)s->o.batch, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

int qsp_controller_solve(qsp_solver* s, const double* x0, const int32_t* index_time) {
    if (!s || !x0 || !index_time) return fail(QSP_ERR_ARG, "qsp_controller_solve: null argument");
    if (!s->have_traj) return fail(QSP_ERR_STATE, "qsp_controller_solve: no reference trajectory");
    if (s->n_shapes < 1) return fail(QSP_ERR_STATE, "qsp_controller_solve: no shapes set");
    const size_t B = s->o.batch;
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(s->index_time.ensure(B * 4));
    HIPCHK(hipMemcpyAsync(s->x0.p, x0, B * 4 * 8, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipMemcpyAsync(s->index_time.p, index_time, B * 4, hipMemcpyHostToDevice, s->stream));
    HIPCHK(launch_controller_step(s, 0));
    return run_timed(s, controller_args(s));
}

// ------------------------------------------------------- delay compensation
int qsp_set_delay_comp(qsp_solver* s, double delay) {
    if (!s || !(delay >= 0.0)) return fail(QSP_ERR_ARG, "qsp_set_delay_comp: delay must be >= 0");
    const double cols = std::ceil(delay / s->o.Ts);   // delay_buff_comp = ceil(delay / sample_time) (:108)
    if (cols > 4096.0) return fail(QSP_ERR_ARG, "qsp_set_delay_comp: more than 4096 delay samples");
    HIPCHK(hipSetDevice(s->o.device));
    s->D = (int32_t)cols;
    const size_t bytes = (size_t)s->o.batch * (size_t)(s->D > 0 ? s->D : 1) * 2 * 8;
    HIPCHK(s->ubc.ensure(bytes));
    HIPCHK(hipMemsetAsync(s->ubc.p, 0, bytes, s->stream));   // u_buff_contr = zeros (:109)
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

int qsp_get_delay_comp(qsp_solver* s, int32_t* cols) {
    if (!s || !cols) return fail(QSP_ERR_ARG, "qsp_get_delay_comp: null argument");
    *cols = s->D;
    return QSP_OK;
}

static ClosedLoopArgs cl_args(qsp_solver* s) {
    ClosedLoopArgs a;
    std::memset(&a, 0, sizeof a);
    a.shapes = s->shapes.as<ShapeDev>();
    a.n_shapes = s->n_shapes;
    a.sid = s->shape_id.as<int32_t>();
    a.B = s->o.batch;
    a.Ts = s->o.Ts;
    a.D = s->D;
    a.ubc = s->ubc.as<double>();
    return a;
}

int qsp_delay_buffer_sim(qsp_solver* s, const double* x, double* x_sim) {
    if (!s || !x || !x_sim) return fail(QSP_ERR_ARG, "qsp_delay_buffer_sim: null argument");
    if (s->n_shapes < 1) return fail(QSP_ERR_STATE, "qsp_delay_buffer_sim: no shapes set");
    const size_t B = s->o.batch;
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(s->cl_x.ensure(B * 4 * 8));
    HIPCHK(s->cl_xsim.ensure(B * 4 * 8));
    HIPCHK(hipMemcpyAsync(s->cl_x.p, x, B * 4 * 8, hipMemcpyHostToDevice, s->stream));
    ClosedLoopArgs a = cl_args(s);
    a.x = s->cl_x.as<double>();
    a.xs = s->cl_xsim.as<double>();
    HIPCHK(launch_delay_sim(a, s->stream));
    HIPCHK(hipMemcpyAsync(x_sim, s->cl_xsim.p, B * 4 * 8, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

int qsp_delay_buffer_push(qsp_solver* s, const double* u) {
    if (!s || !u) return fail(QSP_ERR_ARG, "qsp_delay_buffer_push: null argument");
    if (s->D == 0) return QSP_OK;
    const size_t B = s->o.batch, D = (size_t)s->D;
    std::vector<double> h(B * D * 2);
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(hipMemcpyAsync(h.data(), s->ubc.p, h.size() * 8, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    for (size_t i = 0; i < B; ++i) {   // u_buff_contr = [u, u_buff_contr(:, 1:end-1)]  (helper.m:255)
        double* b = h.data() + i * D * 2;
        std::memmove(b + 2, b, (D - 1) * 2 * 8);
        b[0] = u[2 * i];
        b[1] = u[2 * i + 1];
    }
    HIPCHK(hipMemcpyAsync(s->ubc.p, h.data(), h.size() * 8, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

int qsp_closed_loop_ex(qsp_solver* s, const qsp_closed_loop_opts* o, const double* x0, const int32_t* index0,
                       int32_t n_steps, const double* noise, double* X_traj, double* X_sim, double* U_traj,
                       int32_t* status_traj) {
    if (!s || !x0 || !index0 || !X_traj || !U_traj || n_steps < 1)
        return fail(QSP_ERR_ARG, "qsp_closed_loop: bad argument");
    if (!s->have_traj) return fail(QSP_ERR_STATE, "qsp_closed_loop: no reference trajectory");
    if (s->n_shapes < 1) return fail(QSP_ERR_STATE, "qsp_closed_loop: no shapes set");
    const double plant_delay = o ? o->plant_delay : 0.0;
    if (!(plant_delay >= 0.0) || std::ceil(plant_delay / s->o.Ts) > 4096.0)
        return fail(QSP_ERR_ARG, "qsp_closed_loop: plant_delay must be in [0, 4096 Ts]");
    if (o && o->disturbance && o->t_dist < 1) return fail(QSP_ERR_ARG, "qsp_closed_loop: t_dist must be >= 1");
    const size_t B = s->o.batch, T = (size_t)n_steps;
    const int Dp = (int)std::ceil(plant_delay / s->o.Ts);   // delay_buff_plant (helper.m:211)
    HIPCHK(hipSetDevice(s->o.device));
    DevBuf& dX = s->scratch[9];
    DevBuf& dU = s->scratch[10];
    DevBuf& dS = s->scratch[11];
    DevBuf& dN = s->scratch[3];
    DevBuf& dXs = s->scratch[4];
    HIPCHK(dX.ensure(B * (T + 1) * 4 * 8));
    HIPCHK(dU.ensure(B * T * 2 * 8));
    HIPCHK(dS.ensure(B * T * 4));
    if (X_sim) HIPCHK(dXs.ensure(B * T * 4 * 8));
    if (noise) HIPCHK(dN.ensure(T * B * 4 * 8));
    HIPCHK(s->cl_x.ensure(B * 4 * 8));
    HIPCHK(s->ubp.ensure(B * (size_t)(Dp > 0 ? Dp : 1) * 2 * 8));
    if (s->D > 0) HIPCHK(s->ubc.ensure(B * (size_t)s->D * 2 * 8));
    HIPCHK(s->index_time.ensure(B * 4));
    HIPCHK(hipMemcpyAsync(s->cl_x.p, x0, B * 4 * 8, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipMemcpyAsync(s->index_time.p, index0, B * 4, hipMemcpyHostToDevice, s->stream));
    if (noise) HIPCHK(hipMemcpyAsync(dN.p, noise, T * B * 4 * 8, hipMemcpyHostToDevice, s->stream));
    const bool dist = o && o->disturbance;
    if (dist && o->amplitude) {
        HIPCHK(s->cl_amp.ensure(B * 8));
        HIPCHK(hipMemcpyAsync(s->cl_amp.p, o->amplitude, B * 8, hipMemcpyHostToDevice, s->stream));
    }
    // initial_condition_update -> clear_variables: the first solve is a cold start (main.m:79);
    // the plant's buffer starts at zero (closed_loop_matlab's u_buff_plant, helper.m:211-212); the
    // controller's u_buff_contr is left as it is: the reference zeroes it only in set_delay_comp
    // (NMPC_controller.m:106-110; qsp_set_delay_comp), so a second run continues from the first's
    HIPCHK(hipMemsetAsync(s->warm_valid.p, 0, B, s->stream));
    if (Dp > 0) HIPCHK(hipMemsetAsync(s->ubp.p, 0, B * (size_t)Dp * 2 * 8, s->stream));
    ClosedLoopArgs c = cl_args(s);
    c.n_steps = n_steps;
    c.x = s->cl_x.as<double>();
    c.xs = s->x0.as<double>();                 // the solver's x0 (constr_x0)
    c.noise = noise ? dN.as<double>() : nullptr;
    c.dist_step = dist ? o->t_dist : 0;
    c.dist_amp = (dist && o->amplitude) ? s->cl_amp.as<double>() : nullptr;
    c.Dp = Dp;
    c.ubp = s->ubp.as<double>();
    c.u0 = s->u0.as<double>();
    c.status = s->status.as<int32_t>();
    c.Xtraj = dX.as<double>();
    c.Xsim = X_sim ? dXs.as<double>() : nullptr;
    c.Utraj = dU.as<double>();
    c.Straj = dS.as<int32_t>();
    HIPCHK(hipEventRecord(s->ev0, s->stream));
    const SolveArgs a = controller_args(s);
    for (int32_t t = 0; t < n_steps; ++t) {
        HIPCHK(launch_closed_loop_pre(c, t, s->stream));                       // disturbance, noise, delay_buffer_sim
        HIPCHK(launch_controller_step(s, t + s->D));                           // y_ref for index0 + t + D
        HIPCHK(launch_sqp(a, s->S, s->stream, take_kernel_events(s), sqp_split(s)));   // NMPC_controller.solve
        HIPCHK(launch_plant(c, t, s->stream));                                 // buffers, plant step, logs
    }
    HIPCHK(hipEventRecord(s->ev1, s->stream));
    HIPCHK(hipMemcpyAsync(X_traj, dX.p, B * (T + 1) * 4 * 8, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipMemcpyAsync(U_traj, dU.p, B * T * 2 * 8, hipMemcpyDeviceToHost, s->stream));
    if (X_sim) HIPCHK(hipMemcpyAsync(X_sim, dXs.p, B * T * 4 * 8, hipMemcpyDeviceToHost, s->stream));
    if (status_traj) HIPCHK(hipMemcpyAsync(status_traj, dS.p, B * T * 4, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    HIPCHK(hipEventElapsedTime(&s->last_ms, s->ev0, s->ev1));
    return QSP_OK;
}

int qsp_closed_loop(qsp_solver* s, const double* x0, const int32_t* index0, int32_t n_steps, const double* noise,
                    double* X_traj, double* U_traj, int32_t* status_traj) {
    return qsp_closed_loop_ex(s, nullptr, x0, index0, n_steps, noise, X_traj, nullptr, U_traj, status_traj);
}

int qsp_reproject_contact(qsp_solver* s, int32_t n, const int32_t* sid, const double* px, const double* py,
                          const double* s0, double* s_out) {
    if (!s || n < 1 || !sid || !px || !py || !s0 || !s_out) return fail(QSP_ERR_ARG, "qsp_reproject_contact: bad argument");
    int r = check_ids(s, n, sid);
    if (r) return r;
    HIPCHK(hipSetDevice(s->o.device));
    auto& sc = s->scratch;
    if ((r = stage_in(s, sc[0], sid, n)) || (r = stage_in(s, sc[1], px, n)) || (r = stage_in(s, sc[2], py, n)) ||
        (r = stage_in(s, sc[5], s0, n)))
        return r;
    HIPCHK(sc[6].ensure((size_t)n * 8));
    HIPCHK(launch_reproject(s->shapes.as<ShapeDev>(), s->n_shapes, sc[0].as<int32_t>(), n, sc[1].as<double>(),
                            sc[2].as<double>(), sc[5].as<double>(), sc[6].as<double>(), s->stream));
    if ((r = stage_out(s, s_out, sc[6], (size_t)n))) return r;
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

// ------------------------------------------------------ device fast path
int qsp_solve_device(qsp_solver* s, const qsp_device_io* io, void* stream) {
    if (!s || !io) return fail(QSP_ERR_ARG, "qsp_solve_device: null argument");
    if (!io->x0 || !io->yref || !io->yref_e || !io->X_in || !io->U_in || !io->u0 || !io->X_out || !io->U_out ||
        !io->PI_out || !io->status || !io->cost)
        return fail(QSP_ERR_ARG, "qsp_solve_device: missing device pointer");
    if (s->n_shapes < 1) return fail(QSP_ERR_STATE, "qsp_solve_device: no shapes set");
    HIPCHK(hipSetDevice(s->o.device));
    SolveArgs a = make_args(s);
    a.x0 = io->x0;
    a.yref = io->yref;
    a.yref_e = io->yref_e;
    a.X_in = io->X_in;
    a.U_in = io->U_in;
    a.PI_in = io->PI_in;
    a.shape_id = io->shape_id ? io->shape_id : s->shape_id.as<int32_t>();
    a.u0 = io->u0;
    a.X_out = io->X_out;
    a.U_out = io->U_out;
    a.PI_out = io->PI_out;
    a.status = io->status;
    a.cost = io->cost;
    if (io->controller) {
        a.flags |= QSP_FLAG_CONTROLLER | QSP_FLAG_SHIFT;
        a.warm_valid = io->warm_valid;
    }
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    HIPCHK(launch_sqp(a, s->S, st, take_kernel_events(s), sqp_split(s)));
    return QSP_OK;
}

int qsp_set_stream_parts(qsp_solver* s, int32_t parts) {
    if (!s || parts < 0 || parts > SQP_MAX_PARTS)
        return fail(QSP_ERR_ARG, "qsp_set_stream_parts: parts must be 0 (auto), 1 or 2");
    s->parts_req = parts;
    return QSP_OK;
}

int qsp_get_stream_parts(qsp_solver* s, int32_t* parts) {
    if (!s || !parts) return fail(QSP_ERR_ARG, "qsp_get_stream_parts: null argument");
    *parts = sqp_split(s)->parts;
    return QSP_OK;
}

int qsp_set_kernel_timing(qsp_solver* s, int32_t max_solves) {
    if (!s || max_solves < 0) return fail(QSP_ERR_ARG, "qsp_set_kernel_timing: bad argument");
    HIPCHK(hipSetDevice(s->o.device));
    for (hipEvent_t e : s->kev) HIPCHK(hipEventDestroy(e));
    s->kev.clear();
    s->kev_solves.clear();
    s->kev_split.clear();
    s->kev_used = 0;
    const size_t n = (size_t)max_solves * (2 * s->o.sqp_iters + 3);
    for (size_t i = 0; i < n; ++i) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        s->kev.push_back(e);
    }
    return QSP_OK;
}

// summed kernel times of the recorded solves (events kept: the pool is re-armed by the caller)
static int kernel_times_of(qsp_solver* s, double* ms, int32_t* launches) {
    for (int k = 0; k < 4; ++k) { ms[k] = 0.0; launches[k] = 0; }
    const int K = s->o.sqp_iters;
    for (size_t j = 0; j < s->kev_solves.size(); ++j) {
        hipEvent_t* e = s->kev.data() + s->kev_solves[j];
        HIPCHK(hipEventSynchronize(e[2 * K + 2]));
        float t;
        HIPCHK(hipEventElapsedTime(&t, e[0], e[1])); ms[0] += t; launches[0] += 1;
        if (s->kev_split[j]) {
            // two-stream loop: timed as a whole, one "launch" per SQP iteration (sorts included)
            HIPCHK(hipEventElapsedTime(&t, e[1], e[2 * K + 1])); ms[2] += t; launches[2] += K;
        } else
        for (int it = 0; it < K; ++it) {
            HIPCHK(hipEventElapsedTime(&t, e[1 + 2 * it], e[2 + 2 * it])); ms[1] += t; launches[1] += 1;
            HIPCHK(hipEventElapsedTime(&t, e[2 + 2 * it], e[3 + 2 * it])); ms[2] += t; launches[2] += 1;
        }
        HIPCHK(hipEventElapsedTime(&t, e[2 * K + 1], e[2 * K + 2])); ms[3] += t; launches[3] += 1;
    }
    return QSP_OK;
}

int qsp_get_kernel_times(qsp_solver* s, double* ms, int32_t* launches) {
    if (!s || !ms || !launches) return fail(QSP_ERR_ARG, "qsp_get_kernel_times: null argument");
    HIPCHK(hipSetDevice(s->o.device));
    const int r = kernel_times_of(s, ms, launches);
    if (r) return r;
    s->kev_solves.clear();
    s->kev_split.clear();
    s->kev_used = 0;
    return QSP_OK;
}

int qsp_synchronize(qsp_solver* s) {
    if (!s) return fail(QSP_ERR_ARG, "qsp_synchronize: null handle");
    HIPCHK(hipSetDevice(s->o.device));
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

// ------------------------------------------------------- building blocks
int qsp_eval_spline(qsp_solver* s, int32_t n, const int32_t* sid, const double* sig, double* C, double* D, double* Dd,
                    double* kappa) {
    if (!s || !sid || !sig || !C || !D || !Dd || !kappa || n < 1) return fail(QSP_ERR_ARG, "qsp_eval_spline: bad argument");
    int r = check_ids(s, n, sid);
    if (r) return r;
    HIPCHK(hipSetDevice(s->o.device));
    auto& sc = s->scratch;
    if ((r = stage_in(s, sc[0], sid, n)) || (r = stage_in(s, sc[1], sig, n))) return r;
    HIPCHK(sc[2].ensure((size_t)n * 16)); HIPCHK(sc[3].ensure((size_t)n * 16));
    HIPCHK(sc[4].ensure((size_t)n * 16)); HIPCHK(sc[5].ensure((size_t)n * 8));
    HIPCHK(launch_spline(s->shapes.as<ShapeDev>(), sc[0].as<int32_t>(), n, sc[1].as<double>(), sc[2].as<double>(),
                         sc[3].as<double>(), sc[4].as<double>(), sc[5].as<double>(), s->stream));
    if ((r = stage_out(s, C, sc[2], (size_t)2 * n)) || (r = stage_out(s, D, sc[3], (size_t)2 * n)) ||
        (r = stage_out(s, Dd, sc[4], (size_t)2 * n)) || (r = stage_out(s, kappa, sc[5], (size_t)n)))
        return r;
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

int qsp_eval_dynamics(qsp_solver* s, int32_t n, const int32_t* sid, const double* x, const double* u, double* f,
                      double* J) {
    if (!s || !sid || !x || !u || !f || !J || n < 1) return fail(QSP_ERR_ARG, "qsp_eval_dynamics: bad argument");
    int r = check_ids(s, n, sid);
    if (r) return r;
    HIPCHK(hipSetDevice(s->o.device));
    auto& sc = s->scratch;
    if ((r = stage_in(s, sc[0], sid, n)) || (r = stage_in(s, sc[1], x, (size_t)4 * n)) ||
        (r = stage_in(s, sc[2], u, (size_t)2 * n)))
        return r;
    HIPCHK(sc[3].ensure((size_t)n * 32)); HIPCHK(sc[4].ensure((size_t)n * 24 * 8));
    HIPCHK(launch_dynamics(s->shapes.as<ShapeDev>(), sc[0].as<int32_t>(), n, sc[1].as<double>(), sc[2].as<double>(),
                           sc[3].as<double>(), sc[4].as<double>(), s->stream));
    if ((r = stage_out(s, f, sc[3], (size_t)4 * n)) || (r = stage_out(s, J, sc[4], (size_t)24 * n))) return r;
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

int qsp_eval_rk4(qsp_solver* s, int32_t n, const int32_t* sid, double h, const double* x, const double* u, double* xn,
                 double* A, double* B) {
    if (!s || !sid || !x || !u || !xn || !A || !B || n < 1) return fail(QSP_ERR_ARG, "qsp_eval_rk4: bad argument");
    int r = check_ids(s, n, sid);
    if (r) return r;
    HIPCHK(hipSetDevice(s->o.device));
    auto& sc = s->scratch;
    if ((r = stage_in(s, sc[0], sid, n)) || (r = stage_in(s, sc[1], x, (size_t)4 * n)) ||
        (r = stage_in(s, sc[2], u, (size_t)2 * n)))
        return r;
    HIPCHK(sc[3].ensure((size_t)n * 32)); HIPCHK(sc[4].ensure((size_t)n * 128)); HIPCHK(sc[5].ensure((size_t)n * 64));
    HIPCHK(launch_rk4(s->shapes.as<ShapeDev>(), sc[0].as<int32_t>(), n, h, sc[1].as<double>(), sc[2].as<double>(),
                      sc[3].as<double>(), sc[4].as<double>(), sc[5].as<double>(), s->stream));
    if ((r = stage_out(s, xn, sc[3], (size_t)4 * n)) || (r = stage_out(s, A, sc[4], (size_t)16 * n)) ||
        (r = stage_out(s, B, sc[5], (size_t)8 * n)))
        return r;
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

int qsp_eval_vbound(qsp_solver* s, int32_t n, const int32_t* sid, const double* sv, double* vb) {
    if (!s || !sid || !sv || !vb || n < 1) return fail(QSP_ERR_ARG, "qsp_eval_vbound: bad argument");
    int r = check_ids(s, n, sid);
    if (r) return r;
    HIPCHK(hipSetDevice(s->o.device));
    auto& sc = s->scratch;
    if ((r = stage_in(s, sc[0], sid, n)) || (r = stage_in(s, sc[1], sv, n))) return r;
    HIPCHK(sc[2].ensure((size_t)n * 8));
    HIPCHK(launch_vbound(s->shapes.as<ShapeDev>(), sc[0].as<int32_t>(), n, s->p.cp, sc[1].as<double>(),
                         sc[2].as<double>(), s->stream));
    if ((r = stage_out(s, vb, sc[2], (size_t)n))) return r;
    HIPCHK(hipStreamSynchronize(s->stream));
    return QSP_OK;
}

int qsp_qp_solve(qsp_solver* s, int32_t nb, const double* A, const double* B, const double* b, const double* H,
                 const double* g, const double* lo, const double* hi, const double* dx0, double* dx, double* du,
                 double* pi, double* lam, int32_t* iters, int32_t* qp_status) {
    if (!s || nb < 1 || !A || !B || !b || !H || !g || !lo || !hi || !dx0 || !dx || !du || !pi || !lam || !iters)
        return fail(QSP_ERR_ARG, "qsp_qp_solve: bad argument");
    const int N = s->o.N;
    SolveParams p = s->p;
    p.tau = 1.0;
    for (int i = 0; i < 6; ++i) p.W[i] = H[i];
    for (int i = 0; i < 4; ++i) p.We[i] = H[6 * N + i];
    // bounds in step space lo = lh - v, hi = uh - v with lh = 0, uh = width, v = -lo
    for (int j = 0; j < 3; ++j) { p.lh[j] = 0.0; p.uh[j] = hi[j] - lo[j]; }
    for (int l = 0; l < nb; ++l) {
        for (int k = 0; k < N; ++k) {
            for (int i = 0; i < 6; ++i)
                if (H[(size_t)l * (6 * N + 4) + 6 * k + i] != p.W[i])
                    return fail(QSP_ERR_ARG, "qsp_qp_solve: stage Hessian must be equal on every stage");
            for (int j = 0; j < 3; ++j) {
                const double w = hi[((size_t)l * N + k) * 3 + j] - lo[((size_t)l * N + k) * 3 + j];
                if (std::fabs(w - p.uh[j]) > 1e-12 * (1.0 + std::fabs(w)))
                    return fail(QSP_ERR_ARG, "qsp_qp_solve: bound widths must be equal on every stage");
            }
            const double* Ak = A + ((size_t)l * N + k) * 16;
            const double st[10] = {Ak[0] - 1.0, Ak[1], Ak[4], Ak[5] - 1.0, Ak[8], Ak[9], Ak[10] - 1.0, Ak[12], Ak[13], Ak[14]};
            for (double v : st)
                if (v != 0.0) return fail(QSP_ERR_ARG, "qsp_qp_solve: A lacks the pusher-slider structure");
        }
        for (int i = 0; i < 4; ++i)
            if (H[(size_t)l * (6 * N + 4) + 6 * N + i] != p.We[i])
                return fail(QSP_ERR_ARG, "qsp_qp_solve: terminal Hessian must be equal on every lane");
    }
    // pack the workspace on the host: stage data SoA, v = -lo through X/U, x0 - X_0 = dx0
    const size_t tot = (size_t)nb * (N + 1);
    std::vector<double> lin(tot * 24, 0.0), X(tot * 4, 0.0), U((size_t)nb * N * 2, 0.0), x0(dx0, dx0 + (size_t)nb * 4);
    for (int l = 0; l < nb; ++l) {
        for (int k = 0; k <= N; ++k) {
            const size_t gi = (size_t)l * (N + 1) + k;
            if (k < N) {
                const double* Ak = A + ((size_t)l * N + k) * 16;
                const double av[6] = {Ak[2], Ak[3], Ak[6], Ak[7], Ak[11], Ak[15]};
                for (int q = 0; q < 6; ++q) lin[(0 + q) * tot + gi] = av[q];
                for (int q = 0; q < 8; ++q) lin[(6 + q) * tot + gi] = B[((size_t)l * N + k) * 8 + q];
                for (int q = 0; q < 4; ++q) lin[(14 + q) * tot + gi] = b[((size_t)l * N + k) * 4 + q];
                for (int q = 0; q < 6; ++q) lin[(18 + q) * tot + gi] = g[(size_t)l * (6 * N + 4) + 6 * k + q];
                X[gi * 4 + 3] = -lo[((size_t)l * N + k) * 3 + 0];
                U[((size_t)l * N + k) * 2 + 0] = -lo[((size_t)l * N + k) * 3 + 1];
                U[((size_t)l * N + k) * 2 + 1] = -lo[((size_t)l * N + k) * 3 + 2];
            } else {
                for (int q = 0; q < 4; ++q) lin[(18 + q) * tot + gi] = g[(size_t)l * (6 * N + 4) + 6 * N + q];
            }
        }
        // dx0 = wx0 - X_0 with X_0 = (0, 0, 0, -lo_s(0))  ->  wx0 = dx0 + X_0
        x0[(size_t)l * 4 + 3] += X[(size_t)l * (N + 1) * 4 + 3];
    }
    HIPCHK(hipSetDevice(s->o.device));
    auto& sc = s->scratch;
    int r;
    if ((r = stage_in(s, sc[0], lin.data(), lin.size())) || (r = stage_in(s, sc[1], X.data(), X.size())) ||
        (r = stage_in(s, sc[2], U.data(), U.size())) || (r = stage_in(s, sc[3], x0.data(), x0.size())))
        return r;
    HIPCHK(sc[4].ensure((size_t)nb * (N + 1) * 32)); HIPCHK(sc[5].ensure((size_t)nb * N * 16));
    HIPCHK(sc[6].ensure((size_t)nb * N * 32)); HIPCHK(sc[7].ensure((size_t)nb * N * 48));
    HIPCHK(sc[8].ensure((size_t)nb * 4));
    HIPCHK(sc[9].ensure((size_t)nb * 4));
    SolveArgs a;
    std::memset(&a, 0, sizeof a);
    a.p = p;
    a.B = nb;
    a.wlin = sc[0].as<double>(); a.wX = sc[1].as<double>(); a.wU = sc[2].as<double>(); a.wx0 = sc[3].as<double>();
    a.qp_dx = sc[4].as<double>(); a.qp_du = sc[5].as<double>(); a.PI_out = sc[6].as<double>();
    a.qp_lam = sc[7].as<double>(); a.qp_iter = sc[8].as<int32_t>();
    a.qp_capped = sc[9].as<int32_t>();
    HIPCHK(launch_qp(a, s->S, s->stream));
    if ((r = stage_out(s, dx, sc[4], (size_t)nb * (N + 1) * 4)) || (r = stage_out(s, du, sc[5], (size_t)nb * N * 2)) ||
        (r = stage_out(s, pi, sc[6], (size_t)nb * N * 4)) || (r = stage_out(s, lam, sc[7], (size_t)nb * N * 6)) ||
        (r = stage_out(s, iters, sc[8], (size_t)nb)))
        return r;
    std::vector<int32_t> qst(qp_status ? (size_t)nb : 0);
    if (qp_status && (r = stage_out(s, qst.data(), sc[9], (size_t)nb))) return r;
    HIPCHK(hipStreamSynchronize(s->stream));
    if (qp_status) {
        for (int l = 0; l < nb; ++l) {
            bool fin = true;
            for (int q = 0; q < (N + 1) * 4; ++q) fin = fin && std::isfinite(dx[(size_t)l * (N + 1) * 4 + q]);
            for (int q = 0; q < N * 2; ++q) fin = fin && std::isfinite(du[(size_t)l * N * 2 + q]);
            // the stage-0 s is fixed (dx_0 = dx0): outside its bounds the QP is infeasible
            const bool infeas = s->p.s0_bound && (dx0[(size_t)l * 4 + 3] < lo[(size_t)l * N * 3] ||
                                                  dx0[(size_t)l * 4 + 3] > hi[(size_t)l * N * 3]);
            qp_status[l] = !fin ? 1 : (infeas ? 3 : qst[l]);
        }
    }
    return QSP_OK;
}

}  // extern "C"
