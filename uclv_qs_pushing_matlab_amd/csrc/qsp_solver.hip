// qsp_solver.hip — batched pusher–slider NMPC solve on gfx950 (FP64).
//
// Lane layout: one NMPC instance owns a group of L = ceil((N+1)/S)
// consecutive lanes of a wavefront; lane `lig` of the group owns the S horizon
// stages k = lig*S .. lig*S+S-1 (stage N is the terminal stage).  Every per-stage
// quantity (stage model, IPM slacks/multipliers, Riccati factors) lives in that
// lane's VGPRs or its LDS column for the whole QP; nothing spills to HBM between
// IPM iterations.  Stage-parallel work (barrier terms, step lengths) runs on all
// lanes at once; the horizon recursions (Riccati backward, state forward, adjoint)
// walk the group lane by lane, handing the 4x4 value function / state step to the
// neighbour lane with one DPP wave shift.  With one stage per lane the walks after the
// factorisation run in closed-loop form (one 4x4 affine map per step).
//
// One solve = prologue (NMPC_controller.solve wrapper) + K x qp_step [linearisation
// (RK4 + sensitivities, one lane per stage) and one QP per instance] + epilogue.
// Before each QP launch the instances are packed into waves by the IPM iteration
// count of their previous QP, longest first (sort_by_iters_kernel, on a histogram the
// QP kernel accumulates).
//
// Algorithm (restating the reference OCP, NMPC_controller.m:174-300):
//   SQP  : nlp_mode 0 — fixed-K full Gauss-Newton steps (BASELINE "SQP-RTI, K iterations");
//          nlp_mode 1 — the reference's 'SQP' + 'merit_backtracking': KKT test with
//          tol 1e-6, l1-merit Armijo backtracking (qp_step<1, true> + merit_ls_kernel)
//   QP   : box-constrained LQ-OCP, Mehrotra predictor-corrector interior point,
//          Riccati factorisation reused by the corrector, whose backward pass runs
//          on the difference to the predictor (stands in for HPIPM);
//          stops on mu < mu_stop and bound residual < res_stop, or at qp_iters
//   model: RK4 (1 step, h = Ts) + forward sensitivities of f (qsp_math.hpp)
// Also here: the device closed loop (plant_kernel, helper.m:195-322), per-lane
// reference generation (straight_lines_kernel) and the building-block kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/qsp_nmpc.h"
#include "qsp_math.hpp"
#include "qsp_kernels.h"

#ifndef QSP_MIN_WAVES
#define QSP_MIN_WAVES 1
#endif

namespace qsp {

// Diagnostic build only (-DQSP_SEGSTAMP, scripts/segstamps.py): wave cycles per QP-kernel segment, summed
// over the waves by lane 0 of each (s_memtime; the stamps themselves cost ~10 % of the wave time).
#ifdef QSP_SEGSTAMP
#ifndef QSP_SEGMASK
#define QSP_SEGMASK 0xffffffffu   // which segments are stamped (fewer stamps: less distortion)
#endif
__device__ unsigned long long g_seg[32];
__device__ __forceinline__ unsigned long long seg_now() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ void seg_add(int i, unsigned long long t0) {
    if (!((QSP_SEGMASK >> i) & 1u)) return;
    const unsigned long long t = seg_now();
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_seg[i], t - t0);
}
#define SEG_T(v) unsigned long long v = seg_now()
#define SEG_ADD(i, v) seg_add(i, v)
#define SEG_NEXT(i, v) do { seg_add(i, v); v = seg_now(); } while (0)
#else
#define SEG_T(v)
#define SEG_ADD(i, v)
#define SEG_NEXT(i, v)
#endif

// ------------------------------------------------------------- group helpers
// Reductions over the L lanes of an instance group (lanes base .. base+L-1), leaving the
// same value in every lane of the group (identical decisions in all lanes of an instance).
// Minima and maxima: a segmented inclusive scan over the whole wave with DPP row shifts
// (1, 2, 4, 8 inside each row of 16) and the row broadcasts of lanes 15 and 31 —
// register-to-register moves on the VALU, no LDS round trip — gathers the group's value in
// its last lane; one shuffle broadcasts it.  A lane takes a shifted value only when its
// source lane lies in the same group, so groups of any length L <= 64 and any alignment
// reduce independently.  Sums: see group_sum.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_move(double v) {
    // lanes without a source (row edge, rows outside ROWS) read 0, which the caller's group
    // mask never takes.  (update_dpp, not mov_dpp: the move must stay outside the masked
    // select — a DPP read from a lane disabled by EXEC does not return that lane's value.)
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS, 0xf, false);
    return __hiloint2double(hi, lo);
}

// Which scan steps a lane takes (its source lane lies in the same group); computed once.
struct GroupScan {
    bool s1, s2, s4, s8, b15, b31;
    int last;   // the group's last lane, where the scan completes
    int base, L;
    __device__ void init(int base_, int L_) {
        base = base_;
        L = L_;
        const int lane = (int)(threadIdx.x & 63);
        const int lig = lane - base_, col = lane & 15, row = lane >> 4;
        s1 = col >= 1 && lig >= 1;
        s2 = col >= 2 && lig >= 2;
        s4 = col >= 4 && lig >= 4;
        s8 = col >= 8 && lig >= 8;
        b15 = (row & 1) && lig > col;          // row_bcast:15 into rows 1, 3 (source 16 row - 1)
        b31 = row >= 2 && lig >= lane - 31;    // row_bcast:31 into rows 2, 3 (source 31)
        last = base_ + L_ - 1;
    }
};

// op(v, take ? o : identity) as a select on the moved value (never a branch: the DPP move
// must execute with every lane enabled)
struct OpMin {
    __device__ double operator()(double v, double o, bool take) const { return (take && o < v) ? o : v; }
};
struct OpMax {
    __device__ double operator()(double v, double o, bool take) const { return (take && o > v) ? o : v; }
};

template <class Op>
__device__ __forceinline__ double group_reduce(double v, const GroupScan& g, Op op) {
    v = op(v, dpp_move<0x111, 0xf>(v), g.s1);    // row_shr:1
    v = op(v, dpp_move<0x112, 0xf>(v), g.s2);    // row_shr:2
    v = op(v, dpp_move<0x114, 0xf>(v), g.s4);    // row_shr:4
    v = op(v, dpp_move<0x118, 0xf>(v), g.s8);    // row_shr:8
    v = op(v, dpp_move<0x142, 0xa>(v), g.b15);   // row_bcast:15
    v = op(v, dpp_move<0x143, 0xc>(v), g.b31);   // row_bcast:31
    return __shfl(v, g.last);
}
// Sums keep a log-step shuffle tree towards the group's first lane: its association depends
// only on the lane's place in the group, so an instance's result does not depend on where
// the wave packing puts it (a row-aligned scan would round differently at another offset;
// min and max are exact in any order).
__device__ __forceinline__ double group_sum(double v, const GroupScan& g) {
    const int lane = (int)(threadIdx.x & 63);
    const int lig = lane - g.base;
    for (int off = 1; off < g.L; off <<= 1) {
        const double o = __shfl(v, lane + off);
        v += (lig + off < g.L) ? o : 0.0;
    }
    return __shfl(v, g.base);
}
__device__ __forceinline__ double group_min(double v, const GroupScan& g) { return group_reduce(v, g, OpMin()); }
__device__ __forceinline__ double group_max(double v, const GroupScan& g) { return group_reduce(v, g, OpMax()); }

// rcp(x): 1/x from the hardware reciprocal and two Newton steps (qsp_fp.hpp; ≈ 5 instructions
// instead of the ≈ 10 of the IEEE division sequence, and the correctly rounded 1/x)

// symmetric 4x4 stored as 10 entries: (0,0)(0,1)(0,2)(0,3)(1,1)(1,2)(1,3)(2,2)(2,3)(3,3)
__device__ __forceinline__ int sidx(int i, int j) {
    if (i > j) { int t = i; i = j; j = t; }
    return i == 0 ? j : (i == 1 ? 3 + j : (i == 2 ? 5 + j : 9));
}

// Wave packing.  wnit holds an instance's last four IPM iteration counts c1 | c2 << 8 |
// c3 << 16 | c4 << 24 (c1 the last; 0 = not yet recorded).  The fixed-K SQP settles into
// period-2 cycles on many lanes, so the count two iterations back predicts the coming QP
// better than the last one (bench workload, oracle: equal to it on 71 % of the QPs against
// 58 %).  The key orders by the prediction p = c2 where the lane repeats with period 2
// (c2 == c4), else c1, longest first (LPT, so a launch does not end on a tail of long waves),
// ties by c2.  Over 50 SQP iterations of 3 072 bench lanes (3 instances per wave) waves then
// run 1.060x the mean iteration count, against 1.065x ordering by (c1, c2), 1.094x by c1 alone
// and 1.244x unsorted (perfect prediction: 1.001x).
constexpr int PACK_KEYS_MAX = 1024;   // (maxkey + 1)^2 keys
// key levels: IPM counts above 31 share the last level (qp_iters up to 50 and more: the
// acados default cap; such QPs are rare, ~0.1 % of the bench workload's)
__host__ __device__ __forceinline__ int pack_maxkey(int qp_iters) { return qp_iters < 31 ? qp_iters : 31; }
__device__ __forceinline__ int pack_key(int packed, int maxkey) {
    const int c1 = packed & 0xff, c2 = (packed >> 8) & 0xff, c4 = (packed >> 24) & 0xff;
    const int pred = (c4 != 0 && c2 == c4) ? c2 : c1;
    const int p = min(max(pred, 0), maxkey), q = min(max(c2, 0), maxkey);
    return (maxkey - p) * (maxkey + 1) + (maxkey - q);
}
__device__ __forceinline__ int pack_record(int old, int nit) { return (int)(((unsigned)old << 8) | (unsigned)(nit & 0xff)); }

// ------------------------------------------------------------- per-lane state
// Registers hold what the horizon recursions read on every step (stage model,
// gradient, Riccati factors); LDS holds what only the stage-parallel phases touch
// (iterate, slacks/multipliers, barrier terms, QP solution pieces).
constexpr int BLOCK = 64;                  // threads per workgroup: one wave (see launch_qp_step)
enum LdsField : int {
    F_T = 0,      // 6  slacks        s_lo s_hi un_lo un_hi ut_lo ut_hi
    F_LM = 6,     // 6  multipliers
    F_V = 12,     // 3  bounded components of the SQP iterate (s_k, u_n, u_t)
    F_DU = 15,    // 2  damped QP control step
    F_RT = 17,    // 6  1 / slack, refreshed whenever the slacks change
    F_VA = 23,    // 3  affine-predictor bounded components (ds, dun, dut)
    F_VN = 26,    // 3  corrector bounded components
    F_DX = 23,    // 4  final QP state step (written after the IPM: aliases F_VA / F_VN)
    F_HG = 29,    // 6  barrier Hessian (0..2) / gradient (3..5) additions
    F_COUNT = 35
};
// S = 1: the matrix-core factor walk's stage records overlay F_VA .. F_HG (free while the predictor
// factorises) and mfw_extra<S>() more fields (factor_walk_mfma)
// (S = 1: two, so eight one-wave workgroups and a packing-sort workgroup still share a CU's LDS; S = 2:
// three, every horizon up to N = 127)
template <int S>
constexpr int mfw_extra() { return S == 1 ? 2 : 4; }
template <int S>
constexpr int lds_bytes() { return (F_COUNT * S + mfw_extra<S>()) * BLOCK * 8; }

template <int S>
struct Stage {
    double g[S][6];          // cost gradient (stage: tau W (y - y_ref); terminal: We (x - y_ref_e))
    double a[S][6];          // free entries of A_k (qsp_math.hpp rk4)
    double B[S][8];
    double bb[S][4];         // defect phi(x_k,u_k) - x_{k+1}
    double K[S][8], Rn[S][3], kk[S][2];   // Rn = -R~^-1
    double* lds;             // this thread's column of the workgroup's LDS block
    __device__ __forceinline__ double& f(int field, int ls, int i) const { return lds[((field + i) * S + ls) * BLOCK]; }
    __device__ __forceinline__ double& t(int ls, int q) const { return f(F_T, ls, q); }
    __device__ __forceinline__ double& lm(int ls, int q) const { return f(F_LM, ls, q); }
    __device__ __forceinline__ double& v(int ls, int i) const { return f(F_V, ls, i); }
    __device__ __forceinline__ double& du(int ls, int i) const { return f(F_DU, ls, i); }
    __device__ __forceinline__ double& dxs(int ls, int i) const { return f(F_DX, ls, i); }
    __device__ __forceinline__ double& hg(int ls, int i) const { return f(F_HG, ls, i); }
    __device__ __forceinline__ double& rt(int ls, int q) const { return f(F_RT, ls, q); }
};

struct Ctx {
    int lane, L, grp, lig, base, N;
    bool real;
    int inst;
    GroupScan gs;
};

template <int S>
__device__ __forceinline__ int kof(const Ctx& c, int ls) { return c.lig * S + ls; }

// Is bound side j (0 = s, 1 = u_n, 2 = u_t) of stage k part of the QP?  Stages 0..N-1; the s
// bound at stage 0 only with stage0_s_bound (s_0 is fixed by x0 there: the pair is a
// constant slack that enters the complementarity measure, NMPC_controller.m:237,251-252).
__device__ __forceinline__ bool bnd_act(const Ctx& c, const SolveParams& p, int k, int j) {
    return (k < c.N) && (j > 0 || k >= 1 || p.s0_bound != 0);
}

// bounds of the QP step of slot ls: lo = lh - v, hi = uh - v, v = (s, u_n, u_t)
template <int S>
__device__ __forceinline__ void bnd_lohi(const SolveParams& p, const Stage<S>& st, int ls, double lo[3], double hi[3]) {
    const double v0 = st.v(ls, 0), v1 = st.v(ls, 1), v2 = st.v(ls, 2);
    lo[0] = p.lh[0] - v0; hi[0] = p.uh[0] - v0;
    lo[1] = p.lh[1] - v1; hi[1] = p.uh[1] - v1;
    lo[2] = p.lh[2] - v2; hi[2] = p.uh[2] - v2;
}

// chain hand-over along the wavefront without an LDS round trip (DPP wave shift)
// (lanes without a source keep their own value, so the move can be done in place)
__device__ __forceinline__ double wave_from_next(double v) {   // lane i <- lane i+1
    const int l = __double2loint(v), h = __double2hiint(v);
    const int lo = __builtin_amdgcn_update_dpp(l, l, 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(h, h, 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
// lane i <- lane i+1's v; lanes without a source keep `old`.  With old = the value
// the register held before the step, a hand-over inside a divergent region needs no
// extra copy to merge the lanes that sat the step out.
__device__ __forceinline__ double wave_from_next(double old, double v) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
// lane i <- lane i-1's v; lane 0 keeps `old` (the walks never read it there), so the
// result can take old's register in a loop without a copy
__device__ __forceinline__ double wave_from_prev(double old, double v) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_from_prev(double v) {   // lane i <- lane i-1
    const int l = __double2loint(v), h = __double2hiint(v);
    const int lo = __builtin_amdgcn_update_dpp(l, l, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(h, h, 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// --------------------------------------------------------- Riccati primitives
// Terminal value function: P = diag(We), p = g_N
__device__ __forceinline__ void ric_terminal(const SolveParams& p, const double g[6], double P[10], double pv[4]) {
#pragma unroll
    for (int i = 0; i < 10; ++i) P[i] = 0.0;
    P[0] = p.We[0]; P[4] = p.We[1]; P[7] = p.We[2]; P[9] = p.We[3];
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = g[i];
}

// One backward factorisation step exploiting A = [[1,0,a0,a1],[0,1,a2,a3],[0,0,1,a4],[0,0,0,a5]].
// Hx, Hu: diagonal stage Hessian (incl. barrier); gx, gu: gradient (incl. barrier).
// Every sum is one left-to-right FMA chain from its additive term (or its first product).
__device__ __forceinline__ void ric_factor_step(const double a[6], const double B[8], const double bb[4],
                                                const double Hx[4], const double Hu[2],
                                                const double gx[4], const double gu[2],
                                                double P[10], double pv[4],
                                                double K[8], double Rn[3], double kk[2], bool upd = true) {
    // full symmetric P
    double Pm[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) Pm[i][j] = P[sidx(i, j)];
    // PA (columns 0, 1 of A are e0, e1)
    double PA[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        PA[i][0] = Pm[i][0];
        PA[i][1] = Pm[i][1];
        PA[i][2] = qfma(Pm[i][1], a[2], qfma(Pm[i][0], a[0], Pm[i][2]));
        PA[i][3] = qfma(Pm[i][3], a[5], qfma(Pm[i][2], a[4], qfma(Pm[i][1], a[3], Pm[i][0] * a[1])));
    }
    // PB
    double PB[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            PB[i][j] = qfma(Pm[i][3], B[6 + j], qfma(Pm[i][2], B[4 + j], qfma(Pm[i][1], B[2 + j], Pm[i][0] * B[j])));
    // pp = p + P b
    double pp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        pp[i] = qfma(Pm[i][3], bb[3], qfma(Pm[i][2], bb[2], qfma(Pm[i][1], bb[1], qfma(Pm[i][0], bb[0], pv[i]))));
    // R~ = Hu + B'PB (sym), S~ = B'PA (2x4), r~ = gu + B'pp
    const double R00 = qfma(B[6], PB[3][0], qfma(B[4], PB[2][0], qfma(B[2], PB[1][0], qfma(B[0], PB[0][0], Hu[0]))));
    const double R01 = qfma(B[6], PB[3][1], qfma(B[4], PB[2][1], qfma(B[2], PB[1][1], B[0] * PB[0][1])));
    const double R11 = qfma(B[7], PB[3][1], qfma(B[5], PB[2][1], qfma(B[3], PB[1][1], qfma(B[1], PB[0][1], Hu[1]))));
    // S~ = B'PA = (PB)'A with the structure of A
    double St[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        St[i][0] = PB[0][i];
        St[i][1] = PB[1][i];
        St[i][2] = qfma(PB[1][i], a[2], qfma(PB[0][i], a[0], PB[2][i]));
        St[i][3] = qfma(PB[3][i], a[5], qfma(PB[2][i], a[4], qfma(PB[1][i], a[3], PB[0][i] * a[1])));
    }
    double rt[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
        rt[i] = qfma(B[6 + i], pp[3], qfma(B[4 + i], pp[2], qfma(B[2 + i], pp[1], qfma(B[i], pp[0], gu[i]))));
    // Q~ = Hx + A'PA  (upper triangle), q~ = gx + A'pp
    double Qt[10];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const double c0 = PA[0][j], c1 = PA[1][j], c2 = PA[2][j], c3 = PA[3][j];
        if (j >= 0) Qt[sidx(0, j)] = c0;
        if (j >= 1) Qt[sidx(1, j)] = c1;
        if (j >= 2) Qt[sidx(2, j)] = qfma(a[2], c1, qfma(a[0], c0, j == 2 ? Hx[2] + c2 : c2));
        if (j >= 3) Qt[sidx(3, j)] = qfma(a[5], c3, qfma(a[4], c2, qfma(a[3], c1, qfma(a[1], c0, Hx[3]))));
    }
    Qt[0] += Hx[0]; Qt[4] += Hx[1];
    double qt[4];
    qt[0] = gx[0] + pp[0];
    qt[1] = gx[1] + pp[1];
    qt[2] = qfma(a[2], pp[1], qfma(a[0], pp[0], gx[2] + pp[2]));
    qt[3] = qfma(a[5], pp[3], qfma(a[4], pp[2], qfma(a[3], pp[1], qfma(a[1], pp[0], gx[3]))));
    // Rn = -R~^-1 (kept negated: the sign folds into the multiplies)
    const double idet = rcp(qfma(R00, R11, -(R01 * R01)));
    Rn[0] = (-R11) * idet; Rn[1] = R01 * idet; Rn[2] = (-R00) * idet;
    // K = -R~^-1 S~ ; kk = -R~^-1 r~
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        K[j] = qfma(Rn[1], St[1][j], Rn[0] * St[0][j]);
        K[4 + j] = qfma(Rn[2], St[1][j], Rn[1] * St[0][j]);
    }
    kk[0] = qfma(Rn[1], rt[1], Rn[0] * rt[0]);
    kk[1] = qfma(Rn[2], rt[1], Rn[1] * rt[0]);
    // P = Q~ + S~'K ; p = q~ + K'r~ (not at stage 0: nothing reads P_0, p_0; upd is uniform)
    if (!upd) return;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) P[sidx(i, j)] = qfma(St[1][i], K[4 + j], qfma(St[0][i], K[j], Qt[sidx(i, j)]));
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = qfma(K[4 + i], rt[1], qfma(K[i], rt[0], qt[i]));
}

// Vector-only backward step of the Mehrotra corrector, on the DIFFERENCE to the predictor:
// the corrector changes only the gradient, by dg = (0, 0, 0, dgx3; dgu0, dgu1) (barrier
// correction terms), and the recursion is linear in the gradient with the same factors, so
//   dr = dgu + B' dp,  dq = dgx + A' dp,  dkk = Rn dr,  dp <- dq + K' dr,  dp_N = 0
// (P b cancels in the difference; kk_corr = kk_pred + dkk).
__device__ __forceinline__ void ric_delta_step(const double a[6], const double B[8], double dgx3, const double dgu[2],
                                               const double K[8], const double Rn[3], double pv[4], double dkk[2]) {
    double rt[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
        rt[i] = qfma(B[6 + i], pv[3], qfma(B[4 + i], pv[2], qfma(B[2 + i], pv[1], qfma(B[i], pv[0], dgu[i]))));
    double qt[4];
    qt[0] = pv[0];
    qt[1] = pv[1];
    qt[2] = qfma(a[2], pv[1], qfma(a[0], pv[0], pv[2]));
    qt[3] = qfma(a[5], pv[3], qfma(a[4], pv[2], qfma(a[3], pv[1], qfma(a[1], pv[0], dgx3))));
    dkk[0] = qfma(Rn[1], rt[1], Rn[0] * rt[0]);
    dkk[1] = qfma(Rn[2], rt[1], Rn[1] * rt[0]);
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = qfma(K[4 + i], rt[1], qfma(K[i], rt[0], qt[i]));
}

// dx_{k+1} = A dx + B du + b
__device__ __forceinline__ void dyn_step(const double a[6], const double B[8], const double bb[4],
                                         const double du[2], double dx[4]) {
    const double n0 = qfma(B[1], du[1], qfma(B[0], du[0], qfma(a[1], dx[3], qfma(a[0], dx[2], bb[0] + dx[0]))));
    const double n1 = qfma(B[3], du[1], qfma(B[2], du[0], qfma(a[3], dx[3], qfma(a[2], dx[2], bb[1] + dx[1]))));
    const double n2 = qfma(B[5], du[1], qfma(B[4], du[0], qfma(a[4], dx[3], bb[2] + dx[2])));
    const double n3 = qfma(B[7], du[1], qfma(B[6], du[0], qfma(a[5], dx[3], bb[3])));
    dx[0] = n0; dx[1] = n1; dx[2] = n2; dx[3] = n3;
}

// ------------------------------------- S = 1: the factorisation on the FP64 matrix cores
// The factor walk's step is a handful of 4x4 products, which v_mfma_f64_4x4x4_4b_f64 computes for
// four independent blocks of 16 lanes at once: lane l holds element (l >> 4, l & 3) of block
// (l >> 2) & 3 of each operand, and the A operand is read transposed (mfma4(X, Y, C) = X'Y + C per
// block; scripts/ubench/mfma_f64_probe.hip).  Block b walks instance min(b, G - 1) of the wave with
// its value function held one element per lane, so a step costs eleven matrix-core products and
// ~45 VALU instead of the lane walk's ~210 VALU on 1 of 21 lanes.
// The stage data reaches the blocks through LDS: before the walk every stage lane writes a
// 27-double record (MfwSlot) over the fields that are free while the predictor factorises (F_VA ..
// F_HG and mfw_extra<S>() more); the block lanes read their operand elements from it, one step ahead,
// and write the stage's K and [R~ | r~] back over its first 16 slots, which the stage lane collects
// after the walk (forming -R~^-1 and kk itself, in parallel).  The records of a wave's G instances do not fit at once: the walk runs in two
// phases (stages H .. N-1 with the terminal record, then 0 .. H-1).
// (a record row-major in the order the block lanes read it: [B | b] row by row, so the lanes of two matrix
// rows read at most six consecutive doubles per operand, which the three instances' records -- 9 apart
// mod 32 at N = 20 -- keep on disjoint LDS banks)
enum MfwSlot : int { R_G = 0, R_A = 12, R_GX = 18, R_HX3 = 22, R_HU = 23, R_GU = 25, MFW_REC = 27 };
enum MfwOut : int { O_K = 0, O_Z = 8, O_COUNT = 16 };   // K (2 x 4), rows 0, 1 of Z = [R~ | r~ | .]
// the operand constants (A's ones and zeros, the zero column of [B | b | 0], Hx's fixed diagonal), at the
// end of the region: the lanes whose operand element is one read it there instead of from the record
enum MfwConst : int { C_ONE = 0, C_ZERO = 1, C_HX = 2, C_COUNT = 5 };
static_assert((F_COUNT - F_VA + mfw_extra<1>()) * BLOCK >= 33 * MFW_REC + C_COUNT, "S = 1: records of G (N/2 + 1) stages, 12 <= N <= 31");
static_assert(((F_COUNT - F_VA) * 2 + mfw_extra<2>()) * BLOCK >= 64 * MFW_REC + C_COUNT, "S = 2: records of G (N/2 + 1) stages, N <= 127");

__device__ __forceinline__ double mfma4(double a, double b, double c) {   // a'b + c per 4x4 block
    return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
// The walk hands data between lanes of the one wave through LDS (stage lanes publish, block lanes read,
// and back).  LDS executes a wave's instructions in order; this makes the order explicit to the compiler
// (no instruction on a single wave).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int CTRL>
__device__ __forceinline__ double quad_bcast(double v) {   // DPP quad_perm: one lane of each quad to all four
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

// LDS doubles the stage records may occupy: F_VA .. F_HG of every slot plus the extra fields.
template <int S>
constexpr int mfw_region() { return ((F_COUNT - F_VA) * S + mfw_extra<S>()) * BLOCK; }
// Which horizons factorise on the matrix cores: one instance per 16-lane block (G <= 4: at one
// stage per lane N >= 12, at two N >= 24), the records of a phase in the region.  One stage per lane
// takes the walk as its ALT kernel variant; two stages per lane by a uniform switch, since
// ALT is the factorisation scan there.
// The instances' record regions start IS doubles apart, IS >= CM records: a stride whose multiples put
// the instances' reads of one operand (at most six consecutive doubles per half wave) on disjoint LDS banks
// (32 doubles): 9 ... 11 or 21 ... 23 mod 32 for three instances, 8 or 24 for four, 6 ... 26 for two.
__host__ __device__ __forceinline__ int mfw_stride(int CM, int G) {
    const int rs = CM * MFW_REC;
    for (int is = rs;; ++is) {
        const int m = is & 31;
        if (G <= 1 || (G == 2 && m >= 6 && m <= 26) || (G == 3 && ((m >= 9 && m <= 11) || (m >= 21 && m <= 23))) ||
            (G >= 4 && (m == 8 || m == 24)))
            return is;
    }
}
__host__ __device__ __forceinline__ bool mfw_fits(int N, int S) {
    const int L = (N + S) / S, G = 64 / L, H = (N + 1) / 2, CM = N + 1 - H;
    const int cap = S == 1 ? mfw_region<1>() : mfw_region<2>();
    return G <= 4 && (G - 1) * mfw_stride(CM, G) + CM * MFW_REC + C_COUNT <= cap && (S == 2 || N <= 31);
}
__host__ __device__ __forceinline__ bool mfw_use(const SolveParams& p, int S) { return p.mfw_on[S - 1] != 0; }
// (host, whenever N or mfma_walk change: the kernels read the choice and the stride instead of searching it)
void mfw_prepare(SolveParams& p) {
    for (int S = 1; S <= 2; ++S) {
        const int L = (p.N + S) / S, G = 64 / L, H = (p.N + 1) / 2, CM = p.N + 1 - H;
        p.mfw_on[S - 1] = p.mfma_walk != 0 && mfw_fits(p.N, S);
        p.mfw_is[S - 1] = G >= 1 && G <= 4 ? mfw_stride(CM, G) : CM * MFW_REC;
    }
}

template <int S>
__device__ __forceinline__ void factor_walk_mfma(const Ctx& c, const SolveParams& p, Stage<S>& st, const double (&hx3)[S],
                                                 const double (&hu)[S][2], const double (&gx3)[S], const double (&gu)[S][2]) {
    const int N = c.N, G = 64 / c.L;
    const int H = (N + 1) / 2, CM = N + 1 - H;   // phase split; records per instance and phase
    const int IS = p.mfw_is[S - 1];               // doubles from one instance's records to the next's (mfw_prepare)
    double* const reg = st.lds - (threadIdx.x & 63) + F_VA * S * BLOCK;
    // block-lane geometry and the record slot of each operand element (-1: structural constant)
    // (an opaque lane id: derived from c.lane, the geometry would be hoisted out of the IPM loop and
    // kept live through it)
    int l = c.lane;
    asm volatile("" : "+v"(l));
    const int b = (l >> 2) & 3, r = l >> 4, cc = l & 3;
    const int bg = b < G ? b : G - 1;
    const bool wr = b < G;
    // each operand element's record slot (-1: a structural constant, read from the constant slots instead)
    int ao = -1;
    if (cc >= 2 && r < 2) ao = R_A + 2 * r + (cc - 2);
    else if (cc == 3 && r >= 2) ao = R_A + 2 + r;
    const int go = cc < 3 ? R_G + 3 * r + cc : -1;
    const int ho = (r == 3 && cc == 3) ? R_HX3 : -1;   // Q's C (Hx): only hx3 varies
    int zo = -1;                                       // Z's C: Hu on the diagonal, gu in column 2
    if (r < 2 && r == cc) zo = R_HU + r;
    else if (r < 2 && cc == 2) zo = R_GU + r;
    const int qo = cc == 2 ? R_GX + r : -1;            // q~'s C: gx in column 2 (p lives there only)
    double* const cst = reg + mfw_region<S>() - C_COUNT;
    const int ac = r == cc ? C_ONE : C_ZERO, hc = r == cc && r < 3 ? C_HX + r : C_ZERO;
    if (c.lane < C_COUNT)   // the constants (the region's other fields change between walks)
        cst[c.lane] = c.lane == C_ONE ? 1.0 : (c.lane == C_ZERO ? 0.0 : p.tau * p.W[c.lane < C_HX ? 0 : c.lane - C_HX]);
    double P = 0.0, pv = 0.0;
    for (int ph = 0; ph < 2; ++ph) {
        const int kb = ph == 0 ? H : 0, ke = ph == 0 ? N : H - 1;   // records kb .. ke
        // publish: the stage lanes write the records of their slots' stages (one stage per lane written
        // as the lane test: the slot loop, the same test, costs the S = 1 kernel 2 % in issue order)
        if constexpr (S == 1) {
            if (c.grp < G && c.lig >= kb && c.lig <= ke) {
                double* rw = reg + c.grp * IS + (c.lig - kb) * MFW_REC;
                if (c.lig < N) {
#pragma unroll
                    for (int q = 0; q < 6; ++q) rw[R_A + q] = st.a[0][q];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        rw[R_G + 3 * q] = st.B[0][2 * q];
                        rw[R_G + 3 * q + 1] = st.B[0][2 * q + 1];
                        rw[R_G + 3 * q + 2] = st.bb[0][q];
                    }
#pragma unroll
                    for (int q = 0; q < 3; ++q) rw[R_GX + q] = st.g[0][q];
                    rw[R_GX + 3] = gx3[0];
                    rw[R_HX3] = hx3[0];
                    rw[R_HU] = hu[0][0];
                    rw[R_HU + 1] = hu[0][1];
                    rw[R_GU] = gu[0][0];
                    rw[R_GU + 1] = gu[0][1];
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) rw[R_GX + q] = st.g[0][q];   // terminal: p_N = g_N
                }
            }
        } else {
    #pragma unroll
            for (int ls = 0; ls < S; ++ls) {
                const int k = kof<S>(c, ls);
                if (c.grp < G && k >= kb && k <= ke) {
                    double* rw = reg + c.grp * IS + (k - kb) * MFW_REC;
                    if (k < N) {
    #pragma unroll
                        for (int q = 0; q < 6; ++q) rw[R_A + q] = st.a[ls][q];
    #pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            rw[R_G + 3 * q] = st.B[ls][2 * q];
                            rw[R_G + 3 * q + 1] = st.B[ls][2 * q + 1];
                            rw[R_G + 3 * q + 2] = st.bb[ls][q];
                        }
    #pragma unroll
                        for (int q = 0; q < 3; ++q) rw[R_GX + q] = st.g[ls][q];
                        rw[R_GX + 3] = gx3[ls];
                        rw[R_HX3] = hx3[ls];
                        rw[R_HU] = hu[ls][0];
                        rw[R_HU + 1] = hu[ls][1];
                        rw[R_GU] = gu[ls][0];
                        rw[R_GU + 1] = gu[ls][1];
                    } else {
    #pragma unroll
                        for (int q = 0; q < 4; ++q) rw[R_GX + q] = st.g[ls][q];   // terminal: p_N = g_N
                    }
                }
            }
        }
        wave_lds_sync();
        const double* rb = reg + bg * IS;   // this block's records of the phase
        if (ph == 0) {
            P = r == cc ? (r == 0 ? p.We[0] : (r == 1 ? p.We[1] : (r == 2 ? p.We[2] : p.We[3]))) : 0.0;
            pv = cc == 2 ? rb[(N - kb) * MFW_REC + R_GX + r] : 0.0;   // p_N = g_N (column 2)
        }
        const int kf = ph == 0 ? N - 1 : H - 1;
        // one step of the walk from its operand elements (Am: A, G2: [B | b | 0], CH and CZ: the C operands
        // of Q and Z, gq: gx); p lives in column 2 of pv, zero in the others, so T2 takes it as its C operand
        auto step = [&](int k, double Am, double G2, double CH, double CZ, double gq) {
            double* rk = reg + bg * IS + (k - kb) * MFW_REC;
            const double T1 = mfma4(P, Am, 0.0);                    // P'A
            const double T2 = mfma4(P, G2, pv);                     // P'[B | b | 0] + [0 | 0 | p | 0]
            const double Y = mfma4(G2, T1, 0.0);                    // rows 0, 1: S~ = B'P'A
            const double Z = mfma4(G2, T2, CZ);                     // rows 0, 1: [R~ | r~]
            const double Q = mfma4(Am, T1, CH);                     // Hx + A'P'A
            const double Qt = mfma4(T1, Am, CH);                    // its transpose (below)
            const double pp = cc == 2 ? T2 : 0.0;                   // p + P'b (column 2)
            const double qv = mfma4(Am, pp, gq);                    // q~ = gx + A'pp (column 2; the others +0)
            // R~ on the lanes of rows 0 and 1: v_permlane16_swap puts row 0 of Z into rows 0, 1 of its
            // first result and row 1 into rows 0, 1 of the second; quad broadcasts pick columns
            const auto slo = __builtin_amdgcn_permlane16_swap(__double2loint(Z), __double2loint(Z), false, false);
            const auto shi = __builtin_amdgcn_permlane16_swap(__double2hiint(Z), __double2hiint(Z), false, false);
            const double w0 = __hiloint2double(shi[0], slo[0]), w1 = __hiloint2double(shi[1], slo[1]);
            const double R00 = quad_bcast<0x00>(w0), R01 = quad_bcast<0x55>(w0), R11 = quad_bcast<0x55>(w1);
            // K = -R~^-1 S~ = (Xa'S~) / det with Xa = -adj R~: the product does not wait for the reciprocal
            const double det = qfma(R00, R11, -(R01 * R01));
            const double Xa = (r < 2 && cc < 2) ? (r != cc ? R01 : (r == 0 ? -R11 : -R00)) : 0.0;
            const double Ka = mfma4(Xa, Y, 0.0);
            const double idet = rcp(det);
            const double Kf = Ka * (r < 2 ? idet : 0.0);            // rows 0, 1: K; rows 2, 3: 0
            // (rows 2, 3 hold no R~: their idet is not finite, and Kf's zero rows enter P and p)
            // stage k's K and [R~ | r~] over the record's first slots (its operands are already read)
            if (wr && r < 2) {
                rk[O_K + 4 * r + cc] = Kf;
                rk[O_Z + 4 * r + cc] = Z;
            }
            if (k > 0) {   // P_k, p_k (nothing reads P_0, p_0)
                // P keeps its upper triangle and takes the lower one from the transposed products
                // (K'S~ + Q~', Q~' = T1'A + Hx: the same products in the same order, so bit for bit the
                // transpose): a symmetric P as the lane walk's.  Left to drift apart, the two triangles
                // cost the ill-conditioned QPs up to 1e3x the walk's error (tests/test_gpu_parity.py).
                const double RT = r < 2 && cc == 2 ? Z : 0.0;       // r~ (column 2)
                const double Pu = mfma4(Y, Kf, Q);                  // Q~ + S~'K
                const double Pl = mfma4(Kf, Y, Qt);                 // its transpose
                P = r <= cc ? Pu : Pl;
                pv = mfma4(Kf, RT, qv);                             // q~ + K'r~ (column 2; the others +0)
            }
        };
        // two operand sets, each read one step ahead, so the prefetch never waits on the step it feeds.
        // A lane reads each operand element through its own pointer: a record slot, stepping one record
        // down per step, or a constant slot, standing still (stride 0) -- no per-step selects
        const double* r0 = rb + (kf - kb) * MFW_REC;
        const double *pa = ao >= 0 ? r0 + ao : cst + ac, *pg = go >= 0 ? r0 + go : cst + C_ZERO;
        const double *ph_ = ho >= 0 ? r0 + ho : cst + hc, *pz = zo >= 0 ? r0 + zo : cst + C_ZERO;
        const double* pq = qo >= 0 ? r0 + qo : cst + C_ZERO;
        const int sa = ao >= 0 ? MFW_REC : 0, sg = go >= 0 ? MFW_REC : 0, sh = ho >= 0 ? MFW_REC : 0;
        const int sz = zo >= 0 ? MFW_REC : 0, sq = qo >= 0 ? MFW_REC : 0;
        double aA = *pa, gA = *pg, hA = *ph_, zA = *pz, qA = *pq, aB = 0.0, gB = 0.0, hB = 0.0, zB = 0.0, qB = 0.0;
        pa -= sa; pg -= sg; ph_ -= sh; pz -= sz; pq -= sq;
        // (the reads one record past the phase's last stage land inside the workgroup's LDS and go unused)
        for (int k = kf;; k -= 2) {
            aB = *pa; gB = *pg; hB = *ph_; zB = *pz; qB = *pq;
            pa -= sa; pg -= sg; ph_ -= sh; pz -= sz; pq -= sq;
            step(k, aA, gA, hA, zA, qA);
            if (k == kb) break;
            aA = *pa; gA = *pg; hA = *ph_; zA = *pz; qA = *pq;
            pa -= sa; pg -= sg; ph_ -= sh; pz -= sz; pq -= sq;
            step(k - 1, aB, gB, hB, zB, qB);
            if (k - 1 == kb) break;
        }
        wave_lds_sync();
        // collect: the stage lanes take their slots' factors (stages k < N)
        if constexpr (S == 1) {
            if (c.grp < G && c.lig >= kb && c.lig <= ke && c.lig < N) {
                const double* rr = reg + c.grp * IS + (c.lig - kb) * MFW_REC;
#pragma unroll
                for (int q = 0; q < 8; ++q) st.K[0][q] = rr[O_K + q];
                // Rn = -R~^-1 and kk = -R~^-1 r~ from the R~ the walk inverted (the same operations)
                const double* rz = rr + O_Z;
                const double R00 = rz[0], R01 = rz[1], rt0 = rz[2], R11 = rz[5], rt1 = rz[6];
                const double idet = rcp(qfma(R00, R11, -(R01 * R01)));
                st.Rn[0][0] = (-R11) * idet;
                st.Rn[0][1] = R01 * idet;
                st.Rn[0][2] = (-R00) * idet;
                st.kk[0][0] = qfma(st.Rn[0][1], rt1, st.Rn[0][0] * rt0);
                st.kk[0][1] = qfma(st.Rn[0][2], rt1, st.Rn[0][1] * rt0);
            }
        } else {
    #pragma unroll
            for (int ls = 0; ls < S; ++ls) {
                const int k = kof<S>(c, ls);
                if (c.grp < G && k >= kb && k <= ke && k < N) {
                    const double* rr = reg + c.grp * IS + (k - kb) * MFW_REC;
    #pragma unroll
                    for (int q = 0; q < 8; ++q) st.K[ls][q] = rr[O_K + q];
                    // Rn = -R~^-1 and kk = -R~^-1 r~ from the R~ the walk inverted (the same operations)
                    const double* rz = rr + O_Z;
                    const double R00 = rz[0], R01 = rz[1], rt0 = rz[2], R11 = rz[5], rt1 = rz[6];
                    const double idet = rcp(qfma(R00, R11, -(R01 * R01)));
                    st.Rn[ls][0] = (-R11) * idet;
                    st.Rn[ls][1] = R01 * idet;
                    st.Rn[ls][2] = (-R00) * idet;
                    st.kk[ls][0] = qfma(st.Rn[ls][1], rt1, st.Rn[ls][0] * rt0);
                    st.kk[ls][1] = qfma(st.Rn[ls][2], rt1, st.Rn[ls][1] * rt0);
                }
            }
        }
        wave_lds_sync();   // the next phase's records overwrite these
    }
    // the overlaid fields read later: the terminal and padding slots' F_VA / F_VN stay zero (the
    // forward passes write them on the stages k < N only; qp_ipm's start defines them)
    // (one stage per lane: written as the lane test, which keeps the kernel within two waves per SIMD
    // (249 registers); the unrolled slot loop, the same test, costs it the second wave)
    if constexpr (S == 1) {
        if (c.lig >= N) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                st.f(F_VA, 0, q) = 0.0;
                st.f(F_VN, 0, q) = 0.0;
            }
        }
    } else {
#pragma unroll
        for (int ls = 0; ls < S; ++ls) {
            if (kof<S>(c, ls) >= N) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    st.f(F_VA, ls, q) = 0.0;
                    st.f(F_VN, ls, q) = 0.0;
                }
            }
        }
    }
}

// ------------------------------------------------ S = 2: the affine passes as scans
// With two stages per lane (N + 1 > 32: configs[4]) the kernel runs one wave per SIMD, where a
// serial lane walk is latency-bound.  The forward passes and the corrector's difference pass are
// affine recursions, so they run as Hillis-Steele scans over the group's lanes instead
// (scripts/ubench/fwd_scan_s2.hip: 0.50x the walk's time at that occupancy).  Partner maps move by
// ds_bpermute; every composition is a fixed FMA order, restated by the oracle's twin.
struct Aff { double F[16], c[4]; };   // x -> F x + c

__device__ __forceinline__ double lane_read(double v, int src) {
    const int lo = __shfl(__double2loint(v), src), hi = __shfl(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ void aff_read(const Aff& e, int src, Aff& f) {
#pragma unroll
    for (int q = 0; q < 16; ++q) f.F[q] = lane_read(e.F[q], src);
#pragma unroll
    for (int q = 0; q < 4; ++q) f.c[q] = lane_read(e.c[q], src);
}
// g <- g o f (f applied first), in place row by row: row i of the result needs only row i of g
__device__ __forceinline__ void aff_compose(Aff& g, const Aff& f) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double r[5];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            r[j] = qfma(g.F[4 * i + 3], f.F[12 + j], qfma(g.F[4 * i + 2], f.F[8 + j],
                        qfma(g.F[4 * i + 1], f.F[4 + j], g.F[4 * i] * f.F[j])));
        r[4] = qfma(g.F[4 * i + 3], f.c[3], qfma(g.F[4 * i + 2], f.c[2], qfma(g.F[4 * i + 1], f.c[1],
                    qfma(g.F[4 * i], f.c[0], g.c[i]))));
#pragma unroll
        for (int j = 0; j < 4; ++j) g.F[4 * i + j] = r[j];
        g.c[i] = r[4];
    }
}
__device__ __forceinline__ void aff_apply(const Aff& m, const double x[4], double y[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
        y[i] = qfma(m.F[4 * i + 3], x[3], qfma(m.F[4 * i + 2], x[2], qfma(m.F[4 * i + 1], x[1], qfma(m.F[4 * i], x[0], m.c[i]))));
}
__device__ __forceinline__ void aff_identity(Aff& m) {
#pragma unroll
    for (int q = 0; q < 16; ++q) m.F[q] = (q % 5 == 0) ? 1.0 : 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) m.c[q] = 0.0;
}
// closed-loop forward map of a stage: dx -> (A + B K) dx + (B kk + b)
__device__ __forceinline__ void aff_forward(const double a[6], const double B[8], const double bb[4], const double K[8],
                                            const double kk[2], Aff& m) {
    const double Am[4][4] = {{1.0, 0.0, a[0], a[1]}, {0.0, 1.0, a[2], a[3]}, {0.0, 0.0, 1.0, a[4]}, {0.0, 0.0, 0.0, a[5]}};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) m.F[4 * i + q] = qfma(B[2 * i + 1], K[4 + q], qfma(B[2 * i], K[q], Am[i][q]));
        m.c[i] = qfma(B[2 * i + 1], kk[1], qfma(B[2 * i], kk[0], bb[i]));
    }
}
// backward map of the corrector's difference recursion: dp -> (A + B K)' dp + (K' dgu + dgx3 e3)
__device__ __forceinline__ void aff_delta(const double a[6], const double B[8], const double K[8], double dgx3,
                                          const double dgu[2], Aff& m) {
    const double Am[4][4] = {{1.0, 0.0, a[0], a[1]}, {0.0, 1.0, a[2], a[3]}, {0.0, 0.0, 1.0, a[4]}, {0.0, 0.0, 0.0, a[5]}};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) m.F[4 * q + i] = qfma(B[2 * i + 1], K[4 + q], qfma(B[2 * i], K[q], Am[i][q]));
        m.c[i] = qfma(K[4 + i], dgu[1], qfma(K[i], dgu[0], i == 3 ? dgx3 : 0.0));
    }
}

// ---------------------------------- S = 2: the factorisation as an associative scan
// The conditional value-function element of a stage (Sarkka & Garcia-Fernandez, "Temporal
// parallelization of dynamic programming and linear quadratic control", IEEE TAC 2023):
//   e_k = (A, b, C, eta, J) = (A_k, c_k - B Hu^-1 gu, B Hu^-1 B', -gx, diag Hx),
//   e_N = (0, 0, 0, -g_N, We);
// combining e_ij with e_jk (M = (I + C_ij J_jk)^-1):
//   A = A_jk M A_ij, b = A_jk M (b_ij + C_ij eta_jk) + b_jk, C = A_jk M C_ij A_jk' + C_jk,
//   eta = A_ij' M' (eta_jk - J_jk b_ij) + eta_ij, J = A_ij' M' J_jk A_ij + J_ij.
// The suffix product over stages k..N holds the value function of stage k: P_k = J, p_k = -eta.
// (scripts/ubench/riccati_scan_s2.hip: 0.125 ms vs the walk's 0.149 ms per factorisation of the
// configs[4] batch.)
struct VElem { double A[16], b[4], C[10], eta[4], J[10]; };
constexpr int VELEM_N = 44;

__device__ __forceinline__ void velem_stage(const double a[6], const double B[8], const double bb[4], const double Hx[4],
                                            const double Hu[2], const double gx[4], const double gu[2], VElem& e) {
    const double F[16] = {1.0, 0.0, a[0], a[1], 0.0, 1.0, a[2], a[3], 0.0, 0.0, 1.0, a[4], 0.0, 0.0, 0.0, a[5]};
#pragma unroll
    for (int q = 0; q < 16; ++q) e.A[q] = F[q];
    // IEEE division, not rcp: the pivots below are often 1 + tiny, where rcp's refinement of the hardware
    // estimate ends one ulp off the correctly rounded 1/x (scripts/ubench/rcp_check.hip); the division
    // is the correctly rounded 1/x the oracle's rcp computes
    const double ih0 = 1.0 / Hu[0], ih1 = 1.0 / Hu[1];
    const double v0 = ih0 * gu[0], v1 = ih1 * gu[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        e.b[i] = qfma(-B[2 * i + 1], v1, qfma(-B[2 * i], v0, bb[i]));
        e.eta[i] = -gx[i];
        const double w0 = B[2 * i] * ih0, w1 = B[2 * i + 1] * ih1;
#pragma unroll
        for (int j = i; j < 4; ++j) {
            e.C[sidx(i, j)] = qfma(w1, B[2 * j + 1], w0 * B[2 * j]);
            e.J[sidx(i, j)] = (i == j) ? Hx[i] : 0.0;
        }
    }
}
__device__ __forceinline__ void velem_terminal(const double We[4], const double g[6], VElem& e) {
#pragma unroll
    for (int q = 0; q < 16; ++q) e.A[q] = 0.0;
#pragma unroll
    for (int q = 0; q < 10; ++q) { e.C[q] = 0.0; e.J[q] = 0.0; }
#pragma unroll
    for (int q = 0; q < 4; ++q) { e.b[q] = 0.0; e.eta[q] = -g[q]; e.J[sidx(q, q)] = We[q]; }
}
// e <- e (x) f  (e the earlier stages, f the later ones), in place
__device__ __forceinline__ void velem_combine(VElem& e, const VElem& f) {
    // T = I + C_ij J_jk, inverted in place by Gauss-Jordan without pivoting (C, J symmetric positive
    // semidefinite: the eigenvalues of I + C J are >= 1)
    double T[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            T[i][j] = qfma(e.C[sidx(i, 3)], f.J[sidx(3, j)], qfma(e.C[sidx(i, 2)], f.J[sidx(2, j)],
                      qfma(e.C[sidx(i, 1)], f.J[sidx(1, j)], qfma(e.C[sidx(i, 0)], f.J[sidx(0, j)], i == j ? 1.0 : 0.0))));
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const double piv = 1.0 / T[c][c];
        T[c][c] = 1.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) T[c][j] *= piv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            const double fct = T[r][c];
            T[r][c] = 0.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) T[r][j] = qfma(-fct, T[c][j], T[r][j]);
        }
    }
    // TA = A_jk M ; U = A_ij' M'
    double TA[4][4], Um[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            TA[i][j] = qfma(f.A[4 * i + 3], T[3][j], qfma(f.A[4 * i + 2], T[2][j], qfma(f.A[4 * i + 1], T[1][j], f.A[4 * i] * T[0][j])));
            Um[i][j] = qfma(e.A[12 + i], T[j][3], qfma(e.A[8 + i], T[j][2], qfma(e.A[4 + i], T[j][1], e.A[i] * T[j][0])));
        }
    // w = b_ij + C_ij eta_jk ; z = eta_jk - J_jk b_ij
    double w[4], z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        w[i] = qfma(e.C[sidx(i, 3)], f.eta[3], qfma(e.C[sidx(i, 2)], f.eta[2], qfma(e.C[sidx(i, 1)], f.eta[1], qfma(e.C[sidx(i, 0)], f.eta[0], e.b[i]))));
        z[i] = qfma(-f.J[sidx(i, 3)], e.b[3], qfma(-f.J[sidx(i, 2)], e.b[2], qfma(-f.J[sidx(i, 1)], e.b[1], qfma(-f.J[sidx(i, 0)], e.b[0], f.eta[i]))));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        e.b[i] = qfma(TA[i][3], w[3], qfma(TA[i][2], w[2], qfma(TA[i][1], w[1], qfma(TA[i][0], w[0], f.b[i]))));
        e.eta[i] = qfma(Um[i][3], z[3], qfma(Um[i][2], z[2], qfma(Um[i][1], z[1], qfma(Um[i][0], z[0], e.eta[i]))));
    }
    // J = (U J_jk) A_ij + J_ij  (needs the old A_ij: before A is replaced)
    {
        double Y[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                Y[i][j] = qfma(Um[i][3], f.J[sidx(3, j)], qfma(Um[i][2], f.J[sidx(2, j)], qfma(Um[i][1], f.J[sidx(1, j)], Um[i][0] * f.J[sidx(0, j)])));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = i; j < 4; ++j)
                e.J[sidx(i, j)] = qfma(Y[i][3], e.A[12 + j], qfma(Y[i][2], e.A[8 + j], qfma(Y[i][1], e.A[4 + j], qfma(Y[i][0], e.A[j], e.J[sidx(i, j)]))));
    }
    // C = (TA C_ij) A_jk' + C_jk
    {
        double X[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                X[i][j] = qfma(TA[i][3], e.C[sidx(3, j)], qfma(TA[i][2], e.C[sidx(2, j)], qfma(TA[i][1], e.C[sidx(1, j)], TA[i][0] * e.C[sidx(0, j)])));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = i; j < 4; ++j)
                e.C[sidx(i, j)] = qfma(X[i][3], f.A[4 * j + 3], qfma(X[i][2], f.A[4 * j + 2], qfma(X[i][1], f.A[4 * j + 1], qfma(X[i][0], f.A[4 * j], f.C[sidx(i, j)]))));
    }
    // A = TA A_ij, column by column (column j of the result needs column j of A_ij only)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const double c0 = e.A[j], c1 = e.A[4 + j], c2 = e.A[8 + j], c3 = e.A[12 + j];
#pragma unroll
        for (int i = 0; i < 4; ++i) e.A[4 * i + j] = qfma(TA[i][3], c3, qfma(TA[i][2], c2, qfma(TA[i][1], c1, TA[i][0] * c0)));
    }
}
__device__ __forceinline__ void velem_read(const VElem& e, int src, VElem& f) {
    const double* s = &e.A[0];
    double* d = &f.A[0];
#pragma unroll
    for (int q = 0; q < VELEM_N; ++q) d[q] = lane_read(s[q], src);
}

// ------------------------------------------------------------------ QP core
// Barrier terms of slot ls into LDS (predictor): hg[0..2] Hessian additions, hg[3..5]
// gradient additions.  The corrector changes only the gradient (corrector_terms).
template <int S>
__device__ __forceinline__ void barrier_terms(const Ctx& c, const SolveParams& p, const Stage<S>& st, int ls) {
    const int k = kof<S>(c, ls);
    double lo[3], hi[3];
    bnd_lohi<S>(p, st, ls, lo, hi);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool act = bnd_act(c, p, k, j);
        const double ll = st.lm(ls, 2 * j), lh = st.lm(ls, 2 * j + 1);
        const double sl = ll * st.rt(ls, 2 * j), sh = lh * st.rt(ls, 2 * j + 1);
        const double gadd = qfma(-sh, hi[j], -sl * lo[j]) + (lh - ll);
        st.hg(ls, j) = act ? sl + sh : 0.0;
        st.hg(ls, 3 + j) = act ? gadd : 0.0;
    }
}

// The step length is the largest alpha with t + alpha dt >= 0 and l + alpha dl >= 0,
// tracked as a ratio num/den without dividing (den > 0): a candidate t/(-dt) replaces
// num/den when t * den < num * (-dt).
// Affine (predictor) slack/multiplier directions of slot ls from its bounded QP solution
// components (F_VA), unmasked, kept in registers for the rest of the IPM iteration:
// at/al[2j] lower, [2j+1] upper bound of component j.  Also folds the masked directions
// into the step-length ratio num/den.
template <int S>
__device__ __forceinline__ void affine_dirs(const Ctx& c, const SolveParams& p, const Stage<S>& st, int ls,
                                            double at[6], double al[6], double& num, double& den) {
    const int k = kof<S>(c, ls);
    double lo[3], hi[3];
    bnd_lohi<S>(p, st, ls, lo, hi);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool act = bnd_act(c, p, k, j);
        const double tl = st.t(ls, 2 * j), th = st.t(ls, 2 * j + 1);
        const double ll = st.lm(ls, 2 * j), lh = st.lm(ls, 2 * j + 1);
        const double sl = ll * st.rt(ls, 2 * j), sh = lh * st.rt(ls, 2 * j + 1);
        const double v = st.f(F_VA, ls, j);
        at[2 * j] = v - lo[j] - tl;
        at[2 * j + 1] = hi[j] - v - th;
        al[2 * j] = qfma(-sl, at[2 * j], -ll);
        al[2 * j + 1] = qfma(-sh, at[2 * j + 1], -lh);
        const double dtl = act ? at[2 * j] : 0.0, dth = act ? at[2 * j + 1] : 0.0;
        const double dll = act ? al[2 * j] : 0.0, dlh = act ? al[2 * j + 1] : 0.0;
        if (dtl < 0.0 && tl * den < num * -dtl) { num = tl; den = -dtl; }
        if (dth < 0.0 && th * den < num * -dth) { num = th; den = -dth; }
        if (dll < 0.0 && ll * den < num * -dll) { num = ll; den = -dll; }
        if (dlh < 0.0 && lh * den < num * -dlh) { num = lh; den = -dlh; }
    }
}

// Complementarity after the affine step aa (Mehrotra's mu_aff), from the cached directions.
template <int S>
__device__ __forceinline__ double affine_mu_part(const Ctx& c, const SolveParams& p, const Stage<S>& st, int ls,
                                                 const double at[6],
                                                 const double al[6], double aa, double part) {
    const int k = kof<S>(c, ls);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool act = bnd_act(c, p, k, j);
        const double tl = st.t(ls, 2 * j), th = st.t(ls, 2 * j + 1);
        const double ll = st.lm(ls, 2 * j), lh = st.lm(ls, 2 * j + 1);
        const double dtl = act ? at[2 * j] : 0.0, dth = act ? at[2 * j + 1] : 0.0;
        const double dll = act ? al[2 * j] : 0.0, dlh = act ? al[2 * j + 1] : 0.0;
        part = qfma(qfma(aa, dtl, tl), qfma(aa, dll, ll), part);
        part = qfma(qfma(aa, dth, th), qfma(aa, dlh, lh), part);
    }
    return part;
}

// Corrector barrier gradient change of slot ls from the cached affine directions (the
// Hessian is the predictor's): hg[3+j] = c_h / t_h - c_l / t_l, c = sigma mu - dt_aff dl_aff.
template <int S>
__device__ __forceinline__ void corrector_terms(const Ctx& c, const SolveParams& p, const Stage<S>& st, int ls,
                                                const double at[6],
                                                const double al[6], double smu) {
    const int k = kof<S>(c, ls);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool act = bnd_act(c, p, k, j);
        const double cl = qfma(-at[2 * j], al[2 * j], smu), ch = qfma(-at[2 * j + 1], al[2 * j + 1], smu);
        st.hg(ls, 3 + j) = act ? qfma(ch, st.rt(ls, 2 * j + 1), -(cl * st.rt(ls, 2 * j))) : 0.0;
    }
}

// Corrector directions of slot ls (masked) from its bounded QP solution components (F_VN) and
// the cached affine directions; folded into the ratio num/den and kept for the update.
template <int S>
__device__ __forceinline__ void corrector_dirs(const Ctx& c, const SolveParams& p, const Stage<S>& st, int ls,
                                               const double at[6], const double al[6], double smu, double dt[6],
                                               double dl[6], double& num, double& den) {
    const int k = kof<S>(c, ls);
    double lo[3], hi[3];
    bnd_lohi<S>(p, st, ls, lo, hi);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool act = bnd_act(c, p, k, j);
        const double tl = st.t(ls, 2 * j), th = st.t(ls, 2 * j + 1);
        const double ll = st.lm(ls, 2 * j), lh = st.lm(ls, 2 * j + 1);
        const double rtl = st.rt(ls, 2 * j), rth = st.rt(ls, 2 * j + 1);
        const double sl = ll * rtl, sh = lh * rth;
        const double v = st.f(F_VN, ls, j);
        double dtl = v - lo[j] - tl, dth = hi[j] - v - th;
        double dll = qfma(-sl, dtl, -ll), dlh = qfma(-sh, dth, -lh);
        dll = qfma(qfma(-at[2 * j], al[2 * j], smu), rtl, dll);
        dlh = qfma(qfma(-at[2 * j + 1], al[2 * j + 1], smu), rth, dlh);
        dtl = act ? dtl : 0.0; dth = act ? dth : 0.0;
        dll = act ? dll : 0.0; dlh = act ? dlh : 0.0;
        if (dtl < 0.0 && tl * den < num * -dtl) { num = tl; den = -dtl; }
        if (dth < 0.0 && th * den < num * -dth) { num = th; den = -dth; }
        if (dll < 0.0 && ll * den < num * -dll) { num = ll; den = -dll; }
        if (dlh < 0.0 && lh * den < num * -dlh) { num = lh; den = -dlh; }
        dt[2 * j] = dtl; dt[2 * j + 1] = dth;
        dl[2 * j] = dll; dl[2 * j + 1] = dlh;
    }
}

// Step of slot ls: t += alpha dt (and its reciprocal), l += alpha dl.
template <int S>
__device__ __forceinline__ void apply_step(const Stage<S>& st, int ls, const double dt[6], const double dl[6],
                                           double alpha) {
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        const double tn = qfma(alpha, dt[q], st.t(ls, q));
        st.t(ls, q) = tn;
        st.rt(ls, q) = rcp(tn);
        st.lm(ls, q) = qfma(alpha, dl[q], st.lm(ls, q));
    }
}

// Backward pass over the group (factorisation, or the corrector's difference recursion),
// then forward pass writing the bounded components of the solution into LDS field `out`
// (F_VA / F_VN).
template <int S, bool FACTOR, bool ALT = false>
__device__ __forceinline__ void riccati_solve(const Ctx& c, const SolveParams& p, Stage<S>& st, const double dx0[4],
                                              int out, double (&M)[S][16]) {
    SEG_T(t_rs);
    double P[10], pv[4];
#pragma unroll
    for (int i = 0; i < 10; ++i) P[i] = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = 0.0;
    // Branch-free walk: every lane evaluates the step on its own slot data; only the
    // lane whose turn it is (lig == j) keeps its factors, and only its chain value is
    // consumed by the neighbour after the hand-over.  The terminal stage k = N sits in
    // slot N % S of the last lane; the walk starts there.
    const int lsN = c.N - (c.L - 1) * S;
    if (FACTOR) {
#pragma unroll
        for (int ls = 0; ls < S; ++ls)
            if (ls == lsN) ric_terminal(p, st.g[ls], P, pv);
    }   // corrector difference: dp_N = 0
    // the barrier-modified diagonal and gradient entries are fixed during the walk: formed
    // once per slot instead of at every step
    double hx3[S], hu[S][2], gx3[S], gu[S][2];
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        if (FACTOR) {
            hx3[ls] = qfma(p.tau, p.W[3], st.hg(ls, 0));
            hu[ls][0] = qfma(p.tau, p.W[4], st.hg(ls, 1));
            hu[ls][1] = qfma(p.tau, p.W[5], st.hg(ls, 2));
            gx3[ls] = st.g[ls][3] + st.hg(ls, 3);
            gu[ls][0] = st.g[ls][4] + st.hg(ls, 4);
            gu[ls][1] = st.g[ls][5] + st.hg(ls, 5);
        } else {
            gx3[ls] = st.hg(ls, 3);
            gu[ls][0] = st.hg(ls, 4);
            gu[ls][1] = st.hg(ls, 5);
        }
    }
    if constexpr (S == 1 && !FACTOR) {
        // corrector difference walk in closed-loop form: dp_k = e_k + (A + B K)' dp_{k+1} with
        // e = dg_x + K' dg_u (ric_delta_step with dr = dg_u + B' dp substituted), a 4x4 map per
        // step; each lane keeps the dp that reaches it and forms dkk = Rn (dg_u + B' dp)
        // afterwards, in parallel
        const double* K = st.K[0];
        double e[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) e[i] = qfma(K[4 + i], gu[0][1], qfma(K[i], gu[0][0], i == 3 ? gx3[0] : 0.0));
        // Step j runs on lanes lig <= j only: lane j-1 takes lane j's value, while lane j,
        // whose source lane j+1 sits the step out, keeps its old value (a DPP read from a
        // disabled lane returns `old`) — so every lane ends holding the dp that reached it.
        // (step 0 would only form dp_0, which nothing reads: lane 0 holds dp_1 after step 1)
        for (int j = c.L - 2; j >= 1; --j) {
            if (c.lig <= j) {
                double n[4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    n[i] = qfma(M[0][12 + i], pv[3], qfma(M[0][8 + i], pv[2], qfma(M[0][4 + i], pv[1], qfma(M[0][i], pv[0], e[i]))));
#pragma unroll
                for (int i = 0; i < 4; ++i) pv[i] = wave_from_next(pv[i], n[i]);
            }
        }
        const double* dpk = pv;
        if (c.lig < c.N) {
            const double* B = st.B[0];
            const double* Rn = st.Rn[0];
            double rt[2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
                rt[i] = qfma(B[6 + i], dpk[3], qfma(B[4 + i], dpk[2], qfma(B[2 + i], dpk[1], qfma(B[i], dpk[0], gu[0][i]))));
            st.kk[0][0] = qfma(Rn[1], rt[1], qfma(Rn[0], rt[0], st.kk[0][0]));
            st.kk[0][1] = qfma(Rn[2], rt[1], qfma(Rn[1], rt[0], st.kk[0][1]));
        }
    } else if constexpr (S == 2 && !FACTOR) {
        // corrector difference pass as a suffix scan of the lanes' backward maps, dp_N = 0: lane j's
        // map is slot 1's then slot 0's (identity past the horizon); U_j = D_j o D_{j+1} o ...
        const int k0 = 2 * c.lig;
        Aff d;
        {
            Aff m1;
            aff_delta(st.a[0], st.B[0], st.K[0], gx3[0], gu[0], d);
            aff_delta(st.a[1], st.B[1], st.K[1], gx3[1], gu[1], m1);
            if (k0 + 1 < c.N) aff_compose(d, m1);
            else if (!(k0 < c.N)) aff_identity(d);
        }
        for (int off = 1; off < c.L; off <<= 1) {
            const bool take = c.lig + off < c.L;
            Aff f;
            aff_read(d, take ? c.lane + off : c.lane, f);
            if (take) aff_compose(d, f);
        }
        // dp_{2j+2}: the next lane's suffix map applied to dp_N = 0 (its constant); then each slot's
        // dkk from the dp reaching it, slot 1 first (ric_delta_step also steps dp to the slot)
        double pvs[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double nx = wave_from_next(d.c[i]);
            pvs[i] = (c.lig + 1 < c.L) ? nx : 0.0;
        }
#pragma unroll
        for (int ls = 1; ls >= 0; --ls) {
            if (kof<S>(c, ls) < c.N) {
                double dkk[2];
                ric_delta_step(st.a[ls], st.B[ls], gx3[ls], gu[ls], st.K[ls], st.Rn[ls], pvs, dkk);
                st.kk[ls][0] += dkk[0];
                st.kk[ls][1] += dkk[1];
            }
        }
    } else if constexpr (S == 2 && FACTOR && ALT) {
        // factorisation as a suffix scan of the lanes' value-function elements: lane j combines its
        // two stages' elements (slot 0's, then slot 1's; the terminal element where k = N, none past
        // it), Hillis-Steele levels give E_{2j:N}, the next lane's result E_{2j+2:N} gives slot 1's
        // E_{2j+1:N}; then each slot forms K, Rn, kk from its successor's value function
        const int k0 = 2 * c.lig, k1 = k0 + 1;
        VElem e, e1;
        {
            const double Hx0[4] = {p.tau * p.W[0], p.tau * p.W[1], p.tau * p.W[2], hx3[0]};
            const double gxa[4] = {st.g[0][0], st.g[0][1], st.g[0][2], gx3[0]};
            if (k0 < c.N) velem_stage(st.a[0], st.B[0], st.bb[0], Hx0, hu[0], gxa, gu[0], e);
            else velem_terminal(p.We, st.g[0], e);
            const double Hx1[4] = {p.tau * p.W[0], p.tau * p.W[1], p.tau * p.W[2], hx3[1]};
            const double gxb[4] = {st.g[1][0], st.g[1][1], st.g[1][2], gx3[1]};
            if (k1 < c.N) velem_stage(st.a[1], st.B[1], st.bb[1], Hx1, hu[1], gxb, gu[1], e1);
            else velem_terminal(p.We, st.g[1], e1);
            if (k1 <= c.N) {
                VElem t = e1;
                velem_combine(e, t);
            }
        }
        for (int off = 1; off < c.L; off <<= 1) {
            const bool take = c.lig + off < c.L;
            VElem f;
            velem_read(e, take ? c.lane + off : c.lane, f);
            if (take) velem_combine(e, f);
        }
        {
            VElem f;
            velem_read(e, c.lig + 1 < c.L ? c.lane + 1 : c.lane, f);
            if (k1 < c.N) {
                velem_combine(e1, f);
                double Pn[10], pn[4];
#pragma unroll
                for (int q = 0; q < 10; ++q) Pn[q] = f.J[q];
#pragma unroll
                for (int q = 0; q < 4; ++q) pn[q] = -f.eta[q];
                const double gx[4] = {st.g[1][0], st.g[1][1], st.g[1][2], gx3[1]};
                const double Hx[4] = {p.tau * p.W[0], p.tau * p.W[1], p.tau * p.W[2], hx3[1]};
                ric_factor_step(st.a[1], st.B[1], st.bb[1], Hx, hu[1], gx, gu[1], Pn, pn, st.K[1], st.Rn[1], st.kk[1], false);
            }
            if (k0 < c.N) {
                double Pn[10], pn[4];
#pragma unroll
                for (int q = 0; q < 10; ++q) Pn[q] = e1.J[q];
#pragma unroll
                for (int q = 0; q < 4; ++q) pn[q] = -e1.eta[q];
                const double gx[4] = {st.g[0][0], st.g[0][1], st.g[0][2], gx3[0]};
                const double Hx[4] = {p.tau * p.W[0], p.tau * p.W[1], p.tau * p.W[2], hx3[0]};
                ric_factor_step(st.a[0], st.B[0], st.bb[0], Hx, hu[0], gx, gu[0], Pn, pn, st.K[0], st.Rn[0], st.kk[0], false);
            }
        }
    } else if constexpr (S == 1 && FACTOR && ALT) {
        factor_walk_mfma<1>(c, p, st, hx3, hu, gx3, gu);
    } else {
    bool walked = false;
    if constexpr (S == 2 && FACTOR) {
        if (mfw_use(p, 2)) {   // uniform (two stages per lane: ALT is the factorisation scan)
            factor_walk_mfma<2>(c, p, st, hx3, hu, gx3, gu);
            walked = true;
        }
    }
    if (!walked)
    for (int j = c.L - 1; j >= 0; --j) {
        // Lanes above j already hold their final factors and sit the step out (exec
        // mask); lanes below j compute a throw-away step that their own turn overwrites.
        // Writing the factors in place this way needs no per-step selects.
        // The hand-over runs inside the same region: lane j-1 (active) reads lane j (active).
        if (c.lig <= j) {
            double Pc[10], pvc[4];
#pragma unroll
            for (int i = 0; i < 10; ++i) Pc[i] = P[i];
#pragma unroll
            for (int i = 0; i < 4; ++i) pvc[i] = pv[i];
#pragma unroll
            for (int ls = S - 1; ls >= 0; --ls) {
                if (j == c.L - 1 && ls >= lsN) continue;     // terminal / padding slots of the last lane
                if (FACTOR) {
                    const double gx[4] = {st.g[ls][0], st.g[ls][1], st.g[ls][2], gx3[ls]};
                    const double Hx[4] = {p.tau * p.W[0], p.tau * p.W[1], p.tau * p.W[2], hx3[ls]};
                    ric_factor_step(st.a[ls], st.B[ls], st.bb[ls], Hx, hu[ls], gx, gu[ls], Pc, pvc, st.K[ls],
                                    st.Rn[ls], st.kk[ls], j > 0 || ls > 0);
                } else {
                    double dkk[2];
                    ric_delta_step(st.a[ls], st.B[ls], gx3[ls], gu[ls], st.K[ls], st.Rn[ls], pvc, dkk);
                    // in place only on the lane's own turn (a throw-away step must not accumulate)
                    if (c.lig == j) {
                        st.kk[ls][0] += dkk[0];
                        st.kk[ls][1] += dkk[1];
                    }
                }
            }
            // hand-over to lane j-1 (none after step 0: lane 0 reads a disabled lane there).  The
            // first step of a last lane without a stage (lsN == 0) leaves P at the terminal
            // diag(We) every lane already holds, so only p moves then.
            if (j > 0) {
                if (FACTOR && !(j == c.L - 1 && lsN == 0)) {
#pragma unroll
                    for (int i = 0; i < 10; ++i) P[i] = wave_from_next(P[i], Pc[i]);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) pv[i] = wave_from_next(pv[i], pvc[i]);
            }
        }
    }
    }
    SEG_NEXT(FACTOR ? 2 : 6, t_rs);
    if constexpr (S == 1) {
        // forward in closed-loop form: dx_{k+1} = (A + B K) dx_k + (B kk + b), so a step is
        // one 4x4 affine map (16 FMA) instead of du = kk + K dx followed by the dynamics;
        // each lane keeps the dx of its own stage and forms du = kk + K dx afterwards, in
        // parallel.  A + B K is built once per factorisation (the corrector reuses it).
        if (FACTOR) {
            const double* a = st.a[0];
            const double* B = st.B[0];
            const double* K = st.K[0];
            const double Am[4][4] = {{1.0, 0.0, a[0], a[1]}, {0.0, 1.0, a[2], a[3]}, {0.0, 0.0, 1.0, a[4]},
                                     {0.0, 0.0, 0.0, a[5]}};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q) M[0][4 * i + q] = qfma(B[2 * i + 1], K[4 + q], qfma(B[2 * i], K[q], Am[i][q]));
        }
        double cv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) cv[i] = qfma(st.B[0][2 * i + 1], st.kk[0][1], qfma(st.B[0][2 * i], st.kk[0][0], st.bb[0][i]));
        double dx[4] = {dx0[0], dx0[1], dx0[2], dx0[3]};
        // Step j runs on lanes j <= lig < L-1 only (the terminal lane never steps, so the
        // next group's first lane reads a disabled source): lane j+1 takes lane j's value and
        // lane j keeps its own, so every lane ends holding the dx of its stage.
        for (int j = 0; j < c.L - 1; ++j) {
            if (c.lig >= j && c.lig < c.L - 1) {
                double n[4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    n[i] = qfma(M[0][4 * i + 3], dx[3], qfma(M[0][4 * i + 2], dx[2], qfma(M[0][4 * i + 1], dx[1], qfma(M[0][4 * i], dx[0], cv[i]))));
#pragma unroll
                for (int i = 0; i < 4; ++i) dx[i] = wave_from_prev(dx[i], n[i]);
            }
        }
        const double* dxk = dx;
        if (c.lig < c.N) {
            const double* K = st.K[0];
            st.f(out, 0, 0) = dxk[3];
            st.f(out, 0, 1) = qfma(K[3], dxk[3], qfma(K[2], dxk[2], qfma(K[1], dxk[1], qfma(K[0], dxk[0], st.kk[0][0]))));
            st.f(out, 0, 2) = qfma(K[7], dxk[3], qfma(K[6], dxk[2], qfma(K[5], dxk[1], qfma(K[4], dxk[0], st.kk[0][1]))));
        }
        SEG_ADD(FACTOR ? 3 : 7, t_rs);
        return;
    }
    if constexpr (S == 2) {
        // forward pass as a prefix scan of the lanes' closed-loop maps (slot 0's, then slot 1's):
        // T_j = E_j o T_{j-1}; the state entering lane j is T_{j-1}(dx0) (dx0 at lane 0), then
        // slot 0 forms du = kk + K dx and steps the dynamics, slot 1 forms its du
        Aff e;
        {
            Aff m1;
            aff_forward(st.a[0], st.B[0], st.bb[0], st.K[0], st.kk[0], e);
            aff_forward(st.a[1], st.B[1], st.bb[1], st.K[1], st.kk[1], m1);
            aff_compose(m1, e);
            e = m1;
        }
        for (int off = 1; off < c.L; off <<= 1) {
            const bool take = c.lig >= off;
            Aff f;
            aff_read(e, take ? c.lane - off : c.lane, f);
            if (take) aff_compose(e, f);
        }
        double dx[4];
        {
            double y[4];
            aff_apply(e, dx0, y);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double pr = wave_from_prev(y[i]);
                dx[i] = c.lig == 0 ? dx0[i] : pr;
            }
        }
#pragma unroll
        for (int ls = 0; ls < 2; ++ls) {
            double du[2];
            du[0] = qfma(st.K[ls][3], dx[3], qfma(st.K[ls][2], dx[2], qfma(st.K[ls][1], dx[1], qfma(st.K[ls][0], dx[0], st.kk[ls][0]))));
            du[1] = qfma(st.K[ls][7], dx[3], qfma(st.K[ls][6], dx[2], qfma(st.K[ls][5], dx[1], qfma(st.K[ls][4], dx[0], st.kk[ls][1]))));
            if (kof<S>(c, ls) < c.N) {
                st.f(out, ls, 0) = dx[3];
                st.f(out, ls, 1) = du[0];
                st.f(out, ls, 2) = du[1];
            }
            if (ls == 0) dyn_step(st.a[0], st.B[0], st.bb[0], du, dx);
        }
        return;
    }
    // forward: every slot of lanes 0 .. L-2 is a stage k < N; the last lane holds lsN of them
    double dx[4] = {dx0[0], dx0[1], dx0[2], dx0[3]};
    for (int j = 0; j < c.L; ++j) {
        const bool act = (c.lig == j);
#pragma unroll
        for (int ls = 0; ls < S; ++ls) {
            if (j == c.L - 1 && ls >= lsN) continue;
            double du[2];
            du[0] = qfma(st.K[ls][3], dx[3], qfma(st.K[ls][2], dx[2], qfma(st.K[ls][1], dx[1], qfma(st.K[ls][0], dx[0], st.kk[ls][0]))));
            du[1] = qfma(st.K[ls][7], dx[3], qfma(st.K[ls][6], dx[2], qfma(st.K[ls][5], dx[1], qfma(st.K[ls][4], dx[0], st.kk[ls][1]))));
            if (act) {
                st.f(out, ls, 0) = dx[3];
                st.f(out, ls, 1) = du[0];
                st.f(out, ls, 2) = du[1];
            }
            dyn_step(st.a[ls], st.B[ls], st.bb[ls], du, dx);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) dx[i] = wave_from_prev(dx[i]);
    }
}

enum QpExit : int { QP_EXIT_CONV = 0, QP_EXIT_CAP = 1, QP_EXIT_STALL = 2, QP_EXIT_DIVERGED = 3 };

// Mehrotra predictor-corrector IPM on the current linearisation.  Leaves the
// damped control step in LDS (F_DU) and the slacks/multipliers in F_T / F_LM.
// Returns the number of iterations taken by this lane's instance and, in `exit`, why it stopped
// (group-uniform): QP_EXIT_CONV the stop test was met; QP_EXIT_CAP the iteration cap (its last
// iterate is used, as HPIPM's at iter_max); QP_EXIT_STALL the step length stayed below
// qp_stall_alpha for qp_stall_iters iterations (locally infeasible linearisation, HPIPM's
// min-step exit; the last iterate is used as at the cap); QP_EXIT_DIVERGED mu left
// [0, qp_mu_max) (multipliers growing without bound, or non-finite): a QP failure (acados
// ACADOS_QP_FAILURE, status 4), stopped while its iterate is still finite.  A stopped instance's
// state is frozen while the rest of its wave iterates (no update with alpha = 0, which would turn
// an infinite direction into NaN).
//
// Stop test (HPIPM's four exit residuals, ocp_qp_ipm): complementarity mu < mu_stop, bound
// residual < res_stop, stationarity < qp_tol_stat, equality < qp_tol_eq.  The three linear
// residuals are those of the IPM iterate (z, pi, lam, t) with start z = 0, pi = 0, lam =
// mu0 / t: every Newton step solves them exactly and the update scales all of them by
// (1 - alpha), so each is its start value times prod(1 - alpha) (tracked, not recomputed:
// r0 = bound residual of the floored slacks, rg0 = max|g + C' lam|, rb0 = max(|dx0|, |b|)); the
// test r * prod < tol is applied as prod < min(tol / r) over the three.
template <int S, bool ALT = false>
__device__ int qp_ipm(const Ctx& c, const SolveParams& p, Stage<S>& st, const double dx0[4], int& exit,
                      bool skip = false) {
    SEG_T(t_ipm);
    const double m = 2.0 * (3.0 * c.N - (p.s0_bound ? 0.0 : 1.0));
    // initial point.  r0 = largest bound residual of the infeasible start (t - d where the
    // slack had to be floored at t_min); every update scales all residuals by (1 - alpha)
    double r0 = 0.0, rg0 = 0.0, rb0 = 0.0;
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        double lo[3], hi[3];
        bnd_lohi<S>(p, st, ls, lo, hi);
        double gl[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const bool act = bnd_act(c, p, k, j);
            const double tl = fmax(-lo[j], p.t_min), th = fmax(hi[j], p.t_min);
            if (act) r0 = fmax(r0, fmax(tl + lo[j], th - hi[j]));
            const double rl = rcp(tl), rh = rcp(th);
            st.t(ls, 2 * j) = act ? tl : 1.0;
            st.t(ls, 2 * j + 1) = act ? th : 1.0;
            st.rt(ls, 2 * j) = act ? rl : 1.0;
            st.rt(ls, 2 * j + 1) = act ? rh : 1.0;
            st.lm(ls, 2 * j) = act ? p.mu0 * rl : 0.0;
            st.lm(ls, 2 * j + 1) = act ? p.mu0 * rh : 0.0;
            gl[j] = act ? qfma(p.mu0, rh, -(p.mu0 * rl)) : 0.0;
        }
        // start-point stationarity g + C' lam (bounded components s, u_n, u_t) and equality
        // (defects; x0 on the first stage); the padding slots past the terminal stage hold zeros
        if (k <= c.N) {
            rg0 = fmax(rg0, fmax(fmax(fabs(st.g[ls][0]), fabs(st.g[ls][1])), fmax(fabs(st.g[ls][2]), fabs(st.g[ls][3] + gl[0]))));
            rg0 = fmax(rg0, fmax(fabs(st.g[ls][4] + gl[1]), fabs(st.g[ls][5] + gl[2])));
            rb0 = fmax(rb0, fmax(fmax(fabs(st.bb[ls][0]), fabs(st.bb[ls][1])), fmax(fabs(st.bb[ls][2]), fabs(st.bb[ls][3]))));
            if (k == 0) rb0 = fmax(rb0, fmax(fmax(fabs(dx0[0]), fabs(dx0[1])), fmax(fabs(dx0[2]), fabs(dx0[3]))));
        }
        st.du(ls, 0) = 0.0;
        st.du(ls, 1) = 0.0;
        // the forward walks never write the terminal / padding slots: define them, so no
        // stale LDS content (another block's data, possibly NaN bit patterns) is ever read
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            st.f(F_VA, ls, q) = 0.0;
            st.f(F_VN, ls, q) = 0.0;
        }
    }
    // the three linear residuals share the scale prod(1 - alpha): one threshold on it
    // (x / 0 = inf: a residual that starts at zero never binds)
    double rs_stop = p.res_stop / group_max(r0, c.gs);
    const double rs_g = p.qp_tol_stat / group_max(rg0, c.gs), rs_b = p.qp_tol_eq / group_max(rb0, c.gs);
    // a NaN start residual compares false here and leaves rs_stop as it was (the fmax accumulation
    // above drops NaN anyway); a NaN QP is caught by the divergence exit (NaN mu) or the non-finite
    // solution check after the loop, not by this threshold
    rs_stop = rs_g < rs_stop ? rs_g : rs_stop;
    rs_stop = rs_b < rs_stop ? rs_b : rs_stop;
    double rscale = 1.0;
    int nit = 0, stall = 0;
    bool conv = false, stalled = false, div = false;
    SEG_ADD(13, t_ipm);
    for (int it = 0;; ++it) {
        SEG_T(t_seg);
        double tl_sum = 0.0;
#pragma unroll
        for (int ls = 0; ls < S; ++ls)
#pragma unroll
            for (int q = 0; q < 6; ++q) tl_sum = qfma(st.t(ls, q), st.lm(ls, q), tl_sum);
        const double mu = group_sum(tl_sum, c.gs) / m;
        // divergence first (mu non-finite or past qp_mu_max: a NaN mu would pass the stop test),
        // then the stop test, then the stall exit (locally infeasible QP: the step length stays
        // tiny while mu grows)
        div = !skip && !(mu < p.qp_mu_max);
        conv = !div && (skip || (!(mu >= p.mu_stop) && !(rscale >= rs_stop)));
        stalled = !conv && !div && p.qp_stall_iters > 0 && stall >= p.qp_stall_iters;
        const bool done = conv || div || stalled;
        // the cap is tested after the last step too (conv reports it), then the loop ends
        if (it == p.qp_iters || __ballot(!done) == 0ull) break;
        nit += done ? 0 : 1;
#ifdef QSP_SEGSTAMP
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_seg[31], 1ull);
#endif
        SEG_NEXT(0, t_seg);
        // ---- predictor
#pragma unroll
        for (int ls = 0; ls < S; ++ls) barrier_terms<S>(c, p, st, ls);
        SEG_NEXT(1, t_seg);
        double M[S][16];   // closed-loop matrices A + B K (S = 1), shared by both forward walks
        riccati_solve<S, true, ALT>(c, p, st, dx0, F_VA, M);
        SEG_T(t_seg2);
        // affine directions: computed once, kept in registers through the corrector
        double at[S][6], al[S][6];
        double num = 1.0, den = 1.0;
#pragma unroll
        for (int ls = 0; ls < S; ++ls) affine_dirs<S>(c, p, st, ls, at[ls], al[ls], num, den);
        const double aa = group_min(num / den, c.gs);
        double ma = 0.0;
#pragma unroll
        for (int ls = 0; ls < S; ++ls) ma = affine_mu_part<S>(c, p, st, ls, at[ls], al[ls], aa, ma);
        const double mua = group_sum(ma, c.gs) / m;
        const double r = mua / mu;
        const double sg = fmax(r * r * r, p.sigma_min);
        const double smu = sg * mu;
        SEG_NEXT(4, t_seg2);
        // ---- corrector
#pragma unroll
        for (int ls = 0; ls < S; ++ls) corrector_terms<S>(c, p, st, ls, at[ls], al[ls], smu);
        SEG_ADD(5, t_seg2);
        riccati_solve<S, false, ALT>(c, p, st, dx0, F_VN, M);
        SEG_T(t_seg3);
        double dt[S][6], dl[S][6];
        num = 1.0; den = p.frac;       // initial bound 1/frac
#pragma unroll
        for (int ls = 0; ls < S; ++ls) corrector_dirs<S>(c, p, st, ls, at[ls], al[ls], smu, dt[ls], dl[ls], num, den);
        double alpha = p.frac * group_min(num / den, c.gs);
        alpha = fmin(alpha, 1.0);
        // a finished instance sits the rest of the wave's loop out with its state frozen
        if (!done) {
            stall = alpha < p.qp_stall_alpha ? stall + 1 : 0;
            rscale *= 1.0 - alpha;
#pragma unroll
            for (int ls = 0; ls < S; ++ls) {
                apply_step<S>(st, ls, dt[ls], dl[ls], alpha);
                st.du(ls, 0) = qfma(alpha, st.f(F_VN, ls, 1) - st.du(ls, 0), st.du(ls, 0));
                st.du(ls, 1) = qfma(alpha, st.f(F_VN, ls, 2) - st.du(ls, 1), st.du(ls, 1));
            }
        }
        SEG_ADD(8, t_seg3);
    }
    exit = conv ? QP_EXIT_CONV : (div ? QP_EXIT_DIVERGED : (stalled ? QP_EXIT_STALL : QP_EXIT_CAP));
    return nit;
}

// State step of the damped QP solution (rollout of the affine dynamics), into LDS F_DX.
template <int S>
__device__ __forceinline__ void qp_rollout(const Ctx& c, Stage<S>& st, const double dx0[4]) {
    double dx[4] = {dx0[0], dx0[1], dx0[2], dx0[3]};
    for (int j = 0; j < c.L; ++j) {
        if (c.lig == j) {
#pragma unroll
            for (int ls = 0; ls < S; ++ls) {
                const int k = j * S + ls;
                if (k <= c.N) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) st.dxs(ls, i) = dx[i];
                }
                if (k < c.N) {
                    const double du[2] = {st.du(ls, 0), st.du(ls, 1)};
                    dyn_step(st.a[ls], st.B[ls], st.bb[ls], du, dx);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) dx[i] = wave_from_prev(dx[i]);
    }
}

// One step of the adjoint recursion  pi_{k-1} = Hx dx_k + gx_k + A_k' pi_k + (lam_hi - lam_lo)_s
__device__ __forceinline__ void adjoint_step(const SolveParams& p, const double a[6], const double dx[4],
                                             const double g[6], double dlam_s, double pi[4]) {
    double np[4];
    np[0] = qfma(p.tau * p.W[0], dx[0], g[0]) + pi[0];
    np[1] = qfma(p.tau * p.W[1], dx[1], g[1]) + pi[1];
    np[2] = qfma(p.tau * p.W[2], dx[2], g[2]) + (qfma(a[2], pi[1], a[0] * pi[0]) + pi[2]);
    np[3] = qfma(p.tau * p.W[3], dx[3], g[3]) + qfma(a[5], pi[3], qfma(a[4], pi[2], qfma(a[3], pi[1], a[1] * pi[0])));
    np[3] += dlam_s;
#pragma unroll
    for (int i = 0; i < 4; ++i) pi[i] = np[i];
}

// Dynamics multipliers by the adjoint recursion; writes PI (B x N x 4).
//   pi_{N-1} = We dx_N + g_N ; pi_{k-1} = Hx dx_k + gx_k + A_k' pi_k + (lam_hi - lam_lo)_s
template <int S>
__device__ __forceinline__ void qp_adjoint_store(const Ctx& c, const SolveParams& p, const Stage<S>& st,
                                                 double* PI, bool write, bool shift) {
    double pi[4] = {0, 0, 0, 0};
    for (int j = c.L - 1; j >= 0; --j) {
        if (c.lig == j) {
#pragma unroll
            for (int ls = S - 1; ls >= 0; --ls) {
                const int k = j * S + ls;
                if (k == c.N) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) pi[i] = qfma(p.We[i], st.dxs(ls, i), st.g[ls][i]);
                } else if (k < c.N) {
                    if (write && (!shift || k >= 1)) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) PI[(size_t)(shift ? k - 1 : k) * 4 + i] = pi[i];
                    }
                    if (write && shift && k == c.N - 1) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) PI[(size_t)k * 4 + i] = pi[i];
                    }
                    if (k >= 1) {
                        const double dxk[4] = {st.dxs(ls, 0), st.dxs(ls, 1), st.dxs(ls, 2), st.dxs(ls, 3)};
                        adjoint_step(p, st.a[ls], dxk, st.g[ls], st.lm(ls, 1) - st.lm(ls, 0), pi);
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) pi[i] = wave_from_next(pi[i]);
    }
}

// ------------------------------------------------------------------ kernels
// One solve = prologue, K x (linearize, qp), epilogue; all on one stream.
// Workspace (SolveArgs::w*): SQP iterate X/U, wrapped x0, stage data in SoA.
enum LinField : int { L_A = 0, L_B = 6, L_BB = 14, L_G = 18, L_COUNT = 24 };

// Shape of instance i.  Ids from qsp_solve_device are device data that the host cannot
// validate without a round trip, so they are clamped into the table here.
__device__ __forceinline__ const ShapeDev& shape_of(const SolveArgs& A, int i) {
    const int id = A.shape_id ? A.shape_id[i] : 0;
    return A.shapes[id < 0 ? 0 : (id >= A.n_shapes ? A.n_shapes - 1 : id)];
}

// nlp_mode 1 workspace (SoA over (instance, stage), like wlin)
enum NlpField : int { W_PI = 0, W_LAM = 4, W_NU = 10, W_ETA = 14, W_COUNT = 20 };

// NLP multipliers and merit weights at the start of a solve (oracle sqp_solve: PI from the
// initial guess, LAM and the weights zero).
__device__ __forceinline__ void nlp_init(const SolveArgs& A, int i, bool use_pi) {
    const int N = A.p.N;
    const size_t tot = (size_t)A.B * (N + 1);
    for (int k = 0; k <= N; ++k) {
        const size_t si = (size_t)i * (N + 1) + k;
        for (int q = 0; q < 4; ++q)
            A.wnlp[(W_PI + q) * tot + si] = (use_pi && A.PI_in && k < N) ? A.PI_in[((size_t)i * N + k) * 4 + q] : 0.0;
        for (int q = W_LAM; q < W_COUNT; ++q) A.wnlp[q * tot + si] = 0.0;
    }
    A.wdone[i] = 0;
    if (A.wres)
        for (int q = 0; q < 4; ++q) A.wres[(size_t)i * 4 + q] = 0.0;
}

// With the stage-0 s bound in the QP (stage0_s_bound), s_0 = x0's s is a fixed quantity of
// every QP: outside [lh_s, uh_s] every QP of the solve is infeasible.  The instance then does
// not iterate (wdone = 3: status QSP_STATUS_QP_FAIL, sqp_iter 0, the initial guess returned),
// as the oracle's sqp_solve.  (Called after nlp_init, which clears wdone.)
__device__ __forceinline__ void s0_feasible(const SolveArgs& A, int i, double s0) {
    const SolveParams& p = A.p;
    if (p.s0_bound && A.wdone && !(s0 >= p.lh[0] && s0 <= p.uh[0])) {
        A.wdone[i] = 3;
        A.sqp_iter[i] = 0;
    }
}

// NMPC_controller.solve prologue (NMPC_controller.m:332-384) or acados-level init copy.
__global__ void prologue_kernel(SolveArgs A) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.B) return;
    const SolveParams& p = A.p;
    const int N = p.N;
    const ShapeDev& sh = shape_of(A, i);
    double x0[4];
    for (int c = 0; c < 4; ++c) x0[c] = A.x0[(size_t)i * 4 + c];
    double* X = A.wX + (size_t)i * (N + 1) * 4;
    double* U = A.wU + (size_t)i * N * 2;
    A.qp_iter[i] = 0;
    if (A.qp_capped) A.qp_capped[i] = 0;
    if (A.qp_stalled) A.qp_stalled[i] = 0;
    if (A.wdone) A.wdone[i] = 0;
    if (A.wnit) A.wnit[i] = 0;
    if (!(A.flags & QSP_FLAG_CONTROLLER)) {
        for (int q = 0; q < (N + 1) * 4; ++q) X[q] = A.X_in[(size_t)i * (N + 1) * 4 + q];
        for (int q = 0; q < N * 2; ++q) U[q] = A.U_in[(size_t)i * N * 2 + q];
        for (int c = 0; c < 4; ++c) A.wx0[(size_t)i * 4 + c] = x0[c];
        if (p.nlp_mode == 1) nlp_init(A, i, true);
        s0_feasible(A, i, x0[3]);
        return;
    }
    x0[3] = qfma(-sh.b, (x0[3] < 0.0) ? 1.0 : 0.0, mat_mod(x0[3], sh.b));   // :332
    for (int c = 0; c < 4; ++c) A.wx0[(size_t)i * 4 + c] = x0[c];
    const bool cold = (A.warm_valid == nullptr || A.warm_valid[i] == 0);
    if (p.nlp_mode == 1) nlp_init(A, i, !cold);                             // :351-355 (PI = 0 cold)
    for (int k = 0; k < N; ++k) {                                            // :351-355
        U[2 * k] = cold ? p.cp.u_n_lb : A.U_in[((size_t)i * N + k) * 2];
        U[2 * k + 1] = cold ? 0.0 : A.U_in[((size_t)i * N + k) * 2 + 1];
    }
    double xc[4] = {x0[0], x0[1], x0[2], x0[3]};
    for (int k = 0; k <= N; ++k) {                                           // :357-380
        for (int c = 0; c < 4; ++c) X[4 * k + c] = xc[c];
        if (k == N) break;
        const double vb = v_bound(sh, p.cp, xc[3]);
        const double ut_old = U[2 * k + 1];
        if (fabs(ut_old) > vb) {
            const double sgn = ut_old > 0.0 ? 1.0 : -1.0;
            U[2 * k + 1] = sgn * vb;
            U[2 * k] = U[2 * k + 1] * U[2 * k] / ut_old;
        }
        DynOut d;
        dynamics<false>(sh, xc[2], xc[3], U[2 * k], U[2 * k + 1], d);
        for (int c = 0; c < 4; ++c) xc[c] = qfma(p.Ts, d.f[c], xc[c]);
    }
    s0_feasible(A, i, x0[3]);
}

// The QP of one SQP iteration in the register/LDS-resident lane-group layout:
// load stage data, Mehrotra IPM, roll out the damped step, update the SQP iterate.
// Dynamics multipliers of the QP solution, one per stage lane (S = 1): lane k < N
// returns pi_k (same adjoint recursion as qp_adjoint_store).
__device__ __forceinline__ void qp_adjoint_lane(const Ctx& c, const SolveParams& p, const Stage<1>& st,
                                                double piq[4]) {
    double pi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; ++i) piq[i] = 0.0;
    for (int j = c.L - 1; j >= 0; --j) {
        if (c.lig == j) {
            if (j == c.N) {
#pragma unroll
                for (int i = 0; i < 4; ++i) pi[i] = qfma(p.We[i], st.dxs(0, i), st.g[0][i]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) piq[i] = pi[i];
                if (j >= 1) {
                    const double dxk[4] = {st.dxs(0, 0), st.dxs(0, 1), st.dxs(0, 2), st.dxs(0, 3)};
                    adjoint_step(p, st.a[0], dxk, st.g[0], st.lm(0, 1) - st.lm(0, 0), pi);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) pi[i] = wave_from_next(pi[i]);
    }
}

// l1 merit contribution of stage k (oracle merit_eval): stage cost, nu'|defect|,
// eta'(bound violation) on (s_k, u_n, u_t); the terminal lane adds the terminal cost.
__device__ __forceinline__ double merit_stage(const SolveParams& p, int k, const double x[4], const double u[2],
                                              const double* yr, const double* ye, const double def[4],
                                              const double nu[4], const double eta[6]) {
    if (k == p.N) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) { const double r = x[i] - ye[i]; s = qfma(p.We[i] * r, r, s); }
        return 0.5 * s;
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) { const double r = x[i] - yr[i]; s = qfma(p.W[i] * r, r, s); }
#pragma unroll
    for (int i = 0; i < 2; ++i) { const double r = u[i] - yr[4 + i]; s = qfma(p.W[4 + i] * r, r, s); }
    double ph = 0.5 * p.tau * s;
#pragma unroll
    for (int i = 0; i < 4; ++i) ph = qfma(nu[i], fabs(def[i]), ph);
    const double v[3] = {x[3], u[0], u[1]};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (j == 0 && k == 0 && !p.s0_bound) continue;
        const double vl = p.lh[j] - v[j], vh = v[j] - p.uh[j];
        if (vl > 0.0) ph = qfma(eta[2 * j], vl, ph);
        if (vh > 0.0) ph = qfma(eta[2 * j + 1], vh, ph);
    }
    return ph;
}

// ------------------------------------------------------------------ nlp_mode 1
// acados 'SQP' + 'merit_backtracking' (NMPC_controller.m:271-276), restated in the
// oracle's sqp_solve.  One SQP iteration = linearize, qp_step<1, true> (KKT test of the
// current iterate -> converged instances freeze; QP; its solution into wqp), and
// merit_ls_kernel (merit weights from the QP multipliers, Armijo backtracking on the l1
// merit function, damped multiplier update).  One stage per lane: lane k of a group owns
// stage k, every per-stage term is lane-parallel, horizon sums/maxima are group reductions.
enum QpField : int { Q_DX = 0, Q_DU = 4, Q_PI = 6, Q_LAM = 10, Q_COUNT = 16 };

// KKT residuals of the NLP at the current iterate against tol_* (max norms over the
// horizon); `nlp` points at this lane's stage in the W_* SoA (stride tot).  res (the instance's
// 4 doubles, or nullptr): the residuals are recorded there (acados' res_stat/eq/ineq/comp
// statistics of the last test, qsp_get_residuals).
__device__ bool nlp_converged(const Ctx& c, const SolveParams& p, const Stage<1>& st, const double* nlp, size_t tot,
                              double* res) {
    const int N = p.N;
    const int k = c.lig;
    const bool stg = k < N;
    double PIk[4], LAMk[6];
#pragma unroll
    for (int q = 0; q < 4; ++q) PIk[q] = nlp[(W_PI + q) * tot];
#pragma unroll
    for (int q = 0; q < 6; ++q) LAMk[q] = nlp[(W_LAM + q) * tot];
    double PIp[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) PIp[q] = wave_from_prev(PIk[q]);   // pi_{k-1}
    double rs = 0.0, re = 0.0, ri = 0.0, rc = 0.0;
    if (stg) {
        const double* B = st.B[0];
        const double* a = st.a[0];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const double r = (st.g[0][4 + i] + qfma(B[6 + i], PIk[3], qfma(B[4 + i], PIk[2], qfma(B[2 + i], PIk[1], B[i] * PIk[0])))) +
                             (LAMk[2 * (1 + i) + 1] - LAMk[2 * (1 + i)]);
            rs = fmax(rs, fabs(r));
        }
        if (k >= 1) {
            const double at[4] = {PIk[0], PIk[1], qfma(a[2], PIk[1], a[0] * PIk[0]) + PIk[2],
                                  qfma(a[5], PIk[3], qfma(a[4], PIk[2], qfma(a[3], PIk[1], a[1] * PIk[0])))};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                double r = st.g[0][i] - PIp[i] + at[i];
                if (i == 3) r += LAMk[1] - LAMk[0];
                rs = fmax(rs, fabs(r));
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) re = fmax(re, fabs(st.bb[0][i]));
        const double v[3] = {st.v(0, 0), st.v(0, 1), st.v(0, 2)};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (j == 0 && k == 0 && !p.s0_bound) continue;
            const double sl = v[j] - p.lh[j], sh_ = p.uh[j] - v[j];
            ri = fmax(ri, fmax(-sl, -sh_));
            rc = fmax(rc, fmax(fabs(LAMk[2 * j] * sl), fabs(LAMk[2 * j + 1] * sh_)));
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) rs = fmax(rs, fabs(st.g[0][i] - PIp[i]));
    }
    rs = group_max(rs, c.gs);
    re = group_max(re, c.gs);
    ri = group_max(ri, c.gs);
    rc = group_max(rc, c.gs);
    if (res && c.real && c.lig == 0) {
        res[0] = rs;
        res[1] = re;
        res[2] = ri;
        res[3] = rc;
    }
    return rs < p.tol_stat && re < p.tol_eq && ri < p.tol_ineq && rc < p.tol_comp;
}

// The SQP's reaction to a QP's exit (both SQP kernels): counts of capped and stalled QPs; a
// diverged QP (status 4, acados ACADOS_QP_FAILURE) or a non-finite solution (status 1) stops the
// instance's SQP with its last iterate, as the oracle's sqp_solve does.  Returns that failure.
template <int S>
__device__ __forceinline__ bool qp_outcome(const SolveArgs& A, const Ctx& c, const Stage<S>& st, int iv, int it,
                                           int exit, bool skip) {
    const int N = c.N;
    if (c.real && c.lig == 0 && !skip) {
        if (A.qp_capped && exit == QP_EXIT_CAP) A.qp_capped[iv] += 1;
        if (A.qp_stalled && exit == QP_EXIT_STALL) A.qp_stalled[iv] += 1;
    }
    if (!A.wdone) return false;
    double bad = 0.0;
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
#pragma unroll
        for (int q = 0; q < 4; ++q) bad = (k > N || isfinite(st.dxs(ls, q))) ? bad : 1.0;
        bad = (k >= N || (isfinite(st.du(ls, 0)) && isfinite(st.du(ls, 1)))) ? bad : 1.0;
    }
    const double badg = group_max(bad, c.gs);   // every lane takes part in the DPP scan
    const bool div = exit == QP_EXIT_DIVERGED;
    const bool failed = !skip && (div || badg > 0.0);
    if (failed && c.real && c.lig == 0) {
        A.wdone[iv] = div ? 4 : 2;
        A.sqp_iter[iv] = it;
    }
    return failed;
}

template <int S, bool MERIT = false, bool LIN = false, bool ALT = false>
__global__ void __launch_bounds__(BLOCK, QSP_MIN_WAVES) qp_step_kernel(SolveArgs A, int it) {
    SEG_T(t_k);
    extern __shared__ double smem[];
    const SolveParams& p = A.p;
    Ctx c;
    c.lane = threadIdx.x & 63;
    c.N = p.N;
    c.L = (p.N + S) / S;                 // ceil((N+1)/S)
    const int G = 64 / c.L;
    c.grp = c.lane / c.L;
    c.lig = c.lane - c.grp * c.L;
    c.base = c.grp * c.L;
    c.gs.init(c.base, c.L);
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    c.inst = wave * G + c.grp;
    c.real = (c.grp < G) && (c.inst < A.nI);
    // instances are packed into waves in the order of their previous IPM iteration count
    // (sort_by_iters_kernel), so the instances sharing a wave finish together
    const int slot = A.i0 + (c.real ? c.inst : A.nI - 1);
    const int iv = A.wperm ? A.wperm[slot] : slot;
    const int N = p.N;
    const size_t tot = (size_t)A.B * (N + 1);
    Stage<S> st;
    st.lds = smem + threadIdx.x;
    if (A.flags & QSP_FLAG_POISON) {
        for (int f = 0; f < F_COUNT * S + mfw_extra<S>(); ++f) st.lds[f * BLOCK] = __builtin_nan("");
    }
    double* X = A.wX + (size_t)iv * (N + 1) * 4;
    double* U = A.wU + (size_t)iv * N * 2;
    // frozen instances (converged in nlp_mode 1, or a failed QP earlier) are not iterated
    const bool was_done = A.wdone && A.wdone[iv] != 0;
    const bool lin_live = c.real && !was_done;   // fused linearisation only where it is used
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        const int kc = k <= N ? k : N;
        const int ku = k < N ? k : N - 1;
        if constexpr (LIN) {
            // the SQP iteration's linearisation, one stage per slot (RK4 + sensitivities): the
            // stage data stays in registers instead of a 24-double HBM round trip
            if (kc < N && lin_live) {
                const double xk[4] = {X[4 * kc], X[4 * kc + 1], X[4 * kc + 2], X[4 * kc + 3]};
                const double uk[2] = {U[2 * kc], U[2 * kc + 1]};
#ifdef QSP_SEGSTAMP
                {   // (diagnostic build: the iterate's loads complete before the stamp)
                    double w = xk[0] + xk[1] + xk[2] + xk[3] + uk[0] + uk[1];
                    asm volatile("" : "+v"(w));
                    SEG_NEXT(14, t_k);
                }
#endif
                Lin Ln;
                rk4<true>(shape_of(A, iv), p.Ts, xk, uk, Ln);
#ifdef QSP_SEGSTAMP
                {
                    double w = Ln.a[0] + Ln.B[0] + Ln.xn[0];
                    asm volatile("" : "+v"(w));
                    SEG_NEXT(15, t_k);
                }
#endif
                const double* yr = A.yref + ((size_t)iv * N + kc) * 6;
#pragma unroll
                for (int q = 0; q < 6; ++q) st.a[ls][q] = Ln.a[q];
#pragma unroll
                for (int q = 0; q < 8; ++q) st.B[ls][q] = Ln.B[q];
#pragma unroll
                for (int q = 0; q < 4; ++q) st.bb[ls][q] = Ln.xn[q] - X[4 * (kc + 1) + q];
#pragma unroll
                for (int q = 0; q < 4; ++q) st.g[ls][q] = p.tau * p.W[q] * (xk[q] - yr[q]);
#pragma unroll
                for (int q = 0; q < 2; ++q) st.g[ls][4 + q] = p.tau * p.W[4 + q] * (uk[q] - yr[4 + q]);
            } else {   // terminal stage (or an instance that does not iterate): no dynamics
                const double* ye = A.yref_e + (size_t)iv * 4;
#pragma unroll
                for (int q = 0; q < 6; ++q) st.a[ls][q] = 0.0;
#pragma unroll
                for (int q = 0; q < 8; ++q) st.B[ls][q] = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) st.bb[ls][q] = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) st.g[ls][q] = p.We[q] * (X[4 * N + q] - ye[q]);
                st.g[ls][4] = 0.0;
                st.g[ls][5] = 0.0;
            }
        } else {
            const double* in = A.wlin + (size_t)iv * (N + 1) + kc;
#pragma unroll
            for (int q = 0; q < 6; ++q) st.a[ls][q] = in[(L_A + q) * tot];
#pragma unroll
            for (int q = 0; q < 8; ++q) st.B[ls][q] = in[(L_B + q) * tot];
#pragma unroll
            for (int q = 0; q < 4; ++q) st.bb[ls][q] = in[(L_BB + q) * tot];
#pragma unroll
            for (int q = 0; q < 6; ++q) st.g[ls][q] = in[(L_G + q) * tot];
        }
        st.v(ls, 0) = X[4 * kc + 3];
        st.v(ls, 1) = U[2 * ku];
        st.v(ls, 2) = U[2 * ku + 1];
    }
    if constexpr (MERIT && LIN) {
        // the line search (merit_ls_kernel) evaluates the defect and gradient at the same point
        if (lin_live && c.lig <= N) {
            double* out = A.wlin + (size_t)iv * (N + 1) + c.lig;
#pragma unroll
            for (int q = 0; q < 4; ++q) out[(L_BB + q) * tot] = st.bb[0][q];
#pragma unroll
            for (int q = 0; q < 6; ++q) out[(L_G + q) * tot] = st.g[0][q];
        }
    }
    double dx0[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) dx0[q] = A.wx0[(size_t)iv * 4 + q] - X[q];   // used by lane lig == 0
    // padding lanes (no instance) must not hold their wave in the IPM loop: they mirror
    // instance B-1 with group reductions over foreign lanes and need not converge
    bool skip = was_done || !c.real;
    if constexpr (MERIT) {
        static_assert(S == 1, "nlp_mode 1 uses one stage per lane");
        // nlp_mode 1: KKT test of the current iterate; converged instances freeze
        const bool conv = !was_done && nlp_converged(c, p, st, A.wnlp + (size_t)iv * (N + 1) + c.lig, tot,
                                                     A.wres ? A.wres + (size_t)iv * 4 : nullptr);
        skip = was_done || conv || !c.real;
        if (conv && c.real && c.lig == 0) {
            A.wdone[iv] = 1;
            A.sqp_iter[iv] = it;
        }
    }
    int exit;
    SEG_NEXT(10, t_k);
    const int nit = qp_ipm<S, ALT>(c, p, st, dx0, exit, skip);
    SEG_NEXT(11, t_k);
    qp_rollout<S>(c, st, dx0);
    const bool failed = qp_outcome<S>(A, c, st, iv, it, exit, skip);
    if (A.wnit && c.real && c.lig == 0) {
        // wave-packing record and key of this instance for the next launch
        // (sort_by_iters_kernel); an instance that did not iterate keeps its record
        const int old = A.wnit[iv];
        const int rec = (MERIT || !(skip || failed)) ? pack_record(old, nit) : old;
        A.wnit[iv] = rec;
        if (A.whist) atomicAdd(&A.whist[(it & 1) * PACK_KEYS_MAX + pack_key(rec, pack_maxkey(p.qp_iters))], 1);
    }
    if constexpr (MERIT) {
        // QP solution (step, dynamics and bound multipliers) for the line-search kernel
        double piq[4];
        qp_adjoint_lane(c, p, st, piq);
        if (c.real && !skip && !failed) {
            const size_t si = (size_t)iv * (N + 1) + c.lig;
            double* w = A.wqp + si;
#pragma unroll
            for (int q = 0; q < 4; ++q) w[(Q_DX + q) * tot] = st.dxs(0, q);
#pragma unroll
            for (int q = 0; q < 2; ++q) w[(Q_DU + q) * tot] = c.lig < N ? st.du(0, q) : 0.0;
#pragma unroll
            for (int q = 0; q < 4; ++q) w[(Q_PI + q) * tot] = piq[q];
#pragma unroll
            for (int q = 0; q < 6; ++q) w[(Q_LAM + q) * tot] = c.lig < N ? st.lm(0, q) : 0.0;
        }
        if (c.real && c.lig == 0) A.qp_iter[iv] += nit;
        return;
    }
    const bool last = it + 1 >= p.sqp_iters;
    if (A.qp_dx) {
        // QP-level interface (qsp_qp_solve): report the QP solution itself
        if (last) qp_adjoint_store<S>(c, p, st, A.PI_out + (size_t)iv * N * 4, c.real, false);
        if (!c.real) return;
#pragma unroll
        for (int ls = 0; ls < S; ++ls) {
            const int k = kof<S>(c, ls);
            if (k <= N)
                for (int q = 0; q < 4; ++q) A.qp_dx[((size_t)iv * (N + 1) + k) * 4 + q] = st.dxs(ls, q);
            if (k < N) {
                for (int q = 0; q < 2; ++q) A.qp_du[((size_t)iv * N + k) * 2 + q] = st.du(ls, q);
                for (int q = 0; q < 6; ++q) A.qp_lam[((size_t)iv * N + k) * 6 + q] = st.lm(ls, q);
            }
            if (k == 0) A.qp_iter[iv] = nit;
            // QP status: 0 stop test met, 2 cap, 4 stall (min step), 5 diverged (qsp_qp_solve)
            if (k == 0 && A.qp_capped)
                A.qp_capped[iv] = exit == QP_EXIT_CONV ? 0 : (exit == QP_EXIT_CAP ? 2 : (exit == QP_EXIT_STALL ? 4 : 5));
        }
        return;
    }
    // multipliers of every successful QP (the output holds the last one, also for an
    // instance that stops early)
    qp_adjoint_store<S>(c, p, st, A.PI_out + (size_t)iv * N * 4, c.real && !skip && !failed,
                        (A.flags & QSP_FLAG_SHIFT) != 0);
    if (!c.real || skip || failed) return;
#pragma unroll
    for (int ls = 0; ls < S; ++ls) {
        const int k = kof<S>(c, ls);
        if (k <= N)
            for (int q = 0; q < 4; ++q) X[4 * k + q] += st.dxs(ls, q);
        if (k < N) {
            U[2 * k] += st.du(ls, 0);
            U[2 * k + 1] += st.du(ls, 1);
        }
        if (k == 0) A.qp_iter[iv] += nit;
    }
    SEG_ADD(12, t_k);
}

// Small batches (fewer waves than the chip's 2 048 wave slots), nlp_mode 0: the whole SQP loop
// in one launch.  Every wave keeps its instances for all K iterations, so a solve costs the
// slowest wave's own sum of IPM iterations instead of the sum over iterations of the slowest
// wave of the batch (no packing sort, no grid-wide boundary between SQP iterations).  The
// per-iteration arithmetic is qp_step_kernel<S, false, true>'s (same helpers, same order), so
// the results are bit-identical to the per-iteration launches (tests/test_gpu_fullsize.py).
template <int S, bool ALT = false>
__global__ void __launch_bounds__(BLOCK, QSP_MIN_WAVES) sqp_loop_kernel(SolveArgs A) {
    extern __shared__ double smem[];
    const SolveParams& p = A.p;
    const int N = p.N;
    if (A.flags & QSP_FLAG_POISON) {
        for (int f = 0; f < F_COUNT * S + mfw_extra<S>(); ++f) smem[threadIdx.x + f * BLOCK] = __builtin_nan("");
    }
    bool stopped = false;   // group-uniform: a failed QP stops the instance's SQP
    for (int it = 0; it < p.sqp_iters; ++it) {
        if (it > 0) __syncthreads();   // the neighbour lanes' X, U stores of the last iteration
        // debug: re-poisoned at every SQP iteration, so a read of a word the current iteration
        // did not write shows up (the last iteration's finite values would hide it)
        if (it > 0 && (A.flags & QSP_FLAG_POISON)) {
            for (int f = 0; f < F_COUNT * S + mfw_extra<S>(); ++f) smem[threadIdx.x + f * BLOCK] = __builtin_nan("");
        }
        // lane geometry and addresses re-derived every iteration from an opaque lane id: hoisted
        // out of the loop they would stay live through the interior point (register budget)
        int lane = threadIdx.x & 63;
        asm volatile("" : "+v"(lane));
        Ctx c;
        c.lane = lane;
        c.N = N;
        c.L = (N + S) / S;
        const int G = 64 / c.L;
        c.grp = c.lane / c.L;
        c.lig = c.lane - c.grp * c.L;
        c.base = c.grp * c.L;
        c.gs.init(c.base, c.L);
        const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
        c.inst = wave * G + c.grp;
        c.real = (c.grp < G) && (c.inst < A.nI);
        const int iv = A.i0 + (c.real ? c.inst : A.nI - 1);
        double* X = A.wX + (size_t)iv * (N + 1) * 4;
        double* U = A.wU + (size_t)iv * N * 2;
        if (it == 0) stopped = A.wdone[iv] != 0;
        // a fresh register block per iteration: the factor walk writes K, Rn, kk in place under
        // a lane mask, which would otherwise keep the last iteration's values live
        Stage<S> st;
        st.lds = smem + threadIdx.x;
        const bool lin_live = c.real && !stopped;
#pragma unroll
        for (int ls = 0; ls < S; ++ls) {
            const int k = kof<S>(c, ls);
            const int kc = k <= N ? k : N;
            const int ku = k < N ? k : N - 1;
            if (kc < N && lin_live) {
                const double xk[4] = {X[4 * kc], X[4 * kc + 1], X[4 * kc + 2], X[4 * kc + 3]};
                const double uk[2] = {U[2 * kc], U[2 * kc + 1]};
                Lin Ln;
                rk4<true>(shape_of(A, iv), p.Ts, xk, uk, Ln);
                const double* yr = A.yref + ((size_t)iv * N + kc) * 6;
#pragma unroll
                for (int q = 0; q < 6; ++q) st.a[ls][q] = Ln.a[q];
#pragma unroll
                for (int q = 0; q < 8; ++q) st.B[ls][q] = Ln.B[q];
#pragma unroll
                for (int q = 0; q < 4; ++q) st.bb[ls][q] = Ln.xn[q] - X[4 * (kc + 1) + q];
#pragma unroll
                for (int q = 0; q < 4; ++q) st.g[ls][q] = p.tau * p.W[q] * (xk[q] - yr[q]);
#pragma unroll
                for (int q = 0; q < 2; ++q) st.g[ls][4 + q] = p.tau * p.W[4 + q] * (uk[q] - yr[4 + q]);
            } else {
                const double* ye = A.yref_e + (size_t)iv * 4;
#pragma unroll
                for (int q = 0; q < 6; ++q) st.a[ls][q] = 0.0;
#pragma unroll
                for (int q = 0; q < 8; ++q) st.B[ls][q] = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) st.bb[ls][q] = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) st.g[ls][q] = p.We[q] * (X[4 * N + q] - ye[q]);
                st.g[ls][4] = 0.0;
                st.g[ls][5] = 0.0;
            }
            st.v(ls, 0) = X[4 * kc + 3];
            st.v(ls, 1) = U[2 * ku];
            st.v(ls, 2) = U[2 * ku + 1];
        }
        double dx0[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) dx0[q] = A.wx0[(size_t)iv * 4 + q] - X[q];
        const bool skip = stopped || !c.real;
        int exit;
        const int nit = qp_ipm<S, ALT>(c, p, st, dx0, exit, skip);
        qp_rollout<S>(c, st, dx0);
        const bool failed = qp_outcome<S>(A, c, st, iv, it, exit, skip);
        qp_adjoint_store<S>(c, p, st, A.PI_out + (size_t)iv * N * 4, c.real && !skip && !failed,
                            (A.flags & QSP_FLAG_SHIFT) != 0);
        if (c.real && !skip && !failed) {
#pragma unroll
            for (int ls = 0; ls < S; ++ls) {
                const int k = kof<S>(c, ls);
                if (k <= N)
                    for (int q = 0; q < 4; ++q) X[4 * k + q] += st.dxs(ls, q);
                if (k < N) {
                    U[2 * k] += st.du(ls, 0);
                    U[2 * k + 1] += st.du(ls, 1);
                }
                if (k == 0) A.qp_iter[iv] += nit;
            }
        }
        stopped = stopped || failed;
    }
}

// Counting sort of the instances by their packing key (pack_key) in one pass over the
// instances: the histogram of the keys was accumulated by the QP launch itself (whist,
// parity q); every block forms the exclusive prefix of the histogram (a block-wide scan),
// places its instances at the key's prefix plus a block offset taken from the running
// counters, and block 0 clears the other parity's histogram and counters for the next
// launch.  The order inside a key is arbitrary and does not affect any result (instances
// are independent).  Sorts the instance range [i0, i0 + B) into perm[i0 ...] (one part of a
// split SQP loop, with the part's own whist).
__global__ void __launch_bounds__(256) sort_by_iters_kernel(int i0, int B, int maxkey, const int32_t* nit,
                                                            int32_t* perm, int32_t* whist, int q) {
    constexpr int KPT = PACK_KEYS_MAX / 256;   // keys per thread in the prefix scan
    __shared__ int pre[PACK_KEYS_MAX], lcount[PACK_KEYS_MAX], part[256];
    const int tid = threadIdx.x;
    const int nkeys = (maxkey + 1) * (maxkey + 1);
    const int32_t* hist = whist + q * PACK_KEYS_MAX;
    int32_t* run = whist + (2 + q) * PACK_KEYS_MAX;
    int h[KPT], sum = 0;
#pragma unroll
    for (int r = 0; r < KPT; ++r) {
        const int k = tid * KPT + r;
        h[r] = k < nkeys ? hist[k] : 0;
        sum += h[r];
        lcount[k] = 0;
    }
    part[tid] = sum;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {   // inclusive scan of the per-thread sums
        const int v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int acc = part[tid] - sum;
#pragma unroll
    for (int r = 0; r < KPT; ++r) {
        pre[tid * KPT + r] = acc;
        acc += h[r];
    }
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + tid;
    int key = 0, pos = 0;
    if (i < B) {
        key = pack_key(nit[i0 + i], maxkey);
        pos = atomicAdd(&lcount[key], 1);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < KPT; ++r) {
        const int k = tid * KPT + r;
        if (lcount[k] > 0) pre[k] += atomicAdd(&run[k], lcount[k]);
    }
    __syncthreads();
    if (i < B) perm[i0 + pre[key] + pos] = i0 + i;
    if (blockIdx.x == 0) {
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            whist[(1 - q) * PACK_KEYS_MAX + tid * KPT + r] = 0;
            whist[(3 - q) * PACK_KEYS_MAX + tid * KPT + r] = 0;
        }
    }
}

__global__ void iota_kernel(int B, int32_t* perm) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < B) perm[i] = i;
}

// nlp_mode 1 line search and update (one stage per lane, no LDS): merit weights
// nu = max(|pi|, (nu + |pi|)/2), eta likewise from the QP bound multipliers; phi(0) and
// its directional derivative; alpha <- ls_alpha_red * alpha until
// phi(alpha) <= phi(0) + ls_eps alpha dphi or alpha would drop below ls_alpha_min (then
// the last alpha tried is taken); X, U, PI, LAM updated with that alpha.
__global__ void __launch_bounds__(64) merit_ls_kernel(SolveArgs A) {
    const SolveParams& p = A.p;
    Ctx c;
    c.lane = threadIdx.x & 63;
    c.N = p.N;
    c.L = p.N + 1;
    const int G = 64 / c.L;
    c.grp = c.lane / c.L;
    c.lig = c.lane - c.grp * c.L;
    c.base = c.grp * c.L;
    c.gs.init(c.base, c.L);
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    c.inst = wave * G + c.grp;
    c.real = (c.grp < G) && (c.inst < A.nI);
    // the QP launch's wave packing (instances ordered by their predicted IPM count) also groups
    // the line searches: a wave backtracks until the last of its instances accepts a step
    const int slot = A.i0 + (c.real ? c.inst : A.nI - 1);
    const int iv = A.wperm ? A.wperm[slot] : slot;
    const int N = p.N;
    const int k = c.lig <= N ? c.lig : N;
    const bool stg = k < N;
    const int ku = stg ? k : N - 1;
    const size_t tot = (size_t)A.B * (N + 1);
    const size_t si = (size_t)iv * (N + 1) + k;
    // converged instances (this or an earlier iteration) keep their iterate; the QP kernel
    // wrote no step for them
    const bool skip = !c.real || A.wdone[iv] != 0;
    const ShapeDev& sh = shape_of(A, iv);
    double* X = A.wX + (size_t)iv * (N + 1) * 4;
    double* U = A.wU + (size_t)iv * N * 2;
    // what the backtracking loop reads stays in registers; the multipliers are read again
    // for the update after it (fewer live registers: more waves per SIMD)
    double xk[4], uk[2], dxk[4], duk[2], bb[4], g[6];
    double NUk[4], ETAk[6];
#pragma unroll
    for (int q = 0; q < 4; ++q) xk[q] = X[4 * k + q];
    uk[0] = U[2 * ku];
    uk[1] = U[2 * ku + 1];
    const double* w = A.wqp + si;
    const double* in = A.wlin + si;
    const double* nl = A.wnlp + si;
#pragma unroll
    for (int q = 0; q < 4; ++q) dxk[q] = skip ? 0.0 : w[(Q_DX + q) * tot];
#pragma unroll
    for (int q = 0; q < 2; ++q) duk[q] = (skip || !stg) ? 0.0 : w[(Q_DU + q) * tot];
#pragma unroll
    for (int q = 0; q < 4; ++q) bb[q] = in[(L_BB + q) * tot];
#pragma unroll
    for (int q = 0; q < 6; ++q) g[q] = in[(L_G + q) * tot];
#pragma unroll
    for (int q = 0; q < 4; ++q) NUk[q] = nl[(W_NU + q) * tot];
#pragma unroll
    for (int q = 0; q < 6; ++q) ETAk[q] = nl[(W_ETA + q) * tot];
    if (stg) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double a = skip ? 0.0 : fabs(w[(Q_PI + q) * tot]), wq = 0.5 * (NUk[q] + a);
            NUk[q] = a > wq ? a : wq;
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const double a = skip ? 0.0 : fabs(w[(Q_LAM + q) * tot]), wq = 0.5 * (ETAk[q] + a);
            ETAk[q] = a > wq ? a : wq;
        }
    }
    const double* yr = A.yref + ((size_t)iv * N + ku) * 6;
    const double* ye = A.yref_e + (size_t)iv * 4;
    double dph = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) dph = qfma(g[i], dxk[i], dph);
    if (stg) {
        dph = qfma(g[5], duk[1], qfma(g[4], duk[0], dph));
#pragma unroll
        for (int i = 0; i < 4; ++i) dph = qfma(-NUk[i], fabs(bb[i]), dph);
        const double v[3] = {xk[3], uk[0], uk[1]};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (j == 0 && k == 0 && !p.s0_bound) continue;
            const double lo = p.lh[j] - v[j], hi = p.uh[j] - v[j];
            if (lo > 0.0) dph = qfma(-ETAk[2 * j], lo, dph);
            if (hi < 0.0) dph = qfma(ETAk[2 * j + 1], hi, dph);
        }
    }
    const double phi0 = group_sum(merit_stage(p, k, xk, uk, yr, ye, bb, NUk, ETAk), c.gs);
    const double dphi = group_sum(dph, c.gs);
    double alpha = 1.0;
    bool fin = skip;
    while (__ballot(!fin) != 0ull) {
        double xt[4], ut[2], xnx[4], def[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) xt[q] = qfma(alpha, dxk[q], xk[q]);
        ut[0] = qfma(alpha, duk[0], uk[0]);
        ut[1] = qfma(alpha, duk[1], uk[1]);
#pragma unroll
        for (int q = 0; q < 4; ++q) xnx[q] = wave_from_next(xt[q]);   // x_{k+1} + alpha dx_{k+1}
        if (stg) {
            Lin Lt;
            rk4<false>(sh, p.Ts, xt, ut, Lt);
#pragma unroll
            for (int q = 0; q < 4; ++q) def[q] = Lt.xn[q] - xnx[q];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) def[q] = 0.0;
        }
        const double phi = group_sum(merit_stage(p, k, xt, ut, yr, ye, def, NUk, ETAk), c.gs);
        if (!fin) {
            if (phi <= qfma(p.ls_eps * alpha, dphi, phi0)) {
                fin = true;
            } else {
                const double an = alpha * p.ls_alpha_red;
                if (an < p.ls_alpha_min) fin = true;      // accept the last step tried
                else alpha = an;
            }
        }
    }
    if (skip) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) X[4 * k + q] = qfma(alpha, dxk[q], xk[q]);
    if (stg) {
        U[2 * k] = qfma(alpha, duk[0], uk[0]);
        U[2 * k + 1] = qfma(alpha, duk[1], uk[1]);
        double* nw = A.wnlp + si;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double pk = nw[(W_PI + q) * tot];
            nw[(W_PI + q) * tot] = qfma(alpha, w[(Q_PI + q) * tot] - pk, pk);
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const double lk = nw[(W_LAM + q) * tot];
            nw[(W_LAM + q) * tot] = qfma(alpha, w[(Q_LAM + q) * tot] - lk, lk);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) nw[(W_NU + q) * tot] = NUk[q];
#pragma unroll
        for (int q = 0; q < 6; ++q) nw[(W_ETA + q) * tot] = ETAk[q];
    }
}

// status, cost, u0 and the (optionally shifted, NMPC_controller.m:397-399) outputs.
__global__ void epilogue_kernel(SolveArgs A) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.B) return;
    const SolveParams& p = A.p;
    const int N = p.N;
    const double* X = A.wX + (size_t)i * (N + 1) * 4;
    const double* U = A.wU + (size_t)i * N * 2;
    const double* yref = A.yref + (size_t)i * N * 6;
    const double* ye = A.yref_e + (size_t)i * 4;
    bool bad = false;
    double cost = 0.0;
    for (int k = 0; k < N; ++k) {
        double s = 0.0;
        for (int q = 0; q < 4; ++q) { const double r = X[4 * k + q] - yref[6 * k + q]; s = qfma(p.W[q] * r, r, s); bad |= !isfinite(X[4 * k + q]); }
        for (int q = 0; q < 2; ++q) { const double r = U[2 * k + q] - yref[6 * k + 4 + q]; s = qfma(p.W[4 + q] * r, r, s); bad |= !isfinite(U[2 * k + q]); }
        cost = qfma(0.5 * p.tau, s, cost);
    }
    double s = 0.0;
    for (int q = 0; q < 4; ++q) { const double r = X[4 * N + q] - ye[q]; s = qfma(p.We[q] * r, r, s); bad |= !isfinite(X[4 * N + q]); }
    cost = qfma(0.5, s, cost);
    A.cost[i] = cost;
    // wdone: 1 converged, 2 non-finite QP solution, 3 infeasible stage-0 bound, 4 diverged QP
    // (sqp_iter written then)
    const int fr = A.wdone ? A.wdone[i] : 0;
    if (fr == 3 || fr == 4) A.status[i] = QSP_STATUS_QP_FAIL;
    else if (p.nlp_mode == 1) A.status[i] = (bad || fr == 2) ? 1 : (fr == 1 ? 0 : 2);
    else A.status[i] = (bad || fr == 2) ? 1 : 0;
    if (fr == 0) A.sqp_iter[i] = p.sqp_iters;
    A.u0[(size_t)i * 2] = U[0];
    A.u0[(size_t)i * 2 + 1] = U[1];
    const int sh = (A.flags & QSP_FLAG_SHIFT) ? 1 : 0;
    double* Xo = A.X_out + (size_t)i * (N + 1) * 4;
    double* Uo = A.U_out + (size_t)i * N * 2;
    for (int k = 0; k <= N; ++k) {
        const int src = (k + sh <= N) ? k + sh : N;
        for (int q = 0; q < 4; ++q) Xo[4 * k + q] = X[4 * src + q];
    }
    for (int k = 0; k < N; ++k) {
        const int src = (k + sh < N) ? k + sh : N - 1;
        for (int q = 0; q < 2; ++q) Uo[2 * k + q] = U[2 * src + q];
    }
    if (p.nlp_mode == 1) {
        // dynamics multipliers of the NLP iterate (shifted like X/U in controller mode)
        const size_t tot = (size_t)A.B * (N + 1);
        double* Po = A.PI_out + (size_t)i * N * 4;
        for (int k = 0; k < N; ++k) {
            const int src = (k + sh < N) ? k + sh : N - 1;
            for (int q = 0; q < 4; ++q) Po[4 * k + q] = A.wnlp[(W_PI + q) * tot + (size_t)i * (N + 1) + src];
        }
    }
    if (A.warm_valid && (A.flags & QSP_FLAG_CONTROLLER)) A.warm_valid[i] = 1;
}

// ------------------------------------------------------- closed-loop plant
// helper.m:195-322 (closed_loop_matlab), one thread per lane, around each NMPC_controller.solve:
//   closed_loop_pre_kernel: the disturbance (:221-236), sim_noise (:240-242), the trajectory log
//     and the controller's delay prediction delay_buffer_sim (NMPC_controller.m:112-120) into the
//     solver's x0;
//   plant_kernel: the controller input buffer push (helper.m:255), the plant x(:,i+1) = x(:,i) +
//     Ts * evalModelVariableShape(x(:,i), u) with the plant's own delay buffer (:289-307), logs.

// |C(s) - p|^2 with C at the floor-mod of s (evalSpline, bspline_shape.m:192-199)
__device__ __forceinline__ double contact_phi(const ShapeDev& sh, double s, double px, double py) {
    SplineEval e;
    spline_eval(sh, mat_mod(s, sh.b), e);
    const double ex = e.C[0] - px, ey = e.C[1] - py;
    return qfma(ey, ey, ex * ex);
}

// The contact point after a lateral disturbance: argmin_s |C(s) - p|^2 from s0 (fminunc in the
// reference, helper.m:230; restated as a damped Newton iteration, as the oracle's reproject_contact)
__device__ double reproject_contact(const ShapeDev& sh, double px, double py, double s0) {
    double s = s0, phi = contact_phi(sh, s, px, py);
    for (int it = 0; it < 60; ++it) {
        SplineEval e;
        spline_eval(sh, mat_mod(s, sh.b), e);
        const double ex = e.C[0] - px, ey = e.C[1] - py;
        const double g = 2.0 * qfma(ey, e.D[1], ex * e.D[0]);
        const double h = 2.0 * qfma(ey, e.Dd[1], qfma(ex, e.Dd[0], qfma(e.D[1], e.D[1], e.D[0] * e.D[0])));
        if (fabs(g) < 1e-14) break;
        double step = h > 0.0 ? -g / h : (g > 0.0 ? -0.05 : 0.05) * sh.b;
        const double smax = 0.25 * sh.b;
        step = fmin(fmax(step, -smax), smax);
        bool ok = false;
        double sn = s, phin = phi;
        for (int k = 0; k < 60; ++k) {
            sn = s + step;
            phin = contact_phi(sh, sn, px, py);
            if (phin < phi) { ok = true; break; }
            step *= 0.5;
        }
        if (!ok) break;
        s = sn;
        phi = phin;
        if (fabs(step) < 1e-13 * sh.b) break;
    }
    return s;
}

__device__ __forceinline__ const ShapeDev& shape_clamped(const ShapeDev* shapes, int n_shapes, const int32_t* sid, int i) {
    const int id = sid ? sid[i] : 0;   // clamped like shape_of (the table may have shrunk since the ids were set)
    return shapes[id < 0 ? 0 : (id >= n_shapes ? n_shapes - 1 : id)];
}

__global__ void closed_loop_pre_kernel(ClosedLoopArgs a, int t) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.B) return;
    const ShapeDev& sh = shape_clamped(a.shapes, a.n_shapes, a.sid, i);
    double x[4] = {a.x[(size_t)i * 4], a.x[(size_t)i * 4 + 1], a.x[(size_t)i * 4 + 2], a.x[(size_t)i * 4 + 3]};
    if (a.dist_step > 0 && t + 1 == a.dist_step) {
        // y += amplitude; new contact: the spline point nearest (-xwidth/2, C_y(s) - amplitude),
        // from s0_spline = 0 (one disturbance per run), wrapped into [-b, b) (:224-234)
        const double amp = a.dist_amp ? a.dist_amp[i] : 0.0;
        x[1] += amp;
        SplineEval e;
        spline_eval(sh, mat_mod(x[3], sh.b), e);
        const double sn = reproject_contact(sh, -0.5 * sh.xwidth, e.C[1] - amp, 0.0);
        x[3] = qfma(-sh.b, sn < 0.0 ? 1.0 : 0.0, mat_mod(sn, sh.b));
    }
    if (a.noise)
        for (int c = 0; c < 4; ++c) x[c] += a.noise[((size_t)t * a.B + i) * 4 + c];
    for (int c = 0; c < 4; ++c) {
        a.x[(size_t)i * 4 + c] = x[c];
        a.Xtraj[((size_t)i * (a.n_steps + 1) + t) * 4 + c] = x[c];
    }
    // delay_buffer_sim: D Euler steps with the buffered inputs, oldest (u_buff_contr(:, end)) first
    for (int k = 1; k <= a.D; ++k) {
        const double* u = a.ubc + ((size_t)i * a.D + (a.D - k)) * 2;
        DynOut d;
        dynamics<false>(sh, x[2], x[3], u[0], u[1], d);
        for (int c = 0; c < 4; ++c) x[c] = qfma(a.Ts, d.f[c], x[c]);
    }
    for (int c = 0; c < 4; ++c) a.xs[(size_t)i * 4 + c] = x[c];
    if (a.Xsim)
        for (int c = 0; c < 4; ++c) a.Xsim[((size_t)i * a.n_steps + t) * 4 + c] = x[c];
}

__global__ void plant_kernel(ClosedLoopArgs a, int t) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.B) return;
    const ShapeDev& sh = shape_clamped(a.shapes, a.n_shapes, a.sid, i);
    double xi[4] = {a.x[(size_t)i * 4], a.x[(size_t)i * 4 + 1], a.x[(size_t)i * 4 + 2], a.x[(size_t)i * 4 + 3]};
    const double u[2] = {a.u0[(size_t)i * 2], a.u0[(size_t)i * 2 + 1]};
    // u_buff_contr = [u, u_buff_contr(:, 1:end-1)]
    if (a.D > 0) {
        double* b = a.ubc + (size_t)i * a.D * 2;
        for (int k = a.D - 1; k >= 1; --k) { b[2 * k] = b[2 * (k - 1)]; b[2 * k + 1] = b[2 * (k - 1) + 1]; }
        b[0] = u[0];
        b[1] = u[1];
    }
    double ua[2] = {u[0], u[1]};
    if (a.Dp > 0) {   // the plant applies u_buff_plant(:, end), then pushes u
        double* b = a.ubp + (size_t)i * a.Dp * 2;
        ua[0] = b[2 * (a.Dp - 1)];
        ua[1] = b[2 * (a.Dp - 1) + 1];
        for (int k = a.Dp - 1; k >= 1; --k) { b[2 * k] = b[2 * (k - 1)]; b[2 * k + 1] = b[2 * (k - 1) + 1]; }
        b[0] = u[0];
        b[1] = u[1];
    }
    DynOut d;
    dynamics<false>(sh, xi[2], xi[3], ua[0], ua[1], d);
    for (int c = 0; c < 4; ++c) {
        const double v = qfma(a.Ts, d.f[c], xi[c]);
        a.x[(size_t)i * 4 + c] = v;
        if (t + 1 == a.n_steps) a.Xtraj[((size_t)i * (a.n_steps + 1) + t + 1) * 4 + c] = v;
    }
    a.Utraj[((size_t)i * a.n_steps + t) * 2] = u[0];
    a.Utraj[((size_t)i * a.n_steps + t) * 2 + 1] = u[1];
    if (a.Straj) a.Straj[(size_t)i * a.n_steps + t] = a.status[i];
}

// NMPC_controller.delay_buffer_sim alone (qsp_delay_buffer_sim)
__global__ void delay_sim_kernel(ClosedLoopArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.B) return;
    const ShapeDev& sh = shape_clamped(a.shapes, a.n_shapes, a.sid, i);
    double x[4] = {a.x[(size_t)i * 4], a.x[(size_t)i * 4 + 1], a.x[(size_t)i * 4 + 2], a.x[(size_t)i * 4 + 3]};
    for (int k = 1; k <= a.D; ++k) {
        const double* u = a.ubc + ((size_t)i * a.D + (a.D - k)) * 2;
        DynOut d;
        dynamics<false>(sh, x[2], x[3], u[0], u[1], d);
        for (int c = 0; c < 4; ++c) x[c] = qfma(a.Ts, d.f[c], x[c]);
    }
    for (int c = 0; c < 4; ++c) a.xs[(size_t)i * 4 + c] = x[c];
}

__global__ void reproject_kernel(const ShapeDev* shapes, int n_shapes, const int32_t* sid, int n, const double* px,
                                 const double* py, const double* s0, double* s) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    s[i] = reproject_contact(shape_clamped(shapes, n_shapes, sid, i), px[i], py[i], s0[i]);
}

hipError_t launch_closed_loop_pre(const ClosedLoopArgs& a, int t, hipStream_t stream) {
    hipLaunchKernelGGL(closed_loop_pre_kernel, dim3((a.B + 127) / 128), dim3(128), 0, stream, a, t);
    return hipGetLastError();
}

hipError_t launch_plant(const ClosedLoopArgs& a, int t, hipStream_t stream) {
    hipLaunchKernelGGL(plant_kernel, dim3((a.B + 127) / 128), dim3(128), 0, stream, a, t);
    return hipGetLastError();
}

hipError_t launch_delay_sim(const ClosedLoopArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(delay_sim_kernel, dim3((a.B + 127) / 128), dim3(128), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_reproject(const ShapeDev* shapes, int n_shapes, const int32_t* sid, int n, const double* px,
                            const double* py, const double* s0, double* s, hipStream_t stream) {
    hipLaunchKernelGGL(reproject_kernel, dim3((n + 127) / 128), dim3(128), 0, stream, shapes, n_shapes, sid, n, px, py,
                       s0, s);
    return hipGetLastError();
}

// ------------------------------------------------- reference generation
// TrajectoryGenerator.straight_line (TrajectoryGenerator.m:39-79), one thread per
// (lane, sample): quintic time scaling s(t) = 6 tau^5 - 15 tau^4 + 10 tau^3, tau = t / tf
// (:39-42), x(t) = x0 + s(t) (xf - x0) on (x, y, theta); rows [x y theta 0 0 0] as
// main.m:165-178 builds y_ref (s_ref = 0, u_ref = 0).  auto_angle: theta follows its own
// quintic over tf / 2 and then holds its final value (:58-66).
__device__ __forceinline__ double quintic(double t, double tf) {
    const double tau = t / tf;
    return qfma(qfma(6.0, tau, -15.0), tau, 10.0) * tau * tau * tau;
}

__global__ void straight_lines_kernel(int B, int T, const double* x0, const double* xf, double t0, double tf,
                                      double Ts, int auto_angle, double* traj) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (size_t)B * T) return;
    const int i = (int)(g / T), k = (int)(g - (size_t)i * T);
    const double t = qfma((double)k, Ts, t0);
    const double* a = x0 + (size_t)i * 3;
    const double* b = xf + (size_t)i * 3;
    const double s = quintic(t, tf);
    double* out = traj + g * 6;
    out[0] = qfma(s, b[0] - a[0], a[0]);
    out[1] = qfma(s, b[1] - a[1], a[1]);
    if (auto_angle) {
        const double tfa = 0.5 * tf;
        const int ka = (int)floor((tfa - t0) / Ts + 1e-9);      // last sample of t0:Ts:tf/2
        const double ta = qfma((double)(k < ka ? k : ka), Ts, t0);
        out[2] = qfma(quintic(ta, tf), b[2] - a[2], a[2]);
    } else {
        out[2] = qfma(s, b[2] - a[2], a[2]);
    }
    out[3] = 0.0;
    out[4] = 0.0;
    out[5] = 0.0;
}

hipError_t launch_straight_lines(int B, int T, const double* x0, const double* xf, double t0, double tf, double Ts,
                                 int auto_angle, double* traj, hipStream_t stream) {
    const size_t n = (size_t)B * T;
    hipLaunchKernelGGL(straight_lines_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, B, T, x0, xf,
                       t0, tf, Ts, auto_angle, traj);
    return hipGetLastError();
}

// ----------------------------------------------------- building-block kernels
__global__ void spline_kernel(const ShapeDev* shapes, const int32_t* sid, int n, const double* s,
                              double* C, double* D, double* Dd, double* kappa) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ShapeDev& sh = shapes[sid[i]];
    SplineEval e;
    spline_eval(sh, s[i], e);
    for (int c = 0; c < 2; ++c) { C[2 * i + c] = e.C[c]; D[2 * i + c] = e.D[c]; Dd[2 * i + c] = e.Dd[c]; }
    kappa[i] = angle_rate_of(e);
}

__global__ void dynamics_kernel(const ShapeDev* shapes, const int32_t* sid, int n, const double* x, const double* u,
                                double* f, double* J) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ShapeDev& sh = shapes[sid[i]];
    DynOut d;
    dynamics<true>(sh, x[4 * i + 2], x[4 * i + 3], u[2 * i], u[2 * i + 1], d);
    for (int r = 0; r < 4; ++r) {
        f[4 * i + r] = d.f[r];
        double* Jr = J + (size_t)24 * i + 6 * r;
        Jr[0] = 0.0; Jr[1] = 0.0;
        Jr[2] = r < 2 ? d.Jth[r] : 0.0;
        Jr[3] = d.Js[r]; Jr[4] = d.Jun[r]; Jr[5] = d.Jut[r];
    }
}

__global__ void rk4_kernel(const ShapeDev* shapes, const int32_t* sid, int n, double h, const double* x, const double* u,
                           double* xn, double* Aout, double* Bout) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ShapeDev& sh = shapes[sid[i]];
    double xi[4] = {x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]};
    double ui[2] = {u[2 * i], u[2 * i + 1]};
    Lin L;
    rk4<true>(sh, h, xi, ui, L);
    double* Ai = Aout + (size_t)16 * i;
    const double Afull[16] = {1.0, 0.0, L.a[0], L.a[1], 0.0, 1.0, L.a[2], L.a[3],
                              0.0, 0.0, 1.0, L.a[4], 0.0, 0.0, 0.0, L.a[5]};
    for (int q = 0; q < 16; ++q) Ai[q] = Afull[q];
    for (int q = 0; q < 8; ++q) Bout[(size_t)8 * i + q] = L.B[q];
    for (int q = 0; q < 4; ++q) xn[4 * i + q] = L.xn[q];
}

__global__ void vbound_kernel(const ShapeDev* shapes, const int32_t* sid, int n, CtrlParams cp, const double* s,
                              double* vb) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    vb[i] = v_bound(shapes[sid[i]], cp, s[i]);
}

// ------------------------------------------------------------------ launchers
// The QP kernels take more than 64 KB of dynamic LDS, which a kernel must be allowed once per
// device (one bit per device in `done`; handles on several devices may share a process).
static hipError_t lds_attr_once(const void* kernel, int bytes, std::atomic<uint64_t>& done) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}

// LIN: the SQP iteration's linearisation runs inside the QP kernel (nlp_mode 0); without
// it the kernel reads the stage data the workspace holds (qsp_qp_solve).
// ALT: the alternative factorisation of the stage count — S = 2: the associative scan
// (SolveParams::factor_scan); S = 1: the walk on the matrix cores (mfw_use)
template <int S, bool LIN, bool ALT = false>
static hipError_t launch_qp_step(const SolveArgs& a, int it, hipStream_t stream) {
    const int L = (a.p.N + S) / S;
    const int G = 64 / L;
    const int waves = (a.nI + G - 1) / G;
    const int blocks = (waves * 64 + BLOCK - 1) / BLOCK;
    static std::atomic<uint64_t> attr{0};
    const hipError_t e = lds_attr_once((const void*)qp_step_kernel<S, false, LIN, ALT>, lds_bytes<S>(), attr);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((qp_step_kernel<S, false, LIN, ALT>), dim3(blocks), dim3(BLOCK), lds_bytes<S>(), stream, a, it);
    return hipGetLastError();
}

template <int S, bool ALT = false>
static hipError_t launch_sqp_loop(const SolveArgs& a, hipStream_t stream) {
    const int L = (a.p.N + S) / S;
    const int G = 64 / L;
    const int waves = (a.nI + G - 1) / G;
    const int blocks = (waves * 64 + BLOCK - 1) / BLOCK;
    static std::atomic<uint64_t> attr{0};
    const hipError_t e = lds_attr_once((const void*)sqp_loop_kernel<S, ALT>, lds_bytes<S>(), attr);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((sqp_loop_kernel<S, ALT>), dim3(blocks), dim3(BLOCK), lds_bytes<S>(), stream, a);
    return hipGetLastError();
}

// sqp_loop_kernel keeps more state live across its SQP loop than qp_step_kernel and runs at
// 1 wave/SIMD (256 VGPRs + AGPRs), so it pays only while its waves fit the SIMDs (4 per CU:
// 1 024 on a whole MI355X) in one round.  Measured (scripts/fused_sweep.sh, N = 20, K = 50,
// S = 1, solves/s per-iteration launches -> fused): B = 1 024 58.7k -> 76.5k; 2 048 115k ->
// 123k; 3 072 (1 024 waves) 173k -> 224k; 4 096 (1 366 waves, two rounds) 227k -> 169k.
int sqp_fused_auto(int B, int N, int S, int nlp_mode, int cus) {
    const int G = 64 / lanes_per_instance(N, S);
    const long waves = ((long)B + G - 1) / G;
    return (nlp_mode == 0 && (S == 1 || S == 2) && waves <= 4L * cus) ? 1 : 0;
}

static hipError_t launch_qp_any(const SolveArgs& a, int S, int it, hipStream_t stream, bool lin) {
    switch (S) {
        case 1:
            if (mfw_use(a.p, 1))
                return lin ? launch_qp_step<1, true, true>(a, it, stream) : launch_qp_step<1, false, true>(a, it, stream);
            return lin ? launch_qp_step<1, true>(a, it, stream) : launch_qp_step<1, false>(a, it, stream);
        case 2:
            if (a.p.factor_scan)
                return lin ? launch_qp_step<2, true, true>(a, it, stream) : launch_qp_step<2, false, true>(a, it, stream);
            return lin ? launch_qp_step<2, true>(a, it, stream) : launch_qp_step<2, false>(a, it, stream);
        default: return hipErrorInvalidValue;
    }
}

int lanes_per_instance(int N, int S) { return (N + S) / S; }

#ifdef QSP_SEGSTAMP
// diagnostic build: read (and optionally clear) the segment cycle sums
extern "C" int qsp_debug_segments(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seg), sizeof(g_seg)) != hipSuccess) return -2;
    if (reset) {
        static const unsigned long long zero[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_seg), zero, sizeof(zero)) != hipSuccess) return -2;
    }
    return 0;
}
#endif

int factor_walk_kind(const SolveParams& p, int S) {
    if (S == 2 && p.factor_scan) return QSP_WALK_SCAN;
    return (S == 1 || S == 2) && mfw_use(p, S) ? QSP_WALK_MFMA : QSP_WALK_LANE;
}

static hipError_t launch_sqp_merit(const SolveArgs& a, int it, hipStream_t stream) {
    const int L = a.p.N + 1;
    const int G = 64 / L;
    const int waves = (a.nI + G - 1) / G;
    const int blocks = (waves * 64 + BLOCK - 1) / BLOCK;
    static std::atomic<uint64_t> attr{0}, attr_alt{0};
    if (mfw_use(a.p, 1)) {
        const hipError_t ea = lds_attr_once((const void*)qp_step_kernel<1, true, true, true>, lds_bytes<1>(), attr_alt);
        if (ea != hipSuccess) return ea;
        hipLaunchKernelGGL((qp_step_kernel<1, true, true, true>), dim3(blocks), dim3(BLOCK), lds_bytes<1>(), stream, a, it);
    } else {
        const hipError_t ea = lds_attr_once((const void*)qp_step_kernel<1, true, true>, lds_bytes<1>(), attr);
        if (ea != hipSuccess) return ea;
        hipLaunchKernelGGL((qp_step_kernel<1, true, true>), dim3(blocks), dim3(BLOCK), lds_bytes<1>(), stream, a, it);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(merit_ls_kernel, dim3(waves), dim3(64), 0, stream, a);   // one wave per workgroup
    return hipGetLastError();
}

// Two parts once the batch fills the wave slots of the device (2 waves/SIMD) at least once;
// below that the waves of one launch already run side by side and splitting only adds launches.
// Measured (scripts/parts_sweep.sh, N = 20, K = 50, solves/s one part -> two parts): B = 4 096
// (1 366 waves) 226k -> 218k; B = 8 192 323k -> 361k; B = 16 384 423k -> 505k; B = 32 768
// 473k -> 509k; B = 65 536 491k -> 512k; N = 50, B = 16 384 (S = 2) 69.7k -> 74.8k; merit
// SQP (max_iter 30) B = 65 536 619k -> 672k, and at N = 10 1.42M -> 1.65M.
int sqp_parts_auto(int B, int N, int S, int cus) {
    const int G = 64 / lanes_per_instance(N, S);
    const long waves = ((long)B + G - 1) / G;
    return waves >= 8L * cus ? 2 : 1;   // 2 waves/SIMD x 4 SIMDs per CU: 2 048 slots on a whole MI355X
}

// One part's SQP loop on `stream`: (packing sort, QP [+ line search]) x sqp_iters over the
// instance range of `as`.  mark(): kernel-boundary events (single-part loop only).
template <class Mark>
static hipError_t sqp_iteration(const SolveArgs& as, int S, bool sorted, int it, hipStream_t stream, Mark&& mark) {
    hipError_t e = hipSuccess;
    if (sorted && it > 0) {
        hipLaunchKernelGGL(sort_by_iters_kernel, dim3((as.nI + 255) / 256), dim3(256), 0, stream, as.i0, as.nI,
                           pack_maxkey(as.p.qp_iters), as.wnit, as.wperm, as.whist, (it - 1) & 1);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = mark();
    if (e == hipSuccess)
        e = as.p.nlp_mode == 1 ? launch_sqp_merit(as, it, stream) : launch_qp_any(as, S, it, stream, true);
    if (e == hipSuccess) e = mark();
    return e;
}

hipError_t launch_sqp(const SolveArgs& a, int S, hipStream_t stream, hipEvent_t* ev, const SqpStreams* split) {
    const int G = 64 / lanes_per_instance(a.p.N, S);
    // parts of whole waves (the last part takes the remainder); at least one wave each
    int P = split ? split->parts : 1;
    if (P > SQP_MAX_PARTS) P = SQP_MAX_PARTS;
    const int wtot = (a.B + G - 1) / G;
    if (P > wtot) P = wtot;
    for (int q = 1; q < P; ++q)
        if (!split->aux[q - 1] || !split->join[q - 1] || !split->fork) P = 1;
    const bool fused = split && split->fused && a.p.nlp_mode == 0 && a.wdone && (S == 1 || S == 2);
    if (fused) P = 1;
    const bool two = P > 1;
    const int K = a.p.sqp_iters;
    int ne = 0;
    auto mark = [&]() { return ev ? hipEventRecord(ev[ne++], stream) : hipSuccess; };
    auto nomark = []() { return hipSuccess; };
    const unsigned gb = (unsigned)((a.B + 127) / 128);
    hipError_t e = mark();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(prologue_kernel, dim3(gb), dim3(128), 0, stream, a);
    e = hipGetLastError();
    const bool sorted = !fused && a.wperm && a.wnit && a.whist;
    SolveArgs as = a;
    as.i0 = 0;
    as.nI = a.B;
    if (!sorted) {   // identity order: the QP kernels must not read an unsorted permutation
        as.whist = nullptr;
        as.wperm = nullptr;
    }
    if (e == hipSuccess && sorted) {
        hipLaunchKernelGGL(iota_kernel, dim3(gb), dim3(128), 0, stream, a.B, a.wperm);
        e = hipGetLastError();
        if (e == hipSuccess)
            e = hipMemsetAsync(a.whist, 0, P * 4 * PACK_KEYS_MAX * sizeof(int32_t), stream);
    }
    if (e == hipSuccess) e = mark();
    if (fused) {
        if (e == hipSuccess)
            e = S == 1 ? (mfw_use(as.p, 1) ? launch_sqp_loop<1, true>(as, stream) : launch_sqp_loop<1>(as, stream))
                       : (as.p.factor_scan ? launch_sqp_loop<2, true>(as, stream) : launch_sqp_loop<2>(as, stream));
        ne = 2 * K + 1;
        if (e == hipSuccess) e = mark();
    } else if (!two) {
        for (int it = 0; it < K && e == hipSuccess; ++it) e = sqp_iteration(as, S, sorted, it, stream, mark);
    } else {
        // fork: the other parts wait for the prologue, then every part iterates independently
        SolveArgs ap[SQP_MAX_PARTS];
        hipStream_t sp[SQP_MAX_PARTS];
        for (int q = 0; q < P; ++q) {
            const int w0 = (int)((long)wtot * q / P), w1 = (int)((long)wtot * (q + 1) / P);
            ap[q] = as;
            ap[q].i0 = w0 * G;
            ap[q].nI = (q + 1 < P ? w1 * G : a.B) - w0 * G;
            if (sorted) ap[q].whist = a.whist + q * 4 * PACK_KEYS_MAX;
            sp[q] = q == 0 ? stream : split->aux[q - 1];
        }
        if (e == hipSuccess) e = hipEventRecord(split->fork, stream);
        for (int q = 1; q < P && e == hipSuccess; ++q) e = hipStreamWaitEvent(sp[q], split->fork, 0);
        for (int it = 0; it < K && e == hipSuccess; ++it)
            for (int q = 0; q < P && e == hipSuccess; ++q) e = sqp_iteration(ap[q], S, sorted, it, sp[q], nomark);
        for (int q = 1; q < P && e == hipSuccess; ++q) {
            e = hipEventRecord(split->join[q - 1], sp[q]);
            if (e == hipSuccess) e = hipStreamWaitEvent(stream, split->join[q - 1], 0);
        }
        ne = 2 * K + 1;
        if (e == hipSuccess) e = mark();
    }
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(epilogue_kernel, dim3(gb), dim3(128), 0, stream, a);
    e = hipGetLastError();
    if (e == hipSuccess) e = mark();
    return e;
}

// One QP (qsp_qp_solve): the workspace already holds the stage data.
hipError_t launch_qp(const SolveArgs& a, int S, hipStream_t stream) {
    SolveArgs as = a;
    as.i0 = 0;
    as.nI = a.B;
    return launch_qp_any(as, S, a.p.sqp_iters - 1, stream, false);
}

hipError_t launch_spline(const ShapeDev* shapes, const int32_t* sid, int n, const double* s, double* C, double* D,
                         double* Dd, double* kappa, hipStream_t stream) {
    hipLaunchKernelGGL(spline_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, shapes, sid, n, s, C, D, Dd, kappa);
    return hipGetLastError();
}
hipError_t launch_dynamics(const ShapeDev* shapes, const int32_t* sid, int n, const double* x, const double* u,
                           double* f, double* J, hipStream_t stream) {
    hipLaunchKernelGGL(dynamics_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, shapes, sid, n, x, u, f, J);
    return hipGetLastError();
}
hipError_t launch_rk4(const ShapeDev* shapes, const int32_t* sid, int n, double h, const double* x, const double* u,
                      double* xn, double* A, double* B, hipStream_t stream) {
    hipLaunchKernelGGL(rk4_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, shapes, sid, n, h, x, u, xn, A, B);
    return hipGetLastError();
}
hipError_t launch_vbound(const ShapeDev* shapes, const int32_t* sid, int n, CtrlParams cp, const double* s, double* vb,
                         hipStream_t stream) {
    hipLaunchKernelGGL(vbound_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, shapes, sid, n, cp, s, vb);
    return hipGetLastError();
}

}  // namespace qsp
