"""Batched acados-style OCP solver object over the HIP C ABI.

`OcpSolver` stands where the reference creates `acados_ocp(ocp_model, ocp_opts)`
(acados_nmpc/NMPC_controller.m:302-305) and drives it with `.set/.solve/.get`
(:154-157, 170, 334-348, 382-394, 403, 420; helper.m:253, 264-269).  Every per-lane
quantity carries a leading batch dimension B; one call solves B OCPs on the GPU.
Field names and stage semantics follow the acados MATLAB interface; unknown fields
raise KeyError, wrong shapes raise ValueError (the reference's MEX raises MATLAB
errors in both cases); numerical failure is reported per lane through 'status'.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, f64, i32, ptr


class OcpSolver:
    # nlp_solver_type (NMPC_controller.m:271): 'SQP_RTI' = fixed-K full steps (the BASELINE
    # metric), 'SQP' = merit backtracking + KKT tolerances (the reference's own options)
    NLP_MODES = {"SQP_RTI": 0, "SQP": 1}

    def __init__(self, N=20, batch=1, Ts=0.05, sqp_iters=50, qp_iters=20, stages_per_lane=0, device=0,
                 cost_scale_Ts=True, mu0=1.0, t_min=1e-2, frac=0.995, sigma_min=1e-2, mu_stop=1e-10, res_stop=1e-10,
                 qp_tol_stat=1e-10, qp_tol_eq=1e-10, stage0_s_bound=True, qp_stall_iters=3, qp_stall_alpha=1e-3,
                 qp_mu_max=1e100, factor_scan=False,
                 nlp_solver_type="SQP_RTI", tol=1e-6, ls_alpha_min=0.05, ls_alpha_red=0.7, ls_eps=1e-4,
                 qp_solver_cond_N=None, timings=False):
        # qp_solver_cond_N (NMPC_controller.m:276) selects HPIPM's partial condensing, a different
        # factorisation of the same QP.  The kernel factorises stage-wise at every value: condensed
        # blocks measured 1.16-3.1x slower (profiles/r03/cond_block.txt).  The
        # value is checked (1..N) and kept as .qp_solver_cond_N.
        if qp_solver_cond_N is not None and (int(qp_solver_cond_N) != qp_solver_cond_N
                                             or not 1 <= qp_solver_cond_N <= N):
            raise ValueError("qp_solver_cond_N must be an integer in 1..N")
        self.qp_solver_cond_N = int(N if qp_solver_cond_N is None else qp_solver_cond_N)
        L = _lib.lib()
        o = _lib.Options()
        L.qsp_default_options(C.byref(o))
        o.N, o.batch, o.Ts = int(N), int(batch), float(Ts)
        o.sqp_iters, o.qp_iters, o.stages_per_lane, o.device = int(sqp_iters), int(qp_iters), int(stages_per_lane), int(device)
        o.cost_scale_Ts = 1 if cost_scale_Ts else 0
        o.mu0, o.t_min, o.frac, o.sigma_min, o.mu_stop = mu0, t_min, frac, sigma_min, mu_stop
        o.res_stop = res_stop
        o.qp_tol_stat, o.qp_tol_eq = float(qp_tol_stat), float(qp_tol_eq)
        o.stage0_s_bound = 1 if stage0_s_bound else 0
        o.qp_stall_iters, o.qp_stall_alpha = int(qp_stall_iters), float(qp_stall_alpha)
        o.qp_mu_max = float(qp_mu_max)
        # two stages per lane (N + 1 > 32): the factorisation as an associative scan (faster, less
        # accurate; include/qsp_nmpc.h)
        o.factor_scan = 1 if factor_scan else 0
        if nlp_solver_type not in self.NLP_MODES:
            raise ValueError(f"nlp_solver_type must be one of {tuple(self.NLP_MODES)}")
        o.nlp_mode = self.NLP_MODES[nlp_solver_type]
        o.tol_stat = o.tol_eq = o.tol_ineq = o.tol_comp = float(tol)
        o.ls_alpha_min, o.ls_alpha_red, o.ls_eps = float(ls_alpha_min), float(ls_alpha_red), float(ls_eps)
        h = C.c_void_p()
        check(L.qsp_create(C.byref(o), C.byref(h)), "qsp_create")
        self._L, self._h, self.opts = L, h, o
        self.N, self.B, self.Ts = o.N, o.batch, o.Ts
        Bn, Nn = self.B, self.N
        self._x0 = np.zeros((Bn, 4))
        self._yref = np.zeros((Bn, Nn, 6))
        self._yref_e = np.zeros((Bn, 4))
        self._X = np.zeros((Bn, Nn + 1, 4))
        self._U = np.zeros((Bn, Nn, 2))
        self._PI = np.zeros((Bn, Nn, 4))
        self._W = np.array([1.0, 1.0, 1e-3, 0.0, 1e-3, 1e-3])
        self._We = np.array([2e5, 2e5, 20.0, 0.0])
        self._lh = np.array([-0.06, 0.0, -0.05])
        self._uh = np.array([0.011, 0.03, 0.05])
        self._dirty = set(["x0", "yref", "init"])
        self.n_shapes = 0
        # timings=True: per-kernel HIP events around every solve, for get('time_lin'/'time_qp_sol')
        self._timings = bool(timings)
        self._last_times = None

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None):
            self._L.qsp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def layout(self):
        S, L = C.c_int32(), C.c_int32()
        check(self._L.qsp_get_layout(self._h, C.byref(S), C.byref(L)), "qsp_get_layout")
        return S.value, L.value

    FACTOR_WALKS = {0: "lane walk", 1: "matrix cores (v_mfma_f64_4x4x4_4b_f64)", 2: "associative scan"}

    def factor_walk(self):
        """How the QPs walk the horizon, as the library reports it (qsp_get_factor_walk, QSP_WALK_*)."""
        w = C.c_int32()
        check(self._L.qsp_get_factor_walk(self._h, C.byref(w)), "qsp_get_factor_walk")
        return self.FACTOR_WALKS[w.value]

    # --------------------------------------------------------------- model
    def set_shapes(self, shapes, shape_id=None):
        arr = (_lib.Shape * len(shapes))(*shapes)
        check(self._L.qsp_set_shapes(self._h, arr, len(shapes)), "qsp_set_shapes")
        self.n_shapes = len(shapes)
        if shape_id is not None:
            self.set_shape_ids(shape_id)

    def set_shape_ids(self, shape_id):
        sid = i32(np.broadcast_to(np.asarray(shape_id, np.int32), (self.B,)))
        check(self._L.qsp_set_shape_ids(self._h, ptr(sid)), "qsp_set_shape_ids")

    # ----------------------------------------------------------------- set
    def _lanes(self, v, width):
        v = np.asarray(v, np.float64)
        if v.shape == (width,) or v.shape == (width, 1):
            return np.broadcast_to(v.reshape(width), (self.B, width))
        if v.shape == (self.B, width):
            return v
        raise ValueError(f"expected ({width},) or ({self.B},{width}), got {v.shape}")

    def set(self, field, value, stage=None):
        N = self.N
        if field == "constr_x0":
            self._x0[:] = self._lanes(value, 4)
            self._dirty.add("x0")
        elif field == "cost_y_ref":
            if stage is None:
                v = np.asarray(value, np.float64)
                if v.shape not in ((self.B, N, 6), (N, 6)):
                    raise ValueError(f"cost_y_ref without stage expects (B,N,6) or (N,6), got {v.shape}")
                self._yref[:] = v
            else:
                if not 0 <= stage < N:
                    raise ValueError(f"cost_y_ref stage {stage} out of range 0..{N - 1}")
                self._yref[:, stage] = self._lanes(value, 6)
            self._dirty.add("yref")
        elif field == "cost_y_ref_e":
            if stage is not None and stage != N:
                raise ValueError("cost_y_ref_e is only defined at stage N")
            self._yref_e[:] = self._lanes(value, 4)
            self._dirty.add("yref")
        elif field == "cost_W":
            W = np.asarray(value, np.float64)
            if W.ndim == 2:
                if np.any(W != np.diag(np.diag(W))):
                    raise ValueError("cost_W: only diagonal weights are supported")
                W = np.diag(W)
            if stage == N:
                if W.shape != (4,):
                    raise ValueError("cost_W at stage N must be 4x4")
                self._We[:] = W
            else:
                if W.shape != (6,):
                    raise ValueError("cost_W must be 6x6")
                self._W[:] = W
            check(self._L.qsp_set_cost_W(self._h, ptr(f64(self._W)), ptr(f64(self._We))), "qsp_set_cost_W")
        elif field in ("constr_lh", "constr_uh"):
            v = np.asarray(value, np.float64).reshape(3)
            (self._lh if field == "constr_lh" else self._uh)[:] = v
            check(self._L.qsp_set_constr_h(self._h, ptr(f64(self._lh)), ptr(f64(self._uh))), "qsp_set_constr_h")
        elif field == "init_x":
            v = np.asarray(value, np.float64)
            self._X[:] = v.reshape(self._X.shape) if v.size == self._X.size else np.broadcast_to(v, self._X.shape)
            self._dirty.add("init")
        elif field == "init_u":
            v = np.asarray(value, np.float64)
            self._U[:] = v.reshape(self._U.shape) if v.size == self._U.size else np.broadcast_to(v, self._U.shape)
            self._dirty.add("init")
        elif field == "init_pi":
            v = np.asarray(value, np.float64)
            self._PI[:] = v.reshape(self._PI.shape) if v.size == self._PI.size else np.broadcast_to(v, self._PI.shape)
            self._dirty.add("init")
        else:
            raise KeyError(f"OcpSolver.set: unknown field '{field}'")

    def set_ctrl_params(self, v_alpha, d_v_bound, t_angle0, u_n_lb, u_t_ub):
        check(self._L.qsp_set_ctrl_params(self._h, v_alpha, d_v_bound, t_angle0, u_n_lb, u_t_ub), "qsp_set_ctrl_params")

    # --------------------------------------------------------------- solve
    def _flush(self):
        if "x0" in self._dirty:
            check(self._L.qsp_set_x0(self._h, ptr(f64(self._x0))), "qsp_set_x0")
        if "yref" in self._dirty:
            check(self._L.qsp_set_yref(self._h, ptr(f64(self._yref)), ptr(f64(self._yref_e))), "qsp_set_yref")
        if "init" in self._dirty:
            check(self._L.qsp_set_init(self._h, ptr(f64(self._X)), ptr(f64(self._U)), ptr(f64(self._PI))),
                  "qsp_set_init")
        self._dirty.clear()

    def _timed(self, fn, *args):
        if self._timings:
            self.set_kernel_timing(1)
        fn(*args)
        if self._timings:
            self._last_times = self.kernel_times()

    def solve(self):
        self._flush()
        self._timed(lambda: check(self._L.qsp_solve(self._h), "qsp_solve"))

    # ----------------------------------------------------------------- get
    def get(self, field, stage=None):
        B, N = self.B, self.N
        if field in ("x", "u", "pi"):
            shape = {"x": (B, N + 1, 4), "u": (B, N, 2), "pi": (B, N, 4)}[field]
            out = np.zeros(shape)
            fn = {"x": self._L.qsp_get_x, "u": self._L.qsp_get_u, "pi": self._L.qsp_get_pi}[field]
            check(fn(self._h, ptr(out)), f"get('{field}')")
            return out if stage is None else out[:, stage]
        if field in ("status", "sqp_iter", "qp_iter", "qp_capped", "qp_stalled"):
            out = np.zeros(B, np.int32)
            fn = {"status": self._L.qsp_get_status, "sqp_iter": self._L.qsp_get_sqp_iter,
                  "qp_iter": self._L.qsp_get_qp_iter, "qp_capped": self._L.qsp_get_qp_capped,
                  "qp_stalled": self._L.qsp_get_qp_stalled}[field]
            check(fn(self._h, ptr(out)), f"get('{field}')")
            return out
        if field == "residuals":   # acados res_stat/eq/ineq/comp of the last KKT test (nlp_mode 1)
            out = np.zeros((B, 4))
            check(self._L.qsp_get_residuals(self._h, ptr(out)), "get('residuals')")
            return out
        if field == "time_tot":
            ms = C.c_double()
            check(self._L.qsp_get_time_tot(self._h, C.byref(ms)), "get('time_tot')")
            return ms.value * 1e-3
        if field in ("time_lin", "time_qp_sol"):                # helper.m:264-269, seconds
            if self._last_times is None:
                raise KeyError(f"get('{field}') needs OcpSolver(..., timings=True) and a solve")
            key = "linearize" if field == "time_lin" else "qp_step"
            return self._last_times[key][0] * 1e-3
        raise KeyError(f"OcpSolver.get: unknown field '{field}'")

    def get_u0(self):
        out = np.zeros((self.B, 2))
        check(self._L.qsp_get_u0(self._h, ptr(out)), "qsp_get_u0")
        return out

    def get_cost(self):
        out = np.zeros(self.B)
        check(self._L.qsp_get_cost(self._h, ptr(out)), "qsp_get_cost")
        return out

    # --------------------------------------------------- controller level
    def set_reference_trajectory(self, traj):
        """traj: 6 x T (MATLAB layout) or T x 6."""
        t = np.asarray(traj, np.float64)
        if t.shape[0] == 6 and t.ndim == 2 and t.shape[1] != 6:
            t = t.T
        t = f64(t)
        if t.ndim != 2 or t.shape[1] != 6:
            raise ValueError("reference trajectory must be 6 x T")
        check(self._L.qsp_set_reference_trajectory(self._h, ptr(t), t.shape[0]), "qsp_set_reference_trajectory")
        self._traj_shape = t.shape

    def set_reference_trajectories(self, traj):
        """Per-lane reference tables: (B, T, 6)."""
        t = f64(traj)
        if t.ndim != 3 or t.shape[0] != self.B or t.shape[2] != 6:
            raise ValueError(f"per-lane references must be (B={self.B}, T, 6), got {t.shape}")
        check(self._L.qsp_set_reference_trajectories(self._h, ptr(t), t.shape[1]), "qsp_set_reference_trajectories")
        self._traj_shape = t.shape

    def gen_straight_lines(self, x0, xf, t0, tf, auto_angle=False):
        """Device-generated TrajectoryGenerator.straight_line per lane (x0, xf: (B, 3)); returns T."""
        a = f64(self._lanes(x0, 3))
        b = f64(self._lanes(xf, 3))
        T = C.c_int32()
        check(self._L.qsp_gen_straight_lines(self._h, ptr(a), ptr(b), float(t0), float(tf), int(bool(auto_angle)),
                                             C.byref(T)), "qsp_gen_straight_lines")
        self._traj_shape = (self.B, T.value, 6)
        return T.value

    def get_reference_trajectories(self):
        out = np.zeros(self._traj_shape)
        check(self._L.qsp_get_reference_trajectories(self._h, ptr(out)), "qsp_get_reference_trajectories")
        return out

    def controller_solve(self, x0, index_time):
        x0 = f64(self._lanes(x0, 4))
        idx = i32(np.broadcast_to(np.asarray(index_time, np.int32), (self.B,)))
        self._timed(lambda: check(self._L.qsp_controller_solve(self._h, ptr(x0), ptr(idx)), "qsp_controller_solve"))
        return self.get_u0()

    def closed_loop(self, x0, n_steps, index0=1, noise=None, plant_delay=0.0, disturbance=False, t_dist=0,
                    amplitude=None):
        """Device-resident closed loop (helper.m:195-322): returns X (B, n+1, 4) (plant states after
        disturbance and noise), Xsim (B, n, 4) (the delay-predicted states the solver sees), U (B, n, 2),
        status (B, n).  noise: (n, B, 4) additive state noise before each solve, or None; plant_delay [s];
        disturbance at the 1-based step t_dist with per-lane amplitude (y offset + contact re-projection)."""
        n = int(n_steps)
        x0 = f64(self._lanes(x0, 4))
        idx = i32(np.broadcast_to(np.asarray(index0, np.int32), (self.B,)))
        nz = None if noise is None else f64(noise, (n, self.B, 4))
        amp = None if amplitude is None else f64(np.broadcast_to(np.asarray(amplitude, np.float64), (self.B,)))
        o = _lib.ClosedLoopOpts()
        o.plant_delay, o.disturbance, o.t_dist = float(plant_delay), 1 if disturbance else 0, int(t_dist)
        o.amplitude = None if amp is None else amp.ctypes.data
        X = np.zeros((self.B, n + 1, 4))
        Xs = np.zeros((self.B, n, 4))
        U = np.zeros((self.B, n, 2))
        st = np.zeros((self.B, n), np.int32)
        check(self._L.qsp_closed_loop_ex(self._h, C.byref(o), ptr(x0), ptr(idx), n, ptr(nz), ptr(X), ptr(Xs), ptr(U),
                                         ptr(st)), "qsp_closed_loop_ex")
        return dict(X=X, Xsim=Xs, U=U, status=st)

    # ------------------------------------------------ delay compensation
    def set_delay_comp(self, delay):
        """set_delay_comp (NMPC_controller.m:106-110): delay_buff_comp = ceil(delay / Ts)."""
        check(self._L.qsp_set_delay_comp(self._h, float(delay)), "qsp_set_delay_comp")

    def delay_cols(self):
        d = C.c_int32()
        check(self._L.qsp_get_delay_comp(self._h, C.byref(d)), "qsp_get_delay_comp")
        return d.value

    def delay_buffer_sim(self, x):
        """delay_buffer_sim (NMPC_controller.m:112-120) on the device, per lane."""
        x = f64(self._lanes(x, 4))
        out = np.zeros((self.B, 4))
        check(self._L.qsp_delay_buffer_sim(self._h, ptr(x), ptr(out)), "qsp_delay_buffer_sim")
        return out

    def delay_buffer_push(self, u):
        """u_buff_contr = [u, u_buff_contr(:, 1:end-1)] (helper.m:255)."""
        u = f64(self._lanes(u, 2))
        check(self._L.qsp_delay_buffer_push(self._h, ptr(u)), "qsp_delay_buffer_push")

    def reproject_contact(self, px, py, s0, shape_id=None):
        px = f64(px).ravel()
        n = len(px)
        py = f64(np.broadcast_to(py, (n,)))
        s0 = f64(np.broadcast_to(s0, (n,)))
        out = np.zeros(n)
        check(self._L.qsp_reproject_contact(self._h, n, ptr(self._sid(shape_id, n)), ptr(px), ptr(py), ptr(s0),
                                            ptr(out)), "qsp_reproject_contact")
        return out

    def controller_reset(self):
        check(self._L.qsp_controller_reset(self._h), "qsp_controller_reset")

    # --------------------------------------------------------- device path
    def solve_device(self, io, stream=None):
        check(self._L.qsp_solve_device(self._h, C.byref(io), C.c_void_p(stream) if stream else None), "qsp_solve_device")

    def synchronize(self):
        check(self._L.qsp_synchronize(self._h), "qsp_synchronize")

    def set_stream_parts(self, parts):
        """SQP loop in 1 or 2 parts on their own HIP streams (0 = auto); results are identical."""
        check(self._L.qsp_set_stream_parts(self._h, int(parts)), "qsp_set_stream_parts")

    def stream_parts(self):
        p = C.c_int32()
        check(self._L.qsp_get_stream_parts(self._h, C.byref(p)), "qsp_get_stream_parts")
        return p.value

    def set_kernel_timing(self, max_solves):
        """Record HIP events at every kernel boundary of the next `max_solves` solves."""
        check(self._L.qsp_set_kernel_timing(self._h, int(max_solves)), "qsp_set_kernel_timing")

    KERNELS = ("prologue", "linearize", "qp_step", "epilogue")

    def kernel_times(self):
        """{kernel: (total_ms, launches)} over the timed solves since the last call."""
        ms = (C.c_double * 4)()
        n = (C.c_int32 * 4)()
        check(self._L.qsp_get_kernel_times(self._h, ms, n), "qsp_get_kernel_times")
        return {k: (ms[i], n[i]) for i, k in enumerate(self.KERNELS)}

    # ----------------------------------------------------- building blocks
    def _sid(self, shape_id, n):
        return i32(np.broadcast_to(np.asarray(0 if shape_id is None else shape_id, np.int32), (n,)))

    def eval_spline(self, sigma, shape_id=None):
        s = f64(sigma).ravel()
        n = len(s)
        Cv, D, Dd, kap = np.zeros((n, 2)), np.zeros((n, 2)), np.zeros((n, 2)), np.zeros(n)
        check(self._L.qsp_eval_spline(self._h, n, ptr(self._sid(shape_id, n)), ptr(s), ptr(Cv), ptr(D), ptr(Dd),
                                      ptr(kap)), "qsp_eval_spline")
        return Cv, D, Dd, kap

    def eval_dynamics(self, x, u, shape_id=None):
        x = f64(x).reshape(-1, 4)
        u = f64(u).reshape(-1, 2)
        n = len(x)
        f, J = np.zeros((n, 4)), np.zeros((n, 4, 6))
        check(self._L.qsp_eval_dynamics(self._h, n, ptr(self._sid(shape_id, n)), ptr(x), ptr(u), ptr(f), ptr(J)),
              "qsp_eval_dynamics")
        return f, J

    def eval_rk4(self, x, u, h=None, shape_id=None):
        x = f64(x).reshape(-1, 4)
        u = f64(u).reshape(-1, 2)
        n = len(x)
        xn, A, Bm = np.zeros((n, 4)), np.zeros((n, 4, 4)), np.zeros((n, 4, 2))
        check(self._L.qsp_eval_rk4(self._h, n, ptr(self._sid(shape_id, n)), self.Ts if h is None else h, ptr(x),
                                   ptr(u), ptr(xn), ptr(A), ptr(Bm)), "qsp_eval_rk4")
        return xn, A, Bm

    def eval_vbound(self, s, shape_id=None):
        s = f64(s).ravel()
        n = len(s)
        vb = np.zeros(n)
        check(self._L.qsp_eval_vbound(self._h, n, ptr(self._sid(shape_id, n)), ptr(s), ptr(vb)), "qsp_eval_vbound")
        return vb

    def qp_solve(self, A, B, b, H, g, lo, hi, dx0):
        N = self.N
        nb = A.shape[0]
        arrs = [f64(a) for a in (A, B, b, H, g, lo, hi, dx0)]
        dx, du = np.zeros((nb, N + 1, 4)), np.zeros((nb, N, 2))
        pi, lam = np.zeros((nb, N, 4)), np.zeros((nb, N, 6))
        iters = np.zeros(nb, np.int32)
        qst = np.zeros(nb, np.int32)
        check(self._L.qsp_qp_solve(self._h, nb, *[ptr(a) for a in arrs], ptr(dx), ptr(du), ptr(pi), ptr(lam),
                                   ptr(iters), ptr(qst)), "qsp_qp_solve")
        return dict(dx=dx, du=du, pi=pi, lam=lam, iters=iters, qp_status=qst)
