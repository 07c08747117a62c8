"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Loads oracle/build/libqsp_oracle.so (built by oracle/Makefile).  Used by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg only.

Two restatements of the reference path share one interface:
  Oracle(...)            the literal restatement (qsp_oracle.c: full basis sum, forward AD,
                         a dense Riccati interior point) -- pins the formulas;
  Oracle(..., twin=True) the kernel-order twin (qsp_twin.c: the device library's formulation
                         and operation order, explicit fma) -- reproduces the device bit for bit.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from .shapes_np import shape_table

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libqsp_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
    return _lib


def _threads(n):
    """OpenMP threads of a call: n, or (n = 0) the job's share -- OMP_NUM_THREADS, else the CPUs of the
    affinity mask.  Always explicit, because omp_set_num_threads persists in the process: a call
    with n = 1 (a thread-scaling sample) would otherwise leave every later call on one thread."""
    if n and n > 0:
        return int(n)
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


class Opts(C.Structure):
    _fields_ = [
        ("N", C.c_int32), ("sqp_iters", C.c_int32), ("qp_iters", C.c_int32), ("stage0_s_bound", C.c_int32),
        ("Ts", C.c_double), ("tau", C.c_double),
        ("W", C.c_double * 6), ("We", C.c_double * 4), ("lh", C.c_double * 3), ("uh", C.c_double * 3),
        ("mu0", C.c_double), ("t_min", C.c_double), ("frac", C.c_double),
        ("sigma_min", C.c_double), ("mu_stop", C.c_double),
        ("v_alpha", C.c_double), ("d_v", C.c_double), ("t_angle0", C.c_double),
        ("u_n_lb", C.c_double), ("u_t_ub", C.c_double),
        ("nlp_mode", C.c_int32), ("pad_", C.c_int32),
        ("tol_stat", C.c_double), ("tol_eq", C.c_double), ("tol_ineq", C.c_double), ("tol_comp", C.c_double),
        ("ls_alpha_min", C.c_double), ("ls_alpha_red", C.c_double), ("ls_eps", C.c_double),
        ("res_stop", C.c_double),
        ("qp_tol_stat", C.c_double), ("qp_tol_eq", C.c_double),
        ("qp_stall_alpha", C.c_double), ("qp_stall_iters", C.c_int32), ("stages_per_lane", C.c_int32),
        ("qp_mu_max", C.c_double),
        ("model_probe", C.c_double), ("probe_seed", C.c_int32), ("factor_scan", C.c_int32),
        ("lane_walk", C.c_int32),
    ]


def make_opts(N=20, sqp_iters=50, qp_iters=20, Ts=0.05, tau=None,
              W=(1.0, 1.0, 1e-3, 0.0, 1e-3, 1e-3), We=(2e5, 2e5, 20.0, 0.0),
              lh=(-0.06, 0.0, -0.05), uh=(0.011, 0.03, 0.05),
              mu0=1.0, t_min=1e-2, frac=0.995, sigma_min=1e-2, mu_stop=1e-10, res_stop=1e-10, v_alpha=1.0, d_v=0.0, t_angle0=3.0,
              u_n_lb=0.0, u_t_ub=0.05, nlp_mode=0, tol=1e-6, ls_alpha_min=0.05, ls_alpha_red=0.7, ls_eps=1e-4,
              qp_tol_stat=1e-10, qp_tol_eq=1e-10, stage0_s_bound=1, qp_stall_alpha=1e-3, qp_stall_iters=3,
              qp_mu_max=1e100, stages_per_lane=0, model_probe=0.0, probe_seed=0, factor_scan=0, lane_walk=0):
    o = Opts()
    o.N, o.sqp_iters, o.qp_iters, o.stage0_s_bound = N, sqp_iters, qp_iters, int(stage0_s_bound)
    o.qp_tol_stat, o.qp_tol_eq = qp_tol_stat, qp_tol_eq
    o.qp_stall_alpha, o.qp_stall_iters = qp_stall_alpha, int(qp_stall_iters)
    o.qp_mu_max, o.stages_per_lane = qp_mu_max, int(stages_per_lane)
    o.model_probe, o.probe_seed = float(model_probe), int(probe_seed)
    o.factor_scan = int(factor_scan)
    o.lane_walk = int(lane_walk)
    o.Ts = Ts
    o.tau = Ts if tau is None else tau
    o.W[:] = W
    o.We[:] = We
    o.lh[:] = lh
    o.uh[:] = uh
    o.mu0, o.t_min, o.frac = mu0, t_min, frac
    o.sigma_min, o.mu_stop = sigma_min, mu_stop
    o.res_stop = res_stop
    o.v_alpha, o.d_v, o.t_angle0 = v_alpha, d_v, t_angle0
    o.u_n_lb, o.u_t_ub = u_n_lb, u_t_ub
    o.nlp_mode = nlp_mode
    o.tol_stat = o.tol_eq = o.tol_ineq = o.tol_comp = tol
    o.ls_alpha_min, o.ls_alpha_red, o.ls_eps = ls_alpha_min, ls_alpha_red, ls_eps
    return o


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    def __init__(self, names=("santal", "balea", "montana", "pulirapid"), max_ctrl=64, tab=None, twin=False):
        # tab: optional explicit shape table (n_ctrl, ctrl, knots, params) instead of named PLY objects
        self.tab = shape_table(names, max_ctrl) if tab is None else tab
        t = self.tab
        self._n = np.ascontiguousarray(t["n_ctrl"], np.int32)
        self._c = np.ascontiguousarray(t["ctrl"], np.float64)
        self._k = np.ascontiguousarray(t["knots"], np.float64)
        self._pr = np.ascontiguousarray(t["params"], np.float64)
        self._mc = int(max_ctrl)
        self.L = lib()
        self.twin = bool(twin)
        self._pre = "tw_" if twin else "or_"

    def _f(self, name):
        return getattr(self.L, self._pre + name)

    def _shape_args(self):
        return (_p(self._n), _p(self._c), _p(self._k), _p(self._pr), C.c_int(self._mc))

    @staticmethod
    def _ids(shape_id, n):
        sid = np.zeros(n, np.int32) if shape_id is None else np.asarray(shape_id, np.int32)
        if sid.shape == ():
            sid = np.full(n, int(sid), np.int32)
        return np.ascontiguousarray(sid)

    def spline(self, s, shape_id=None):
        s = np.ascontiguousarray(s, np.float64).ravel()
        n = len(s)
        sid = self._ids(shape_id, n)
        Cv, dC, D, dD = (np.zeros((n, 2)) for _ in range(4))
        kap = np.zeros(n)
        if self.twin:   # (C, C', C'', kappa): the device's spline outputs
            self.L.tw_spline_eval(*self._shape_args(), C.c_int32(n), _p(sid), _p(s), _p(Cv), _p(D), _p(dD), _p(kap))
            return Cv, D, dD, kap
        self.L.or_spline_eval(*self._shape_args(), C.c_int32(n), _p(sid), _p(s), _p(Cv), _p(dC), _p(D), _p(dD), _p(kap))
        return Cv, dC, D, dD, kap

    def dynamics(self, x, u, shape_id=None):
        x = np.ascontiguousarray(x, np.float64).reshape(-1, 4)
        u = np.ascontiguousarray(u, np.float64).reshape(-1, 2)
        n = len(x)
        sid = self._ids(shape_id, n)
        f = np.zeros((n, 4))
        J = np.zeros((n, 4, 6))
        self._f('dynamics')(*self._shape_args(), C.c_int32(n), _p(sid), _p(x), _p(u), _p(f), _p(J))
        return f, J

    def rk4(self, x, u, h=0.05, shape_id=None):
        x = np.ascontiguousarray(x, np.float64).reshape(-1, 4)
        u = np.ascontiguousarray(u, np.float64).reshape(-1, 2)
        n = len(x)
        sid = self._ids(shape_id, n)
        xn = np.zeros((n, 4))
        A = np.zeros((n, 4, 4))
        B = np.zeros((n, 4, 2))
        self._f('rk4')(*self._shape_args(), C.c_int32(n), _p(sid), C.c_double(h), _p(x), _p(u), _p(xn), _p(A), _p(B))
        return xn, A, B

    def vbound(self, s, opts, shape_id=None):
        s = np.ascontiguousarray(s, np.float64).ravel()
        n = len(s)
        sid = self._ids(shape_id, n)
        vb = np.zeros(n)
        self._f('vbound')(*self._shape_args(), C.byref(opts), C.c_int32(n), _p(sid), _p(s), _p(vb))
        return vb

    def qp(self, opts, A, B, b, H, g, lo, hi, act, dx0):
        N = opts.N
        nb = A.shape[0]
        arrs = [np.ascontiguousarray(a, np.float64) for a in (A, B, b, H, g, lo, hi)]
        act = np.ascontiguousarray(act, np.uint8)
        dx0 = np.ascontiguousarray(dx0, np.float64)
        dx = np.zeros((nb, N + 1, 4))
        du = np.zeros((nb, N, 2))
        pi = np.zeros((nb, N, 4))
        lam = np.zeros((nb, N, 6))
        iters = np.zeros(nb, np.int32)
        qst = np.zeros(nb, np.int32)
        r = self._f('qp_batch')(C.byref(opts), C.c_int32(nb), *[_p(a) for a in arrs], _p(act), _p(dx0),
                               _p(dx), _p(du), _p(pi), _p(lam), _p(iters), _p(qst))
        return dict(dx=dx, du=du, pi=pi, lam=lam, iters=iters, fail=r, qp_status=qst)

    def ocp_solve(self, opts, x0, yref, yref_e, X=None, U=None, PI=None, shape_id=None, nthreads=0):
        N = opts.N
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 4)
        nb = len(x0)
        sid = self._ids(shape_id, nb)
        yref = np.ascontiguousarray(np.broadcast_to(yref, (nb, N, 6)), np.float64)
        yref_e = np.ascontiguousarray(np.broadcast_to(yref_e, (nb, 4)), np.float64)
        X = np.zeros((nb, N + 1, 4)) if X is None else np.array(X, np.float64, copy=True).reshape(nb, N + 1, 4)
        U = np.zeros((nb, N, 2)) if U is None else np.array(U, np.float64, copy=True).reshape(nb, N, 2)
        PI = np.zeros((nb, N, 4)) if PI is None else np.array(PI, np.float64, copy=True).reshape(nb, N, 4)
        lam = np.zeros((nb, N, 6))
        status = np.zeros(nb, np.int32)
        iters = np.zeros(nb, np.int32)
        qp_iter = np.zeros(nb, np.int32)
        cost = np.zeros(nb)
        capped = np.zeros(nb, np.int32)
        stalled = np.zeros(nb, np.int32)
        self._f("ocp_solve")(*self._shape_args(), C.byref(opts), C.c_int32(nb), _p(sid), _p(x0), _p(yref), _p(yref_e),
                             _p(X), _p(U), _p(PI), _p(lam), _p(status), _p(iters), _p(qp_iter), _p(cost),
                             C.c_int(_threads(nthreads)), _p(capped), _p(stalled))
        return dict(X=X, U=U, PI=PI, lam=lam, status=status, iters=iters, qp_iter=qp_iter, cost=cost, qp_capped=capped,
                    qp_stalled=stalled)

    def controller_solve(self, opts, x0, traj, index_time, warm, shape_id=None, nthreads=0, delay_cols=0):
        """warm: dict with X (nb,N+1,4), U (nb,N,2), PI (nb,N,4), valid (nb,) uint8 — updated in place.
        traj: (T, 6) shared, or (nb, T, 6) per lane (twin only)."""
        N = opts.N
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 4)
        nb = len(x0)
        sid = self._ids(shape_id, nb)
        per_lane = np.ndim(traj) == 3
        if per_lane and not self.twin:
            raise ValueError("per-lane reference tables: twin only")
        traj = np.ascontiguousarray(traj, np.float64)
        T = traj.shape[1] if per_lane else traj.reshape(-1, 6).shape[0]
        idx = np.ascontiguousarray(np.broadcast_to(np.asarray(index_time, np.int32), (nb,)), np.int32)
        u0 = np.zeros((nb, 2))
        status = np.zeros(nb, np.int32)
        iters = np.zeros(nb, np.int32)
        qp_iter = np.zeros(nb, np.int32)
        cost = np.zeros(nb)
        capped = np.zeros(nb, np.int32)
        stalled = np.zeros(nb, np.int32)
        args = [*self._shape_args(), C.byref(opts), C.c_int32(nb), _p(sid), _p(x0), _p(traj), C.c_int32(T), _p(idx),
                _p(warm["X"]), _p(warm["U"]), _p(warm["PI"]), _p(warm["valid"]), _p(u0), _p(status), _p(iters),
                _p(qp_iter), _p(cost), C.c_int(_threads(nthreads)), _p(capped), C.c_int32(int(delay_cols))]
        if self.twin:
            self.L.tw_controller_solve(*args, C.c_int32(int(per_lane)), _p(stalled))
        else:
            self.L.or_controller_solve(*args, _p(stalled))
        return dict(u0=u0, status=status, iters=iters, qp_iter=qp_iter, cost=cost, qp_capped=capped, qp_stalled=stalled)

    def controller_solve_ext(self, opts, x0, traj, index_time, warm, shape_id=None, nthreads=0, delay_cols=0,
                             precision="quad"):
        """controller_solve of the LITERAL restatement evaluated in extended precision (qsp_oracle.c
        built with OR_EXT: "long" = long double, "quad" = __float128); double in/out."""
        if self.twin:
            raise ValueError("extended precision: literal restatement only")
        N = opts.N
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 4)
        nb = len(x0)
        sid = self._ids(shape_id, nb)
        traj = np.ascontiguousarray(traj, np.float64).reshape(-1, 6)
        idx = np.ascontiguousarray(np.broadcast_to(np.asarray(index_time, np.int32), (nb,)), np.int32)
        u0 = np.zeros((nb, 2))
        status = np.zeros(nb, np.int32)
        iters = np.zeros(nb, np.int32)
        qp_iter = np.zeros(nb, np.int32)
        cost = np.zeros(nb)
        fn = {"long": self.L.orx_controller_solve_l, "quad": self.L.orx_controller_solve_q}[precision]
        r = fn(*self._shape_args(), C.c_int32(len(self._n)), C.byref(opts), C.c_int32(nb), _p(sid), _p(x0), _p(traj),
               C.c_int32(len(traj)), _p(idx), _p(warm["X"]), _p(warm["U"]), _p(warm["PI"]), _p(warm["valid"]), _p(u0),
               _p(status), _p(iters), _p(qp_iter), _p(cost), C.c_int(_threads(nthreads)), C.c_int32(int(delay_cols)))
        if r != 0:
            raise ValueError("orx_controller_solve: bad arguments")
        return dict(u0=u0, status=status, iters=iters, qp_iter=qp_iter, cost=cost)

    def closed_loop(self, opts, x0, traj, n_steps, index0=1, shape_id=None, noise=None, delay_cols=0,
                    plant_delay_cols=0, dist_step=0, dist_amp=None, xwidth=None, nthreads=0, ubc0=None):
        """helper.m:195-322 closed loop (see or_closed_loop).  Returns X (nb, n+1, 4), Xsim (nb, n, 4),
        U (nb, n, 2), status (nb, n)."""
        x0 = np.ascontiguousarray(x0, np.float64).reshape(-1, 4)
        nb, n = len(x0), int(n_steps)
        sid = self._ids(shape_id, nb)
        traj = np.ascontiguousarray(traj, np.float64).reshape(-1, 6)
        idx = np.ascontiguousarray(np.broadcast_to(np.asarray(index0, np.int32), (nb,)), np.int32)
        nz = None if noise is None else np.ascontiguousarray(noise, np.float64).reshape(n, nb, 4)
        amp = np.ascontiguousarray(np.broadcast_to(np.asarray(0.0 if dist_amp is None else dist_amp, np.float64), (nb,)))
        xw = np.ascontiguousarray(np.zeros(len(self._n)) if xwidth is None else np.asarray(xwidth, np.float64))
        X = np.zeros((nb, n + 1, 4))
        Xs = np.zeros((nb, n, 4))
        U = np.zeros((nb, n, 2))
        st = np.zeros((nb, n), np.int32)
        args = [*self._shape_args(), C.byref(opts), C.c_int32(nb), _p(sid), _p(x0), _p(traj),
                C.c_int32(len(traj)), _p(idx), C.c_int32(n), None if nz is None else _p(nz),
                C.c_int32(int(delay_cols)), C.c_int32(int(plant_delay_cols)), C.c_int32(int(dist_step)),
                _p(amp), _p(xw), _p(X), _p(Xs), _p(U), _p(st), C.c_int(_threads(nthreads))]
        if self.twin:   # ubc0: the controller's input buffer at the start (B x delay_cols x 2; None: zeros)
            u0b = None if ubc0 is None else np.ascontiguousarray(ubc0, np.float64).reshape(nb, int(delay_cols), 2)
            r = self.L.tw_closed_loop(*args, None if u0b is None else _p(u0b))
        else:
            if ubc0 is not None:
                raise ValueError("ubc0: twin only")
            r = self.L.or_closed_loop(*args)
        if r != 0:
            raise ValueError("or_closed_loop: bad arguments")
        return dict(X=X, Xsim=Xs, U=U, status=st)

    def reproject_contact(self, px, py, s0, shape_id=None):
        px = np.ascontiguousarray(px, np.float64).ravel()
        n = len(px)
        py = np.ascontiguousarray(np.broadcast_to(py, (n,)), np.float64)
        s0 = np.ascontiguousarray(np.broadcast_to(s0, (n,)), np.float64)
        sid = self._ids(shape_id, n)
        s = np.zeros(n)
        self._f('reproject_contact')(*self._shape_args(), C.c_int32(n), _p(sid), _p(px), _p(py), _p(s0), _p(s))
        return s

    @staticmethod
    def new_warm(nb, N):
        return dict(X=np.zeros((nb, N + 1, 4)), U=np.zeros((nb, N, 2)), PI=np.zeros((nb, N, 4)),
                    valid=np.zeros(nb, np.uint8))
