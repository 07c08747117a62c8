"""CPU: the oracle's kernel-order twin (oracle/qsp_twin.c) against the literal restatement
(oracle/qsp_oracle.c) and the committed fixtures.

The twin is what the GPU is compared with bit for bit (tests/test_gpu_twin.py); these tests pin
the twin itself to the reference's formulas: its building blocks (span-based de Boor,
hand-derived Jacobian, RK4 with sensitivities) agree with the literal full-basis + forward-AD
restatement to rounding; its QP meets the KKT conditions; its SQP reproduces the golden runs of
BASELINE configs[0] and main.m's controller; its closed loop composes as helper.m's; and its two
lane-layout orders (one or two stages per lane) differ only at rounding level.  Parity against
acados stays unpinned."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, config2_x0, straight_traj
from oracle.oracle import Oracle, make_opts

NAMES = ("santal", "balea", "montana", "pulirapid")


def _fma(a, b, c):
    """a * b + c rounded once (exact rational arithmetic, then one correctly rounded conversion)."""
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


@pytest.fixture(scope="module")
def twin():
    return Oracle(NAMES, twin=True)


def _states(rng, n, b):
    x = np.stack([rng.uniform(-0.05, 0.05, n), rng.uniform(-0.05, 0.05, n), rng.uniform(-np.pi, np.pi, n),
                  rng.uniform(-1.5 * b, 1.5 * b, n)], 1)
    u = np.stack([rng.uniform(0.0, 0.03, n), rng.uniform(-0.05, 0.05, n)], 1)
    return x, u


def test_building_blocks_match_literal(oracle, twin):
    rng = np.random.default_rng(4)
    for sid in range(4):
        b = oracle.tab["params"][sid, 0]
        knots = oracle.tab["knots"][sid, :oracle.tab["n_ctrl"][sid] + 4]
        s = np.concatenate([rng.uniform(0, b, 800), knots, [b, np.nextafter(b, 0)]])
        C, D, Dd, kap = twin.spline(s, sid)
        Co, _, Do, dDo, kapo = oracle.spline(s, sid)
        np.testing.assert_allclose(C, Co, rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(D, Do, rtol=1e-11, atol=1e-13)
        np.testing.assert_allclose(Dd, dDo, rtol=1e-9, atol=1e-9)
        ok = np.isfinite(kapo)
        np.testing.assert_allclose(kap[ok], kapo[ok], rtol=1e-9, atol=1e-9)
        x, u = _states(rng, 3000, b)
        u[:50] = 0.0
        f, J = twin.dynamics(x, u, sid)
        fo, Jo = oracle.dynamics(x, u, sid)
        np.testing.assert_allclose(f, fo, rtol=1e-10, atol=1e-14)
        np.testing.assert_allclose(J, Jo, rtol=1e-8, atol=1e-10)
        assert np.all(f[:50] == 0.0)                     # rho = 0/0: every indicator false
        xn, A, B = twin.rk4(x, u, 0.05, sid)
        xo, Ao, Bo = oracle.rk4(x, u, 0.05, sid)
        np.testing.assert_allclose(xn, xo, rtol=1e-11, atol=1e-14)
        np.testing.assert_allclose(A, Ao, rtol=1e-8, atol=1e-10)
        np.testing.assert_allclose(B, Bo, rtol=1e-8, atol=1e-10)
        sv = rng.uniform(-2 * b, 2 * b, 500)
        np.testing.assert_allclose(twin.vbound(sv, make_opts(), sid), oracle.vbound(sv, make_opts(), sid),
                                   rtol=1e-9, atol=1e-12)


def test_sincos_against_libm(twin):
    """The library's own sin/cos (qsp_fp.hpp, restated in the twin): within one ulp of libm on the
    model's angle range -- seen through f, whose theta dependence is R(theta) G."""
    x = np.zeros((2000, 4))
    x[:, 2] = np.linspace(-20.0, 20.0, 2000)
    x[:, 3] = 0.05
    u = np.tile([0.01, 0.001], (2000, 1))
    f, _ = twin.dynamics(x, u, 0)
    f0, _ = twin.dynamics(x * np.array([1, 1, 0, 1]), u, 0)
    c, s = np.cos(x[:, 2]), np.sin(x[:, 2])
    ref = np.stack([c * f0[:, 0] - s * f0[:, 1], s * f0[:, 0] + c * f0[:, 1]], 1)
    np.testing.assert_allclose(f[:, :2], ref, rtol=0, atol=4 * np.finfo(float).eps * np.abs(f0[:, :2]).max())


@pytest.mark.parametrize("S", [1, 2])
def test_qp_kkt(twin, S):
    """The twin's QP solutions (both lane-layout orders) meet the KKT conditions as the literal
    oracle's do (tests/test_oracle.py::test_qp_kkt: 1e-8 relative plus the dual-accuracy floor)."""
    from qp_data import build_qp
    N, nb = 20, 32
    op = make_opts(N=N, sqp_iters=3, stages_per_lane=S)
    x0 = config2_x0(nb, 5)
    yref = np.repeat(straight_traj()[None, :N], nb, 0)
    yref_e = yref[:, N - 1, :4].copy()
    r = twin.ocp_solve(op, x0, yref, yref_e, X=np.repeat(x0[:, None], N + 1, 1))
    A, B, b, H, g, lo, hi, act, dx0 = build_qp(twin, op, r["X"], r["U"], yref, yref_e, x0)
    s = twin.qp(op, A.reshape(nb, N, 16), B.reshape(nb, N, 8), b, H, g, lo, hi, act, dx0)
    assert np.all(s["qp_status"] == 0)
    eps = np.finfo(float).eps
    for i in range(nb):
        dx, du, pi, lam = s["dx"][i], s["du"][i], s["pi"][i], s["lam"][i]
        np.testing.assert_allclose(dx[0], dx0[i], atol=1e-15)
        v = np.stack([dx[:N, 3], du[:, 0], du[:, 1]], 1)
        t = np.stack([v - lo[i], hi[i] - v], 2).reshape(N, 6)
        sig = np.where(np.repeat(act[i], 2, 1) > 0, np.abs(lam) / np.maximum(np.abs(t), 1e-300), 0.0)
        floor = N * sig.max() * eps * max(np.abs(lo[i]).max(), np.abs(hi[i]).max())
        worst = 0.0
        for k in range(N):
            np.testing.assert_allclose(dx[k + 1], A[i, k] @ dx[k] + B[i, k] @ du[k] + b[i, k], atol=1e-12)
            sl = slice(0 if k >= 1 else 0, 3)
            assert np.all(v[k, sl] >= lo[i, k, sl] - 1e-8) and np.all(v[k, sl] <= hi[i, k, sl] + 1e-8)
            rs = H[i, 6 * k + 4:6 * k + 6] * du[k] + g[i, 6 * k + 4:6 * k + 6] + B[i, k].T @ pi[k] \
                - lam[k, 2::2] + lam[k, 3::2]
            worst = max(worst, np.abs(rs).max())
        assert worst <= 1e-8 * (1 + np.abs(g[i]).max()) + floor, (i, worst, floor)


def test_config0_rti_golden(twin):
    """BASELINE configs[0] (201 control steps, one SQP-RTI iteration each) against the literal
    oracle's golden trace: the formulations differ by rounding, which one iteration per step
    cannot amplify."""
    g = np.load(os.path.join(GOLDEN, "config1_rti_full.npz"))
    op = make_opts(N=20, sqp_iters=1)
    warm = twin.new_warm(1, 20)
    xs = np.zeros((1, 4))
    traj = straight_traj()
    for i in range(1, 202):
        r = twin.controller_solve(op, xs, traj, i, warm)
        np.testing.assert_allclose(r["u0"][0], g["U"][i - 1], rtol=0, atol=1e-8)   # measured 5.0e-9
        fx, _ = twin.dynamics(xs, r["u0"])
        xs = xs + 0.05 * fx
    np.testing.assert_allclose(xs[0], g["X"][-1], atol=1e-10)                        # measured 1.1e-12


def test_main_m_sqp_closed_loop(twin):
    """main.m's own controller (Hp = 10, merit-backtracking SQP, max_iter 30, tol 1e-6), 201 steps,
    against the literal oracle's golden run: same statuses on at least 97 % of the steps and u0 within
    1e-6 where both converged (the merit SQP stops at the tolerance, so the two formulations' answers
    differ by less than it)."""
    g = np.load(os.path.join(GOLDEN, "main_m_sqp_closed_loop.npz"))
    op = make_opts(N=10, sqp_iters=30, nlp_mode=1)
    warm = twin.new_warm(1, 10)
    xs = np.zeros((1, 4))
    traj = straight_traj()
    st, U = [], []
    for i in range(1, 202):
        r = twin.controller_solve(op, xs, traj, i, warm)
        st.append(r["status"][0])
        U.append(r["u0"][0])
        fx, _ = twin.dynamics(xs, r["u0"])
        xs = xs + 0.05 * fx
    st, U = np.array(st), np.array(U)
    assert np.mean(st == g["status"]) >= 0.97
    both = (st == 0) & (g["status"] == 0)
    assert both.mean() > 0.75
    assert np.abs(U - g["U"])[both].max() < 1e-6
    assert abs(xs[0, 0] - 0.1) < 2e-3


def test_layouts_differ_by_rounding_only(twin):
    """One or two stages per lane (S = 1 or 2) change the order of the Riccati walks' sums, so the
    twin follows the library's choice (S = 1 for N + 1 <= 32); at one SQP iteration the two orders
    agree to rounding."""
    N, nb = 20, 256
    x0 = config2_x0(nb, 8)
    traj = straight_traj()
    sid = np.arange(nb) % 4
    u = []
    for S in (1, 2):
        r = twin.controller_solve(make_opts(N=N, sqp_iters=1, stages_per_lane=S), x0, traj, 1, twin.new_warm(nb, N),
                                  shape_id=sid)
        u.append(r["u0"])
    np.testing.assert_allclose(u[0], u[1], rtol=0, atol=1e-12)


def test_mfma_walk_matches_lane_walk(twin, monkeypatch):
    """The matrix-core factorisation (the default at one stage per lane, 12 <= N <= 31) against the lane
    walk (QSP_MFMA_WALK=0), both measured against the literal formulas in __float128: three SQP-RTI
    iterations of 64 lanes, mixed shapes, at the range's lower edge and the bench horizon.  The two walks
    associate every product differently (their answers part after the first iteration) and are equally
    accurate: the same lanes sit beyond 1e-9 of exact arithmetic (the ill-conditioned ones, also for the
    literal restatement), and the median error is the same.  Measured: 4 and 3 such lanes, medians
    3.1e-13 / 3.8e-13 for the matrix cores, 3.1e-13 / 5.5e-13 for the lane walk."""
    nb = 64
    x0 = config2_x0(nb, 13)
    sid = np.arange(nb) % 4
    traj = straight_traj()
    lit = Oracle(NAMES)
    for N in (15, 20):
        op = make_opts(N=N, sqp_iters=3)
        q = lit.controller_solve_ext(op, x0, traj, 1, lit.new_warm(nb, N), shape_id=sid, precision="quad")["u0"]
        err = {}
        for mw in ("1", "0"):
            monkeypatch.setenv("QSP_MFMA_WALK", mw)
            u = twin.controller_solve(op, x0, traj, 1, twin.new_warm(nb, N), shape_id=sid)["u0"]
            err[mw] = np.abs(u - q).max(1)
        assert not np.array_equal(err["1"], err["0"]), f"N={N}: the two walks should round differently"
        assert np.array_equal(err["1"] > 1e-9, err["0"] > 1e-9), f"N={N}"
        assert np.median(err["1"]) < 2 * np.median(err["0"]) + 1e-15, (N, np.median(err["1"]), np.median(err["0"]))


def test_mfma_walk_matches_lane_walk_two_stages_per_lane(twin):
    """The same check at two stages per lane (N + 1 > 32: configs[4]'s layout), where the matrix-core
    factorisation is also the default (round 5): N = 32, 50 and 127, three SQP-RTI iterations of 64 lanes
    against the literal formulas in __float128, the twin in the device's matrix-core order and in the lane
    walk's (or_opts.lane_walk).  Measured: lanes beyond 1e-9 of quad 6 / 8 / 5 (matrix cores), 5 / 8 / 4
    (lane walk), 5 / 9 / 6 (the double literal); medians 3.1e-13 / 1.0e-13 / 4.3e-13 against 2.6e-13 /
    9.2e-14 / 6.9e-13; the largest error smaller with the matrix cores at every horizon (6.9e-6 / 1.8e-4 /
    2.5e-4 against 1.2e-5 / 5.5e-4 / 1.6e-3)."""
    nb = 64
    x0 = config2_x0(nb, 13)
    sid = np.arange(nb) % 4
    traj = straight_traj()
    lit = Oracle(NAMES)
    for N in (32, 50, 127):
        op = make_opts(N=N, sqp_iters=3)
        q = lit.controller_solve_ext(op, x0, traj, 1, lit.new_warm(nb, N), shape_id=sid, precision="quad")["u0"]
        dl = np.abs(lit.controller_solve(op, x0, traj, 1, lit.new_warm(nb, N), shape_id=sid)["u0"] - q).max(1)
        err = {}
        for lw in (0, 1):
            u = twin.controller_solve(make_opts(N=N, sqp_iters=3, lane_walk=lw), x0, traj, 1, twin.new_warm(nb, N),
                                      shape_id=sid)["u0"]
            err[lw] = np.abs(u - q).max(1)
        assert not np.array_equal(err[0], err[1]), f"N={N}: the two walks should round differently"
        far = [int(np.sum(e > 1e-9)) for e in (err[0], err[1], dl)]
        assert max(far) - min(far) <= 2, (N, far)
        assert np.median(err[0]) < 2 * np.median(err[1]) + 1e-15, (N, np.median(err[0]), np.median(err[1]))
        assert err[0].max() <= 2 * err[1].max(), (N, err[0].max(), err[1].max())


def test_s2_scans_across_horizons(twin):
    """The S = 2 layout's scans (forward and corrector-difference passes as Hillis-Steele scans over
    the group's lanes, at any lane count L = ceil((N+1)/2), powers of two or not) against the S = 1
    lane walks for N = 2 ... 63, and against the literal restatement for N = 64 ... 127, where S = 1
    no longer fits a wavefront: one SQP iteration, 64 lanes, mixed shapes.  Measured: <= 1e-17."""
    nb = 64
    x0 = config2_x0(nb, 11)
    sid = np.arange(nb) % 4
    traj = straight_traj()
    for N in (2, 3, 5, 8, 11, 16, 17, 31, 32, 33, 47, 50, 63):
        u = [twin.controller_solve(make_opts(N=N, sqp_iters=1, stages_per_lane=S), x0, traj, 1, twin.new_warm(nb, N),
                                   shape_id=sid)["u0"] for S in (1, 2)]
        np.testing.assert_allclose(u[1], u[0], rtol=0, atol=1e-15, err_msg=f"N={N}")
    lit = Oracle(NAMES)
    for N in (64, 100, 127):
        r = twin.controller_solve(make_opts(N=N, sqp_iters=1, stages_per_lane=2), x0, traj, 1, twin.new_warm(nb, N),
                                  shape_id=sid)
        q = lit.controller_solve(make_opts(N=N, sqp_iters=1), x0, traj, 1, lit.new_warm(nb, N), shape_id=sid)
        np.testing.assert_allclose(r["u0"], q["u0"], rtol=0, atol=1e-15, err_msg=f"N={N}")


def test_divergence_exit(twin):
    """qp_mu_max below mu0 = 1: the first QP of every lane diverges by definition -> status 4
    (acados ACADOS_QP_FAILURE), sqp_iter 0, and the SQP keeps its initial iterate (u0 = the
    warm-start rollout's first control, here the cold start's (0, 0))."""
    N, nb = 20, 64
    x0 = config2_x0(nb, 12)
    r = twin.controller_solve(make_opts(N=N, qp_mu_max=0.5), x0, straight_traj(), 1, twin.new_warm(nb, N),
                              shape_id=np.arange(nb) % 4)
    assert np.all(r["status"] == 4) and np.all(r["iters"] == 0) and np.all(r["qp_iter"] == 0)
    assert np.all(r["u0"] == 0.0)


def test_closed_loop_composition(twin):
    """The twin's closed loop (helper.m:195-322) equals its step-by-step composition of
    controller_solve + the Euler plant with a fused multiply-add, and with a controller delay of D
    columns it reads column i + D and predicts with the buffered inputs."""
    N, nb, T = 10, 4, 6
    x0 = config2_x0(nb, 2)
    sid = np.arange(nb) % 4
    traj = straight_traj()
    op = make_opts(N=N, sqp_iters=2)
    r = twin.closed_loop(op, x0, traj, T, shape_id=sid)
    w = twin.new_warm(nb, N)
    x = x0.copy()
    for t in range(T):
        ro = twin.controller_solve(op, x, traj, 1 + t, w, shape_id=sid)
        np.testing.assert_array_equal(ro["u0"], r["U"][:, t])
        f, _ = twin.dynamics(x, ro["u0"], sid)
        x = np.array([[_fma(0.05, f[i, c], x[i, c]) for c in range(4)] for i in range(nb)])
    np.testing.assert_array_equal(x, r["X"][:, -1])
    rd = twin.closed_loop(op, x0, traj, 2, shape_id=sid, delay_cols=2)
    np.testing.assert_array_equal(rd["U"][:, 0], r["U"][:, 0])
    # a non-empty controller buffer at the start (as a second run after set_delay_comp would leave it)
    ub = np.tile([0.01, 0.002], (nb, 2, 1))
    rb = twin.closed_loop(op, x0, traj, 2, shape_id=sid, delay_cols=2, ubc0=ub)
    assert not np.array_equal(rb["Xsim"][:, 0], rd["Xsim"][:, 0])


def test_factor_scan_s2_matches_walk_at_one_iteration(twin):
    """The S = 2 factorisation as an associative scan (factor_scan) against the walk at one SQP
    iteration (the cold QP, before any amplification), N = 2 ... 127 with the terminal stage in either
    slot.  Measured <= 1e-17: the scan's rounding (about two digits more than the walk's)
    shows only once the SQP iterates."""
    nb = 64
    x0 = config2_x0(nb, 11)
    sid = np.arange(nb) % 4
    traj = straight_traj()
    for N in (2, 3, 5, 17, 32, 33, 50, 63, 100, 127):
        u = [twin.controller_solve(make_opts(N=N, sqp_iters=1, stages_per_lane=2, factor_scan=fs), x0, traj, 1,
                                   twin.new_warm(nb, N), shape_id=sid)["u0"] for fs in (0, 1)]
        np.testing.assert_allclose(u[1], u[0], rtol=0, atol=1e-15, err_msg=f"N={N}")
