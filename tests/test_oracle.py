"""CPU: the oracle against the committed golden fixtures, the reference's data files,
the survey-time values derived from them, and mathematical invariants.

Parity against acados is UNPINNED (acados/CasADi/MATLAB are not runnable here); these
checks pin the oracle to what can be pinned."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, config2_x0, straight_traj
from oracle.oracle import make_opts
from oracle.shapes_np import load_object

NAMES = ("santal", "balea", "montana", "pulirapid")


def test_shape_tables_match_golden():
    gold = json.load(open(os.path.join(GOLDEN, "shapes.json")))
    for n in NAMES:
        o = load_object(n)
        g = gold[n]
        assert len(o["P"]) == g["n"]
        np.testing.assert_array_equal(o["P"], np.array(g["P"]))
        np.testing.assert_array_equal(o["S"], np.array(g["S"]))
        assert o["b"] == g["b"] and o["c"] == g["c"] and o["mu"] == g["mu"]


def test_shape_values_from_reference_data():
    # control points, knot counts, contour lengths, c_ellipse
    expect = {"santal": (37, 0.281899, 0.027811, 0.19), "balea": (37, 0.222486, 0.0071409, 0.20),
              "montana": (35, 0.285079, 0.020867, 0.10), "pulirapid": (56, 0.596013, 0.023260, 0.10)}
    for n, (nc, b, c, mu) in expect.items():
        o = load_object(n)
        assert len(o["P"]) == nc and len(o["S"]) == nc + 4
        assert abs(o["b"] - b) < 5e-7 and abs(o["c"] - c) / c < 5e-5 and o["mu"] == mu
        np.testing.assert_array_equal(o["P"][0], o["P"][-1])          # closed contour
        assert np.all(np.diff(o["S"]) >= 0) and o["S"][0] == 0 and o["S"][-1] == o["b"]


def test_santal_contact_geometry(oracle):
    # C(0) = (-0.031, 0.024463), t(0) = (0, 1), gamma_l = 0.7176, gamma_r = 0.3492
    C, dC, D, dD, kap = oracle.spline([0.0], 0)
    np.testing.assert_allclose(C[0], [-0.031, 0.024463], atol=5e-7)
    t = D[0] / np.linalg.norm(D[0])
    np.testing.assert_allclose(t, [0.0, 1.0], atol=1e-12)
    # pure pushing at s = 0 is slide-right: s_dot = -gamma_r u_n
    f, _ = oracle.dynamics([[0, 0, 0, 0]], [[0.01, 0.0]], 0)
    assert abs(-f[0, 3] / 0.01 - 0.3492) < 5e-4


def test_spline_invariants(oracle):
    for sid, n in enumerate(NAMES):
        o = load_object(n)
        C, dC, D, dD, _ = oracle.spline([0.0, o["b"]], sid)
        np.testing.assert_allclose(C[0], o["P"][0], atol=1e-15)     # C(0) = P_1 (clamped)
        assert np.all(C[1] == 0.0) and np.all(D[1] == 0.0)           # C(b) = 0: half-open indicator
        s = np.linspace(0, o["b"], 400, endpoint=False)
        C, dC, D, dD, _ = oracle.spline(s, sid)
        np.testing.assert_allclose(dC, D, rtol=1e-9, atol=1e-9)      # d/ds FC == FC_dot
        # the derivative of FC_dot agrees with a central difference away from knots
        h = 1e-7
        Cp = oracle.spline(s + h, sid)[2]
        Cm = oracle.spline(s - h, sid)[2]
        fd = (Cp - Cm) / (2 * h)
        knots = np.asarray(o["S"])
        far = np.min(np.abs(s[:, None] - knots[None, :]), axis=1) > 1e-5
        np.testing.assert_allclose(dD[far], fd[far], rtol=1e-5, atol=1e-4)


def test_dynamics_invariants(oracle):
    rng = np.random.default_rng(0)
    for sid, n in enumerate(NAMES):
        b = load_object(n)["b"]
        x = np.stack([rng.uniform(-.1, .1, 200), rng.uniform(-.1, .1, 200), rng.uniform(-3, 3, 200),
                      rng.uniform(-b, b, 200)], 1)
        f, J = oracle.dynamics(x, np.zeros((200, 2)), sid)
        assert np.all(f == 0.0) and np.all(J == 0.0)                 # rho = 0/0: no mode active
        u = np.stack([rng.uniform(1e-3, .03, 200), rng.uniform(-.05, .05, 200)], 1)
        f, J = oracle.dynamics(x, u, sid)
        assert np.all(J[:, :, :2] == 0.0)                            # f independent of (x, y)
        assert np.all(J[:, 2:, 2] == 0.0)                            # theta_dot, s_dot independent of theta
        # forward-mode AD vs central differences (away from mode switches)
        h = 1e-7
        for c in range(6):
            dx = np.zeros((200, 4)); du = np.zeros((200, 2))
            (dx if c < 4 else du)[:, c % 4 if c < 4 else c - 4] = h
            fp, _ = oracle.dynamics(x + dx, u + du, sid)
            fm, _ = oracle.dynamics(x - dx, u - du, sid)
            fd = (fp - fm) / (2 * h)
            # drop points whose mode changes inside the stencil (Jacobian jumps there)
            ok = np.all(np.abs(fd - J[:, :, c]) < 1e-5 * (1 + np.abs(J[:, :, c])), axis=1)
            assert ok.mean() > 0.97, (n, c, ok.mean())


def test_motion_cone_continuity(oracle):
    # f is continuous across the cone edges rho = gamma_l and rho = gamma_r:
    # locate each edge by bisection on the sticking indicator (s_dot == 0 exactly while
    # sticking) and check that f does not jump there
    x = np.array([[0.0, 0.0, 0.1, 0.03]])
    un = 0.01

    def f_at(rho):
        return oracle.dynamics(x, [[un, un * rho]], sid)[0][0]

    for sid in range(4):
        for lo, hi in ((0.0, 50.0), (0.0, -50.0)):
            assert f_at(lo)[3] == 0.0 or f_at(hi)[3] != 0.0
            if f_at(lo)[3] != 0.0:
                continue                      # rho = 0 already sliding for this shape/point
            for _ in range(200):
                mid = 0.5 * (lo + hi)
                if f_at(mid)[3] == 0.0:
                    lo = mid
                else:
                    hi = mid
            jump = np.abs(f_at(hi) - f_at(lo)).max()
            assert jump < 1e-9, (sid, lo, hi, jump)


def test_rk4_sensitivities_vs_fd(oracle):
    rng = np.random.default_rng(1)
    x = np.stack([rng.uniform(-.05, .05, 100), rng.uniform(-.05, .05, 100), rng.uniform(-1, 1, 100),
                  rng.uniform(-.05, .05, 100)], 1)
    u = np.stack([rng.uniform(1e-3, .03, 100), rng.uniform(-.05, .05, 100)], 1)
    xn, A, B = oracle.rk4(x, u, 0.05, 0)
    h = 1e-7
    for c in range(6):
        dx = np.zeros((100, 4)); du = np.zeros((100, 2))
        (dx if c < 4 else du)[:, c if c < 4 else c - 4] = h
        fp = oracle.rk4(x + dx, u + du, 0.05, 0)[0]
        fm = oracle.rk4(x - dx, u - du, 0.05, 0)[0]
        fd = (fp - fm) / (2 * h)
        an = A[:, :, c] if c < 4 else B[:, :, c - 4]
        ok = np.all(np.abs(fd - an) < 1e-5 * (1 + np.abs(an)), axis=1)
        assert ok.mean() > 0.95


def test_model_points_golden(oracle):
    g = np.load(os.path.join(GOLDEN, "model_points.npz"))
    f, J = oracle.dynamics(g["x"], g["u"], g["sid"])
    np.testing.assert_array_equal(f, g["f"])
    np.testing.assert_array_equal(J, g["J"])
    xn, A, B = oracle.rk4(g["x"], g["u"], 0.05, g["sid"])
    np.testing.assert_array_equal(xn, g["xn"])
    np.testing.assert_array_equal(A, g["A"])
    C, dC, D, dD, kap = oracle.spline(g["sigma"], g["sid"])
    np.testing.assert_array_equal(C, g["C"])
    np.testing.assert_array_equal(kap, g["kappa"])


def test_qp_kkt(oracle):
    """KKT of the oracle's QP solutions (HPIPM-style stop: mu, bound, stationarity and equality
    residuals, cap 50).  Stationarity is checked on every QP that met the stop test, against
    1e-8 relative plus the dual-accuracy floor every primal-dual IPM has here: an active bound's
    multiplier comes from lam/t * (v - lo - t), whose difference carries eps*|v| of rounding, so
    lam is known to ~ (lam/t) eps |v| ~ eps |v| lam^2 / mu, and the adjoint sums that over the
    horizon (it grows as mu_stop shrinks, ~1e-3 absolute at mu = 1e-10 on
    the QPs with lam ~ 100 active s bounds; most QPs sit far below it)."""
    from qp_data import build_qp
    N, nb = 20, 32
    op = make_opts(N=N, sqp_iters=3)
    x0 = config2_x0(nb, 5)
    traj = straight_traj()
    yref = np.repeat(traj[None, :N], nb, 0)
    yref_e = yref[:, N - 1, :4].copy()
    r = oracle.ocp_solve(op, x0, yref, yref_e, X=np.repeat(x0[:, None], N + 1, 1))
    A, B, b, H, g, lo, hi, act, dx0 = build_qp(oracle, op, r["X"], r["U"], yref, yref_e, x0)
    s = oracle.qp(op, A, B, b, H, g, lo, hi, act, dx0)
    assert s["fail"] == 0
    conv = s["qp_status"] == 0                  # stop test met (2: iteration cap)
    assert conv.all()
    eps = np.finfo(float).eps
    plain = []
    for i in np.where(conv)[0]:
        dx, du, pi, lam = s["dx"][i], s["du"][i], s["pi"][i], s["lam"][i]
        np.testing.assert_allclose(dx[0], dx0[i], atol=1e-15)
        v = np.stack([dx[:N, 3], du[:, 0], du[:, 1]], 1)
        t = np.stack([v - lo[i], hi[i] - v], 2).reshape(N, 6)
        sig = np.where(np.repeat(act[i], 2, 1) > 0, np.abs(lam) / np.maximum(np.abs(t), 1e-300), 0.0)
        floor = N * sig.max() * eps * max(np.abs(lo[i]).max(), np.abs(hi[i]).max())
        scale = 1 + np.abs(g[i]).max()
        worst = 0.0
        for k in range(N):
            # dynamics
            np.testing.assert_allclose(dx[k + 1], A[i, k] @ dx[k] + B[i, k] @ du[k] + b[i, k], atol=1e-12)
            # bounds (IPM: interior up to the final barrier parameter)
            sl = slice(0 if (k >= 1 or act[i, 0, 0]) else 1, 3)
            assert np.all(v[k, sl] >= lo[i, k, sl] - 1e-8) and np.all(v[k, sl] <= hi[i, k, sl] + 1e-8)
            # stationarity w.r.t. u_k
            rs = H[i, 6 * k + 4:6 * k + 6] * du[k] + g[i, 6 * k + 4:6 * k + 6] + B[i, k].T @ pi[k] \
                - lam[k, 2::2] + lam[k, 3::2]
            worst = max(worst, np.abs(rs).max())
        assert worst <= 1e-8 * scale + floor, (i, worst, floor)
        plain.append(worst <= 1e-8 * scale)
    # the floor binds only on the QPs with strongly active bounds
    assert np.mean(plain) >= 0.75, np.mean(plain)


def test_config1_closed_loop_golden(oracle):
    gold = json.load(open(os.path.join(GOLDEN, "config1_closed_loop.json")))
    traj = straight_traj()
    for N in (10, 20):
        op = make_opts(N=N, sqp_iters=5)
        warm = oracle.new_warm(1, N)
        xs = np.zeros((1, 4))
        for i in range(1, 21):
            r = oracle.controller_solve(op, xs, traj, i, warm)
            np.testing.assert_allclose(r["u0"][0], gold[f"N{N}"]["u0"][i - 1], rtol=0, atol=1e-12)
            fx, _ = oracle.dynamics(xs, r["u0"])
            xs = xs + 0.05 * fx
        np.testing.assert_allclose(xs[0], gold[f"N{N}"]["x_final"], atol=1e-12)
        # the slider follows the 0.01 m/s reference: x(1 s) ~ 0.010 m
        assert abs(xs[0, 0] - 0.01) < 2e-3


def test_config2_batch_golden(oracle):
    g = np.load(os.path.join(GOLDEN, "config2_batch64.npz"))
    N = 20
    r = oracle.controller_solve(make_opts(N=N, sqp_iters=50), g["x0"], straight_traj(), 1,
                                oracle.new_warm(len(g["x0"]), N))
    st = g["stable"]
    np.testing.assert_allclose(r["u0"][st], g["u0"][st], atol=1e-12)
    assert np.all(r["status"] == 0)
    assert np.all(g["u0"][:, 0] >= -1e-9) and np.all(g["u0"][:, 0] <= 0.03 + 1e-9)      # u_n bounds
    assert np.all(np.abs(g["u0"][:, 1]) <= 0.05 + 1e-9)                                  # u_t bounds


def test_vbound_definition(oracle):
    op = make_opts()
    s = np.linspace(-0.3, 0.3, 301)
    vb = oracle.vbound(s, op, 0)
    kap = oracle.spline(np.mod(s, load_object("santal")["b"]), 0)[4]
    ref = np.minimum(1.0 / (np.abs(np.abs(kap) - 3.0) + 1e-4), 0.05)
    np.testing.assert_allclose(vb, ref, rtol=1e-12)


@pytest.mark.parametrize("name", ["santal", "balea", "montana", "pulirapid"])
def test_tangent_angle_curvature_finite_differences(oracle, name):
    """The reference's own curvature check (acados_nmpc/t_angle_curvatures.m:1-27): the tangent
    angle atan2(C'_y, C'_x) on s = 0:1e-3:b, its differences unwrapped where |d| > 3 pi / 2 and
    divided by ds, against the analytic kappa (d/ds of the angle, bspline_shape.m:137-152) at the
    interval midpoints, away from the knots (C'' of a cubic spline is only continuous there)."""
    sid = ["santal", "balea", "montana", "pulirapid"].index(name)
    b = load_object(name)["b"]
    h = 1e-3
    s = np.arange(0.0, b, h)
    _, dC, _, _, _ = oracle.spline(s, sid)
    ang = np.arctan2(dC[:, 1], dC[:, 0])
    d = np.diff(ang)
    d[np.abs(d) > 1.5 * np.pi] -= 2 * np.pi * np.sign(d[np.abs(d) > 1.5 * np.pi])
    fd = d / np.diff(s)
    kap = oracle.spline(s[:-1] + h / 2, sid)[4]
    # skip the intervals that hold a knot (shapes_np.knots_for: uniform interior spacing)
    knots = np.unique(load_object(name)["S"])
    near = np.min(np.abs((s[:-1] + h / 2)[:, None] - knots[None, :]), 1) < h
    ok = ~near & np.isfinite(kap)
    scale = np.max(np.abs(kap[ok]))
    assert ok.sum() > 0.5 * len(ok)
    # midpoint rule: O(h^2 kappa'') on smooth intervals
    assert np.median(np.abs(fd[ok] - kap[ok])) < 1e-3 * scale
    assert np.mean(np.abs(fd[ok] - kap[ok]) < 1e-2 * scale + 1e-6) > 0.97
    assert np.max(np.abs(fd[ok] - kap[ok])) < 3e-2 * scale


def _eval_bspline_m(s, S, i, p):
    """acados_nmpc/eval_bspline.m:1-33 (= bspline_shape.m:40-72) restated literally: 1-based i,
    the zero-support guard first (also at p = 0), the half-open indicator, the 0/0 guards."""
    if S[i + p] == S[i - 1]:
        return 0.0
    if p == 0:
        return float(s < S[i]) * float(s >= S[i - 1])
    a = _eval_bspline_m(s, S, i, p - 1)
    c = _eval_bspline_m(s, S, i + 1, p - 1)
    m1 = 0.0 if S[i + p - 1] == S[i - 1] else (s - S[i - 1]) / (S[i + p - 1] - S[i - 1])
    m2 = 0.0 if S[i + p] == S[i] else (S[i + p] - s) / (S[i + p] - S[i])
    return m1 * a + m2 * c


@pytest.mark.parametrize("name", ["santal", "balea", "montana", "pulirapid"])
def test_spline_matches_literal_eval_bspline(oracle, name):
    """The oracle's C(s) and C'(s) against eval_bspline.m's recursion summed as getSymbolicSpline
    (bspline_shape.m:74-83) and getSymboliSplineDot (:85-104) do, at sampled points, at every
    knot (the half-open indicator's side) and at s = b (every basis function zero)."""
    sid = ["santal", "balea", "montana", "pulirapid"].index(name)
    o = load_object(name)
    S, P, b, p = list(o["S"]), o["P"], o["b"], 3
    n = len(P)
    s = np.r_[np.random.default_rng(7).uniform(0.0, b, 24), np.unique(S)]
    C, _, D, _, _ = oracle.spline(s, sid)
    for q, sq in enumerate(s):
        Cm = np.zeros(2)
        for i in range(1, n + 1):
            Cm = Cm + _eval_bspline_m(sq, S, i, p) * P[i - 1]
        Dm = np.zeros(2)
        for i in range(2, n + 1):
            cj = 0.0 if S[i + p - 1] == S[i - 1] else p * (P[i - 1] - P[i - 2]) / (S[i + p - 1] - S[i - 1])
            Dm = Dm + cj * _eval_bspline_m(sq, S, i, p - 1)
        np.testing.assert_array_equal(C[q], Cm)                        # same sum, same order: bit for bit
        np.testing.assert_allclose(D[q], Dm, rtol=0, atol=2e-15)        # the oracle divides the knot span once
        if sq == b:
            assert np.all(Cm == 0.0) and np.all(C[q] == 0.0)


def test_decagon_fixture_known_answers():
    """test_bspline_class.m's decagon: clamped-end values, end tangent, convex hull,
    mirror symmetry of the uniform knot vector, C(b) = 0 (half-open indicator)."""
    from conftest import decagon_table
    from oracle.oracle import Oracle
    tab, P, S, b = decagon_table()
    orc = Oracle(tab=tab)
    assert len(P) == 11 and len(S) == 15
    np.testing.assert_allclose(b, 10 * 2 * np.sin(np.pi / 10), rtol=1e-15)
    C0, _, D0, _, _ = orc.spline(np.array([0.0]), 0)
    np.testing.assert_allclose(C0[0], P[0], atol=1e-15)                       # clamped start
    np.testing.assert_allclose(D0[0], 3 * (P[1] - P[0]) / (S[4] - S[1]), rtol=1e-13)
    s = np.linspace(0, b, 2001)[1:-1]
    Cs, _, Ds, _, _ = orc.spline(s, 0)
    assert np.all(np.hypot(Cs[:, 0], Cs[:, 1]) <= 1.0 + 1e-12)                 # convex hull
    Cm, _, _, _, _ = orc.spline(b - s, 0)
    np.testing.assert_allclose(Cm[:, 0], Cs[:, 0], atol=1e-13)                 # y -> -y, s -> b - s
    np.testing.assert_allclose(Cm[:, 1], -Cs[:, 1], atol=1e-13)
    Cb, _, _, _, _ = orc.spline(np.array([b]), 0)
    assert np.all(Cb == 0.0)


def test_config1_rti_full_golden(oracle):
    """BASELINE configs[0]: 201 control steps, one SQP-RTI iteration each."""
    g = np.load(os.path.join(GOLDEN, "config1_rti_full.npz"))
    op = make_opts(N=20, sqp_iters=1)
    warm = oracle.new_warm(1, 20)
    xs = np.zeros((1, 4))
    traj = straight_traj()
    for i in range(1, 202):
        r = oracle.controller_solve(op, xs, traj, i, warm)
        np.testing.assert_allclose(r["u0"][0], g["U"][i - 1], rtol=0, atol=1e-12)
        fx, _ = oracle.dynamics(xs, r["u0"])
        xs = xs + 0.05 * fx
    np.testing.assert_allclose(xs[0], g["X"][-1], atol=1e-12)
    assert abs(xs[0, 0] - 0.1) < 2e-3                       # reaches the 0.10 m waypoint


def test_main_m_sqp_closed_loop_golden(oracle):
    """main.m's own setup (Hp = 10, merit-backtracking SQP, max_iter 30), 201 steps."""
    g = np.load(os.path.join(GOLDEN, "main_m_sqp_closed_loop.npz"))
    op = make_opts(N=10, sqp_iters=30, nlp_mode=1)
    warm = oracle.new_warm(1, 10)
    xs = np.zeros((1, 4))
    traj = straight_traj()
    for i in range(1, 202):
        r = oracle.controller_solve(op, xs, traj, i, warm)
        np.testing.assert_allclose(r["u0"][0], g["U"][i - 1], rtol=0, atol=1e-12)
        assert r["status"][0] == g["status"][i - 1] and r["iters"][0] == g["iters"][i - 1]
        fx, _ = oracle.dynamics(xs, r["u0"])
        xs = xs + 0.05 * fx
    assert np.mean(g["status"] == 0) > 0.8 and abs(xs[0, 0] - 0.1) < 2e-3


def test_reference_table_prefix_and_closed_loop_composition(oracle):
    """set_reference_trajectory with delay_buff_comp D (NMPC_controller.m:425-431): D zero columns
    prepended, the u_t-reference row copied from the first real column; the oracle's closed loop
    equals the step-by-step composition of controller_solve + Euler plant (helper.m:195-322) when
    no delay is set, and with D > 0 the solve at step i reads column i + D (= the original i)."""
    traj = straight_traj()
    traj[:, 5] = 0.003
    N, nb, T = 10, 4, 6
    x0 = config2_x0(nb, 2)
    sid = np.arange(nb) % 4
    op = make_opts(N=N, sqp_iters=2)
    # prefix columns: index 1 with D = 3 reads columns 1..3 of the prefix, then the table
    w1, w2 = oracle.new_warm(nb, N), oracle.new_warm(nb, N)
    pre = np.zeros((3 + len(traj), 6))
    pre[3:] = traj
    pre[:3, 5] = traj[0, 5]
    a = oracle.controller_solve(op, x0, traj, 1, w1, shape_id=sid, delay_cols=3)
    b = oracle.controller_solve(op, x0, pre, 1, w2, shape_id=sid)
    np.testing.assert_array_equal(a["u0"], b["u0"])
    r = oracle.closed_loop(op, x0, traj, T, shape_id=sid)
    w = oracle.new_warm(nb, N)
    x = x0.copy()
    for t in range(T):
        ro = oracle.controller_solve(op, x, traj, 1 + t, w, shape_id=sid)
        np.testing.assert_array_equal(ro["u0"], r["U"][:, t])
        f, _ = oracle.dynamics(x, ro["u0"], sid)
        x = x + 0.05 * f
    np.testing.assert_array_equal(x, r["X"][:, -1])
    # delay D: the first solve sees x advanced by D steps of zero input (= x, f(x, 0) = 0) and the
    # original columns, so it equals the undelayed first step
    rd = oracle.closed_loop(op, x0, traj, 2, shape_id=sid, delay_cols=2)
    np.testing.assert_array_equal(rd["U"][:, 0], r["U"][:, 0])


def test_model_probe(oracle):
    """The model probe (or_opts.model_probe, used by bench.py's parity leg): off by default and at 0,
    deterministic per seed whatever the thread count, and a perturbation of the model's size only
    (u0 of a one-iteration solve moves by at most ~1e-9)."""
    N, nb = 20, 24
    x0 = config2_x0(nb, 41)
    traj = straight_traj()

    def run(threads=4, **kw):
        return oracle.controller_solve(make_opts(N=N, sqp_iters=1, **kw), x0, traj, 1, oracle.new_warm(nb, N),
                                       nthreads=threads)["u0"]
    base = run()
    assert np.array_equal(run(model_probe=0.0, probe_seed=7), base)
    p1 = run(model_probe=1e-14, probe_seed=1)
    assert not np.array_equal(p1, base)
    assert np.abs(p1 - base).max() < 1e-9
    assert np.array_equal(run(threads=1, model_probe=1e-14, probe_seed=1), p1)
    assert not np.array_equal(run(model_probe=1e-14, probe_seed=2), p1)
    assert np.array_equal(run(), base)      # the probe does not leak into the next solve
