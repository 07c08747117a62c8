"""GPU: device-resident closed loop (qsp_closed_loop, helper.m:195-322) against the committed
config-1 golden trace and against the oracle's controller + Euler plant, batched over
mixed shapes with sim_noise."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, config2_x0, straight_traj

pytestmark = pytest.mark.gpu

NAMES = ("santal", "balea", "montana", "pulirapid")


@pytest.mark.parametrize("N", [10, 20])
def test_closed_loop_config1_golden(N):
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    gold = json.load(open(os.path.join(GOLDEN, "config1_closed_loop.json")))[f"N{N}"]
    s = OcpSolver(N=N, batch=4, sqp_iters=5)
    s.set_shapes([make_shape("santal")])
    s.set_reference_trajectory(straight_traj())
    r = s.closed_loop(np.zeros(4), 20)
    s.close()
    # 20 closed-loop steps of K = 5 full SQP steps amplify rounding (two formulations of the
    # spline and the Jacobian): 1e-8 on u0 and x (BASELINE asks 1e-6)
    for lane in range(4):      # identical lanes give identical trajectories
        np.testing.assert_allclose(r["U"][lane], gold["u0"], rtol=0, atol=1e-8)
        np.testing.assert_allclose(r["X"][lane, -1], gold["x_final"], atol=1e-9)
    assert np.all(r["status"] == 0)


def test_closed_loop_batched_noise(oracle):
    from oracle.oracle import make_opts
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N, nb, K, T = 20, 96, 2, 12
    x0 = config2_x0(nb, 31)
    sid = np.arange(nb) % 4
    rng = np.random.default_rng(5)
    noise = rng.standard_normal((T, nb, 4)) * np.array([1e-5, 1e-5, 1e-3, 1e-4])   # helper.m:243-245
    traj = straight_traj()
    s = OcpSolver(N=N, batch=nb, sqp_iters=K)
    s.set_shapes([make_shape(n) for n in NAMES], shape_id=sid)
    s.set_reference_trajectory(traj)
    r = s.closed_loop(x0, T, index0=1, noise=noise)
    s.close()
    op = make_opts(N=N, sqp_iters=K)

    def oracle_loop(xs):
        warm = oracle.new_warm(nb, N)
        x = xs + noise[0]
        X, U, ST = [x], [], []
        for t in range(T):
            ro = oracle.controller_solve(op, x, traj, 1 + t, warm, shape_id=sid)
            f, _ = oracle.dynamics(x, ro["u0"], sid)
            x = x + 0.05 * f + (noise[t + 1] if t + 1 < T else 0.0)
            X.append(x)
            U.append(ro["u0"])
            ST.append(ro["status"])
        oracle_loop.status = np.stack(ST, 1)
        return np.stack(X, 1), np.stack(U, 1)
    Xo, Uo = oracle_loop(x0)
    So = oracle_loop.status
    # closed-loop stable lanes: the oracle's own trace does not move under 1e-13 perturbations
    stable = np.ones(nb, bool)
    for f in (1e-13, -1e-13):
        _, Up = oracle_loop(x0 * (1 + f))
        stable &= np.abs(Up - Uo).max(axis=(1, 2)) < 1e-9
    assert stable.mean() > 0.4, stable.mean()
    du = np.abs(r["U"] - Uo).max(axis=(1, 2))
    dx = np.abs(r["X"] - Xo).max(axis=(1, 2))
    assert du[stable].max() < 1e-6, np.sort(du[stable])[-4:]
    assert dx[stable].max() < 1e-8, np.sort(dx[stable])[-4:]
    # a lane whose s leaves [lh_s, uh_s] gets an infeasible stage-0 bound: status 4, as the oracle
    assert set(np.unique(r["status"])) <= {0, 4}
    assert np.all(r["status"][stable] == So[stable])


def test_closed_loop_config1_rti_full():
    """BASELINE configs[0] on the device: 201 steps of one SQP-RTI iteration, one call."""
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    g = np.load(os.path.join(GOLDEN, "config1_rti_full.npz"))
    s = OcpSolver(N=20, batch=2, sqp_iters=1)
    s.set_shapes([make_shape("santal")])
    s.set_reference_trajectory(straight_traj())
    r = s.closed_loop(np.zeros(4), 201)
    s.close()
    for lane in range(2):
        np.testing.assert_allclose(r["U"][lane], g["U"], rtol=0, atol=1e-8)
        np.testing.assert_allclose(r["X"][lane], g["X"], rtol=0, atol=1e-8)
    assert np.all(r["status"] == 0)


def test_closed_loop_main_m_sqp():
    """main.m's own controller (Hp = 10, 'sqp' + 'merit_backtracking', max_iter 30), 201 steps
    on the device in one call, against the committed oracle trace."""
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    g = np.load(os.path.join(GOLDEN, "main_m_sqp_closed_loop.npz"))
    s = OcpSolver(N=10, batch=3, sqp_iters=30, nlp_solver_type="SQP")
    s.set_shapes([make_shape("santal")])
    s.set_reference_trajectory(straight_traj())
    r = s.closed_loop(np.zeros(4), 201)
    s.close()
    for lane in range(3):
        np.testing.assert_allclose(r["U"][lane], g["U"], rtol=0, atol=1e-7)
        np.testing.assert_allclose(r["X"][lane], g["X"], rtol=0, atol=1e-7)
        assert np.mean(r["status"][lane] == g["status"]) > 0.95


def test_c_host_closed_loop(tmp_path):
    """The same configs[0] closed loop from a plain-C host (integration/c/qsp_demo.c, built by
    __graft_entry__.build()) through the C ABI alone, against the committed golden trace."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "integration", "c", "qsp_demo")
    ply = os.path.join(root, "uclv_qs_pushing_matlab_amd", "data", "planar_surface_santal_36_uniformed.ply")
    out = tmp_path / "u.txt"
    assert os.path.exists(exe), "integration/c/qsp_demo not built (run __graft_entry__.build())"
    r = subprocess.run([exe, ply, str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    g = np.load(os.path.join(GOLDEN, "config1_rti_full.npz"))
    np.testing.assert_allclose(np.loadtxt(out), g["U"], rtol=0, atol=1e-8)


XWIDTH = {"santal": 0.068, "balea": 0.071, "montana": 0.057, "pulirapid": 0.13}   # object_selection.m


def _cl_setup(nb, N, K, seed):
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    x0 = config2_x0(nb, seed)
    sid = np.arange(nb) % 4
    s = OcpSolver(N=N, batch=nb, sqp_iters=K)
    s.set_shapes([make_shape(n) for n in NAMES], shape_id=sid)
    s.set_reference_trajectory(straight_traj())
    return s, x0, sid


def _stable_lanes(oracle, run, x0):
    ref = run(x0)
    st = np.ones(len(x0), bool)
    for f in (1e-13, -1e-13):
        rp = run(x0 * (1 + f))
        st &= np.abs(rp["U"] - ref["U"]).max(axis=(1, 2)) < 1e-9
    return ref, st


@pytest.mark.parametrize("delay,plant_delay", [(0.1, 0.0), (0.1, 0.1), (0.0, 0.15), (0.35, 0.35)])
def test_closed_loop_delay_matches_oracle(oracle, delay, plant_delay):
    """A17 + helper.m's plant delay: set_delay_comp (delay_buff_comp = ceil(delay/Ts) prefix columns,
    delay_buffer_sim with the buffered inputs, oldest first) and the plant's u_buff_plant, on the
    device closed loop, against the oracle's or_closed_loop (helper.m:195-322 restated)."""
    from oracle.oracle import make_opts
    N, nb, K, T = 20, 32, 2, 14
    s, x0, sid = _cl_setup(nb, N, K, 41)
    s.set_delay_comp(delay)
    D = s.delay_cols()
    Dp = int(np.ceil(plant_delay / 0.05))
    assert D == int(np.ceil(delay / 0.05))
    r = s.closed_loop(x0, T, plant_delay=plant_delay)
    s.close()
    op = make_opts(N=N, sqp_iters=K)
    run = lambda x: oracle.closed_loop(op, x, straight_traj(), T, shape_id=sid, delay_cols=D,  # noqa: E731
                                       plant_delay_cols=Dp)
    ref, st = _stable_lanes(oracle, run, x0)
    assert st.mean() > 0.5, st.mean()
    np.testing.assert_array_equal(r["status"][st], ref["status"][st])
    assert np.abs(r["U"] - ref["U"]).max(axis=(1, 2))[st].max() < 1e-6
    assert np.abs(r["X"] - ref["X"]).max(axis=(1, 2))[st].max() < 1e-8
    assert np.abs(r["Xsim"] - ref["Xsim"]).max(axis=(1, 2))[st].max() < 1e-8
    if D > 0:   # the prediction moved the state (the buffer held earlier inputs)
        assert np.abs(r["Xsim"][:, D + 1:] - r["X"][:, D + 1:-1]).max() > 1e-6


def test_closed_loop_disturbance_matches_oracle(oracle):
    """helper.m:221-236: at step t_dist, y += amplitude and the contact point is re-projected onto
    the contour (s nearest to (-xwidth/2, C_y(s) - amplitude), from s0 = 0); then the loop goes on."""
    from oracle.oracle import make_opts
    N, nb, K, T, td = 20, 24, 2, 10, 4
    s, x0, sid = _cl_setup(nb, N, K, 43)
    amp = np.linspace(-0.02, 0.02, nb)
    r = s.closed_loop(x0, T, disturbance=True, t_dist=td, amplitude=amp)
    s.close()
    op = make_opts(N=N, sqp_iters=K)
    xw = [XWIDTH[n] for n in NAMES]
    run = lambda x: oracle.closed_loop(op, x, straight_traj(), T, shape_id=sid, dist_step=td,  # noqa: E731
                                       dist_amp=amp, xwidth=xw)
    ref, st = _stable_lanes(oracle, run, x0)
    assert st.mean() > 0.5, st.mean()
    # the disturbed state itself (step td, before the solve), re-projected s included, as the literal
    # oracle to 1e-8 on the stable lanes (the first td - 1 closed-loop steps carry the two
    # formulations' rounding differences; bit-for-bit equality with the kernel-order twin is
    # tests/test_gpu_twin.py::test_closed_loop_variants_bit_identical).  Measured: <= 2.4e-10 on every
    # stable lane; lane 0 is not one -- its closed loop is chaotic before the disturbance (its pre-disturbance state
    # already differs by 3.4e-6 between the two formulations, so its re-projected s by 2.7e-6; the
    # round-3 note blamed the Newton stop, but the re-projection adds nothing measurable)
    assert not st[0]
    np.testing.assert_allclose(r["X"][st, td - 1, :], ref["X"][st, td - 1, :], rtol=0, atol=1e-8)
    assert np.abs(r["U"] - ref["U"]).max(axis=(1, 2))[st].max() < 1e-6
    assert np.abs(r["X"] - ref["X"]).max(axis=(1, 2))[st].max() < 1e-8
    # the re-projected s is wrapped into [-b, b) (helper.m:233)
    b = oracle.tab["params"][sid, 0]
    assert np.all(np.abs(r["X"][:, td - 1, 3]) <= b)


def test_reproject_contact_matches_oracle(oracle):
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    gpu = OcpSolver(N=10, batch=1)
    gpu.set_shapes([make_shape(n) for n in NAMES])
    rng = np.random.default_rng(9)
    n = 400
    sid = rng.integers(0, 4, n)
    b = oracle.tab["params"][sid, 0]
    s_true = rng.uniform(0, 1, n) * b
    C = oracle.spline(s_true, sid)[0]
    px = C[:, 0] + rng.normal(0, 2e-3, n)
    py = C[:, 1] + rng.normal(0, 2e-3, n)
    s0 = s_true + rng.uniform(-0.02, 0.02, n)
    so = oracle.reproject_contact(px, py, s0, sid)
    sg = gpu.reproject_contact(px, py, s0, sid)
    gpu.close()
    np.testing.assert_allclose(sg, so, rtol=0, atol=1e-8)
    # stationary point of |C(s) - p|^2: the tangent is orthogonal to C(s) - p
    Cs, dCs, D, dD, _ = oracle.spline(np.mod(so, b), sid)
    g = (Cs[:, 0] - px) * D[:, 0] + (Cs[:, 1] - py) * D[:, 1]
    assert np.abs(g).max() < 1e-8


def test_delay_buffer_mirror(oracle):
    """NMPC_controller.delay_buffer_sim + the helper's buffer push through the controller mirror."""
    from uclv_qs_pushing_matlab_amd.controller import NMPCController
    from uclv_qs_pushing_matlab_amd.model import PusherSliderModel
    from uclv_qs_pushing_matlab_amd.objects import object_selection
    plant = PusherSliderModel("real_plant", object_selection("santal"), 0.0, object_name="santal")
    c = NMPCController("nmpc", plant, 0.05, 10, batch=3, nlp_solver_type="SQP_RTI", sqp_iters=2)
    c.create_ocp_solver()
    c.set_delay_comp(0.12)
    assert c.delay_buff_comp == 3
    x = config2_x0(3, 5)
    np.testing.assert_array_equal(c.delay_buffer_sim(plant, x), x)        # empty buffer: zero inputs, f(x, 0) = 0
    us = [np.array([[0.01, 0.002]] * 3) * (k + 1) for k in range(4)]
    for u in us:
        c.push_u_buffer(u)
    xs = c.delay_buffer_sim(plant, x)
    ref = x.copy()
    for u in (us[1], us[2], us[3]):                                       # oldest of the 3 kept first
        f, _ = oracle.dynamics(ref, u)
        ref = ref + 0.05 * f
    np.testing.assert_allclose(xs, ref, rtol=0, atol=1e-12)


def test_closed_loop_bench_line():
    """bench.py --closed-loop (SURVEY §8(f) row 1 measured): one JSON line, every sampled closed loop
    bit-identical to the twin's (X, U, status over all 201 steps of main.m's scenario)."""
    import subprocess
    import sys
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--closed-loop", "--global-batch", "192",
                          "--steps", "1", "--cpu-seconds", "1"], capture_output=True, text=True, timeout=200, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["unit"] == "lane-steps/s" and d["value"] > 0
    p = d["parity"]
    assert p["lanes"] >= 16 and p["bit_identical_trajectory_lanes"] == p["lanes"], p
