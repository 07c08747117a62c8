"""GPU: per-lane reference tables and the device TrajectoryGenerator.straight_line
(TrajectoryGenerator.m:39-79) against the host mirror; controller solves staged from
per-lane tables against the oracle lane by lane."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NAMES = ("santal", "balea", "montana", "pulirapid")


@pytest.mark.parametrize("auto_angle", [False, True])
def test_device_straight_lines_match_mirror(auto_angle):
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    from uclv_qs_pushing_matlab_amd.trajectory import TrajectoryGenerator
    B = 16
    rng = np.random.default_rng(9)
    x0 = rng.uniform(-0.05, 0.05, (B, 3))
    xf = x0 + rng.uniform(0.02, 0.2, (B, 3))
    s = OcpSolver(N=10, batch=B)
    s.set_shapes([make_shape("santal")])
    T = s.gen_straight_lines(x0, xf, 0.0, 10.0, auto_angle)
    assert T == 201
    tab = s.get_reference_trajectories()
    s.close()
    for i in range(B):
        tg = TrajectoryGenerator(0.05, 0.01)
        tg.set_target(x0[i], xf[i], 0.0, 10.0)
        _, ref = tg.straight_line(auto_angle)
        np.testing.assert_allclose(tab[i, :, :3], ref.T, rtol=1e-14, atol=1e-15)
        assert np.all(tab[i, :, 3:] == 0.0)


def test_controller_with_per_lane_references(oracle):
    from oracle.oracle import make_opts
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N, B, K = 20, 8, 3
    rng = np.random.default_rng(4)
    x0 = np.zeros((B, 3))
    xf = np.stack([rng.uniform(0.05, 0.15, B), rng.uniform(-0.05, 0.05, B), np.zeros(B)], 1)
    sid = np.arange(B) % 4
    s = OcpSolver(N=N, batch=B, sqp_iters=K)
    s.set_shapes([make_shape(n) for n in NAMES], shape_id=sid)
    s.gen_straight_lines(x0, xf, 0.0, 10.0)
    tab = s.get_reference_trajectories()
    idx = rng.integers(1, 150, B).astype(np.int32)
    xs = np.concatenate([tab[np.arange(B), idx - 1, :3], np.zeros((B, 1))], 1)
    u = s.controller_solve(xs, idx)
    s.close()
    op = make_opts(N=N, sqp_iters=K)
    for i in range(B):
        r = oracle.controller_solve(op, xs[i:i + 1], tab[i], int(idx[i]), oracle.new_warm(1, N), shape_id=sid[i:i + 1])
        assert np.abs(u[i] - r["u0"][0]).max() < 1e-8, (i, u[i], r["u0"][0])
