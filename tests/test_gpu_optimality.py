"""GPU: the solver's converged answers are local minima of the OCP, checked without the oracle's
solver (only its RK4 is used, to roll candidate control trajectories out).

This restates the reference's own optimality probe, `helper.debug_cost_function`
(`helper.m:369-451`). That probe grid-searches u_0 over [u_n_lb:0.005:u_n_ub] x
[u_t_lb:0.005:u_t_ub] with the rest of the control trajectory fixed, rolls each candidate out
and compares its cost with the solver's u_0. The reference used the fixed-shape `eval_model`
there (`PusherSliderModel.m:200`). Here the probe uses the OCP's own model (RK4 of f,
`PusherSliderModel.m:503-603`) and its cost (`NMPC_controller.m:185-218`, stage term x Ts), on a
grid local enough for a nonconvex problem.
* u_0 on a 9 x 9 grid of +-2e-4 around the solution;
* every stage at once: U* + eps d for random d, projected onto the input bounds.
Candidates whose rollout leaves the s bound are skipped (the probe compares feasible points
only). On lanes where the merit SQP converged (status 0, KKT tolerances 1e-6), no feasible
candidate may cost less than the solution beyond rounding."""
import numpy as np
import pytest

from conftest import config2_x0, straight_traj

pytestmark = pytest.mark.gpu

NAMES = ("santal", "balea", "montana", "pulirapid")
W = np.array([1.0, 1.0, 1e-3, 0.0, 1e-3, 1e-3])      # main.m:82-86 (x 0.01 folded), NMPC_controller.m:16-18
WE = np.array([2e5, 2e5, 20.0, 0.0])
LH = np.array([-0.06, 0.0, -0.05])                   # NMPC_controller.m:23-26, 83-84
UH = np.array([0.011, 0.03, 0.05])
TS = 0.05


def _rollout_cost(oracle, x0, U, sid, yref, yref_e):
    """Cost and s-feasibility of candidate control trajectories U (m, N, 2) from x0."""
    m, N = U.shape[0], U.shape[1]
    x = np.repeat(x0[None], m, 0)
    J = np.zeros(m)
    feas = np.ones(m, bool)
    for k in range(N):
        e = np.concatenate([x, U[:, k]], 1) - yref[k]
        J += 0.5 * TS * (W * e * e).sum(1)
        if k >= 1:
            feas &= (x[:, 3] >= LH[0]) & (x[:, 3] <= UH[0])
        x = oracle.rk4(x, U[:, k], TS, np.full(m, sid))[0]
    e = x - yref_e
    return J + 0.5 * (WE * e * e).sum(1), feas


def test_converged_solutions_are_local_minima(oracle):
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N, nb, K = 20, 64, 30
    x0 = config2_x0(nb, 21)
    sid = np.arange(nb) % 4
    traj = straight_traj()
    yref = np.repeat(traj[None, :N], nb, 0)
    yref_e = yref[:, N - 1, :4].copy()
    s = OcpSolver(N=N, batch=nb, sqp_iters=K, nlp_solver_type="SQP")
    s.set_shapes([make_shape(n) for n in NAMES], shape_id=sid)
    s.set("constr_x0", x0)
    s.set("cost_y_ref", yref)
    s.set("cost_y_ref_e", yref_e)
    s.set("init_x", np.repeat(x0[:, None], N + 1, 1))
    s.set("init_u", np.zeros((nb, N, 2)))
    s.solve()
    U, status = s.get("u"), s.get("status")
    s.close()
    conv = np.nonzero(status == 0)[0]
    assert len(conv) >= 10, len(conv)
    rng = np.random.default_rng(5)
    grid = np.linspace(-2e-4, 2e-4, 9)
    worst_grid, worst_dir = np.inf, np.inf
    for l in conv:
        J0, f0 = _rollout_cost(oracle, x0[l], U[l][None], sid[l], yref[l], yref_e[l])
        assert f0[0], l
        cand = np.repeat(U[l][None], len(grid) ** 2, 0)
        cand[:, 0, 0] += np.repeat(grid, len(grid))
        cand[:, 0, 1] += np.tile(grid, len(grid))
        ok = np.all((cand[:, 0] >= LH[1:]) & (cand[:, 0] <= UH[1:]), 1)
        Jg, fg = _rollout_cost(oracle, x0[l], cand[ok], sid[l], yref[l], yref_e[l])
        worst_grid = min(worst_grid, ((Jg[fg] - J0[0]) / J0[0]).min())
        d = rng.standard_normal((64, N, 2))
        cand = np.clip(np.concatenate([U[l][None] + 1e-4 * d, U[l][None] - 1e-4 * d]), LH[1:], UH[1:])
        Jd, fd = _rollout_cost(oracle, x0[l], cand, sid[l], yref[l], yref_e[l])
        assert fd.sum() >= 16, (l, fd.sum())
        worst_dir = min(worst_dir, ((Jd[fd] - J0[0]) / J0[0]).min())
    # oracle's own converged solutions: grid -1.9e-12, projected directions +5.6e-4 (no descent)
    assert worst_grid > -1e-9, worst_grid
    assert worst_dir > -1e-9, worst_dir
