"""GPU: the reference-interface mirrors (PusherSliderModel, NMPCController,
TrajectoryGenerator) driving the HIP path, main.m-style, against the committed
oracle golden closed loop (config 1) and the oracle's model functions."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _plant(name="santal"):
    from uclv_qs_pushing_matlab_amd.model import PusherSliderModel
    from uclv_qs_pushing_matlab_amd.objects import object_selection
    return PusherSliderModel("plant", object_selection(name), object_name=name)


def test_model_mirror_matches_oracle(oracle):
    plant = _plant()
    rng = np.random.default_rng(3)
    x = np.stack([rng.uniform(-0.05, 0.05, 300), rng.uniform(-0.05, 0.05, 300), rng.uniform(-3, 3, 300),
                  rng.uniform(-0.2, 0.2, 300)], 1)
    u = np.stack([rng.uniform(0, 0.03, 300), rng.uniform(-0.05, 0.05, 300)], 1)
    f = plant.evalModelVariableShape(x, u)
    fo, Jo = oracle.dynamics(x, u, 0)
    np.testing.assert_allclose(f, fo, rtol=1e-10, atol=1e-14)
    np.testing.assert_allclose(plant.jacobian(x, u), Jo, rtol=1e-8, atol=1e-10)
    s = np.linspace(0, plant.SP.b, 97)
    # FC wraps with MATLAB mod (bspline_shape.m:147): FC(b) = FC(0)
    np.testing.assert_allclose(plant.SP.FC(s), oracle.spline(np.mod(s, plant.SP.b), 0)[0], rtol=1e-12, atol=1e-15)
    R = plant.SP.R_NT(s[:-1])
    np.testing.assert_allclose(np.einsum("nij,nik->njk", R, R), np.broadcast_to(np.eye(2), R.shape), atol=1e-12)


@pytest.mark.parametrize("N", [10, 20])
def test_controller_mirror_config1_golden(N):
    """main.m:150-199 with the mirrors: waypoint reference, NMPCController.solve, Euler plant."""
    from uclv_qs_pushing_matlab_amd.controller import NMPCController
    from uclv_qs_pushing_matlab_amd.trajectory import TrajectoryGenerator
    gold = json.load(open(os.path.join(GOLDEN, "config1_closed_loop.json")))[f"N{N}"]
    plant = _plant()
    ctrl = NMPCController("nmpc", plant, 0.05, N, batch=1, nlp_solver_type="SQP_RTI", sqp_iters=5)
    ctrl.create_ocp_solver()
    tg = TrajectoryGenerator(0.05, 0.01)
    tg.set_target(np.zeros(4), np.zeros(5), 0.0, 10.0)
    tg.waypoints_ = np.array([[0, 0, 0], [0.10, 0, 0]])
    tg.waypoints_velocities = [0.010]
    _, traj = tg.waypoints_gen()
    y_ref = np.zeros((6, traj.shape[1]))
    y_ref[:3] = traj[:3]
    ctrl.initial_condition_update(np.zeros(4))          # main.m:79, clears y_ref (NMPC_controller.m:144-151)
    ctrl.set_reference_trajectory(y_ref)                # main.m:178
    x = np.zeros(4)
    for i in range(1, 21):
        u = ctrl.solve(x, i)[0]
        np.testing.assert_allclose(u, gold["u0"][i - 1], rtol=0, atol=1e-8, err_msg=f"step {i}")
        x = x + 0.05 * plant.evalModelVariableShape(x[None], u[None])[0]
    np.testing.assert_allclose(x, gold["x_final"], atol=1e-9)
    assert len(ctrl.cost_function_vect) == 20


def test_helper_closed_loop_mirror():
    """helper.closed_loop_matlab over the mirrors reproduces the config-1 golden trace."""
    from uclv_qs_pushing_matlab_amd.controller import NMPCController
    from uclv_qs_pushing_matlab_amd.helper import closed_loop_matlab
    gold = json.load(open(os.path.join(GOLDEN, "config1_closed_loop.json")))["N20"]
    plant = _plant()
    ctrl = NMPCController("nmpc", plant, 0.05, 20, batch=2, nlp_solver_type="SQP_RTI", sqp_iters=5)
    ctrl.create_ocp_solver()
    ctrl.initial_condition_update(np.zeros(4))
    y_ref = np.zeros((6, 201))
    y_ref[0] = 0.01 * np.arange(201) * 0.05
    ctrl.set_reference_trajectory(y_ref)
    out = closed_loop_matlab(plant, ctrl, np.zeros(4), 10.0)
    u_n, u_t, found = out[6], out[7], out[10]
    assert u_n.shape == (2, 201) and np.all(found)
    np.testing.assert_allclose(np.stack([u_n[0, :20], u_t[0, :20]], 1), gold["u0"], atol=1e-9)
    # the slider tracks the 0.01 m/s line
    assert abs(out[0][0, -1] - 0.01 * 10.0) < 0.02


def test_acados_timing_fields():
    """get('time_tot'/'time_lin'/'time_qp_sol') as helper.m:264-269 prints them."""
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    from conftest import straight_traj
    s = OcpSolver(N=20, batch=64, sqp_iters=5, timings=True)
    s.set_shapes([make_shape("santal")])
    s.set_reference_trajectory(straight_traj())
    s.controller_solve(np.zeros((64, 4)), 1)
    tt, tl, tq = s.get("time_tot"), s.get("time_lin"), s.get("time_qp_sol")
    s.close()
    # nlp_mode 0 linearises inside the qp_step kernel: time_lin is the wave-packing sort only
    assert 0 <= tl < tt and 0 < tq < tt and tl + tq <= tt * 1.05
