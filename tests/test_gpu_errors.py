"""GPU: argument and state errors of the C ABI raise (no silent fallback), and device-side
shape ids from qsp_solve_device are clamped into the shape table."""
import ctypes as C

import numpy as np
import pytest

from conftest import straight_traj

pytestmark = pytest.mark.gpu


def test_state_and_argument_errors():
    from uclv_qs_pushing_matlab_amd import _lib
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    s = OcpSolver(N=10, batch=4)
    with pytest.raises(_lib.QspError, match="no shapes"):
        s.solve()
    with pytest.raises(_lib.QspError, match="reference"):
        s.controller_solve(np.zeros((4, 4)), 1)
    s.set_shapes([make_shape("santal"), make_shape("balea")])
    with pytest.raises(_lib.QspError, match="out of range"):
        s.set_shape_ids([0, 1, 2, 0])
    with pytest.raises(_lib.QspError, match="out of range"):
        s.eval_spline(np.zeros(3), [0, 5, 1])
    bad = make_shape("santal")
    bad.n_ctrl = 80
    with pytest.raises(_lib.QspError, match="n_ctrl"):
        s.set_shapes([bad])
    L = _lib.lib()
    assert L.qsp_set_reference_trajectory(s.handle, None, 10) == -1
    with pytest.raises(_lib.QspError, match="nlp_mode 1"):
        s.get("residuals")
    s.close()
    # residuals before the first solve: zeros (qsp_nmpc.h), not uninitialised device memory
    for poison in ("0", "1"):
        import os
        os.environ["QSP_DEBUG_POISON"] = poison
        try:
            m = OcpSolver(N=10, batch=5, nlp_solver_type="SQP")
        finally:
            os.environ.pop("QSP_DEBUG_POISON")
        np.testing.assert_array_equal(m.get("residuals"), np.zeros((5, 4)))
        m.close()
    s = OcpSolver(N=10, batch=4)
    s.set_shapes([make_shape("santal")])
    with pytest.raises(ValueError):
        s.set("cost_y_ref", np.zeros((3, 3)))
    with pytest.raises(KeyError):
        s.get("no_such_field")
    s.close()


def test_device_shape_ids_are_clamped():
    import torch
    from uclv_qs_pushing_matlab_amd._lib import DeviceIO
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N, B = 10, 6
    names = ("santal", "balea")
    s = OcpSolver(N=N, batch=B, sqp_iters=2)
    s.set_shapes([make_shape(n) for n in names])
    dev = torch.device("cuda", 0)
    traj = straight_traj()
    x0 = torch.zeros((B, 4), dtype=torch.float64, device=dev)
    yref = torch.as_tensor(np.broadcast_to(traj[None, :N], (B, N, 6)).copy(), device=dev)
    yref_e = yref[:, N - 1, :4].contiguous()
    outs = {k: torch.zeros(sh, dtype=torch.float64, device=dev) for k, sh in
            (("X_in", (B, N + 1, 4)), ("U_in", (B, N, 2)), ("u0", (B, 2)), ("X_out", (B, N + 1, 4)),
             ("U_out", (B, N, 2)), ("PI_out", (B, N, 4)), ("cost", (B,)))}
    status = torch.zeros(B, dtype=torch.int32, device=dev)

    def run(ids):
        sid = torch.as_tensor(np.asarray(ids, np.int32), device=dev)
        io = DeviceIO()
        io.x0, io.yref, io.yref_e = x0.data_ptr(), yref.data_ptr(), yref_e.data_ptr()
        for k, v in outs.items():
            setattr(io, k, v.data_ptr())
        io.shape_id, io.status, io.controller = sid.data_ptr(), status.data_ptr(), 1
        s.solve_device(io, None)
        s.synchronize()
        return outs["u0"].cpu().numpy().copy()
    u_bad = run([-3, 0, 1, 1, 7, 100])
    u_ok = run([0, 0, 1, 1, 1, 1])
    s.close()
    np.testing.assert_array_equal(u_bad, u_ok)
    assert np.all(status.cpu().numpy() == 0)


@pytest.mark.parametrize("mode,S,fused", [("SQP_RTI", 1, "0"), ("SQP_RTI", 1, "1"), ("SQP_RTI", 2, "0"),
                                          ("SQP_RTI", 2, "1"), ("SQP", 1, "0")])
def test_no_uninitialised_reads(monkeypatch, mode, S, fused):
    """QSP_DEBUG_POISON=1 fills every workspace buffer and the QP kernels' LDS with NaN
    before use (the fused SQP-loop kernel re-poisons its LDS at every SQP iteration): a kernel
    that reads a word it never wrote would change the result.  Both the per-iteration QP
    kernel (QSP_FUSED_LOOP=0, which every bench-size batch uses) and the fused loop."""
    monkeypatch.setenv("QSP_FUSED_LOOP", fused)
    from conftest import config2_x0
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N, B = 20, 70
    x0 = config2_x0(B, 77)
    sid = np.arange(B) % 4

    def run():
        s = OcpSolver(N=N, batch=B, sqp_iters=6, stages_per_lane=S, nlp_solver_type=mode)
        s.set_shapes([make_shape(n) for n in ("santal", "balea", "montana", "pulirapid")], shape_id=sid)
        s.set_reference_trajectory(straight_traj())
        u1 = s.controller_solve(x0, 1)
        u2 = s.controller_solve(x0 * 0.9, 2)          # warm path
        out = (u1, u2, s.get("status"), s.get("x"), s.get("pi"))
        s.close()
        return out
    clean = run()
    monkeypatch.setenv("QSP_DEBUG_POISON", "1")
    poisoned = run()
    for a, b in zip(clean, poisoned):
        np.testing.assert_array_equal(a, b)
    assert np.all(clean[2] == (0 if mode == "SQP_RTI" else clean[2]))


@pytest.mark.parametrize("mode,B", [("SQP_RTI", 8192), ("SQP", 8192), ("SQP_RTI", 96)])
def test_qp_iters_beyond_packing_levels(mode, B):
    """qp_iters > 31 (acados' default cap is 50): the wave-packing keys clamp their levels at 31,
    the packing stays on (per-iteration launches, two stream parts at B = 8 192), and every lane
    gets the bits it gets when solved in a batch of its own kind (instances are independent)."""
    from conftest import config2_x0
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N = 20
    x0 = config2_x0(B, 91)
    sid = np.arange(B) % 4
    names = ("santal", "balea", "montana", "pulirapid")

    def run(n, qp_iters):
        s = OcpSolver(N=N, batch=n, sqp_iters=8, qp_iters=qp_iters, nlp_solver_type=mode)
        s.set_shapes([make_shape(q) for q in names], shape_id=sid[:n])
        s.set_reference_trajectory(straight_traj())
        u = s.controller_solve(x0[:n], 1)
        out = (u, s.get("status"), s.get("qp_iter"), s.get("qp_capped"), s.stream_parts())
        s.close()
        return out
    u, st, qi, cap, parts = run(B, 40)
    assert np.all(np.isfinite(u)) and set(np.unique(st)) <= {0, 2}
    u_s, st_s, qi_s, cap_s, _ = run(64, 40)
    np.testing.assert_array_equal(u[:64], u_s)
    np.testing.assert_array_equal(qi[:64], qi_s)
    np.testing.assert_array_equal(cap[:64], cap_s)
    if B >= 8192:
        assert parts == 2


def test_stage0_s_bound_infeasible(oracle):
    """stage0_s_bound (default on, acados bgh at stage 0): an x0 whose s lies outside
    [lh_s, uh_s] = [-0.06, 0.011] makes every QP infeasible -> status 4 (ACADOS_QP_FAILURE),
    sqp_iter 0, the other lanes unaffected; with the option off the lane solves (status 0)."""
    from conftest import config2_x0
    from oracle.oracle import make_opts
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N, B, K = 20, 8, 5
    x0 = config2_x0(B, 3)
    x0[2, 3] = 0.05          # above uh_s
    x0[5, 3] = -0.07         # below lh_s
    traj = straight_traj()
    res = {}
    for on in (True, False):
        s = OcpSolver(N=N, batch=B, sqp_iters=K, stage0_s_bound=on)
        s.set_shapes([make_shape("santal")])
        s.set_reference_trajectory(traj)
        u = s.controller_solve(x0, 1)
        res[on] = (u, s.get("status"), s.get("sqp_iter"))
        s.close()
        r = oracle.controller_solve(make_opts(N=N, sqp_iters=K, stage0_s_bound=int(on)), x0, traj, 1,
                                    oracle.new_warm(B, N))
        ok = np.ones(B, bool)
        ok[[2, 5]] = False        # with the option off their QPs are infeasible from stage 1 on: junk iterates
        np.testing.assert_array_equal(res[on][1][ok], r["status"][ok])
        np.testing.assert_array_equal(res[on][2][ok], r["iters"][ok])
        np.testing.assert_allclose(u[ok], r["u0"][ok], rtol=0, atol=1e-5)   # K = 5 full steps
        if on:
            np.testing.assert_array_equal(res[on][1], r["status"])
            np.testing.assert_allclose(u[[2, 5]], r["u0"][[2, 5]], rtol=0, atol=1e-12)   # the initial guess
    u, st, it = res[True]
    assert list(np.where(st != 0)[0]) == [2, 5] and np.all(st[[2, 5]] == 4) and np.all(it[[2, 5]] == 0)
    assert np.all(res[False][1] == 0)
