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


@pytest.mark.parametrize("mode,S", [("SQP_RTI", 1), ("SQP_RTI", 2), ("SQP", 1)])
def test_no_uninitialised_reads(monkeypatch, mode, S):
    """QSP_DEBUG_POISON=1 fills every workspace buffer and the QP kernels' LDS with NaN
    before use: a kernel that reads a word it never wrote would change the result."""
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
