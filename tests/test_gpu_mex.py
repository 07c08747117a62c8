"""The MATLAB boundary, functionally: integration/matlab/qsp_nmpc_mex.c compiled unmodified against
a functional stand-in for the MEX API (tests/stubs/mex_stub.c; MATLAB is not in this image) and
driven like NMPC_controller_hip.m + main.m (tests/stubs/mex_driver.c): the reference's solver
options by default (sqp + merit backtracking, max_iter 30, tol 1e-6, NMPC_controller.m:271-276),
Hp = 10, santal, 201 closed-loop steps, status / sqp_iter / time_lin / time_qp_sol read back
(helper.m:253-269), argument checks raising MEX errors.  The trace must match main.m's golden run
(tests/golden/main_m_sqp_closed_loop.npz, oracle)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu


def test_mex_gateway_drives_main_m(tmp_path):
    exe = tmp_path / "mex_driver"
    lib = os.path.join(ROOT, "uclv_qs_pushing_matlab_amd")
    subprocess.check_call(["gcc", "-std=c99", "-D_DEFAULT_SOURCE", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           "-I", os.path.join(ROOT, "tests", "stubs"),
                           os.path.join(ROOT, "integration", "matlab", "qsp_nmpc_mex.c"),
                           os.path.join(ROOT, "tests", "stubs", "mex_stub.c"),
                           os.path.join(ROOT, "tests", "stubs", "mex_driver.c"),
                           "-L", lib, "-lqsp_nmpc", f"-Wl,-rpath,{lib}", "-lm", "-o", str(exe)])
    ply = os.path.join(lib, "data", "planar_surface_santal_36_uniformed.ply")
    out = tmp_path / "out.bin"
    r = subprocess.run([str(exe), ply, str(out)], capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    raw = out.read_bytes()
    S = 201
    U = np.frombuffer(raw, np.float64, S * 2, 0).reshape(S, 2)
    X = np.frombuffer(raw, np.float64, (S + 1) * 4, S * 16).reshape(S + 1, 4)
    off = S * 16 + (S + 1) * 32
    st = np.frombuffer(raw, np.int32, S, off)
    it = np.frombuffer(raw, np.int32, S, off + 4 * S)
    errors, t_lin, t_qp, t_tot = np.frombuffer(raw, np.float64, 4, off + 8 * S)
    res = np.frombuffer(raw, np.float64, S * 4, off + 8 * S + 32).reshape(S, 4)
    assert errors == 7
    gold = np.load(os.path.join(GOLDEN, "main_m_sqp_closed_loop.npz"))
    np.testing.assert_allclose(U, gold["U"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(X, gold["X"], rtol=0, atol=1e-7)
    np.testing.assert_array_equal(st, gold["status"])
    assert np.mean(it == gold["iters"]) > 0.95
    assert t_qp > 0 and t_lin > 0 and t_tot >= t_qp
    # get('residuals'): the KKT residuals of each step's last test -- all below tol 1e-6 where the
    # SQP converged, at least one at or above it where it stopped at max_iter
    conv, capped = st == 0, st == 2
    assert np.all(res[conv] < 1e-6)
    assert np.all(res[capped].max(1) >= 1e-6)
