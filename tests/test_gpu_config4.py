"""BASELINE configs[4] at its full size: N = 50, B = 16 384, the curved x_finals.mat reference with a
random start index per lane, four shapes mixed per lane, K = 50 SQP-RTI iterations (bench.py
--config 4's input law and seed), on the host-boundary controller path.

* every status is 0 and u0 is finite;
* lanes are independent: a shuffled batch gives every lane the same bits, and so does a small
  batch holding some of the same lanes (the layout at N = 50 is two stages per lane, and the
  packing moves instances between waves and groups);
* u0 agrees with the literal oracle on the first 1 024 lanes wherever neither implementation moves
  under the probe criterion of tests/test_gpu_config2.py (full-step SQP at N = 50 settles on fewer
  lanes); where they disagree, tests/test_extended_oracle.py and bench's configs4.parity_literal
  adjudicate in extended precision."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NAMES = ("santal", "balea", "montana", "pulirapid")


def _solver(B, N, K):
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    s = OcpSolver(N=N, batch=B, sqp_iters=K)
    s.set_shapes([make_shape(n) for n in NAMES])
    return s


def test_config4_full_batch(oracle):
    from bench import SEED, config4_inputs
    from oracle.oracle import make_opts
    B, N, K = 16384, 50, 50
    x0, _, _, sid, traj, idx = config4_inputs(B, N, SEED)
    s = _solver(B, N, K)
    assert s.layout()[0] == 2
    s.set_reference_trajectory(traj)
    s.set_shape_ids(sid)
    u = s.controller_solve(x0, idx)
    st = s.get("status")
    perm = np.random.default_rng(4).permutation(B)
    s.set_shape_ids(sid[perm])
    s.controller_reset()
    up = s.controller_solve(x0[perm], idx[perm])
    s.close()
    assert np.all(st == 0) and np.all(np.isfinite(u))
    np.testing.assert_array_equal(up, u[perm])
    pick = np.r_[0:5, B // 2:B // 2 + 3, B - 5:B]
    small = _solver(len(pick), N, K)
    small.set_reference_trajectory(traj)
    small.set_shape_ids(sid[pick])
    us = small.controller_solve(x0[pick], idx[pick])
    small.close()
    np.testing.assert_array_equal(us, u[pick])

    # the literal restatement (oracle/qsp_oracle.c) on the first 1 024 lanes, with the probe criterion
    # in both implementations: the oracle's own response to three 1e-13 relative x0 perturbations and
    # mu_stop 1.5e-10, the GPU's to the same x0 perturbations
    nl = 1024

    def run(xx, **kw):
        return oracle.controller_solve(make_opts(N=N, sqp_iters=K, **kw), xx, traj, idx[:nl],
                                       oracle.new_warm(nl, N), shape_id=sid[:nl])
    ref = run(x0[:nl])
    xdev = np.zeros(nl)
    for f in (1e-13, -1e-13, 3e-13):
        xdev = np.maximum(xdev, np.abs(run(x0[:nl] * (1 + f))["u0"] - ref["u0"]).max(1))
    dev = np.maximum(xdev, np.abs(run(x0[:nl], mu_stop=1.5e-10)["u0"] - ref["u0"]).max(1))
    s = _solver(nl, N, K)
    s.set_reference_trajectory(traj)
    s.set_shape_ids(sid[:nl])
    gdev = np.zeros(nl)
    for f in (1e-13, -1e-13, 3e-13):
        s.controller_reset()
        gdev = np.maximum(gdev, np.abs(s.controller_solve(x0[:nl] * (1 + f), idx[:nl]) - u[:nl]).max(1))
    s.close()
    nonchaotic = (dev < 1e-9) & (ref["status"] == 0)
    d = np.abs(u[:nl] - ref["u0"]).max(1)
    # measured (twin = GPU bit for bit, 1 024 lanes): N = 50's full-step SQP settles on fewer lanes
    # than N = 20 -- 37 % of them move by > 1e-6 under the 1e-13 x0 probes, in both implementations,
    # 73 % of the oracle's once mu_stop moves too -- and on every lane that neither implementation's
    # probes move, the two agree within 1e-6 (240 lanes at 1e-9, 278 at 1e-6, none off)
    assert nonchaotic.sum() >= 200, nonchaotic.sum()
    assert d[nonchaotic].max() < 1e-6, np.sort(d[nonchaotic])[-5:]
    both = (dev <= 1e-6) & (gdev <= 1e-6)
    assert both.sum() >= 250, both.sum()
    assert np.all(d[both] <= 1e-6), np.flatnonzero(both & (d > 1e-6))[:10]
    assert abs(np.mean(gdev > 1e-6) - np.mean(xdev > 1e-6)) < 0.05, (np.mean(gdev > 1e-6), np.mean(xdev > 1e-6))
