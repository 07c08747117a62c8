"""BASELINE configs[4] at its full size: N = 50, B = 16 384, the curved x_finals.mat reference with a
random start index per lane, four shapes mixed per lane, K = 50 SQP-RTI iterations (bench.py
--config 4's input law and seed), on the host-boundary controller path.

* every status is 0 and u0 is finite;
* lanes are independent: a shuffled batch gives every lane the same bits, and so does a small
  batch holding some of the same lanes (the layout at N = 50 is two stages per lane, and the
  packing moves instances between waves and groups);
* u0 agrees with the oracle on the first lanes that the oracle itself reproduces (the probe
  criterion of tests/test_gpu_config2.py; full-step SQP at N = 50 settles on fewer lanes)."""
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

    nl = 64

    def run(xx, **kw):
        return oracle.controller_solve(make_opts(N=N, sqp_iters=K, **kw), xx, traj, idx[:nl],
                                       oracle.new_warm(nl, N), shape_id=sid[:nl])
    ref = run(x0[:nl])
    dev = np.zeros(nl)
    for f in (1e-13, -1e-13, 3e-13):
        dev = np.maximum(dev, np.abs(run(x0[:nl] * (1 + f))["u0"] - ref["u0"]).max(1))
    dev = np.maximum(dev, np.abs(run(x0[:nl], mu_stop=1.5e-10)["u0"] - ref["u0"]).max(1))
    nonchaotic = (dev < 1e-9) & (ref["status"] == 0)
    d = np.abs(u[:nl] - ref["u0"]).max(1)
    assert nonchaotic.sum() >= 10, nonchaotic.sum()
    assert np.mean(d[nonchaotic] < 1e-6) >= 0.95, np.sort(d[nonchaotic])[-5:]
