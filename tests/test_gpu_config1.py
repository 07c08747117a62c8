"""BASELINE configs[1] in full against the oracle: B = 4 096 random x0 around santal (the config-2
x0 law of main.m:53-56, bench.py's seed), the straight reference of main.m:150-164, N = 20, K = 50
SQP-RTI iterations, cold-start NMPC_controller.solve, on the host-boundary controller path (the
bench's configs1 leg). Every lane is checked against the oracle with the probe criterion of
tests/test_gpu_config2.py: on lanes whose oracle answer survives 1e-13 x0 perturbations and
mu_stop 1.5e-10, u0 agrees within 1e-6 (BASELINE); on all lanes, the GPU agrees with the oracle
about as often as the perturbed oracle agrees with itself; and the GPU's own response to the same
perturbations marks the same lanes as chaotic, which are the lanes where the two disagree."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_config1_full_batch_parity(oracle):
    from bench import config1_inputs
    from oracle.oracle import make_opts
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N, K = 20, 50
    x0, traj, sid = config1_inputs(N)
    B = len(x0)
    assert B == 4096
    s = OcpSolver(N=N, batch=B, sqp_iters=K)
    s.set_shapes([make_shape("santal")], shape_id=sid)
    s.set_reference_trajectory(traj)
    u0 = s.controller_solve(x0, 1).copy()
    status, capped = s.get("status"), s.get("qp_capped")
    # the GPU's own sensitivity to the same 1e-13 x0 perturbations
    gpu_dev = np.zeros(B)
    for f in (1e-13, -1e-13, 3e-13):
        s.controller_reset()
        gpu_dev = np.maximum(gpu_dev, np.abs(s.controller_solve(x0 * (1 + f), 1) - u0).max(1))
    s.close()
    assert np.all(status == 0)

    def run(xx, **kw):
        return oracle.controller_solve(make_opts(N=N, sqp_iters=K, **kw), xx, traj, 1, oracle.new_warm(B, N),
                                       shape_id=sid)
    ref = run(x0)
    # the literal oracle's only failure (lane 1949, SQP iteration 11) is a QP that diverges -- its
    # 2x2 stage inverse breaks down and mu turns non-finite -- which both implementations report as
    # a QP failure (status 4, acados ACADOS_QP_FAILURE), never as status 1; the lane is chaotic (a
    # 1e-13 perturbation of its x0 lets the oracle solve it), and the device solves it
    assert set(np.unique(ref["status"])) <= {0, 4}
    np.testing.assert_array_equal(np.flatnonzero(ref["status"]), [1949])
    self_dev = np.zeros(B)
    st_moves = np.zeros(B, bool)
    for f in (1e-13, -1e-13, 3e-13):
        rp = run(x0 * (1 + f))
        self_dev = np.maximum(self_dev, np.abs(rp["u0"] - ref["u0"]).max(1))
        st_moves |= rp["status"] != ref["status"]
    assert st_moves[1949]
    mu_dev = np.abs(run(x0, mu_stop=1.5e-10)["u0"] - ref["u0"]).max(1)
    stable = (self_dev <= 1e-6) & (gpu_dev <= 1e-6) & ~st_moves
    np.testing.assert_array_equal(status[stable], ref["status"][stable])
    nonchaotic = (self_dev < 1e-9) & (mu_dev < 1e-9) & (ref["status"] == 0)
    d = np.abs(u0 - ref["u0"]).max(1)
    assert nonchaotic.mean() > 0.6, nonchaotic.mean()
    assert np.mean(d[nonchaotic] < 1e-6) >= 0.99, np.sort(d[nonchaotic])[-5:]
    assert np.mean(capped[nonchaotic] == ref["qp_capped"][nonchaotic]) >= 0.95
    assert np.mean(d <= 1e-6) >= np.mean(self_dev <= 1e-6) - 0.03, (np.mean(d <= 1e-6), np.mean(self_dev <= 1e-6))
    # the disagreement is the formulation's sensitivity, seen the same way by both implementations:
    # equal chaotic fractions (measured 10.8 % GPU, 10.9 % oracle), largely the same lanes (Jaccard
    # 0.81), and the GPU and oracle differ by more than 1e-6 almost only where at least one of them
    # moves under the probes (measured: 1 lane of 4 096 off while stable in both)
    gc, rc = gpu_dev > 1e-6, self_dev > 1e-6
    assert abs(gc.mean() - rc.mean()) < 0.02, (gc.mean(), rc.mean())
    assert (gc & rc).sum() / max((gc | rc).sum(), 1) > 0.7
    assert np.mean((d > 1e-6) & ~gc & ~rc) <= 0.001, np.nonzero((d > 1e-6) & ~gc & ~rc)[0][:10]
