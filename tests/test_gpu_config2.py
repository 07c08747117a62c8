"""BASELINE configs[2]'s exact workload against the oracle: bench.py's input law (seed, x0
ranges of main.m:53-56, shape_id = lane mod 4 over santal/balea/montana/pulirapid), N = 20,
K = 50 SQP-RTI iterations, cold-start NMPC_controller.solve, the full B = 65 536 batch on the
GPU (two stream parts, per-iteration launches: the bench's code path); the first lanes are
checked against the oracle.

Parity is asserted on the lanes the oracle itself can reproduce: lanes whose oracle u0 moves
by > 1e-9 under 1e-13 relative perturbations of x0, or when the IPM stop test mu_stop moves
from 1e-10 to 1.5e-10, are chaotic (the full-step SQP amplifies rounding there, and the QPs'
central-path bias in the flat u_t direction depends on where the IPM stops; measured
independent of the QP stop rule).  On all lanes together the GPU must
agree with the oracle about as often as the perturbed oracle agrees with itself."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NAMES = ("santal", "balea", "montana", "pulirapid")


def test_config2_exact_law_parity(oracle):
    import torch
    from bench import make_inputs
    from oracle.oracle import make_opts
    from uclv_qs_pushing_matlab_amd._lib import DeviceIO
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    B, N, K, nl = 65536, 20, 50, 768
    x0, yref, yref_e, sid, traj = make_inputs(B, N, 20250303 + 3)
    s = OcpSolver(N=N, batch=B, sqp_iters=K)
    s.set_shapes([make_shape(n) for n in NAMES])
    assert s.stream_parts() == 2
    dev = torch.device("cuda", 0)
    t = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731
    bufs = dict(x0=t(x0), yref=t(yref), yref_e=t(yref_e), X_in=torch.zeros((B, N + 1, 4), dtype=torch.float64, device=dev),
                U_in=torch.zeros((B, N, 2), dtype=torch.float64, device=dev), shape_id=t(sid, torch.int32),
                u0=torch.empty((B, 2), dtype=torch.float64, device=dev),
                X_out=torch.empty((B, N + 1, 4), dtype=torch.float64, device=dev),
                U_out=torch.empty((B, N, 2), dtype=torch.float64, device=dev),
                PI_out=torch.empty((B, N, 4), dtype=torch.float64, device=dev),
                status=torch.empty((B,), dtype=torch.int32, device=dev), cost=torch.empty((B,), dtype=torch.float64, device=dev))
    io = DeviceIO()
    for k, v in bufs.items():
        setattr(io, k, v.data_ptr())
    io.controller = 1
    io.warm_valid = None
    s.solve_device(io)
    s.synchronize()
    u0 = bufs["u0"].cpu().numpy()
    status = bufs["status"].cpu().numpy()
    capped = s.get("qp_capped")
    s.close()
    assert np.all(status == 0)
    assert capped.sum() < 0.01 * B * K          # QPs stopped by the cap (qp_iters 20) are rare
    # the device-resident path (qsp_solve_device, the bench's) against the kernel-order twin: every
    # lane bit for bit
    from oracle.oracle import Oracle
    tw = Oracle(NAMES, twin=True)
    rt = tw.controller_solve(make_opts(N=N, sqp_iters=K), x0, traj, 1, tw.new_warm(B, N), shape_id=sid)
    np.testing.assert_array_equal(u0, rt["u0"])
    np.testing.assert_array_equal(status, rt["status"])
    np.testing.assert_array_equal(capped, rt["qp_capped"])

    def run(xx, **kw):
        return oracle.controller_solve(make_opts(N=N, sqp_iters=K, **kw), xx, traj, 1, oracle.new_warm(len(xx), N),
                                       shape_id=sid[:nl])
    ref = run(x0[:nl])
    assert np.all(ref["status"] == 0)
    self_dev = np.zeros(nl)
    for f in (1e-13, -1e-13, 3e-13):
        self_dev = np.maximum(self_dev, np.abs(run(x0[:nl] * (1 + f))["u0"] - ref["u0"]).max(1))
    mu_dev = np.abs(run(x0[:nl], mu_stop=1.5e-10)["u0"] - ref["u0"]).max(1)
    nonchaotic = (self_dev < 1e-9) & (mu_dev < 1e-9)
    d = np.abs(u0[:nl] - ref["u0"]).max(1)
    assert nonchaotic.mean() > 0.7, nonchaotic.mean()
    # the GPU's model evaluations differ from the oracle's by ~1e-12 relative (span-based de Boor +
    # hand-derived Jacobian vs full basis sum + forward AD), more than the 1e-13 probes: a few
    # probe-stable lanes still take another path (3 of 1 024 measured)
    assert np.mean(d[nonchaotic] < 1e-6) >= 0.99, np.sort(d[nonchaotic])[-5:]
    # the same QPs stop at the iteration cap (the chaotic lanes' iterates differ, and with them
    # their QPs)
    assert np.mean(capped[:nl][nonchaotic] == ref["qp_capped"][nonchaotic]) >= 0.95
    # everywhere: the GPU agrees with the oracle as often as the perturbed oracle with itself
    assert np.mean(d <= 1e-6) >= np.mean(self_dev <= 1e-6) - 0.03, (np.mean(d <= 1e-6), np.mean(self_dev <= 1e-6))
