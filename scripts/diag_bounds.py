"""Diagnostic (GPU): lanes of the bench workload whose u0 leaves a bound (QPs stopped by the
IPM iteration cap on chaotic lanes), at K = 50 and K = 49 SQP iterations."""
import sys, numpy as np
sys.path.insert(0, '.')
from bench import make_inputs, SHAPES
from uclv_qs_pushing_matlab_amd.objects import make_shape
from uclv_qs_pushing_matlab_amd.solver import OcpSolver
B, N = 65536, 20
x0, yref, yref_e, sid, traj = make_inputs(B, N, 20250303 + 3)
for K in (50, 49):
    s = OcpSolver(N=N, batch=B, sqp_iters=K)
    s.set_shapes([make_shape(n) for n in SHAPES])
    s.set_reference_trajectory(traj); s.set_shape_ids(sid)
    u1 = s.controller_solve(x0, 1)
    qi = s.get("qp_iter")
    viol = np.maximum.reduce([-u1[:, 0], u1[:, 0] - 0.03, np.abs(u1[:, 1]) - 0.05])
    print("K", K, "viol>1e-9:", int(np.sum(viol > 1e-9)), "max", viol.max(), "mean qp iters", qi.mean() / K)
    s.close()
