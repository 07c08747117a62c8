"""Developer diagnostic: the lane with the largest bound violation of u0 on the bench workload."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import SHAPES, make_inputs  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402
from uclv_qs_pushing_matlab_amd.objects import make_shape  # noqa: E402
from uclv_qs_pushing_matlab_amd.solver import OcpSolver  # noqa: E402

N, B = 20, 65536
x0, yref, yref_e, sid, traj = make_inputs(B, N, 20250303 + 3)
s = OcpSolver(N=N, batch=B, sqp_iters=50)
s.set_shapes([make_shape(n) for n in SHAPES], shape_id=sid)
s.set_reference_trajectory(traj)
u = s.controller_solve(x0, 1)
st, qi = s.get("status"), s.get("qp_iter")
U = s.get("u")
s.close()
viol = np.maximum.reduce([-u[:, 0], u[:, 0] - 0.03, np.abs(u[:, 1]) - 0.05])
i = int(np.argmax(viol))
print("lane", i, "viol", viol[i], "u0", u[i], "status", st[i], "qp_iter", qi[i], "x0", x0[i], "sid", sid[i])
print("U(shifted) first stages", U[i, :4])
orc = Oracle(SHAPES)
for K in (10, 20, 30, 40, 45, 48, 49, 50):
    r = orc.controller_solve(make_opts(N=N, sqp_iters=K), x0[i:i + 1], traj, 1, orc.new_warm(1, N), shape_id=sid[i:i + 1])
    s1 = OcpSolver(N=N, batch=1, sqp_iters=K)
    s1.set_shapes([make_shape(n) for n in SHAPES], shape_id=sid[i:i + 1])
    s1.set_reference_trajectory(traj)
    ug = s1.controller_solve(x0[i:i + 1], 1)
    print(K, "oracle", r["u0"][0], r["status"][0], r["qp_iter"][0], "gpu", ug[0], s1.get("status")[0], s1.get("qp_iter")[0])
    s1.close()
