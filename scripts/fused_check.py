"""Developer tool: fused SQP loop vs per-iteration launches on configs[1]-like lanes with the
library QSP_LIB_PATH points at; prints how many lanes differ (bit identity expected)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def solve(fused, B):
    os.environ["QSP_FUSED_LOOP"] = fused
    from bench import config1_inputs
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    x, traj, sid = config1_inputs(20, B)
    s = OcpSolver(N=20, batch=B, sqp_iters=50)
    s.set_shapes([make_shape("santal")], shape_id=sid)
    s.set_reference_trajectory(traj)
    u = s.controller_solve(x, 1)
    st, qi = s.get("status"), s.get("qp_iter")
    s.close()
    return u, st, qi


B = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
u0, s0, q0 = solve("0", B)
u1, s1, q1 = solve("1", B)
d = np.abs(u0 - u1).max(1)
bad = np.nonzero(d > 0)[0]
print(os.environ.get("QSP_LIB_PATH", "in-tree"), "lanes differing:", len(bad), "first:", bad[:10],
      "status0/1 nonzero:", int((s0 != 0).sum()), int((s1 != 0).sum()),
      "qp_iter differing:", int((q0 != q1).sum()))
