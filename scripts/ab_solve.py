"""Developer tool: one controller solve of bench lanes with the library QSP_LIB_PATH points at,
dumped to an .npz (compare two builds: python scripts/ab_solve.py out.npz [B] [K])."""
import sys

import numpy as np

sys.path.insert(0, ".")
from bench import make_inputs, SHAPES  # noqa: E402
from uclv_qs_pushing_matlab_amd.objects import make_shape  # noqa: E402
from uclv_qs_pushing_matlab_amd.solver import OcpSolver  # noqa: E402

out = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 6
K = int(sys.argv[3]) if len(sys.argv) > 3 else 1
x0, yref, yref_e, sid, traj = make_inputs(B, 20, 20250303 + 3)
s = OcpSolver(N=20, batch=B, sqp_iters=K)
s.set_shapes([make_shape(n) for n in SHAPES])
s.set_reference_trajectory(traj)
s.set_shape_ids(sid)
u = s.controller_solve(x0, 1)
np.savez(out, u0=u, status=s.get("status"), qp_iter=s.get("qp_iter"), x=s.get("x"), u=s.get("u"))
print(out, "status", s.get("status")[:8], "qp_iter", s.get("qp_iter")[:8], "u0", u[:3])
s.close()
