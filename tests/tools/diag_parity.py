"""Developer diagnostic: per-shape GPU-vs-oracle u0 parity for cold-start controller solves."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import SHAPES, config2_x0, straight_traj  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402
from uclv_qs_pushing_matlab_amd.objects import make_shape  # noqa: E402
from uclv_qs_pushing_matlab_amd.solver import OcpSolver  # noqa: E402

N, K, nb = 20, int(sys.argv[1]) if len(sys.argv) > 1 else 50, 256
orc = Oracle(SHAPES)
traj = straight_traj()
for sid, name in enumerate(SHAPES):
    x0 = config2_x0(nb, 5 + sid)
    s = OcpSolver(N=N, batch=nb, sqp_iters=K)
    s.set_shapes([make_shape(n) for n in SHAPES], shape_id=sid)
    s.set_reference_trajectory(traj)
    u_gpu = s.controller_solve(x0, 1)
    X_gpu = s.get("x") if False else None
    op = make_opts(N=N, sqp_iters=K)
    r = orc.controller_solve(op, x0, traj, 1, orc.new_warm(nb, N), shape_id=sid)
    rp = orc.controller_solve(op, x0 * (1 + 1e-13), traj, 1, orc.new_warm(nb, N), shape_id=sid)
    d = np.abs(u_gpu - r["u0"]).max(1)
    stable = np.abs(rp["u0"] - r["u0"]).max(1) < 1e-9
    print(f"{name:10s} K={K} max err {d.max():.2e}  stable {stable.sum()}/{nb}  max err stable {d[stable].max():.2e}  "
          f"#err>1e-6: {(d > 1e-6).sum()}  #stable&err>1e-6: {(stable & (d > 1e-6)).sum()}")
    bad = np.where(stable & (d > 1e-6))[0][:3]
    for i in bad:
        print("   lane", i, "x0", x0[i], "gpu", u_gpu[i], "orc", r["u0"][i])
    s.close()
