"""Developer diagnostic: find bench lanes that are oracle-stable but disagree on the GPU,
then trace them over K for both kernel layouts."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import SHAPES, make_inputs  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402
from uclv_qs_pushing_matlab_amd.objects import make_shape  # noqa: E402
from uclv_qs_pushing_matlab_amd.solver import OcpSolver  # noqa: E402

N, m = 20, 512
x0, yref, yref_e, sid, traj = make_inputs(65536, N, 20250303 + 3)
x0, sid = x0[:m], sid[:m]
orc = Oracle(SHAPES)


def gpu(x, ids, K, S):
    s = OcpSolver(N=N, batch=len(x), sqp_iters=K, stages_per_lane=S)
    s.set_shapes([make_shape(n) for n in SHAPES], shape_id=ids)
    s.set_reference_trajectory(traj)
    u = s.controller_solve(x, 1)
    it = s.get("qp_iter")
    s.close()
    return u, it


def orac(x, ids, K):
    r = orc.controller_solve(make_opts(N=N, sqp_iters=K), x, traj, 1, orc.new_warm(len(x), N), shape_id=ids)
    return r["u0"], r["qp_iter"]


u_o, _ = orac(x0, sid, 50)
stable = np.ones(m, bool)
for f in (1e-13, -1e-13, 3e-13):
    stable &= np.abs(orac(x0 * (1 + f), sid, 50)[0] - u_o).max(1) < 1e-9
for S in (1, 2):
    u_g, _ = gpu(x0, sid, 50, S)
    d = np.abs(u_g - u_o).max(1)
    bad = np.where(stable & (d > 1e-6))[0]
    print(f"S={S}: stable {stable.sum()}  max err stable {d[stable].max():.3e}  bad lanes {bad.tolist()}")
    for i in bad[:2]:
        print(f"  lane {i} shape {sid[i]} x0 {x0[i]}")
        for K in (1, 2, 3, 5, 8, 12, 20, 30, 40, 50):
            ug, ig = gpu(x0[i:i + 1], sid[i:i + 1], K, S)
            uo, io = orac(x0[i:i + 1], sid[i:i + 1], K)
            print(f"    K={K:2d} |du0|={np.abs(ug - uo).max():.3e} qp_iter gpu {int(ig[0])} orc {int(io[0])}  u_gpu {ug[0]} u_orc {uo[0]}")
