"""Developer diagnostic: per-K trace of one lane for both layouts vs the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import SHAPES, make_inputs  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402
from uclv_qs_pushing_matlab_amd.objects import make_shape  # noqa: E402
from uclv_qs_pushing_matlab_amd.solver import OcpSolver  # noqa: E402

N = 20
lane = int(sys.argv[1]) if len(sys.argv) > 1 else 207
x0, yref, yref_e, sid, traj = make_inputs(65536, N, 20250303 + 3)
x0, sid = x0[lane:lane + 1], sid[lane:lane + 1]
orc = Oracle(SHAPES)
for K in range(18, 51):
    row = []
    res = {}
    for S in (1, 2):
        s = OcpSolver(N=N, batch=1, sqp_iters=K, stages_per_lane=S)
        s.set_shapes([make_shape(n) for n in SHAPES], shape_id=sid)
        s.set_reference_trajectory(traj)
        s.controller_solve(x0, 1)
        res[S] = (s.get("u"), int(s.get("qp_iter")[0]))
        s.close()
    w = orc.new_warm(1, N)
    r = orc.controller_solve(make_opts(N=N, sqp_iters=K), x0, traj, 1, w, shape_id=sid)
    Uo = w["U"].reshape(res[1][0].shape)   # shifted, as the GPU's get('u') in controller mode
    msg = f"K={K:2d} qp_iter S1 {res[1][1]} S2 {res[2][1]} orc {int(r['qp_iter'][0])}"
    if Uo is not None:
        msg += f"  |U1-Uo| {np.abs(res[1][0] - Uo).max():.2e} |U2-Uo| {np.abs(res[2][0] - Uo).max():.2e}"
    msg += f"  |U1-U2| {np.abs(res[1][0] - res[2][0]).max():.2e}  u0 S1 {res[1][0].reshape(-1)[0]:.3e} orc {r['u0'][0, 0]:.3e}"
    print(msg, flush=True)
