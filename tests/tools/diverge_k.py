"""Developer tool: u0, IPM iterations and capped-QP counts of chosen bench lanes after K = 1..K_max
SQP-RTI iterations (cold start each), from the library (GPU) or the oracle (--oracle), so the
first iteration at which two implementations part can be found.

  python tests/tools/diverge_k.py out.npz 479,651,2342 [--kmax 50] [--oracle]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("lanes")
ap.add_argument("--kmax", type=int, default=50)
ap.add_argument("--oracle", action="store_true")
a = ap.parse_args()
from bench import SEED, SHAPES, make_inputs  # noqa: E402

lanes = np.array([int(v) for v in a.lanes.split(",")])
B, N = 65536, 20
x0, _, _, sid, traj = make_inputs(B, N, SEED)
x, s = x0[lanes], sid[lanes]
U, QI, CAP, X = [], [], [], []
for K in range(1, a.kmax + 1):
    if a.oracle:
        from oracle.oracle import Oracle, make_opts
        o = Oracle()
        w = o.new_warm(len(lanes), N)
        r = o.controller_solve(make_opts(N=N, sqp_iters=K), x, traj, 1, w, shape_id=s)
        U.append(r["u0"]); QI.append(r["qp_iter"]); CAP.append(r["qp_capped"]); X.append(w["X"].reshape(len(lanes), -1))
    else:
        from uclv_qs_pushing_matlab_amd.objects import make_shape
        from uclv_qs_pushing_matlab_amd.solver import OcpSolver
        so = OcpSolver(N=N, batch=len(lanes), sqp_iters=K)
        so.set_shapes([make_shape(n) for n in SHAPES], shape_id=s)
        so.set_reference_trajectory(traj)
        U.append(so.controller_solve(x, 1)); QI.append(so.get("qp_iter")); CAP.append(so.get("qp_capped"))
        X.append(so.get("x").reshape(len(lanes), -1))
        so.close()
np.savez(a.out, lanes=lanes, u0=np.array(U), qp_iter=np.array(QI), qp_capped=np.array(CAP), X=np.array(X))
print("wrote", a.out)
