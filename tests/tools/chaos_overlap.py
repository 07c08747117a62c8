"""Developer tool (GPU + oracle): configs[1] lanes (B = 4 096, K = 50).  Compares the GPU's own
sensitivity to 1e-13 relative x0 perturbations with the oracle's: the fraction of lanes whose u0
moves by more than 1e-6 in each, and their overlap.  Prints one JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import config1_inputs  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402
from uclv_qs_pushing_matlab_amd.objects import make_shape  # noqa: E402
from uclv_qs_pushing_matlab_amd.solver import OcpSolver  # noqa: E402

N, K = 20, 50
x0, traj, sid = config1_inputs(N)
B = len(x0)
s = OcpSolver(N=N, batch=B, sqp_iters=K)
s.set_shapes([make_shape("santal")], shape_id=sid)
s.set_reference_trajectory(traj)


def gpu(x):
    s.controller_reset()
    return s.controller_solve(x, 1).copy()


o = Oracle()


def orc(x):
    return o.controller_solve(make_opts(N=N, sqp_iters=K), x, traj, 1, o.new_warm(B, N), shape_id=sid)["u0"]


g0, r0 = gpu(x0), orc(x0)
gd, rd = np.zeros(B), np.zeros(B)
for f in (1e-13, -1e-13, 3e-13):
    gd = np.maximum(gd, np.abs(gpu(x0 * (1 + f)) - g0).max(1))
    rd = np.maximum(rd, np.abs(orc(x0 * (1 + f)) - r0).max(1))
s.close()
gc, rc = gd > 1e-6, rd > 1e-6
d = np.abs(g0 - r0).max(1)
out = {"lanes": B, "gpu_chaotic_frac": float(gc.mean()), "oracle_chaotic_frac": float(rc.mean()),
       "both": float((gc & rc).mean()), "jaccard": float((gc & rc).sum() / max((gc | rc).sum(), 1)),
       "gpu_vs_oracle_off_1e-6": float((d > 1e-6).mean()),
       "off_and_chaotic_in_either": float(((d > 1e-6) & (gc | rc)).mean()),
       "off_and_stable_in_both": float(((d > 1e-6) & ~(gc | rc)).mean())}
print(json.dumps(out))
