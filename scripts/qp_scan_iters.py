"""Developer check (GPU box): the first IPM iteration at which the S = 2 factorisation scan's QP (qsp_qp_solve,
factor_scan) parts from the twin's, per instance (tests/test_gpu_twin.py test_qp_bit_identical data)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import config2_x0, straight_traj  # noqa: E402
from qp_data import build_qp  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402
from uclv_qs_pushing_matlab_amd.objects import make_shape  # noqa: E402
from uclv_qs_pushing_matlab_amd.solver import OcpSolver  # noqa: E402

NAMES = ("santal", "balea", "montana", "pulirapid")
twin = Oracle(NAMES, twin=True)
N, S, nb = 20, 2, 192
rng = np.random.default_rng(5 + N + S)
x0 = config2_x0(nb, 17 + N)
X = np.repeat(x0[:, None], N + 1, 1) + rng.normal(0, 2e-3, (nb, N + 1, 4))
U = np.stack([rng.uniform(0, 0.03, (nb, N)), rng.uniform(-0.02, 0.02, (nb, N))], 2)
yref = np.broadcast_to(straight_traj()[None, :N], (nb, N, 6)).copy()
A, B, b, H, g, lo, hi, act, dx0 = build_qp(twin, make_opts(N=N, stages_per_lane=S), X, U, yref, yref[:, -1, :4], x0,
                                           np.arange(nb) % 4)
first = np.full(nb, -1)
for q in range(1, 12):
    s = OcpSolver(N=N, batch=nb, stages_per_lane=S, factor_scan=True, qp_iters=q)
    s.set_shapes([make_shape(n) for n in NAMES])
    r = s.qp_solve(A.reshape(nb, N, 16), B.reshape(nb, N, 8), b, H, g, lo, hi, dx0)
    s.close()
    t = twin.qp(make_opts(N=N, stages_per_lane=S, factor_scan=1, qp_iters=q), A.reshape(nb, N, 16), B.reshape(nb, N, 8),
                b, H, g, lo, hi, act, dx0)
    d = (r["dx"] != t["dx"]).any(axis=(1, 2)) | (r["du"] != t["du"]).any(axis=(1, 2)) | (r["lam"] != t["lam"]).any(axis=(1, 2))
    first[(first < 0) & d] = q
    print(f"qp_iters {q}: instances differing {np.flatnonzero(d).tolist()}", flush=True)
print("first differing iteration per instance:", {int(i): int(first[i]) for i in np.flatnonzero(first >= 0)})
