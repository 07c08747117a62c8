"""Developer measurement: single-call latency of NMPC_controller.solve at small batch."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import SHAPES, make_inputs  # noqa: E402
from uclv_qs_pushing_matlab_amd.objects import make_shape  # noqa: E402
from uclv_qs_pushing_matlab_amd.solver import OcpSolver  # noqa: E402

N = 20
for B in (1, 64, 1024, 8192):
    x0, yref, yref_e, sid, traj = make_inputs(B, N, 7)
    s = OcpSolver(N=N, batch=B, sqp_iters=50)
    s.set_shapes([make_shape(n) for n in SHAPES], shape_id=sid)
    s.set_reference_trajectory(traj)
    for _ in range(3):
        s.controller_reset()
        s.controller_solve(x0, 1)
    ts = []
    for _ in range(20):
        s.controller_reset()
        t0 = time.perf_counter()
        s.controller_solve(x0, 1)
        ts.append(time.perf_counter() - t0)
    print(f"B={B:6d}  wall median {np.median(ts) * 1e3:7.3f} ms  device {s.get('time_tot') * 1e3:7.3f} ms  "
          f"-> {B / np.median(ts):10.0f} solves/s", flush=True)
    s.close()
