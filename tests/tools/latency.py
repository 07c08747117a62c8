"""Developer measurement: single-call latency of NMPC_controller.solve at small batch."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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

# main.m's own controller: one instance, N = 10 (Hp), merit SQP, max_iter 30, tol 1e-6, warm
# started from the previous step (NMPC_controller.solve inside helper.closed_loop_matlab), against
# the oracle on one host thread for the same calls
from oracle.oracle import Oracle, make_opts  # noqa: E402

Nm = 10
x0, yref, yref_e, sid, traj = make_inputs(1, Nm, 7)
s = OcpSolver(N=Nm, batch=1, sqp_iters=30, nlp_solver_type="SQP")
s.set_shapes([make_shape("santal")], shape_id=np.zeros(1, np.int32))
s.set_reference_trajectory(traj)
orc = Oracle(("santal",))
warm = orc.new_warm(1, Nm)
op = make_opts(N=Nm, sqp_iters=30, nlp_mode=1)
tg, tc, its = [], [], []
x = x0.copy()
for step in range(60):
    t0 = time.perf_counter()
    u = s.controller_solve(x, step + 1)
    tg.append(time.perf_counter() - t0)
    its.append(int(s.get("sqp_iter")[0]))
    t0 = time.perf_counter()
    orc.controller_solve(op, x, traj, step + 1, warm, shape_id=np.zeros(1, np.int32), nthreads=1)
    tc.append(time.perf_counter() - t0)
    f, _ = s.eval_dynamics(x, u)
    x = x + 0.05 * f
s.close()
print(f"main.m controller (N=10, merit SQP, max_iter 30), one instance, 60 closed-loop steps: GPU call median "
      f"{np.median(tg[5:]) * 1e3:.3f} ms (max {np.max(tg[5:]) * 1e3:.3f}), oracle on one thread median "
      f"{np.median(tc[5:]) * 1e3:.3f} ms; SQP iterations per call median {np.median(its):.0f}", flush=True)
