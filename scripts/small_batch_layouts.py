"""Small-batch throughput by lane layout and loop form (developer tool, GPU).

For configs[1]-like batches (santal, config-2 x0 law, straight reference, N = 20, K = 50) times
host-boundary controller solves at each batch size for stages per lane S = 1, 2 and the SQP loop
as per-iteration launches (QSP_FUSED_LOOP=0) or the fused loop (QSP_FUSED_LOOP=1), and checks
that every variant returns the same u0 bits as the S = 1 per-iteration form (lanes are
independent of layout only up to the layout's summation order: S = 2 sums a group's terms in
another order, so its u0 is compared by max |diff| instead).

  python scripts/small_batch_layouts.py [--batches 1024,2048,4096] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(B, S, fused, reps, N=20, K=50):
    os.environ["QSP_FUSED_LOOP"] = fused
    from bench import config1_inputs
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    x, traj, sid = config1_inputs(N, B)
    s = OcpSolver(N=N, batch=B, sqp_iters=K, stages_per_lane=S)
    s.set_shapes([make_shape("santal")], shape_id=sid)
    s.set_reference_trajectory(traj)
    s.controller_solve(x, 1)
    s.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        s.controller_reset()
        u = s.controller_solve(x, 1)
    s.synchronize()
    dt = (time.perf_counter() - t) / reps
    lay = s.layout()
    s.close()
    return B / dt, dt, u, lay


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1024,2048,3072,4096,6144,8192")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--stages", default="1,2")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for B in [int(b) for b in a.batches.split(",")]:
        base = None
        for S in [int(v) for v in a.stages.split(",")]:
            for fused in ("0", "1"):
                rate, dt, u, lay = run(B, S, fused, a.reps)
                if base is None:
                    base = u
                d = float(np.abs(u - base).max())
                row = {"B": B, "S": S, "fused": fused, "layout": list(lay), "solves_per_s": round(rate),
                       "ms": round(dt * 1e3, 2), "max_abs_u0_diff_vs_S1_unfused": d}
                rows.append(row)
                print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
