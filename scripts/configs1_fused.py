"""configs[1] (B = 4 096 santal lanes, N = 20, K = 50) with the whole SQP loop in one launch against the
per-iteration launches (developer tool; GPU).  Run once per library build:
    QSP_LIB_PATH=... python scripts/configs1_fused.py --tag NAME [--fused 0|1] [--u0 out.npy]
prints solves/s of host-boundary controller solves (bench.py's configs1 leg) and, with --u0, saves u0 so
builds can be compared bit for bit."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--fused", default=None, choices=(None, "0", "1"))
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--u0", default=None)
    args = ap.parse_args()
    if args.fused is not None:
        os.environ["QSP_FUSED_LOOP"] = args.fused
    import torch
    from bench import config1_inputs
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    x1, traj1, sid1 = config1_inputs(20)
    s = OcpSolver(N=20, batch=len(x1), sqp_iters=50)
    s.set_shapes([make_shape("santal")], shape_id=sid1)
    s.set_reference_trajectory(traj1)
    s.controller_solve(x1, 1)
    s.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        s.controller_reset()
        u = s.controller_solve(x1, 1)
    dt = (time.perf_counter() - t0) / args.reps
    print(f"{args.tag} fused={args.fused} walk={s.factor_walk()} B={len(x1)}: {len(x1) / dt:.0f} solves/s "
          f"({dt * 1e3:.2f} ms per solve)", flush=True)
    s.close()
    if args.u0:
        np.save(args.u0, u)


if __name__ == "__main__":
    main()
