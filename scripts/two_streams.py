"""Developer experiment: does splitting the bench batch over several HIP streams (one solver
handle each) overlap the launch tails of the per-SQP-iteration QP kernels?

    python scripts/two_streams.py [--parts 1 2 4] [--steps 5]

Prints solves/s of the bench workload for each split (same lanes, same K)."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--parts", type=int, nargs="+", default=[1, 2, 4, 1])
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from uclv_qs_pushing_matlab_amd._lib import DeviceIO
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver

    B, N, K = args.batch, args.N, args.K
    dev = torch.device("cuda", 0)
    x0, yref, yref_e, sid, _ = bench.make_inputs(B, N, 20250303 + 3, 0, B)
    t = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731

    def part(lo, hi):
        n = hi - lo
        s = OcpSolver(N=N, batch=n, sqp_iters=K, device=0)
        s.set_shapes([make_shape(nm) for nm in bench.SHAPES])
        keep = dict(x0=t(x0[lo:hi]), yref=t(yref[lo:hi]), yref_e=t(yref_e[lo:hi]), shape_id=t(sid[lo:hi], torch.int32),
                    X_in=torch.zeros((n, N + 1, 4), dtype=torch.float64, device=dev),
                    U_in=torch.zeros((n, N, 2), dtype=torch.float64, device=dev),
                    u0=torch.empty((n, 2), dtype=torch.float64, device=dev),
                    X_out=torch.empty((n, N + 1, 4), dtype=torch.float64, device=dev),
                    U_out=torch.empty((n, N, 2), dtype=torch.float64, device=dev),
                    PI_out=torch.empty((n, N, 4), dtype=torch.float64, device=dev),
                    status=torch.empty((n,), dtype=torch.int32, device=dev),
                    cost=torch.empty((n,), dtype=torch.float64, device=dev))
        io = DeviceIO()
        for k, v in keep.items():
            setattr(io, k, v.data_ptr())
        io.controller = 1
        io.warm_valid = None
        return s, io, keep, torch.cuda.Stream(dev)

    for P in args.parts:
        edges = [B * i // P for i in range(P + 1)]
        parts = [part(edges[i], edges[i + 1]) for i in range(P)]
        for s, io, _, st in parts:
            s.solve_device(io, st.cuda_stream)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            for s, io, _, st in parts:
                s.solve_device(io, st.cuda_stream)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        u0 = torch.cat([p[2]["u0"] for p in parts]).cpu().numpy()
        print(f"parts {P}: {B * args.steps / dt:,.0f} solves/s  ({dt / args.steps * 1e3:.2f} ms per batch)  "
              f"u0 checksum {np.abs(u0).sum():.12e}", flush=True)
        for s, *_ in parts:
            s.close()


if __name__ == "__main__":
    main()
