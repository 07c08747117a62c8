"""Developer tool: configs[1] (B = 4 096) device time under QP-rule variants and input laws."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import SEED, SHAPES, config1_inputs, make_inputs
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    N, K, B = 20, 50, 4096
    x1, traj1, sid1 = config1_inputs(N)
    xm, _, _, sidm, trajm = make_inputs(B, N, SEED)
    for law, (x, sid, traj) in (("mixed", (xm, sidm, trajm)),):
        for kw, parts, fused in ((dict(qp_iters=20), 0, None), (dict(qp_iters=50), 0, None), (dict(qp_iters=50), 2, None),
                                 (dict(qp_iters=50), 1, "1"), (dict(qp_iters=20), 1, "1"), (dict(qp_iters=50), 2, "0")):
            if fused is None:
                os.environ.pop("QSP_FUSED_LOOP", None)
            else:
                os.environ["QSP_FUSED_LOOP"] = fused
            for Bq in (4096, 16384):
                xq = np.resize(x, (Bq, 4)); sq = np.resize(sid, Bq)
                s = OcpSolver(N=N, batch=Bq, sqp_iters=K, **kw)
                s.set_shapes([make_shape(n) for n in SHAPES], shape_id=sq)
                s.set_reference_trajectory(traj)
                s.set_stream_parts(parts)
                s.controller_solve(xq, 1)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    s.controller_reset()
                    s.controller_solve(xq, 1)
                dt = (time.perf_counter() - t0) / 5
                print(law, Bq, kw, "parts", parts, "fused", fused, f"{Bq / dt:.0f} solves/s", flush=True)
                s.close()


if __name__ == "__main__":
    main()
