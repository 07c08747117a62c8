"""Developer tool: solve BASELINE configs[2] on the GPU (bench's input law, two stream parts)
and save u0, status, qp_iter, qp_capped of every lane to gpurun_out/config2_gpu.npz, for
offline comparison with the oracle on the CPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from bench import SEED, SHAPES, make_inputs
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    B, N, K = 65536, 20, 50
    x0, yref, yref_e, sid, traj = make_inputs(B, N, SEED)
    s = OcpSolver(N=N, batch=B, sqp_iters=K)
    s.set_shapes([make_shape(n) for n in SHAPES], shape_id=sid)
    s.set_reference_trajectory(traj)
    u0 = s.controller_solve(x0, 1)
    out = dict(u0=u0, status=s.get("status"), qp_iter=s.get("qp_iter"), qp_capped=s.get("qp_capped"),
               parts=s.stream_parts())
    s.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "config2_gpu.npz"), **out)
    print("saved", {k: (v.shape if hasattr(v, "shape") else v) for k, v in out.items()})


if __name__ == "__main__":
    main()
