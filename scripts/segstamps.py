"""Wave-time breakdown of the QP kernel by segment (developer tool; GPU; the diagnostic build):
    bash scripts/mkvariant.sh seg -DQSP_SEGSTAMP
    QSP_LIB_PATH=$PWD/variants/seg.so python scripts/segstamps.py [--N 20 --batch 65536]
Runs the bench workload's cold-start solve twice and prints, from the second, the wave cycles (s_memtime,
summed over waves by lane 0) spent in each segment of qp_step_kernel, per IPM iteration of a wave and as
a share of the kernel's wave time.  The stamps cost ~10 % of the wave time; the shares are what counts."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {0: "iteration head (mu, stop tests, ballot)", 1: "barrier_terms", 2: "factorisation walk",
         3: "predictor forward walk", 4: "affine directions, step, mu_aff", 5: "corrector_terms",
         6: "corrector difference walk", 7: "corrector forward walk", 8: "corrector directions, step, update",
         10: "kernel head: linearisation, loads", 11: "qp_ipm total", 12: "rollout, adjoint, stores",
         13: "qp_ipm start point", 14: "head: permutation and iterate loads", 15: "head: RK4 + sensitivities"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import numpy as np
    from bench import SEED, SHAPES, make_inputs
    from uclv_qs_pushing_matlab_amd import _lib
    from uclv_qs_pushing_matlab_amd.objects import make_shape
    from uclv_qs_pushing_matlab_amd.solver import OcpSolver
    L = _lib.lib()
    stamped = hasattr(L, "qsp_debug_segments")
    if stamped:
        L.qsp_debug_segments.argtypes = [C.c_void_p, C.c_int]
    x0, _, _, sid, traj = make_inputs(args.batch, args.N, SEED)
    s = OcpSolver(N=args.N, batch=args.batch)
    s.set_shapes([make_shape(n) for n in SHAPES])
    s.set_shape_ids(sid)
    s.set_reference_trajectory(traj)
    seg = np.zeros(32, np.uint64)
    s.controller_solve(x0, 1)
    s.synchronize()
    assert not stamped or L.qsp_debug_segments(seg.ctypes.data, 1) == 0
    s.controller_reset()
    import time
    t0 = time.perf_counter()
    s.controller_solve(x0, 1)
    s.synchronize()
    wall = time.perf_counter() - t0
    s.close()
    if not stamped:
        print(f"solve wall {wall * 1e3:.1f} ms (library without stamps)")
        return
    assert L.qsp_debug_segments(seg.ctypes.data, 1) == 0
    seg = seg.astype(np.float64)
    iters = seg[31]
    kern = seg[10] + seg[11] + seg[12] + seg[14] + seg[15]
    out = {"workload": f"N={args.N} batch={args.batch}", "wall_s": wall, "wave_ipm_iterations": iters,
           "kernel_wave_cycles": kern, "segments": {}}
    print(f"solve wall {wall * 1e3:.1f} ms; wave IPM iterations {iters:.0f}; kernel wave cycles {kern:.3e} "
          f"({kern / iters:.0f} per wave IPM iteration)")
    for i, nm in NAMES.items():
        if seg[i] == 0:
            continue
        out["segments"][nm] = {"cycles": seg[i], "per_wave_iteration": seg[i] / iters, "share_of_kernel": seg[i] / kern}
        print(f"  {i:2d} {nm:40s} {seg[i] / iters:9.0f} cycles/iter  {100 * seg[i] / kern:5.1f} %")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
