"""Oracle study (CPU): does a stricter, HPIPM-style QP termination remove the full-step
SQP's sensitive ('chaotic') lanes on the bench workload?  VERDICT r01 item 1.

For each QP stop rule the oracle solves the bench sample (BASELINE configs[2] law, cold
start, K = 50 SQP-RTI iterations) and reports
  - chaotic: fraction of lanes whose u0 moves > 1e-6 under three 1e-13 relative
    perturbations of x0 (the oracle against itself);
  - unconverged: fraction whose u0 moves > 1e-9 between K-1 and K iterations;
  - capped: fraction of QPs stopped by the iteration cap; mean IPM iterations per QP.
Usage: python tests/tools/qp_termination_study.py [lanes] [threads]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import SHAPES, make_inputs  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402

RULES = {
    "r01 (mu, bound res < 1e-10; cap 20)": dict(qp_iters=20),
    "r01 rule, cap 50": dict(qp_iters=50),
    "HPIPM-acados (stat 1e-6, eq/ineq/comp 1e-8; cap 50)": dict(qp_iters=50, qp_tol_stat=1e-6, qp_tol_eq=1e-8,
                                                                res_stop=1e-8, mu_stop=1e-8),
    "all four 1e-10, cap 50": dict(qp_iters=50, qp_tol_stat=1e-10, qp_tol_eq=1e-10),
    "all four 1e-12, cap 50": dict(qp_iters=50, qp_tol_stat=1e-12, qp_tol_eq=1e-12, res_stop=1e-12, mu_stop=1e-12),
}


def study(nl, threads, N=20, K=50, seed=20250303 + 3):
    x0, _, _, sid, traj = make_inputs(65536, N, seed, 0, nl)
    orc = Oracle(SHAPES)
    out = {}
    for name, kw in RULES.items():
        def run(xx, K_run=K):
            op = make_opts(N=N, sqp_iters=K_run, **kw)
            return orc.controller_solve(op, xx, traj, 1, orc.new_warm(len(xx), N), shape_id=sid, nthreads=threads)
        t0 = time.perf_counter()
        r = run(x0)
        dt = time.perf_counter() - t0
        dev = np.zeros(nl)
        for sgn, f in ((1, 1.0), (-1, 1.0), (1, 3.0)):
            dev = np.maximum(dev, np.abs(run(x0 * (1 + sgn * f * 1e-13))["u0"] - r["u0"]).max(1))
        dk = np.abs(run(x0, K - 1)["u0"] - r["u0"]).max(1)
        out[name] = dict(chaotic=float(np.mean(dev > 1e-6)), sensitive_1e9=float(np.mean(dev > 1e-9)),
                         unconverged=float(np.mean(dk > 1e-9)),
                         chaotic_or_unconverged=float(np.mean((dev > 1e-6) | (dk > 1e-9))),
                         capped_qp_frac=float(r["qp_capped"].sum() / (nl * K)),
                         ipm_iters_per_qp=float(r["qp_iter"].sum() / (nl * K)),
                         status_nonzero=int(np.count_nonzero(r["status"])), seconds=dt)
        print(name, json.dumps(out[name]), flush=True)
    return out


if __name__ == "__main__":
    nl = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    th = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 1)
    res = study(nl, th)
    print(json.dumps({"lanes": nl, "rules": res}))
