"""Which KKT residual keeps the merit SQP (nlp_mode 1: sqp + merit_backtracking, max_iter 30,
tol 1e-6, NMPC_controller.m:271-276) from converging?  Runs the twin and/or the literal oracle on
configs[2]-law lanes with the KKT diagnostics on (or_set_kkt_diag / tw_set_kkt_diag) and prints,
for the lanes ending with status 2, which residuals exceed their tolerance and by how much.
Test tooling (CPU only)."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import SEED, make_inputs  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402

NAMES = ("santal", "balea", "montana", "pulirapid")
FIELDS = ("stat_u", "stat_x", "stat_term", "eq", "ineq", "comp")


def run(impl, B, K, steps, qp_iters, tol, **kw):
    orc = Oracle(NAMES, twin=impl == "twin")
    x0, _, _, sid, traj = make_inputs(B, 20, SEED + 7)
    op = make_opts(N=20, sqp_iters=K, nlp_mode=1, qp_iters=qp_iters, tol=tol, **kw)
    warm = orc.new_warm(B, 20)
    diag = np.zeros((B, 22 if impl == 'literal' else 8))
    setter = getattr(orc.L, ("tw_" if impl == "twin" else "or_") + "set_kkt_diag")
    setter(diag.ctypes.data_as(C.c_void_p))
    out = []
    try:
        for step in range(steps):
            r = orc.controller_solve(op, x0, traj, 1 + step, warm, shape_id=sid)
            out.append((r, diag.copy()))
    finally:
        setter(None)   # process-global pointer: never leave it set past this buffer's lifetime
    return out, sid


def report(r, diag, sid, tol):
    st = r["status"]
    B = len(st)
    print(f"  status: " + ", ".join(f"{v}: {np.mean(st == v):.3f}" for v in np.unique(st)))
    m = st == 2
    if not m.any():
        return
    d = diag[m]
    fail = d[:, :6] >= tol
    print(f"  status-2 lanes: {m.sum()}  (per shape: {np.bincount(sid[m], minlength=4)})")
    for j, f in enumerate(FIELDS):
        v = d[:, j]
        print(f"    {f:9s} fails on {fail[:, j].mean():6.3f}  median {np.median(v):.2e}  p90 {np.quantile(v, .9):.2e}  max {v.max():.2e}")
    only = fail.sum(1) == 1
    for j, f in enumerate(FIELDS):
        print(f"    only {f:9s}: {np.mean(only & fail[:, j]):.3f}")
    print(f"    last line-search alpha: median {np.median(d[:, 7]):.3g}, frac alpha=1 {np.mean(d[:, 7] == 1.0):.3f}, "
          f"frac alpha<0.05 {np.mean(d[:, 7] < 0.05 + 1e-12):.3f}")
    if d.shape[1] > 8:
        print(f"    last line search: dphi < 0 on {np.mean(d[:, 8] < 0):.3f}; phi(last) > phi0 on {np.mean(d[:, 10] > d[:, 9]):.3f}; "
              f"line searches ending at alpha_min per lane: median {np.median(d[:, 11])}, mean {d[:, 11].mean():.1f}")
        print(f"    stages whose motion-cone mode changed at the last linearisation: lanes with any {np.mean(d[:, 16] > 0):.3f}; "
              f"mode changes from SQP iteration 10 on: median {np.median(d[:, 17])}, lanes with any {np.mean(d[:, 17] > 0):.3f}")
        up = d[:, 8] >= 0
        if up.any():
            print(f"    on the {up.sum()} lanes with dphi >= 0: last QP exit {np.unique(d[up, 12], return_counts=True)}; "
                  f"r_u'du median {np.median(d[up, 13]):.2e}, -d'Hd median {np.median(d[up, 14]):.2e}, pi'b - nu|b| median {np.median(d[up, 15]):.2e}, dphi median {np.median(d[up, 8]):.2e}")
    print(f"    qp capped per lane mean {r['qp_capped'][m].mean():.2f}, stalled {r['qp_stalled'][m].mean():.2f}")
    c = st == 0
    if c.any() and diag.shape[1] > 16:
        print(f"  status-0 lanes: mode changes from SQP iteration 10 on: lanes with any {np.mean(diag[c, 17] > 0):.3f}")
    if c.any():
        print(f"  status-0 lanes: sqp_iter median {np.median(r['iters'][c])}, max {r['iters'][c].max()}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", default="twin", choices=("twin", "literal"))
    ap.add_argument("--B", type=int, default=1024)
    ap.add_argument("--K", type=int, default=30)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--qp-iters", type=int, default=50)
    ap.add_argument("--tol", type=float, default=1e-6)
    a = ap.parse_args()
    outs, sid = run(a.impl, a.B, a.K, a.steps, a.qp_iters, a.tol)
    for s, (r, d) in enumerate(outs):
        print(f"{a.impl} step {s}:")
        report(r, d, sid, a.tol)


def closed_loop_breakdown(B=256, seed=None, qp_iters=50):
    """main.m's closed loop (bench.closed_loop_measure's workload) on the twin: per status-2 lane-step,
    which KKT residual failed (tw_set_kkt_diag accumulates them in tw_closed_loop)."""
    from bench import SEED as S0, SHAPES, config2_x0, straight_traj
    tw = Oracle(SHAPES, twin=True)
    x0 = config2_x0(B, S0 if seed is None else seed)
    sid = (np.arange(B) % len(SHAPES)).astype(np.int32)
    op = make_opts(N=10, sqp_iters=30, nlp_mode=1, qp_iters=qp_iters)
    diag = np.zeros((B, 8))
    tw.L.tw_set_kkt_diag(diag.ctypes.data_as(C.c_void_p))
    try:
        r = tw.closed_loop(op, x0, straight_traj(), 201, shape_id=sid, dist_step=300)
    finally:
        tw.L.tw_set_kkt_diag(None)
    n2 = diag[:, 4].sum()
    st = r["status"]
    return {"lane_steps": int(st.size), "status": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
            "status2_fail_frac": {f: float(diag[:, j].sum() / max(n2, 1)) for j, f in enumerate(("stat", "eq", "ineq", "comp"))},
            "status2_stat_only_frac": float(diag[:, 5].sum() / max(n2, 1)),
            "status2_stat_below_1e-3_frac": float(diag[:, 6].sum() / max(n2, 1))}
