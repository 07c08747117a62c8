"""Adjudicate the formulation disagreements with the extended-precision literal restatement.

On the first `n` lanes of the bench workload (BASELINE configs[2], or configs[4] with --config 4):
  * the kernel-order twin (= the GPU bit for bit) and the double literal restatement, each with its
    own response to three 1e-13 relative x0 probes (and the literal's mu_stop and model probes, as
    bench.parity_leg);
  * the literal restatement in __float128 ("quad", 113-bit significand) and long double on every lane
    where twin and literal differ by > 1e-6 -- the exact-arithmetic answer of the same formulas, as
    far as the SQP's amplification of rounding allows (quad and long double agreeing to 1e-6 says it
    does) -- and on a random control sample of the other lanes;
  * per disagreeing lane: does the extended-precision u0 side with the twin (the GPU) or with the
    double literal?
Writes the tally (and, with --fixture, tests/golden/ext_adjudication.json: the stable-in-both lanes
with their u0 from every implementation, which tests/test_extended_oracle.py re-checks).
Test tooling (CPU only)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import SEED, SHAPES, config4_inputs, make_inputs  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402

TOL = 1e-6


def inputs(config, n, seed=SEED):
    if config == 4:
        x0, _, _, sid, traj, idx = config4_inputs(16384, 50, seed)
        return x0[:n], sid[:n], traj, idx[:n], 50
    x0, _, _, sid, traj = make_inputs(65536, 20, seed)
    return x0[:n], sid[:n], traj, np.ones(n, np.int32), 20


def adjudicate(u_tw, u_lit, u_q, u_l):
    """Per lane: 'twin' when quad is within TOL of the twin only, 'literal' when of the literal only,
    'both', 'neither'; ext_stable when long double and quad agree within TOL."""
    dt = np.abs(u_tw - u_q).max(1)
    dl = np.abs(u_lit - u_q).max(1)
    side = np.where((dt <= TOL) & (dl > TOL), "twin", np.where((dl <= TOL) & (dt > TOL), "literal",
                    np.where((dt <= TOL) & (dl <= TOL), "both", "neither")))
    return side, dt, dl, np.abs(u_l - u_q).max(1) <= TOL


def tally(side, mask):
    return {k: int(np.sum(mask & (side == k))) for k in ("twin", "literal", "both", "neither")}


def run(config=2, n=5904, control=64, threads=0, K=50, qp_iters=20):
    x0, sid, traj, idx, N = inputs(config, n)
    orc, tw = Oracle(SHAPES), Oracle(SHAPES, twin=True)
    op = make_opts(N=N, sqp_iters=K, qp_iters=qp_iters)

    def solve(o, x, which, sl=slice(None), **kw):
        oo = make_opts(N=N, sqp_iters=K, qp_iters=qp_iters, **kw) if kw else op
        xs = x[sl]
        w = Oracle.new_warm(len(xs), N)
        if which == "quad" or which == "long":
            return orc.controller_solve_ext(oo, xs, traj, idx[sl], w, shape_id=sid[sl], nthreads=threads,
                                            precision=which)["u0"]
        return o.controller_solve(oo, xs, traj, idx[sl], w, shape_id=sid[sl], nthreads=threads)["u0"]

    t0 = time.time()
    u_tw, u_lit = solve(tw, x0, "d"), solve(orc, x0, "d")
    tw_dev, lit_dev = np.zeros(n), np.zeros(n)
    for sgn, f in ((1, 1.0), (-1, 1.0), (1, 3.0)):
        xp = x0 * (1 + sgn * f * 1e-13)
        tw_dev = np.maximum(tw_dev, np.abs(solve(tw, xp, "d") - u_tw).max(1))
        lit_dev = np.maximum(lit_dev, np.abs(solve(orc, xp, "d") - u_lit).max(1))
    mod_dev = np.abs(solve(orc, x0, "d", mu_stop=1.5e-10) - u_lit).max(1)
    for seed in (1, 2):
        mod_dev = np.maximum(mod_dev, np.abs(solve(orc, x0, "d", model_probe=1e-14, probe_seed=seed) - u_lit).max(1))
    d = np.abs(u_tw - u_lit).max(1)
    dis = np.flatnonzero(d > TOL)
    stable_both = (tw_dev <= TOL) & (lit_dev <= TOL)
    stable_all = stable_both & (mod_dev <= TOL)
    lit_stable = (lit_dev <= TOL) & (mod_dev <= TOL)   # the literal moves under none of its probes
    rng = np.random.default_rng(1)
    agree = np.flatnonzero(d <= TOL)
    ctrl = np.sort(rng.choice(agree, min(control, len(agree)), replace=False))
    t1 = time.time()
    lanes = np.concatenate([dis, ctrl])
    u_q = solve(None, x0, "quad", lanes)
    u_l = solve(None, x0, "long", lanes)
    t2 = time.time()
    side, dt, dl, ext_ok = adjudicate(u_tw[lanes], u_lit[lanes], u_q, u_l)
    m_dis = np.arange(len(lanes)) < len(dis)
    sb = stable_both[lanes]
    sa = stable_all[lanes]
    out = {"config": config, "lanes": int(n), "N": N, "K": K,
           "disagreeing_lanes": int(len(dis)),
           "disagreeing_stable_in_both_lanes": int(np.sum(stable_both[dis])),
           "disagreeing_stable_under_all_probes_lanes": int(np.sum(stable_all[dis])),
           "ext_stable_frac_disagreeing": float(np.mean(ext_ok[m_dis])) if len(dis) else None,
           "all_disagreeing": tally(side, m_dis),
           "disagreeing_ext_stable": tally(side, m_dis & ext_ok),
           "disagreeing_stable_in_both": tally(side, m_dis & sb),
           "disagreeing_stable_under_all_probes": tally(side, m_dis & sa),
           "disagreeing_literal_stable_lanes": int(np.sum(lit_stable[dis])),
           "disagreeing_literal_stable": tally(side, m_dis & lit_stable[lanes]),
           "control_lanes": int(len(ctrl)),
           "control_twin_within_1e-6_of_quad": int(np.sum(dt[~m_dis] <= TOL)),
           "control_literal_within_1e-6_of_quad": int(np.sum(dl[~m_dis] <= TOL)),
           "seconds": {"double": t1 - t0, "extended": t2 - t1}}
    fix = [{"lane": int(lanes[j]), "u0_twin": u_tw[lanes[j]].tolist(), "u0_literal": u_lit[lanes[j]].tolist(),
            "u0_quad": u_q[j].tolist(), "u0_long": u_l[j].tolist(), "side": str(side[j]),
            "stable_under_all_probes": bool(sa[j]), "twin_stable": bool(tw_dev[lanes[j]] <= TOL),
            "literal_stable": bool(lit_stable[lanes[j]])}
           for j in range(len(dis)) if sb[j] or lit_stable[lanes[j]]]
    return out, fix


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n", type=int, default=5904)
    ap.add_argument("--control", type=int, default=64)
    ap.add_argument("--fixture", action="store_true")
    a = ap.parse_args()
    out, fix = run(a.config, a.n, a.control)
    print(json.dumps(out, indent=1))
    if a.fixture:
        path = os.path.join(ROOT, "tests", "golden", f"ext_adjudication_c{a.config}.json")
        with open(path, "w") as f:
            json.dump({"generator": "tests/tools/ext_adjudicate.py", "config": a.config, "lanes_scanned": a.n,
                       "summary": out, "lanes": fix}, f, indent=1)
        print("wrote", path)
