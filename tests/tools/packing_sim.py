"""Developer tool (uses the oracle twin, test infrastructure): wave-packing predictors simulated on
the per-QP IPM iteration counts of bench lanes.

The fixed-K SQP's first k iterations do not depend on K, so the IPM count of QP k of a lane is
qp_iter(K = k) - qp_iter(K = k - 1) of the kernel-order twin (the device's counts bit for bit).
A QP launch costs, per wave, the largest count among the wave's G instances; the instances are
sorted by a key computed from their last four counts (longest first), as sort_by_iters_kernel
does.  Reported: sum over waves and SQP iterations of the wave maximum, over the mean count x
#waves (1.0 = no packing loss).

    python tests/tools/packing_sim.py [lanes] [K]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from bench import SHAPES, make_inputs  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402


def counts(nb, K, N=20, seed=20250303 + 3):
    x0, _, _, sid, traj = make_inputs(nb, N, seed)
    orc = Oracle(list(SHAPES), twin=True)
    tot = np.zeros((K + 1, nb), np.int64)
    for k in range(1, K + 1):
        r = orc.controller_solve(make_opts(N=N, sqp_iters=k), x0, traj, 1, orc.new_warm(nb, N), shape_id=sid)
        tot[k] = r["qp_iter"]
    return np.diff(tot, axis=0)           # (K, nb): IPM count of QP k


def simulate(c, key, G=3):
    K, nb = c.shape
    hist = np.zeros((4, nb), np.int64)   # c1 (last) .. c4
    cost = 0
    for k in range(K):
        order = np.arange(nb) if k == 0 else np.lexsort(tuple(-np.asarray(x) for x in key(hist)[::-1]))
        w = c[k][order]
        pad = (-nb) % G
        w = np.concatenate([w, np.zeros(pad, w.dtype)]).reshape(-1, G)
        cost += w.max(1).sum()
        hist = np.vstack([c[k][None], hist[:3]])
    return cost / (c.sum() / G)


def kd(h):   # the kernel's key: period-2 prediction, ties by c2
    c1, c2, c3, c4 = h
    p = np.where((c4 != 0) & (c2 == c4), c2, c1)
    return (p, c2)


PREDICTORS = {
    "unsorted": None,
    "c1": lambda h: (h[0],),
    "c1,c2": lambda h: (h[0], h[1]),
    "kernel (p2 pred, c2)": kd,
    "p2 pred, c1": lambda h: (kd(h)[0], h[0]),
    "max(c1,c2), c2": lambda h: (np.maximum(h[0], h[1]), h[1]),
    "c2 if c2==c4 or c1==c3, c1": lambda h: (np.where(((h[3] != 0) & (h[1] == h[3])) | ((h[2] != 0) & (h[0] == h[2])),
                                                      h[1], h[0]), h[0]),
    "c1+c2": lambda h: (h[0] + h[1], h[1]),
    "2c2+c1 if p2 else 2c1+c2": lambda h: (np.where((h[3] != 0) & (h[1] == h[3]), 2 * h[1] + h[0], 2 * h[0] + h[1]),),
}


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    c = counts(nb, K)
    print(f"{nb} bench lanes, K = {K}, mean IPM count {c.mean():.3f}")
    for name, key in PREDICTORS.items():
        if key is None:
            r = simulate(c, lambda h: (np.zeros(h.shape[1]),))
        else:
            r = simulate(c, key)
        print(f"{name:32s} {r:.4f}")
    # perfect foresight
    K_, _ = c.shape
    cost = 0
    for k in range(K_):
        w = np.sort(c[k])[::-1]
        pad = (-len(w)) % 3
        cost += np.concatenate([w, np.zeros(pad, w.dtype)]).reshape(-1, 3).max(1).sum()
    print(f"{'perfect foresight':32s} {cost / (c.sum() / 3):.4f}")


if __name__ == "__main__":
    main()


def table_study(c):
    """Keys from the conditional mean of the next count given a history tuple, learned on the even
    lanes and evaluated on the odd ones (upper bound on what a lookup-table predictor buys)."""
    K, nb = c.shape
    tr, te = c[:, 0::2], c[:, 1::2]

    def hists(x):
        out = []
        h = np.zeros((4, x.shape[1]), np.int64)
        for k in range(K):
            out.append(h.copy())
            h = np.vstack([x[k][None], h[:3]])
        return out
    for depth in (1, 2, 3, 4):
        tab = {}
        for k, h in enumerate(hists(tr)):
            for i in range(tr.shape[1]):
                t = tuple(h[:depth, i])
                s = tab.setdefault(t, [0, 0])
                s[0] += tr[k, i]
                s[1] += 1

        def key(h, depth=depth):
            m = np.array([(lambda s: s[0] / s[1] if s else -1.0)(tab.get(tuple(h[:depth, i]))) for i in range(h.shape[1])])
            # unseen histories: fall back to the kernel's prediction
            return (np.where(m < 0, kd(h)[0], m), h[1])
        print(f"table E[next | c1..c{depth}] ({len(tab)} entries): {simulate(te, key):.4f}  (kernel key on the same lanes {simulate(te, kd):.4f})")


if __name__ == "__main__" and os.environ.get("TABLES"):
    table_study(counts(int(sys.argv[1]) if len(sys.argv) > 1 else 3072, 50))
