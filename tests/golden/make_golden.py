"""Generates the committed fixtures in tests/golden/ from the CPU oracle.

Inputs come from the reference's own data files (cad_models/*.ply copied to
uclv_qs_pushing_matlab_amd/data/, acados_nmpc/x_finals.mat -> data/x_finals.npz) and
from the constants of acados_nmpc/main.m / NMPC_controller.m.  The outputs are the
oracle's (acados itself cannot run here: parity against acados is unpinned, see
DESIGN.md §2).  Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import config2_x0, straight_traj  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402
from oracle.shapes_np import load_object  # noqa: E402

NAMES = ("santal", "balea", "montana", "pulirapid")


def main():
    # 1. shape tables (PusherSliderModel.m:84-132)
    shapes = {}
    for n in NAMES:
        o = load_object(n)
        shapes[n] = dict(n=len(o["P"]), P=o["P"].tolist(), S=o["S"].tolist(), b=o["b"], c=o["c"], mu=o["mu"])
    with open(os.path.join(HERE, "shapes.json"), "w") as f:
        json.dump(shapes, f, indent=1)

    orc = Oracle(NAMES)
    rng = np.random.default_rng(20250303)
    # 2. model points: f, J, RK4 + sensitivities, spline, v_bound
    n = 256
    sid = rng.integers(0, 4, n).astype(np.int32)
    b = orc.tab["params"][sid, 0]
    x = np.stack([rng.uniform(-0.05, 0.05, n), rng.uniform(-0.05, 0.05, n), rng.uniform(-np.pi, np.pi, n),
                  rng.uniform(-1.2, 1.2, n) * b], 1)
    u = np.stack([rng.uniform(0, 0.03, n), rng.uniform(-0.05, 0.05, n)], 1)
    u[:8] = 0.0
    u[8:16, 0] = 0.0
    f, J = orc.dynamics(x, u, sid)
    xn, A, B = orc.rk4(x, u, 0.05, sid)
    sg = rng.uniform(0, 1, n) * b
    C, dC, D, dD, kap = orc.spline(sg, sid)
    vb = orc.vbound(x[:, 3], make_opts(), sid)
    np.savez_compressed(os.path.join(HERE, "model_points.npz"), sid=sid, x=x, u=u, f=f, J=J, xn=xn, A=A, B=B,
                        sigma=sg, C=C, D=D, dD=dD, kappa=kap, vbound=vb)

    # 3. config 1 (santal, x0 = 0, straight reference): closed loop of NMPC_controller.solve,
    #    reference horizon Hp = 10 and BASELINE N = 20, K = 5 SQP-RTI iterations per call
    traj = straight_traj()
    out = {}
    for N in (10, 20):
        op = make_opts(N=N, sqp_iters=5)
        warm = orc.new_warm(1, N)
        xs = np.zeros((1, 4))
        us, costs = [], []
        for i in range(1, 21):
            r = orc.controller_solve(op, xs, traj, i, warm)
            us.append(r["u0"][0].tolist())
            costs.append(float(r["cost"][0]))
            fx, _ = orc.dynamics(xs, r["u0"])
            xs = xs + 0.05 * fx                       # plant: helper.m:292-307 (Euler, same f)
        out[f"N{N}"] = dict(u0=us, cost=costs, x_final=xs[0].tolist())
    with open(os.path.join(HERE, "config1_closed_loop.json"), "w") as f:
        json.dump(out, f, indent=1)

    # 4. config-2 mini batch (64 lanes, K = 50), with the oracle's own stability mask
    nb, N = 64, 20
    x0 = config2_x0(nb, 20250303 + 2)
    op = make_opts(N=N, sqp_iters=50)
    base = orc.controller_solve(op, x0, traj, 1, orc.new_warm(nb, N))
    stable = np.ones(nb, bool)
    for pert in (lambda v: v * (1 + 1e-13), lambda v: v * (1 - 1e-13), lambda v: v + 1e-15):
        r = orc.controller_solve(op, pert(x0), traj, 1, orc.new_warm(nb, N))
        stable &= np.abs(r["u0"] - base["u0"]).max(1) < 1e-9
    np.savez_compressed(os.path.join(HERE, "config2_batch64.npz"), x0=x0, u0=base["u0"], cost=base["cost"],
                        qp_iter=base["qp_iter"], stable=stable)

    # 5. BASELINE configs[0] exactly: santal, N = 20, one SQP-RTI iteration per control step,
    #    the full 10 s straight-line run (201 steps, helper.m:195-322 with x0 = 0)
    N, T = 20, 201
    op = make_opts(N=N, sqp_iters=1)
    warm = orc.new_warm(1, N)
    xs = np.zeros((1, 4))
    U, X = [], [xs[0].copy()]
    for i in range(1, T + 1):
        r = orc.controller_solve(op, xs, traj, i, warm)
        fx, _ = orc.dynamics(xs, r["u0"])
        xs = xs + 0.05 * fx
        U.append(r["u0"][0].copy())
        X.append(xs[0].copy())
    np.savez_compressed(os.path.join(HERE, "config1_rti_full.npz"), U=np.array(U), X=np.array(X))

    # 6. main.m as the reference runs it: santal, Hp = 10 (main.m:41), the 'sqp' +
    #    'merit_backtracking' options of create_ocp_opts (max_iter 30, tol 1e-6), 201 steps
    N = 10
    op = make_opts(N=N, sqp_iters=30, nlp_mode=1)
    warm = orc.new_warm(1, N)
    xs = np.zeros((1, 4))
    U, X, ST, IT = [], [xs[0].copy()], [], []
    for i in range(1, T + 1):
        r = orc.controller_solve(op, xs, traj, i, warm)
        fx, _ = orc.dynamics(xs, r["u0"])
        xs = xs + 0.05 * fx
        U.append(r["u0"][0].copy())
        X.append(xs[0].copy())
        ST.append(int(r["status"][0]))
        IT.append(int(r["iters"][0]))
    np.savez_compressed(os.path.join(HERE, "main_m_sqp_closed_loop.npz"), U=np.array(U), X=np.array(X),
                        status=np.array(ST, np.int32), iters=np.array(IT, np.int32))
    print("golden fixtures written to", HERE, "stable lanes:", int(stable.sum()), "/", nb)


if __name__ == "__main__":
    main()
