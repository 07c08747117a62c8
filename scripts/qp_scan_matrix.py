import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from conftest import config2_x0, straight_traj
from qp_data import build_qp
from oracle.oracle import Oracle, make_opts
from uclv_qs_pushing_matlab_amd.objects import make_shape
from uclv_qs_pushing_matlab_amd.solver import OcpSolver
NAMES = ("santal", "balea", "montana", "pulirapid")
twin = Oracle(NAMES, twin=True)
for N in (20, 50):
    S = 2
    rng = np.random.default_rng(5 + N + S)
    nb = 192
    x0 = config2_x0(nb, 17 + N)
    X = np.repeat(x0[:, None], N + 1, 1) + rng.normal(0, 2e-3, (nb, N + 1, 4))
    U = np.stack([rng.uniform(0, 0.03, (nb, N)), rng.uniform(-0.02, 0.02, (nb, N))], 2)
    traj = straight_traj()
    yref = np.broadcast_to(traj[None, :N], (nb, N, 6)).copy()
    sid = np.arange(nb) % 4
    A, B, b, H, g, lo, hi, act, dx0 = build_qp(twin, make_opts(N=N, stages_per_lane=S), X, U, yref, yref[:, -1, :4], x0, sid)
    G, T = {}, {}
    for fs in (0, 1):
        s = OcpSolver(N=N, batch=nb, stages_per_lane=S, factor_scan=bool(fs))
        s.set_shapes([make_shape(n) for n in NAMES])
        G[fs] = s.qp_solve(A.reshape(nb, N, 16), B.reshape(nb, N, 8), b, H, g, lo, hi, dx0)
        s.close()
        T[fs] = twin.qp(make_opts(N=N, stages_per_lane=S, factor_scan=fs), A.reshape(nb, N, 16), B.reshape(nb, N, 8), b, H, g, lo, hi, act, dx0)
    for gf in (0, 1):
        for tf in (0, 1):
            print(N, "gpu scan", gf, "twin scan", tf, "dx differing", int(np.sum(G[gf]["dx"] != T[tf]["dx"])), "iters differ", int(np.sum(G[gf]["iters"] != T[tf]["iters"])))
    d = (G[1]["dx"] != T[1]["dx"]).any(axis=(1, 2)) | (G[1]["du"] != T[1]["du"]).any(axis=(1, 2))
    L = (N + 2) // 2
    Gw = 64 // L
    lanes = np.flatnonzero(d)
    print(N, "differing instances", lanes.tolist(), "group in wave", (lanes % Gw).tolist(),
          "iters", G[1]["iters"][lanes].tolist(), "max |ddx|", float(np.abs(G[1]["dx"] - T[1]["dx"]).max()))
    for i in lanes[:3]:
        ks = np.flatnonzero((G[1]["dx"][i] != T[1]["dx"][i]).any(1))
        print("   instance", i, "stages with dx differing", ks.tolist())
