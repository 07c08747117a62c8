"""Developer tool: mean IPM iterations per QP, capped/failed QPs and u0 movement under changes of the
interior-point parameters (oracle, first 1 024 bench lanes, K = 50).  Run: python tests/tools/ipm_param_study.py"""
import sys, time, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from bench import make_inputs, SEED
from oracle.oracle import Oracle, make_opts
o = Oracle()
B, N, K = 65536, 20, 50
n = 1024
x0, _, _, sid, traj = make_inputs(B, N, SEED)
x, s = x0[:n], sid[:n]
def run(**kw):
    r = o.controller_solve(make_opts(N=N, sqp_iters=K, **kw), x, traj, 1, o.new_warm(n, N), shape_id=s)
    return r["qp_iter"].mean() / K, r["qp_capped"].sum() / (n * K), (r["status"] != 0).sum(), r["u0"]
base = run()
print("base", base[:3])
for kw in [dict(mu0=10.0), dict(mu0=0.1), dict(mu0=100.0), dict(sigma_min=1e-3), dict(sigma_min=0.1), dict(frac=0.999), dict(frac=0.99), dict(t_min=1e-1), dict(t_min=1e-3)]:
    t = time.time(); r = run(**kw)
    print(kw, "ipm/qp %.3f capped %.4f failed %d  u0 moved>1e-6: %.3f" % (r[0], r[1], r[2], np.mean(np.abs(r[3] - base[3]).max(1) > 1e-6)), round(time.time() - t, 1))
