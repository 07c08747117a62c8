"""Developer check (GPU box): scripts/ubench/velem_check.hip's device element arithmetic against the
twin's tw_velem_check on the same cases, bit for bit; prints the first differing case and field."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.oracle import lib  # noqa: E402

rng = np.random.default_rng(1)
n = 20000
c = np.zeros((n, 68))
for o in (0, 30):
    c[:, o:o + 6] = rng.normal(0, 0.05, (n, 6)); c[:, o + 5] += 1.0
    c[:, o + 6:o + 14] = rng.normal(0, 0.05, (n, 8))
    c[:, o + 14:o + 18] = rng.normal(0, 1e-3, (n, 4))
    c[:, o + 18:o + 22] = np.array([0.05, 0.05, 5e-5, 0.0]) + 10 ** rng.uniform(-12, 14, (n, 4)) * (rng.random((n, 4)) < 0.5)
    c[:, o + 22:o + 24] = 5e-5 + 10 ** rng.uniform(-12, 14, (n, 2)) * (rng.random((n, 2)) < 0.5)
    c[:, o + 24:o + 28] = rng.normal(0, 1e-2, (n, 4))
    c[:, o + 28:o + 30] = rng.normal(0, 1e-4, (n, 2))
c[:, 60:64] = [2e5, 2e5, 20.0, 0.0]
c[n // 2:, 60] = -1.0   # second half: general element (x) general element
for o in (0, 30):       # near-converged interior points: barrier terms from 1e-20 to 1e30
    m = rng.random((n, 4)) < 0.3
    c[:, o + 18:o + 22] += np.where(m, 10 ** rng.uniform(-20, 30, (n, 4)), 0.0)
    m = rng.random((n, 2)) < 0.3
    c[:, o + 22:o + 24] += np.where(m, 10 ** rng.uniform(-20, 30, (n, 2)), 0.0)
    c[:, o + 24:o + 30] *= np.where(rng.random((n, 6)) < 0.3, 10 ** rng.uniform(-5, 15, (n, 6)), 1.0)
c[:, 64:68] = rng.normal(0, 1e2, (n, 4))
inp, outp = "/tmp/velem_in.bin", "/tmp/velem_out.bin"
c.tofile(inp)
exe = os.path.join(ROOT, "scripts", "ubench", "velem_check")
subprocess.check_call([exe, inp, outp])
g = np.fromfile(outp).reshape(n, 88)
t = np.zeros((n, 88))
lib().tw_velem_check(C.c_int32(n), c.ctypes.data_as(C.c_void_p), t.ctypes.data_as(C.c_void_p))
names = [f"A{q}" for q in range(16)] + [f"b{q}" for q in range(4)] + [f"C{q}" for q in range(10)] + \
        [f"eta{q}" for q in range(4)] + [f"J{q}" for q in range(10)]
bad = np.argwhere(g != t)
print(f"cases {n}: differing entries {len(bad)}, cases {len(np.unique(bad[:, 0])) if len(bad) else 0}")
for i, q in bad[:12]:
    print(f"  case {i} {'1st' if q < 44 else '2nd'} combine {names[q % 44]}: gpu {g[i, q]!r} twin {t[i, q]!r}")

# the same on realistic cases: consecutive stage pairs of the OCP's Gauss-Newton QPs (tests/test_gpu_twin.py
# test_qp_bit_identical's data) with the interior point's first barrier terms (mu0 / t^2 on every bound)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import config2_x0, straight_traj  # noqa: E402
from qp_data import build_qp  # noqa: E402
from oracle.oracle import Oracle, make_opts  # noqa: E402
tw = Oracle(("santal", "balea", "montana", "pulirapid"), twin=True)
N, nb = 20, 192
rng = np.random.default_rng(5 + N + 2)
x0 = config2_x0(nb, 17 + N)
X = np.repeat(x0[:, None], N + 1, 1) + rng.normal(0, 2e-3, (nb, N + 1, 4))
U = np.stack([rng.uniform(0, 0.03, (nb, N)), rng.uniform(-0.02, 0.02, (nb, N))], 2)
yref = np.broadcast_to(straight_traj()[None, :N], (nb, N, 6)).copy()
A, B, b, H, g, lo, hi, act, dx0 = build_qp(tw, make_opts(N=N, stages_per_lane=2), X, U, yref, yref[:, -1, :4], x0,
                                           np.arange(nb) % 4)
tl, th = np.maximum(-lo, 1e-2), np.maximum(hi, 1e-2)
hb = 1.0 / tl ** 2 + 1.0 / th ** 2
gb = -1.0 / tl + 1.0 / th
cases = []
for i in range(nb):
    for k in range(N - 1):
        row = []
        for kk in (k, k + 1):
            Ak = A[i, kk]
            a6 = [Ak[0, 2], Ak[0, 3], Ak[1, 2], Ak[1, 3], Ak[2, 3], Ak[3, 3]]
            Hx = list(H[i, 6 * kk:6 * kk + 3]) + [H[i, 6 * kk + 3] + hb[i, kk, 0]]
            Hu = [H[i, 6 * kk + 4] + hb[i, kk, 1], H[i, 6 * kk + 5] + hb[i, kk, 2]]
            gx = list(g[i, 6 * kk:6 * kk + 3]) + [g[i, 6 * kk + 3] + gb[i, kk, 0]]
            gu = [g[i, 6 * kk + 4] + gb[i, kk, 1], g[i, 6 * kk + 5] + gb[i, kk, 2]]
            row += a6 + list(B[i, kk].reshape(8)) + list(b[i, kk]) + Hx + Hu + gx + gu
        row += list(H[i, 6 * N:]) + list(g[i, 6 * N:])
        cases.append(row)
c = np.array(cases)
n = len(c)
c.tofile(inp)
subprocess.check_call([exe, inp, outp])
g2 = np.fromfile(outp).reshape(n, 88)
t2 = np.zeros((n, 88))
lib().tw_velem_check(C.c_int32(n), c.ctypes.data_as(C.c_void_p), t2.ctypes.data_as(C.c_void_p))
bad = np.argwhere(g2 != t2)
print(f"QP cases {n}: differing entries {len(bad)}, cases {len(np.unique(bad[:, 0])) if len(bad) else 0}")
for i, q in bad[:12]:
    print(f"  case {i} {'1st' if q < 44 else '2nd'} combine {names[q % 44]}: gpu {g2[i, q]!r} twin {t2[i, q]!r}")
