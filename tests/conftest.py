import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Oracle
    return Oracle()


def config2_x0(nb, seed):
    """BASELINE config 2 initial-state law (main.m:53-56 ranges)."""
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(-0.0065, 0.0260, nb), rng.uniform(-0.0197, 0.0124, nb),
                     np.deg2rad(rng.uniform(-8.05, 9.30, nb)), rng.uniform(-0.0382, 0.0011, nb)], 1)


def straight_traj(T_end=10.0, Ts=0.05, v=0.01):
    """Config-1 reference: x_ref(t) = [v t, 0, 0, 0 | 0, 0], t = 0:Ts:T_end (main.m:150-175)."""
    t = np.arange(0.0, T_end + 1e-9, Ts)
    traj = np.zeros((len(t), 6))
    traj[:, 0] = v * t
    return traj


def decagon_table(max_ctrl=64):
    """Control polygon of acados_nmpc/test_bspline_class.m:22-25 (unit circle at
    theta = 0:pi/5:2*pi, 11 points, first = last) with the knot rule of :29-33 /
    PusherSliderModel.m:113-132; c and mu are placeholders (spline tests only)."""
    from oracle.shapes_np import knots_for
    th = np.arange(0.0, 2 * np.pi + 1e-12, np.pi / 5)
    P = np.stack([np.cos(th), np.sin(th)], 1)
    S, b = knots_for(P)
    n = len(P)
    ctrl = np.zeros((1, max_ctrl, 2))
    ctrl[0, :n] = P
    knots = np.zeros((1, max_ctrl + 4))
    knots[0, :n + 4] = S
    return dict(n_ctrl=np.array([n], np.int32), ctrl=ctrl, knots=knots, params=np.array([[b, 0.03, 0.2]]),
                max_ctrl=max_ctrl, names=["decagon"]), P, S, b
