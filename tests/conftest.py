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
