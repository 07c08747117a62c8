"""The multi-GPU path of bench.py on the HIP library, started as the driver's 8-GPU run would be
started by hand: `python bench.py --gpus 2` launches its own two ranks (one process each; here
both on device 0 of the one-GPU box, QSP_DIST_BACKEND=gloo for the exchange); they each solve their
contiguous shard of a global batch, then all-gather u0/status with bench's gather_lanes; the
gathered u0 must equal a single-process solve of the whole batch bit for bit (instances are
independent).  On the 8-GPU node the same code runs with the nccl (RCCL) backend."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_bench_gather_matches_single_process(tmp_path):
    total = 6144
    common = ["--global-batch", str(total), "--steps", "1", "--warmup", "0", "--no-cpu", "--no-configs1"]
    env = dict(os.environ, QSP_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    two = tmp_path / "two.npz"
    one = tmp_path / "one.npz"
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dump-u0", str(two)] + common
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    import json
    rec = json.loads(line)
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == total and rec["gather_ms"] is not None
    assert "configs[3]" in rec["config"]["workload"]
    assert len([ln for ln in r.stdout.splitlines() if ln.startswith("{")]) == 1   # rank 0 only
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dump-u0", str(one)] + common,
                        cwd=ROOT, env=dict(os.environ), capture_output=True, text=True, timeout=200)
    assert r1.returncode == 0, r1.stderr[-3000:]
    a, b = np.load(two), np.load(one)
    assert a["u0"].shape == (total, 2)
    np.testing.assert_array_equal(a["u0"], b["u0"])
    np.testing.assert_array_equal(a["status"], b["status"])
