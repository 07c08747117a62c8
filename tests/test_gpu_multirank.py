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


def test_rccl_branch_world1_matches_single_process(tmp_path):
    """The nccl (RCCL) branch of bench.py as the 8-GPU node runs it — process group on the nccl
    backend, barriers and the MAX all_reduce on device tensors, gather_lanes on device u0/status —
    executed on the box's one GPU at world size 1 (RCCL refuses two ranks on one device), started by
    torch.distributed.run.  The gathered u0/status must equal a plain single-process run bit for bit."""
    import json
    import socket
    total = 6144
    common = ["--global-batch", str(total), "--steps", "1", "--warmup", "0", "--no-cpu", "--no-configs1",
              "--no-configs4", "--no-closed-loop"]
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, QSP_DIST_FORCE="1", MASTER_ADDR="127.0.0.1")
    env.pop("QSP_DIST_BACKEND", None)
    env.pop("WORLD_SIZE", None)
    rc = tmp_path / "rccl.npz"
    one = tmp_path / "one.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--dump-u0", str(rc)] + common
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["gather_ms"] is not None   # the gather ran (over RCCL)
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dump-u0", str(one)] + common,
                        cwd=ROOT, env=dict(os.environ), capture_output=True, text=True, timeout=200)
    assert r1.returncode == 0, r1.stderr[-3000:]
    assert json.loads([ln for ln in r1.stdout.splitlines() if ln.startswith("{")][-1])["gather_ms"] is None
    a, b = np.load(rc), np.load(one)
    np.testing.assert_array_equal(a["u0"], b["u0"])
    np.testing.assert_array_equal(a["status"], b["status"])
