"""CPU, world_size 2 (and 3) over gloo: the multi-GPU layout of bench.py -- its input law per
shard (bench.make_inputs), its shard split and its u0/status gather
(uclv_qs_pushing_matlab_amd.sharding.shard_range / gather_lanes), the max-over-ranks timing --
reproduces the single-process result.  The per-shard solve here is the CPU oracle (no GPU in
this container); tests/test_gpu_multirank.py runs the same path on the HIP library."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from bench import config2_x0, shard_range, straight_traj


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bench import make_inputs
    from oracle.oracle import Oracle, make_opts
    from uclv_qs_pushing_matlab_amd.sharding import gather_lanes
    lo, hi = shard_range(total, world, rank)
    x0, _, _, sid, traj = make_inputs(total, 10, 123, lo, hi)
    orc = Oracle()
    r = orc.controller_solve(make_opts(N=10, sqp_iters=2), x0, traj, 1, orc.new_warm(hi - lo, 10),
                             shape_id=sid, nthreads=1)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    u0 = gather_lanes(torch.as_tensor(r["u0"]), total, dist, world, rank)
    st = gather_lanes(torch.as_tensor(r["status"]), total, dist, world, rank)
    if rank == 0:
        out.put((float(t), u0.numpy(), st.numpy()))
    dist.destroy_process_group()


def test_shard_range_covers_all_lanes():
    for total in (1, 7, 64, 65536 * 8 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world,total", [(2, 24), (3, 25)])
def test_multi_rank_gloo_matches_single_process(world, total):
    from bench import make_inputs
    from oracle.oracle import Oracle, make_opts
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    tmax, u0, st = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == float(world)                          # max over ranks
    orc = Oracle()
    x0, _, _, sid, traj = make_inputs(total, 10, 123)
    ref = orc.controller_solve(make_opts(N=10, sqp_iters=2), x0, traj, 1, orc.new_warm(total, 10),
                               shape_id=sid, nthreads=1)
    np.testing.assert_array_equal(u0, ref["u0"])           # shards unequal at total = 25: padded gather
    np.testing.assert_array_equal(st, ref["status"])


def test_make_inputs_shards_match_single_process():
    from bench import make_inputs
    full = make_inputs(1000, 20, 7)
    for world in (2, 3, 8):
        parts = [make_inputs(1000, 20, 7, *shard_range(1000, world, r)) for r in range(world)]
        for q in range(4):
            np.testing.assert_array_equal(np.concatenate([p[q] for p in parts]), full[q])


def test_bench_gpus_flag_launches_ranks_or_fails_loudly():
    """bench.py --gpus N (no WORLD_SIZE) starts its own N ranks; with fewer visible GPUs than N it
    refuses (exit 2) before touching a device -- here, in a container without GPUs."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "QSP_DIST_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("GPUs visible: the launch itself is tests/test_gpu_multirank.py's")
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) visible" in r.stderr


class _MockNccl:
    """Stands in for torch.distributed on the nccl (RCCL) backend for gather_lanes: checks what RCCL
    requires of an all_gather -- one output per rank, every tensor of the input's shape, dtype and
    device, the input not moved off its device -- and delivers the ranks' padded shards."""

    def __init__(self, world, pads=None):
        self.world, self.pads, self.seen = world, pads, []

    def all_gather(self, parts, pad):
        assert len(parts) == self.world
        for p in parts:
            assert p.shape == pad.shape and p.dtype == pad.dtype and p.device == pad.device
        self.seen.append((tuple(pad.shape), pad.dtype, pad.device))
        if self.pads is not None:
            for p, q in zip(parts, self.pads):
                p.copy_(q)


@pytest.mark.parametrize("world,total", [(8, 262144), (8, 262147), (2, 5)])
@pytest.mark.parametrize("dtype", ["float64", "int32"])
def test_gather_lanes_nccl_branch_shapes(world, total, dtype):
    """bench.py's gather on the nccl backend hands gather_lanes device tensors (d_u0 B x 2 FP64, d_st B
    int32, red_dev = the rank's GPU).  Without a GPU here: the same call on 'meta' tensors (device
    tensors that hold no data) must build padded buffers of the largest shard's shape, dtype and
    device -- so the first 8-GPU run cannot fail on this branch -- and, on CPU tensors with a mock
    collective, reassemble the global lane order exactly (unequal shards at 262 147 lanes)."""
    import torch
    from uclv_qs_pushing_matlab_amd.sharding import gather_lanes
    dt = getattr(torch, dtype)
    cap = max(h - l for l, h in (shard_range(total, world, r) for r in range(world)))
    tail = (2,) if dtype == "float64" else ()
    for rank in range(world):
        lo, hi = shard_range(total, world, rank)
        m = _MockNccl(world)
        out = gather_lanes(torch.empty((hi - lo,) + tail, dtype=dt, device="meta"), total, m, world, rank)
        assert m.seen == [((cap,) + tail, dt, torch.device("meta"))]
        assert out.shape == (total,) + tail and out.dtype == dt and out.device.type == "meta"
    full = torch.arange(total * (2 if tail else 1), dtype=dt).reshape((total,) + tail)
    pads = []
    for r in range(world):
        lo, hi = shard_range(total, world, r)
        p = torch.zeros((cap,) + tail, dtype=dt)
        p[: hi - lo] = full[lo:hi]
        pads.append(p)
    for rank in (0, world - 1):
        lo, hi = shard_range(total, world, rank)
        out = gather_lanes(full[lo:hi].clone(), total, _MockNccl(world, pads), world, rank)
        assert torch.equal(out, full)
    with pytest.raises(ValueError):
        gather_lanes(torch.empty((cap + 1,) + tail, dtype=dt), total, _MockNccl(world), world, 0)
