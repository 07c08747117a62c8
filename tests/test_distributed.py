"""CPU, world_size 2 over gloo: the multi-GPU layout of bench.py (independent lane
shards, max-over-ranks timing, optional gather of u0) reproduces the single-process
result.  The per-shard solve here is the CPU oracle (no GPU in this container)."""
import os
import socket

import numpy as np
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
    from oracle.oracle import Oracle, make_opts
    lo, hi = shard_range(total, world, rank)
    x0 = config2_x0(total, 123)[lo:hi]
    orc = Oracle()
    r = orc.controller_solve(make_opts(N=10, sqp_iters=2), x0, straight_traj(), 1, orc.new_warm(hi - lo, 10),
                             shape_id=np.arange(lo, hi) % 4, nthreads=1)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    parts = [None] * world
    dist.all_gather_object(parts, (lo, r["u0"]))
    if rank == 0:
        out.put((float(t), parts))
    dist.destroy_process_group()


def test_shard_range_covers_all_lanes():
    for total in (1, 7, 64, 65536 * 8 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_gloo_matches_single_process():
    from oracle.oracle import Oracle, make_opts
    total, world = 24, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    tmax, parts = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 2.0                                   # max over ranks
    u0 = np.concatenate([u for _, u in sorted(parts, key=lambda t: t[0])])
    orc = Oracle()
    x0 = config2_x0(total, 123)
    ref = orc.controller_solve(make_opts(N=10, sqp_iters=2), x0, straight_traj(), 1, orc.new_warm(total, 10),
                               shape_id=np.arange(total) % 4, nthreads=1)
    np.testing.assert_array_equal(u0, ref["u0"])


def test_make_inputs_shards_match_single_process():
    from bench import make_inputs
    full = make_inputs(1000, 20, 7)
    for world in (2, 3, 8):
        parts = [make_inputs(1000, 20, 7, *shard_range(1000, world, r)) for r in range(world)]
        for q in range(4):
            np.testing.assert_array_equal(np.concatenate([p[q] for p in parts]), full[q])
