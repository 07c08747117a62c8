"""Lane sharding across GPUs: one process per GPU, each solving a contiguous
shard of the global lane set with no collective on the data path; the only exchange is the
final gather of u0 and status (north_star: "RCCL over xGMI only for the trivial gather").

Lanes are independent NMPC instances, so a shard's results are bit-identical to the same lanes
solved in a single process (tests/test_distributed.py, tests/test_gpu_multirank.py).
"""
import torch


def shard_range(total, world, rank):
    """Contiguous, balanced shard [lo, hi) of `total` lanes for `rank` (covers every lane once)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_lanes(local, total, dist, world, rank):
    """All-gather of a per-lane tensor (n_local, ...) into the global (total, ...) tensor in
    lane order, on every rank.  One collective per tensor: the shards are padded to the
    largest shard so the exchange is a single fixed-size all_gather (RCCL over xGMI with the
    nccl backend and device tensors; gloo with host tensors)."""
    sizes = [shard_range(total, world, r) for r in range(world)]
    cap = max(h - l for l, h in sizes)
    lo, hi = sizes[rank]
    if local.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: local shard has {local.shape[0]} lanes, expected {hi - lo}")
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: hi - lo] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([parts[r][: h - l] for r, (l, h) in enumerate(sizes)])
