"""Multi-GPU batch planning: one process per GPU, batch sharded.

Problems are independent, so there is no per-iteration communication.  The
collectives (torch.distributed: "nccl" = RCCL over xGMI on the GPUs, "gloo" in
the CPU tests) are exactly the four §8e lists:

1. broadcast of the shared environment (obstacles, and start/goal when rank 0
   owns them) from rank 0 — broadcast_environment;
2. none inside the optimiser (K, dK, F are rebuilt deterministically per rank);
3. gather of the per-rank α / trajectories / statistics to rank 0, which writes
   the batch files — gather_batch (shards padded to the largest one; the other
   ranks receive nothing);
4. the scalar reductions of the benchmark (max elapsed, Σ iterations) —
   reduce_timing.

shard(B, world, rank) gives rank r the rows [lo, hi) of the global batch:
contiguous, in rank order, the first B mod world ranks one row larger.
"""
import os

import numpy as np


def world_info():
    """(world, rank, local_rank) from the torchrun environment (1, 0, 0 when absent)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(B, world, rank):
    base, extra = divmod(int(B), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _dist():
    import torch.distributed as dist
    return dist


def broadcast_environment(obstacles, start=None, goal=None, device="cpu", src=0):
    """Rank src's obstacles (O×2 or B×O×2) and optional start/goal (B×D) on every rank.

    Shapes must agree across ranks (the batch size is a CLI argument); values come from src."""
    import torch
    dist = _dist()
    out = []
    for a in (obstacles, start, goal):
        if a is None:
            out.append(None)
            continue
        t = torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device)
        dist.broadcast(t, src=src)
        out.append(t.cpu().numpy())
    return tuple(out)


def gather_batch(arrays, B, device="cpu", dst=0):
    """Gather per-rank shards (dict name -> array with leading dim = this rank's shard size) to rank
    `dst`: there, global arrays (leading dim B, rank order); None on every other rank."""
    import torch
    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    sizes = [shard(B, world, r)[1] - shard(B, world, r)[0] for r in range(world)]
    mx = max(sizes)
    out = {}
    for name, a in arrays.items():
        a = np.ascontiguousarray(a)
        if a.shape[0] != sizes[rank]:
            raise ValueError(f"{name}: rank {rank} holds {a.shape[0]} rows, shard is {sizes[rank]}")
        dt = a.dtype
        buf = np.zeros((mx,) + a.shape[1:], dtype=dt)
        buf[: a.shape[0]] = a
        t = torch.from_numpy(buf).to(device)
        parts = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
        dist.gather(t, parts, dst=dst)
        if rank == dst:
            out[name] = np.concatenate([p.cpu().numpy()[: sizes[r]] for r, p in enumerate(parts)], axis=0)
    return out if rank == dst else None


def reduce_timing(elapsed, iterations, device="cpu"):
    """(max elapsed over ranks, Σ executed iterations over ranks)."""
    import torch
    dist = _dist()
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    it = torch.tensor([float(iterations)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(it, op=dist.ReduceOp.SUM)
    return float(t.item()), float(it.item())
