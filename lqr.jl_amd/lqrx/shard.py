"""Batch sharding over GPUs and the final gather to rank 0.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on ROCm; "gloo" in
the CPU tests).  Trajectories are independent, so a batch is split into contiguous shards
with no collective during the solve.  Afterwards only the SMALL per-trajectory outputs are
brought to rank 0 — `info` (4 B) and P₁ (n²·8 B), optionally X / U — while the gains K stay
sharded where they were computed (cfg4: 68.5 GB of K per 65536 trajectories; gathering it
would cost ~7× the solve).  RCCL has no gather primitive; torch's `gather` on the nccl
backend is a grouped send/recv, which is the exchange §8(e) prescribes.
"""
from __future__ import annotations

__all__ = ["shard_range", "gather_to_root"]


def shard_range(batch: int, rank: int, world: int) -> tuple[int, int]:
    """(first trajectory, count) of `rank`'s contiguous shard; the first batch % world
    ranks take one extra trajectory, so every shard differs by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} / world {world}")
    base, extra = divmod(batch, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


def gather_to_root(fields: dict, batch: int, root: int = 0, group=None) -> dict | None:
    """Gather per-trajectory outputs of every rank's shard to `root`, in trajectory order.

    fields: name → 1-D tensor holding this rank's shard, `count` trajectories × a fixed
    per-trajectory size (ABI layout, batch slowest).  batch: the GLOBAL batch (shards as
    shard_range).  Returns name → tensor of the whole batch on root, None elsewhere.
    Shards are padded to the largest shard so every rank sends the same element count."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [shard_range(batch, r, world)[1] for r in range(world)]
    cmax = max(counts)
    out = {} if rank == root else None
    for name, t in fields.items():
        t = t.reshape(-1)
        mine = counts[rank]
        if mine and t.numel() % mine:
            raise ValueError(f"{name}: {t.numel()} elements is not a multiple of {mine} trajectories")
        per = t.numel() // mine if mine else 0
        per = int(max(per, 0))
        # every rank must agree on the per-trajectory size: take the max (empty shards send 0s)
        p = torch.tensor([per], dtype=torch.int64, device=t.device)
        dist.all_reduce(p, op=dist.ReduceOp.MAX, group=group)
        per = int(p.item())
        buf = torch.zeros(cmax * per, dtype=t.dtype, device=t.device)
        buf[: t.numel()] = t
        parts = [torch.empty_like(buf) for _ in range(world)] if rank == root else None
        dist.gather(buf, parts, dst=root, group=group)
        if rank == root:
            out[name] = torch.cat([parts[r][: counts[r] * per] for r in range(world)])
    return out
