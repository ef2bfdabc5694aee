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

import os
import time

__all__ = ["shard_range", "gather_to_root", "dist_env", "init_ranks", "timed_steps",
           "max_over_ranks", "sum_over_ranks", "timed_gather", "finish_ranks"]


def dist_env() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the launcher's environment (torch.distributed.run sets
    RANK / WORLD_SIZE / LOCAL_RANK; a plain `python bench.py` is rank 0 of 1)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_ranks(backend: str = "nccl", device=None) -> tuple[int, int, int]:
    """One process per GPU: join the process group when WORLD_SIZE > 1 ("nccl" = RCCL over
    xGMI on ROCm; "gloo" in the CPU tests).  Returns dist_env()."""
    rank, world, local = dist_env()
    if world > 1:
        import torch.distributed as dist
        kw = {"device_id": device} if device is not None and backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def _barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def timed_steps(step, steps: int, warmup: int, sync=lambda: None, world: int = 1,
                on_start=None, on_stop=None) -> float:
    """The bench contract's timed region: `warmup` untimed steps, then exactly `steps`
    steps bracketed on both sides by sync() + a barrier across ranks + sync().  on_start /
    on_stop run inside the bracket right before the first and after the last timed step
    (HIP events on the launch stream).  Returns this rank's wall seconds; the job time is
    max_over_ranks() of it."""
    for _ in range(warmup):
        step()
    sync()
    _barrier(world)
    sync()
    t0 = time.perf_counter()
    if on_start:
        on_start()
    for _ in range(steps):
        step()
    if on_stop:
        on_stop()
    sync()
    _barrier(world)
    sync()
    return time.perf_counter() - t0


def max_over_ranks(x: float, world: int = 1, device=None) -> float:
    """MAX of a float over ranks (all-reduce); identity for world == 1."""
    if world == 1:
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(xs: list[int], world: int = 1, device=None) -> list[int]:
    """Element-wise SUM of small integer counters over ranks; identity for world == 1."""
    if world == 1:
        return [int(x) for x in xs]
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(xs), dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return [int(v) for v in t.tolist()]


def timed_gather(fields: dict, batch: int, world: int, sync=lambda: None, device=None) -> dict:
    """§8(e)'s one exchange, timed apart from the solve: gather_to_root() of the small
    per-trajectory outputs, bracketed by sync + barrier; time = MAX over ranks.  Returns
    {"ms", "bytes_to_root", "got"} (got: the gathered tensors on rank 0, None elsewhere)."""
    sync()
    _barrier(world)
    t0 = time.perf_counter()
    got = gather_to_root(fields, batch)
    sync()
    ms = max_over_ranks(time.perf_counter() - t0, world, device) * 1e3
    per_rank = sum(f.numel() * f.element_size() for f in fields.values())
    return {"ms": ms, "bytes_to_root": per_rank * (world - 1), "got": got}


def finish_ranks(world: int):
    """Final barrier and process-group teardown (no-op for world == 1)."""
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


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
    # `root` is a rank within `group`; dist.gather's dst is a global rank
    dst = root if group is None else dist.get_global_rank(group, root)
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
        dist.gather(buf, parts, dst=dst, group=group)
        if rank == root:
            out[name] = torch.cat([parts[r][: counts[r] * per] for r in range(world)])
    return out
