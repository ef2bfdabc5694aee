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
           "max_over_ranks", "sum_over_ranks", "timed_gather", "finish_ranks", "spawn_ranks",
           "rank_partition", "profiler_preload"]


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_child(rank, world, port, fn, args):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rc = fn(*args)
    raise SystemExit(int(rc or 0))


_TOOL_ENV = ("ROCP_TOOL_LIBRARIES", "HSA_TOOLS_LIB", "ROCPROFILER_LIBRARY", "ROCP_TOOL_LIB")


def profiler_preload() -> str | None:
    """The profiler / HSA-tool preload active in this process's environment, if any
    (rocprofv3 sets LD_PRELOAD to its tool library and ROCP_TOOL_LIBRARIES; an HSA tool sets
    HSA_TOOLS_LIB).  Such a tool initialises the GPU before the program's own code runs."""
    pre = os.environ.get("LD_PRELOAD", "")
    for lib in pre.replace(":", " ").split():
        if "rocprof" in os.path.basename(lib):
            return f"LD_PRELOAD={lib}"
    for k in _TOOL_ENV:
        if os.environ.get(k):
            return f"{k}={os.environ[k]}"
    return None


def spawn_ranks(nprocs: int, fn, *args, port: int | None = None, timeout: float | None = None) -> int:
    """One process per GPU without an external launcher: start `nprocs` fresh interpreters
    (multiprocessing "spawn": fork + exec of python by THIS process, which must not have
    touched the GPU yet) with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT set — what torch.distributed.run would set — each running fn(*args).  Waits
    for all; returns 0 if every rank exited 0, else the first non-zero exit code (a rank
    killed by a signal gives 128 + signal).  If one rank fails the others are terminated
    rather than left hanging in a collective."""
    import multiprocessing as mp
    import time as _t

    tool = profiler_preload()
    if tool:
        # under rocprofv3 (or any HSA tool preload) this process has been GPU-initialised by
        # the tool before main() ran; starting ranks from it is the exec this pool forbids
        raise RuntimeError(f"spawn_ranks: a profiler/tool preload is active ({tool}); profile one "
                           "rank (--gpus 1) or launch the ranks with torch.distributed.run")
    ctx = mp.get_context("spawn")
    port = port or _free_port()
    procs = [ctx.Process(target=_rank_child, args=(r, nprocs, port, fn, args)) for r in range(nprocs)]
    for p in procs:
        p.start()
    t0 = _t.monotonic()
    rc = 0
    while any(p.is_alive() for p in procs):
        for p in procs:
            p.join(0.2)
            if p.exitcode not in (None, 0) and rc == 0:
                rc = p.exitcode if p.exitcode > 0 else 128 - p.exitcode
        if rc or (timeout is not None and _t.monotonic() - t0 > timeout):
            rc = rc or 124
            for p in procs:
                if p.is_alive():
                    p.terminate()
            for p in procs:
                p.join(30)
            break
    for p in procs:
        if p.exitcode not in (None, 0) and rc == 0:
            rc = p.exitcode if p.exitcode > 0 else 128 - p.exitcode
    return rc


def rank_partition(batch: int, rank: int, world: int, scaling: str = "strong") -> tuple[int, int, int]:
    """(first trajectory, count, global batch) of this rank's contiguous shard.  "strong": the
    GLOBAL `batch` is split by shard_range (cfg4 65536 → 8192 per GPU at 8);
    "weak": every rank solves `batch` trajectories of its own (first = rank·batch)."""
    if scaling == "strong":
        first, cnt = shard_range(batch, rank, world)
        return first, cnt, batch
    if scaling == "weak":
        return rank * batch, batch, batch * world
    raise ValueError(f"scaling must be 'strong' or 'weak' (got {scaling!r})")


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
