"""World-size-2 `gloo` tests (CPU) of the multi-GPU bench path: ranks shard the batch by
trajectory index (traj0 = rank·batch) with no data-path collective; the only collectives
are the timing barrier and the MAX-over-ranks of the wall time.  The shards must tile the
single-process batch exactly, and per-rank oracle solves of the shards must equal the
single-process solve (independent problems ⇒ sharding cannot change results)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, root, q):
    import sys

    sys.path[:0] = [os.path.join(root, "lqr.jl_amd"), root]
    import torch
    import lqrx
    from oracle import oracle as orc

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, m, N, per = 6, 3, 12, 5
    d = lqrx.random_batch(n, m, N, per, seed=77, traj0=rank * per)
    out = orc.dp_solve_abi(d, N)
    wall = torch.tensor([0.1 * (rank + 1)], dtype=torch.float64)
    dist.barrier()
    dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    q.put((rank, d["A"], out["K"], float(wall.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_gloo(lqrx):
    import lqrx as L
    from oracle import oracle as orc

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = L.random_batch(6, 3, 12, 10, seed=77)
    ref = orc.dp_solve_abi(full, 12)
    assert np.array_equal(np.concatenate([res[0][1], res[1][1]]), full["A"])
    assert np.array_equal(np.concatenate([res[0][2], res[1][2]]), ref["K"])
    assert res[0][3] == pytest.approx(0.2) and res[1][3] == pytest.approx(0.2)


def _gather_worker(rank, world, port, root, batch, q):
    import sys

    sys.path[:0] = [os.path.join(root, "lqr.jl_amd"), root]
    import torch
    import lqrx
    from lqrx.shard import gather_to_root, shard_range
    from oracle import oracle as orc

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, m, N = 4, 2, 9
    first, cnt = shard_range(batch, rank, world)
    if cnt:
        d = lqrx.random_batch(n, m, N, cnt, seed=31, traj0=first)
        o = orc.dp_solve_abi(d, N)
        fields = {"info": torch.from_numpy(o["info"]), "P": torch.from_numpy(o["P"]),
                  "U": torch.from_numpy(o["U"])}
    else:
        fields = {"info": torch.zeros(0, dtype=torch.int32), "P": torch.zeros(0, dtype=torch.float64),
                  "U": torch.zeros(0, dtype=torch.float64)}
    got = gather_to_root(fields, batch)
    q.put((rank, None if got is None else {k: v.numpy() for k, v in got.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 11), (3, 7), (3, 2)])
def test_gather_to_root_gloo(lqrx, world, batch):
    """Final gather: ragged contiguous shards (shard_range), info + P_1 + U of
    every shard reach rank 0 in trajectory order and equal the single-process solve; other
    ranks receive nothing.  (3, 2) has an empty shard."""
    import lqrx as L
    from lqrx.shard import shard_range
    from oracle import oracle as orc

    spans = [shard_range(batch, r, world) for r in range(world)]
    assert spans[0][0] == 0 and sum(c for _, c in spans) == batch
    assert all(spans[r][0] + spans[r][1] == spans[r + 1][0] for r in range(world - 1))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, root, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res[r] is None for r in range(1, world))
    ref = orc.dp_solve_abi(L.random_batch(4, 2, 9, batch, seed=31), 9)
    for k in ("info", "P", "U"):
        assert np.array_equal(res[0][k], ref[k]), k


def _bench_scaffold_worker(rank, world, port, root, per, q):
    """bench.py's rank logic (lqrx.shard: init_ranks, timed_steps, sum/max_over_ranks,
    timed_gather, finish_ranks) with the oracle as the per-rank solver."""
    import sys
    import time

    sys.path[:0] = [os.path.join(root, "lqr.jl_amd"), root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch
    import lqrx
    from lqrx import shard as SH
    from oracle import oracle as orc

    r, w, local = SH.init_ranks("gloo")
    assert (r, w, local) == (rank, world, rank)
    n, m, N = 4, 2, 10
    d = lqrx.random_batch(n, m, N, per, seed=91, traj0=rank * per)    # bench's weak sharding
    calls = []
    res = {}

    def step():
        calls.append(1)
        res.update(orc.dp_solve_abi(d, N))
        time.sleep(0.02 * (rank + 1))                                  # ranks finish unevenly

    wall = SH.timed_steps(step, steps=3, warmup=2, world=w)
    nonfinite = int(sum((~np.isfinite(res[k])).sum() for k in ("K", "X", "U")))
    bad = int((res["info"] != 0).sum())
    nf, nb = SH.sum_over_ranks([nonfinite, bad + rank], w)
    job = SH.max_over_ranks(wall, w)
    g = SH.timed_gather({"info": torch.from_numpy(res["info"]), "P": torch.from_numpy(res["P"])},
                        per * w, w)
    got = g["got"]
    q.put((rank, len(calls), wall, job, nf, nb, g["ms"], g["bytes_to_root"],
           None if got is None else {k: v.numpy() for k, v in got.items()}))
    SH.finish_ranks(w)


def test_bench_rank_scaffolding_gloo(lqrx):
    """The multi-GPU bench path minus the GPU: warmup + exactly `steps` timed steps per rank,
    job time = MAX over ranks (≥ the slowest rank's own wall), counters summed over ranks,
    the timed final gather delivers rank-ordered info + P₁ equal to a one-process solve."""
    import lqrx as L
    from oracle import oracle as orc

    world, per = 2, 3
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_scaffold_worker, args=(r, world, port, root, per, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {r[0]: r for r in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        _, ncalls, wall, job, nf, nb, gms, gbytes, got = res[r]
        assert ncalls == 5                                   # 2 warmup + 3 timed
        assert job >= max(res[k][2] for k in range(world)) - 1e-9
        assert job >= 3 * 0.02 * world                       # slowest rank's sleeps
        assert nf == 0 and nb == sum(range(world))           # SUM over ranks
        assert gms > 0 and gbytes == per * (4 + 4 * 4 * 8) * (world - 1)
        assert (got is None) == (r != 0)
    ref = orc.dp_solve_abi(L.random_batch(4, 2, 10, per * world, seed=91), 10)
    assert np.array_equal(res[0][8]["info"], ref["info"])
    assert np.array_equal(res[0][8]["P"], ref["P"])


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


@pytest.mark.parametrize("scaling,batch", [("strong", 65536), ("strong", 11), ("weak", 5)])
def test_bench_launcher_spawns_ranks_gloo(scaling, batch):
    """`python bench.py --gpus 2` without a launcher: bench.py spawns the two ranks itself
    (lqrx.shard.spawn_ranks, before any GPU call), each joins the process group, and rank 0
    reports n_gpus == 2; strong scaling splits the GLOBAL batch into shards that tile it,
    weak scaling gives every rank `batch` of its own (--dry-run: gloo, no solve)."""
    rc, line, err = _run_bench(["--gpus", "2", "--dry-run", "--batch", str(batch), "--steps", "2",
                                "--warmup", "1", "--scaling", scaling])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2 and line["scaling"] == scaling
    spans = [tuple(s) for s in line["shards"]]
    if scaling == "strong":
        assert line["global_batch"] == batch
        assert spans[0][0] == 0 and spans[0][0] + spans[0][1] == spans[1][0]
        assert spans[1][0] + spans[1][1] == batch and abs(spans[0][1] - spans[1][1]) <= 1
    else:
        assert spans == [(0, batch), (batch, batch)] and line["global_batch"] == 2 * batch


def test_bench_launcher_world_mismatch_exits_nonzero():
    """A launcher-set WORLD_SIZE that disagrees with --gpus is an error (exit 2), not a
    silent one-rank run."""
    rc, line, _ = _run_bench(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0"})
    assert rc == 2 and line is None


def test_spawn_ranks_reports_failure():
    """A failing rank makes spawn_ranks return non-zero (and stops the other rank)."""
    from lqrx.shard import spawn_ranks
    assert spawn_ranks(2, _fail_on_rank1, timeout=120) == 3


def _fail_on_rank1():
    import time
    if os.environ["RANK"] == "1":
        return 3
    time.sleep(30)
    return 0
