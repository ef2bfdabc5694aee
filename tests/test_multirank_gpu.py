"""The multi-rank GPU path of bench.py, executed on the one GPU of the test box.

The driver's N = 2…8 scaling run uses RCCL with one GPU per rank; a one-GPU box cannot host
that, so these tests run the SAME code with two ranks sharing cuda:0 over gloo
(`--dist-backend gloo`: host-staged collectives and gather).  Everything else is the N > 1
device path the scaling run executes: per-rank device shards from the counter-based generator
at `traj0`, the barrier + MAX-over-ranks timing, the device-side output scans summed over
ranks, the timed info + P₁ gather to rank 0 and its sampled parity against the CPU oracle,
rank 0's own sampled parity and its cpu_baseline.

Both launchers are covered: bench.py spawning its own ranks (`--gpus 2`, no WORLD_SIZE) and
`torch.distributed.run` (what the driver runs).  Each test starts the launcher as a child
process (never an exec from this GPU-initialised process) under a timeout.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# cfg4's shape (n=32 m=16 N=256 are bench.py's defaults — and must stay implicit: torchrun's
# own parser would take "--n" for an abbreviation of its --nnodes / --nproc-per-node)
ARGS = ["--gpus", "2", "--dist-backend", "gloo", "--batch", "2049", "--steps", "2", "--warmup", "1",
        "--cpu-seconds", "1"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout            # rank 0 prints exactly one line
    return json.loads(lines[0])


def _check(line, batch=2049):
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    cfg = line["config"]
    assert cfg["global_batch"] == batch and cfg["dist_backend"] == "gloo"
    # the shards tile the global batch: contiguous, in rank order, sizes differing by ≤ 1
    sh = [tuple(s) for s in cfg["shards"]]
    assert sh[0][0] == 0 and sh[0][0] + sh[0][1] == sh[1][0] and sh[1][0] + sh[1][1] == batch
    assert abs(sh[0][1] - sh[1][1]) <= 1
    assert line["value"] > 0 and line["ms_per_step"] > 0
    chk = line["check"]
    assert chk["nonfinite"] == 0 and chk["info_nonzero"] == 0
    assert chk["sampled_parity"]["pass"], chk["sampled_parity"]
    g = line["gather"]
    assert g is not None and g["delivered"] == batch and g["root_info_nonzero"] == 0
    assert g["sampled_parity"]["pass"], g["sampled_parity"]
    assert batch - 1 in g["sampled_parity"]["indices"]         # rank 1's last trajectory
    assert g["bytes_to_root"] > 0
    cpu = line["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["kind"] == "port"


def test_bench_two_ranks_spawned(lqrx, gpu_ok):
    """`python bench.py --gpus 2`: the bench spawns its two ranks itself."""
    _check(_run([sys.executable, "-u", "bench.py"] + ARGS))


def test_bench_two_ranks_torchrun(lqrx, gpu_ok):
    """The driver's launcher: torch.distributed.run --nproc-per-node 2 bench.py --gpus 2."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py"] + ARGS
    _check(_run(cmd))
