#!/usr/bin/env python3
"""bench.py — batched LQR (Riccati backward + forward rollout) throughput on MI355X.

Metric (BASELINE.json): LQR trajectories/sec, n=32 m=16 N=256 B=65536 fp64.
A "step" = one lqrx_dp_solve launch over the rank's whole shard (inputs resident in HBM,
outputs K/P/X/U written to HBM).  One process per GPU: under torch.distributed.run (RANK /
WORLD_SIZE set by the launcher) or, for a plain `python bench.py --gpus N`, N ranks spawned
by this script before anything touches a GPU (lqrx.shard.spawn_ranks).  The batch is
sharded (independent problems, no data-path collective): by default the GLOBAL
`--batch` is split into contiguous shards (lqrx.shard.shard_range; strong scaling — cfg4
65536 → 8192 per GPU at 8), with `--scaling weak` every rank solves `--batch` trajectories
of its own.  Shards come from the same counter-based generator at the shard's first
trajectory index, so the union of the shards is the one-GPU batch.

Prints ONE JSON line on rank 0 (contract in the task description), with a `roofline`
object for the Riccati kernel (fp64 compute roofline: algorithmic flops per launch ÷ the
kernel's own HIP-event-timed duration on the launch stream) and a `cpu_baseline` object
(the CPU oracle — a restatement of the reference path — timed on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lqr.jl_amd"))
sys.path.insert(0, ROOT)

METRIC = "LQR trajectories/sec (Riccati bwd+fwd), n=32 m=16 N=256 B=65536; 1/2/4/8 GPU"
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 vector = FP64 matrix (spec); MI355X_MICROARCH.md
PEAK_FP32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0
ACHIEVABLE_HBM_GBS = 6290.0   # measured float4 copy rate (MI355X_MICROARCH.md)


def dp_flops_per_traj(n, m, N):
    """(N−1)[4n³+8n²m+4nm²+m³/3+2n²+2m²] + (N−1)(2n²+4nm)."""
    return (N - 1) * (4 * n**3 + 8 * n**2 * m + 4 * n * m**2 + m**3 / 3 + 2 * n**2 + 2 * m**2) \
        + (N - 1) * (2 * n**2 + 4 * n * m)


def dp_bytes_per_traj(n, m, N, s=8, tv=False):
    """SURVEY.md §8(d), time-invariant: read (3n²+nm+m²+n)s, write ((N−1)mn+Nn+(N−1)m+n²)s;
    time-varying: A, B, Q, R read once per knot (×(N−1))."""
    rd = (2 * n * n + n * m + m * m) * ((N - 1) if tv else 1) + n * n + n
    return rd * s + ((N - 1) * m * n + N * n + (N - 1) * m + n * n) * s


def _dp_kernel_name(n, m, bt, tv, lin=False, f64=False):
    """Which DP kernel lqrx_dp_solve dispatches to (mirrors dp_launch / dp_lane_launch)."""
    if n <= 4 and m <= 4:
        small = os.environ.get("LQRX_DP_SMALL", "")
        hex_ = not tv and not lin and small.startswith("h")
        if hex_:
            return "dp_hex_kernel"
        quad = n >= 3 and not tv and (small.startswith("q") or (not small.startswith("l") and bt <= 16384))
        return "dp_quad_kernel" if quad else "dp_lane_kernel"
    if n > 64 or m > 32:
        return "dp_big_kernel"      # workgroup per trajectory, past the register tiles
    if f64 and n == 64 and m in (16, 32) and os.environ.get("LQRX_DP_WG4", "") != "0":
        return "dp_wg4_kernel"      # four waves per trajectory (lqrx_dp.hip; TV / LIN variants: round 6)
    return "dp_riccati_kernel"


def cpu_baseline(n, m, N, target_s=12.0, threads=None, tv=False, linear=False):
    """Time the CPU oracle (C restatement of dynamic_programming.jl, OpenMP over the batch)
    on a bounded sample of the same workload; returns traj/s and the sample description.
    tv: per-knot A_k, B_k, Q_k, R_k streamed by the oracle (oracle_dp_solve_batch_tv with
    tv_AB = tv_QR = 1); linear: the q, r, qf terms (oracle_dp_solve_one_lin) — the same
    problem class the GPU line solves."""
    import numpy as np
    import lqrx
    from oracle import oracle as orc

    threads = threads or max(1, min(16, os.cpu_count() or 1))
    orc.load()

    def problem(bt):
        d = lqrx.random_batch(n, m, N, bt, seed=20260104)
        if linear:
            rng = np.random.default_rng(7)
            d.update(q=rng.standard_normal(bt * n), r=rng.standard_normal(bt * m),
                     qf=rng.standard_normal(bt * n))
        if tv:
            for k in ("A", "B", "Q", "R") + (("q", "r") if linear else ()):
                v = np.asarray(d[k]).reshape(bt, 1, -1)
                d[k] = np.ascontiguousarray(np.broadcast_to(v, (bt, N - 1, v.shape[-1]))).ravel()
            d.update(tv_AB=1, tv_QR=1)
        return d

    solve = orc.dp_solve_lin_abi if linear else orc.dp_solve_abi
    probe = threads * 2
    d = problem(probe)
    t0 = time.perf_counter()
    solve(d, N, nthreads=threads)
    dt = time.perf_counter() - t0
    per = dt / probe
    sample = int(max(probe, min(65536 if not tv else 8192, target_s / max(per, 1e-9))))
    sample = (sample // threads) * threads or threads
    d = problem(sample)
    t0 = time.perf_counter()
    solve(d, N, nthreads=threads)
    dt = time.perf_counter() - t0
    what = ", ".join(w for w, on in (("time-varying per-knot A_k B_k Q_k R_k", tv),
                                     ("linear cost terms q r qf", linear)) if on)
    return dict(value=sample / dt, unit="trajectories/s", cores=threads, kind="port",
                sample=f"{sample} trajectories of n={n} m={m} N={N} fp64{' (' + what + ')' if what else ''}, "
                       f"oracle/lqr_oracle.c (op-for-op C restatement of dynamic_programming.jl), OpenMP "
                       f"{threads} threads, {dt:.1f} s")


def kkt_structure(name, N, n=None, m=None):
    """The KKT block structure of the kkt workload: the Dubins car of BASELINE configs[2], the
    reference's own known-answer structure DoubleIntegrator(3, N) (test/problems.jl:14-56), or
    "dense": the trajectory structure (conblocks.jl:403-425) at any n, m with dense random
    dynamics blocks — BASELINE configs[4]'s banded KKT at n=64 m=32 N=512."""
    import lqrx.kkt as K
    if name == "dense":
        return K.trajectory_structure(n, m, N)
    return K.dubins_structure(N) if name == "dubins" else K.double_integrator_structure(3, N)


def kkt_big_flops(st):
    """Flops of one large-block KKT solve, per trajectory, in two counts.
    reference: the op count of the reference's calls (cholesky_solver.jl _solve!): shur! as
      ldiv + r = YJ·g + the full YYt = Y·JYt gemm (jacobian_blocks.jl:231-242), cholesky! with
      potrf/trsm/gemm per block (cholesky_solve.jl:47-67), forward/backward substitution
      (:93-143) and the primal recovery (cholesky_solver.jl:201-236);
    minimal: the same with every symmetric product counted once (YYt's upper triangle, the
      syrk updates) — what an implementation that exploits symmetry must execute; the roofline
      `achieved` uses this one so the fraction cannot exceed what the hardware can do."""
    import numpy as np
    ref = mini = 0.0
    for k in range(st.N):
        p1, ps, p2, w = int(st.n1[k]), int(st.p[k]), int(st.n2[k]), int(st.w[k])
        r = p1 + ps + p2
        sub = (w * r + 2.0 * r * w                                  # ldiv, r = YJ·g
               + p1 * p1 * ps + ps ** 3 / 3.0 + p1 * p1 * p2        # trsm D, potrf B, trsm F
               + 2.0 * p1 * ps * p2 + ps * ps * p2 + p2 ** 3 / 3.0  # E − DᵀF, trsm E, potrf C
               + 4.0 * (p1 * ps + ps * ps / 2 + p1 * p2 + ps * p2 + p2 * p2 / 2)   # fwd + bwd subst
               + 2.0 * r * w + w)                                    # residual + ldiv
        ref += sub + 2.0 * r * r * w + 2.0 * p1 * ps * ps + 2.0 * p1 * p2 * p2 + 2.0 * ps * p2 * p2
        mini += sub + r * (r + 1.0) * w + p1 * ps * (ps + 1.0) + p1 * p2 * (p2 + 1.0) + ps * p2 * (p2 + 1.0)
    return ref, mini


def cpu_baseline_kkt_dense(st, target_s=12.0, threads=None):
    """CPU oracle (C restatement of _solve!, fp64, OpenMP) on a bounded sample of the
    large-block workload (host-generated trajectories of the same structure)."""
    import lqrx.kkt as K
    from oracle import oracle as orc

    threads = threads or max(1, min(16, os.cpu_count() or 1))
    os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
    pb = K.random_kkt(st, threads, seed=1, h_mode=K.H_DIAG, dyn="dense")
    t0 = time.perf_counter()
    orc.kkt_solve_batch(os_, threads, pb.Y, pb.y, pb.H, pb.g, h_mode=2, nthreads=threads)
    dt = time.perf_counter() - t0                    # one round: `threads` solves in parallel
    rounds = int(max(1, min(4, target_s / max(dt, 1e-9))))
    sample = threads * rounds
    if rounds > 1:
        pb = K.random_kkt(st, sample, seed=2, h_mode=K.H_DIAG, dyn="dense")
        t0 = time.perf_counter()
        orc.kkt_solve_batch(os_, sample, pb.Y, pb.y, pb.H, pb.g, h_mode=2, nthreads=threads)
        dt = time.perf_counter() - t0
    return dict(value=sample / dt, unit="trajectories/s", cores=threads, kind="port",
                sample=f"{sample} KKT solves n={st.n} m={st.m} N={st.N} (trajectory structure, dense "
                       f"dynamics), fp64, oracle/lqr_oracle.c (C restatement of _solve!), OpenMP "
                       f"{threads} threads, {dt:.1f} s")


def cpu_baseline_kkt(N, target_s=12.0, threads=None, structure="dubins", h_mode=2):
    """CPU oracle (C restatement of cholesky_solver.jl _solve!) on a bounded sample."""
    import lqrx.kkt as K
    from oracle import oracle as orc

    threads = threads or max(1, min(16, os.cpu_count() or 1))
    st = kkt_structure(structure, N)
    os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
    probe = 256
    pb = K.random_kkt(st, probe, seed=1, h_mode=h_mode)
    t0 = time.perf_counter()
    orc.kkt_solve_batch(os_, probe, pb.Y, pb.y, pb.H, pb.g, h_mode=h_mode, nthreads=threads)
    per = (time.perf_counter() - t0) / probe
    sample = int(max(probe, min(1 << 18, target_s / max(per, 1e-9))))
    pb = K.random_kkt(st, sample, seed=2, h_mode=h_mode)
    t0 = time.perf_counter()
    orc.kkt_solve_batch(os_, sample, pb.Y, pb.y, pb.H, pb.g, h_mode=h_mode, nthreads=threads)
    dt = time.perf_counter() - t0
    return dict(value=sample / dt, unit="trajectories/s", cores=threads, kind="port",
                sample=f"{sample} {'Dubins' if structure == 'dubins' else 'DoubleIntegrator(3)'} KKT solves "
                       f"N={N}, oracle/lqr_oracle.c (C restatement "
                       f"of _solve!), OpenMP {threads} threads, {dt:.1f} s")


TRAFFIC_FILES = ("traffic_r06.json", "traffic_r05.json", "traffic_r04.json", "traffic_r03.json", "traffic_r02.json")


def traffic_lookup(key, path=None):
    """roofline.traffic: PMC HBM bytes per launch of this exact workload from the committed
    profiles/traffic_*.json (FETCH_SIZE×2 + WRITE_SIZE passes, tools/traffic_json.py), newest
    round first, with where it came from — the file, the key, the commit it was measured at, the
    PMC run, the kernels measured and their sources' code digests; traffic_validate() below
    drops a figure that no longer describes the line's kernel."""
    paths = [path] if path else [os.path.join(ROOT, "profiles", f) for f in TRAFFIC_FILES]
    for p in paths:
        if not os.path.exists(p):
            continue
        try:
            e = json.load(open(p)).get(key)
        except Exception:
            e = None
        if e and e.get("hbm_bytes_per_launch"):
            return e["hbm_bytes_per_launch"], {"file": os.path.relpath(p, ROOT), "key": key,
                                               "measured_at_head": e.get("measured_at_head"),
                                               "pmc_source": e.get("source"),
                                               "kernels": e.get("kernels"), "sources": e.get("sources")}
    return None, {"file": None, "key": key, "note": "no PMC FETCH/WRITE pass recorded for this workload"}


def traffic_validate(roof):
    """Keep roofline.traffic only while it describes the kernel this line timed: the entry must
    name its measured kernels and the code digests of their sources (round 5 on), the line's
    dominant kernel must be one of them, and the tree's code digests of those sources must still
    match.  Otherwise traffic is null and traffic_source says why (the stale figure is kept
    beside it as stale_bytes_per_launch)."""
    tsrc = roof.get("traffic_source")
    if not isinstance(tsrc, dict) or roof.get("traffic") is None:
        return
    kernels, sources = tsrc.pop("kernels", None), tsrc.pop("sources", None)
    why = None
    if not kernels or not sources:
        why = "entry records no measured kernels / source digests (measured before round 5)"
    else:
        want = re.findall(r"\b(\w+_kernel)\b", roof.get("kernel") or "")[:1]
        bases = {re.findall(r"(\w+)", k.split("<")[0])[-1] for k in kernels}
        if want and want[0] not in bases:
            why = f"measured kernels {sorted(bases)} do not include this line's {want[0]}"
        else:
            from lqrx import _lib as _L
            now = _L.kernel_source_digest(list(sources), ROOT)
            changed = sorted(f for f, d in sources.items() if now.get(f) != d)
            if changed:
                why = "kernel code changed since the measurement: " + ", ".join(changed)
    if why:
        tsrc["stale"] = why
        tsrc["stale_bytes_per_launch"] = roof["traffic"]
        roof["traffic"] = None
    else:
        tsrc["verified"] = "kernel and source code digests match the measurement"


def _sample_index(batch, k=64):
    k = min(k, batch)
    import numpy as np
    return np.unique(np.linspace(0, batch - 1, k).round().astype(np.int64))


def check_dp_sample(out, sub, idx, n, m, N, bt, tol, threads):
    """Checker (outside the timed region): the timed launch's K, P₁, X, U for a strided
    sample of trajectories (first and last included) against the CPU oracle on the same
    inputs — K/P per knot relative, X/U on the trajectory's scale."""
    import numpy as np
    import torch
    from lqrx.dp import from_abi
    from oracle import oracle as orc

    ti = torch.from_numpy(idx).to(out["K"].device)
    pick = lambda x, w: x.view(bt, w).index_select(0, ti).cpu().numpy().astype(np.float64)
    s = len(idx)
    lin = "q" in sub
    ref = (orc.dp_solve_lin_abi if lin else orc.dp_solve_abi)(dict(sub, n=n, m=m, N=N, batch=s), N,
                                                             nthreads=threads)

    def knot_err(a, b):
        a, b = a.reshape(s, a.shape[1], -1), b.reshape(s, b.shape[1], -1)
        den = np.abs(b).max(axis=2)
        den[den == 0] = 1.0
        return float((np.abs(a - b).max(axis=2) / den).max())

    def traj_err(a, b):
        a, b = a.reshape(s, -1), b.reshape(s, -1)
        return float((np.abs(a - b).max(axis=1) / np.maximum(1.0, np.abs(b).max(axis=1))).max())

    e = dict(K=knot_err(from_abi(pick(out["K"], (N - 1) * m * n), (s, N - 1, m, n)),
                        from_abi(ref["K"], (s, N - 1, m, n))),
             P=knot_err(pick(out["P"], n * n)[:, None], ref["P"].reshape(s, 1, n * n)),
             X=traj_err(pick(out["X"], N * n), ref["X"]),
             U=traj_err(pick(out["U"], (N - 1) * m), ref["U"]))
    if lin:   # feedforward d and p_1 on their trajectory's scale (they cross zero)
        e["d"] = traj_err(pick(out["d"], (N - 1) * m), ref["d"])
        e["p"] = traj_err(pick(out["p"], n), ref["p"])
    return {"trajectories": s, "last_index": int(idx[-1]), "max_rel_err": e, "tol": tol,
            "pass": bool(max(e.values()) <= tol),
            "oracle": "oracle/lqr_oracle.c (restatement of dynamic_programming.jl:54-72)"}


def check_kkt_sample(out, pb, st, idx, bt, threads):
    """Checker: the timed launch's δz, λ for a strided sample against the C oracle of
    cholesky_solver.jl _solve! (1e-10 relative)."""
    import numpy as np
    import torch
    from oracle import oracle as orc

    ti = torch.from_numpy(idx).to(out["dz"].device)
    s = len(idx)
    dz = out["dz"].view(bt, -1).index_select(0, ti).cpu().numpy()
    lam = out["lam"].view(bt, -1).index_select(0, ti).cpu().numpy()
    ref = orc.kkt_solve_batch(orc.KktStructure(st.n, st.m, st.N, st.p), s, pb.Y[idx], pb.y[idx],
                              pb.H[idx], pb.g[idx], h_mode=pb.h_mode, nthreads=threads)
    rel = lambda a, b: float((np.abs(a - b.reshape(a.shape)).max(axis=1)
                              / np.maximum(1e-300, np.abs(b.reshape(a.shape)).max(axis=1))).max())
    e = dict(dz=rel(dz, ref["dz"]), lam=rel(lam, ref["lam"]))
    return {"trajectories": s, "last_index": int(idx[-1]), "max_rel_err": e, "tol": 1e-10,
            "pass": bool(max(e.values()) <= 1e-10),
            "oracle": "oracle/lqr_oracle.c (restatement of cholesky_solver.jl _solve!)"}


def check_kkt_dense_sample(out, t, st, idx, bt, threads, f64):
    """Checker for the large-block workload: the sampled trajectories' inputs copied back from
    HBM (as the kernel saw them, fp32 or fp64) and solved by the fp64 C oracle; fp64 1e-10,
    fp32 1e-4 relative per trajectory (tests/test_kkt_big_gpu.py)."""
    import numpy as np
    import torch
    from oracle import oracle as orc

    ti = torch.from_numpy(idx).to(out["dz"].device)
    s = len(idx)
    pick = lambda x: x.view(bt, -1).index_select(0, ti).double().cpu().numpy()
    Y, y, H, g = (pick(t[k]) for k in ("Y", "y", "H", "g"))
    ref = orc.kkt_solve_batch(orc.KktStructure(st.n, st.m, st.N, st.p), s, Y, y, H, g, h_mode=2,
                              nthreads=threads)
    dz, lam = pick(out["dz"]), pick(out["lam"])

    def rel(a, b):
        b = b.reshape(a.shape)
        return float((np.abs(a - b).max(axis=1) / np.maximum(1e-300, np.abs(b).max(axis=1))).max())
    e = dict(dz=rel(dz, ref["dz"]), lam=rel(lam, ref["lam"]))
    tol = 1e-10 if f64 else 1e-4
    return {"trajectories": s, "last_index": int(idx[-1]), "max_rel_err": e, "tol": tol,
            "pass": bool(max(e.values()) <= tol and (ref["info"] == 0).all()),
            "oracle": "oracle/lqr_oracle.c (restatement of cholesky_solver.jl _solve!), fp64 on the same inputs"}


def check_gathered_P(P, n, m, N, batch, seed, f64, threads, k=8):
    """Checker for the §8(e) gather: P₁ of a strided sample of the GLOBAL batch (first and
    last trajectory included, so every shard boundary region of a 2-rank run is crossed) as it
    arrived on rank 0, against the CPU oracle on the same counter-generated inputs."""
    import numpy as np
    import torch
    import lqrx
    from oracle import oracle as orc

    idx = _sample_index(batch, k)
    Pg = P.view(batch, n * n).index_select(0, torch.from_numpy(idx).to(P.device)).double().cpu().numpy()
    worst = 0.0
    for j, i in enumerate(idx):
        d = lqrx.random_batch(n, m, N, 1, seed=seed, traj0=int(i), dtype=lqrx.F64 if f64 else lqrx.F32)
        ref = orc.dp_solve_abi(d, N, nthreads=threads)["P"].reshape(-1)
        worst = max(worst, float(np.abs(Pg[j] - ref).max() / max(np.abs(ref).max(), 1e-300)))
    tol = 1e-10 if f64 else 1e-4
    return {"trajectories": len(idx), "indices": [int(i) for i in idx], "max_rel_err_P1": worst,
            "tol": tol, "pass": bool(worst <= tol)}


def nonfinite_count(out, keys):
    """Whole-batch scan of the timed launch's outputs on the device."""
    import torch
    return int(sum(int((~torch.isfinite(out[k])).sum().item()) for k in keys if k in out))


def _rank_main(argv):
    """Entry of a rank spawned by main() (lqrx.shard.spawn_ranks sets RANK / WORLD_SIZE)."""
    return main(argv)


def dry_run(args):
    """--dry-run: the launcher, rank set-up, partitioning and MAX-over-ranks of the bench on
    the CPU (gloo), no GPU and no solve — what tests/test_multirank.py drives at world 2."""
    from lqrx import shard as SH
    import torch.distributed as dist

    rank, world, _ = SH.init_ranks("gloo")
    first, cnt, gb = SH.rank_partition(args.batch, rank, world, args.scaling)
    wall = SH.timed_steps(lambda: time.sleep(0.001), args.steps, args.warmup, world=world)
    wall = SH.max_over_ranks(wall, world)
    spans = [None] * world
    if world > 1:
        dist.all_gather_object(spans, (first, cnt))
    else:
        spans = [(first, cnt)]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "scaling": args.scaling, "global_batch": gb,
                          "shards": spans, "steps": args.steps, "wall_s": wall}), flush=True)
    SH.finish_ranks(world)
    return 0


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--m", type=int, default=16)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--batch", type=int, default=65536,
                    help="trajectories: the global batch (--scaling strong, default) or per GPU (weak)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong: the global --batch split over the GPUs (SURVEY §8(e)); weak: --batch per GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + partition + timing scaffolding only, on the CPU (gloo), no solve")
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--seed", type=int, default=20260104)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tv", action="store_true",
                    help="dp: time-varying problem (per-knot A_k, B_k, Q_k, R_k; knot_stride 1, "
                         "SURVEY §8(f) rank 1); default batch 16384 (65536 would need 376 GB)")
    ap.add_argument("--linear", action="store_true",
                    help="dp: linear cost terms q, r, qf (lqrx_dp_solve_linear, SURVEY §8(f) rank 1)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend for N > 1: nccl (= RCCL over xGMI, one GPU per rank) or "
                         "gloo with host-staged collectives (lets several ranks share one GPU: the "
                         "multi-rank test on a one-GPU box)")
    ap.add_argument("--no-gather", action="store_true",
                    help="skip the final info + P_1 gather to rank 0 (N > 1)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic table (default: profiles/traffic_r06.json, then the older rounds'; a "
                         "figure is reported only while its kernel's code is unchanged, see traffic_validate)")
    ap.add_argument("--kkt-structure", choices=["dubins", "di", "dense"], default="dubins",
                    help="kkt workload: Dubins (configs[2]), DoubleIntegrator(3,N) (test/problems.jl), or "
                         "dense: the trajectory structure at --n/--m with dense dynamics, generated in HBM "
                         "(configs[4]: --n 64 --m 32 --N 512 --batch 8192 --dtype f32)")
    ap.add_argument("--graph", action="store_true",
                    help="replay one captured HIP graph per step (no per-call host work in the timed loop); "
                         "dp, cartpole, kkt and ls workloads — the sqp step synchronises with the host "
                         "every pass and cannot be captured")
    ap.add_argument("--kkt-hmode", type=int, choices=[0, 1, 2], default=2,
                    help="kkt workload (dubins / di): BlockCholesky mode of H — 2 diagonal (default), 1 "
                         "block-diagonal, 0 dense (block_cholesky.jl:19-159)")
    ap.add_argument("--kkt-layout", type=int, choices=[0, 1], default=0,
                    help="kkt workload: ABI layout 0 (per trajectory, the reference's blocks) or 1 "
                         "(batch fastest, SoA)")
    ap.add_argument("--sqp-model", choices=["dubins", "cartpole"], default="dubins",
                    help="sqp workload: Dubins car (test/dubins_sqp.jl, mu 10, N 101) or the swing-up "
                         "Cartpole() of test/problems.jl:58-88 (mu 1, N 101, tf 5)")
    ap.add_argument("--workload", choices=["dp", "cartpole", "kkt", "sqp", "ls"], default="dp",
                    help="dp = random dense LQR (BASELINE configs[3], the headline); "
                         "cartpole = configs[1] (n=4 m=1 N=101 B=4096); "
                         "kkt = Dubins block-tridiagonal KKT solve (configs[2], B=16384); "
                         "sqp = Dubins SQP around the KKT solve (SURVEY §8(f) ranks 2-3, B=16384); "
                         "ls = condensed least-squares LQR on cartpole (SURVEY §8(f) rank 4, B=4096)")
    args = ap.parse_args(argv)
    if args.graph and args.workload == "sqp":
        ap.error("--graph: the sqp workload reads its active count back to the host every loop pass "
                 "(lqrx_sqp.hip), which a HIP graph capture cannot contain; use dp, cartpole, kkt or ls")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: spawn one rank per GPU now, before this process touches a GPU
        from lqrx import shard as SH
        return SH.spawn_ranks(args.gpus, _rank_main, argv)
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    if args.dry_run:
        return dry_run(args)
    if args.tv and args.batch == 65536:
        args.batch = 16384
    if args.workload in ("cartpole", "ls"):
        args.n, args.m, args.N = 4, 1, 101
        if args.batch == 65536:
            args.batch = 4096
    if args.workload in ("kkt", "sqp") and not (args.workload == "kkt" and args.kkt_structure == "dense"):
        args.n, args.m = 3, 2                       # Dubins car (test/dubins.jl)
        if args.workload == "sqp" and args.sqp_model == "cartpole":
            args.n, args.m = 4, 1
        if args.workload == "kkt" and args.kkt_structure == "di":
            args.n, args.m = 6, 3                   # DoubleIntegrator(3) (test/problems.jl)
        if args.batch == 65536:
            args.batch = 16384
        if args.N == 256:
            args.N = 101

    import torch
    import lqrx

    from lqrx import shard as SH

    rank, world, local = SH.dist_env()
    # one GPU per rank; with fewer visible GPUs than ranks (the gloo rehearsal on a one-GPU
    # box) ranks share devices round-robin — device_count() does not initialise the GPU
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise RuntimeError("bench.py: no GPU visible")
    local = local % ndev
    if args.dist_backend == "nccl" and world > ndev:
        raise RuntimeError(f"bench.py: {world} ranks over {ndev} GPUs needs --dist-backend gloo "
                           "(RCCL takes one GPU per rank)")
    torch.cuda.set_device(local)
    SH.init_ranks(args.dist_backend, torch.device("cuda", local))
    # device of the collectives' tensors: the GPU for RCCL, the host for gloo
    cdev = torch.device("cuda", local) if args.dist_backend == "nccl" else None
    lib = lqrx.load()
    if lib.lqrx_device_available() != 1:
        raise RuntimeError("liblqrx.so sees no gfx950 device")

    # this rank's contiguous shard: [traj0, traj0 + bt) of the global batch
    traj0, bt, global_batch = SH.rank_partition(args.batch, rank, world, args.scaling)
    if bt < 1:
        raise ValueError(f"global batch {args.batch} < {world} ranks")
    n, m, N = args.n, args.m, args.N
    f64 = args.dtype == "f64"
    dev = torch.device("cuda", local)
    # a created stream, not the null stream: launches on the legacy default stream pay an
    # implicit device-wide ordering (measured: cfg2 step 0.113 ms vs 0.082 ms kernel)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    if args.workload == "ls":
        from lqrx import ls as LS
        from lqrx.models import cartpole_batch
        from lqrx.dp import to_abi
        cb = cartpole_batch(bt, N, seed=args.seed + rank)
        t = {k: torch.from_numpy(to_abi(getattr(cb, k)).ravel()).to(dev) for k in ("A", "B", "Q", "R", "Qf")}
        t["x0"] = torch.from_numpy(cb.x0.ravel()).to(dev)
        t.update(n=n, m=m, batch=bt)
        out = LS.ls_solve_device(t, N, hu_mode=LS.HU_ZERO, stream=sh)

        def step():
            LS.ls_solve_device(t, N, hu_mode=LS.HU_ZERO, stream=sh, out=out)
    elif args.workload in ("dp", "cartpole"):
        tdt = torch.float64 if f64 else torch.float32
        if args.workload == "dp":
            host = lqrx.random_batch(n, m, N, bt, seed=args.seed, traj0=traj0,
                                     dtype=lqrx.F64 if f64 else lqrx.F32)
        else:
            from lqrx.models import cartpole_batch
            from lqrx.dp import to_abi
            cb = cartpole_batch(bt, N, seed=args.seed + rank)
            npdt = "float64" if f64 else "float32"
            host = {k: to_abi(getattr(cb, k)).astype(npdt).ravel()
                    for k in ("A", "B", "Q", "R", "Qf")}
            host["x0"] = cb.x0.astype(npdt).ravel()
        t = {k: torch.from_numpy(host[k]).to(dev) for k in ("A", "B", "Q", "R", "Qf", "x0")}
        t.update(n=n, m=m, batch=bt)
        chk_idx = _sample_index(bt)
        widths = dict(A=n * n, B=n * m, Q=n * n, R=m * m, Qf=n * n, x0=n)
        if args.linear:   # linear cost terms, same counter-based style: seeded per rank
            import numpy as np
            rng = np.random.default_rng(args.seed + 17 * rank)
            npdt = "float64" if f64 else "float32"
            host.update(q=rng.standard_normal(bt * n).astype(npdt), r=rng.standard_normal(bt * m).astype(npdt),
                        qf=rng.standard_normal(bt * n).astype(npdt))
            widths.update(q=n, r=m, qf=n)
        chk_sub = {k: host[k].reshape(bt, w)[chk_idx].astype("float64").ravel()
                   for k, w in widths.items()}
        if args.linear:
            for k in ("q", "r", "qf"):
                t[k] = torch.from_numpy(host[k]).to(dev)
        del host
        if args.tv:
            # per-knot fields: every knot's block is its own copy in HBM (the kernel streams
            # all N−1 of them), values = the time-invariant draw
            for k in ("A", "B", "Q", "R") + (("q", "r") if args.linear else ()):
                v = t[k].view(bt, 1, -1)
                t[k] = v.expand(bt, N - 1, v.shape[-1]).contiguous().view(-1)
            t.update(tv_AB=1, tv_QR=1)
        out = lqrx.dp_solve_device(t, N, p_mode=0, stream=sh)   # allocates outputs once

        def step():
            lqrx.dp_solve_device(t, N, p_mode=0, stream=sh, out=out)
    elif args.workload == "sqp":
        import lqrx.sqp as Q
        if args.sqp_model == "cartpole":
            sqp_prob = Q.CartpoleSQP(N, mu=1.0)
            x0_, xf_, Z0_ = Q.random_cartpole_batch(sqp_prob, bt, seed=args.seed + rank)
        else:
            dt_, x0_, xf_, Z0_ = Q.random_dubins_batch(N, bt, seed=args.seed + rank)
            sqp_prob = Q.DubinsSQP(N, dt_, mu=10.0)
        z0 = torch.from_numpy(Z0_.ravel()).to(dev)
        t = dict(Z=z0.clone(), x0=torch.from_numpy(x0_.ravel()).to(dev),
                 xf=torch.from_numpy(xf_.ravel()).to(dev),
                 lam=torch.empty(bt * Q.num_multipliers(N, sqp_prob.model), dtype=torch.float64, device=dev),
                 iters=torch.empty(bt, dtype=torch.int32, device=dev),
                 status=torch.empty(bt, dtype=torch.int32, device=dev))
        out = {"info": t["status"]}

        def step():
            t["Z"].copy_(z0)                                  # same problem every step
            Q.sqp_solve_device(sqp_prob, t, stream=sh)
    elif args.kkt_structure == "dense":
        # large-block KKT (configs[4]): inputs generated in HBM, fp64 or fp32
        import lqrx.kkt as K
        st = kkt_structure("dense", N, n, m)
        tdt = torch.float64 if f64 else torch.float32
        t = K.random_kkt_device(st, bt, args.seed + 1000 * rank, dev, tdt)
        ws = torch.empty(K.workspace_size(st, bt, K.H_DIAG, 1, 0, lqrx.F64 if f64 else lqrx.F32),
                         dtype=torch.uint8, device=dev)
        out = K.kkt_solve_device(st, t, K.H_DIAG, 1, stream=sh, workspace=ws)
        pb = None

        def step():
            K.kkt_solve_device(st, t, K.H_DIAG, 1, stream=sh, out=out, workspace=ws)
    else:
        import lqrx.kkt as K
        st = kkt_structure(args.kkt_structure, N)
        hm = args.kkt_hmode
        pb = K.random_kkt(st, bt, seed=args.seed + rank, h_mode=hm)
        kl = args.kkt_layout
        # layout 1: the same data as [element][batch] (transposed on the device, untimed)
        t = {k: (torch.from_numpy(getattr(pb, k)).to(dev).t().contiguous().view(-1) if kl else
                 torch.from_numpy(getattr(pb, k).ravel()).to(dev)) for k in ("Y", "y", "H", "g")}
        t["batch"] = bt
        # caller-owned workspace (lqrx_kkt_solve_ws): a step is the kernel alone, as a serving
        # loop would run it (the pool path adds ~0.05 ms of stream-ordered alloc/free per call)
        ws = torch.empty(K.workspace_size(st, bt, hm, 1, kl), dtype=torch.uint8, device=dev)
        out = K.kkt_solve_device(st, t, hm, 1, stream=sh, workspace=ws, layout=kl)

        def step():
            K.kkt_solve_device(st, t, hm, 1, stream=sh, out=out, workspace=ws, layout=kl)

    if args.graph:
        # one step captured as a HIP graph (torch.cuda.graph on the launch stream) and replayed
        # per step: the serving form, same kernels and work, none of the per-call host work
        # (ctypes marshalling, ~8 µs) that outlasts a sub-0.1-ms kernel in the timed loop
        step()
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            step()
        step = graph.replay
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    sync = lambda: torch.cuda.synchronize(dev)
    wall = SH.timed_steps(step, args.steps, args.warmup, sync, world,
                          on_start=lambda: ev0.record(stream), on_stop=lambda: ev1.record(stream))
    kern_ms = ev0.elapsed_time(ev1) / args.steps       # stream-timed launch duration
    bad = int((out["info"] != 0).sum().item()) if args.workload != "sqp" else \
        int((out["info"] == 2).sum().item())                  # SQP: line-search failures
    # output checks, outside the timed region: the whole batch scanned on the device for
    # non-finite values; a strided sample compared with the CPU oracle (rank 0)
    nonfinite = nonfinite_count(out if args.workload != "sqp" else t,
                                ("K", "P", "X", "U", "d", "p", "dz", "lam", "Z"))
    nonfinite, bad = SH.sum_over_ranks([nonfinite, bad], world, cdev)
    sampled = None
    if rank == 0 and args.workload in ("dp", "cartpole", "kkt"):
        thr = max(1, min(16, os.cpu_count() or 1))
        if args.workload == "kkt" and args.kkt_structure == "dense":
            sampled = check_kkt_dense_sample(out, t, st, _sample_index(bt, 4), bt, thr, f64)
        elif args.workload == "kkt":
            o = out if not args.kkt_layout else \
                {k: out[k].view(-1, bt).t().contiguous().view(-1) for k in ("dz", "lam")}
            sampled = check_kkt_sample(o, pb, st, _sample_index(bt), bt, thr)
        else:   # (a --tv run repeats the time-invariant draw per knot: same oracle problem)
            sampled = check_dp_sample(out, chk_sub, chk_idx, n, m, N, bt,
                                      1e-10 if f64 else 1e-4, thr)

    # final gather, timed separately from the solve: info + P_1 of every
    # shard to rank 0 over RCCL (grouped send/recv); K stays sharded
    gather = None
    if world > 1 and args.workload in ("dp", "cartpole") and not args.no_gather:
        # a failure here propagates: the rank exits non-zero (spawn_ranks / the launcher
        # report it) instead of printing a line with the error folded into a field
        fields = {"info": out["info"], "P": out["P"]}
        if cdev is None:       # gloo: host-staged (the copy is inside the timed gather)
            fields = {k: v.cpu() for k, v in fields.items()}
        g = SH.timed_gather(fields, global_batch, world, sync, cdev)
        got = g.pop("got")
        gather = dict(g, what="info + P_1 of every shard to rank 0 (torch.distributed.gather "
                              "= RCCL send/recv); K stays sharded",
                      backend=args.dist_backend,
                      root_info_nonzero=int((got["info"] != 0).sum().item()) if got is not None else None)
        if got is not None and got["info"].numel() != global_batch:
            raise RuntimeError(f"gather delivered {got['info'].numel()} of {global_batch} trajectories")
        if got is not None:
            gather["delivered"] = int(got["info"].numel())
            if args.workload == "dp":
                gather["sampled_parity"] = check_gathered_P(got["P"], n, m, N, global_batch, args.seed, f64,
                                                            max(1, min(16, os.cpu_count() or 1)))
        del got
    shards = None
    if world > 1:
        import torch.distributed as dist
        shards = [None] * world
        dist.all_gather_object(shards, (traj0, bt))

    wall = SH.max_over_ranks(wall, world, cdev)
    total = global_batch * args.steps
    value = total / wall
    ms_per_step = wall / args.steps * 1e3

    if rank == 0:
        tsrc = None
        if args.workload == "sqp":
            import lqrx.kkt as K
            import lqrx.sqp as Q
            sY, sy, sH, sg = K.trajectory_structure(n, m, N).sizes(K.H_DIAG)
            it_max = int(t["iters"].max().item()) + 1                # loop passes (last = check only)
            # algorithmic bytes per trajectory and loop pass: assembly (z, λ in; Y, y, H, g out),
            # Newton KKT (41 KB class), SOC KKT (Y, y in; δẑ, λ out), line search (z, δz, g, δẑ, λ)
            per_it = ((sg + sy) + (sY + sy + sH + sg)
                      + (sY + sy + sH + sg + sg + sy) + (sY + sy + sg + sy)
                      + (4 * sg + 2 * sy)) * 8
            alg_bytes = per_it * it_max * bt
            achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": achieved / PEAK_HBM_GBS, "traffic": None,
                    "kernel": "whole SQP step (assembly + 2 KKT + line search per pass)",
                    "kernel_ms": kern_ms, "alg_bytes_per_traj": alg_bytes / bt, "loop_passes": it_max}
            mname = "Cartpole swing-up" if args.sqp_model == "cartpole" else "Dubins"
            metric = f"{mname} SQP solves/sec (n={n} m={m} N={N}, <=10 steps, L1-merit line search + SOC)"
            workload = f"{mname} SQP around the KKT solve (SURVEY.md 8(f) ranks 2-3)"
            cpu = None
            if not args.no_cpu_baseline:
                sys.path.insert(0, ROOT)
                import numpy as np
                from oracle import sqp_oracle as S
                model = S.CARTPOLE if args.sqp_model == "cartpole" else S.DUBINS
                nb = 4
                t0c = time.perf_counter()
                refs = [S.solve(S.TrajSQP(N, sqp_prob.dt, sqp_prob.Q, sqp_prob.R, sqp_prob.Qf, x0_[b], xf_[b],
                                          mu=sqp_prob.mu, model=model), Z0_[b]) for b in range(nb)]
                el = time.perf_counter() - t0c
                cpu = {"value": nb / el, "unit": "trajectories/s", "cores": 1, "kind": "port",
                       "sample": f"{nb} trajectories, oracle/sqp_oracle.py (numpy dense KKT restatement of "
                                 f"test/dubins_sqp.jl), {el:.1f} s"}
                # the same trajectories of the last GPU step against the oracle (status, steps,
                # iterate within 1e-8 relative)
                zg = t["Z"].view(bt, -1)[:nb].cpu().numpy()
                sg_, ig_ = t["status"][:nb].cpu().numpy(), t["iters"][:nb].cpu().numpy()
                errs = [float(np.abs(zg[b] - r["z"]).max() / np.abs(r["z"]).max()) for b, r in enumerate(refs)]
                ok = all(sg_[b] == r["status"] and ig_[b] == r["iters"] for b, r in enumerate(refs))
                sampled = {"n": nb, "max_rel_err_z": max(errs), "tol": 1e-8,
                           "status_iters_equal": bool(ok), "pass": bool(ok and max(errs) <= 1e-8)}
        elif args.workload == "ls":
            Nm, Nn = (N - 1) * m, N * n
            # reference op count (least_squares.jl:171-182): ĀᵀĀ as a dense gemm, Āᵀb̄, potrf, potrs
            fl = 2.0 * Nn * Nm * Nm + 2.0 * Nn * Nm + Nm ** 3 / 3.0 + 2.0 * Nm * Nm
            achieved = fl * bt / (kern_ms * 1e-3) / 1e12
            traffic, tsrc = traffic_lookup(f"ls_cartpole_N{N}_B{bt}_f64", args.traffic_json)
            roof = {"traffic_source": tsrc, "bound": "mfma", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / PEAK_FP64_TFLOPS, "traffic": traffic,
                    "kernel": "ls_condensed_kernel (fp64 VALU, LDS-resident H)", "kernel_ms": kern_ms,
                    "flops_per_traj": fl}
            metric = f"condensed least-squares LQR solves/sec (cartpole n=4 m=1 N={N} B={bt}, Hu=0 as a fresh solver)"
            workload = "LeastSquaresSolver solve! on cartpole (SURVEY.md 8(f) rank 4)"
            cpu = None
            if not args.no_cpu_baseline:
                sys.path.insert(0, ROOT)
                from oracle import ls_oracle as LO
                nb, t0c = 0, time.perf_counter()
                while time.perf_counter() - t0c < min(args.cpu_seconds, 5.0) and nb < bt:
                    LO.ls_solve(cb.A[nb], cb.B[nb], cb.Q[nb], cb.R[nb], cb.Qf[nb], cb.x0[nb], N)
                    nb += 1
                el = time.perf_counter() - t0c
                cpu = {"value": nb / el, "unit": "trajectories/s", "cores": 1, "kind": "port",
                       "sample": f"{nb} cartpole trajectories, oracle/ls_oracle.py (numpy restatement of "
                                 f"least_squares.jl solve!, OpenBLAS), {el:.1f} s"}
        elif args.workload == "kkt" and args.kkt_structure == "dense":
            import lqrx.kkt as K
            sY, sy, sH, sg = st.sizes(K.H_DIAG)
            es = 8 if f64 else 4
            alg_bytes = (sY + sy + sH + sg + sg + sy) * es * bt      # inputs + dz + λ
            fl_ref, fl_min = kkt_big_flops(st)
            peak = PEAK_FP64_TFLOPS if f64 else PEAK_FP32_TFLOPS
            achieved = fl_min * bt / (kern_ms * 1e-3) / 1e12
            t_hbm = alg_bytes / (PEAK_HBM_GBS * 1e9)
            t_fl = fl_min * bt / (peak * 1e12)
            traffic, tsrc = traffic_lookup(f"kkt_dense_n{n}_m{m}_N{N}_B{bt}_{args.dtype}", args.traffic_json)
            # fp64 trajectory structures with a compile-time direct-kernel shape (lqrx_kkt_fil.hip
            # fil_dispatch) run kkt_fild_kernel, HBM-bound; everything else the large-block path
            # (the other small ones, up to n=8 m=4, the padded direct kernel: Shape<…, PAD>)
            padded = f64 and N >= 4 and n <= 8 and m <= 4 and (n, m) not in ((5, 2), (7, 3))
            if f64 and N >= 4 and ((n, m) in ((5, 2), (7, 3)) or padded):
                roof = {"bound": "hbm", "achieved": alg_bytes / (kern_ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS,
                        "unit": "GB/s", "frac": alg_bytes / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                        "kernel": ("kkt_fild_kernel<Shape<…, PAD>> (padded direct kernel, lqrx_kkt_fil.hip)"
                                   if padded else "kkt_fild_kernel (compile-time direct shape, lqrx_kkt_fil.hip)")}
            else:
                big = max(n, m) <= 64 and n + m <= 128        # blocks the large-block kernels take
                kname = ("kb_fuse_mid_kernel (interior knots) + kb_bwd_kernel, kb_schur/kb_factor at the "
                         "ends (lqrx_kkt_big.hip)" if big else
                         "kkt_wg_kernel (workgroup per trajectory, blocks past 64 rows, lqrx_kkt_wg.hip)")
                roof = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                        "frac": achieved / peak, "kernel": kname}
            roof.update({"traffic": traffic, "traffic_source": tsrc, "kernel_ms": kern_ms,
                    "flops_per_traj_minimal": fl_min, "flops_per_traj_reference": fl_ref,
                    "reference_count_tflops": fl_ref * bt / (kern_ms * 1e-3) / 1e12,
                    "alg_bytes_per_launch": alg_bytes, "hbm_gbs_alg": alg_bytes / (kern_ms * 1e-3) / 1e9,
                    "t_hbm_ms": t_hbm * 1e3, "t_flop_ms": t_fl * 1e3,
                    "frac_of_binding": max(t_hbm, t_fl) / (kern_ms * 1e-3)})
            metric = (f"KKT solves/sec (banded block-tridiagonal _solve!, trajectory structure n={n} m={m} "
                      f"N={N}, {args.dtype})")
            workload = ("large-block banded KKT solve, cholesky_solver.jl _solve! (BASELINE.json configs[4]"
                        + (")" if (n, m, N, args.dtype) == (64, 32, 512, "f32") else " shape family)"))
            cpu = cpu_baseline_kkt_dense(st, target_s=args.cpu_seconds) \
                if not args.no_cpu_baseline else None
        elif args.workload == "kkt":
            import lqrx.kkt as K
            hm = args.kkt_hmode
            sY, sy, sH, sg = st.sizes(hm)
            alg_bytes = (sY + sy + sH + sg + sg + sy) * 8 * bt     # inputs + dz + λ
            achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
            traffic, tsrc = traffic_lookup(f"kkt_{args.kkt_structure}_N{N}_B{bt}_f64"
                                           + ("_soa" if args.kkt_layout else "")
                                           + (f"_h{hm}" if hm != 2 else ""), args.traffic_json)
            kname = ("kkt_fil_kernel" if args.kkt_structure == "dubins" else "kkt_fild_kernel") if N >= 4 \
                else "kkt_staged_kernel"
            if hm != 2 and args.kkt_structure == "di" and N >= 4:
                kname = "kkt_hpre_kernel + kkt_fild_kernel + kkt_hpost_kernel (dense H = UᵀU passes)"
            roof = {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": achieved / PEAK_HBM_GBS, "traffic": traffic, "traffic_source": tsrc,
                    "kernel": kname,
                    "kernel_ms": kern_ms,
                    "alg_bytes_per_traj": alg_bytes / bt}
            if args.kkt_structure == "dubins":
                metric = "KKT solves/sec (Dubins n=3 m=2 N=101 block-tridiagonal _solve!)"
                workload = "Dubins constrained KKT inner solve (BASELINE.json configs[2])" + \
                    (", ABI layout 1 (batch-fastest SoA)" if args.kkt_layout else "")
            else:
                metric = f"KKT solves/sec (DoubleIntegrator(3,{N}) n=6 m=3 block-tridiagonal _solve!)"
                workload = "DoubleIntegrator KKT structure of test/cholesky_solve.jl (non-baseline)"
            if hm != 2:
                metric = metric[:-1] + f", {('dense', 'block-diagonal')[hm]} H)"
                workload += f", BlockCholesky mode {hm}"
            cpu = cpu_baseline_kkt(N, target_s=args.cpu_seconds, structure=args.kkt_structure, h_mode=hm) \
                if not args.no_cpu_baseline else None
        else:
            flops = dp_flops_per_traj(n, m, N) * bt
            achieved = flops / (kern_ms * 1e-3) / 1e12
            peak = PEAK_FP64_TFLOPS if f64 else PEAK_FP32_TFLOPS
            traffic, tsrc = traffic_lookup(f"n{n}_m{m}_N{N}_B{bt}_{args.dtype}" + ("_tv" if args.tv else "")
                                           + ("_lin" if args.linear else ""), args.traffic_json)
            roof = {"bound": "mfma", "achieved": achieved, "peak": peak,
                    "unit": "TFLOP/s", "frac": achieved / peak, "traffic": traffic,
                    "kernel": _dp_kernel_name(n, m, bt, args.tv or args.linear, f64=f64),
                    "kernel_ms": kern_ms,
                    "flops_per_traj": dp_flops_per_traj(n, m, N),
                    "alg_bytes_per_launch": dp_bytes_per_traj(n, m, N, 8 if f64 else 4, args.tv) * bt}
            if (n, m, args.dtype) == (32, 16, "f64") and not (args.tv or args.linear):
                # executed work beside the reference-op-count fraction: the fast symmetric form
                # issues 129 v_mfma_f64_16x16x4 (2048 flop each) per knot (PMC SQ_INSTS_MFMA,
                # profiles/r02/dp_cfg4_r02_pmc_summary.txt) — the MFMA pipe's real utilisation
                ex = 129 * 2048.0 * (N - 1)
                roof["executed_mfma_flops_per_traj"] = ex
                roof["executed_frac"] = ex * bt / (kern_ms * 1e-3) / 1e12 / peak
            if args.tv:
                # time-varying: per-knot A_k, B_k, Q_k, R_k make the launch HBM-bound (SURVEY
                # §8(d) 4-TV row: t_HBM vs t_FLOP near the ridge) — report the HBM roofline on
                # the §8(d) algorithmic bytes, the fp64 fraction beside it, and the bytes the
                # path must move at least (the rollout re-reads A_k, B_k and K_k: DESIGN §3.1)
                ab = dp_bytes_per_traj(n, m, N, 8 if f64 else 4, True) * bt
                s_ = 8 if f64 else 4
                min_traffic = ab + bt * (N - 1) * (n * n + n * m + m * n) * s_
                hbm = ab / (kern_ms * 1e-3) / 1e9
                roof = {"bound": "hbm", "achieved": hbm, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": hbm / PEAK_HBM_GBS, "traffic": traffic,
                        "kernel": _dp_kernel_name(n, m, bt, True, f64=f64), "kernel_ms": kern_ms,
                        "alg_bytes_per_launch": ab, "min_traffic_bytes_per_launch": min_traffic,
                        "min_traffic_frac": min_traffic / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                        "fp64_tflops": achieved, "fp64_frac": achieved / peak}
            elif n <= 4 and m <= 4:
                # n ≤ 4 (cfg2 cartpole): AI ≈ 6 flop/B is below the ridge, so the roofline is
                # HBM — but the launch is latency-bound: 16 (hex), 4 (quad) or 1 (lane) lanes
                # per trajectory give B·lanes/64 waves (cfg2: 1024 = one per SIMD with hex),
                # each running a serial N-knot chain; report that beside the HBM fraction
                ab = dp_bytes_per_traj(n, m, N, 8 if f64 else 4, False) * bt
                hbm = ab / (kern_ms * 1e-3) / 1e9
                kname = _dp_kernel_name(n, m, bt, False, args.linear, f64=f64)
                lanes = {"dp_hex_kernel": 16, "dp_quad_kernel": 4}.get(kname, 1)
                waves = -(-bt * lanes // 64)
                roof = {"bound": "hbm", "achieved": hbm, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": hbm / PEAK_HBM_GBS, "traffic": traffic, "kernel": kname,
                        "kernel_ms": kern_ms, "alg_bytes_per_launch": ab,
                        "fp64_tflops": achieved, "fp64_frac": achieved / peak,
                        "latency_bound": {"waves": waves, "cus": 256, "waves_per_cu": waves / 256,
                                          "knot_chain_us": kern_ms * 1e3 / N,
                                          "note": "one serial N-knot chain per trajectory; the chip "
                                                  "holds the whole batch at once"}}
            headline = (n, m, N, bt, args.dtype) == (32, 16, 256, 65536, "f64") and not args.tv \
                and not args.linear
            if args.workload == "cartpole":
                metric = f"LQR trajectories/sec (Riccati bwd+fwd), cartpole n=4 m=1 N={N} B={bt}"
                workload = "cartpole LQR, RK3-linearised (BASELINE.json configs[1])"
            elif headline:
                metric = METRIC
                workload = ("random dense time-invariant LQR, Riccati backward pass + forward "
                            "rollout (BASELINE.json configs[3])")
            else:
                metric = (f"LQR trajectories/sec (Riccati bwd+fwd), n={n} m={m} N={N} B={bt} {args.dtype}"
                          + (", time-varying A_k B_k Q_k R_k" if args.tv else "")
                          + (", linear cost terms q r qf" if args.linear else ""))
                cfg5 = (n, m, N, args.dtype) == (64, 32, 512, "f32")
                workload = (("random dense time-varying LQR (SURVEY §8(f) rank 1)" if args.tv else
                             "random dense time-invariant LQR") + ", Riccati backward pass + forward rollout"
                            + (" (BASELINE.json configs[4], per GPU)" if cfg5 else " (non-baseline shape)"))
            cpu = cpu_baseline(n, m, N, target_s=args.cpu_seconds, tv=args.tv, linear=args.linear) \
                if not args.no_cpu_baseline else None
        if tsrc is not None:
            roof.setdefault("traffic_source", tsrc)
        traffic_validate(roof)
        if roof.get("bound") == "hbm":
            # beside the 8 TB/s spec: the measured achievable streaming rate
            # (MI355X_MICROARCH.md: float4 copy, 6.29 TB/s); peak and frac stay on the spec
            roof["achievable_peak"] = ACHIEVABLE_HBM_GBS
            roof["frac_of_achievable"] = roof["achieved"] / ACHIEVABLE_HBM_GBS
            if roof.get("traffic"):
                roof["traffic_rate_frac_of_achievable"] = \
                    roof["traffic"] / (roof["kernel_ms"] * 1e-3) / 1e9 / ACHIEVABLE_HBM_GBS
        line = {
            "metric": metric, "value": value, "unit": "trajectories/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic (counter-based random problems, "
                                          "SURVEY.md §8(d) generator)",
            "config": {"workload": workload, "n": n, "m": m, "N": N, "batch_per_gpu": bt,
                       "global_batch": global_batch, "parallelism": f"batch-sharded x{world}",
                       "shard_rank0": [traj0, bt], "shards": shards,
                       "dist_backend": args.dist_backend if world > 1 else None,
                       "hip_graph": bool(args.graph)},
            "roofline": roof,
            "cpu_baseline": cpu,
            "check": {"nonfinite": nonfinite, "info_nonzero": bad, "sampled_parity": sampled},
            "gather": gather,
        }
        if gather is not None and "ms" in gather:
            line["value_solve_plus_gather"] = total / (wall + gather["ms"] * 1e-3)
        try:   # build provenance: the library's compiled-in source hash vs this tree's
            from lqrx import _lib as _L
            bi = _L.build_info()
            line["build"] = {"library": bi["info"], "matches_tree": bi["matches_tree"]}
        except Exception as exc:   # noqa: BLE001 — reporting only
            line["build"] = {"error": str(exc)}
        print(json.dumps(line), flush=True)
    SH.finish_ranks(world)
    return 0


if __name__ == "__main__":
    sys.exit(main())
