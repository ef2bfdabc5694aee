"""GPU parity: batched block-tridiagonal KKT solve (liblqrx.so, C ABI) vs the CPU oracle.

Oracle = oracle/lqr_oracle.c restating cholesky_solver.jl:166-236, jacobian_blocks.jl:
220-286, cholesky_solve.jl:47-143, block_cholesky.jl:55-101 (pinned in test_oracle.py by
the reference's test/cholesky_solve.jl:18-44 identities).  Tolerance: fp64, max|δz − ref| /
max|ref| ≤ 1e-10 and the same for the multipliers.
"""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
TOL = 1e-10


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _ref(st, pb, ginv):
    os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
    return orc.kkt_solve_batch(os_, pb.batch, pb.Y, pb.y, pb.H, pb.g, h_mode=pb.h_mode, ginv=ginv,
                               nthreads=8)


@pytest.mark.parametrize("N,batch", [(101, 256), (11, 67), (3, 5)])   # N=2 Dubins is over-constrained (9 rows, 8 vars)
@pytest.mark.parametrize("h_mode", [2, 0, 1])
def test_kkt_dubins_parity(lqrx, gpu_ok, N, batch, h_mode):
    import lqrx.kkt as K

    st = K.dubins_structure(N)
    pb = K.random_kkt(st, batch, seed=100 + N + h_mode, h_mode=h_mode)
    got = K.kkt_solve(pb)
    ref = _ref(st, pb, 1)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert rel(got["dz"], ref["dz"].reshape(batch, -1)) <= TOL
    assert rel(got["lam"], ref["lam"].reshape(batch, -1)) <= TOL


@pytest.mark.parametrize("D,N", [(3, 101), (2, 12)])
def test_kkt_double_integrator_parity(lqrx, gpu_ok, D, N):
    """The reference's own known-answer structure (test/cholesky_solve.jl on
    DoubleIntegrator(3,101))."""
    import lqrx.kkt as K

    st = K.double_integrator_structure(D, N)
    pb = K.random_kkt(st, 37, seed=9, h_mode=2)
    got = K.kkt_solve(pb)
    ref = _ref(st, pb, 1)
    assert (got["info"] == 0).all()
    assert rel(got["dz"], ref["dz"].reshape(37, -1)) <= TOL
    assert rel(got["lam"], ref["lam"].reshape(37, -1)) <= TOL


def test_kkt_soc_parity(lqrx, gpu_ok):
    """second_order_correction! variant (Ginv = false)."""
    import lqrx.kkt as K

    st = K.dubins_structure(101)
    pb = K.random_kkt(st, 128, seed=3, h_mode=2)
    got = K.second_order_correction(pb)
    ref = _ref(st, pb, 0)
    assert rel(got["dz"], ref["dz"].reshape(128, -1)) <= TOL
    assert rel(got["lam"], ref["lam"].reshape(128, -1)) <= TOL


def test_kkt_info_non_spd(lqrx, gpu_ok):
    import lqrx.kkt as K

    st = K.dubins_structure(11)
    pb = K.random_kkt(st, 4, seed=2, h_mode=0)
    pb.H[2, :] = -pb.H[2, :]
    got = K.kkt_solve(pb)
    assert got["rc"] == 1 and got["info"][2] != 0
    assert got["info"][0] == 0 and got["info"][1] == 0 and got["info"][3] == 0


def test_kkt_alternating_structures(lqrx, gpu_ok):
    """Repeated solves that alternate block structures and batch sizes in one process.
    Regression for a stale device structure table (per-call pool allocation + async copy
    from pageable memory) that corrupted every later solve of one structure."""
    import lqrx.kkt as K

    cases = []
    for N, batch, h, seed in [(11, 4, 0, 18), (101, 256, 2, 5), (11, 67, 1, 3), (3, 5, 2, 4)]:
        st = K.dubins_structure(N)
        pb = K.random_kkt(st, batch, seed=seed, h_mode=h)
        ref = _ref(st, pb, 1)
        cases.append((pb, ref["dz"].reshape(batch, -1), ref["lam"].reshape(batch, -1)))
    for _ in range(8):
        for pb, rd, rl in cases:
            got = K.kkt_solve(pb)
            assert rel(got["dz"], rd) <= TOL and rel(got["lam"], rl) <= TOL


@pytest.mark.parametrize("model,N,batch", [("dubins", 4, 130), ("dubins", 5, 64), ("dubins", 6, 1),
                                           ("dubins", 101, 16384 + 3), ("cartpole", 6, 130), ("cartpole", 7, 1),
                                           ("cartpole", 101, 4096 + 5), ("di", 4, 70), ("di", 101, 1000),
                                           ("t52", 6, 67), ("t52", 101, 4096 + 7), ("t73", 8, 130), ("t73", 101, 1000)])
@pytest.mark.parametrize("h_mode,ginv", [(2, 1), (0, 1), (2, 0)])
def test_kkt_fil_shapes(lqrx, gpu_ok, model, N, batch, h_mode, ginv):
    """The compile-time-shaped first/interior/last kernel (lqrx_kkt_fil.hip) at its edge
    cases: the shortest horizon it serves (N = 4), one trajectory, ragged last waves, the
    full cfg3 batch; Ginv = 0 is the second-order-correction variant.  The cartpole shape
    (n 4, m 1; the device SQP's structure) is instantiated for diagonal H (dense H → the
    H = UᵀU pre-pass around that kernel, round 4; the generic kernel before); N ≥ 6 (N = 4 is
    over-constrained: 20 rows, 19 vars; at N = 5 the system is square and a few of the random
    problems lose 1e-5 to rounding in the oracle and the generic kernel alike — measured,
    tools/kkt_shape_diag.py; at N = 6, 7 it is near-square — 28 rows, 29 vars at N = 6 — and
    with dense H the Z = YU⁻¹ form and the oracle's H⁻¹Yᵀ form round apart by up to ~2e-10, so
    those trajectories are held to the refined truth as below).
    DoubleIntegrator(3) (the structure of test/cholesky_solve.jl) runs the direct variant
    kkt_fild_kernel for diagonal H / SOC, the large-block kernel for dense H, and so do the
    trajectory structures (5, 2, N) and (7, 3, N) ("t52", "t73"); at N = 4 DoubleIntegrator(3)'s
    S reaches cond ~7e6 and the oracle itself is 4.6e-11 from the exact solution, so the
    trajectories past 1e-10 are held to the refined truth instead (tests/kkt_truth.py)."""
    import lqrx.kkt as K
    from kkt_truth import check

    if model == "dubins":
        st = K.dubins_structure(N)
    elif model == "cartpole":
        st = K.trajectory_structure(4, 1, N)
    elif model == "t52":
        st = K.trajectory_structure(5, 2, N)
    elif model == "t73":
        st = K.trajectory_structure(7, 3, N)
    else:
        st = K.double_integrator_structure(3, N)
    pb = K.random_kkt(st, batch, seed=7 * N + h_mode, h_mode=h_mode)
    got = K.kkt_solve(pb, ginv=ginv)
    ref = _ref(st, pb, ginv)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    check(st, pb, ginv, got, ref, TOL,
          fallback=(model == "di" and N == 4) or (model == "cartpole" and N <= 7 and h_mode == 0))


def test_kkt_workspace_entry(lqrx, gpu_ok):
    """lqrx_kkt_solve_ws (caller workspace, no allocation inside) equals lqrx_kkt_solve bit for
    bit on the FIL and generic paths; a short workspace is rejected with -10."""
    import ctypes as C
    import torch
    import lqrx.kkt as K

    for st, bt in ((K.dubins_structure(101), 300), (K.double_integrator_structure(3, 11), 70)):
        pb = K.random_kkt(st, bt, seed=5, h_mode=K.H_DIAG)
        t = {k: torch.from_numpy(getattr(pb, k).ravel()).cuda() for k in ("Y", "y", "H", "g")}
        t["batch"] = bt
        a = K.kkt_solve_device(st, t, K.H_DIAG, 1)
        nb = K.workspace_size(st, bt, K.H_DIAG, 1)
        ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
        b = K.kkt_solve_device(st, t, K.H_DIAG, 1, workspace=ws)
        torch.cuda.synchronize()
        assert torch.equal(a["dz"], b["dz"]) and torch.equal(a["lam"], b["lam"])
        with pytest.raises(lqrx.LqrxError) as e:
            K.kkt_solve_device(st, t, K.H_DIAG, 1, workspace=ws[: nb - 8])
        assert e.value.code == -10


def test_kkt_meta_cache_overflow(lqrx, gpu_ok):
    """Beyond the structure-table cache (LQRX_META_CACHE, default 4096) a call uploads a
    per-call table on its own stream and frees it stream-ordered — no device-wide sync.
    Exercised with the cache capped at 1, alternating structures and streams."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, LQRX_META_CACHE="1")
    r = subprocess.run([sys.executable, os.path.join(here, "_kkt_meta_overflow.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("model,N,batch", [("dubins", 4, 1), ("dubins", 5, 130), ("dubins", 101, 16384 + 3),
                                           ("cartpole", 7, 70), ("cartpole", 101, 4096 + 5),
                                           ("di3", 4, 70), ("di3", 101, 1000), ("di2", 12, 67),
                                           ("t52", 101, 1000 + 3), ("t73", 9, 70)])
@pytest.mark.parametrize("h_mode,ginv", [(2, 1), (0, 1), (1, 1), (2, 0)])
def test_kkt_layout1_soa(lqrx, gpu_ok, model, N, batch, h_mode, ginv):
    """ABI layout 1 (batch fastest: element e of trajectory t at [e·batch + t]) on the
    compile-time-shaped kernels (LDS-staged Dubins / cartpole, direct DoubleIntegrator(2, 3)):
    bit-identical to layout 0 (same arithmetic, only the staging differs: 512-B element rows
    instead of per-trajectory chunks) and within 1e-10 of the oracle; ragged last waves (dead
    lanes read past the arrays' ends, bounds-checked to 0)."""
    import lqrx.kkt as K

    st = {"dubins": lambda: K.dubins_structure(N), "cartpole": lambda: K.trajectory_structure(4, 1, N),
          "di3": lambda: K.double_integrator_structure(3, N), "di2": lambda: K.double_integrator_structure(2, N),
          "t52": lambda: K.trajectory_structure(5, 2, N), "t73": lambda: K.trajectory_structure(7, 3, N)}[model]()
    if model != "dubins" and h_mode != 2 and ginv:
        # dense H: no SoA shape — staged through layout 0 (transpose in, layout-0 kernels,
        # transpose out): identical to the layout-0 call
        pb = K.random_kkt(st, 67, seed=1, h_mode=h_mode)
        got1 = K.kkt_solve(pb, ginv=ginv, layout=1)
        got0 = K.kkt_solve(pb, ginv=ginv, layout=0)
        assert got1["rc"] == 0 and (got1["info"] == got0["info"]).all()
        assert np.array_equal(got1["dz"], got0["dz"]) and np.array_equal(got1["lam"], got0["lam"])
        return
    pb = K.random_kkt(st, batch, seed=11 * N + h_mode, h_mode=h_mode)
    got1 = K.kkt_solve(pb, ginv=ginv, layout=1)
    got0 = K.kkt_solve(pb, ginv=ginv, layout=0)
    assert got1["rc"] == 0 and (got1["info"] == got0["info"]).all()
    assert np.array_equal(got1["dz"], got0["dz"]) and np.array_equal(got1["lam"], got0["lam"])
    idx = np.unique(np.linspace(0, batch - 1, min(batch, 64)).round().astype(int))
    sub = K.KktProblem(st, len(idx), h_mode, pb.Y[idx], pb.y[idx], pb.H[idx], pb.g[idx])
    ref = _ref(st, sub, ginv)
    assert rel(got1["dz"][idx], ref["dz"].reshape(len(idx), -1)) <= TOL
    assert rel(got1["lam"][idx], ref["lam"].reshape(len(idx), -1)) <= TOL


@pytest.mark.parametrize("case", ["t53", "dubins_N3", "big_f32", "big_f64_dense", "wg_f64"])
def test_kkt_layout1_staged(lqrx, gpu_ok, case):
    """Layout 1 outside the compile-time SoA shapes (other structures, N < 4, fp32, the
    large-block and workgroup kernels) is staged: the SoA arrays are transposed to layout 0 in
    scratch, solved by the layout-0 kernel family and transposed back — bit-identical to the
    layout-0 call, and within tolerance of the oracle."""
    import dataclasses
    import lqrx.kkt as K

    st, hm, dt, dyn, tol = {
        "t53": (K.trajectory_structure(5, 3, 12), K.H_DIAG, lqrx.F64, "small", TOL),
        "dubins_N3": (K.dubins_structure(3), K.H_DIAG, lqrx.F64, "small", TOL),
        "big_f32": (K.trajectory_structure(16, 8, 9), K.H_DIAG, lqrx.F32, "dense", 1e-4),
        "big_f64_dense": (K.trajectory_structure(16, 8, 9), K.H_DENSE, lqrx.F64, "dense", TOL),
        "wg_f64": (K.trajectory_structure(72, 36, 5), K.H_DIAG, lqrx.F64, "dense", TOL),
    }[case]
    pb = K.random_kkt(st, 37, seed=2, h_mode=hm, dyn=dyn)
    if dt == lqrx.F32:
        f = lambda a: np.asarray(a, np.float32).astype(np.float64)
        pb = dataclasses.replace(pb, Y=f(pb.Y), y=f(pb.y), H=f(pb.H), g=f(pb.g))
    got1 = K.kkt_solve(pb, layout=1, dtype=dt)
    got0 = K.kkt_solve(pb, layout=0, dtype=dt)
    assert got1["rc"] == 0 and (got1["info"] == 0).all()
    assert np.array_equal(got1["dz"], got0["dz"]) and np.array_equal(got1["lam"], got0["lam"])
    ref = _ref(st, pb, 1)
    assert rel(got1["dz"], ref["dz"].reshape(pb.batch, -1)) <= tol
    assert rel(got1["lam"], ref["lam"].reshape(pb.batch, -1)) <= tol


@pytest.mark.parametrize("case", ["t53", "big_f64"])
def test_kkt_layout1_staged_workspace(lqrx, gpu_ok, case):
    """A staged layout-1 call through lqrx_kkt_solve_ws takes its transposed arrays from the
    caller's workspace (lqrx_kkt_workspace_size counts them: more than the layout-0 call needs),
    gives the pool call's result bit for bit, and a workspace short of the staged arrays is
    rejected with -10."""
    import torch
    import lqrx.kkt as K

    st, dyn = {"t53": (K.trajectory_structure(5, 3, 12), "small"),
               "big_f64": (K.trajectory_structure(16, 8, 9), "dense")}[case]
    bt = 37
    pb = K.random_kkt(st, bt, seed=3, h_mode=K.H_DIAG, dyn=dyn)
    t = {k: torch.from_numpy(getattr(pb, k)).cuda().t().contiguous().view(-1) for k in ("Y", "y", "H", "g")}
    t["batch"] = bt
    n1 = K.workspace_size(st, bt, K.H_DIAG, 1, 1)
    n0 = K.workspace_size(st, bt, K.H_DIAG, 1, 0)
    assert n1 > n0
    a = K.kkt_solve_device(st, t, K.H_DIAG, 1, layout=1)
    ws = torch.empty(n1, dtype=torch.uint8, device="cuda")
    b = K.kkt_solve_device(st, t, K.H_DIAG, 1, workspace=ws, layout=1)
    torch.cuda.synchronize()
    assert torch.equal(a["dz"], b["dz"]) and torch.equal(a["lam"], b["lam"])
    with pytest.raises(lqrx.LqrxError) as e:
        K.kkt_solve_device(st, t, K.H_DIAG, 1, workspace=ws[: n1 - 256], layout=1)
    assert e.value.code == -10
