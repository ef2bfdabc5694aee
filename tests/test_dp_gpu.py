"""GPU parity: batched Riccati kernel (liblqrx.so, via the C ABI) vs the CPU oracle.

Oracle = oracle/lqr_oracle.c, restating /root/reference/src/dynamic_programming.jl:28-72.
Tolerance (north star): max|K − K_ref| / max|K_ref| ≤ 1e-10 per knot in fp64, same for P
(and X, U); fp32 runs are held to 1e-4 against the fp64 oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL64 = 1e-10
TOL32 = 1e-4


def relerr_per_knot(a, b):
    """max over knots of max|a−b| / max|b| (leading axes: batch, knot)."""
    a = a.reshape(a.shape[0], a.shape[1], -1)
    b = b.reshape(b.shape[0], b.shape[1], -1)
    num = np.abs(a - b).max(axis=2)
    den = np.abs(b).max(axis=2)
    den[den == 0] = 1.0
    return float((num / den).max())


def run_pair(lqrx, oracle, n, m, N, batch, seed, dtype=0, all_P=True):
    from lqrx.dp import abi_to_batch

    d = lqrx.random_batch(n, m, N, batch, seed)
    b = abi_to_batch(d)
    got = lqrx.solve_batch(b, dtype=dtype, all_P=all_P)
    ref = oracle.dp_solve_abi(d, N, all_P=all_P)
    from lqrx.dp import from_abi

    refK = from_abi(ref["K"], (batch, N - 1, m, n))
    refP = from_abi(ref["P"], (batch, N, n, n) if all_P else (batch, n, n))
    refX = ref["X"].reshape(batch, N, n)
    refU = ref["U"].reshape(batch, N - 1, m)
    return got, dict(K=refK, P=refP, X=refX, U=refU, info=ref["info"])


@pytest.mark.parametrize("n,m,N,batch", [
    (4, 1, 101, 64),      # cartpole-sized (cfg1/cfg2 shape)
    (6, 3, 30, 37),       # DoubleIntegrator(3) shape, ragged batch
    (16, 16, 12, 5),      # exact single tiles
    (17, 5, 9, 3),        # padded 2×1 tiles
    (32, 16, 16, 8),      # cfg4 shape, short horizon
    (32, 16, 256, 4),     # cfg4 shape, full horizon
    (32, 32, 20, 3),      # 2×2 tiles
    (64, 32, 12, 2),      # cfg5 shape (4×2 tiles), fp64
    (48, 20, 9, 3),       # padded 3×2 → 4×2 tiles
])
def test_dp_parity_f64(lqrx, oracle, gpu_ok, n, m, N, batch):
    got, ref = run_pair(lqrx, oracle, n, m, N, batch, seed=1000 + n * 7 + m)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert relerr_per_knot(got["K"], ref["K"]) <= TOL64
    P = got["P"]
    assert relerr_per_knot(P, ref["P"]) <= TOL64
    assert relerr_per_knot(got["X"][:, :, None], ref["X"][:, :, None]) <= TOL64 or \
        np.abs(got["X"] - ref["X"]).max() <= TOL64 * max(1.0, np.abs(ref["X"]).max())
    assert np.abs(got["U"] - ref["U"]).max() <= TOL64 * max(1.0, np.abs(ref["U"]).max())


@pytest.mark.parametrize("n,m,N,batch,all_P", [
    (64, 32, 40, 5, True),     # dp_wg4_kernel<double, 2>: four waves per trajectory
    (64, 16, 30, 3, True),     # dp_wg4_kernel<double, 1>
    (64, 32, 150, 2, False),   # long horizon (warm-started inverse), P_1 only
])
def test_dp_wg4_parity_f64(lqrx, oracle, gpu_ok, n, m, N, batch, all_P):
    """fp64 n = 64 runs on the four-wave kernel (lqrx_dp.hip dp_wg4_kernel)."""
    got, ref = run_pair(lqrx, oracle, n, m, N, batch, seed=4000 + N, all_P=all_P)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert relerr_per_knot(got["K"], ref["K"]) <= TOL64
    P = got["P"] if all_P else got["P"][:, None]
    assert relerr_per_knot(P, ref["P"] if all_P else ref["P"][:, None]) <= TOL64
    assert np.abs(got["X"] - ref["X"]).max() <= TOL64 * max(1.0, np.abs(ref["X"]).max())
    assert np.abs(got["U"] - ref["U"]).max() <= TOL64 * max(1.0, np.abs(ref["U"]).max())


def test_dp_wg4_matches_one_wave(lqrx, gpu_ok):
    """The four-wave and the one-wave kernel (LQRX_DP_WG4=0) agree to rounding on n=64."""
    import subprocess
    import sys
    import os
    code = ("import numpy as np, lqrx; from lqrx.dp import abi_to_batch; "
            "d = lqrx.random_batch(64, 32, 24, 3, seed=9); "
            "g = lqrx.solve_batch(abi_to_batch(d), all_P=True); "
            "np.save(__import__('sys').argv[1], np.concatenate([g['K'].ravel(), g['P'].ravel()]))")
    outs = []
    for flag in ("1", "0"):
        f = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"wg4_{flag}_{os.getpid()}.npy")
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env = dict(os.environ, LQRX_DP_WG4=flag,
                   PYTHONPATH=os.pathsep.join([os.path.join(root, "lqr.jl_amd"), os.environ.get("PYTHONPATH", "")]))
        subprocess.run([sys.executable, "-c", code, f], env=env, check=True, timeout=120)
        outs.append(np.load(f))
        os.remove(f)
    a, b = outs
    assert np.abs(a - b).max() <= 1e-11 * np.abs(b).max()


def test_dp_wg4_non_spd_sets_info(lqrx, gpu_ok):
    from lqrx.dp import abi_to_batch

    n, m, N, bt = 64, 32, 8, 3
    d = lqrx.random_batch(n, m, N, bt, seed=13)
    b = abi_to_batch(d)
    b.R[1] = -100.0 * np.eye(m)
    b.B[1] *= 1e-3
    got = lqrx.solve_batch(b)
    assert got["rc"] == 1
    assert got["info"][1] == N - 1
    assert got["info"][0] == 0 and got["info"][2] == 0


def test_dp_p1_only(lqrx, oracle, gpu_ok):
    """p_mode 0 returns P_1 = solver.P after solve! (dynamic_programming.jl:63)."""
    got, ref = run_pair(lqrx, oracle, 32, 16, 40, 6, seed=5, all_P=False)
    assert relerr_per_knot(got["P"][:, None], ref["P"][:, None]) <= TOL64


@pytest.mark.parametrize("n,m,N,batch", [(32, 16, 64, 4), (4, 1, 101, 16), (64, 32, 40, 3)])
def test_dp_parity_f32(lqrx, oracle, gpu_ok, n, m, N, batch):
    got, ref = run_pair(lqrx, oracle, n, m, N, batch, seed=77, dtype=1)
    assert relerr_per_knot(got["K"].astype(np.float64), ref["K"]) <= TOL32
    assert relerr_per_knot(got["P"].astype(np.float64), ref["P"]) <= TOL32


def test_dp_non_spd_sets_info(lqrx, oracle, gpu_ok):
    """A non-SPD R makes E = R + BᵀPB indefinite at the first backward knot: the kernel
    reports it per trajectory (the reference discards potrf's info)."""
    from lqrx.dp import abi_to_batch

    n, m, N, bt = 6, 3, 10, 4
    d = lqrx.random_batch(n, m, N, bt, seed=3)
    b = abi_to_batch(d)
    b.R[1] = -100.0 * np.eye(m)      # trajectory 1 is broken
    b.B[1] *= 1e-3
    got = lqrx.solve_batch(b)
    assert got["rc"] == 1
    assert got["info"][1] == N - 1
    assert got["info"][0] == 0 and got["info"][2] == 0 and got["info"][3] == 0


def test_dp_deterministic(lqrx, gpu_ok):
    from lqrx.dp import abi_to_batch

    d = lqrx.random_batch(32, 16, 32, 16, seed=11)
    b = abi_to_batch(d)
    a1 = lqrx.solve_batch(b)
    a2 = lqrx.solve_batch(b)
    assert np.array_equal(a1["K"], a2["K"]) and np.array_equal(a1["X"], a2["X"])


def test_reference_call_shape_diagonal_costs(lqrx, oracle, gpu_ok):
    """The reference's own call sequence (test/dp.jl:14-20) through the C ABI:
    sol = LQRSolution(prob); solver = DPSolver(prob); solve!(sol, solver, prob) — here
    LQRSolution.of / DPSolver.of / lqrx.solve — with LQRProblem's Q, Qf, R given as
    Diagonal (lqr_problem.jl:1-4 allows TQ, TR = Diagonal; test/problems.jl builds them that
    way), densified on the way into the ABI.  sol.K[k] is knot k's m×n gain."""
    from lqrx.dp import from_abi, to_abi

    n, m, N, dt = 4, 2, 51, 0.1                    # DoubleIntegrator(2) (test/problems.jl:14-56)
    I2 = np.eye(2)
    A = np.block([[I2, dt * I2], [0 * I2, I2]])
    B = np.vstack([0.5 * dt * dt * I2, dt * I2])
    q = np.array([10.0, 10.0, 1.0, 1.0])
    prob = lqrx.LQRProblem(Qf=10 * q, Q=q, R=np.full(m, 0.1), A=A, B=B, x0=np.array([1.0, -1, 0, 0.5]),
                           u0=np.zeros(m), tf=5.0, N=N)
    sol = lqrx.LQRSolution.of(prob)
    solver = lqrx.DPSolver.of(prob)
    lqrx.solve(sol, solver, prob)
    d = dict(A=to_abi(A[None]).ravel(), B=to_abi(B[None]).ravel(), Q=to_abi(np.diag(q)[None]).ravel(),
             R=to_abi(np.diag(np.full(m, 0.1))[None]).ravel(), Qf=to_abi(np.diag(10 * q)[None]).ravel(),
             x0=prob.x0.copy(), n=n, m=m, N=N, batch=1)
    ref = oracle.dp_solve_abi(d, N)
    K = from_abi(ref["K"], (1, N - 1, m, n))[0]
    assert sol.info == 0
    for k in (0, N // 2, N - 2):
        assert sol.K[k].shape == (m, n)
        assert np.abs(sol.K[k] - K[k]).max() <= TOL64 * np.abs(K[k]).max()
    assert np.abs(sol.X - ref["X"].reshape(N, n)).max() <= TOL64 * np.abs(ref["X"]).max()
    assert np.abs(sol.P - from_abi(ref["P"], (1, n, n))[0]).max() <= TOL64 * np.abs(ref["P"]).max()


@pytest.mark.parametrize("n,m,bt", [(4, 2, 5), (3, 1, 70), (12, 5, 9), (32, 16, 3), (80, 40, 2)])
def test_per_knot_compute_gain_ctg(lqrx, gpu_ok, n, m, bt):
    """The reference's per-knot surface (test/dp.jl:16-17): compute_gain!(K, solver, prob) and
    compute_ctg!(K, solver, prob) (dynamic_programming.jl:34-52) through lqrx_dp_compute_ctg —
    from solver.P = 0 (a fresh solver, as the test calls them) and from a random SPD P, batched
    over every kernel family (n ≤ 4, register tiles, workgroup) — against the formulas in fp64
    numpy: K = (R + BᵀPB)⁻¹BᵀPA, P_ = Q + AᵀPA − AᵀPB·K."""
    from lqrx.dp import abi_to_batch, compute_ctg_batch

    b = abi_to_batch(lqrx.random_batch(n, m, 3, bt, seed=5 + n))
    rng = np.random.default_rng(n)
    G = rng.standard_normal((bt, n, n))
    for P in (np.zeros((bt, n, n)), G @ np.swapaxes(G, 1, 2) / n + np.eye(n)):
        out = compute_ctg_batch(b.A, b.B, b.Q, b.R, P)
        assert out["rc"] == 0 and (out["info"] == 0).all()
        PB, PA = P @ b.B, P @ b.A
        E = b.R + np.swapaxes(b.B, 1, 2) @ PB
        K = np.linalg.solve(E, np.swapaxes(b.B, 1, 2) @ PA)
        Pn = b.Q + np.swapaxes(b.A, 1, 2) @ PA - np.swapaxes(b.A, 1, 2) @ PB @ K
        assert np.abs(out["K"] - K).max() <= 1e-10 * max(1.0, np.abs(K).max())
        assert np.abs(out["P_"] - Pn).max() <= 1e-10 * max(1.0, np.abs(Pn).max())
        g = compute_ctg_batch(b.A, b.B, b.Q, b.R, P, gain_only=True)
        assert g["P_"] is None and np.array_equal(g["K"], out["K"])


def test_per_knot_reference_call_shape(lqrx, gpu_ok):
    """test/dp.jl:14-17 verbatim in shape: sol = LQRSolution(prob); solver = DPSolver(prob);
    compute_gain!(sol.K[1], solver, prob); compute_ctg!(sol.K[1], solver, prob) — on a fresh
    solver (P = 0) the gain is 0 and P_ = Q; with solver.P = Qf it is solve!'s last knot."""
    n, m, N, dt = 4, 2, 11, 0.1
    I2 = np.eye(2)
    A = np.block([[I2, dt * I2], [0 * I2, I2]])
    B = np.vstack([0.5 * dt * dt * I2, dt * I2])
    q = np.array([10.0, 10.0, 1.0, 1.0])
    prob = lqrx.LQRProblem(Qf=10 * q, Q=q, R=np.full(m, 0.1), A=A, B=B, x0=np.array([1.0, -1, 0, 0.5]),
                           u0=np.zeros(m), tf=1.0, N=N)
    sol = lqrx.LQRSolution.of(prob)
    solver = lqrx.DPSolver.of(prob)
    lqrx.compute_gain(sol.K[0], solver, prob)
    assert np.abs(sol.K[0]).max() == 0.0
    lqrx.compute_ctg(sol.K[0], solver, prob)
    assert np.abs(solver.P_ - np.diag(q)).max() <= 1e-14
    solver.P[...] = np.diag(10 * q)
    lqrx.compute_ctg(sol.K[0], solver, prob)
    full = lqrx.LQRSolution.of(prob)
    lqrx.solve(full, lqrx.DPSolver.of(prob), prob)
    assert np.abs(sol.K[0] - full.K[N - 2]).max() <= 1e-12 * np.abs(full.K[N - 2]).max()


def test_gpu_run_uses_library_built_from_tree(lqrx, gpu_ok):
    """On the GPU box: the library these GPU tests load was built from the sources shipped
    with them (lqrx_build_info's source hash = the tree's; see tests/test_abi.py)."""
    from lqrx import _lib

    b = _lib.build_info()
    print(b["info"])
    assert b["matches_tree"], b
