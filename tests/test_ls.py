"""Condensed least-squares LQR and the sparse KKT formulation.

CPU (oracle pinning):
  * oracle/ls_oracle.py against the known answers of /root/reference/test/least_squares.jl
    (:10-12 T / L / Hx end blocks with A = 0.99 I, B = 1; :16-17 build_toeplitz ≡
    build_least_squares!; :19-24 Ā ≈ Hx·T, b̄ ≈ Hx·L·x0; :30-37 normal equations of a
    fresh solver, Hu = 0) on the DoubleIntegrator(3, 101) fixture of test/problems.jl:14-56;
  * LS with Hu = blkdiag(R) reproduces the DP oracle's rollout (the same LQR optimum);
  * the sparse restatement (sparse_solver.jl:267-292) equals the KAT-pinned block oracle.
GPU (parity through the C ABI): ls_condensed_kernel vs the oracle for every Hu mode,
buildAb!'s Ā/b̄, info codes, ragged batches; SparseSolver (block gather → kkt kernel)
vs the sparse oracle.  Tolerances are written per test: the condensed normal equations
square the conditioning, so U is compared at rel 1e-9 on problems with cond(H) ≤ 1e6
(measured in the test), Ā/b̄ at 1e-12.
"""
import numpy as np
import pytest

from oracle import ls_oracle as LO
from oracle import oracle as orc


def _di_fixture(D=3):
    """test/problems.jl:14-40 DoubleIntegrator(D, N): RK3 of the linear double integrator is
    exact, dt = (N−1)/tf = 50 as the script computes it (:18)."""
    dt = 50.0
    A = np.block([[np.eye(D), dt * np.eye(D)], [np.zeros((D, D)), np.eye(D)]])
    B = np.vstack([0.5 * dt * dt * np.eye(D), dt * np.eye(D)])
    Q = np.diag([10.0] * D + [1.0] * D)
    R = 0.1 * np.eye(D)
    return A, B, Q, R, 10 * Q, np.concatenate([np.ones(D), np.zeros(D)])


def _stable_problem(rng, n, m):
    G = rng.standard_normal((n, n))
    A = np.eye(n) + 0.1 / np.sqrt(n) * G
    A /= max(1.0, 1.02 * np.abs(np.linalg.eigvals(A)).max())
    B = rng.standard_normal((n, m)) / np.sqrt(n)
    Gq = rng.standard_normal((n, n))
    Q = np.eye(n) + Gq.T @ Gq / n
    Gr = rng.standard_normal((m, m))
    R = np.eye(m) + Gr.T @ Gr / m
    return A, B, Q, R, 10 * Q, rng.standard_normal(n)


# ------------------------------------------------------------------ CPU: oracle pinning
def test_ls_oracle_known_answers():
    A, B, Q, R, Qf, x0 = _di_fixture()
    n, m, N = 6, 3, 101
    # :8-12 with prob.A = 0.99 I, prob.B = 1
    A1, B1 = 0.99 * np.eye(n), np.ones((n, m))
    T, L = LO.build_toeplitz(A1, B1, N)
    Hx, Hu = LO.block_costs(Q, R, Qf, N)
    assert np.allclose(T[-n:, :m], np.linalg.matrix_power(A1, N - 2) @ B1, rtol=1e-12)
    assert np.allclose(L[-n:, :], np.linalg.matrix_power(A1, N - 1), rtol=1e-12)
    assert np.allclose(Hx[-n:, -n:], np.sqrt(Qf), rtol=1e-12)       # diagonal Qf
    # :16-17 build_toeplitz ≡ build_least_squares!'s T, L (same function body here)
    # :19-24 buildAb! ≡ Hx·T, Hx·L·x0
    Ab, bb = LO.buildAb(A1, B1, Q, Qf, x0, N)
    assert np.allclose(Ab, Hx @ T, rtol=1e-12, atol=1e-12 * np.abs(Ab).max())
    assert np.allclose(bb, Hx @ L @ x0, rtol=1e-12, atol=1e-12 * np.abs(bb).max())
    # :28-37 a fresh solver (Hu = 0) on the DoubleIntegrator problem: normal equations
    out = LO.ls_solve(A, B, Q, R, Qf, x0, N)
    assert out["info"] == 0
    U = out["U"].reshape(-1)
    Ab, bb = out["Ab"], out["bb"]
    res = np.abs(Ab.T @ (Ab @ U + bb)).max()
    # the script's absolute 1e-12 is stated at its own scale; ‖Āᵀb̄‖∞ = 1.5e8 here
    assert res <= 1e-11 * np.abs(Ab.T @ bb).max()
    # :lsq build: Ā, b̄ equal buildAb!'s; Hu = chol(R).U afterwards
    o2 = LO.ls_solve(A, B, Q, R, Qf, x0, 21, hu=LO.HU_CHOL_R, matbuild="lsq")
    o3 = LO.ls_solve(A, B, Q, R, Qf, x0, 21, hu=LO.HU_CHOL_R, matbuild="Ab")
    assert np.allclose(o2["Ab"], o3["Ab"], rtol=1e-12, atol=1e-12 * np.abs(o2["Ab"]).max())
    assert np.allclose(o2["U"], o3["U"], rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("n,m,N", [(4, 1, 101), (3, 2, 30), (6, 3, 12)])
def test_ls_oracle_equals_dp(n, m, N):
    """LS with Hu = blkdiag(R) minimises the DP cost: same U, X as the DP oracle."""
    rng = np.random.default_rng(100 + n)
    A, B, Q, R, Qf, x0 = _stable_problem(rng, n, m)
    o = LO.ls_solve(A, B, Q, R, Qf, x0, N, hu=LO.HU_R)
    d = dict(n=n, m=m, batch=1, A=A.T.reshape(-1), B=B.T.reshape(-1), Q=Q.T.reshape(-1),
             R=R.T.reshape(-1), Qf=Qf.T.reshape(-1), x0=x0)
    ref = orc.dp_solve_abi(d, N)
    Ud = ref["U"].reshape(N - 1, m)
    assert np.abs(o["U"] - Ud).max() <= 1e-10 * np.abs(Ud).max()
    assert np.abs(o["X"] - ref["X"].reshape(N, n)).max() <= 1e-10 * np.abs(o["X"]).max()


@pytest.mark.parametrize("name", ["dubins", "di_small"])
@pytest.mark.parametrize("h_mode", [0, 2])
def test_sparse_oracle_equals_block_oracle(lqrx, name, h_mode):
    import lqrx.kkt as K

    st = {"dubins": K.dubins_structure(21), "di_small": K.double_integrator_structure(2, 12)}[name]
    pb = K.random_kkt(st, 1, seed=5 + h_mode, h_mode=h_mode)
    D, d, G, g = LO.blocks_to_global(st, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode)
    sp_ = LO.sparse_solve(D, d, G, g)
    ost = orc.KktStructure(st.n, st.m, st.N, st.p)
    blk = orc.kkt_solve_one(ost, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=h_mode)
    assert np.abs(sp_["dz"] - blk["dz"]).max() <= 1e-10 * np.abs(blk["dz"]).max()
    assert np.abs(sp_["lam"] - blk["lam"]).max() <= 1e-10 * np.abs(blk["lam"]).max()
    soc = LO.sparse_soc(D, d)
    bsoc = orc.kkt_solve_one(ost, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=h_mode, ginv=0)
    assert np.abs(soc - bsoc["dz"]).max() <= 1e-10 * np.abs(soc).max()


def test_sparse_gather_roundtrip(lqrx):
    """SparseSolver.blocks (host gather, no compute) inverts the global assembly exactly."""
    import lqrx.kkt as K

    st = K.dubins_structure(11)
    for h_mode in (0, 2):
        pb = K.random_kkt(st, 2, seed=3, h_mode=h_mode)
        glob = [LO.blocks_to_global(st, pb.Y[b], pb.y[b], pb.H[b], pb.g[b], h_mode) for b in range(2)]
        back = K.SparseSolver(st, h_mode).blocks(*[[gl[i] for gl in glob] for i in range(4)])
        for f in ("Y", "y", "H", "g"):
            assert np.array_equal(getattr(back, f), getattr(pb, f)), f


def test_ls_lds_limits(lqrx):
    """Nm = (N−1)m ≤ 192 with the problem in LDS; larger problems (up to Nm = 1024) keep H in
    global scratch (blocked factor) and need far less LDS — including the reference's own LS
    test problem, DoubleIntegrator() n=6 m=3 N=101 (test/least_squares.jl:2), Nm = 300."""
    from lqrx import ls

    assert ls.lds_bytes(4, 1, 101) <= 163840      # cartpole N=101 fits one CU
    assert ls.lds_bytes(2, 2, 97) <= 163840       # Nm = 192: the largest LDS-resident H
    assert ls.lds_bytes(6, 3, 101) <= 163840      # DoubleIntegrator(3,101): Nm = 300, global H
    assert ls.lds_bytes(4, 1, 193) <= 163840      # Nm = 192 but H would overflow LDS: global H
    ls.LeastSquaresSolver.of(lqrx.LQRProblem(*[np.eye(6)] * 3 + [np.eye(6), np.ones((6, 3)),
                                                                  np.zeros(6)], N=101))
    for n, m, N in ((2, 2, 98), (4, 1, 193), (1, 1, 1025)):
        ls.LeastSquaresSolver.of(lqrx.LQRProblem(np.eye(n), np.eye(n), np.eye(m), np.eye(n),
                                                 np.ones((n, m)), np.zeros(n), N=N))
    with pytest.raises(lqrx.LqrxError) as e:                # Nm = 1025 > 1024
        ls.LeastSquaresSolver.of(lqrx.LQRProblem(np.eye(1), np.eye(1), np.eye(1), np.eye(1),
                                                 np.ones((1, 1)), np.zeros(1), N=1026))
    assert e.value.code == lqrx._lib.ERR_UNSUPPORTED


def double_integrator_ls(N=101, D=3):
    """RobotZoo.DoubleIntegrator(D) (test/problems.jl:14-56) as the LS path sees it: exact
    discretisation of ẍ = u at dt = tf/(N−1), tf = 2; Q = diag(10·1_D, 1_D), R = 0.1·I,
    Qf = 10Q, x0 = [1_D; 0_D] (problems.jl:20-27)."""
    dt = 2.0 / (N - 1)
    I = np.eye(D)
    A = np.block([[I, dt * I], [0 * I, I]])
    B = np.vstack([0.5 * dt * dt * I, dt * I])
    Q = np.diag([10.0] * D + [1.0] * D)
    return A, B, Q, 0.1 * np.eye(D), 10 * Q, np.concatenate([np.ones(D), np.zeros(D)])


def test_ls_rejects_non_symmetric(lqrx):
    """cholesky() throws for a non-Hermitian Q/Qf/R (least_squares.jl:50-52); the kernel
    reads only upper triangles, so the host mirror checks (exactly, like ishermitian)."""
    from lqrx import ls
    from lqrx.dp import LQRBatch

    rng = np.random.default_rng(5)
    A, B, Q, R, Qf, x0 = _batch(rng, 4, 1, 3)
    Q[2, 0, 1] += 1e-3
    with pytest.raises(ValueError, match="Q of trajectory 2"):
        ls.ls_solve_batch(LQRBatch(A, B, Q, R, Qf, x0, 20))


# ------------------------------------------------------------------ GPU parity
def _batch(rng, n, m, bt):
    ps = [_stable_problem(rng, n, m) for _ in range(bt)]
    st = lambda i: np.stack([p[i] for p in ps])
    return st(0), st(1), st(2), st(3), st(4), st(5)


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,N,bt", [(4, 1, 101, 37), (3, 2, 40, 64), (6, 3, 12, 5), (2, 1, 2, 3),
                                      (8, 4, 16, 9), (16, 4, 8, 5),    # n·m + n > 64, LDS path
                                      (2, 2, 97, 4)])                  # Nm = 192: the LS cap
@pytest.mark.parametrize("hu", [0, 1, 2])
def test_ls_gpu_parity(lqrx, gpu_ok, n, m, N, bt, hu):
    from lqrx import ls
    from lqrx.dp import LQRBatch

    rng = np.random.default_rng(7 * n + m + N)
    A, B, Q, R, Qf, x0 = _batch(rng, n, m, bt)
    out = ls.ls_solve_batch(LQRBatch(A, B, Q, R, Qf, x0, N), hu_mode=hu)
    assert out["rc"] == 0 and (out["info"] == 0).all()
    for b in range(bt):
        o = LO.ls_solve(A[b], B[b], Q[b], R[b], Qf[b], x0[b], N, hu=hu)
        cond = np.linalg.cond(o["H"])
        assert cond <= 1e6, cond
        # rel 1e-9: two fp64 Cholesky solves of the same normal equations, cond(H) ≤ 1e6
        assert np.abs(out["U"][b] - o["U"]).max() <= 1e-9 * np.abs(o["U"]).max()
        assert np.abs(out["X"][b] - o["X"]).max() <= 1e-9 * np.abs(o["X"]).max()


@pytest.mark.gpu
def test_ls_gpu_buildAb_and_dp_identity(lqrx, gpu_ok):
    """Ā, b̄ as buildAb! leaves them (least_squares.jl:58-103), and LS(Hu = R) ≡ DP on the
    device (the two kernels share no code)."""
    import torch
    from lqrx import ls
    from lqrx.dp import LQRBatch, solve_batch, to_abi

    rng = np.random.default_rng(11)
    n, m, N, bt = 4, 1, 60, 16
    A, B, Q, R, Qf, x0 = _batch(rng, n, m, bt)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(to_abi(v).reshape(-1)).to(dev) for k, v in
         dict(A=A, B=B, Q=Q, R=R, Qf=Qf).items()}
    t["x0"] = torch.from_numpy(np.ascontiguousarray(x0).reshape(-1)).to(dev)
    t.update(n=n, m=m, batch=bt)
    out = ls.ls_solve_device(t, N, hu_mode=ls.HU_R, with_Ab=True)
    torch.cuda.synchronize()
    Ab = out["Ab"].cpu().numpy().reshape(bt, (N - 1) * m, N * n)
    bb = out["bb"].cpu().numpy().reshape(bt, N * n)
    for b in range(bt):
        Abr, bbr = LO.buildAb(A[b], B[b], Q[b], Qf[b], x0[b], N)
        assert np.abs(Ab[b].T - Abr).max() <= 1e-12 * np.abs(Abr).max()
        assert np.abs(bb[b] - bbr).max() <= 1e-12 * np.abs(bbr).max()
    dp = solve_batch(LQRBatch(A, B, Q, R, Qf, x0, N))
    U = out["U"].cpu().numpy().reshape(bt, N - 1, m)
    assert np.abs(U - dp["U"]).max() <= 1e-9 * np.abs(dp["U"]).max()


@pytest.mark.gpu
def test_ls_gpu_info(lqrx, gpu_ok):
    from lqrx import ls
    from lqrx.dp import LQRBatch

    rng = np.random.default_rng(3)
    n, m, N, bt = 4, 1, 20, 6
    A, B, Q, R, Qf, x0 = _batch(rng, n, m, bt)
    Q[1] = -np.eye(n)                       # cholesky(Q) throws upstream → info −1
    B[3] = 0.0                              # H = ĀᵀĀ + 0 singular → potrf pivot 1
    out = ls.ls_solve_batch(LQRBatch(A, B, Q, R, Qf, x0, N), hu_mode=ls.HU_ZERO)
    assert out["rc"] == 1
    assert out["info"][1] == -1 and out["info"][3] == 1
    ok = [0, 2, 4, 5]
    assert (out["info"][ok] == 0).all()
    for b in (1, 3):                        # failed trajectories: NaN, never stale memory
        assert np.isnan(out["U"][b]).all() and np.isnan(out["X"][b]).all()
    for b in ok:
        o = LO.ls_solve(A[b], B[b], Q[b], R[b], Qf[b], x0[b], N)
        assert np.abs(out["U"][b] - o["U"]).max() <= 1e-8 * np.abs(o["U"]).max()


@pytest.mark.gpu
def test_ls_gpu_solver_surface(lqrx, gpu_ok):
    """LeastSquaresSolver state: :Ab on a fresh solver (Hu = 0), then :lsq (Hu = chol(R).U),
    which persists for the next :Ab solve (least_squares.jl:44, :121, :158-172)."""
    from lqrx import ls

    rng = np.random.default_rng(5)
    A, B, Q, R, Qf, x0 = _stable_problem(rng, 4, 1)
    prob = lqrx.LQRProblem(Qf, Q, R, A, B, x0, N=51)
    solver = ls.LeastSquaresSolver.of(prob)
    sol = ls.Primals.of(prob)
    ls.ls_solve(sol, solver, prob)
    o0 = LO.ls_solve(A, B, Q, R, Qf, x0, 51, hu=LO.HU_ZERO)
    assert np.abs(sol.U - o0["U"]).max() <= 1e-9 * np.abs(o0["U"]).max()
    solver.opts["matbuild"] = "lsq"
    ls.ls_solve(sol, solver, prob)
    solver.opts["matbuild"] = "Ab"
    ls.ls_solve(sol, solver, prob)
    o1 = LO.ls_solve(A, B, Q, R, Qf, x0, 51, hu=LO.HU_CHOL_R)
    assert solver.hu_mode == ls.HU_CHOL_R
    assert np.abs(sol.U - o1["U"]).max() <= 1e-9 * np.abs(o1["U"]).max()
    assert sol.Z.shape == (51 * 4 + 50,)
    solver.opts["solve_type"] = "naive"
    with pytest.raises(ValueError):
        ls.ls_solve(sol, solver, prob)


@pytest.mark.gpu
@pytest.mark.parametrize("name,h_mode", [("dubins", 2), ("dubins", 0), ("di_small", 1), ("di", 2)])
def test_sparse_solver_gpu(lqrx, gpu_ok, name, h_mode):
    """("di", 2) is test/sparse_solver.jl's own problem structure, DoubleIntegrator(3, 101)
    with diagonal costs (dense_cost=false)."""
    import lqrx.kkt as K

    st = {"dubins": K.dubins_structure(31), "di_small": K.double_integrator_structure(2, 12),
          "di": K.double_integrator_structure(3, 101)}[name]
    bt = 4
    pb = K.random_kkt(st, bt, seed=21, h_mode=h_mode)
    glob = [LO.blocks_to_global(st, pb.Y[b], pb.y[b], pb.H[b], pb.g[b], h_mode) for b in range(bt)]
    D, d, G, g = ([gl[i] for gl in glob] for i in range(4))
    solver = K.SparseSolver(st, h_mode)
    out = solver.solve(D, d, G, g)
    soc = solver.second_order_correction(D, d)
    assert out["rc"] == 0
    for b in range(bt):
        ref = LO.sparse_solve(D[b], d[b], G[b], g[b])
        assert np.abs(out["dz"][b] - ref["dz"]).max() <= 1e-10 * np.abs(ref["dz"]).max()
        assert np.abs(out["lam"][b] - ref["lam"]).max() <= 1e-10 * np.abs(ref["lam"]).max()
        rs = LO.sparse_soc(D[b], d[b])
        assert np.abs(soc["dz"][b] - rs).max() <= 1e-10 * np.abs(rs).max()


@pytest.mark.gpu
@pytest.mark.parametrize("hu", [0, 1, 2])
def test_ls_gpu_reference_double_integrator(lqrx, gpu_ok, hu):
    """The reference's own LS test problem (test/least_squares.jl:29-38: DoubleIntegrator(),
    n=6 m=3 N=101, Nm = 300 — the global-H blocked path): U, X against the numpy oracle, and
    the optimality condition that test asserts, ‖Āᵀ(ĀU + b̄) + Hu·U‖∞ < 1e-12 (scaled)."""
    import torch
    from lqrx import ls
    from lqrx.dp import to_abi

    A, B, Q, R, Qf, x0 = double_integrator_ls()
    n, m, N, bt = 6, 3, 101, 6
    rng = np.random.default_rng(4)
    X0 = x0[None] + 0.1 * rng.standard_normal((bt, n))
    st = lambda M: np.repeat(M[None], bt, axis=0)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(to_abi(st(v)).reshape(-1)).to(dev) for k, v in dict(A=A, B=B, Q=Q, R=R, Qf=Qf).items()}
    t["x0"] = torch.from_numpy(np.ascontiguousarray(X0).reshape(-1)).to(dev)
    t.update(n=n, m=m, batch=bt)
    out = ls.ls_solve_device(t, N, hu_mode=hu, with_Ab=True)
    torch.cuda.synchronize()
    assert int((out["info"] != 0).sum()) == 0
    U = out["U"].cpu().numpy().reshape(bt, (N - 1) * m)
    X = out["X"].cpu().numpy().reshape(bt, N, n)
    Ab = out["Ab"].cpu().numpy().reshape(bt, (N - 1) * m, N * n)
    bb = out["bb"].cpu().numpy().reshape(bt, N * n)
    for b in range(bt):
        o = LO.ls_solve(A, B, Q, R, Qf, X0[b], N, hu=hu)
        assert np.linalg.cond(o["H"]) <= 1e6
        assert np.abs(U[b] - o["U"].ravel()).max() <= 1e-9 * np.abs(o["U"]).max()
        assert np.abs(X[b] - o["X"]).max() <= 1e-9 * np.abs(o["X"]).max()
        Abar = Ab[b].T
        Hu = np.kron(np.eye(N - 1), {0: np.zeros((m, m)), 1: np.linalg.cholesky(R).T, 2: R}[hu])
        res = Abar.T @ (Abar @ U[b] + bb[b]) + Hu @ U[b]
        scale = np.abs(Abar.T @ Abar).max() * np.abs(U[b]).max()
        assert np.abs(res).max() <= 1e-12 * max(1.0, scale)


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,N,bt", [(4, 1, 193, 3), (2, 2, 98, 5), (3, 2, 150, 2), (2, 1, 400, 2)])
def test_ls_gpu_big_path_parity(lqrx, gpu_ok, n, m, N, bt):
    """Problems past the LDS-resident kernel (Nm > 192 or H > LDS): global H, blocked factor."""
    from lqrx import ls
    from lqrx.dp import LQRBatch

    rng = np.random.default_rng(3 * n + m + N)
    A, B, Q, R, Qf, x0 = _batch(rng, n, m, bt)
    out = ls.ls_solve_batch(LQRBatch(A, B, Q, R, Qf, x0, N), hu_mode=2)
    assert out["rc"] == 0 and (out["info"] == 0).all()
    for b in range(bt):
        o = LO.ls_solve(A[b], B[b], Q[b], R[b], Qf[b], x0[b], N, hu=2)
        cond = np.linalg.cond(o["H"])
        tol = 1e-9 if cond <= 1e6 else 1e-15 * cond * 10
        assert np.abs(out["U"][b] - o["U"]).max() <= tol * np.abs(o["U"]).max(), cond
        assert np.abs(out["X"][b] - o["X"]).max() <= tol * np.abs(o["X"]).max(), cond


@pytest.mark.gpu
def test_ls_gpu_big_path_info(lqrx, gpu_ok):
    from lqrx import ls
    from lqrx.dp import LQRBatch

    rng = np.random.default_rng(9)
    n, m, N, bt = 3, 2, 120, 4
    A, B, Q, R, Qf, x0 = _batch(rng, n, m, bt)
    Q[1] = -np.eye(n)
    B[2] = 0.0
    out = ls.ls_solve_batch(LQRBatch(A, B, Q, R, Qf, x0, N), hu_mode=ls.HU_ZERO)
    assert out["rc"] == 1 and out["info"][1] == -1 and out["info"][2] == 1
    assert out["info"][0] == 0 and out["info"][3] == 0
    for b in (1, 2):
        assert np.isnan(out["U"][b]).all() and np.isnan(out["X"][b]).all()
