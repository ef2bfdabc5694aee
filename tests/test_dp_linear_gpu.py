"""GPU parity: DP with linear cost terms (lqrx_dp_solve_linear) vs the CPU oracle.

SURVEY §8(f) rank 1 ("time-varying LQR … and cost linear terms").  The reference
LQRProblem has no linear terms; the oracle (oracle/lqr_oracle.c oracle_dp_solve_one_lin)
extends dynamic_programming.jl:28-72 in its own op order — d is one more potrs column of
chol_solve! (:42), p follows :51 — and is pinned against the dense QP optimum and its
costates (tests/test_oracle.py::test_dp_oracle_linear_equals_dense_kkt).
Tolerance as the plain DP: 1e-10 relative per knot in fp64 for K and P; d and p are
vectors that change sign along the horizon (a knot's max|d_k| can be ~0 for m = 1), so
they are held to 1e-10 relative to their trajectory's max (X, U likewise); fp32 1e-4.
Kernels: n ≤ 4 dp_lane_kernel<…, LIN>, n ≥ 5 dp_riccati_kernel<…, VAR_TV | VAR_LIN>.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL64 = 1e-10
TOL32 = 1e-4


def relerr_per_knot(a, b):
    a = a.reshape(a.shape[0], a.shape[1], -1)
    b = b.reshape(b.shape[0], b.shape[1], -1)
    num = np.abs(a - b).max(axis=2)
    den = np.abs(b).max(axis=2)
    den[den == 0] = 1.0
    return float((num / den).max())


def lin_problem(lqrx, n, m, N, bt, seed, tv_QR=False, tv_AB=False):
    """random_batch + linear terms (flat ABI arrays) and, with tv_*, per-knot fields."""
    from lqrx.dp import from_abi, to_abi

    d = lqrx.random_batch(n, m, N, bt, seed)
    rng = np.random.default_rng(seed + 7)
    kq = N - 1 if tv_QR else 1
    d["q"] = rng.standard_normal(bt * kq * n)
    d["r"] = rng.standard_normal(bt * kq * m)
    d["qf"] = rng.standard_normal(bt * n)
    if tv_QR:
        s = 1.0 + 0.5 * rng.random((bt, N - 1, 1, 1))
        Q = from_abi(d["Q"], (bt, n, n))[:, None] * s
        R = from_abi(d["R"], (bt, m, m))[:, None] * s
        d["Q"] = to_abi(Q.reshape(-1, n, n)).ravel()
        d["R"] = to_abi(R.reshape(-1, m, m)).ravel()
        d["tv_QR"] = 1
    if tv_AB:
        A = from_abi(d["A"], (bt, n, n))[:, None] + 0.02 * rng.standard_normal((bt, N - 1, n, n))
        B = from_abi(d["B"], (bt, n, m))[:, None] * (1.0 + 0.1 * rng.random((bt, N - 1, 1, 1)))
        d["A"] = to_abi(A.reshape(-1, n, n)).ravel()
        d["B"] = to_abi(B.reshape(-1, n, m)).ravel()
        d["tv_AB"] = 1
    return d


def to_batch(d, N):
    from lqrx.dp import LQRBatch, from_abi

    n, m, bt = d["n"], d["m"], d["batch"]
    kab = N - 1 if d.get("tv_AB") else 1
    kq = N - 1 if d.get("tv_QR") else 1
    sh = lambda a, r, c, k: from_abi(a, (bt, k, r, c)) if k > 1 else from_abi(a, (bt, r, c))
    vec = lambda a, w, k: a.reshape(bt, k, w) if k > 1 else a.reshape(bt, w)
    return LQRBatch(sh(d["A"], n, n, kab), sh(d["B"], n, m, kab), sh(d["Q"], n, n, kq),
                    sh(d["R"], m, m, kq), from_abi(d["Qf"], (bt, n, n)), d["x0"].reshape(bt, n), N,
                    q=vec(d["q"], n, kq), r=vec(d["r"], m, kq), qf=d["qf"].reshape(bt, n))


def relerr_traj(a, b):
    """max over trajectories of max|a−b| / max|b| over the whole trajectory."""
    a = a.reshape(a.shape[0], -1)
    b = b.reshape(b.shape[0], -1)
    den = np.abs(b).max(axis=1)
    den[den == 0] = 1.0
    return float((np.abs(a - b).max(axis=1) / den).max())


def check(got, ref, n, m, N, bt, all_P, tol):
    from lqrx.dp import from_abi

    assert (got["info"] == 0).all() and (ref["info"] == 0).all()
    assert relerr_per_knot(got["K"], from_abi(ref["K"], (bt, N - 1, m, n))) <= tol
    assert relerr_traj(got["d"], ref["d"].reshape(bt, N - 1, m)) <= tol
    if all_P:
        assert relerr_per_knot(got["P"], from_abi(ref["P"], (bt, N, n, n))) <= tol
        assert relerr_traj(got["p"], ref["p"].reshape(bt, N, n)) <= tol
    else:
        assert relerr_per_knot(got["P"][:, None], from_abi(ref["P"], (bt, 1, n, n))) <= tol
        assert relerr_traj(got["p"], ref["p"].reshape(bt, n)) <= tol
    for k, w in (("X", n), ("U", m)):
        r = ref[k].reshape(got[k].shape)
        assert np.abs(got[k] - r).max() <= tol * max(1.0, np.abs(r).max()), k


@pytest.mark.parametrize("n,m,N,bt,tvq,tvab,all_P", [
    (4, 1, 101, 67, False, False, True),    # cartpole shape, lane kernel (quad is skipped)
    (3, 2, 40, 9, True, False, True),       # Dubins shape, per-knot Q, R, q, r
    (2, 2, 30, 5, True, True, False),       # fully time-varying, p_1 only
    (6, 3, 30, 7, False, False, True),      # MFMA 1×1 tiles (DoubleIntegrator(3) shape)
    (17, 5, 12, 3, True, True, True),       # padded 2×1 tiles, time-varying
    (32, 16, 64, 4, False, False, True),    # cfg4 shape
    (32, 16, 256, 3, True, False, False),   # cfg4 shape, full horizon, per-knot q, r
    (64, 32, 12, 2, False, False, True),    # cfg5 shape (4×2 tiles), fp64
])
def test_dp_linear_parity_f64(lqrx, oracle, gpu_ok, n, m, N, bt, tvq, tvab, all_P):
    d = lin_problem(lqrx, n, m, N, bt, 3100 + 11 * n + m, tvq, tvab)
    got = lqrx.solve_batch(to_batch(d, N), all_P=all_P)
    assert got["rc"] == 0
    ref = oracle.dp_solve_lin_abi(d, N, all_P=all_P)
    check(got, ref, n, m, N, bt, all_P, TOL64)


@pytest.mark.parametrize("n,m,N,bt", [(4, 2, 50, 70), (32, 16, 40, 3), (64, 32, 14, 2)])   # 64: four-wave TV + LIN
def test_dp_linear_layout1(lqrx, oracle, gpu_ok, n, m, N, bt):
    """Layout 1 (SoA) for the linear arrays too: bit-identical to layout 0."""
    d = lin_problem(lqrx, n, m, N, bt, 77 + n, tv_QR=True)
    b = to_batch(d, N)
    a0 = lqrx.solve_batch(b, all_P=True, layout=0)
    a1 = lqrx.solve_batch(b, all_P=True, layout=1)
    for k in ("K", "P", "X", "U", "d", "p", "info"):
        assert np.array_equal(a0[k], a1[k]), k


# fp32 lane shapes are fully/well actuated: at n = 4, m = 1 the §8(d) generator's weakly
# actuated trajectories amplify rounding (tests/test_dp_lane_gpu.py) and the plain fp32
# kernel itself is far from the fp64 oracle there
@pytest.mark.parametrize("n,m,N,bt", [(4, 4, 101, 40), (3, 2, 60, 40), (32, 16, 64, 3), (64, 32, 30, 2)])
def test_dp_linear_parity_f32(lqrx, oracle, gpu_ok, n, m, N, bt):
    d = lin_problem(lqrx, n, m, N, bt, 500 + n)
    got = lqrx.solve_batch(to_batch(d, N), dtype=1, all_P=True)
    ref = oracle.dp_solve_lin_abi(d, N, all_P=True)
    check(got, ref, n, m, N, bt, True, TOL32)


@pytest.mark.parametrize("n,m", [(4, 1), (32, 16)])
def test_dp_linear_zero_terms_equal_plain(lqrx, gpu_ok, n, m):
    """q = r = qf = 0: K, P, X, U equal the plain lqrx_dp_solve within 1e-11 (different
    kernel instantiation — for n ≤ 4 the quad kernel's column form) and d = p = 0 exactly."""
    N, bt = 40, 6
    d = lin_problem(lqrx, n, m, N, bt, 9)
    for k in ("q", "r", "qf"):
        d[k] = np.zeros_like(d[k])
    b = to_batch(d, N)
    a = lqrx.solve_batch(b, all_P=True)
    b.q = b.r = b.qf = None
    c = lqrx.solve_batch(b, all_P=True)
    for k in ("K", "P", "X", "U"):
        assert np.abs(a[k] - c[k]).max() <= 1e-11 * max(1.0, np.abs(c[k]).max()), k
    assert not a["d"].any() and not a["p"].any()


def test_dp_linear_device_stream(lqrx, oracle, gpu_ok):
    """Device-pointer entry point on a created stream (what bench.py and a Julia ccall with
    CuArrays use), compared to the oracle."""
    import torch

    n, m, N, bt = 32, 16, 48, 5
    d = lin_problem(lqrx, n, m, N, bt, 123)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(np.asarray(d[k])).to(dev) for k in ("A", "B", "Q", "R", "Qf", "x0", "q", "r", "qf")}
    t.update(n=n, m=m, batch=bt)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        out = lqrx.dp_solve_device(t, N, p_mode=1, stream=s.cuda_stream)
    s.synchronize()
    from lqrx.dp import from_abi
    got = dict(K=from_abi(out["K"].cpu().numpy(), (bt, N - 1, m, n)),
               P=from_abi(out["P"].cpu().numpy(), (bt, N, n, n)),
               X=out["X"].cpu().numpy().reshape(bt, N, n), U=out["U"].cpu().numpy().reshape(bt, N - 1, m),
               d=out["d"].cpu().numpy().reshape(bt, N - 1, m), p=out["p"].cpu().numpy().reshape(bt, N, n),
               info=out["info"].cpu().numpy())
    ref = oracle.dp_solve_lin_abi(d, N, all_P=True)
    check(got, ref, n, m, N, bt, True, TOL64)


@pytest.mark.parametrize("small", ["lane", "quad"])
@pytest.mark.parametrize("n,m,N,bt,tvq", [(4, 1, 101, 67, False), (3, 2, 60, 33, False),
                                          (4, 4, 40, 20, False), (4, 2, 50, 19, True)])
def test_dp_linear_small_kernels(lqrx, oracle, gpu_ok, monkeypatch, small, n, m, N, bt, tvq):
    """Both n ≤ 4 kernels with linear terms (LQRX_DP_SMALL forces the choice; time-varying
    problems always take the lane kernel)."""
    monkeypatch.setenv("LQRX_DP_SMALL", small)
    d = lin_problem(lqrx, n, m, N, bt, 900 + n * 5 + m, tv_QR=tvq)
    for all_P in (True, False):
        got = lqrx.solve_batch(to_batch(d, N), all_P=all_P)
        ref = oracle.dp_solve_lin_abi(d, N, all_P=all_P)
        check(got, ref, n, m, N, bt, all_P, TOL64)


@pytest.mark.parametrize("n,m,N,bt,tvq", [(4, 1, 2, 1, False), (32, 16, 2, 3, True), (6, 2, 3, 65, False),
                                          (3, 1, 5, 130, True), (64, 32, 2, 1, False)])
def test_dp_linear_edge_shapes(lqrx, oracle, gpu_ok, n, m, N, bt, tvq):
    """Shortest horizons (N = 2: one backward knot), single trajectories and ragged waves."""
    d = lin_problem(lqrx, n, m, N, bt, 4400 + 7 * n + N, tv_QR=tvq)
    for all_P in (True, False):
        got = lqrx.solve_batch(to_batch(d, N), all_P=all_P)
        ref = oracle.dp_solve_lin_abi(d, N, all_P=all_P)
        check(got, ref, n, m, N, bt, all_P, TOL64)


def test_dp_linear_empty_batch(lqrx, gpu_ok):
    """batch = 0 is a valid no-op, as for lqrx_dp_solve."""
    import ctypes as C
    from lqrx import _lib

    d = _lib.DpDesc(8, 4, 10, 0, 0, 0, 0, 0, 0)
    ln = _lib.DpLinear(None, None, None, None, None)
    assert lqrx.load().lqrx_dp_solve_linear(C.byref(d), *([None] * 6), C.byref(ln), *([None] * 4), None, None) == 0


def test_dp_linear_single_problem_api(lqrx, oracle, gpu_ok):
    """The reference-shaped surface: LQRProblem(q=, r=, qf=) → solve(sol, DPSolver, prob)
    fills sol.d (feedforward) and sol.p (linear cost-to-go) beside K, X, U, P."""
    from lqrx.dp import DPSolver, LQRProblem, LQRSolution, from_abi

    n, m, N = 6, 2, 30
    d = lin_problem(lqrx, n, m, N, 1, 2024)
    prob = LQRProblem(Qf=from_abi(d["Qf"], (1, n, n))[0], Q=from_abi(d["Q"], (1, n, n))[0],
                      R=from_abi(d["R"], (1, m, m))[0], A=from_abi(d["A"], (1, n, n))[0],
                      B=from_abi(d["B"], (1, n, m))[0], x0=d["x0"].copy(), N=N,
                      q=d["q"].copy(), r=d["r"].copy(), qf=d["qf"].copy())
    sol = LQRSolution.of(prob, all_P=True)
    lqrx.solve(sol, DPSolver.of(prob), prob)
    ref = oracle.dp_solve_lin_abi(d, N, all_P=True)
    got = dict(K=sol.K[None], P=sol.P[None], X=sol.X[None], U=sol.U[None], d=sol.d[None], p=sol.p[None],
               info=np.array([sol.info]))
    check(got, ref, n, m, N, 1, True, TOL64)
