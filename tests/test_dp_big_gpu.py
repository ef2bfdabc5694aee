"""GPU parity: DP shapes past the register-tiled kernels (n > 64 or m > 32, up to 512) on the
workgroup-per-trajectory kernel (lqrx_dp_big.hip), against the CPU oracle of
/root/reference/src/dynamic_programming.jl:28-72 — the reference handles any (n, m).

Same tolerances as the other DP kernels: K, P per knot within 1e-10 relative in fp64 (this
kernel keeps the reference op order, so it tracks the oracle to rounding), X, U on the
trajectory's scale; fp32 within 1e-4 of the fp64 oracle.
"""
import numpy as np
import pytest

from test_dp_gpu import TOL32, TOL64, relerr_per_knot, run_pair
from test_dp_linear_gpu import check, lin_problem, to_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,m,N,batch", [
    (65, 4, 12, 3),       # one past the 4×2 tile grid in n
    (16, 33, 10, 2),      # one past it in m
    (96, 48, 20, 3),
    (128, 64, 8, 2),
    (80, 1, 30, 5),
])
def test_dp_big_parity_f64(lqrx, oracle, gpu_ok, n, m, N, batch):
    got, ref = run_pair(lqrx, oracle, n, m, N, batch, seed=7000 + n + m)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert relerr_per_knot(got["K"], ref["K"]) <= TOL64
    assert relerr_per_knot(got["P"], ref["P"]) <= TOL64
    assert np.abs(got["X"] - ref["X"]).max() <= TOL64 * max(1.0, np.abs(ref["X"]).max())
    assert np.abs(got["U"] - ref["U"]).max() <= TOL64 * max(1.0, np.abs(ref["U"]).max())


def test_dp_big_parity_f32(lqrx, oracle, gpu_ok):
    got, ref = run_pair(lqrx, oracle, 72, 36, 16, 3, seed=71, dtype=1)
    assert relerr_per_knot(got["K"].astype(np.float64), ref["K"]) <= TOL32
    assert relerr_per_knot(got["P"].astype(np.float64), ref["P"]) <= TOL32


def test_dp_big_p1_layout1_time_varying(lqrx, oracle, gpu_ok):
    """p_mode 0, layout 1 (through the stream-ordered transpose) and per-knot A_k, B_k, Q_k,
    R_k with linear cost terms on the big kernel."""
    n, m, N, bt = 70, 8, 9, 3
    d = lin_problem(lqrx, n, m, N, bt, 555, tv_QR=True, tv_AB=True)
    b = to_batch(d, N)
    for all_P in (True, False):
        got = lqrx.solve_batch(b, all_P=all_P)
        ref = oracle.dp_solve_lin_abi(d, N, all_P=all_P)
        check(got, ref, n, m, N, bt, all_P, TOL64)
    g0 = lqrx.solve_batch(b, all_P=True, layout=0)
    g1 = lqrx.solve_batch(b, all_P=True, layout=1)
    for k in ("K", "P", "X", "U", "d", "p"):
        assert np.array_equal(g0[k], g1[k]), k


def test_dp_big_info(lqrx, oracle, gpu_ok):
    """A non-SPD R (the reference discards potrf's info) is reported at the first backward
    knot, as by the other kernels."""
    from lqrx.dp import abi_to_batch

    n, m, N, bt = 66, 3, 6, 2
    d = lqrx.random_batch(n, m, N, bt, seed=3)
    b = abi_to_batch(d)
    b.R[1] = -1e3 * np.eye(m)           # E = R + BᵀQfB stays indefinite
    got = lqrx.solve_batch(b)
    assert got["rc"] == 1 and got["info"][0] == 0 and got["info"][1] == N - 1


def test_dp_big_unsupported(lqrx, gpu_ok):
    import ctypes as C
    from lqrx import _lib

    d = _lib.DpDesc(513, 4, 5, 0, 2, 0, 0, 0, 0)
    assert lqrx.load().lqrx_dp_solve(C.byref(d), *([None] * 10), None, None) == _lib.ERR_UNSUPPORTED


def test_dp_big_chunked_batch(lqrx, oracle, gpu_ok, monkeypatch):
    """The batch runs in scratch-bounded chunks (≤ 4 GiB each); LQRX_DP_BIG_CHUNK forces
    chunks of 2 trajectories: results equal the one-chunk solve bit for bit."""
    from lqrx.dp import abi_to_batch

    n, m, N, bt = 70, 6, 7, 5
    b = abi_to_batch(lqrx.random_batch(n, m, N, bt, seed=12))
    one = lqrx.solve_batch(b, all_P=True)
    monkeypatch.setenv("LQRX_DP_BIG_CHUNK", "2")
    many = lqrx.solve_batch(b, all_P=True)
    for k in ("K", "P", "X", "U", "info"):
        assert np.array_equal(one[k], many[k]), k
