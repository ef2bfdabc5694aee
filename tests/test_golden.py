"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture bit-exactly (regression pin of the restatement).
GPU: the HIP path matches every fixture within the north-star tolerance (1e-10 rel, fp64).
"""
import glob
import os

import numpy as np
import pytest

from oracle import oracle as orc

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DP = sorted(glob.glob(os.path.join(HERE, "dp_*.npz")))
KKT = sorted(glob.glob(os.path.join(HERE, "kkt_*.npz")))


def _kkt_struct(f):
    import lqrx.kkt as K

    return K.ConstraintBlocks(int(f["n"]), int(f["m"]), int(f["N"]), f["p"])


@pytest.mark.parametrize("path", DP, ids=os.path.basename)
def test_dp_fixture_oracle_exact(lqrx, path):
    f = np.load(path)
    d = {k: f[k] for k in ("A", "B", "Q", "R", "Qf", "x0")}
    d.update(n=int(f["n"]), m=int(f["m"]), batch=int(f["batch"]))
    out = orc.dp_solve_abi(d, int(f["N"]), all_P=True)
    for k in ("K", "P", "X", "U"):
        assert np.array_equal(out[k], f[k]), k


@pytest.mark.parametrize("path", KKT, ids=os.path.basename)
def test_kkt_fixture_oracle_exact(lqrx, path):
    f = np.load(path)
    st = _kkt_struct(f)
    os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
    out = orc.kkt_solve_batch(os_, int(f["batch"]), f["Y"], f["y"], f["H"], f["g"],
                              h_mode=int(f["h_mode"]), ginv=int(f["ginv"]))
    assert np.array_equal(out["dz"], f["dz"]) and np.array_equal(out["lam"], f["lam"])


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


@pytest.mark.gpu
@pytest.mark.parametrize("path", DP, ids=os.path.basename)
def test_dp_fixture_gpu(lqrx, gpu_ok, path):
    from lqrx.dp import abi_to_batch, from_abi

    f = np.load(path)
    n, m, N, bt = int(f["n"]), int(f["m"]), int(f["N"]), int(f["batch"])
    d = {k: f[k] for k in ("A", "B", "Q", "R", "Qf", "x0")}
    d.update(n=n, m=m, N=N, batch=bt)
    got = lqrx.solve_batch(abi_to_batch(d), all_P=True)
    K = from_abi(f["K"], (bt, N - 1, m, n))
    P = from_abi(f["P"], (bt, N, n, n))
    for t in range(bt):
        for k in range(N - 1):
            assert _rel(got["K"][t, k], K[t, k]) <= 1e-10
        for k in range(N):
            assert _rel(got["P"][t, k], P[t, k]) <= 1e-10
    assert _rel(got["X"], f["X"].reshape(bt, N, n)) <= 1e-10
    assert _rel(got["U"], f["U"].reshape(bt, N - 1, m)) <= 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("path", KKT, ids=os.path.basename)
def test_kkt_fixture_gpu(lqrx, gpu_ok, path):
    import lqrx.kkt as K

    f = np.load(path)
    st = _kkt_struct(f)
    bt = int(f["batch"])
    pb = K.KktProblem(st, bt, int(f["h_mode"]), f["Y"].reshape(bt, -1), f["y"].reshape(bt, -1),
                      f["H"].reshape(bt, -1), f["g"].reshape(bt, -1))
    got = K.kkt_solve(pb, ginv=int(f["ginv"]))
    assert _rel(got["dz"], f["dz"].reshape(bt, -1)) <= 1e-10
    assert _rel(got["lam"], f["lam"].reshape(bt, -1)) <= 1e-10


LS = sorted(glob.glob(os.path.join(HERE, "ls_*.npz")))


@pytest.mark.parametrize("path", LS, ids=os.path.basename)
def test_ls_fixture_oracle(lqrx, path):
    """The condensed least-squares restatement reproduces its fixtures (numpy/OpenBLAS: to
    rounding, not bit-exact — BLAS summation order is not pinned)."""
    from oracle import ls_oracle as LO

    f = np.load(path)
    for b in range(f["A"].shape[0]):
        o = LO.ls_solve(f["A"][b], f["B"][b], f["Q"][b], f["R"][b], f["Qf"][b], f["x0"][b],
                        int(f["N"]), hu=int(f["hu"]))
        assert _rel(o["U"], f["U"][b]) <= 1e-12 and _rel(o["X"], f["X"][b]) <= 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("path", LS, ids=os.path.basename)
def test_ls_fixture_gpu(lqrx, gpu_ok, path):
    """ls_condensed_kernel on the fixture inputs: U, X within 1e-9 relative (cond(H) of the
    cartpole N=41 fixtures ≤ 2e6; two Cholesky solves of the same normal equations)."""
    from lqrx import ls
    from lqrx.dp import LQRBatch

    f = np.load(path)
    out = ls.ls_solve_batch(LQRBatch(f["A"], f["B"], f["Q"], f["R"], f["Qf"], f["x0"], int(f["N"])),
                            hu_mode=int(f["hu"]))
    assert out["rc"] == 0
    assert _rel(out["U"], f["U"]) <= 1e-9 and _rel(out["X"], f["X"]) <= 1e-9
