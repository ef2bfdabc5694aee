"""GPU parity: the fp64 n = 64 four-wave DP kernel's time-varying and linear-term variants
(lqrx_dp.hip dp_wg4_kernel<double, MT, VAR_TV | VAR_LIN>, round 6) against the CPU oracle.

The reference runs any (n, m) in fp64 with per-knot data (dynamic_programming.jl:54-72 over the
constrained_problem.jl:3-4 layout); before round 6 only the time-invariant n = 64 problem ran on
four waves and the time-varying / linear-term ones fell back to the one-wave kernel that spills
2–3 KB per lane.  Oracle: oracle/lqr_oracle.c (dp_solve_abi with tv_AB / tv_QR, and
dp_solve_lin_abi for q, r, qf — the op-for-op restatement of :28-72, extended by one potrs column
for d, §3.7).  Tolerance as every fp64 DP test: 1e-10 relative per knot (K, P), 1e-10 on the
trajectory's scale for X, U, d, p.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from test_dp_lane_gpu import _tv_batch
from test_dp_linear_gpu import check, lin_problem, to_batch

pytestmark = pytest.mark.gpu

TOL64 = 1e-10


def relerr_per_knot(a, b):
    a = a.reshape(a.shape[0], a.shape[1], -1)
    b = b.reshape(b.shape[0], b.shape[1], -1)
    den = np.abs(b).max(axis=2)
    den[den == 0] = 1.0
    return float((np.abs(a - b).max(axis=2) / den).max())


@pytest.mark.parametrize("m,tv_ab,tv_qr,N,bt,all_P", [
    (32, True, True, 40, 3, True),      # dp_wg4_kernel<double, 2, VAR_TV>
    (16, True, True, 33, 2, True),      # <double, 1, VAR_TV>
    (32, True, False, 24, 2, False),    # per-knot A_k, B_k only, P_1 only
    (32, False, True, 21, 2, True),     # per-knot Q_k, R_k only
    (32, True, True, 2, 3, True),       # N = 2: one backward knot, no prefetch
    (16, True, True, 3, 2, False),      # N = 3: the A double buffer's both halves once
])
def test_wg4_time_varying_parity(lqrx, oracle, gpu_ok, m, tv_ab, tv_qr, N, bt, all_P):
    from lqrx.dp import from_abi, to_abi

    n = 64
    b = _tv_batch(lqrx, n, m, N, bt, seed=310 + m + N, tv_ab=tv_ab, tv_qr=tv_qr)
    got = lqrx.solve_batch(b, all_P=all_P)
    d = {k: to_abi(getattr(b, k)).ravel() for k in ("A", "B", "Q", "R", "Qf")}
    d.update(x0=b.x0.ravel(), n=n, m=m, batch=bt, tv_AB=int(tv_ab), tv_QR=int(tv_qr))
    ref = oracle.dp_solve_abi(d, N, all_P=all_P)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert relerr_per_knot(got["K"], from_abi(ref["K"], (bt, N - 1, m, n))) <= TOL64
    if all_P:
        assert relerr_per_knot(got["P"], from_abi(ref["P"], (bt, N, n, n))) <= TOL64
    else:
        assert relerr_per_knot(got["P"][:, None], from_abi(ref["P"], (bt, 1, n, n))) <= TOL64
    refX = ref["X"].reshape(bt, N, n)
    refU = ref["U"].reshape(bt, N - 1, m)
    assert np.abs(got["X"] - refX).max() <= TOL64 * max(1.0, np.abs(refX).max())
    assert np.abs(got["U"] - refU).max() <= TOL64 * max(1.0, np.abs(refU).max())


@pytest.mark.parametrize("m,N,bt,tvq,tvab,all_P", [
    (32, 30, 2, False, False, True),    # dp_wg4_kernel<double, 2, VAR_LIN>
    (16, 25, 3, False, False, False),   # <double, 1, VAR_LIN>, p_1 only
    (32, 20, 2, True, False, True),     # per-knot Q, R, q, r: <double, 2, VAR_TV | VAR_LIN>
    (16, 18, 2, True, True, True),      # fully time-varying with linear terms
    (32, 2, 2, True, True, False),      # N = 2
])
def test_wg4_linear_parity(lqrx, oracle, gpu_ok, m, N, bt, tvq, tvab, all_P):
    n = 64
    d = lin_problem(lqrx, n, m, N, bt, 5200 + 3 * m + N, tvq, tvab)
    got = lqrx.solve_batch(to_batch(d, N), all_P=all_P)
    assert got["rc"] == 0
    ref = oracle.dp_solve_lin_abi(d, N, all_P=all_P)
    check(got, ref, n, m, N, bt, all_P, TOL64)


def test_wg4_time_varying_info_middle_knot(lqrx, oracle, gpu_ok):
    """An indefinite E at a middle knot k0 of a time-varying n = 64 problem: the four waves'
    Newton–Schulz verdicts are AND-ed, the exact sweep on wave 0 reports info = k0 (potrf's info,
    dynamic_programming.jl:29) and the knots solved before the break still match the oracle."""
    from lqrx.dp import from_abi, to_abi

    n, m, N, k0, bt = 64, 32, 24, 11, 3
    b = _tv_batch(lqrx, n, m, N, bt, seed=77, tv_ab=True, tv_qr=True)
    b.R = np.array(b.R)
    b.B = np.array(b.B)
    b.R[1, k0 - 1] = -100.0 * np.eye(m)
    b.B[1, k0 - 1] *= 1e-3
    got = lqrx.solve_batch(b, all_P=True)
    d = {k: to_abi(getattr(b, k)).ravel() for k in ("A", "B", "Q", "R", "Qf")}
    d.update(x0=b.x0.ravel(), n=n, m=m, batch=bt, tv_AB=1, tv_QR=1)
    ref = oracle.dp_solve_abi(d, N, all_P=True)
    assert ref["info"][1] == k0 and (np.delete(ref["info"], 1) == 0).all()
    assert got["rc"] == 1 and got["info"][1] == k0 and (np.delete(got["info"], 1) == 0).all()
    refK = from_abi(ref["K"], (bt, N - 1, m, n))
    assert relerr_per_knot(got["K"][[0, 2]], refK[[0, 2]]) <= TOL64
    assert relerr_per_knot(got["K"][1:2, k0:], refK[1:2, k0:]) <= TOL64


_CODE = """
import sys, numpy as np, lqrx
sys.path.insert(0, sys.argv[2])
from test_dp_linear_gpu import lin_problem, to_batch
d = lin_problem(lqrx, 64, 32, 22, 2, 9, tv_QR=True, tv_AB=True)
g = lqrx.solve_batch(to_batch(d, 22), all_P=True)
np.save(sys.argv[1], np.concatenate([g[k].ravel() for k in ("K", "P", "X", "U", "d", "p")]))
"""


def test_wg4_variants_match_one_wave(lqrx, gpu_ok):
    """The four-wave TV + LIN kernel and the one-wave kernel (LQRX_DP_WG4=0) agree to rounding."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for flag in ("1", "0"):
        f = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"wg4v_{flag}_{os.getpid()}.npy")
        env = dict(os.environ, LQRX_DP_WG4=flag,
                   PYTHONPATH=os.pathsep.join([os.path.join(root, "lqr.jl_amd"), os.environ.get("PYTHONPATH", "")]))
        subprocess.run([sys.executable, "-c", _CODE, f, os.path.join(root, "tests")], env=env, check=True,
                       timeout=120)
        outs.append(np.load(f))
        os.remove(f)
    a, b = outs
    assert np.abs(a - b).max() <= 1e-11 * np.abs(b).max()


_SWEEP = """
import sys, numpy as np, lqrx
sys.path.insert(0, sys.argv[1])
from oracle import oracle as orc
from lqrx.dp import abi_to_batch, from_abi
n, m, N, bt = (int(v) for v in sys.argv[2:6])
d = lqrx.random_batch(n, m, N, bt, seed=n + 7 * m)
got = lqrx.solve_batch(abi_to_batch(d), all_P=True)
ref = orc.dp_solve_abi(d, N, all_P=True)
K = from_abi(ref["K"], (bt, N - 1, m, n)); P = from_abi(ref["P"], (bt, N, n, n))
ek = np.abs(got["K"] - K).max() / np.abs(K).max(); ep = np.abs(got["P"] - P).max() / np.abs(P).max()
ex = np.abs(got["X"] - ref["X"].reshape(bt, N, n)).max() / max(1.0, np.abs(ref["X"]).max())
print(n, m, ek, ep, ex)
sys.exit(0 if (got["rc"] == 0 and (got["info"] == 0).all() and max(ek, ep, ex) <= 1e-10) else 1)
"""


@pytest.mark.parametrize("n,m,N,bt", [(64, 32, 20, 3), (64, 16, 17, 2), (32, 16, 30, 4), (17, 5, 12, 3)])
def test_exact_sweep_every_knot(lqrx, gpu_ok, n, m, N, bt):
    """LQRX_DP_NS_OFF=1 (tests only): no Newton–Schulz step, every knot takes the exact LDLᵀ sweep
    and its verdict path — in the four-wave kernel (m = 32: the wave-3 verdict barrier, then the
    sweep on wave 0 at every knot) and the one-wave kernel — still equal to the oracle at 1e-10."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LQRX_DP_NS_OFF="1",
               PYTHONPATH=os.pathsep.join([os.path.join(root, "lqr.jl_amd"), root, os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, "-c", _SWEEP, root, str(n), str(m), str(N), str(bt)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
