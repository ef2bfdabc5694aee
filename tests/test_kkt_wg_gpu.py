"""GPU parity of the workgroup-per-trajectory KKT kernel (lqr.jl_amd/csrc/lqrx_kkt_wg.hip) —
block sizes past the large-block register tiles (n1, p, n2 > 64 or w > 128, up to 512 / 1024)
— against the CPU oracle (oracle/lqr_oracle.c: the reference's block Cholesky at any block
size, cholesky_solve.jl:47-143, jacobian_blocks.jl:220-286, cholesky_solver.jl:166-236).

Tolerances as test_kkt_big_gpu.py: fp64 within 1e-10 relative per trajectory; fp32 against the
fp64 oracle on the same fp32-rounded inputs within 1e-4.  The last test forces the kernel
(LQRX_KKT_WG=1, read once per process — one child process) onto small structures so that
every option (dense / block-diagonal / diagonal H, SOC, stage constraints, info, chunking)
is exercised on it at oracle-cheap sizes.
"""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
TOL = 1e-10
F32_TOL = 1e-4


def traj_rel(a, b):
    a = np.asarray(a, np.float64).reshape(b.shape)
    den = np.maximum(np.abs(b).max(axis=1), 1e-300)
    return float((np.abs(a - b).max(axis=1) / den).max())


def _ref(st, pb, ginv=1):
    os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
    r = orc.kkt_solve_batch(os_, pb.batch, pb.Y, pb.y, pb.H, pb.g, h_mode=pb.h_mode, ginv=ginv, nthreads=8)
    return dict(dz=r["dz"].reshape(pb.batch, -1), lam=r["lam"].reshape(pb.batch, -1), info=r["info"])


def _round32(pb):
    import dataclasses
    f = lambda a: np.asarray(a, np.float32).astype(np.float64)
    return dataclasses.replace(pb, Y=f(pb.Y), y=f(pb.y), H=f(pb.H), g=f(pb.g))


@pytest.mark.parametrize("n,m,N", [(96, 48, 64), (72, 40, 17), (128, 64, 9)])
def test_wg_kkt_f64_trajectory(lqrx, gpu_ok, n, m, N):
    """n = 96, m = 48, N = 64 (blocks of 96 rows, w = 144) and neighbours,
    diagonal H, fp64."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, N)
    pb = K.random_kkt(st, 3, seed=n + N, h_mode=K.H_DIAG, dyn="dense")
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert got["rc"] == 0 and (got["info"] == 0).all() and (ref["info"] == 0).all()
    assert traj_rel(got["dz"], ref["dz"]) <= TOL
    assert traj_rel(got["lam"], ref["lam"]) <= TOL


@pytest.mark.parametrize("n,m,N", [(96, 48, 64), (80, 16, 33)])
def test_wg_kkt_f32(lqrx, gpu_ok, n, m, N):
    """fp32 past the large-block kernels."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, N)
    pb = _round32(K.random_kkt(st, 3, seed=7 * n + N, h_mode=K.H_DIAG, dyn="dense"))
    got = K.kkt_solve(pb, dtype=lqrx.F32)
    ref = _ref(st, pb)
    assert got["dz"].dtype == np.float32
    assert got["rc"] == 0 and (got["info"] == 0).all()
    e = max(traj_rel(got["dz"], ref["dz"]), traj_rel(got["lam"], ref["lam"]))
    print(f"fp32 n={n} m={m} N={N}: max rel err {e:.3e}")
    assert e <= F32_TOL


@pytest.mark.parametrize("n,m,N", [(70, 30, 9), (72, 40, 7), (67, 20, 5)])
@pytest.mark.parametrize("ginv", [1, 0])
def test_wg_kkt_f32_ragged_w(lqrx, gpu_ok, n, m, N, ginv):
    """the fp32 diagonal-H Gram path with w mod 16 in 3..8 — w = 100 for
    (70, 30), the last knot's w = 72 for (72, 40), w = 87 for (67, 20).  In fp32 one lane's
    k index steps by 1 per slice, so a partial 16-column k-tile still needs all 4 slices; the
    round-5 slice count ceil(w/4) dropped columns 16t+2, 16t+3 (…) of the last tile."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, N)
    assert any(int(w) % 16 in range(3, 9) for w in st.w)
    pb = _round32(K.random_kkt(st, 3, seed=11 * n + m, h_mode=K.H_DIAG, dyn="dense"))
    got = K.kkt_solve(pb, dtype=lqrx.F32, ginv=ginv)
    ref = _ref(st, pb, ginv=ginv)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    e = max(traj_rel(got["dz"], ref["dz"]), traj_rel(got["lam"], ref["lam"]))
    print(f"fp32 n={n} m={m} N={N} ginv={ginv}: max rel err {e:.3e}")
    assert e <= F32_TOL


@pytest.mark.parametrize("n,m,N,h_mode", [(80, 40, 9, 0), (66, 20, 7, 1), (40, 100, 6, 0)])
def test_wg_kkt_dense_h(lqrx, gpu_ok, n, m, N, h_mode):
    """Dense / block-diagonal H_k (potrf per knot, H⁻¹ by potrs) with blocks past 64 rows or
    w past 128 (n = 40, m = 100: w = 140)."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, N)
    pb = K.random_kkt(st, 3, seed=n + m + h_mode, h_mode=h_mode, dyn="dense")
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert traj_rel(got["dz"], ref["dz"]) <= TOL
    assert traj_rel(got["lam"], ref["lam"]) <= TOL


def test_wg_kkt_stage_constraints_and_soc(lqrx, gpu_ok):
    """Interior stage constraints of 70 rows (B, D, E blocks and the B̃ factor past 64) and the
    second-order correction (ginv = 0: H = I, r = 0)."""
    import lqrx.kkt as K

    n, m, N, ps = 72, 80, 9, 70
    st = K.ConstraintBlocks(n, m, N, [n] + [ps] * (N - 2) + [n])
    pb = K.random_kkt(st, 3, seed=ps, h_mode=K.H_DIAG, dyn="dense")
    for ginv in (1, 0):
        got = K.kkt_solve(pb, ginv=ginv)
        ref = _ref(st, pb, ginv=ginv)
        assert got["rc"] == 0 and (got["info"] == 0).all()
        assert traj_rel(got["dz"], ref["dz"]) <= TOL, ginv
        assert traj_rel(got["lam"], ref["lam"]) <= TOL, ginv


def test_wg_kkt_info(lqrx, gpu_ok):
    """info on the workgroup kernel: a negative diagonal cost block makes a Schur pivot fail
    (k+1 of the first failing knot), untouched trajectories stay 0 and match the oracle."""
    import lqrx.kkt as K

    st = K.trajectory_structure(70, 30, 11)
    pb = K.random_kkt(st, 3, seed=3, h_mode=K.H_DIAG, dyn="dense")
    og = int(np.sum(st.w[:5]))
    pb.H[1, og:og + st.w[5]] = -5.0
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert got["rc"] == 1
    assert list(got["info"]) == list(ref["info"]), (got["info"], ref["info"])
    assert got["info"][0] == 0 and got["info"][2] == 0 and got["info"][1] > 0
    ok = [0, 2]
    assert traj_rel(got["dz"][ok], ref["dz"][ok]) <= TOL


def test_wg_kkt_past_limits_unsupported(lqrx, gpu_ok):
    """Blocks past 512 rows return LQRX_ERR_UNSUPPORTED from the validation."""
    import ctypes as C
    import lqrx.kkt as K

    st = K.trajectory_structure(513, 4, 3)
    n = C.c_size_t(0)
    assert lqrx.load().lqrx_kkt_workspace_size(C.byref(st.desc(2, K.H_DIAG, 1, 0, lqrx.F64)), C.byref(n)) == -101


_FORCE_SCRIPT = r"""
import sys, dataclasses, numpy as np
sys.path[:0] = [sys.argv[1] + "/lqr.jl_amd", sys.argv[1]]
import lqrx, lqrx.kkt as K
from oracle import oracle as orc

def rel(a, b):
    a = np.asarray(a, np.float64).reshape(b.shape)
    return float((np.abs(a - b).max(axis=1) / np.maximum(np.abs(b).max(axis=1), 1e-300)).max())

bad = 0
cases = [  # n, m, N, stage rows, h_mode, ginv, dtype
    (16, 8, 21, 0, 2, 1, lqrx.F64), (16, 8, 21, 0, 0, 1, lqrx.F64), (7, 3, 41, 0, 1, 1, lqrx.F64),
    (20, 24, 23, 17, 2, 1, lqrx.F64), (8, 4, 17, 3, 0, 0, lqrx.F64), (3, 2, 101, 0, 0, 1, lqrx.F64),
    (32, 16, 13, 0, 2, 1, lqrx.F32), (16, 8, 9, 5, 0, 1, lqrx.F32), (64, 32, 5, 0, 2, 1, lqrx.F64),
]
for n, m, N, ps, hm, ginv, dt in cases:
    st = K.trajectory_structure(n, m, N) if ps == 0 else K.ConstraintBlocks(n, m, N, [n] + [ps] * (N - 2) + [n])
    pb = K.random_kkt(st, 5, seed=n + N + hm, h_mode=hm, dyn="dense" if n >= 8 else "small")
    if dt == lqrx.F32:
        f = lambda a: np.asarray(a, np.float32).astype(np.float64)
        pb = dataclasses.replace(pb, Y=f(pb.Y), y=f(pb.y), H=f(pb.H), g=f(pb.g))
    got = K.kkt_solve(pb, ginv=ginv, dtype=dt)
    r = orc.kkt_solve_batch(orc.KktStructure(n, m, N, st.p), 5, pb.Y, pb.y, pb.H, pb.g, h_mode=hm, ginv=ginv,
                            nthreads=4)
    e = max(rel(got["dz"], r["dz"].reshape(5, -1)), rel(got["lam"], r["lam"].reshape(5, -1)))
    tol = 1e-10 if dt == lqrx.F64 else 1e-4
    ok = e <= tol and got["rc"] == 0 and (np.asarray(got["info"]) == 0).all()
    print(n, m, N, ps, hm, ginv, dt, "rel err %.3e" % e, "ok" if ok else "FAIL")
    bad += not ok

# info: a non-SPD dense H_k → −(k+1); a failing Schur pivot → k+1 (oracle convention)
st = K.trajectory_structure(16, 8, 15)
pb = K.random_kkt(st, 3, seed=9, h_mode=K.H_DENSE, dyn="dense")
w = st.w.astype(int)
o = int(np.sum(w[:6] * w[:6]))
pb.H[2, o:o + w[6] * w[6]] *= -1.0
got = K.kkt_solve(pb)
r = orc.kkt_solve_batch(orc.KktStructure(16, 8, 15, st.p), 3, pb.Y, pb.y, pb.H, pb.g, h_mode=0, nthreads=4)
print("dense-H info", list(got["info"]), list(r["info"]))
bad += list(got["info"]) != list(r["info"]) or r["info"][2] != -7
sys.exit(1 if bad else 0)
"""


def test_wg_kkt_forced_on_small_structures(lqrx, gpu_ok, tmp_path):
    """LQRX_KKT_WG=1 routes every layout-0 call to the workgroup kernel; LQRX_KKT_WG_CHUNK=2
    runs the 5-trajectory batches in 3 chunks through one scratch block."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "force_wg.py"
    f.write_text(_FORCE_SCRIPT)
    env = dict(os.environ, LQRX_KKT_WG="1", LQRX_KKT_WG_CHUNK="2")
    p = subprocess.run([sys.executable, str(f), root], env=env, capture_output=True, text=True, timeout=300)
    print(p.stdout)
    assert p.returncode == 0, p.stdout + p.stderr
