"""GPU parity: trajectory-form KKT structures outside the compile-time shapes, on the padded
direct kernel (kkt_fild_kernel<Shape<…, PAD>>, lqrx_kkt_fil.hip) — blocks zero-padded in
registers up to a bin (4,2,4,1,4) / (6,3,6,1,6) / (8,4,8,1,8), the structure's own sizes at run time
— and round 5's exact direct shapes for trajectory_structure(6, 2, N) and (8, 4, N).

Reference: the block structure ConstraintBlocks builds (conblocks.jl:403-425) for any (n, m)
and stage constraints; the solve is cholesky_solver.jl:166-236 on it.  Oracle: oracle/
lqr_oracle.c (fp64), tolerance 1e-10 relative as in test_kkt_gpu.py.  The large-block path
(LQRX_KKT_PAD=0 in a child process) must agree with the padded kernel to the same tolerance.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
TOL = 1e-10
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def _ref(st, pb, ginv):
    os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
    return orc.kkt_solve_batch(os_, pb.batch, pb.Y, pb.y, pb.H, pb.g, h_mode=pb.h_mode, ginv=ginv, nthreads=8)


def _structure(K, n, m, N, kind):
    if kind == "traj":                       # initial state, dynamics, goal
        return K.trajectory_structure(n, m, N)
    if kind == "stage":                      # + a one-row stage constraint on the interior knots
        return K.ConstraintBlocks(n, m, N, [n] + [1] * (N - 2) + [n])
    if kind == "nogoal":                     # no terminal constraint (PN = 0)
        return K.ConstraintBlocks(n, m, N, [n] + [0] * (N - 2) + [0])
    raise ValueError(kind)


CASES = [
    # (n, m, N, kind, batch): every bin, ragged batches, short horizons (stage rows only where
    # the system stays well posed: n + PK(N−2) ≤ m(N−1))
    (2, 1, 11, "traj", 67),
    (3, 1, 21, "traj", 130),
    (4, 2, 101, "traj", 64),
    (4, 2, 6, "stage", 33),
    (3, 2, 9, "nogoal", 70),
    (5, 1, 31, "traj", 65),
    (6, 2, 101, "traj", 96),             # exact direct shape (6,2,6,0,6) since round 5
    (6, 3, 40, "traj", 17),
    (5, 3, 12, "stage", 40),
    (6, 1, 4, "nogoal", 9),
    (8, 4, 21, "traj", 66),              # exact direct shape (8,4,8,0,8) since round 5
    (8, 4, 13, "stage", 33),             # bin (8,4,8,1,8)
    (7, 2, 12, "stage", 31),
    (8, 3, 5, "nogoal", 5),
]


@pytest.mark.parametrize("n,m,N,kind,batch", CASES)
@pytest.mark.parametrize("ginv", [1, 0])
def test_kkt_padded_parity(lqrx, gpu_ok, n, m, N, kind, batch, ginv):
    import lqrx.kkt as K

    st = _structure(K, n, m, N, kind)
    pb = K.random_kkt(st, batch, seed=1000 + 7 * n + m + N, h_mode=2)
    got = K.kkt_solve(pb) if ginv else K.second_order_correction(pb)
    ref = _ref(st, pb, ginv)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert np.isfinite(got["dz"]).all() and np.isfinite(got["lam"]).all()
    assert rel(got["dz"], ref["dz"].reshape(batch, -1)) <= TOL
    assert rel(got["lam"], ref["lam"].reshape(batch, -1)) <= TOL


def test_kkt_padded_layout1_staged(lqrx, gpu_ok):
    """Layout 1 (SoA) of a padded structure: staged to layout 0, bit-identical results."""
    import lqrx.kkt as K

    st = K.trajectory_structure(5, 1, 33)          # padded bin (6,3,6,1,6)
    pb = K.random_kkt(st, 70, seed=5, h_mode=2)
    a = K.kkt_solve(pb, layout=0)
    b = K.kkt_solve(pb, layout=1)
    assert a["rc"] == 0 and b["rc"] == 0
    assert np.array_equal(a["dz"], b["dz"]) and np.array_equal(a["lam"], b["lam"])


@pytest.mark.parametrize("n,m,N,batch", [(6, 2, 37, 70), (8, 4, 29, 65)])
@pytest.mark.parametrize("ginv", [1, 0])
def test_kkt_exact_traj_shapes_layouts(lqrx, gpu_ok, n, m, N, batch, ginv):
    """Round 5's exact direct shapes (6,2,6,0,6) and (8,4,8,0,8) — trajectory_structure(6, 2, N)
    and (8, 4, N) — in both ABI layouts (layout 1 native, SoA) against the oracle."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, N)
    pb = K.random_kkt(st, batch, seed=70 + n + N + ginv, h_mode=2)
    ref = _ref(st, pb, ginv)
    for layout in (0, 1):
        got = K.kkt_solve(pb, ginv=ginv, layout=layout)
        assert got["rc"] == 0 and (got["info"] == 0).all()
        assert rel(got["dz"], ref["dz"].reshape(batch, -1)) <= TOL
        assert rel(got["lam"], ref["lam"].reshape(batch, -1)) <= TOL


def test_kkt_padded_matches_large_block_path(lqrx, gpu_ok, tmp_path):
    """The same problem with the padded kernel switched off (LQRX_KKT_PAD=0: the 16-padded
    large-block kernels of lqrx_kkt_big.hip) — both within 1e-10 of the oracle and of each
    other."""
    import lqrx.kkt as K

    st = K.trajectory_structure(6, 2, 51)
    pb = K.random_kkt(st, 40, seed=77, h_mode=2)
    got = K.kkt_solve(pb)
    np.savez(tmp_path / "pb.npz", Y=pb.Y, y=pb.y, H=pb.H, g=pb.g)
    code = (
        "import sys, numpy as np; sys.path[:0] = [%r, %r];"
        "import lqrx.kkt as K;"
        "st = K.trajectory_structure(6, 2, 51); z = np.load(%r);"
        "pb = K.KktProblem(st, 40, 2, z['Y'], z['y'], z['H'], z['g']);"
        "r = K.kkt_solve(pb); np.savez(%r, dz=r['dz'], lam=r['lam'], rc=r['rc'])"
    ) % (ROOT, os.path.join(ROOT, "lqr.jl_amd"), str(tmp_path / "pb.npz"), str(tmp_path / "big.npz"))
    env = dict(os.environ, LQRX_KKT_PAD="0")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    big = np.load(tmp_path / "big.npz")
    assert int(big["rc"]) == 0
    assert rel(got["dz"], big["dz"]) <= TOL and rel(got["lam"], big["lam"]) <= TOL


# ---------------------------------------------------------------- dense / block-diagonal H
# BlockCholesky modes 0 and 1 (block_cholesky.jl:55-77) on the diagonal-H kernels through the
# H = UᵀU pre-pass (Z = Y U⁻¹, gz = U⁻ᵀg) and the δz = U⁻¹δz' post-pass (fil::kkt_hpre_kernel).
DENSE = [
    ("di3", None, None, 101, 50),        # DoubleIntegrator(3): exact direct shape (6,3,6,1,6)
    ("di2", None, None, 12, 37),         # DoubleIntegrator(2): exact (4,2,4,1,4)
    ("traj", 6, 2, 101, 40),             # exact (6,2,6,0,6)
    ("traj", 5, 1, 41, 40),              # padded bin (6,3,6,1,6)
    ("traj", 5, 2, 31, 65),              # exact (5,2,5,0,5)
    ("traj", 4, 1, 21, 70),              # cartpole's shape: the LDS-staged FIL kernel (diagonal only)
    ("stage", 3, 2, 9, 20),              # padded bin (4,2,4,1,4)
]


def _dense_structure(K, kind, n, m, N):
    if kind == "di3":
        return K.double_integrator_structure(3, N)
    if kind == "di2":
        return K.double_integrator_structure(2, N)
    return _structure(K, n, m, N, kind)


@pytest.mark.parametrize("kind,n,m,N,batch", DENSE)
@pytest.mark.parametrize("h_mode", [0, 1])
def test_kkt_dense_h_parity(lqrx, gpu_ok, kind, n, m, N, batch, h_mode):
    import lqrx.kkt as K

    st = _dense_structure(K, kind, n, m, N)
    pb = K.random_kkt(st, batch, seed=300 + N + h_mode, h_mode=h_mode)
    got = K.kkt_solve(pb)
    ref = _ref(st, pb, 1)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert rel(got["dz"], ref["dz"].reshape(batch, -1)) <= TOL
    assert rel(got["lam"], ref["lam"].reshape(batch, -1)) <= TOL


@pytest.mark.parametrize("knot", [0, 5, 20])
def test_kkt_dense_h_info(lqrx, gpu_ok, knot):
    """A non-SPD H_k reports info = −(k+1) for that trajectory only, as the large-block path's
    dense-H pre-pass does (kb hfac, lqrx_kkt_big.hip)."""
    import lqrx.kkt as K

    st = K.double_integrator_structure(3, 21)
    pb = K.random_kkt(st, 6, seed=11, h_mode=0)
    w = st.w
    oH = int(np.sum(w[:knot] * w[:knot]))
    wk = int(w[knot])
    pb.H[3, oH:oH + wk * wk] *= -1.0
    got = K.kkt_solve(pb)
    assert got["rc"] == 1
    assert int(got["info"][3]) == -(knot + 1)
    assert (np.delete(got["info"], 3) == 0).all()


def test_kkt_dense_h_info_wins_over_earlier_pivot(lqrx, gpu_ok):
    """A Schur pivot failure at knot 2 (a zero stage-constraint row) AND a non-SPD H_10: the H
    failure is reported, −11, as the oracle (and the reference, which factors every H_k in
    shur! before cholesky! meets a pivot) and the large-block / workgroup routes report it."""
    import lqrx.kkt as K

    st = K.double_integrator_structure(3, 21)
    pb = K.random_kkt(st, 6, seed=12, h_mode=0)
    rows, w = st.n1 + st.p + st.n2, st.w
    oY = int(np.sum(rows[:2] * w[:2]))                    # knot 2's Y block, column-major rows × w
    for c in range(int(w[2])):
        pb.Y[3, oY + c * int(rows[2]) + int(st.n1[2])] = 0.0   # its stage row (C, after D2)
    oH = int(np.sum(w[:10] * w[:10]))
    pb.H[3, oH:oH + int(w[10]) ** 2] *= -1.0
    got = K.kkt_solve(pb)
    ref = _ref(st, pb, 1)
    assert int(ref["info"][3]) == -11
    assert int(got["info"][3]) == -11
    assert (np.delete(got["info"], 3) == 0).all()
