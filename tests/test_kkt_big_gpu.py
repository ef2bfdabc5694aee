"""GPU parity of the large-block MFMA KKT kernels (lqr.jl_amd/csrc/lqrx_kkt_big.hip) against
the CPU oracle (oracle/lqr_oracle.c: cholesky_solver.jl:166-236, jacobian_blocks.jl:220-286,
cholesky_solve.jl:47-143 — any block size, as the reference's LAPACK path).

Tolerances: fp64 δz and λ within 1e-10 of the oracle, relative per trajectory (max-abs error
over the trajectory ÷ its max-abs value).  fp32 (BASELINE configs[4]'s precision) against the
fp64 oracle run on the SAME fp32-rounded inputs, within F32_TOL = 1e-4 relative per
trajectory: single precision accumulated over the forward and backward sweeps of up to 512
knots (measured worst case 4.8e-6 at n=64 m=32 N=512).
"""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
TOL = 1e-10
F32_TOL = 1e-4
CASES = [(8, 4), (16, 8), (32, 16), (64, 32)]


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


@pytest.mark.parametrize("n,m", CASES)
@pytest.mark.parametrize("N", [2, 5, 37])
def test_big_kkt_f64_trajectory(lqrx, gpu_ok, n, m, N):
    """Trajectory structure (initial condition, dynamics, goal — conblocks.jl:403-425) with
    dense random dynamics blocks, diagonal H: the fp64 path of the large-block kernels."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, N)
    if N == 2 and n > m:
        pytest.skip("N = 2 with a goal is over-constrained for n > m (rows > variables)")
    pb = K.random_kkt(st, 5, seed=10 * n + N, h_mode=K.H_DIAG, dyn="dense")
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert got["rc"] == 0 and (got["info"] == 0).all() and (ref["info"] == 0).all()
    assert traj_rel(got["dz"], ref["dz"]) <= TOL
    assert traj_rel(got["lam"], ref["lam"]) <= TOL


def test_big_kkt_f64_cfg5_shape_N512(lqrx, gpu_ok):
    """BASELINE configs[4]'s KKT shape (n=64, m=32, w=96) over the full N=512 horizon, fp64."""
    import lqrx.kkt as K

    st = K.trajectory_structure(64, 32, 512)
    pb = K.random_kkt(st, 3, seed=512, h_mode=K.H_DIAG, dyn="dense")
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert traj_rel(got["dz"], ref["dz"]) <= TOL
    assert traj_rel(got["lam"], ref["lam"]) <= TOL


@pytest.mark.parametrize("n,m", CASES)
@pytest.mark.parametrize("N", [9, 128])
def test_big_kkt_f32(lqrx, gpu_ok, n, m, N):
    """fp32 (dtype LQRX_F32) against the fp64 oracle on the same fp32-rounded inputs."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, N)
    pb = _round32(K.random_kkt(st, 6, seed=7 * n + N, h_mode=K.H_DIAG, dyn="dense"))
    got = K.kkt_solve(pb, dtype=lqrx.F32)
    ref = _ref(st, pb)
    assert got["dz"].dtype == np.float32
    assert got["rc"] == 0 and (got["info"] == 0).all()
    e = max(traj_rel(got["dz"], ref["dz"]), traj_rel(got["lam"], ref["lam"]))
    print(f"fp32 n={n} m={m} N={N}: max rel err {e:.3e}")
    assert e <= F32_TOL


def test_big_kkt_f32_cfg5_N512(lqrx, gpu_ok):
    """configs[4] shape and precision over the full horizon (n=64 m=32 N=512 fp32)."""
    import lqrx.kkt as K

    st = K.trajectory_structure(64, 32, 512)
    pb = _round32(K.random_kkt(st, 4, seed=55, h_mode=K.H_DIAG, dyn="dense"))
    got = K.kkt_solve(pb, dtype=lqrx.F32)
    ref = _ref(st, pb)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    e = max(traj_rel(got["dz"], ref["dz"]), traj_rel(got["lam"], ref["lam"]))
    print(f"fp32 cfg5 N=512: max rel err {e:.3e}")
    assert e <= F32_TOL


@pytest.mark.parametrize("n,m,ps", [(8, 4, 3), (16, 8, 5), (32, 16, 14), (20, 24, 17)])
def test_big_kkt_stage_constraints(lqrx, gpu_ok, n, m, ps):
    """Interior stage constraints (C rows in every block: B, D, E Schur blocks, B̃ factor and
    Ẽ at every knot), block sizes off the 16 grid.  ps ≤ ((N−1)m − n)/(N−2) keeps the rows of
    D no more than its columns (D H⁻¹ Dᵀ nonsingular)."""
    import lqrx.kkt as K

    N = 23
    st = K.ConstraintBlocks(n, m, N, [n] + [ps] * (N - 2) + [n])
    pb = K.random_kkt(st, 4, seed=ps + n, h_mode=K.H_DIAG, dyn="dense")
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert traj_rel(got["dz"], ref["dz"]) <= TOL
    assert traj_rel(got["lam"], ref["lam"]) <= TOL


@pytest.mark.parametrize("n,m", [(16, 8), (64, 32)])
def test_big_kkt_soc(lqrx, gpu_ok, n, m):
    """second_order_correction! (Ginv = false, cholesky_solver.jl:254-273): H = I, r = 0."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, 17)
    pb = K.random_kkt(st, 3, seed=n, h_mode=K.H_DIAG, dyn="dense")
    got = K.kkt_solve(pb, ginv=0)
    ref = _ref(st, pb, ginv=0)
    assert traj_rel(got["dz"], ref["dz"]) <= TOL
    assert traj_rel(got["lam"], ref["lam"]) <= TOL


@pytest.mark.parametrize("n,m,N", [(5, 3, 101), (7, 2, 101)])
def test_generic_structures_without_compile_time_shape(lqrx, gpu_ok, n, m, N):
    """Structures outside the compile-time shapes and past the small lane kernels (their
    (8,8,8,12,16) maxima spilled to scratch) now run on the large-block kernels."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, N)
    pb = K.random_kkt(st, 70, seed=n, h_mode=K.H_DIAG)
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert got["rc"] == 0
    assert traj_rel(got["dz"], ref["dz"]) <= TOL
    assert traj_rel(got["lam"], ref["lam"]) <= TOL


def test_big_kkt_info_first_failing_knot(lqrx, gpu_ok):
    """A negative cost weight makes a Schur pivot block indefinite part-way along the horizon:
    info = the first knot whose potrf fails (cholesky_solve.jl:53/62), equal to the oracle's;
    untouched trajectories stay 0."""
    import lqrx.kkt as K

    st = K.trajectory_structure(16, 8, 21)
    pb = K.random_kkt(st, 4, seed=3, h_mode=K.H_DIAG, dyn="dense")
    sg = int(np.sum(st.w))
    og = int(np.sum(st.w[:9]))
    pb.H[1, og:og + st.w[9]] = -5.0                    # knot 9 of trajectory 1
    pb.H[3, og + int(st.w[9]):og + int(st.w[9]) + int(st.w[10])] *= -1.0   # knot 10 of trajectory 3
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert got["rc"] == 1
    assert list(got["info"]) == list(ref["info"]), (got["info"], ref["info"])
    assert got["info"][0] == 0 and got["info"][2] == 0 and got["info"][1] > 0 and got["info"][3] > 0
    ok = [0, 2]
    assert traj_rel(got["dz"][ok], ref["dz"][ok]) <= TOL


def test_big_kkt_device_workspace(lqrx, gpu_ok):
    """Device entry (torch tensors, fp64 and fp32) with a caller-owned workspace
    (lqrx_kkt_solve_ws) equals the library-pool call bit for bit and the oracle."""
    import torch
    import lqrx.kkt as K

    st = K.trajectory_structure(32, 16, 19)
    bt = 9
    pb = K.random_kkt(st, bt, seed=4, h_mode=K.H_DIAG, dyn="dense")
    ref = _ref(_round32(pb).st, _round32(pb))
    dev = torch.device("cuda", 0)
    for dt, tol in ((torch.float64, TOL), (torch.float32, F32_TOL)):
        src = _round32(pb) if dt == torch.float32 else pb
        t = {k: torch.from_numpy(np.ascontiguousarray(getattr(src, k).ravel())).to(dev, dt) for k in ("Y", "y", "H", "g")}
        t["batch"] = bt
        ws = torch.empty(K.workspace_size(st, bt, K.H_DIAG, dtype=lqrx.F32 if dt == torch.float32 else lqrx.F64),
                         dtype=torch.uint8, device=dev)
        a = K.kkt_solve_device(st, t, K.H_DIAG, workspace=ws)
        b = K.kkt_solve_device(st, t, K.H_DIAG)
        torch.cuda.synchronize()
        assert torch.equal(a["dz"], b["dz"]) and torch.equal(a["lam"], b["lam"])
        r = ref if dt == torch.float32 else _ref(st, pb)
        assert traj_rel(a["dz"].view(bt, -1).double().cpu().numpy(), r["dz"]) <= tol
        assert traj_rel(a["lam"].view(bt, -1).double().cpu().numpy(), r["lam"]) <= tol


_CHUNK_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1] + "/lqr.jl_amd", sys.argv[1]]
import lqrx, lqrx.kkt as K
from oracle import oracle as orc
st = K.trajectory_structure(16, 8, 13)
pb = K.random_kkt(st, 11, seed=8, h_mode=K.H_DIAG, dyn="dense")
got = K.kkt_solve(pb)
ref = orc.kkt_solve_batch(orc.KktStructure(16, 8, 13, st.p), 11, pb.Y, pb.y, pb.H, pb.g, h_mode=2, nthreads=4)
e = np.abs(got["dz"] - ref["dz"].reshape(11, -1)).max() / np.abs(ref["dz"]).max()
print("chunked rel err", e)
sys.exit(0 if e <= 1e-10 and (got["info"] == 0).all() else 1)
"""


def test_big_kkt_slab_chunks(lqrx, gpu_ok, tmp_path):
    """A slab cap smaller than the batch needs (LQRX_KKT_BIG_SLAB_MB, read once per process —
    hence one child process) runs the batch in consecutive chunks through one slab."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "chunk.py"
    f.write_text(_CHUNK_SCRIPT)
    env = dict(os.environ, LQRX_KKT_BIG_SLAB_MB="0")     # 0 MB → one trajectory per chunk
    p = subprocess.run([sys.executable, str(f), root], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr


@pytest.mark.parametrize("n,m,N,h_mode", [(5, 2, 101, 0), (7, 3, 41, 1), (6, 3, 33, 0), (16, 8, 21, 0),
                                          (32, 16, 13, 1), (64, 32, 9, 0)])
def test_big_kkt_dense_h(lqrx, gpu_ok, n, m, N, h_mode):
    """Dense (h_mode 0) and block-diagonal (1) cost Hessians (BlockCholesky, block_cholesky.jl:
    55-77) on the large-block path: the hfac pre-pass factors each H_k (w up to 96 here, eight
    16-blocks), the sweeps run on Z = Y U⁻¹ and gz = U⁻ᵀg, and δz = −U⁻¹(Zᵀλ + gz).  Covers the
    structures the scratch-spilling lane<8,8,8,12,16> kernel used to serve with a dense H."""
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, N)
    pb = K.random_kkt(st, 4, seed=n + N + h_mode, h_mode=h_mode, dyn="dense" if n >= 8 else "small")
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    assert traj_rel(got["dz"], ref["dz"]) <= TOL
    assert traj_rel(got["lam"], ref["lam"]) <= TOL


def test_big_kkt_dense_h_f32(lqrx, gpu_ok):
    """fp32 with a dense H (n=32, m=16: w = 48)."""
    import lqrx.kkt as K

    st = K.trajectory_structure(32, 16, 33)
    pb = _round32(K.random_kkt(st, 3, seed=5, h_mode=K.H_DENSE, dyn="dense"))
    got = K.kkt_solve(pb, dtype=lqrx.F32)
    ref = _ref(st, pb)
    assert got["rc"] == 0 and (got["info"] == 0).all()
    e = max(traj_rel(got["dz"], ref["dz"]), traj_rel(got["lam"], ref["lam"]))
    print(f"fp32 dense H: max rel err {e:.3e}")
    assert e <= F32_TOL


def test_big_kkt_dense_h_info(lqrx, gpu_ok):
    """A non-SPD H_k reports info = −(k+1) for its first knot (the oracle's convention; the
    reference's potrf! at block_cholesky.jl:63 discards it), ahead of any Schur failure."""
    import lqrx.kkt as K

    st = K.trajectory_structure(16, 8, 15)
    pb = K.random_kkt(st, 3, seed=9, h_mode=K.H_DENSE, dyn="dense")
    w = st.w.astype(int)
    o = int(np.sum(w[:6] * w[:6]))
    pb.H[2, o:o + w[6] * w[6]] *= -1.0                   # H at knot 6 (0-based) of trajectory 2
    got = K.kkt_solve(pb)
    ref = _ref(st, pb)
    assert ref["info"][2] == -7
    assert list(got["info"]) == list(ref["info"])
    assert traj_rel(got["dz"][:2], ref["dz"][:2]) <= TOL


_FUSED_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1] + "/lqr.jl_amd", sys.argv[1]]
import lqrx, lqrx.kkt as K
from oracle import oracle as orc
worst = 0.0
for n, m, N, dt in ((16, 8, 21, lqrx.F64), (64, 32, 9, lqrx.F64), (32, 16, 13, lqrx.F32), (8, 4, 17, lqrx.F32),
                    (40, 12, 11, lqrx.F64), (64, 32, 33, lqrx.F32)):
    st = K.trajectory_structure(n, m, N)
    pb = K.random_kkt(st, 3, seed=n + N, h_mode=K.H_DIAG, dyn="dense")
    if dt == lqrx.F32:
        import dataclasses
        f = lambda a: np.asarray(a, np.float32).astype(np.float64)
        pb = dataclasses.replace(pb, Y=f(pb.Y), y=f(pb.y), H=f(pb.H), g=f(pb.g))
    got = K.kkt_solve(pb, dtype=dt)
    ref = orc.kkt_solve_batch(orc.KktStructure(n, m, N, st.p), 3, pb.Y, pb.y, pb.H, pb.g, h_mode=2, nthreads=4)
    r = ref["dz"].reshape(3, -1)
    e = (np.abs(np.asarray(got["dz"], np.float64) - r).max(axis=1) / np.abs(r).max(axis=1)).max()
    tol = 1e-10 if dt == lqrx.F64 else 1e-4
    print(n, m, N, dt, "rel err", e)
    if not (e <= tol and (got["info"] == 0).all()):
        sys.exit(1)
"""


@pytest.mark.parametrize("split,fuse", [("0", "1"), ("1", "0"), ("1", "1")])
def test_big_kkt_fused_and_split_forward(lqrx, gpu_ok, tmp_path, split, fuse):
    """Every forward sweep of the large-block path on the trajectory structure: the split path
    with the interior knots on the fused one-wave Schur+factor kernel (default), the split path
    with Schur images + kb_factor_mid_kernel (LQRX_KKT_FUSE=0), and the one-workgroup-per-
    trajectory kernel (LQRX_KKT_SPLIT=0, which every structure with stage constraints at
    interior knots takes), fp64 and fp32, against the oracle (one child process each: the
    switches are read once per process)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "fused.py"
    f.write_text(_FUSED_SCRIPT)
    env = dict(os.environ, LQRX_KKT_SPLIT=split, LQRX_KKT_FUSE=fuse)
    p = subprocess.run([sys.executable, str(f), root], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr


@pytest.mark.parametrize("n,m,dt", [(5, 2, "f32"), (6, 3, "f32"), (6, 3, "f64")])
def test_big_kkt_y_tail_nan(lqrx, gpu_ok, n, m, dt):
    """Knot widths off the 4-column k-slice (w = n + m interior, w = n at the last knot) on the
    split Schur kernel, with Y a view followed by NaN-filled memory: the k-slices past a knot's
    last column must read 0 through the buffer descriptor's bound (the slice offset rides in
    the range-checked VGPR offset), not the memory after the block — at the batch's last knot
    that is past the caller's Y (a soffset slice read it, and 0·NaN poisoned the
    Schur tiles)."""
    import torch
    import lqrx.kkt as K

    st = K.trajectory_structure(n, m, 11)
    bt = 5
    pb = K.random_kkt(st, bt, seed=n + m, h_mode=K.H_DIAG)
    f32 = dt == "f32"
    if f32:
        pb = _round32(pb)
    tdt = torch.float32 if f32 else torch.float64
    dev = torch.device("cuda", 0)
    sY = pb.Y.size
    ybuf = torch.full((sY + 4096,), float("nan"), dtype=tdt, device=dev)
    ybuf[:sY] = torch.from_numpy(pb.Y.ravel()).to(dev, tdt)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(pb, k).ravel())).to(dev, tdt) for k in ("y", "H", "g")}
    t.update(Y=ybuf[:sY], batch=bt)
    got = K.kkt_solve_device(st, t, K.H_DIAG)
    torch.cuda.synchronize()
    ref = _ref(st, pb)
    dz = got["dz"].view(bt, -1).double().cpu().numpy()
    lam = got["lam"].view(bt, -1).double().cpu().numpy()
    assert np.isfinite(dz).all() and np.isfinite(lam).all()
    tol = F32_TOL if f32 else TOL
    assert traj_rel(dz, ref["dz"]) <= tol
    assert traj_rel(lam, ref["lam"]) <= tol
