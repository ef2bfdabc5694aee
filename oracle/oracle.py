"""CPU ORACLE (test infrastructure only) — Python side.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker.  Wraps oracle/liblqr_oracle.so (the plain-C restatement in lqr_oracle.c, which
cites the reference lines it follows) and adds numpy identities used to PIN it:

  * dp_dense_kkt:  the DP rollout must equal the optimum of the equality-constrained QP
      min Σ ½xᵀQx + ½uᵀRu + ½x_Nᵀ Qf x_N  s.t. x1 = x0, x_{k+1} = A x_k + B u_k
    solved densely (the reference's own DP≡KKT equivalence).
  * kkt_dense: the dense quantities test/cholesky_solve.jl:18-44 compares against
      S = D H⁻¹Dᵀ, r = D H⁻¹g − d, λ = −S⁻¹r, δz = −H⁻¹(Dᵀλ + g), full KKT solve.
Parity status: KKT pinned by the reference's known-answer identities; DP pinned by
identities only (the reference's DP test holds no assertion and Julia is unavailable).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblqr_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = C.CDLL(LIB_PATH)
        vp, i32, i64 = C.c_void_p, C.c_int, C.c_int64
        lib.oracle_dp_solve_batch.restype = i64
        lib.oracle_dp_solve_batch.argtypes = [i32, i32, i32, i64] + [vp] * 8 + [i32, vp, vp, vp,
                                                                                 i32]
        lib.oracle_dp_solve_batch_tv.restype = i64
        lib.oracle_dp_solve_batch_tv.argtypes = [i32, i32, i32, i64] + [vp] * 8 + [
            i32, vp, vp, vp, i32, i32, i32]
        lib.oracle_dp_solve_batch_lin.restype = i64
        lib.oracle_dp_solve_batch_lin.argtypes = [i32, i32, i32, i64] + [vp] * 8 + [
            i32, vp, vp, vp, i32, i32, i32] + [vp] * 5
        lib.oracle_kkt_solve_one.restype = i32
        lib.oracle_kkt_solve_one.argtypes = [i32, vp, vp, vp, vp, vp, vp, i32, vp, vp, i32, vp,
                                             vp, vp, vp, vp]
        lib.oracle_kkt_solve_batch.restype = i64
        lib.oracle_kkt_solve_batch.argtypes = [i32, vp, vp, vp, vp, i64, vp, vp, i32, vp, vp,
                                               i32, vp, vp, vp, i32]
        lib.oracle_kkt_lower_one.restype = i32
        lib.oracle_kkt_lower_one.argtypes = [i32, vp, vp, vp, vp, vp, vp, i32, vp, vp, i32, vp,
                                             vp, vp]
        lib.oracle_num_threads_max.restype = i32
        _lib = lib
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


# ------------------------------------------------------------------------- DP
def dp_solve_abi(d: dict, N: int, all_P: bool = False, nthreads: int = 1) -> dict:
    """Oracle DP on ABI-layout (flat, column-major, batch slowest) float64 inputs.
    d["tv_AB"] / d["tv_QR"] (optional, default 0) select per-knot A,B / Q,R (N−1 knots per
    trajectory, the time-varying extension of SURVEY §8(f))."""
    lib = load()
    n, m, bt = d["n"], d["m"], d["batch"]
    f = lambda k: np.ascontiguousarray(np.asarray(d[k], dtype=np.float64))
    A, B, Q, R, Qf, x0 = (f(k) for k in ("A", "B", "Q", "R", "Qf", "x0"))
    K = np.zeros(bt * (N - 1) * m * n)
    P = np.zeros(bt * n * n * (N if all_P else 1))
    X = np.zeros(bt * N * n)
    U = np.zeros(bt * (N - 1) * m)
    info = np.zeros(bt, np.int32)
    lib.oracle_dp_solve_batch_tv(n, m, N, bt, _p(A), _p(B), _p(Q), _p(R), _p(Qf), _p(x0),
                                 _p(K), _p(P), 1 if all_P else 0, _p(X), _p(U), _p(info),
                                 nthreads, int(d.get("tv_AB", 0)), int(d.get("tv_QR", 0)))
    return dict(K=K, P=P, X=X, U=U, info=info)


def dp_solve_lin_abi(d: dict, N: int, all_P: bool = False, nthreads: int = 1) -> dict:
    """Oracle DP with linear cost terms (oracle_dp_solve_one_lin): d additionally holds the
    flat ABI arrays q (n per knot, N−1 knots when tv_QR), r (m, idem) and qf (n).  Returns
    K, P, X, U, info plus the feedforward d (m per knot) and the linear cost-to-go p."""
    lib = load()
    n, m, bt = d["n"], d["m"], d["batch"]
    f = lambda k: np.ascontiguousarray(np.asarray(d[k], dtype=np.float64))
    A, B, Q, R, Qf, x0, q, r, qf = (f(k) for k in ("A", "B", "Q", "R", "Qf", "x0", "q", "r", "qf"))
    K = np.zeros(bt * (N - 1) * m * n)
    P = np.zeros(bt * n * n * (N if all_P else 1))
    X = np.zeros(bt * N * n)
    U = np.zeros(bt * (N - 1) * m)
    dd = np.zeros(bt * (N - 1) * m)
    p = np.zeros(bt * n * (N if all_P else 1))
    info = np.zeros(bt, np.int32)
    lib.oracle_dp_solve_batch_lin(n, m, N, bt, _p(A), _p(B), _p(Q), _p(R), _p(Qf), _p(x0),
                                  _p(K), _p(P), 1 if all_P else 0, _p(X), _p(U), _p(info),
                                  nthreads, int(d.get("tv_AB", 0)), int(d.get("tv_QR", 0)),
                                  _p(q), _p(r), _p(qf), _p(dd), _p(p))
    return dict(K=K, P=P, X=X, U=U, info=info, d=dd, p=p)


def dp_lapack(A, B, Q, R, Qf, x0, N):
    """dynamic_programming.jl:28-72 for one problem through the same third-party arithmetic
    the reference calls: LAPACK dpotrf/dpotrs 'U' from OpenBLAS (scipy.linalg.lapack — Julia's
    LAPACK.potrf!/potrs! are OpenBLAS too) and OpenBLAS dgemm for the products (numpy @).
    Logical row-major matrices in; returns K (N−1, m, n), P (N, n, n), X (N, n), U (N−1, m)."""
    from scipy.linalg import lapack

    n, m = B.shape
    P = np.array(Qf, dtype=np.float64)                    # :58
    Ks = np.zeros((N - 1, m, n)); Ps = np.zeros((N, n, n)); Ps[N - 1] = P
    for k in range(N - 1, 0, -1):                        # :61
        PB = P @ B                                       # :38
        E = R + B.T @ PB                                 # :39
        PA = P @ A                                       # :40
        K = B.T @ PA                                     # :41
        c, info = lapack.dpotrf(E, lower=0, clean=0)     # :29 potrf!('U', E)
        K, info2 = lapack.dpotrs(c, K, lower=0)          # :30 potrs!('U', E, K)
        APB = A.T @ PB                                   # :50
        P = Q + A.T @ PA - APB @ K                       # :51
        Ks[k - 1] = K
        Ps[k - 1] = P
    X = np.zeros((N, n)); U = np.zeros((N - 1, m)); X[0] = x0
    for k in range(N - 1):                               # :66-70
        U[k] = -Ks[k] @ X[k]
        X[k + 1] = A @ X[k] + B @ U[k]
    return Ks, Ps, X, U


def dp_extended(A, B, Q, R, Qf, N):
    """The backward pass of dynamic_programming.jl:54-64 (compute_gain! :37-43 with
    chol_solve! :28-31, compute_ctg! :48-52, same op order) in x87 80-bit extended precision
    (np.longdouble, unit roundoff 5.4e-20 vs 1.1e-16), batched over trajectories.  Inputs are
    logical (batch, r, c) float64 arrays; returns K (batch, N−1, m, n) and P (batch, N, n, n)
    as longdouble — the near-exact answer that the fp64 oracle and the GPU are both measured
    against when a recursion is ill-conditioned (tests/test_dp_lane_gpu.py)."""
    ld = np.longdouble
    assert np.finfo(ld).eps < 1e-18, "needs x87 extended precision"
    A, B, Q, R, Qf = (np.asarray(x, dtype=ld) for x in (A, B, Q, R, Qf))
    bt, n, m = B.shape
    T = lambda M: np.swapaxes(M, 1, 2)
    P = Qf.copy()
    Ks = np.zeros((bt, N - 1, m, n), dtype=ld)
    Ps = np.zeros((bt, N, n, n), dtype=ld)
    Ps[:, N - 1] = P
    for k in range(N - 1, 0, -1):
        PB = P @ B                                   # :38
        E = R + T(B) @ PB                            # :39
        PA = P @ A                                   # :40
        K = T(B) @ PA                                # :41
        U = np.zeros_like(E)                         # :29 potrf 'U'
        for j in range(m):
            d = E[:, j, j] - (U[:, :j, j] ** 2).sum(axis=1)
            U[:, j, j] = np.sqrt(d)
            for c in range(j + 1, m):
                U[:, j, c] = (E[:, j, c] - (U[:, :j, j] * U[:, :j, c]).sum(axis=1)) / U[:, j, j]
        for i in range(m):                           # :30 potrs: Uᵀ Y = K, then U X = Y
            K[:, i] = (K[:, i] - (U[:, :i, i, None] * K[:, :i]).sum(axis=1)) / U[:, i, i, None]
        for i in range(m - 1, -1, -1):
            K[:, i] = (K[:, i] - (U[:, i, i + 1:, None] * K[:, i + 1:]).sum(axis=1)) / U[:, i, i, None]
        APB = T(A) @ PB                              # :50
        P = Q + T(A) @ PA - APB @ K                  # :51
        Ks[:, k - 1] = K
        Ps[:, k - 1] = P
    return Ks, Ps


def dp_dense_kkt(A, B, Q, R, Qf, x0, N, q=None, r=None, qf=None, with_lam=False):
    """Dense equality-constrained QP optimum of one LQR problem (logical row-major
    matrices).  Returns (X (N,n), U (N-1,m)).  Optional linear cost terms q (n or (N-1,n)),
    r (m or (N-1,m)), qf (n) add gᵀz to the objective; with_lam=True also returns the
    multipliers λ (N, n): λ[0] of the initial condition x₁ = x0 (the optimal cost's gradient
    in x0 is −λ[0] = P₁x₁ + p₁) and λ[k] of x_{k+1} = A x_k + B u_k − x_{k+1}, the costate
    λ[k] = P_{k+1}x_{k+1} + p_{k+1} (0-based knot k)."""
    n, m = B.shape[-2:]
    nz = N * n + (N - 1) * m
    H = np.zeros((nz, nz))
    g = np.zeros(nz)
    ix = lambda k: slice(k * (n + m), k * (n + m) + n)
    iu = lambda k: slice(k * (n + m) + n, k * (n + m) + n + m)
    for k in range(N - 1):
        H[ix(k), ix(k)] = Q
        H[iu(k), iu(k)] = R
        if q is not None:
            g[ix(k)] = q if np.ndim(q) == 1 else q[k]
            g[iu(k)] = r if np.ndim(r) == 1 else r[k]
    H[ix(N - 1), ix(N - 1)] = Qf
    if qf is not None:
        g[ix(N - 1)] = qf
    D = np.zeros((N * n, nz))
    d = np.zeros(N * n)
    D[0:n, ix(0)] = np.eye(n)
    d[0:n] = -x0
    for k in range(N - 1):
        r = slice((k + 1) * n, (k + 2) * n)
        D[r, ix(k)] = A
        D[r, iu(k)] = B
        D[r, ix(k + 1)] = -np.eye(n)
    Kkt = np.block([[H, D.T], [D, np.zeros((N * n, N * n))]])
    sol = np.linalg.solve(Kkt, np.concatenate([-g, -d]))
    z = sol[:nz]
    X = np.stack([z[ix(k)] for k in range(N)])
    U = np.stack([z[iu(k)] for k in range(N - 1)])
    if with_lam:
        return X, U, sol[nz:].reshape(N, n)
    return X, U


# ------------------------------------------------------------------------- KKT
class KktStructure:
    """Per-knot block sizes (conblocks.jl:403-425) for the dynamics + stage-constraint
    structure: n̄ = n (no Lie group), n1 = n for k>1, n2 = n for k<N, w = n + m·(k<N)."""

    def __init__(self, n: int, m: int, N: int, p):
        self.n, self.m, self.N = n, m, N
        p = np.broadcast_to(np.asarray(p, dtype=np.int32), (N,)).copy()
        self.p = p
        self.n1 = np.array([0] + [n] * (N - 1), np.int32)
        self.n2 = np.array([n] * (N - 1) + [0], np.int32)
        self.w = np.array([n + m] * (N - 1) + [n], np.int32)
        self.rows = self.n1 + self.p + self.n2
        self.sY = int(np.sum(self.rows * self.w))
        self.sy = int(np.sum(self.p + self.n2))
        self.sg = int(np.sum(self.w))
        self.P = self.sy

    def sH(self, h_mode):
        return self.sg if h_mode == 2 else int(np.sum(self.w * self.w))


def kkt_solve_one(st: KktStructure, Y, y, H, g, h_mode=2, ginv=1, debug=False):
    lib = load()
    dz = np.zeros(st.sg)
    lam = np.zeros(st.P)
    S = np.zeros(st.P * st.P) if debug else None
    U = np.zeros(st.P * st.P) if debug else None
    r = np.zeros(st.P) if debug else None
    f = lambda a: np.ascontiguousarray(a, dtype=np.float64)
    Y, y, H, g = f(Y), f(y), f(H), f(g)
    info = lib.oracle_kkt_solve_one(st.N, _p(st.n1), _p(st.p), _p(st.n2), _p(st.w), _p(Y), _p(y),
                                    h_mode, _p(H), _p(g), ginv, _p(dz), _p(lam), _p(S), _p(U),
                                    _p(r))
    out = dict(dz=dz, lam=lam, info=info)
    if debug:
        out.update(S=S.reshape(st.P, st.P, order="F"), U=U.reshape(st.P, st.P, order="F"), r=r)
    return out


def kkt_lower_one(st: KktStructure, Y, y, H, g, h_mode=2, ginv=1):
    """KKT-12: the lower-storage block Cholesky (cholesky_solve.jl:5-26) and the lower
    forward/backward substitutions (the commented text :146-168).  Returns the dense lower
    factor L (P×P), yv = L⁻¹r after the forward sweep, xv = S⁻¹r after the backward sweep,
    and info."""
    lib = load()
    L = np.zeros(st.P * st.P)
    yv = np.zeros(st.P)
    xv = np.zeros(st.P)
    f = lambda a: np.ascontiguousarray(a, dtype=np.float64)
    Y, y, H, g = f(Y), f(y), f(H), f(g)
    info = lib.oracle_kkt_lower_one(st.N, _p(st.n1), _p(st.p), _p(st.n2), _p(st.w), _p(Y), _p(y),
                                    h_mode, _p(H), _p(g), ginv, _p(L), _p(yv), _p(xv))
    return dict(L=L.reshape(st.P, st.P, order="F"), y=yv, x=xv, info=info)


def kkt_solve_batch(st: KktStructure, bt, Y, y, H, g, h_mode=2, ginv=1, nthreads=1):
    lib = load()
    dz = np.zeros(bt * st.sg)
    lam = np.zeros(bt * st.P)
    info = np.zeros(bt, np.int32)
    f = lambda a: np.ascontiguousarray(a, dtype=np.float64)
    Y, y, H, g = f(Y), f(y), f(H), f(g)
    lib.oracle_kkt_solve_batch(st.N, _p(st.n1), _p(st.p), _p(st.n2), _p(st.w), bt, _p(Y), _p(y),
                               h_mode, _p(H), _p(g), ginv, _p(dz), _p(lam), _p(info), nthreads)
    return dict(dz=dz, lam=lam, info=info)


def kkt_dense(st: KktStructure, Y, y, H, g, h_mode=2):
    """Dense assembly (copy_blocks!, conblocks.jl:429-442; build_H!) and the dense
    quantities of test/cholesky_solve.jl:18-44."""
    N = st.N
    NN, P = st.sg, st.P
    D = np.zeros((P, NN))
    d = np.zeros(P)
    Hd = np.zeros((NN, NN))
    gd = np.zeros(NN)
    oY = oy = oH = og = 0
    off1 = off2 = 0
    for k in range(N):
        rows, w = int(st.rows[k]), int(st.w[k])
        Yk = np.asarray(Y[oY:oY + rows * w]).reshape(w, rows).T
        D[off1:off1 + rows, off2:off2 + w] = Yk
        n1 = int(st.n1[k])
        d[off1 + n1:off1 + rows] = y[oy:oy + rows - n1]
        if h_mode == 2:
            Hd[off2:off2 + w, off2:off2 + w] = np.diag(H[oH:oH + w])
            oH += w
        else:
            Hd[off2:off2 + w, off2:off2 + w] = np.asarray(H[oH:oH + w * w]).reshape(w, w).T
            oH += w * w
        gd[off2:off2 + w] = g[og:og + w]
        oY += rows * w
        oy += rows - n1
        og += w
        off1 += n1 + int(st.p[k])
        off2 += w
    HiDt = np.linalg.solve(Hd, D.T)
    S = D @ HiDt
    r = D @ np.linalg.solve(Hd, gd) - d
    lam = -np.linalg.solve(S, r)
    dz = -np.linalg.solve(Hd, D.T @ lam + gd)
    full = np.linalg.solve(np.block([[Hd, D.T], [D, np.zeros((P, P))]]), np.concatenate([-gd, -d]))
    return dict(D=D, d=d, H=Hd, g=gd, S=S, r=r, lam=lam, dz=dz, full=full)
