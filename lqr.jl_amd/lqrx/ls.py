"""Host-side mirror of the reference's condensed least-squares LQR surface, backed by the
HIP kernel ``ls_condensed_kernel`` (lqr.jl_amd/csrc/lqrx_ls.hip) — SURVEY.md §8(f) rank 4.

Reference surface (Julia, /root/reference/src/least_squares.jl):
  LeastSquaresSolver(prob)               :30-56   opts :solve_type => :cholesky,
                                                  :matbuild => :Ab; Hu = 0
  buildAb!(solver, prob)                 :58-103
  build_least_squares!(solver, prob)     :105-134 also fills Hu with chol(R).U blocks
  solve!(sol, solver, prob)              :158-192 H = ĀᵀĀ + Hu, y = −Āᵀb̄, potrf/potrs, rollout!

Hu is solver state in the reference: zero for a fresh solver, chol(R).U blocks once a
:lsq build ran (and it stays so for later :Ab solves).  ``LeastSquaresSolver.hu_mode``
tracks exactly that; ``hu_mode = HU_R`` (extension) gives the LQR cost, whose optimum is
the DP rollout.  The :naive solve type throws in the reference (it assigns a flat vector
into a Vector of views) and is rejected here.  No CPU fallback: compute is liblqrx.so.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .dp import LQRBatch, LQRProblem, to_abi

__all__ = ["LeastSquaresSolver", "Primals", "HU_ZERO", "HU_CHOL_R", "HU_R", "ls_solve",
           "ls_solve_batch", "ls_solve_device", "lds_bytes"]

HU_ZERO, HU_CHOL_R, HU_R = 0, 1, 2


@dataclass
class Primals:
    """Primals(n, m, N, tf) (lqr_problem.jl:46-75): Z = [x_1; u_1; …; x_{N−1}; u_{N−1}; x_N]
    with the X / U views; here X (N, n) and U (N−1, m) arrays plus the interleaved Z."""

    X: np.ndarray
    U: np.ndarray
    info: int = 0

    @classmethod
    def of(cls, prob: LQRProblem):
        n, m, N = prob.size()
        return cls(np.zeros((N, n)), np.zeros((N - 1, m)))

    @property
    def Z(self):
        N, n = self.X.shape
        parts = []
        for k in range(N - 1):
            parts += [self.X[k], self.U[k]]
        parts.append(self.X[N - 1])
        return np.concatenate(parts)

    @property
    def U_(self):
        return self.U.reshape(-1)


@dataclass
class LeastSquaresSolver:
    """LeastSquaresSolver(prob) (least_squares.jl:30-56).  The Julia struct owns dense
    scratch (H, Ā, b̄, T, L, Hx, Hu); here it lives in the kernel's LDS, so the solver keeps
    the shape, the options and the Hu state."""

    n: int
    m: int
    N: int
    opts: dict = field(default_factory=lambda: {"solve_type": "cholesky", "matbuild": "Ab"})
    hu_mode: int = HU_ZERO

    @classmethod
    def of(cls, prob: LQRProblem):
        n, m, N = prob.size()
        if (N - 1) * m > MAX_NM:
            raise _lib.LqrxError(_lib.ERR_UNSUPPORTED,
                                 f"n={n} m={m} N={N}: (N-1)m = {(N - 1) * m} > {MAX_NM} (LS kernel cap)")
        if lds_bytes(n, m, N) > 163840:
            raise _lib.LqrxError(_lib.ERR_UNSUPPORTED,
                                 f"n={n} m={m} N={N}: the condensed problem exceeds one CU's LDS")
        return cls(n, m, N)


MAX_NM = 1024     # (N−1)·m cap of ls_condensed_kernel (LS_BIG_MAX_NM, lqrx_ls.hip; above 192 H lives in
                  # global scratch with a blocked factor)


def lds_bytes(n: int, m: int, N: int) -> int:
    return int(_lib.load().lqrx_ls_lds_bytes(n, m, N))


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _check_symmetric(b: LQRBatch):
    """LeastSquaresSolver(prob) factors Q, Qf (and R) with cholesky() (least_squares.jl:50-52),
    which throws for a non-Hermitian matrix; the kernel reads only the upper triangles, so the
    check is made here, exactly as ishermitian() does (no tolerance)."""
    for name in ("Q", "Qf", "R"):
        a = np.asarray(getattr(b, name), dtype=np.float64)
        if not np.array_equal(a, np.swapaxes(a, -1, -2)):
            bad = int(np.flatnonzero([not np.array_equal(x, x.T) for x in a])[0])
            raise ValueError(f"{name} of trajectory {bad} is not symmetric "
                             "(cholesky() throws PosDefException there)")


def ls_solve_batch(b: LQRBatch, hu_mode: int = HU_ZERO) -> dict:
    """Batched solve! through lqrx_ls_solve_host.  Returns U (batch, N−1, m),
    X (batch, N, n), info (batch,), rc."""
    lib = _lib.load()
    n, m, N = b.size()
    if b.time_varying() != (0, 0):
        raise ValueError("LeastSquaresSolver is time-invariant (least_squares.jl:58-103)")
    bt = b.batch
    _check_symmetric(b)
    ins = [to_abi(np.asarray(x, dtype=np.float64)) for x in (b.A, b.B, b.Q, b.R, b.Qf)]
    x0 = np.ascontiguousarray(np.asarray(b.x0, dtype=np.float64))
    U = np.zeros(bt * (N - 1) * m)
    X = np.zeros(bt * N * n)
    info = np.zeros(bt, np.int32)
    d = _lib.LsDesc(n, m, N, hu_mode, bt)
    rc = _lib.check(lib.lqrx_ls_solve_host(C.byref(d), *[_ptr(a) for a in ins], _ptr(x0),
                                           _ptr(U), _ptr(X), _ptr(info)))
    return dict(U=U.reshape(bt, N - 1, m), X=X.reshape(bt, N, n), info=info, rc=rc)


def ls_solve(sol: Primals, solver: LeastSquaresSolver, prob: LQRProblem) -> Primals:
    """solve!(sol, ::LeastSquaresSolver, prob) (least_squares.jl:158-192)."""
    st = solver.opts.get("solve_type", "cholesky")
    if st != "cholesky":
        raise ValueError(f"solve_type {st!r}: only :cholesky is a working path upstream")
    mb = solver.opts.get("matbuild", "Ab")
    if mb == "lsq":               # build_least_squares! fills Hu with chol(R).U (:121)
        solver.hu_mode = HU_CHOL_R if solver.hu_mode == HU_ZERO else solver.hu_mode
    elif mb != "Ab":
        raise ValueError(f"matbuild {mb!r} (expected 'Ab' or 'lsq')")
    out = ls_solve_batch(LQRBatch.of([prob]), solver.hu_mode)
    sol.U[...] = out["U"][0]
    sol.X[...] = out["X"][0]
    sol.info = int(out["info"][0])
    return sol


def ls_solve_device(t: dict, N: int, hu_mode: int = HU_ZERO, stream: int | None = None,
                    out: dict | None = None, with_Ab: bool = False) -> dict:
    """Device-pointer entry on torch tensors in ABI layout (flat float64 A, B, Q, R, Qf, x0
    on the GPU; ints n, m, batch).  with_Ab also returns buildAb!'s Ā and b̄."""
    import torch

    lib = _lib.load()
    n, m, bt = t["n"], t["m"], t["batch"]
    dev = t["A"].device
    f64 = torch.float64
    if out is None:
        out = dict(U=torch.empty(bt * (N - 1) * m, dtype=f64, device=dev),
                   X=torch.empty(bt * N * n, dtype=f64, device=dev),
                   info=torch.empty(bt, dtype=torch.int32, device=dev))
        if with_Ab:
            out["Ab"] = torch.empty(bt * N * n * (N - 1) * m, dtype=f64, device=dev)
            out["bb"] = torch.empty(bt * N * n, dtype=f64, device=dev)
    d = _lib.LsDesc(n, m, N, hu_mode, bt)
    p = lambda x: C.c_void_p(x.data_ptr()) if x is not None else None
    rc = lib.lqrx_ls_solve(C.byref(d), p(t["A"]), p(t["B"]), p(t["Q"]), p(t["R"]), p(t["Qf"]),
                           p(t["x0"]), p(out["U"]), p(out["X"]), p(out["info"]),
                           p(out.get("Ab")), p(out.get("bb")),
                           C.c_void_p(stream) if stream else None)
    _lib.check(rc)
    out["rc"] = rc
    return out
