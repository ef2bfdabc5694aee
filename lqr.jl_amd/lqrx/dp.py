"""Host-side mirror of the reference's DP (Riccati) surface, backed by the HIP kernels.

Reference surface (Julia, /root/reference/src):
  LQRProblem{n,m,T}(Qf, Q, R, A, B, x0, u0, tf, N)        lqr_problem.jl:1-11
  size(prob) = (n, m, N); num_vars(prob) = N n + (N-1) m   lqr_problem.jl:21-25
  DPSolver(prob)                                           dynamic_programming.jl:13-23
  LQRSolution (exported, undefined upstream: fields K, X, U as used by :62-69)
  solve!(sol, solver, prob)                                dynamic_programming.jl:54-72
  compute_gain!(K, solver, prob), compute_ctg!(K, solver, prob)      :34-52 (per knot)
Extension (no upstream counterpart): linear cost terms q, r, qf on
LQRProblem / LQRBatch → feedforward d and linear cost-to-go p (lqrx_dp_solve_linear).

Array conventions here: a single problem uses plain (rows, cols) numpy matrices; batches
use numpy arrays shaped (batch, rows, cols).  The C ABI wants Julia column-major with the
batch slowest; ``to_abi``/``from_abi`` convert (a transpose of the last two axes).
Every compute call goes through liblqrx.so — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib

__all__ = ["LQRProblem", "LQRSolution", "DPSolver", "solve", "solve_batch", "LQRBatch",
           "random_batch", "to_abi", "from_abi", "dp_solve_device", "compute_gain", "compute_ctg",
           "compute_ctg_batch"]


def to_abi(a: np.ndarray) -> np.ndarray:
    """(batch, r, c) row-major logical matrices → contiguous column-major-per-matrix."""
    a = np.asarray(a)
    if a.ndim == 2:  # vectors (batch, r)
        return np.ascontiguousarray(a)
    return np.ascontiguousarray(np.swapaxes(a, -1, -2))


def to_soa(flat: np.ndarray, batch: int) -> np.ndarray:
    """Layout-0 flat buffer (batch slowest) → ABI layout 1 (batch fastest): [S][batch]."""
    return np.ascontiguousarray(np.asarray(flat).reshape(batch, -1).T)


def from_soa(soa: np.ndarray, batch: int) -> np.ndarray:
    """ABI layout 1 ([S][batch]) → the layout-0 flat buffer."""
    return np.ascontiguousarray(np.asarray(soa).reshape(-1, batch).T).ravel()


def from_abi(a: np.ndarray, shape: tuple) -> np.ndarray:
    """Inverse of to_abi: flat ABI buffer → (…, r, c) logical matrices."""
    *lead, r, c = shape
    return np.swapaxes(np.asarray(a).reshape(*lead, c, r), -1, -2)


@dataclass
class LQRProblem:
    """Finite-horizon LQR problem (lqr_problem.jl:1-11).  Time-invariant as upstream;
    A/B (and Q/R) may instead carry a leading knot axis of length N-1 (per-knot A_k, B_k,
    the LCRProblem layout of constrained_problem.jl:3-4)."""

    Qf: np.ndarray
    Q: np.ndarray
    R: np.ndarray
    A: np.ndarray
    B: np.ndarray
    x0: np.ndarray
    u0: np.ndarray | None = None
    tf: float = 1.0
    N: int = 2
    # linear cost terms (extension): stage ½xᵀQx + qᵀx + ½uᵀRu + rᵀu, terminal + qfᵀx;
    # q, r time-invariant or with a leading knot axis N-1 (then Q, R must carry one too)
    q: np.ndarray | None = None
    r: np.ndarray | None = None
    qf: np.ndarray | None = None

    def size(self):
        n, m = self.B.shape[-2:]
        return n, m, self.N

    def num_vars(self):
        n, m, N = self.size()
        return N * n + (N - 1) * m


@dataclass
class LQRSolution:
    """Output container the reference exports but never defines.

    K[k] (m×n) for k = 1..N-1 stored at index k-1; X[k] (n), U[k] (m); P = P_1 (what
    solver.P holds after solve!) or all P_k when constructed with all_P=True.
    """

    K: np.ndarray
    X: np.ndarray
    U: np.ndarray
    P: np.ndarray
    info: int = 0
    d: np.ndarray | None = None   # feedforward (linear terms): u_k = −K_k x_k − d_k
    p: np.ndarray | None = None   # linear cost-to-go p_1 (or every p_k with all_P)

    @classmethod
    def of(cls, prob: LQRProblem, all_P: bool = False):
        n, m, N = prob.size()
        lin = prob.q is not None
        return cls(np.zeros((N - 1, m, n)), np.zeros((N, n)), np.zeros((N - 1, m)),
                   np.zeros((N, n, n)) if all_P else np.zeros((n, n)),
                   d=np.zeros((N - 1, m)) if lin else None,
                   p=(np.zeros((N, n)) if all_P else np.zeros(n)) if lin else None)


@dataclass
class DPSolver:
    """DPSolver(prob) (dynamic_programming.jl:13-23).  The Julia struct owns scratch
    (P, P_, PA, PB, APB, E); here the products live in registers/LDS inside the kernel, so
    the solver records the problem shape and dtype plus the two matrices the reference's
    per-knot surface reads and writes: P (the cost-to-go compute_gain!/compute_ctg! start
    from, zero as upstream) and P_ (what compute_ctg! produces)."""

    n: int
    m: int
    N: int
    dtype: int = _lib.F64
    P: np.ndarray | None = None
    P_: np.ndarray | None = None

    @classmethod
    def of(cls, prob: LQRProblem, dtype: int = _lib.F64):
        n, m, N = prob.size()
        return cls(n, m, N, dtype, np.zeros((n, n)), np.zeros((n, n)))


@dataclass
class LQRBatch:
    """A batch of LQRProblems with the same (n, m, N), arrays shaped (batch, r, c)."""

    A: np.ndarray
    B: np.ndarray
    Q: np.ndarray
    R: np.ndarray
    Qf: np.ndarray
    x0: np.ndarray
    N: int
    extra: dict = field(default_factory=dict)
    q: np.ndarray | None = None    # (batch, n) or (batch, N-1, n) — linear terms (extension)
    r: np.ndarray | None = None    # (batch, m) or (batch, N-1, m)
    qf: np.ndarray | None = None   # (batch, n)

    @property
    def batch(self):
        return self.A.shape[0]

    def size(self):
        return self.B.shape[-2], self.B.shape[-1], self.N

    def time_varying(self):
        """(tv_AB, tv_QR): 1 where the fields carry a knot axis, A (batch, N-1, n, n) —
        the per-knot LCRProblem layout (constrained_problem.jl:3-4), SURVEY §8(f) rank 1."""
        return int(np.ndim(self.A) == 4), int(np.ndim(self.Q) == 4)

    @classmethod
    def of(cls, probs: list[LQRProblem]):
        """Stack problems; a 1-D Q, Qf or R is a diagonal (the reference's LQRProblem allows
        TQ, TR = Diagonal, lqr_problem.jl:1-4) and is densified."""
        def field_(p, f):
            a = np.asarray(getattr(p, f), dtype=np.float64)
            return np.diag(a) if f in ("Q", "Qf", "R") and a.ndim == 1 else a
        st = lambda f: np.stack([field_(p, f) for p in probs])
        lin = probs[0].q is not None
        return cls(st("A"), st("B"), st("Q"), st("R"), st("Qf"), st("x0"), probs[0].N,
                   q=st("q") if lin else None, r=st("r") if lin else None,
                   qf=st("qf") if lin else None)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _devices(devices):
    """(int32 array, ctypes pointer, count) for a devices= argument."""
    dv = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
    return dv, dv.ctypes.data_as(C.c_void_p), C.c_int32(len(dv))


def solve_batch(b: LQRBatch, dtype: int = _lib.F64, all_P: bool = False, layout: int = 0,
                devices=None):
    """Batched solve! through lqrx_dp_solve_host.  Returns dict of logical arrays
    K (batch, N-1, m, n), P (batch, n, n) or (batch, N, n, n), X (batch, N, n),
    U (batch, N-1, m), info (batch,), and the ABI return code.  layout = 1 hands the
    library batch-fastest (SoA) buffers (the conversion here is host-side bookkeeping; the
    result is the same logical arrays).  devices = [d0, d1, …] shards the batch over those
    GPUs in one call (lqrx_dp_solve[_linear]_host_devices; repeats allowed)."""
    lib = _lib.load()
    n, m, N = b.size()
    bt = b.batch
    tvAB, tvQR = b.time_varying()
    npdt = np.float64 if dtype == _lib.F64 else np.float32
    ins = [to_abi(np.asarray(x, dtype=npdt)) for x in (b.A, b.B, b.Q, b.R, b.Qf)]
    x0 = np.ascontiguousarray(np.asarray(b.x0, dtype=npdt))
    if layout == 1:
        ins = [to_soa(a, bt) for a in ins]
        x0 = to_soa(x0, bt)
    K = np.zeros(bt * (N - 1) * m * n, npdt)
    P = np.zeros(bt * n * n * (N if all_P else 1), npdt)
    X = np.zeros(bt * N * n, npdt)
    U = np.zeros(bt * (N - 1) * m, npdt)
    info = np.zeros(bt, np.int32)
    d = _lib.DpDesc(n, m, N, dtype, bt, layout, 1 if all_P else 0, tvAB, tvQR)
    lin = b.q is not None
    if lin:   # linear cost terms: lqrx_dp_solve_linear_host
        if b.r is None or b.qf is None:
            raise ValueError("linear cost terms need q, r and qf together")
        kq = N - 1 if tvQR else 1
        vec = lambda a, w: np.ascontiguousarray(np.asarray(a, dtype=npdt).reshape(bt * kq * w))
        q, r = vec(b.q, n), vec(b.r, m)
        qf = np.ascontiguousarray(np.asarray(b.qf, dtype=npdt).reshape(bt * n))
        if layout == 1:
            q, r, qf = to_soa(q, bt), to_soa(r, bt), to_soa(qf, bt)
        dff = np.zeros(bt * (N - 1) * m, npdt)
        pv = np.zeros(bt * n * (N if all_P else 1), npdt)
        ln = _lib.DpLinear(_ptr(q).value, _ptr(r).value, _ptr(qf).value, _ptr(dff).value,
                           _ptr(pv).value)
        args = (C.byref(d), *[_ptr(a) for a in ins], _ptr(x0), C.byref(ln), _ptr(K), _ptr(P),
                _ptr(X), _ptr(U), _ptr(info))
        if devices is None:
            rc = _lib.check(lib.lqrx_dp_solve_linear_host(*args))
        else:
            dv, dp_, nd = _devices(devices)
            rc = _lib.check(lib.lqrx_dp_solve_linear_host_devices(*args, dp_, nd))
    else:
        args = (C.byref(d), *[_ptr(a) for a in ins], _ptr(x0), _ptr(K), _ptr(P), _ptr(X), _ptr(U),
                _ptr(info))
        if devices is None:
            rc = _lib.check(lib.lqrx_dp_solve_host(*args))
        else:
            dv, dp_, nd = _devices(devices)
            rc = _lib.check(lib.lqrx_dp_solve_host_devices(*args, dp_, nd))
    if layout == 1:
        K, P, X, U = (from_soa(a, bt) for a in (K, P, X, U))
        if lin:
            dff, pv = from_soa(dff, bt), from_soa(pv, bt)
    out = dict(K=from_abi(K, (bt, N - 1, m, n)),
               P=from_abi(P, (bt, N, n, n) if all_P else (bt, n, n)),
               X=X.reshape(bt, N, n), U=U.reshape(bt, N - 1, m), info=info, rc=rc)
    if lin:
        out["d"] = dff.reshape(bt, N - 1, m)
        out["p"] = pv.reshape(bt, N, n) if all_P else pv.reshape(bt, n)
    return out


def solve(sol: LQRSolution, solver: DPSolver, prob: LQRProblem) -> LQRSolution:
    """solve!(sol, solver, prob) — dynamic_programming.jl:54-72 (one problem)."""
    all_P = sol.P.ndim == 3
    out = solve_batch(LQRBatch.of([prob]), solver.dtype, all_P)
    sol.K[...] = out["K"][0]
    sol.X[...] = out["X"][0]
    sol.U[...] = out["U"][0]
    sol.P[...] = out["P"][0]
    sol.info = int(out["info"][0])
    if prob.q is not None:
        sol.d = out["d"][0]
        sol.p = out["p"][0]
    return sol


def compute_ctg_batch(A, B, Q, R, P, dtype: int = _lib.F64, gain_only: bool = False):
    """compute_ctg! (dynamic_programming.jl:45-52; compute_gain! :34-43 with gain_only) for a
    batch through lqrx_dp_compute_ctg_host: A (batch, n, n), B (batch, n, m), Q, R, and
    P = solver.P (batch, n, n).  Returns K (batch, m, n), P_ (batch, n, n) (None with
    gain_only), info (batch,), rc."""
    lib = _lib.load()
    A = np.asarray(A)
    bt, n, m = A.shape[0], A.shape[-1], np.asarray(B).shape[-1]
    # the kernels' symmetric fast form needs symmetric P and Q (include/lqrx.h precondition);
    # the tolerance is relative to the largest entry and never tighter than 100 ulp of the
    # working dtype (an fp32 AᵀPA is symmetric only to fp32 rounding); Q never enters K, so a
    # gain-only call does not check it
    rtol = max(1e-10, 100.0 * float(np.finfo(np.float64 if dtype == _lib.F64 else np.float32).eps))
    for name, M in (("P", P),) + (() if gain_only else (("Q", Q),)):
        M = np.asarray(M, dtype=np.float64)
        if np.abs(M - np.swapaxes(M, -1, -2)).max(initial=0.0) > rtol * max(np.abs(M).max(initial=0.0), 1e-300):
            raise ValueError(f"compute_ctg: {name} must be symmetric (the Riccati cost-to-go / cost "
                             "Hessian; lqrx_dp_compute_ctg precondition)")
    npdt = np.float64 if dtype == _lib.F64 else np.float32
    ins = [to_abi(np.asarray(x, dtype=npdt)) for x in (A, B, Q, R, P)]
    K = np.zeros(bt * m * n, npdt)
    Pn = None if gain_only else np.zeros(bt * n * n, npdt)
    info = np.zeros(bt, np.int32)
    d = _lib.DpDesc(n, m, 2, dtype, bt, 0, 0, 0, 0)
    rc = _lib.check(lib.lqrx_dp_compute_ctg_host(C.byref(d), *[_ptr(a) for a in ins], _ptr(K),
                                                 None if Pn is None else _ptr(Pn), _ptr(info)))
    return dict(K=from_abi(K, (bt, m, n)), P_=None if Pn is None else from_abi(Pn, (bt, n, n)),
                info=info, rc=rc)


def compute_gain(K: np.ndarray, solver: DPSolver, prob: LQRProblem) -> np.ndarray:
    """compute_gain!(K, solver, prob) — dynamic_programming.jl:34-43: K = E⁻¹BᵀPA from
    P = solver.P (test/dp.jl:16 calls it on a fresh solver, P = 0)."""
    b = LQRBatch.of([prob])                       # densifies Diagonal Q / R
    out = compute_ctg_batch(b.A, b.B, b.Q, b.R, np.asarray(solver.P)[None], solver.dtype, gain_only=True)
    K[...] = out["K"][0]
    return K


def compute_ctg(K: np.ndarray, solver: DPSolver, prob: LQRProblem) -> np.ndarray:
    """compute_ctg!(K, solver, prob) — dynamic_programming.jl:45-52: the gain as above and
    solver.P_ = Q + AᵀPA − APB·K."""
    b = LQRBatch.of([prob])
    out = compute_ctg_batch(b.A, b.B, b.Q, b.R, np.asarray(solver.P)[None], solver.dtype)
    K[...] = out["K"][0]
    solver.P_[...] = out["P_"][0]
    return K


def random_batch(n: int, m: int, N: int, batch: int, seed: int, traj0: int = 0,
                 dtype: int = _lib.F64) -> dict:
    """Synthetic random-dense batch from the library's counter-based generator, returned
    in ABI layout (flat arrays) — the same bytes the bench feeds the kernel."""
    lib = _lib.load()
    npdt = np.float64 if dtype == _lib.F64 else np.float32
    A = np.empty(batch * n * n, npdt); B = np.empty(batch * n * m, npdt)
    Q = np.empty(batch * n * n, npdt); R = np.empty(batch * m * m, npdt)
    Qf = np.empty(batch * n * n, npdt); x0 = np.empty(batch * n, npdt)
    _lib.check(lib.lqrx_make_random_dp(n, m, batch, traj0, seed, dtype, _ptr(A), _ptr(B),
                                       _ptr(Q), _ptr(R), _ptr(Qf), _ptr(x0)))
    return dict(A=A, B=B, Q=Q, R=R, Qf=Qf, x0=x0, n=n, m=m, N=N, batch=batch)


def abi_to_batch(d: dict) -> LQRBatch:
    n, m, N, bt = d["n"], d["m"], d["N"], d["batch"]
    return LQRBatch(from_abi(d["A"], (bt, n, n)), from_abi(d["B"], (bt, n, m)),
                    from_abi(d["Q"], (bt, n, n)), from_abi(d["R"], (bt, m, m)),
                    from_abi(d["Qf"], (bt, n, n)), d["x0"].reshape(bt, n), N)


def dp_solve_device(t: dict, N: int, p_mode: int = 0, stream: int | None = None,
                    out: dict | None = None, layout: int = 0) -> dict:
    """Device-pointer entry point on torch tensors already in ABI layout (flat; layout 1 =
    batch fastest, every input and output).

    t: dict with torch tensors A, B, Q, R, Qf, x0 on the GPU and ints n, m, batch; with
    tensors q, r, qf as well it runs lqrx_dp_solve_linear and also returns d and p.
    Returns dict of output tensors (K, P, X, U, info[, d, p]).  `stream` is a raw hipStream_t
    (torch.cuda.current_stream().cuda_stream); None = the null stream, synchronous.
    """
    import torch

    lib = _lib.load()
    n, m, bt = t["n"], t["m"], t["batch"]
    tdt = t["A"].dtype
    dtype = _lib.F64 if tdt == torch.float64 else _lib.F32
    dev = t["A"].device
    if out is None:
        out = dict(K=torch.empty(bt * (N - 1) * m * n, dtype=tdt, device=dev),
                   P=torch.empty(bt * n * n * (N if p_mode else 1), dtype=tdt, device=dev),
                   X=torch.empty(bt * N * n, dtype=tdt, device=dev),
                   U=torch.empty(bt * (N - 1) * m, dtype=tdt, device=dev),
                   info=torch.empty(bt, dtype=torch.int32, device=dev))
    d = _lib.DpDesc(n, m, N, dtype, bt, layout, p_mode, int(t.get("tv_AB", 0)), int(t.get("tv_QR", 0)))
    p = lambda x: C.c_void_p(x.data_ptr())
    st = C.c_void_p(stream) if stream else None
    if t.get("q") is not None:
        if "d" not in out:
            out["d"] = torch.empty(bt * (N - 1) * m, dtype=tdt, device=dev)
            out["p"] = torch.empty(bt * n * (N if p_mode else 1), dtype=tdt, device=dev)
        ln = _lib.DpLinear(t["q"].data_ptr(), t["r"].data_ptr(), t["qf"].data_ptr(),
                           out["d"].data_ptr(), out["p"].data_ptr())
        rc = lib.lqrx_dp_solve_linear(C.byref(d), p(t["A"]), p(t["B"]), p(t["Q"]), p(t["R"]),
                                      p(t["Qf"]), p(t["x0"]), C.byref(ln), p(out["K"]),
                                      p(out["P"]), p(out["X"]), p(out["U"]), p(out["info"]), st)
    else:
        rc = lib.lqrx_dp_solve(C.byref(d), p(t["A"]), p(t["B"]), p(t["Q"]), p(t["R"]), p(t["Qf"]),
                               p(t["x0"]), p(out["K"]), p(out["P"]), p(out["X"]), p(out["U"]),
                               p(out["info"]), st)
    _lib.check(rc)
    out["rc"] = rc
    return out
