"""Batched Dubins-car SQP on the device (SURVEY.md §8(f) ranks 2–3) — host mirror of the
reference's CholeskySolver outer loop around the KKT path.

Reference (Julia, /root/reference):
  solve!/step!: ≤ 10 steps, convergence before each step   src/cholesky_solver.jl:109-153
  update!: cost + constraint expansion (TrajOptCore)         src/cholesky_solver.jl:155-164
  _solve! (the KKT kernel)                                   src/cholesky_solver.jl:166-182
  second_order_correction! (ginv = 0 KKT)                    src/cholesky_solver.jl:254-273
  f, c, merit ϕ = f + μ‖c‖₁, line search + SOC               test/dubins_sqp.jl:37-97
Compute goes through liblqrx.so (lqrx_dubins_sqp_solve[_host]); no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib

__all__ = ["DubinsSQP", "dubins_sqp_solve", "dubins_sqp_solve_device", "CONVERGED", "LIMIT",
           "LS_FAILED", "num_vars", "num_multipliers"]

CONVERGED, LIMIT, LS_FAILED = 0, 1, 2


def num_vars(N: int) -> int:
    """N·n + (N−1)·m (cholesky_solver.jl:104 num_vars) for the Dubins car n = 3, m = 2."""
    return 5 * N - 2


def num_multipliers(N: int) -> int:
    """initial state + N−1 dynamics + goal, 3 rows each."""
    return 3 * (N + 1)


@dataclass
class DubinsSQP:
    """Problem data shared by the batch (LQRObjective weights, horizon) + solver options."""

    N: int
    dt: float
    Q: tuple = (1e-2, 1e-2, 1e-2)
    R: tuple = (1e-1, 1e-1)
    Qf: tuple = (100.0, 100.0, 100.0)
    mu: float = 1.0            # dubins_sqp.jl:59
    max_iters: int = 10        # cholesky_solver.jl:111
    tol_p: float = 1e-5        # :131-132
    tol_d: float = 1e-5

    def desc(self, batch: int) -> _lib.SqpDesc:
        return _lib.SqpDesc(self.N, self.max_iters, batch, self.dt, (C.c_double * 3)(*self.Q),
                            (C.c_double * 2)(*self.R), (C.c_double * 3)(*self.Qf), self.mu,
                            self.tol_p, self.tol_d)


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def dubins_sqp_solve(prob: DubinsSQP, Z0, x0, xf) -> dict:
    """Host arrays: Z0 (batch, 5N−2), x0, xf (batch, 3).  Returns z, lam, iters, status."""
    lib = _lib.load()
    Z = np.ascontiguousarray(Z0, dtype=np.float64).copy()
    bt = Z.shape[0]
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    xf = np.ascontiguousarray(xf, dtype=np.float64)
    lam = np.zeros((bt, num_multipliers(prob.N)))
    it = np.zeros(bt, np.int32)
    st = np.zeros(bt, np.int32)
    _lib.check(lib.lqrx_dubins_sqp_solve_host(C.byref(prob.desc(bt)), _ptr(Z), _ptr(x0), _ptr(xf), _ptr(lam),
                                              _ptr(it), _ptr(st)))
    return dict(z=Z, lam=lam, iters=it, status=st)


def dubins_sqp_solve_device(prob: DubinsSQP, t: dict, stream: int | None = None) -> dict:
    """Device entry on torch tensors: t has Z (in/out), x0, xf, lam, iters, status."""
    lib = _lib.load()
    bt = t["x0"].numel() // 3
    p = lambda x: C.c_void_p(x.data_ptr())
    _lib.check(lib.lqrx_dubins_sqp_solve(C.byref(prob.desc(bt)), p(t["Z"]), p(t["x0"]), p(t["xf"]),
                                         p(t["lam"]), p(t["iters"]), p(t["status"]),
                                         C.c_void_p(stream) if stream else None))
    return t


def initial_guess(N: int, dt: float, x0, xf) -> np.ndarray:
    """States interpolated from x0 to xf, controls at the straight-line speed and turn rate
    (a guess that violates the dynamics; the SQP removes the violation)."""
    x0, xf = np.asarray(x0, float), np.asarray(xf, float)
    z = np.zeros(num_vars(N))
    T = dt * (N - 1)
    v = np.hypot(*(xf[:2] - x0[:2])) / T
    om = (xf[2] - x0[2]) / T
    for k in range(N):
        s = k / (N - 1)
        z[5 * k:5 * k + 3] = (1 - s) * x0 + s * xf
        if k < N - 1:
            z[5 * k + 3:5 * k + 5] = [v, om]
    return z


def random_dubins_batch(N: int, batch: int, seed: int, tf: float = 3.0):
    """Synthetic cfg3-shaped SQP batch: x0 ~ N(0, 0.1²), goals uniform in [−4, 4]² × [−3, 3],
    perturbed straight-line guesses.  Returns dt, x0, xf, Z0 (numpy, batch-major)."""
    rng = np.random.default_rng(seed)
    dt = tf / (N - 1)
    x0 = 0.1 * rng.standard_normal((batch, 3))
    xf = np.stack([rng.uniform(-4, 4, batch), rng.uniform(-4, 4, batch), rng.uniform(-3, 3, batch)], 1)
    Z0 = np.stack([initial_guess(N, dt, x0[b], xf[b]) for b in range(batch)])
    Z0 += 0.3 * rng.standard_normal(Z0.shape)
    return dt, x0, xf, Z0
