"""Batched trajectory-optimisation SQP on the device (SURVEY.md §8(f) ranks 2–3) — host
mirror of the reference's CholeskySolver outer loop around the KKT path, for the reference's
test models: the Dubins car (test/dubins_sqp.jl, BASELINE cfg3), the cartpole
(test/problems.jl:58-88 Cartpole(), test/cartpole.jl) and the double integrator with its
interior-knot linear constraint (test/problems.jl:14-56 DoubleIntegrator(D)).

Reference (Julia, /root/reference):
  solve!/step!: ≤ 10 steps, convergence before each step   src/cholesky_solver.jl:109-153
  update!: cost + constraint expansion (TrajOptCore)         src/cholesky_solver.jl:155-164
  _solve! (the KKT kernel)                                   src/cholesky_solver.jl:166-182
  second_order_correction! (ginv = 0 KKT)                    src/cholesky_solver.jl:254-273
  f, c, merit ϕ = f + μ‖c‖₁, line search + SOC               test/dubins_sqp.jl:37-97
Compute goes through liblqrx.so (lqrx_sqp_solve[_host]); no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib

__all__ = ["SQPProblem", "DubinsSQP", "CartpoleSQP", "DoubleIntegratorSQP", "sqp_solve", "sqp_solve_device", "dubins_sqp_solve",
           "dubins_sqp_solve_device", "CONVERGED", "LIMIT", "LS_FAILED", "MODEL_DUBINS", "MODEL_CARTPOLE",
           "model_dims", "num_vars", "num_multipliers", "cartpole_rollout_guess"]

CONVERGED, LIMIT, LS_FAILED = 0, 1, 2
MODEL_DUBINS, MODEL_CARTPOLE = 0, 1           # LQRX_MODEL_*
MODEL_DOUBLE_INTEGRATOR = {1: 2, 2: 3, 3: 4}  # D → LQRX_MODEL_DOUBLE_INTEGRATOR{D}
_DIMS = {MODEL_DUBINS: (3, 2), MODEL_CARTPOLE: (4, 1), 2: (2, 1), 3: (4, 2), 4: (6, 3)}
CARTPOLE_PARAMS = (1.0, 0.2, 0.5, 9.81)       # RobotZoo.Cartpole(): mc, mp, l, g


def model_dims(model: int) -> tuple[int, int]:
    """(n, m) of a model (RobotDynamics size(model))."""
    if model not in _DIMS:
        raise ValueError(f"unknown model {model}")
    return _DIMS[model]


def num_vars(N: int, model: int = MODEL_DUBINS) -> int:
    """N·n + (N−1)·m (cholesky_solver.jl:104 num_vars)."""
    n, m = model_dims(model)
    return N * n + (N - 1) * m


def num_multipliers(N: int, model: int = MODEL_DUBINS, stage_rows: int = 0) -> int:
    """initial state + N−1 dynamics + goal, n rows each, + the stage rows of knots 2..N−1."""
    return model_dims(model)[0] * (N + 1) + stage_rows * (N - 2)


@dataclass
class SQPProblem:
    """Problem data shared by the batch (model, LQRObjective diagonal weights, horizon) +
    solver options (CholeskySolver defaults)."""

    model: int
    N: int
    dt: float
    Q: tuple
    R: tuple
    Qf: tuple
    params: tuple = (0.0, 0.0, 0.0, 0.0)
    mu: float = 1.0            # dubins_sqp.jl:59
    max_iters: int = 10        # cholesky_solver.jl:111
    tol_p: float = 1e-5        # :131-132
    tol_d: float = 1e-5
    stage_A: tuple = ()        # A_s (stage_rows × n) rows, shared by the batch; () = none
    stage_b: tuple = ()

    @property
    def stage_rows(self) -> int:
        return len(self.stage_b)

    @property
    def n(self) -> int:
        return model_dims(self.model)[0]

    @property
    def m(self) -> int:
        return model_dims(self.model)[1]

    def desc(self, batch: int) -> _lib.TrajSqpDesc:
        n, m = model_dims(self.model)
        if len(self.Q) != n or len(self.Qf) != n or len(self.R) != m:
            raise ValueError(f"Q, Qf need {n} entries and R {m} for model {self.model}")
        pad = lambda v: (C.c_double * 8)(*v)
        pk = self.stage_rows
        SA = np.asarray(self.stage_A, float).reshape(pk, n) if pk else np.zeros((0, n))
        return _lib.TrajSqpDesc(self.model, self.N, self.max_iters, pk, batch, self.dt, pad(self.Q), pad(self.R),
                                pad(self.Qf), (C.c_double * 4)(*self.params), self.mu, self.tol_p, self.tol_d,
                                (C.c_double * 32)(*SA.T.ravel()), (C.c_double * 4)(*self.stage_b))


def DubinsSQP(N: int, dt: float, Q=(1e-2,) * 3, R=(1e-1,) * 2, Qf=(100.0,) * 3, mu=1.0, max_iters=10,
              tol_p=1e-5, tol_d=1e-5) -> SQPProblem:
    """The Dubins car problem of test/dubins_sqp.jl (weights of test/problems.jl)."""
    return SQPProblem(MODEL_DUBINS, N, dt, tuple(Q), tuple(R), tuple(Qf), (0.0,) * 4, mu, max_iters, tol_p, tol_d)


def CartpoleSQP(N: int = 101, tf: float = 5.0, Q=(1e-2,) * 4, R=(1e-1,), Qf=(100.0,) * 4,
                params=CARTPOLE_PARAMS, mu=1.0, max_iters=10, tol_p=1e-5, tol_d=1e-5) -> SQPProblem:
    """Cartpole() of test/problems.jl:58-88: Q = 1e-2·I, R = 1e-1·I, Qf = 100·I, dt = tf/(N−1)."""
    return SQPProblem(MODEL_CARTPOLE, N, tf / (N - 1), tuple(Q), tuple(R), tuple(Qf), tuple(params), mu,
                      max_iters, tol_p, tol_d)


def DoubleIntegratorSQP(D: int = 3, N: int = 101, stage_A=None, stage_b=None, tf: float = 2.0, mu=10.0,
                        max_iters=10, tol_p=1e-5, tol_d=1e-5) -> SQPProblem:
    """DoubleIntegrator(D, N) of test/problems.jl:14-56: Q = diag(10·1_D, 1_D), R = 0.1·I,
    Qf = 10Q, dt = (N−1)/tf as the reference writes it (:19), and the planar LinearConstraint
    A_s x = b_s (p = max(D−2, 1) rows; the reference draws A_s = [rand(p,D) rand(p,D)], b = 0)
    on knots 2:N−1.  x0 = [1_D; 0_D] and xf = 0 are the solve's per-trajectory inputs."""
    Q = (10.0,) * D + (1.0,) * D
    p = max(D - 2, 1)
    if stage_A is None:
        stage_A = np.random.default_rng(1).random((p, 2 * D))
    stage_A = np.asarray(stage_A, float)
    stage_b = np.zeros(stage_A.shape[0]) if stage_b is None else np.asarray(stage_b, float)
    return SQPProblem(MODEL_DOUBLE_INTEGRATOR[D], N, (N - 1) / tf, Q, (0.1,) * D, tuple(10.0 * q for q in Q),
                      (0.0,) * 4, mu, max_iters, tol_p, tol_d, tuple(stage_A.ravel()), tuple(stage_b))


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def sqp_solve(prob: SQPProblem, Z0, x0, xf) -> dict:
    """Host arrays: Z0 (batch, N·n + (N−1)·m), x0, xf (batch, n).  Returns z, lam, iters, status."""
    lib = _lib.load()
    n = prob.n
    Z = np.ascontiguousarray(Z0, dtype=np.float64).copy()
    bt = Z.shape[0]
    if Z.shape[1] != num_vars(prob.N, prob.model):
        raise ValueError(f"Z0 has {Z.shape[1]} columns, the problem {num_vars(prob.N, prob.model)}")
    x0 = np.ascontiguousarray(np.broadcast_to(x0, (bt, n)), dtype=np.float64)
    xf = np.ascontiguousarray(np.broadcast_to(xf, (bt, n)), dtype=np.float64)
    lam = np.zeros((bt, num_multipliers(prob.N, prob.model, prob.stage_rows)))
    it = np.zeros(bt, np.int32)
    st = np.zeros(bt, np.int32)
    _lib.check(lib.lqrx_sqp_solve_host(C.byref(prob.desc(bt)), _ptr(Z), _ptr(x0), _ptr(xf), _ptr(lam), _ptr(it),
                                       _ptr(st)))
    return dict(z=Z, lam=lam, iters=it, status=st)


def sqp_solve_device(prob: SQPProblem, t: dict, stream: int | None = None) -> dict:
    """Device entry on torch tensors: t has Z (in/out), x0, xf, lam, iters, status."""
    lib = _lib.load()
    bt = t["x0"].numel() // prob.n
    p = lambda x: C.c_void_p(x.data_ptr())
    _lib.check(lib.lqrx_sqp_solve(C.byref(prob.desc(bt)), p(t["Z"]), p(t["x0"]), p(t["xf"]), p(t["lam"]),
                                  p(t["iters"]), p(t["status"]), C.c_void_p(stream) if stream else None))
    return t


# the round-1 Dubins names
dubins_sqp_solve = sqp_solve
dubins_sqp_solve_device = sqp_solve_device


def initial_guess(N: int, dt: float, x0, xf) -> np.ndarray:
    """Dubins: states interpolated from x0 to xf, controls at the straight-line speed and turn
    rate (a guess that violates the dynamics; the SQP removes the violation)."""
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


def _cartpole_f(x, u, params):
    """RobotZoo.Cartpole ẋ over leading batch dimensions (x[..., 4], u[..., 1])."""
    mc, mp, l, g = params
    s, c = np.sin(x[..., 1]), np.cos(x[..., 1])
    h01 = mp * l * c
    r0 = mp * l * s * x[..., 3] ** 2 + u[..., 0]
    r1 = -mp * g * l * s
    det = (mc + mp) * (mp * l * l) - h01 * h01
    return np.stack([x[..., 2], x[..., 3], ((mp * l * l) * r0 - h01 * r1) / det, ((mc + mp) * r1 - h01 * r0) / det],
                    -1)


def cartpole_rollout_guess(prob: SQPProblem, x0, u0: float = 0.01) -> np.ndarray:
    """The initial trajectory of Cartpole() (problems.jl:80-84): U0 = u0 everywhere and the
    states rolled out from x0 with RK3 (rollout!) — problem set-up on the host, as in the
    reference, before the solver runs.  x0 (4,) → z (NN,); x0 (B, 4) → Z (B, NN)."""
    dt, x = prob.dt, np.asarray(x0, float)
    u = np.full(x.shape[:-1] + (1,), float(u0))
    z = []
    for _ in range(prob.N - 1):
        z += [x, u]
        k1 = _cartpole_f(x, u, prob.params) * dt
        k2 = _cartpole_f(x + k1 / 2, u, prob.params) * dt
        k3 = _cartpole_f(x - k1 + 2 * k2, u, prob.params) * dt
        x = x + (k1 + 4 * k2 + k3) / 6
    z.append(x)
    return np.concatenate(z, -1)


def random_cartpole_batch(prob: SQPProblem, batch: int, seed: int, xf=(0.0, np.pi, 0.0, 0.0)):
    """Synthetic swing-up batch of Cartpole(): x0 ~ N(0, 0.05²) (trajectory 0 at rest, the
    reference's x0), goal xf, rollout guesses.  Returns x0, xf, Z0 (numpy, batch-major)."""
    rng = np.random.default_rng(seed)
    x0 = 0.05 * rng.standard_normal((batch, 4))
    x0[0] = 0.0
    xf = np.broadcast_to(np.asarray(xf, float), (batch, 4)).copy()
    return x0, xf, cartpole_rollout_guess(prob, x0)


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
