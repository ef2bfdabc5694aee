"""Problem construction feeding the hot path (the reference gets these from RobotZoo /
RobotDynamics, which are not available offline; SURVEY.md §8(c) lists the recalled
constants).  Only used to build LQRProblem inputs — never part of the solve.

  Cartpole (RobotZoo): mc = 1, mp = 0.2, l = 0.5, g = 9.81, state [x, θ, ẋ, θ̇];
      q̈ = −H⁻¹(C q̇ + G − B u)
  RK3 (RobotDynamics): k1 = f(x)dt; k2 = f(x + k1/2)dt; k3 = f(x − k1 + 2k2)dt;
      x⁺ = x + (k1 + 4k2 + k3)/6
  LQRProblem(model, Q, R, Qf, z0, N, tf): A, B = linearize(RK3, model, z0)
      (lqr_problem.jl:13-19); Jacobians here by complex-step differentiation (exact to
      rounding for these analytic dynamics, as ForwardDiff is in the reference).
"""
from __future__ import annotations

import numpy as np

from .dp import LQRProblem


def cartpole_dynamics(x, u, mc=1.0, mp=0.2, l=0.5, g=9.81):
    q, qd = x[:2], x[2:]
    s, c = np.sin(q[1]), np.cos(q[1])
    H = np.array([[mc + mp, mp * l * c], [mp * l * c, mp * l * l]], dtype=x.dtype)
    Cm = np.array([[0.0, -mp * qd[1] * l * s], [0.0, 0.0]], dtype=x.dtype)
    G = np.array([0.0, mp * g * l * s], dtype=x.dtype)
    B = np.array([1.0, 0.0], dtype=x.dtype)
    qdd = -np.linalg.solve(H, Cm @ qd + G - B * u[0])
    return np.concatenate([qd, qdd])


def rk3(f, x, u, dt):
    k1 = f(x, u) * dt
    k2 = f(x + k1 / 2, u) * dt
    k3 = f(x - k1 + 2 * k2, u) * dt
    return x + (k1 + 4 * k2 + k3) / 6


def linearize(f, x, u, dt, h=1e-30):
    """Discrete Jacobians (A, B) of rk3(f) at (x, u) by complex-step differentiation."""
    n, m = len(x), len(u)
    A = np.zeros((n, n))
    B = np.zeros((n, m))
    for i in range(n):
        e = np.zeros(n, complex)
        e[i] = 1j * h
        A[:, i] = np.imag(rk3(f, x.astype(complex) + e, u.astype(complex), dt)) / h
    for i in range(m):
        e = np.zeros(m, complex)
        e[i] = 1j * h
        B[:, i] = np.imag(rk3(f, x.astype(complex), u.astype(complex) + e, dt)) / h
    return A, B


def cartpole_problem(N=101, tf=5.0, x0=None, u0=0.01):
    """test/problems.jl:58-88 Cartpole: Q = 1e-2 I, R = 0.1, Qf = 100 I, linearised (RK3)
    at x = 0, u = 0.01 with dt = tf/(N−1)."""
    n, m = 4, 1
    dt = tf / (N - 1)
    xl = np.zeros(n)
    ul = np.array([u0])
    A, B = linearize(cartpole_dynamics, xl, ul, dt)
    Q = 1e-2 * np.eye(n)
    R = 1e-1 * np.eye(m)
    Qf = 100.0 * np.eye(n)
    x0 = np.zeros(n) if x0 is None else np.asarray(x0, dtype=float)
    return LQRProblem(Qf=Qf, Q=Q, R=R, A=A, B=B, x0=x0, u0=ul, tf=tf, N=N)


def cartpole_batch(batch, N=101, seed=0, sigma=0.1):
    """cfg2: the cartpole problem with per-trajectory x0 ~ N(0, σ²)."""
    from .dp import LQRBatch

    p = cartpole_problem(N)
    rng = np.random.default_rng(seed)
    rep = lambda M: np.broadcast_to(M, (batch,) + M.shape).copy()
    return LQRBatch(rep(p.A), rep(p.B), rep(p.Q), rep(p.R), rep(p.Qf),
                    sigma * rng.standard_normal((batch, 4)), N)
