"""Trajectory SQP oracle (Dubins car, cartpole) — TEST INFRASTRUCTURE ONLY (CPU restatement, numpy).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module;
the product path (lqrx.sqp → liblqrx.so) never does.

The reference's explicit SQP specification is /root/reference/test/dubins_sqp.jl:
  objective f(Z)                             :37-42  (LQRObjective: Σ ½(x−xf)ᵀQ(x−xf) + ½uᵀRu,
                                                      terminal ½(x−xf)ᵀQf(x−xf); Q, R, Qf diagonal)
  constraints c(Z)                           :47-55  (x₁ − x0; discrete_dynamics(RK3, x_k, u_k) − x_{k+1})
                                                      plus the goal x_N − xf that the cfg3 block
                                                      structure carries (problems.jl:44-45 GoalConstraint)
  merit ϕ = f + μ‖c‖₁, ϕ′ = ∇fᵀdx − μ‖c‖₁      :58-61
  Newton KKT [∇²f ∇cᵀ; ∇c 0][dx; λ] = −[∇f; c]  :64-70, with ∇²f the cost Hessian (the
                                                      CholeskySolver's expansion, cholesky_solver.jl:155-164)
  backtracking line search + second-order correction  :74-97  (η = 1e-4, ρ = 0.5, 10 tries;
                                                      dx̂ = −Aᵀ(AAᵀ)⁻¹c(x + dx), A = ∇c(x))
and the outer loop of CholeskySolver.solve!/step! (cholesky_solver.jl:109-153): at most
`iters` (10) steps; a trajectory stops when ‖c‖∞ < tol_p and ‖∇f + ∇cᵀλ‖₂ < tol_d, checked
before its step with the λ of its previous Newton solve (zero at the start).  A line search
that finds no acceptable step leaves the iterate unchanged and ends that trajectory
(status 2; the script only warns, :96).

The same loop serves the cartpole of test/problems.jl:58-88 (Cartpole(): Q = 1e-2·I,
R = 1e-1·I, Qf = 100·I, x0 = 0, xf = [0, π, 0, 0], tf = 5, U0 = 0.01 rolled out from x0;
the SQP of test/cartpole.jl drives the same update! / _solve! / L1-merit pieces).

Parity anchor: the reference's own functions above.  TrajOptCore / RobotZoo are absent, so the
models — RobotZoo.DubinsCar: ẋ = [v cosθ, v sinθ, ω]; RobotZoo.Cartpole (mc 1, mp 0.2,
l 0.5, g 9.81): q̈ = −H⁻¹(C q̇ + G − B u) with H = [mc+mp, mp l cθ; mp l cθ, mp l²],
C q̇ = [−mp l sθ θ̇², 0], G = [0, mp g l sθ], B = [1, 0] — and RK3 (RobotDynamics:
k1 = f(x)dt, k2 = f(x + k1/2)dt, k3 = f(x − k1 + 2k2)dt, x⁺ = x + (k1 + 4k2 + k3)/6) are
restated from their published definitions; Jacobians here by complex-step differentiation
(exact to rounding; the device path uses forward-mode dual numbers — an independent check).
The merit weight μ is fixed (the script's μ = 1; TO.update_penalty! is absent).
"""
from __future__ import annotations

import numpy as np

NX, NU = 3, 2          # the Dubins car (module-level names kept for the Dubins helpers)
ETA, RHO, LS_TRIES = 1e-4, 0.5, 10
CARTPOLE_PARAMS = (1.0, 0.2, 0.5, 9.81)   # RobotZoo.Cartpole() defaults: mc, mp, l, g


def dubins(x, u):
    """RobotZoo.DubinsCar continuous dynamics."""
    return np.array([u[0] * np.cos(x[2]), u[0] * np.sin(x[2]), u[1]], dtype=np.result_type(x, u))


def cartpole(x, u, params=CARTPOLE_PARAMS):
    """RobotZoo.Cartpole continuous dynamics, q = [x, θ]: q̈ = −H⁻¹(C q̇ + G − B u)."""
    mc, mp, l, g = params
    s, c = np.sin(x[1]), np.cos(x[1])
    H = np.array([[mc + mp, mp * l * c], [mp * l * c, mp * l * l]], dtype=np.result_type(x, u))
    rhs = np.array([mp * l * s * x[3] ** 2 + u[0], -mp * g * l * s], dtype=H.dtype)
    qdd = np.linalg.solve(H, rhs)
    return np.concatenate([x[2:4], qdd])


class Model:
    """A continuous model f(x, u) with its sizes (the device's LQRX_MODEL_* id in `model_id`)."""

    def __init__(self, name, nx, nu, f, model_id, params=(0.0, 0.0, 0.0, 0.0)):
        self.name, self.nx, self.nu, self.f, self.model_id, self.params = name, nx, nu, f, model_id, params


def double_integrator(D):
    """RobotZoo.DoubleIntegrator(D): x = [q; q̇], ẋ = [q̇; u]."""
    return lambda x, u: np.concatenate([x[D:2 * D], u])


DUBINS = Model("dubins", 3, 2, dubins, 0)
CARTPOLE = Model("cartpole", 4, 1, cartpole, 1, CARTPOLE_PARAMS)
DOUBLE_INTEGRATOR = {D: Model(f"double_integrator{D}", 2 * D, D, double_integrator(D), 1 + D) for D in (1, 2, 3)}


def rk3(x, u, dt, model=DUBINS):
    f = model.f
    k1 = f(x, u) * dt
    k2 = f(x + k1 / 2, u) * dt
    k3 = f(x - k1 + 2 * k2, u) * dt
    return x + (k1 + 4 * k2 + k3) / 6


def rk3_jac(x, u, dt, model=DUBINS, h=1e-30):
    """[A B] = ∂rk3/∂[x u] by complex step."""
    nx, nu = model.nx, model.nu
    J = np.zeros((nx, nx + nu))
    for i in range(nx + nu):
        xc = x.astype(complex)
        uc = u.astype(complex)
        if i < nx:
            xc[i] += 1j * h
        else:
            uc[i - nx] += 1j * h
        J[:, i] = np.imag(rk3(xc, uc, dt, model)) / h
    return J


def rollout(model, x0, U, dt):
    """rollout! (problems.jl:83): states from x0 under the controls U (N−1 × nu)."""
    X = [np.asarray(x0, float)]
    for u in U:
        X.append(rk3(X[-1], np.asarray(u, float), dt, model))
    return X


class TrajSQP:
    """One trajectory's NLP, variables in the reference's order z = [x₁; u₁; …; x_{N-1}; u_{N-1}; x_N]."""

    def __init__(self, N, dt, Q, R, Qf, x0, xf, mu=1.0, model=DUBINS, stage=None):
        """stage = (A_s, b_s): the linear constraint A_s x_k = b_s on the interior knots
        k = 2..N−1 (1-based; DoubleIntegrator()'s LinearConstraint, problems.jl:40-44)."""
        self.model = model
        self.nx, self.nu = model.nx, model.nu
        self.N, self.dt, self.mu = N, dt, mu
        self.Q, self.R, self.Qf = (np.asarray(v, float) for v in (Q, R, Qf))
        self.x0, self.xf = np.asarray(x0, float), np.asarray(xf, float)
        if stage is None:
            stage = (np.zeros((0, self.nx)), np.zeros(0))
        self.SA, self.Sb = np.asarray(stage[0], float).reshape(-1, self.nx), np.asarray(stage[1], float)
        self.pk = self.SA.shape[0]
        self.NN = N * self.nx + (N - 1) * self.nu
        self.P = (N + 1) * self.nx + (N - 2) * self.pk

    def oy(self, k):
        """start of knot k's constraint block [c_k; d_k] (the KKT y / λ order)."""
        return 0 if k == 0 else 2 * self.nx + (k - 1) * (self.pk + self.nx)

    def split(self, z):
        NX, NU = self.nx, self.nu
        w = NX + NU
        X = [z[k * w:k * w + NX] for k in range(self.N - 1)] + [z[(self.N - 1) * w:]]
        U = [z[k * w + NX:(k + 1) * w] for k in range(self.N - 1)]
        return X, U

    def f(self, z):
        X, U = self.split(z)
        J = 0.0
        for k in range(self.N - 1):
            e = X[k] - self.xf
            J += 0.5 * e @ (self.Q * e) + 0.5 * U[k] @ (self.R * U[k])
        e = X[-1] - self.xf
        return J + 0.5 * e @ (self.Qf * e)

    def grad(self, z):
        X, U = self.split(z)
        g = []
        for k in range(self.N - 1):
            g += [self.Q * (X[k] - self.xf), self.R * U[k]]
        g.append(self.Qf * (X[-1] - self.xf))
        return np.concatenate(g)

    def hess_diag(self):
        return np.concatenate([np.concatenate([self.Q, self.R])] * (self.N - 1) + [self.Qf])

    def c(self, z):
        """[x₁ − x0; dyn₁; (A_s x_k − b_s; dyn_k) for k = 2..N−1; x_N − xf]"""
        X, U = self.split(z)
        v = [X[0] - self.x0]
        for k in range(self.N - 1):
            if k > 0:
                v.append(self.SA @ X[k] - self.Sb)
            v.append(rk3(X[k], U[k], self.dt, self.model) - X[k + 1])
        v.append(X[-1] - self.xf)
        return np.concatenate(v)

    def jac(self, z):
        X, U = self.split(z)
        NX, PK = self.nx, self.pk
        A = np.zeros((self.P, self.NN))
        w = NX + self.nu
        A[:NX, :NX] = np.eye(NX)
        for k in range(self.N - 1):
            r = NX if k == 0 else self.oy(k) + PK          # dynamics rows of knot k
            if k > 0:
                A[self.oy(k):self.oy(k) + PK, k * w:k * w + NX] = self.SA
            A[r:r + NX, k * w:(k + 1) * w] = rk3_jac(X[k], U[k], self.dt, self.model)
            A[r:r + NX, (k + 1) * w:(k + 1) * w + NX] = -np.eye(NX)
        A[-NX:, (self.N - 1) * w:] = np.eye(NX)
        return A

    def phi(self, z):
        return self.f(z) + self.mu * np.abs(self.c(z)).sum()

    def newton(self, z):
        """dubins_sqp.jl:64-70 with the cost Hessian: returns dz, λ."""
        A, H = self.jac(z), self.hess_diag()
        NN, P = self.NN, self.P
        K = np.zeros((NN + P, NN + P))
        K[:NN, :NN] = np.diag(H)
        K[:NN, NN:] = A.T
        K[NN:, :NN] = A
        sol = np.linalg.solve(K, -np.concatenate([self.grad(z), self.c(z)]))
        return sol[:NN], sol[NN:]

    def soc(self, z, dz):
        """dx̂ = −Aᵀ(AAᵀ)⁻¹c(x + dx) (dubins_sqp.jl:84-85; second_order_correction!)."""
        A = self.jac(z)
        return -A.T @ np.linalg.solve(A @ A.T, self.c(z + dz))

    def line_search(self, z, dz):
        """dubins_sqp.jl:74-97.  Returns (z_new, accepted, alpha, used_soc)."""
        phi0 = self.phi(z)
        dphi = self.grad(z) @ dz - self.mu * np.abs(self.c(z)).sum()
        a = 1.0
        for _ in range(LS_TRIES):
            if self.phi(z + a * dz) <= phi0 + ETA * a * dphi:
                return z + a * dz, True, a, False
            if a == 1.0:
                dzh = self.soc(z, dz)
                if self.phi(z + dz + dzh) < phi0 + ETA * dphi:
                    return z + dz + dzh, True, a, True
            a *= RHO
        return z, False, 0.0, False

    def residuals(self, z, lam):
        """max_violation and residual (cholesky_solver.jl:129-130, 238-252)."""
        return np.abs(self.c(z)).max(), np.linalg.norm(self.grad(z) + self.jac(z).T @ lam)


class DubinsSQP(TrajSQP):
    """The Dubins car NLP (test/dubins_sqp.jl)."""

    def __init__(self, N, dt, Q, R, Qf, x0, xf, mu=1.0):
        super().__init__(N, dt, Q, R, Qf, x0, xf, mu, DUBINS)


def cartpole_problem(N, mu=1.0, x0=(0.0, 0.0, 0.0, 0.0), xf=(0.0, np.pi, 0.0, 0.0), tf=5.0):
    """Cartpole() of test/problems.jl:58-88 (Q 1e-2·I, R 1e-1·I, Qf 100·I, tf 5) and its
    initial guess: U0 = 0.01 rolled out from x0 (:80-84).  Returns (TrajSQP, z0)."""
    dt = tf / (N - 1)
    p = TrajSQP(N, dt, [1e-2] * 4, [1e-1], [100.0] * 4, x0, xf, mu, CARTPOLE)
    U = np.full((N - 1, 1), 0.01)
    X = rollout(CARTPOLE, p.x0, U, dt)
    z = np.concatenate([np.concatenate([X[k], U[k]]) for k in range(N - 1)] + [X[-1]])
    return p, z


def double_integrator_problem(D=3, N=101, mu=1.0, seed=1, x0=None, xf=None):
    """DoubleIntegrator(D, N) of test/problems.jl:14-56: Q = diag(10·1_D, 1_D), R = 0.1·I,
    Qf = 10Q, x0 = [1_D; 0_D], xf = 0, dt = (N−1)/tf with tf = 2 (as the reference writes it,
    :19), the planar LinearConstraint A = [rand(p,D) rand(p,D)], b = 0, p = max(D−2, 1) on
    knots 2:N−1 (Julia's rand stream is not reproducible here: A from a seeded numpy draw) and
    the goal.  Initial guess: zeros (the reference's Problem holds no trajectory for it).
    Returns (TrajSQP, z0)."""
    model = DOUBLE_INTEGRATOR[D]
    tf = 2.0
    dt = (N - 1) / tf
    p = max(D - 2, 1)
    rng = np.random.default_rng(seed)
    SA = rng.random((p, 2 * D))
    Q = [10.0] * D + [1.0] * D
    x0 = np.concatenate([np.ones(D), np.zeros(D)]) if x0 is None else x0
    xf = np.zeros(2 * D) if xf is None else xf
    prob = TrajSQP(N, dt, Q, [0.1] * D, [10.0 * q for q in Q], x0, xf, mu, model, (SA, np.zeros(p)))
    return prob, np.zeros(prob.NN)


def solve(prob: TrajSQP, z0, iters=10, tol_p=1e-5, tol_d=1e-5):
    """CholeskySolver.solve! loop (cholesky_solver.jl:109-153).  Returns dict z, lam, iters
    (steps taken), status (0 converged, 1 iteration limit, 2 line search failed), hist
    (iterates), soc (per step: second-order correction used)."""
    z, lam = np.array(z0, float), np.zeros(prob.P)
    hist, socs = [z.copy()], []
    for it in range(iters):
        fp, fd = prob.residuals(z, lam)
        if fp < tol_p and fd < tol_d:
            return dict(z=z, lam=lam, iters=it, status=0, hist=hist, soc=socs)
        dz, lam_n = prob.newton(z)
        z_n, ok, _, used = prob.line_search(z, dz)
        if not ok:
            return dict(z=z, lam=lam, iters=it, status=2, hist=hist, soc=socs)
        z, lam = z_n, lam_n
        hist.append(z.copy())
        socs.append(used)
    return dict(z=z, lam=lam, iters=iters, status=1, hist=hist, soc=socs)


def initial_guess(N, dt, x0, xf):
    """States interpolated from x0 to xf, controls at the straight-line speed and turn rate:
    violates the dynamics, so the SQP has work to do."""
    x0, xf = np.asarray(x0, float), np.asarray(xf, float)
    w = NX + NU
    z = np.zeros(N * NX + (N - 1) * NU)
    T = dt * (N - 1)
    v = np.hypot(*(xf[:2] - x0[:2])) / T
    om = (xf[2] - x0[2]) / T
    for k in range(N):
        s = k / (N - 1)
        z[k * w:k * w + NX] = (1 - s) * x0 + s * xf
        if k < N - 1:
            z[k * w + NX:(k + 1) * w] = [v, om]
    return z


def assemble(prob: TrajSQP, z):
    """The Newton step's KKT inputs at z in the liblqrx ABI layout (h_mode 2): per knot
    Y_k = [D2; C; D1] (column-major), y_k = [c; d], H_k (diagonal), g_k — the blocks
    ConstraintBlocks / InvertedQuadratic hold (conblocks.jl:36-98, block_cholesky.jl:82-91,
    126-132), cut from the dense ∇c, c, ∇²f, ∇f above.  Knot k's rows are the constraints
    [λ_{k-1}; μ_k; λ_k] = c[mk : mk+2n], mk = 0 (k = 0) or n·k; its columns are z_k."""
    A, c, g, h = prob.jac(z), prob.c(z), prob.grad(z), prob.hess_diag()
    N, NX, W, PK = prob.N, prob.nx, prob.nx + prob.nu, prob.pk
    Y, y, H, G = [], [], [], []
    for k in range(N):
        w = W if k < N - 1 else NX
        rows = 2 * NX if k in (0, N - 1) else 2 * NX + PK
        mk = 0 if k == 0 else prob.oy(k) - NX
        Y.append(A[mk:mk + rows, W * k:W * k + w].T.ravel())     # column-major
        oy = prob.oy(k)
        y.append(c[oy:oy + (2 * NX if k == 0 else NX if k == N - 1 else PK + NX)])
        H.append(h[W * k:W * k + w])
        G.append(g[W * k:W * k + w])
    return tuple(np.concatenate(v) for v in (Y, y, H, G))
