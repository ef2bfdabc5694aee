"""Trajectory SQP (SURVEY.md §8(f) ranks 2–3), Dubins car and cartpole: oracle self-checks on
CPU, GPU parity of lqrx_sqp_solve (and the round-1 lqrx_dubins_sqp_solve forwarders) against
oracle/sqp_oracle.py (a restatement of test/dubins_sqp.jl:37-97
inside the CholeskySolver loop, cholesky_solver.jl:109-153).

Pinning: the oracle's Newton step is a dense KKT solve; `test_assembly_matches_kkt_oracle`
checks that the block assembly of the same step fed to the KAT-pinned block KKT oracle
(oracle/lqr_oracle.c, pinned by test/cholesky_solve.jl:18-44 in test_oracle.py) gives the same
δz and λ — so assembly layout, signs and multiplier order are pinned by the reference's own
KKT identities.  TrajOptCore/RobotZoo are absent: the Dubins and cartpole models and RK3 are
restated from their published definitions (parity unpinned for those formulas beyond that;
the device differentiates them with dual numbers, the oracle by complex step).

GPU tolerance: iterates and multipliers within 1e-9 relative (rounding of a dense LU vs the
block Cholesky propagates through ≤ 10 nonlinear steps), identical iteration counts and status.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from oracle import sqp_oracle as S


def _problem(N, mu, seed, batch):
    rng = np.random.default_rng(seed)
    dt = 3.0 / (N - 1)
    x0 = 0.1 * rng.standard_normal((batch, 3))
    xf = np.array([3.0, 3.0, np.pi / 2]) + 0.2 * rng.standard_normal((batch, 3))
    probs = [S.DubinsSQP(N, dt, [1e-2] * 3, [1e-1] * 2, [100.0] * 3, x0[b], xf[b], mu=mu) for b in range(batch)]
    Z0 = np.stack([S.initial_guess(N, dt, x0[b], xf[b]) for b in range(batch)])
    return dt, x0, xf, probs, Z0


@pytest.mark.parametrize("N", [4, 11, 101])
def test_assembly_matches_kkt_oracle(N):
    dt, x0, xf, probs, Z0 = _problem(N, 1.0, 3, 3)
    rng = np.random.default_rng(4)
    st = orc.KktStructure(3, 2, N, [3] + [0] * (N - 2) + [3])
    for b, p in enumerate(probs):
        z = Z0[b] + 0.05 * rng.standard_normal(Z0.shape[1])
        dz, lam = p.newton(z)
        Y, y, H, g = p.assemble(z) if hasattr(p, "assemble") else S.assemble(p, z)
        r = orc.kkt_solve_batch(st, 1, Y[None], y[None], H[None], g[None], h_mode=2, ginv=1, nthreads=1)
        assert np.abs(r["dz"].ravel() - dz).max() <= 1e-10 * np.abs(dz).max()
        assert np.abs(r["lam"].ravel() - lam).max() <= 1e-10 * np.abs(lam).max()
        # second-order correction = the ginv = 0 variant on the same blocks with y = c(z + dz)
        _, y2, _, _ = S.assemble(p, z + dz)
        r0 = orc.kkt_solve_batch(st, 1, Y[None], y2[None], H[None], g[None], h_mode=2, ginv=0, nthreads=1)
        soc = p.soc(z, dz)
        assert np.abs(r0["dz"].ravel() - soc).max() <= 1e-10 * max(np.abs(soc).max(), 1e-300)


def test_oracle_sqp_behaviour():
    """The restated loop: full steps converge toward feasibility; with μ = 1 at N = 101 the
    L1 merit is not exact and the line search (SOC, then backtracking) fails — status 2."""
    _, _, _, probs, Z0 = _problem(11, 10.0, 0, 2)
    for p, z0 in zip(probs, Z0):
        r = S.solve(p, z0)
        assert r["status"] == 1 and r["iters"] == 10
        assert p.residuals(r["z"], r["lam"])[0] < 1e-5
    _, _, _, probs, Z0 = _problem(101, 1.0, 1, 1)
    r = S.solve(probs[0], Z0[0])
    assert r["status"] == 2


def test_sqp_desc_validation(lqrx):
    import ctypes as C
    import lqrx.sqp as Q

    lib = lqrx.load()
    for field, val in (("N", 1), ("dt", 0.0), ("max_iters", -1), ("mu", -1.0), ("batch", -1), ("model", 7),
                       ("stage_rows", 3)):
        d = Q.DubinsSQP(11, 0.3).desc(4)
        setattr(d, field, val)
        assert lib.lqrx_sqp_solve(C.byref(d), *([None] * 6), None) == -1, field
    d = Q.DubinsSQP(11, 0.3, R=(0.1, 0.0)).desc(4)
    assert lib.lqrx_sqp_solve(C.byref(d), *([None] * 6), None) == -1
    d = Q.CartpoleSQP(11, params=(1.0, 0.2, 0.0, 9.81)).desc(4)          # l = 0
    assert lib.lqrx_sqp_solve(C.byref(d), *([None] * 6), None) == -1
    d = Q.CartpoleSQP(11, Qf=(1.0, 1.0, 1.0, -1.0)).desc(4)
    assert lib.lqrx_sqp_solve(C.byref(d), *([None] * 6), None) == -1
    d = Q.DubinsSQP(11, 0.3).desc(0)
    assert lib.lqrx_sqp_solve(C.byref(d), *([None] * 6), None) == 0     # empty batch
    d = Q.CartpoleSQP(11).desc(2)
    assert lib.lqrx_sqp_solve(C.byref(d), None, *([None] * 5), None) == -2
    # the round-1 Dubins entry points forward (same validation)
    old = lqrx._lib.SqpDesc(11, 10, 4, 0.3, (C.c_double * 3)(1, 1, 1), (C.c_double * 2)(1, 0), (C.c_double * 3)(1, 1, 1),
                            1.0, 1e-5, 1e-5)
    assert lib.lqrx_dubins_sqp_solve(C.byref(old), *([None] * 6), None) == -1
    old.R[1] = 1.0
    old.batch = 0
    assert lib.lqrx_dubins_sqp_solve(C.byref(old), *([None] * 6), None) == 0
    d = Q.DoubleIntegratorSQP(3, 11).desc(2)
    d.stage_rows = 3                                                    # > 2
    assert lib.lqrx_sqp_solve(C.byref(d), *([None] * 6), None) == -1
    d = Q.DoubleIntegratorSQP(3, 11).desc(2)
    d.stage_A[0] = float("nan")
    assert lib.lqrx_sqp_solve(C.byref(d), *([None] * 6), None) == -1
    nx, nu = C.c_int32(), C.c_int32()
    assert lib.lqrx_sqp_model_dims(1, C.byref(nx), C.byref(nu)) == 0 and (nx.value, nu.value) == (4, 1)
    assert lib.lqrx_sqp_model_dims(0, C.byref(nx), C.byref(nu)) == 0 and (nx.value, nu.value) == (3, 2)
    assert lib.lqrx_sqp_model_dims(4, C.byref(nx), C.byref(nu)) == 0 and (nx.value, nu.value) == (6, 3)
    assert lib.lqrx_sqp_model_dims(5, C.byref(nx), C.byref(nu)) == -1


# ---------------------------------------------------------------- cartpole (problems.jl:58-88)
def _cartpole(N, mu, seed, batch, goal="swingup", tf=5.0):
    """Cartpole() per trajectory: swing-up (xf = [0, π, 0, 0], the reference's problem) or a
    gentle goal the SQP converges to, with x0 perturbed per trajectory (seeded)."""
    rng = np.random.default_rng(seed)
    probs, Z0, x0s, xfs = [], [], [], []
    for b in range(batch):
        x0 = 0.05 * rng.standard_normal(4) if b else np.zeros(4)
        if goal == "swingup":
            xf = np.array([0.0, np.pi, 0.0, 0.0])
        else:
            xf = np.array([rng.uniform(-1, 1), rng.uniform(-0.5, 0.5), 0.0, 0.0])
        p, z0 = S.cartpole_problem(N, mu=mu, x0=x0, xf=xf, tf=tf)
        probs.append(p), Z0.append(z0), x0s.append(x0), xfs.append(xf)
    return probs, np.stack(Z0), np.stack(x0s), np.stack(xfs)


@pytest.mark.parametrize("N", [6, 21])        # N ≥ 5: 4(N+1) constraints ≤ 5N − 1 variables
def test_cartpole_assembly_matches_kkt_oracle(N):
    probs, Z0, _, _ = _cartpole(N, 1.0, 3, 2)
    rng = np.random.default_rng(5)
    st = orc.KktStructure(4, 1, N, [4] + [0] * (N - 2) + [4])
    for b, p in enumerate(probs):
        z = Z0[b] + 0.05 * rng.standard_normal(Z0.shape[1])
        dz, lam = p.newton(z)
        Y, y, H, g = S.assemble(p, z)
        r = orc.kkt_solve_batch(st, 1, Y[None], y[None], H[None], g[None], h_mode=2, ginv=1, nthreads=1)
        assert np.abs(r["dz"].ravel() - dz).max() <= 1e-10 * np.abs(dz).max()
        assert np.abs(r["lam"].ravel() - lam).max() <= 1e-10 * np.abs(lam).max()
        _, y2, _, _ = S.assemble(p, z + dz)
        r0 = orc.kkt_solve_batch(st, 1, Y[None], y2[None], H[None], g[None], h_mode=2, ginv=0, nthreads=1)
        soc = p.soc(z, dz)
        assert np.abs(r0["dz"].ravel() - soc).max() <= 1e-10 * max(np.abs(soc).max(), 1e-300)


def test_cartpole_model_and_guess():
    """The restated cartpole: energy-consistent small-step check (a free pendulum hanging at
    θ = 0 stays put; H q̈ = B u − C q̇ − G holds at a random state), and the host rollout guess
    of lqrx.sqp equals the oracle's rollout (problems.jl:80-84)."""
    import lqrx.sqp as Q

    mc, mp, l, g = S.CARTPOLE_PARAMS
    assert np.allclose(S.cartpole(np.zeros(4), np.zeros(1)), 0.0)
    rng = np.random.default_rng(1)
    x, u = rng.standard_normal(4), rng.standard_normal(1)
    qdd = S.cartpole(x, u)[2:]
    s, c = np.sin(x[1]), np.cos(x[1])
    H = np.array([[mc + mp, mp * l * c], [mp * l * c, mp * l * l]])
    rhs = np.array([u[0] + mp * l * s * x[3] ** 2, -mp * g * l * s])
    assert np.allclose(H @ qdd, rhs, rtol=1e-13, atol=1e-13)
    p, z0 = S.cartpole_problem(21)
    zq = Q.cartpole_rollout_guess(Q.CartpoleSQP(21), np.zeros(4))
    assert np.abs(zq - z0).max() <= 1e-12 * np.abs(z0).max()


def test_cartpole_oracle_behaviour():
    """Gentle goals converge in a few full Newton steps; the reference's swing-up does not
    within the 10 steps of solve! (pure SQP from a near-rest rollout)."""
    probs, Z0, _, _ = _cartpole(21, 1.0, 2, 2, goal="gentle", tf=2.0)
    for p, z0 in zip(probs, Z0):
        r = S.solve(p, z0)
        assert r["status"] == 0 and r["iters"] <= 6
    probs, Z0, _, _ = _cartpole(21, 1.0, 0, 1)
    r = S.solve(probs[0], Z0[0])
    assert r["status"] == 1 and r["iters"] == 10


def _run_gpu(N, mu, seed, batch, iters=10):
    import lqrx.sqp as Q

    dt, x0, xf, probs, Z0 = _problem(N, mu, seed, batch)
    got = Q.dubins_sqp_solve(Q.DubinsSQP(N, dt, mu=mu, max_iters=iters), Z0, x0, xf)
    refs = [S.solve(p, z, iters=iters) for p, z in zip(probs, Z0)]
    return got, refs


@pytest.mark.gpu
@pytest.mark.parametrize("N,mu,seed,batch", [(11, 10.0, 0, 5), (101, 10.0, 1, 3), (4, 1.0, 2, 4), (101, 1.0, 5, 2)])
def test_sqp_gpu_parity(lqrx, gpu_ok, N, mu, seed, batch):
    got, refs = _run_gpu(N, mu, seed, batch)
    for b, r in enumerate(refs):
        assert got["status"][b] == r["status"], (b, got["status"][b], r["status"])
        assert got["iters"][b] == r["iters"]
        scale = np.abs(r["z"]).max()
        assert np.abs(got["z"][b] - r["z"]).max() <= 1e-9 * scale
        if r["iters"]:
            ls = max(np.abs(r["lam"]).max(), 1e-300)
            assert np.abs(got["lam"][b] - r["lam"]).max() <= 1e-9 * ls


@pytest.mark.gpu
def test_sqp_gpu_converges_and_ragged(lqrx, gpu_ok):
    """A batch that is not a multiple of 64 with a loose tolerance: trajectories stop at
    different iterations (frozen ones are not touched again) and each matches the oracle."""
    import lqrx.sqp as Q

    N, batch = 11, 70
    dt, x0, xf, probs, Z0 = _problem(N, 10.0, 9, batch)
    prob = Q.DubinsSQP(N, dt, mu=10.0, tol_p=1e-4, tol_d=2e-3)
    got = Q.dubins_sqp_solve(prob, Z0, x0, xf)
    assert (got["status"] == Q.CONVERGED).any()
    for b in (0, 1, 63, 64, 69):
        r = S.solve(probs[b], Z0[b], tol_p=1e-4, tol_d=2e-3)
        assert got["status"][b] == r["status"] and got["iters"][b] == r["iters"]
        assert np.abs(got["z"][b] - r["z"]).max() <= 1e-9 * np.abs(r["z"]).max()


def _random_goals(N, mu, seed, batch):
    """Goals anywhere in [−4, 4]² × [−3, 3] and a perturbed straight-line guess: exercises the
    full line search (Armijo at α = 1, second-order correction, backtracking)."""
    rng = np.random.default_rng(seed)
    dt = 3.0 / (N - 1)
    x0 = 0.1 * rng.standard_normal((batch, 3))
    xf = np.stack([rng.uniform(-4, 4, batch), rng.uniform(-4, 4, batch), rng.uniform(-3, 3, batch)], 1)
    Z0 = np.stack([S.initial_guess(N, dt, x0[b], xf[b]) for b in range(batch)])
    Z0 += 0.3 * rng.standard_normal(Z0.shape)
    probs = [S.DubinsSQP(N, dt, [1e-2] * 3, [1e-1] * 2, [100.0] * 3, x0[b], xf[b], mu=mu) for b in range(batch)]
    return dt, x0, xf, probs, Z0


@pytest.mark.gpu
@pytest.mark.parametrize("N,mu", [(21, 10.0), (11, 1.0)])
def test_sqp_gpu_line_search_paths(lqrx, gpu_ok, N, mu):
    import lqrx.sqp as Q

    batch = 96
    dt, x0, xf, probs, Z0 = _random_goals(N, mu, 11 + N, batch)
    got = Q.dubins_sqp_solve(Q.DubinsSQP(N, dt, mu=mu), Z0, x0, xf)
    refs = [S.solve(p, z) for p, z in zip(probs, Z0)]
    assert any(any(r["soc"]) for r in refs)               # the SOC branch is covered
    bad = [b for b, r in enumerate(refs)
           if got["status"][b] != r["status"] or got["iters"][b] != r["iters"]
           or np.abs(got["z"][b] - r["z"]).max() > 1e-9 * np.abs(r["z"]).max()]
    assert not bad, bad


# ---------------------------------------------------------------- DoubleIntegrator (problems.jl:14-56)
def _double_integrator(D, N, mu, seed, batch):
    """DoubleIntegrator(D, N) per trajectory, x0 = [1_D; 0_D] for trajectory 0 and perturbed
    for the others; the shared stage matrix of lqrx.sqp.DoubleIntegratorSQP."""
    import lqrx.sqp as Q

    prob = Q.DoubleIntegratorSQP(D, N, mu=mu)
    SA = np.asarray(prob.stage_A).reshape(prob.stage_rows, 2 * D)
    rng = np.random.default_rng(seed)
    probs, Z0, x0s, xfs = [], [], [], []
    for b in range(batch):
        x0 = np.concatenate([np.ones(D), np.zeros(D)]) + (0.2 * rng.standard_normal(2 * D) if b else 0.0)
        p, z0 = S.double_integrator_problem(D, N, mu=mu, x0=x0)
        p.SA = SA
        probs.append(p), Z0.append(z0 + (0.1 * rng.standard_normal(z0.shape) if b % 2 else 0.0))
        x0s.append(x0), xfs.append(np.zeros(2 * D))
    return prob, probs, np.stack(Z0), np.stack(x0s), np.stack(xfs)


@pytest.mark.parametrize("D,N", [(2, 12), (3, 21)])
def test_double_integrator_assembly_matches_kkt_oracle(D, N):
    """The stage-constrained assembly (Y_k = [D2; C; D1] with C = A_s on knots 2..N−1) fed to
    the KAT-pinned block KKT oracle on the DoubleIntegrator structure reproduces the dense
    Newton step — the structure test/cholesky_solve.jl pins (its problem)."""
    import lqrx.kkt as K

    _, probs, Z0, _, _ = _double_integrator(D, N, 10.0, 0, 2)
    st = K.double_integrator_structure(D, N)
    sto = orc.KktStructure(2 * D, D, N, st.p)
    rng = np.random.default_rng(2)
    for b, p in enumerate(probs):
        z = Z0[b] + 0.1 * rng.standard_normal(Z0.shape[1])
        dz, lam = p.newton(z)
        Y, y, H, g = S.assemble(p, z)
        r = orc.kkt_solve_batch(sto, 1, Y[None], y[None], H[None], g[None], h_mode=2, ginv=1, nthreads=1)
        assert np.abs(r["dz"].ravel() - dz).max() <= 1e-9 * np.abs(dz).max()
        assert np.abs(r["lam"].ravel() - lam).max() <= 1e-8 * np.abs(lam).max()


def test_double_integrator_oracle_behaviour():
    """A linear-quadratic problem: with μ = 10 the first full Newton step is the optimum
    (converged at the next check); with μ = 1 the L1 merit is inexact and the line search fails."""
    _, probs, Z0, _, _ = _double_integrator(3, 21, 10.0, 1, 2)
    for p, z0 in zip(probs, Z0):
        r = S.solve(p, z0)
        assert r["status"] == 0 and r["iters"] == 1
    _, probs, Z0, _, _ = _double_integrator(3, 21, 1.0, 1, 1)
    assert S.solve(probs[0], Z0[0])["status"] == 2


@pytest.mark.gpu
@pytest.mark.parametrize("D,N,mu,batch", [(3, 101, 10.0, 4), (2, 12, 10.0, 67), (3, 21, 1.0, 3)])
def test_double_integrator_sqp_gpu_parity(lqrx, gpu_ok, D, N, mu, batch):
    """Device SQP with the interior-knot linear constraint (stage rows in the KKT blocks, the
    generic KKT kernel) against the oracle: status, steps, z, λ (relative 1e-8: dt = (N−1)/tf
    as the reference writes it makes the D = 3, N = 101 system ill-conditioned)."""
    import lqrx.sqp as Q

    prob, probs, Z0, x0, xf = _double_integrator(D, N, mu, 5, batch)
    got = Q.sqp_solve(prob, Z0, x0, xf)
    for b in sorted({0, 1, batch // 2, batch - 1}):
        r = S.solve(probs[b], Z0[b])
        assert got["status"][b] == r["status"] and got["iters"][b] == r["iters"], (b, got["status"][b], r["status"])
        assert np.abs(got["z"][b] - r["z"]).max() <= 1e-8 * np.abs(r["z"]).max()
        if r["iters"]:
            assert np.abs(got["lam"][b] - r["lam"]).max() <= 1e-8 * np.abs(r["lam"]).max()


def _cartpole_gpu(N, mu, seed, batch, goal, tf, iters=10):
    import lqrx.sqp as Q

    probs, Z0, x0, xf = _cartpole(N, mu, seed, batch, goal, tf)
    got = Q.sqp_solve(Q.CartpoleSQP(N, tf=tf, mu=mu, max_iters=iters), Z0, x0, xf)
    refs = [S.solve(p, z, iters=iters) for p, z in zip(probs, Z0)]
    return got, refs


@pytest.mark.gpu
@pytest.mark.parametrize("N,mu,seed,batch,goal,tf", [
    (21, 1.0, 0, 3, "swingup", 5.0),       # Cartpole(N=21) of test/cartpole.jl
    (101, 1.0, 1, 2, "swingup", 5.0),      # Cartpole() default N = 101
    (101, 10.0, 2, 2, "swingup", 5.0),
    (21, 1.0, 3, 5, "gentle", 2.0),
    (51, 10.0, 4, 3, "gentle", 2.0),
])
def test_cartpole_sqp_gpu_parity(lqrx, gpu_ok, N, mu, seed, batch, goal, tf):
    """Status, accepted steps, iterate and multipliers of every trajectory equal the oracle's
    (relative 1e-8: ≤ 10 nonlinear steps of a swing-up amplify the rounding difference of the
    dense LU vs the block Cholesky more than the Dubins car does)."""
    got, refs = _cartpole_gpu(N, mu, seed, batch, goal, tf)
    for b, r in enumerate(refs):
        assert got["status"][b] == r["status"], (b, got["status"][b], r["status"])
        assert got["iters"][b] == r["iters"]
        assert np.abs(got["z"][b] - r["z"]).max() <= 1e-8 * np.abs(r["z"]).max()
        if r["iters"]:
            assert np.abs(got["lam"][b] - r["lam"]).max() <= 1e-8 * max(np.abs(r["lam"]).max(), 1e-300)
    if goal == "gentle":
        assert (got["status"] == 0).all()


@pytest.mark.gpu
def test_cartpole_sqp_gpu_ragged(lqrx, gpu_ok):
    """70 gentle-goal trajectories (not a multiple of 64 waves): each converges and matches."""
    got, refs = _cartpole_gpu(21, 1.0, 7, 70, "gentle", 2.0)
    for b in (0, 1, 63, 64, 69):
        r = refs[b]
        assert got["status"][b] == r["status"] == 0 and got["iters"][b] == r["iters"]
        assert np.abs(got["z"][b] - r["z"]).max() <= 1e-8 * np.abs(r["z"]).max()
