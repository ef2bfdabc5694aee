"""CPU tests that PIN the oracle (oracle/lqr_oracle.c) before anything is compared to it.

KKT path — pinned by the reference's own known-answer identities,
/root/reference/test/cholesky_solve.jl:18-44, reproduced on the same problem structure
(DoubleIntegrator(3,101) from test/problems.jl:14-56) and on the Dubins cfg3 structure:
  :18  S ≈ D*(H\\D')            :19  D*(H\\g) − d ≈ r
  :24  cholesky(S).U ≈ U        :25  U'U ≈ S
  :31  λ ≈ −S\\r                :36  δz ≈ −H\\(D'λ + g)
  :39  ‖D δz + d‖ < 1e-12      :40  ‖H δz + g + D'λ‖ < 1e-12
  :42-44 [H D'; D 0] \\ [−g; −d] equals (δz, λ)
and the second-order-correction variant (cholesky_solver.jl:254-273): δẑ = −Dᵀ(DDᵀ)⁻¹d.

DP path — the reference's DP test (test/dp.jl) has no assertion and Julia is absent, so
the restatement of dynamic_programming.jl is pinned by identities: (1) the rollout U equals
the dense equality-constrained QP optimum; (2) for a long horizon K_1 → the DARE gain.
"""
import numpy as np
import pytest
import scipy.linalg as sla

from oracle import oracle as orc


def _struct(name):
    import lqrx.kkt as K

    return {"di": K.double_integrator_structure(3, 101), "dubins": K.dubins_structure(101),
            "di_small": K.double_integrator_structure(2, 12)}[name]


def _oracle_struct(st):
    o = orc.KktStructure(st.n, st.m, st.N, st.p)
    return o


@pytest.mark.parametrize("name", ["di", "dubins", "di_small"])
@pytest.mark.parametrize("h_mode", [0, 1, 2])
def test_kkt_oracle_known_answers(lqrx, name, h_mode):
    import lqrx.kkt as K

    st = _struct(name)
    pb = K.random_kkt(st, 1, seed=17 + h_mode, h_mode=h_mode)
    os_ = _oracle_struct(st)
    out = orc.kkt_solve_one(os_, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=h_mode, debug=True)
    assert out["info"] == 0
    dn = orc.kkt_dense(os_, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=h_mode)
    D, d, H, g = dn["D"], dn["d"], dn["H"], dn["g"]
    S_dense = D @ np.linalg.solve(H, D.T)
    rtol = 1e-8  # Julia's default ≈ (√eps) used by the reference script
    scale = np.abs(S_dense).max()
    # :18  S ≈ D*(H\D')  (the block storage holds the upper block triangle)
    assert np.abs(np.triu(out["S"]) - np.triu(S_dense)).max() <= rtol * scale
    # :19  D*(H\g) − d ≈ r
    assert np.allclose(out["r"], D @ np.linalg.solve(H, g) - d, rtol=rtol, atol=rtol * np.abs(d).max())
    # :24-25  cholesky(S).U ≈ U ;  U'U ≈ S
    U = np.triu(out["U"])
    Uref = np.linalg.cholesky(S_dense).T
    assert np.abs(U - Uref).max() <= 1e-7 * np.abs(Uref).max()
    assert np.abs(U.T @ U - S_dense).max() <= rtol * scale
    # :31  λ ≈ −S\r
    lam = out["lam"]
    assert np.allclose(lam, dn["lam"], rtol=1e-8, atol=1e-9 * np.abs(dn["lam"]).max())
    # :36  δz ≈ −H\(D'λ + g)
    dz = out["dz"]
    assert np.allclose(dz, -np.linalg.solve(H, D.T @ lam + g), rtol=1e-8, atol=1e-10)
    # :39-40  residuals
    assert np.linalg.norm(D @ dz + d) < 1e-10 * max(1.0, np.abs(d).max())
    assert np.linalg.norm(H @ dz + g + D.T @ lam) < 1e-10 * max(1.0, np.abs(g).max())
    # :42-44 full KKT solve
    NN = len(g)
    assert np.allclose(dn["full"][:NN], dz, rtol=1e-8, atol=1e-10)
    assert np.allclose(dn["full"][NN:], lam, rtol=1e-8, atol=1e-9 * np.abs(lam).max())


@pytest.mark.parametrize("name", ["di", "dubins"])
def test_kkt_oracle_soc(lqrx, name):
    """second_order_correction! (Ginv=false): δẑ = −Dᵀ(DDᵀ)⁻¹d (cholesky_solver.jl:255)."""
    import lqrx.kkt as K

    st = _struct(name)
    pb = K.random_kkt(st, 1, seed=5, h_mode=2)
    os_ = _oracle_struct(st)
    out = orc.kkt_solve_one(os_, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=2, ginv=0)
    dn = orc.kkt_dense(os_, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=2)
    D, d = dn["D"], dn["d"]
    ref = -D.T @ np.linalg.solve(D @ D.T, d)
    assert np.allclose(out["dz"], ref, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("name", ["di", "dubins", "di_small"])
@pytest.mark.parametrize("h_mode", [0, 2])
def test_kkt12_lower_variant(lqrx, name, h_mode):
    """KKT-12: the lower-storage block Cholesky (cholesky_solve.jl:5-26) cross-checks the
    upper one, as test/constraint_blocks.jl:103-133 does:
      :122  L_ ≈ U_'          :123  L_ ≈ cholesky(S0).L     :124  U_ ≈ cholesky(S0).U
      :125  cholesky(S0).L\\d ≈ λ  (after the forward sweep)
      :133  cholesky(S0)\\d ≈ λ    (after the backward sweep)
    with d = the stacked [c; d] right-hand side r of the Schur system; the upper solve
    returns −S⁻¹r (its backward sweep negates, :135-136), the lower one +S⁻¹r."""
    import lqrx.kkt as K

    st = _struct(name)
    pb = K.random_kkt(st, 1, seed=41 + h_mode, h_mode=h_mode)
    os_ = _oracle_struct(st)
    up = orc.kkt_solve_one(os_, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=h_mode, debug=True)
    lo = orc.kkt_lower_one(os_, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=h_mode)
    assert up["info"] == 0 and lo["info"] == 0
    dn = orc.kkt_dense(os_, pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=h_mode)
    S0 = dn["S"]
    S0 = 0.5 * (S0 + S0.T)
    Lref = np.linalg.cholesky(S0)
    L, U = lo["L"], np.triu(up["U"])
    sc = np.abs(Lref).max()
    assert np.array_equal(L, np.tril(L))                       # lower storage only
    assert np.abs(L - U.T).max() <= 1e-12 * sc                  # :122
    assert np.abs(L - Lref).max() <= 1e-9 * sc                  # :123
    assert np.abs(U - Lref.T).max() <= 1e-9 * sc                # :124
    r = up["r"]
    y_ref = sla.solve_triangular(Lref, r, lower=True)
    assert np.allclose(lo["y"], y_ref, rtol=1e-8, atol=1e-10 * np.abs(y_ref).max())   # :125
    x_ref = np.linalg.solve(S0, r)
    assert np.allclose(lo["x"], x_ref, rtol=1e-8, atol=1e-10 * np.abs(x_ref).max())   # :133
    assert np.allclose(lo["x"], -up["lam"], rtol=1e-10, atol=1e-12 * np.abs(x_ref).max())


def test_kkt12_lower_variant_throws_on_indefinite(lqrx):
    """cholesky() in the lower variant throws PosDefException (cholesky_solve.jl:17,21);
    the oracle reports the failing block."""
    import lqrx.kkt as K

    st = K.dubins_structure(11)
    pb = K.random_kkt(st, 1, seed=3, h_mode=2)
    h = pb.H.shape[1]
    pb.H[0, h // 2:] = -np.abs(pb.H[0, h // 2:])              # later knots: negative cost
    lo = orc.kkt_lower_one(_oracle_struct(st), pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=2)
    up = orc.kkt_solve_one(_oracle_struct(st), pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=2)
    assert lo["info"] > 0 and lo["info"] == up["info"]


def test_kkt_oracle_non_spd_info(lqrx):
    """A negative cost Hessian entry must be reported (the reference discards potrf info)."""
    import lqrx.kkt as K

    st = K.dubins_structure(11)
    pb = K.random_kkt(st, 1, seed=2, h_mode=0)
    pb.H[0, :] = -pb.H[0, :]
    out = orc.kkt_solve_one(_oracle_struct(st), pb.Y[0], pb.y[0], pb.H[0], pb.g[0], h_mode=0)
    assert out["info"] != 0


def test_dp_oracle_equals_dense_kkt(lqrx):
    from lqrx.dp import abi_to_batch

    n, m, N, bt = 6, 3, 25, 5
    d = lqrx.random_batch(n, m, N, bt, seed=31)
    out = orc.dp_solve_abi(d, N)
    b = abi_to_batch(d)
    X = out["X"].reshape(bt, N, n)
    U = out["U"].reshape(bt, N - 1, m)
    for t in range(bt):
        Xd, Ud = orc.dp_dense_kkt(b.A[t], b.B[t], b.Q[t], b.R[t], b.Qf[t], b.x0[t], N)
        assert np.abs(U[t] - Ud).max() <= 1e-10 * max(1.0, np.abs(Ud).max())
        assert np.abs(X[t] - Xd).max() <= 1e-10 * max(1.0, np.abs(Xd).max())


def _lin_batch(lqrx, n, m, N, bt, seed, tv):
    """Random batch with linear cost terms, flat ABI arrays (q, r per knot when tv)."""
    d = lqrx.random_batch(n, m, N, bt, seed=seed)
    rng = np.random.default_rng(seed + 1)
    kq = N - 1 if tv else 1
    d["q"] = rng.standard_normal(bt * kq * n)
    d["r"] = rng.standard_normal(bt * kq * m)
    d["qf"] = rng.standard_normal(bt * n)
    if tv:   # per-knot Q, R (the q, r knot layout follows Q, R: ABI knot_stride_QR)
        from lqrx.dp import from_abi, to_abi
        Q = from_abi(d["Q"], (bt, n, n))
        R = from_abi(d["R"], (bt, m, m))
        s = 1.0 + 0.5 * rng.random((bt, N - 1, 1, 1))
        d["Q"] = to_abi((Q[:, None] * s).reshape(bt * (N - 1), n, n)).ravel()
        d["R"] = to_abi((R[:, None] * s).reshape(bt * (N - 1), m, m)).ravel()
        d["tv_QR"] = 1
    return d


@pytest.mark.parametrize("tv", [False, True])
def test_dp_oracle_linear_equals_dense_kkt(lqrx, tv):
    """Linear cost terms: the rollout with u = −Kx − d equals the
    optimum of the QP with gᵀz added, and the value function's gradient P_k x_k + p_k equals
    the QP's costate at every knot (pins K, d, P_k and p_k together)."""
    from lqrx.dp import abi_to_batch, from_abi

    n, m, N, bt = 5, 2, 21, 4
    d = _lin_batch(lqrx, n, m, N, bt, 41, tv)
    out = orc.dp_solve_lin_abi(d, N, all_P=True)
    assert (out["info"] == 0).all()
    X = out["X"].reshape(bt, N, n)
    U = out["U"].reshape(bt, N - 1, m)
    P = from_abi(out["P"], (bt, N, n, n))
    p = out["p"].reshape(bt, N, n)
    A = from_abi(d["A"], (bt, n, n)); B = from_abi(d["B"], (bt, n, m))
    kq = N - 1 if tv else 1
    Q = from_abi(d["Q"], (bt, kq, n, n)); R = from_abi(d["R"], (bt, kq, m, m))
    Qf = from_abi(d["Qf"], (bt, n, n)); x0 = d["x0"].reshape(bt, n)
    q = d["q"].reshape(bt, kq, n); r = d["r"].reshape(bt, kq, m); qf = d["qf"].reshape(bt, n)
    for t in range(bt):
        if tv:   # dense QP with per-knot Q_k, R_k
            Xd, Ud, lam = _dense_tv(A[t], B[t], Q[t], R[t], Qf[t], x0[t], N, q[t], r[t], qf[t])
        else:
            Xd, Ud, lam = orc.dp_dense_kkt(A[t], B[t], Q[t, 0], R[t, 0], Qf[t], x0[t], N,
                                           q[t, 0], r[t, 0], qf[t], with_lam=True)
        sc = max(1.0, np.abs(Xd).max(), np.abs(Ud).max())
        assert np.abs(U[t] - Ud).max() <= 1e-10 * sc
        assert np.abs(X[t] - Xd).max() <= 1e-10 * sc
        grad = np.einsum("kij,kj->ki", P[t], X[t]) + p[t]
        costate = np.concatenate([-lam[:1], lam[1:]])
        assert np.abs(grad - costate).max() <= 1e-9 * max(1.0, np.abs(costate).max())


def _dense_tv(A, B, Q, R, Qf, x0, N, q, r, qf):
    """Dense QP of a problem with per-knot Q_k, R_k, q_k, r_k (A, B time-invariant)."""
    n, m = B.shape
    nz = N * n + (N - 1) * m
    H = np.zeros((nz, nz)); g = np.zeros(nz)
    ix = lambda k: slice(k * (n + m), k * (n + m) + n)
    iu = lambda k: slice(k * (n + m) + n, k * (n + m) + n + m)
    for k in range(N - 1):
        H[ix(k), ix(k)] = Q[k]; H[iu(k), iu(k)] = R[k]
        g[ix(k)] = q[k]; g[iu(k)] = r[k]
    H[ix(N - 1), ix(N - 1)] = Qf; g[ix(N - 1)] = qf
    D = np.zeros((N * n, nz)); dd = np.zeros(N * n)
    D[0:n, ix(0)] = np.eye(n); dd[0:n] = -x0
    for k in range(N - 1):
        rr = slice((k + 1) * n, (k + 2) * n)
        D[rr, ix(k)] = A; D[rr, iu(k)] = B; D[rr, ix(k + 1)] = -np.eye(n)
    sol = np.linalg.solve(np.block([[H, D.T], [D, np.zeros((N * n, N * n))]]),
                          np.concatenate([-g, -dd]))
    z = sol[:nz]
    return (np.stack([z[ix(k)] for k in range(N)]), np.stack([z[iu(k)] for k in range(N - 1)]),
            sol[nz:].reshape(N, n))


def test_dp_oracle_linear_zero_is_plain(lqrx):
    """q = r = qf = 0 reproduces the reference recursion bit for bit (d = 0, p = 0)."""
    n, m, N, bt = 6, 3, 17, 3
    d = _lin_batch(lqrx, n, m, N, bt, 43, False)
    for k in ("q", "r", "qf"):
        d[k] = np.zeros_like(d[k])
    a = orc.dp_solve_lin_abi(d, N, all_P=True)
    b = orc.dp_solve_abi(d, N, all_P=True)
    for k in ("K", "P", "X", "U"):
        assert np.array_equal(a[k], b[k]), k
    assert not a["d"].any() and not a["p"].any()


@pytest.mark.parametrize("n,m,N", [(4, 1, 101), (6, 3, 40), (32, 16, 64)])
def test_dp_oracle_matches_openblas_lapack(lqrx, n, m, N):
    """SURVEY §8(c) third-party boundary: the C oracle's hand-written potrf/potrs/gemm agree
    with OpenBLAS's dpotrf/dpotrs 'U' and dgemm (what Julia's LAPACK.potrf!/potrs! and BLAS
    call) on the reference op order — per knot K_k, P_k within 1e-12 relative, X, U 1e-12."""
    from lqrx.dp import abi_to_batch, from_abi

    bt = 3
    d = lqrx.random_batch(n, m, N, bt, seed=71 + n)
    out = orc.dp_solve_abi(d, N, all_P=True)
    b = abi_to_batch(d)
    K = from_abi(out["K"], (bt, N - 1, m, n)); P = from_abi(out["P"], (bt, N, n, n))
    X = out["X"].reshape(bt, N, n); U = out["U"].reshape(bt, N - 1, m)
    for t in range(bt):
        Kl, Pl, Xl, Ul = orc.dp_lapack(b.A[t], b.B[t], b.Q[t], b.R[t], b.Qf[t], b.x0[t], N)
        kn = lambda a, r: (np.abs(a - r).reshape(len(r), -1).max(1) / np.abs(r).reshape(len(r), -1).max(1)).max()
        assert kn(K[t], Kl) <= 1e-12 and kn(P[t], Pl) <= 1e-12
        assert np.abs(X[t] - Xl).max() <= 1e-12 * max(1.0, np.abs(Xl).max())
        assert np.abs(U[t] - Ul).max() <= 1e-12 * max(1.0, np.abs(Ul).max())


def test_dp_oracle_dare_limit(lqrx):
    """Long horizon: K_1 → (R + BᵀP∞B)⁻¹BᵀP∞A and P_1 → P∞ (scipy solve_discrete_are) on
    well-actuated problems (stable A, full-rank B) whose Riccati recursion
    converges geometrically."""
    from lqrx.dp import from_abi, to_abi

    rng = np.random.default_rng(8)
    n, m, N, bt = 8, 4, 300, 3
    A = rng.standard_normal((bt, n, n)) * 0.3   # ρ(A) < 1: the reference recursion does not
    # symmetrise P, so for open-loop-unstable A its skew part grows like ρ(A)^{2k}
    B = rng.standard_normal((bt, n, m))
    Q = np.broadcast_to(np.eye(n), (bt, n, n)).copy()
    R = np.broadcast_to(np.eye(m), (bt, m, m)).copy()
    d = dict(A=to_abi(A), B=to_abi(B), Q=to_abi(Q), R=to_abi(R), Qf=to_abi(10 * Q),
             x0=rng.standard_normal((bt, n)), n=n, m=m, batch=bt)
    out = orc.dp_solve_abi(d, N)
    K = from_abi(out["K"], (bt, N - 1, m, n))
    P1 = from_abi(out["P"], (bt, n, n))
    for t in range(bt):
        Pinf = sla.solve_discrete_are(A[t], B[t], Q[t], R[t])
        Kinf = np.linalg.solve(R[t] + B[t].T @ Pinf @ B[t], B[t].T @ Pinf @ A[t])
        assert np.abs(K[t, 0] - Kinf).max() <= 1e-9 * np.abs(Kinf).max()
        assert np.abs(P1[t] - Pinf).max() <= 1e-9 * np.abs(Pinf).max()


def test_dp_oracle_all_P_consistent(lqrx):
    """p_mode 1 stores P_k for every knot; P_N = Qf and P_1 equals the p_mode 0 output."""
    from lqrx.dp import from_abi

    n, m, N, bt = 5, 2, 30, 2
    d = lqrx.random_batch(n, m, N, bt, seed=4)
    a = orc.dp_solve_abi(d, N, all_P=True)
    b = orc.dp_solve_abi(d, N, all_P=False)
    Pa = from_abi(a["P"], (bt, N, n, n))
    Pb = from_abi(b["P"], (bt, n, n))
    Qf = from_abi(d["Qf"], (bt, n, n))
    assert np.array_equal(Pa[:, N - 1], Qf)
    assert np.array_equal(Pa[:, 0], Pb)


def lqr_as_kkt(A, B, Q, R, Qf, x0, N):
    """The LQR as the reference's KKT problem (conblocks.jl:403-425 block structure):
    initial-condition stage rows [I 0] at knot 1 (value −x0), dynamics D1_k = [A B],
    D2_{k+1} = [−I 0], H_k = blockdiag(Q, R) (Qf at N), g = 0, linearised at z = 0."""
    import lqrx.kkt as K

    n, m = B.shape
    st = K.ConstraintBlocks(n, m, N, [n] + [0] * (N - 1))
    Y, y, H = [], [], []
    for k in range(N):
        n1, p, n2, w = int(st.n1[k]), int(st.p[k]), int(st.n2[k]), int(st.w[k])
        blk = np.zeros((n1 + p + n2, w))
        if n1:
            blk[:n1, :n] = -np.eye(n)
        if p:
            blk[n1:n1 + p, :n] = np.eye(n)
        if n2:
            blk[n1 + p:, :n] = A
            blk[n1 + p:, n:] = B
        Y.append(blk.T.ravel())
        y.append(np.concatenate([-x0 if p else np.zeros(0), np.zeros(n2)]))
        Hk = np.zeros((w, w))
        Hk[:n, :n] = Qf if k == N - 1 else Q
        if w > n:
            Hk[n:, n:] = R
        H.append(Hk.T.ravel())
    g = np.zeros(int(np.sum(st.w)))
    return st, np.concatenate(Y), np.concatenate(y), np.concatenate(H), g


def test_dp_oracle_equals_kat_pinned_kkt_oracle(lqrx):
    """Transitive pin of the DP restatement: its rollout (X, U) must equal the primal step of
    the KKT restatement — itself pinned above by the reference's test/cholesky_solve.jl
    known answers — on the same LQR written as a constrained QP."""
    from lqrx.dp import abi_to_batch

    n, m, N, bt = 6, 3, 30, 4
    d = lqrx.random_batch(n, m, N, bt, seed=12)
    out = orc.dp_solve_abi(d, N)
    b = abi_to_batch(d)
    X = out["X"].reshape(bt, N, n)
    U = out["U"].reshape(bt, N - 1, m)
    for t in range(bt):
        st, Y, y, H, g = lqr_as_kkt(b.A[t], b.B[t], b.Q[t], b.R[t], b.Qf[t], b.x0[t], N)
        kk = orc.kkt_solve_one(_oracle_struct(st), Y, y, H, g, h_mode=0)
        assert kk["info"] == 0
        z = kk["dz"]
        Xk = np.stack([z[k * (n + m):k * (n + m) + n] for k in range(N)])
        Uk = np.stack([z[k * (n + m) + n:(k + 1) * (n + m)] for k in range(N - 1)])
        assert np.abs(Xk - X[t]).max() <= 1e-10 * max(1.0, np.abs(X[t]).max())
        assert np.abs(Uk - U[t]).max() <= 1e-10 * max(1.0, np.abs(U[t]).max())


def lqr_tv_as_kkt(A, B, Q, R, Qf, x0, N):
    """Time-varying LQR (A[k], B[k], Q[k], R[k] for k = 0..N-2) as the KKT problem of
    lqr_as_kkt (knot k's dynamics rows [A_k B_k], cost blockdiag(Q_k, R_k))."""
    import lqrx.kkt as K

    n, m = B.shape[-2:]
    st = K.ConstraintBlocks(n, m, N, [n] + [0] * (N - 1))
    Y, y, H = [], [], []
    for k in range(N):
        n1, p, n2, w = int(st.n1[k]), int(st.p[k]), int(st.n2[k]), int(st.w[k])
        blk = np.zeros((n1 + p + n2, w))
        if n1:
            blk[:n1, :n] = -np.eye(n)
        if p:
            blk[n1:n1 + p, :n] = np.eye(n)
        if n2:
            blk[n1 + p:, :n] = A[k]
            blk[n1 + p:, n:] = B[k]
        Y.append(blk.T.ravel())
        y.append(np.concatenate([-x0 if p else np.zeros(0), np.zeros(n2)]))
        Hk = np.zeros((w, w))
        Hk[:n, :n] = Qf if k == N - 1 else Q[k]
        if w > n:
            Hk[n:, n:] = R[k]
        H.append(Hk.T.ravel())
    g = np.zeros(int(np.sum(st.w)))
    return st, np.concatenate(Y), np.concatenate(y), np.concatenate(H), g


def test_dp_oracle_time_varying_pinned(lqrx):
    """the time-varying DP restatement (per-knot A_k, B_k, Q_k, R_k)
    (a) reduces bit-exactly to the time-invariant one when every knot repeats the same
    matrices and (b) equals the KAT-pinned KKT oracle on the same time-varying QP."""
    from lqrx.dp import abi_to_batch, to_abi

    n, m, N, bt = 4, 2, 20, 3
    d = lqrx.random_batch(n, m, N, bt, seed=44)
    b = abi_to_batch(d)
    rep = lambda M: np.repeat(M[:, None], N - 1, axis=1)
    dtv = dict(d, A=to_abi(rep(b.A)).ravel(), B=to_abi(rep(b.B)).ravel(),
               Q=to_abi(rep(b.Q)).ravel(), R=to_abi(rep(b.R)).ravel(), tv_AB=1, tv_QR=1)
    a0, a1 = orc.dp_solve_abi(d, N, all_P=True), orc.dp_solve_abi(dtv, N, all_P=True)
    for k in ("K", "P", "X", "U"):
        assert np.array_equal(a0[k], a1[k]), k

    rng = np.random.default_rng(3)
    A = rep(b.A) + 0.1 * rng.standard_normal((bt, N - 1, n, n))
    B = rep(b.B) + 0.1 * rng.standard_normal((bt, N - 1, n, m))
    Q = rep(b.Q) * (1 + rng.random((bt, N - 1, 1, 1)))
    R = rep(b.R) * (1 + rng.random((bt, N - 1, 1, 1)))
    dtv = dict(d, A=to_abi(A).ravel(), B=to_abi(B).ravel(), Q=to_abi(Q).ravel(),
               R=to_abi(R).ravel(), tv_AB=1, tv_QR=1)
    out = orc.dp_solve_abi(dtv, N)
    X = out["X"].reshape(bt, N, n)
    U = out["U"].reshape(bt, N - 1, m)
    for t in range(bt):
        st, Y, y, H, g = lqr_tv_as_kkt(A[t], B[t], Q[t], R[t], b.Qf[t], b.x0[t], N)
        kk = orc.kkt_solve_one(_oracle_struct(st), Y, y, H, g, h_mode=0)
        assert kk["info"] == 0
        z = kk["dz"]
        Xk = np.stack([z[k * (n + m):k * (n + m) + n] for k in range(N)])
        Uk = np.stack([z[k * (n + m) + n:(k + 1) * (n + m)] for k in range(N - 1)])
        assert np.abs(Xk - X[t]).max() <= 1e-10 * max(1.0, np.abs(X[t]).max())
        assert np.abs(Uk - U[t]).max() <= 1e-10 * max(1.0, np.abs(U[t]).max())
