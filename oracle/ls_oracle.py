"""CPU ORACLE (test infrastructure only) — condensed least-squares and sparse-KKT
formulations of the LQR problem.

Loaded only by tests/ and bench.py's cpu_baseline leg, as the checker; never by the product
path (lqrx.ls / lqrx.kkt.sparse_kkt_solve run on the GPU through liblqrx.so).

Plain numpy restatements, each citing the reference lines (/root/reference/src) it follows:

  least_squares.jl
    LeastSquaresSolver(prob)            :30-56   Hx/Hu zero, Qf/Q/R ← cholesky(·).U
    buildAb!(solver, prob)              :58-103  Ā = Hx·T, b̄ = Hx·L·x0 built from powers of A
    build_least_squares!(solver, prob)  :105-134 T (block Toeplitz), L, Hx, Hu ← chol(R).U
    build_toeplitz(T, L, A, B)          :136-156
    solve!(sol, solver, prob)           :158-192 H = ĀᵀĀ + Hu, y = −Āᵀb̄, potrf/potrs 'U'
                                                 (:cholesky); rollout!
    rollout!(sol, A, B, x0)             :197-202
  Quirks kept (they are the reference's observable behaviour): a fresh solver's Hu is zero,
  so the default (:Ab) solve carries NO control cost; Hu holds chol(R).U (not R) once
  build_least_squares! has run (matbuild :lsq), and persists in the solver.  The :naive
  branch (:185-186, `sol.U .= −H\\y`) assigns a flat vector into a Vector of views and
  throws in Julia, so only :cholesky is restated.  `hu=HU_R` (an extension, not in the reference) puts R on the
  diagonal blocks, which makes the optimum the LQR one — equal to the DP rollout.

  sparse_solver.jl
    _solve!(solver)                     :267-292 HD = G⁻¹Dᵀ, Hg = G⁻¹g, S = D·HD,
                                                 r = d − D·Hg, λ = S⁻¹r, δZ = −HD·λ − Hg
    second_order_correction!            :385-401 δx̂ = −Dᵀ(DDᵀ)⁻¹d
    Dblocks / zinds                     :156-165 the block views of the global D
Parity status: the least-squares restatement is pinned by the known answers of
test/least_squares.jl (T, L, Hx end blocks; Ā = Hx·T, b̄ = Hx·L·x0; normal-equation
residual < 1e-12) and by the DP ≡ LS(hu=R) identity; the sparse restatement is pinned
against the KAT-pinned block KKT oracle (same δz, λ).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

HU_ZERO, HU_CHOL_R, HU_R = 0, 1, 2


def _chol_u(M):
    """cholesky(M).U (LinearAlgebra; least_squares.jl:50-52)."""
    return np.linalg.cholesky(np.asarray(M, dtype=np.float64)).T


def build_toeplitz(A, B, N):
    """build_toeplitz / build_least_squares! (least_squares.jl:105-156): T (N·n × (N−1)·m)
    block lower-Toeplitz of A^{i−1−j}B, L (N·n × n) stacked powers A^j.  N = prob.N."""
    n, m = B.shape
    K = N - 1
    T = np.zeros((N * n, K * m))
    L = np.zeros((N * n, n))
    tmpA = np.eye(n)
    for j in range(0, K + 1):              # :141 loop powers of A
        L[j * n:(j + 1) * n, :] = tmpA
        tmpB = tmpA @ B                    # :151 mul!(tmpB, tmpA, B)
        for i in range(1, K - j + 1):      # :146 loop over columns
            r = i + j
            T[r * n:(r + 1) * n, (i - 1) * m:i * m] = tmpB
        tmpA = A @ tmpA                    # :154
    return T, L


def block_costs(Q, R, Qf, N):
    """Hx (block diag of chol(Q).U, chol(Qf).U at the end) and Hu (chol(R).U blocks) as
    build_least_squares! fills them (least_squares.jl:118-124)."""
    n, m = Q.shape[0], R.shape[0]
    K = N - 1
    Sq, Sf, Sr = _chol_u(Q), _chol_u(Qf), _chol_u(R)
    Hx = np.zeros((N * n, N * n))
    Hu = np.zeros((K * m, K * m))
    for j in range(K + 1):
        Hx[j * n:(j + 1) * n, j * n:(j + 1) * n] = Sq if j < K else Sf
        if j < K:
            Hu[j * m:(j + 1) * m, j * m:(j + 1) * m] = Sr
    return Hx, Hu


def buildAb(A, B, Q, Qf, x0, N):
    """buildAb! (least_squares.jl:58-103): Ā[block i+j, block i−1] = S_{i+j}·A^j·B and
    b̄[block j] = S_j·A^j·x0, S = chol(Q).U for rows < N−1, chol(Qf).U for the last."""
    n, m = B.shape
    K = N - 1
    Sq, Sf = _chol_u(Q), _chol_u(Qf)
    Ab = np.zeros((N * n, K * m))
    bb = np.zeros(N * n)
    An = np.eye(n)
    for j in range(K + 1):                         # :70
        Qi = Sq if j < K else Sf                   # :71-75
        tmpA = Qi @ An                             # :78
        bb[j * n:(j + 1) * n] = tmpA @ x0          # :79-80
        tmpB = An @ B                              # :82
        for i in range(1, K - j + 1):              # :83
            row = i + j                            # :84
            Qi = Sq if row < K else Sf             # :90-94
            Ab[row * n:(row + 1) * n, (i - 1) * m:i * m] = Qi @ tmpB   # :95-96
        An = A @ An                                # :101
    return Ab, bb


def ls_solve(A, B, Q, R, Qf, x0, N, hu=HU_ZERO, matbuild="Ab"):
    """solve!(sol, ::LeastSquaresSolver, prob) (least_squares.jl:158-192) + rollout!
    (:197-202).  Returns dict(U (N−1, m), X (N, n), H, y, Ab, bb, info)."""
    A, B, Q, R, Qf, x0 = (np.asarray(a, dtype=np.float64) for a in (A, B, Q, R, Qf, x0))
    n, m = B.shape
    K = N - 1
    if matbuild == "Ab":                           # :161-162
        Ab, bb = buildAb(A, B, Q, Qf, x0, N)
    else:                                          # :163-168
        T, L = build_toeplitz(A, B, N)
        Hx, _ = block_costs(Q, R, Qf, N)
        Ab = Hx @ T
        bb = Hx @ (L @ x0)
    if hu == HU_ZERO:
        Hu = np.zeros((K * m, K * m))
    elif hu == HU_CHOL_R:
        Hu = block_costs(Q, R, Qf, N)[1]
    else:
        Hu = np.kron(np.eye(K), R)
    H = Ab.T @ Ab + Hu                             # :171-172
    y = -(Ab.T @ bb)                               # :173
    info = 0
    # potrf 'U' reads only the upper triangle of H (:181); with Hu = chol(R).U the matrix
    # H .+= Hu is not symmetric, so symmetrise from the upper triangle as LAPACK sees it
    Hs = np.triu(H) + np.triu(H, 1).T
    try:                                           # :177-183 potrf 'U' / potrs 'U'
        Uc = np.linalg.cholesky(Hs).T
        z = np.linalg.solve(Uc.T, y)
        u = np.linalg.solve(Uc, z)
    except np.linalg.LinAlgError:
        info = 1
        u = np.full(K * m, np.nan)
    U = u.reshape(K, m)
    X = np.zeros((N, n))
    X[0] = x0                                      # :198
    for k in range(K):                             # :199-201
        X[k + 1] = A @ X[k] + B @ U[k]
    return dict(U=U, X=X, H=H, y=y, Ab=Ab, bb=bb, info=info)


# --------------------------------------------------------------------- sparse KKT
def blocks_to_global(st, Y, y, H, g, h_mode=2):
    """Global sparse D (P×NN), d, G (NN×NN), g of SparseConstraintSet / the cost views
    (sparse_solver.jl:17-43, :65-111): Dblocks[k] = D[off_k + (1:rows_k), zinds[k]]
    (:156-160), rows ordered [stage_k; dynamics_k] per knot, G block diagonal."""
    N = st.N
    NN, P = int(np.sum(st.w)), int(np.sum(st.p + st.n2))
    D = sp.lil_matrix((P, NN))
    d = np.zeros(P)
    G = sp.lil_matrix((NN, NN))
    gg = np.zeros(NN)
    oY = oy = oH = og = 0
    off1 = off2 = 0
    for k in range(N):
        n1, rows, w = int(st.n1[k]), int(st.n1[k] + st.p[k] + st.n2[k]), int(st.w[k])
        D[off1:off1 + rows, off2:off2 + w] = np.asarray(Y[oY:oY + rows * w]).reshape(w, rows).T
        d[off1 + n1:off1 + rows] = y[oy:oy + rows - n1]
        if h_mode == 2:
            G[off2:off2 + w, off2:off2 + w] = np.diag(H[oH:oH + w])
            oH += w
        else:
            G[off2:off2 + w, off2:off2 + w] = np.asarray(H[oH:oH + w * w]).reshape(w, w).T
            oH += w * w
        gg[off2:off2 + w] = g[og:og + w]
        oY += rows * w
        oy += rows - n1
        og += w
        off1 += n1 + int(st.p[k])
        off2 += w
    return D.tocsc(), d, G.tocsc(), gg


def sparse_solve(D, d, G, g):
    """_solve!(::SparseSolver) (sparse_solver.jl:267-292).  G⁻¹ is formed block by block in
    the reference (calc_Ginv!, :249-265); a sparse LU of G gives the same products."""
    D = sp.csc_matrix(D)
    G = sp.csc_matrix(G)
    lu = spla.splu(G)
    HD = lu.solve(D.T.toarray())                   # :280 HD = Ginv*D'
    Hg = lu.solve(np.asarray(g, dtype=np.float64))  # :281 Hg = Ginv*g
    S = D @ HD                                     # :285
    r = d - D @ Hg                                 # :287
    lam = np.linalg.solve(0.5 * (S + S.T), r)      # :289 Symmetric(S)\r
    dz = -HD @ lam - Hg                            # :291
    return dict(dz=dz, lam=lam, S=S, r=r)


def sparse_soc(D, d):
    """second_order_correction!(::SparseSolver) (sparse_solver.jl:385-401): δx̂ = −Dᵀ(DDᵀ)⁻¹d."""
    D = sp.csc_matrix(D)
    DDt = (D @ D.T).toarray()
    return -(D.T @ np.linalg.solve(DDt, d))
