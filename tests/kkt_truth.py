"""Truth reference for ill-conditioned KKT parity cases (test helper, no GPU).

A few random problems of the near-square structures (DoubleIntegrator(3) at N = 4, cond(S)
up to ~7e6) put the fp64 oracle itself ~5e-11 away from the exact solution, so a flat 1e-10
against the oracle measures two roundings, not the kernel.  For those trajectories the
check falls back to the rule the DP lane tests use: the kernel may be no further
from the truth than C × max(the oracle's own error, tol), the truth being the full KKT system
[H Dᵀ; D 0][δz; λ] = [−g; −d] (test/cholesky_solve.jl:18-44's identities; H = I, g = 0 for the
second-order correction, cholesky_solver.jl:254-273) solved in fp64 with five rounds of
iterative refinement whose residuals are formed in extended precision (numpy longdouble).
"""
import numpy as np

from oracle import oracle as orc

C = 4.0


def _truth_one(os_, pb, t, ginv):
    sl = lambda a: np.asarray(a).reshape(pb.batch, -1)[t]
    dd = orc.kkt_dense(os_, sl(pb.Y), sl(pb.y), sl(pb.H), sl(pb.g), h_mode=pb.h_mode)
    H, D, g, d = dd["H"], dd["D"], dd["g"], dd["d"]
    if not ginv:
        H, g = np.eye(H.shape[0]), np.zeros_like(g)
    NN, P = H.shape[0], D.shape[0]
    A = np.block([[H, D.T], [D, np.zeros((P, P))]])
    b = np.concatenate([-g, -d])
    x = np.linalg.solve(A, b)
    Al, bl = A.astype(np.longdouble), b.astype(np.longdouble)
    for _ in range(5):
        r = (bl - Al @ x.astype(np.longdouble)).astype(np.float64)
        x = x + np.linalg.solve(A, r)
    return x[:NN], x[NN:]


def check(st, pb, ginv, got, ref, tol, scale="batch", fallback=False):
    """Assert δz and λ match the oracle within tol.  Only with fallback=True (the documented
    ill-conditioned case, DoubleIntegrator(3) at N = 4) may an offending trajectory instead be
    within C·max(err_oracle, tol) of the refined truth; otherwise every trajectory must meet
    tol flat, so a regression elsewhere cannot pass at a multiple of it.  scale "batch": errors
    over the batch-wide max |ref| (test_kkt_gpu's rel); "traj": per trajectory."""
    os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
    for key, part in (("dz", 0), ("lam", 1)):
        a = np.asarray(got[key], np.float64).reshape(pb.batch, -1)
        b = np.asarray(ref[key], np.float64).reshape(pb.batch, -1)
        den = (np.full(pb.batch, np.abs(b).max()) if scale == "batch" else np.abs(b).max(axis=1))
        den = np.maximum(den, 1e-300)
        e = np.abs(a - b).max(axis=1) / den
        if not fallback:
            assert (e <= tol).all(), (key, np.nonzero(e > tol)[0][:8].tolist(), float(e.max()))
            continue
        for t in np.nonzero(e > tol)[0]:
            tr = _truth_one(os_, pb, int(t), ginv)[part]
            ek = np.abs(a[t] - tr).max() / den[t]
            eo = np.abs(b[t] - tr).max() / den[t]
            assert ek <= C * max(eo, tol), (key, int(t), e[t], ek, eo)
