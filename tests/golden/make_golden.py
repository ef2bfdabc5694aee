#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz).

Inputs are deterministic (library generator / seeded numpy); expected outputs come from
the CPU oracle (oracle/lqr_oracle.c).  The reference (Julia) cannot run in this container
(no julia binary, unvendored dependencies — SURVEY.md §8(c)), so these are oracle fixtures:
the oracle itself is pinned by tests/test_oracle.py (the reference's test/cholesky_solve.jl
known-answer identities for KKT; DP ≡ the KAT-pinned KKT oracle, dense-QP and DARE
identities for DP).  Re-run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "lqr.jl_amd"), ROOT]

import lqrx  # noqa: E402
import lqrx.kkt as K  # noqa: E402
from lqrx.dp import to_abi  # noqa: E402
from lqrx.models import cartpole_batch  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def dp_fixture(name, d, N):
    out = orc.dp_solve_abi(d, N, all_P=True)
    np.savez_compressed(os.path.join(HERE, name), n=d["n"], m=d["m"], N=N, batch=d["batch"],
                        A=d["A"], B=d["B"], Q=d["Q"], R=d["R"], Qf=d["Qf"], x0=d["x0"],
                        K=out["K"], P=out["P"], X=out["X"], U=out["U"], info=out["info"])


def kkt_fixture(name, st, pb, ginv=1):
    os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
    out = orc.kkt_solve_batch(os_, pb.batch, pb.Y, pb.y, pb.H, pb.g, h_mode=pb.h_mode, ginv=ginv)
    np.savez_compressed(os.path.join(HERE, name), n=st.n, m=st.m, N=st.N, p=st.p,
                        batch=pb.batch, h_mode=pb.h_mode, ginv=ginv, Y=pb.Y, y=pb.y, H=pb.H,
                        g=pb.g, dz=out["dz"], lam=out["lam"], info=out["info"])


def ls_fixture(name, cb, N, hu):
    """Condensed least squares (oracle/ls_oracle.py, least_squares.jl:158-202)."""
    from oracle import ls_oracle as LO

    outs = [LO.ls_solve(cb.A[b], cb.B[b], cb.Q[b], cb.R[b], cb.Qf[b], cb.x0[b], N, hu=hu)
            for b in range(cb.A.shape[0])]
    np.savez_compressed(os.path.join(HERE, name), N=N, hu=hu, A=cb.A, B=cb.B, Q=cb.Q, R=cb.R,
                        Qf=cb.Qf, x0=cb.x0, U=np.stack([o["U"] for o in outs]),
                        X=np.stack([o["X"] for o in outs]))


def main():
    cb = cartpole_batch(4, 101, seed=1)
    d = {k: to_abi(getattr(cb, k)).ravel() for k in ("A", "B", "Q", "R", "Qf")}
    d.update(x0=cb.x0.ravel(), n=4, m=1, batch=4)
    dp_fixture("dp_cartpole_N101.npz", d, 101)
    d = lqrx.random_batch(6, 3, 20, 3, seed=2024)
    dp_fixture("dp_random_n6_m3_N20.npz", d, 20)
    d = lqrx.random_batch(32, 16, 16, 2, seed=2025)
    dp_fixture("dp_random_n32_m16_N16.npz", d, 16)
    st = K.dubins_structure(11)
    kkt_fixture("kkt_dubins_N11_diag.npz", st, K.random_kkt(st, 4, seed=7, h_mode=K.H_DIAG))
    kkt_fixture("kkt_dubins_N11_soc.npz", st, K.random_kkt(st, 4, seed=8, h_mode=K.H_DIAG), ginv=0)
    st = K.double_integrator_structure(2, 12)
    kkt_fixture("kkt_di2_N12_dense.npz", st, K.random_kkt(st, 3, seed=9, h_mode=K.H_DENSE))
    cb = cartpole_batch(3, 41, seed=3)
    for hu in (0, 1, 2):
        ls_fixture(f"ls_cartpole_N41_hu{hu}.npz", cb, 41, hu)


if __name__ == "__main__":
    main()
