"""Per-shape KKT parity table on the GPU (diagnostic): rel. error of δz / λ vs the C oracle for
the FIL shapes across N, batch, Ginv, and the first knot whose δz block is off."""
import sys
import numpy as np

sys.path.insert(0, "lqr.jl_amd")
sys.path.insert(0, ".")
import lqrx.kkt as K
from oracle import oracle as orc


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


for model in sys.argv[1:] or ["cartpole", "di", "dubins"]:
    for N in (4, 5, 6, 7, 8, 11, 101):
        if model == "cartpole":
            st = K.trajectory_structure(4, 1, N)
        elif model == "di":
            st = K.double_integrator_structure(3, N)
        else:
            st = K.dubins_structure(N)
        if model == "cartpole" and N < 5:
            continue
        for batch in (64, 130):
            for ginv in (1, 0):
                pb = K.random_kkt(st, batch, seed=7 * N + 2, h_mode=2)
                got = K.kkt_solve(pb, ginv=ginv)
                so = orc.KktStructure(st.n, st.m, st.N, st.p)
                ref = orc.kkt_solve_batch(so, batch, pb.Y, pb.y, pb.H, pb.g, h_mode=2, ginv=ginv, nthreads=8)
                rd = ref["dz"].reshape(batch, -1)
                rl = ref["lam"].reshape(batch, -1)
                ed, el = rel(got["dz"], rd), rel(got["lam"], rl)
                msg = ""
                if ed > 1e-10:
                    e = np.abs(got["dz"] - rd).max(0)
                    bad = np.nonzero(e > 1e-10 * np.abs(rd).max())[0]
                    tb = np.nonzero(np.abs(got["dz"] - rd).max(1) > 1e-10 * np.abs(rd).max())[0]
                    msg = f" first bad dz idx {bad[:6]} (of {got['dz'].shape[1]}), bad traj {tb[:8]} ({len(tb)})"
                print(f"{model:8s} N={N:3d} B={batch:4d} ginv={ginv} dz {ed:.2e} lam {el:.2e} info {int((got['info'] != 0).sum())}{msg}",
                      flush=True)
