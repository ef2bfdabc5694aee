"""Diagnose intermittent KKT mismatches: alternate two structures so the memory pool hands
back stale buffers, and report where (trajectory, entry) the bad results are."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "lqr.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import lqrx.kkt as K
from oracle import oracle as orc


def case(N, batch, h, seed):
    st = K.dubins_structure(N)
    pb = K.random_kkt(st, batch, seed=seed, h_mode=h)
    os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
    ref = orc.kkt_solve_batch(os_, pb.batch, pb.Y, pb.y, pb.H, pb.g, h_mode=h, ginv=1, nthreads=8)
    return pb, ref["dz"].reshape(batch, -1), ref["lam"].reshape(batch, -1)


A = case(11, 4, 0, 18)
B = case(101, 256, 2, 5)
C = case(11, 67, 1, 3)
tot = 0
first = None
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    for name, (pb, rd, rl) in (("A", A), ("B", B), ("C", C)):
        got = K.kkt_solve(pb)
        d = np.abs(got["dz"] - rd) / np.abs(rd).max()
        l = np.abs(got["lam"] - rl) / np.abs(rl).max()
        if d.max() > 1e-10 or l.max() > 1e-10:
            tot += 1
            first = r if first is None else first
            if tot > 4:
                continue
            bt, bz = np.nonzero(d > 1e-10)
            bl_t, bl = np.nonzero(l > 1e-10)
            print(f"rep {r} {name}: dz err {d.max():.2e} traj {sorted(set(bt.tolist()))[:10]} "
                  f"entries {sorted(set(bz.tolist()))[:40]} | lam err {l.max():.2e} entries "
                  f"{sorted(set(bl.tolist()))[:40]} info {got['info'][:8]}", flush=True)
print("BAD", tot, "first bad rep", first)
