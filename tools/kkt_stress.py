"""Repeat small KKT solves many times in one process and report the worst error vs the
oracle (catches intermittent staging races that a single parity run can miss)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "lqr.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import lqrx.kkt as K
from oracle import oracle as orc

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
worst = 0.0
for N, batch in [(11, 4), (3, 5), (11, 67), (101, 256), (101, 4096)]:
    for h in (0, 1, 2):
        st = K.dubins_structure(N)
        pb = K.random_kkt(st, batch, seed=7 + N + h, h_mode=h)
        os_ = orc.KktStructure(st.n, st.m, st.N, st.p)
        ref = orc.kkt_solve_batch(os_, pb.batch, pb.Y, pb.y, pb.H, pb.g, h_mode=h, ginv=1, nthreads=8)
        rd = ref["dz"].reshape(batch, -1)
        e = 0.0
        bad = 0
        for r in range(reps):
            got = K.kkt_solve(pb)
            er = np.abs(got["dz"] - rd).max() / np.abs(rd).max()
            bad += er > 1e-10
            e = max(e, er)
        worst = max(worst, e)
        print(f"N={N} batch={batch} h={h} worst={e:.2e} bad={bad}/{reps}", flush=True)
print("WORST", worst)
sys.exit(0 if worst <= 1e-10 else 1)
