# debug: TV parity at a given shape, where do GPU results go bad (knot-wise)
import sys, numpy as np
sys.path[:0]=['lqr.jl_amd','.','tests']
import lqrx
from test_dp_lane_gpu import _tv_batch
from test_dp_gpu import relerr_per_knot
from lqrx.dp import to_abi, from_abi
from oracle import oracle as orc
n,m,N,bt=[int(x) for x in sys.argv[1:5]]
for tvab, tvqr in ((1,1),(1,0),(0,1)):
    b=_tv_batch(lqrx,n,m,N,bt,seed=21+n,tv_ab=bool(tvab),tv_qr=bool(tvqr))
    got=lqrx.solve_batch(b, all_P=True)
    d = {k: to_abi(getattr(b, k)).ravel() for k in ("A", "B", "Q", "R", "Qf")}
    d.update(x0=b.x0.ravel(), n=n, m=m, batch=bt, tv_AB=tvab, tv_QR=tvqr)
    ref = orc.dp_solve_abi(d, N, all_P=True)
    K=from_abi(ref["K"], (bt, N-1, m, n)); P=from_abi(ref["P"], (bt, N, n, n))
    print("tv", tvab, tvqr, "info", got["info"], "K nan per knot", np.isnan(got["K"]).any(axis=(2,3)).astype(int).tolist())
    print("   P nan per knot", np.isnan(got["P"]).any(axis=(2,3)).astype(int).tolist())
    ok = ~np.isnan(got["K"]).any()
    if ok: print("   relerr K", relerr_per_knot(got["K"], K), "P", relerr_per_knot(got["P"], P))
import copy
b0=_tv_batch(lqrx,n,m,N,bt,seed=21+n,tv_ab=False,tv_qr=True)
base=lqrx.dp.abi_to_batch(lqrx.random_batch(n,m,N,bt,21+n))
rep=lambda M: np.repeat(M[:,None],N-1,axis=1)
for name, Q, R in (("Q only", b0.Q, rep(base.R)), ("R only", rep(base.Q), b0.R)):
    bb=copy.copy(base); bb.Q=Q; bb.R=R
    got=lqrx.solve_batch(bb, all_P=True)
    print(name, "K nan per knot", np.isnan(got["K"]).any(axis=(2,3)).astype(int).tolist())
