"""Run by tests/test_kkt_gpu.py::test_kkt_meta_cache_overflow in a child process with
LQRX_META_CACHE=1: only the first structure is cached, every other one takes the per-call,
stream-ordered table path (lqrx_api.cpp device_meta).  Alternates structures on the null
stream and on a created stream and checks every solve against the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lqr.jl_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import lqrx  # noqa: E402
import lqrx.kkt as K  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    assert os.environ.get("LQRX_META_CACHE") == "1"
    lqrx.load()
    stream = torch.cuda.Stream()
    cases = []
    for N, batch, h, seed in [(11, 4, 0, 18), (101, 64, 2, 5), (3, 5, 2, 4), (9, 33, 1, 8)]:
        st = K.dubins_structure(N)
        pb = K.random_kkt(st, batch, seed=seed, h_mode=h)
        ref = orc.kkt_solve_batch(orc.KktStructure(st.n, st.m, st.N, st.p), batch, pb.Y, pb.y,
                                  pb.H, pb.g, h_mode=h, nthreads=4)
        t = {k: torch.from_numpy(getattr(pb, k).ravel()).cuda() for k in ("Y", "y", "H", "g")}
        t["batch"] = batch
        cases.append((st, pb, t, ref))
    worst = 0.0
    for it in range(4):
        for st, pb, t, ref in cases:
            if it % 2:
                with torch.cuda.stream(stream):
                    got = K.kkt_solve_device(st, t, pb.h_mode, 1, stream=stream.cuda_stream)
                stream.synchronize()
            else:
                got = K.kkt_solve_device(st, t, pb.h_mode, 1)
                torch.cuda.synchronize()
            for k in ("dz", "lam"):
                a = got[k].cpu().numpy()
                b = ref[k]
                worst = max(worst, float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)))
    print(f"meta overflow path: worst rel err {worst:.2e}")
    sys.exit(0 if worst <= 1e-10 else 1)


if __name__ == "__main__":
    main()
