"""Diagnostic (GPU): dp_hex_kernel vs dp_quad_kernel vs the oracle and the 80-bit recursion
on the cfg2-shaped random batch of test_lane_parity_f64 — which trajectories / knots drift."""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "lqr.jl_amd"), os.path.join(os.path.dirname(__file__), "..")]
import lqrx  # noqa: E402
from lqrx.dp import abi_to_batch  # noqa: E402
from oracle import oracle as orc  # noqa: E402

n, m, N, bt = 4, 1, 101, 4101
d = lqrx.random_batch(n, m, N, bt, 300 + 11 * n + m)
b = abi_to_batch(d)
Kx, Px = orc.dp_extended(b.A, b.B, b.Q, b.R, b.Qf, N)
res = {}
for mode in ("quad", "hex"):
    os.environ["LQRX_DP_SMALL"] = mode
    g = lqrx.solve_batch(b, all_P=True)
    ek = np.abs(np.asarray(g["K"], np.longdouble) - Kx).max(axis=(2, 3)) / np.abs(Kx).max(axis=(2, 3))
    res[mode] = (g, ek.astype(np.float64))
    e = res[mode][1].max(axis=1)
    print(mode, "K err vs 80-bit: max", e.max(), "count>1e-10", (e > 1e-10).sum(), "argmax", e.argmax())
gh, eh = res["hex"]
gq, eq = res["quad"]
t = int(eh.max(axis=1).argmax())
print("worst hex trajectory", t, "quad err there", eq[t].max())
print("per-knot K err (hex, quad) for the worst trajectory, knots N-2 .. 0 every 10:")
for k in range(N - 2, -1, -10):
    print(k, eh[t, k], eq[t, k])
dk = np.abs(gh["K"] - gq["K"]).max(axis=(2, 3))
first = [int(np.nonzero(dk[t] > 0)[0].max()) if (dk[t] > 0).any() else -1 for t in range(bt)]
print("hex vs quad: identical trajectories", sum(f < 0 for f in first), "of", bt)
dP = np.abs(gh["P"] - gq["P"]).max(axis=(2, 3)) / np.abs(gq["P"]).max(axis=(2, 3))
print("relative P diff hex vs quad at knot N-2 (first backward step): max", dP[:, N - 2].max(),
      "at knot N-1 (Qf):", dP[:, N - 1].max())
print("K at knot N-2 rel diff max", (np.abs(gh["K"][:, N - 2] - gq["K"][:, N - 2]).max(axis=(1, 2)) /
                                    np.abs(gq["K"][:, N - 2]).max(axis=(1, 2))).max())
Pt = gh["P"][:, N - 2]
print("hex P_{N-1} symmetric?", np.abs(Pt - np.swapaxes(Pt, 1, 2)).max())
