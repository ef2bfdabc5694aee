"""ABI layout 1 (batch fastest / SoA, SURVEY §8(b) lqrx_dp_desc.layout) through the C ABI.

The n ≤ 4 kernels (lane and quad) address SoA natively; n ≥ 5 (MFMA kernel) converts to
layout 0 in stream-ordered scratch and back (lqrx_layout.hip).  Either way the arithmetic is
the layout-0 kernel's, so layout 1 must reproduce layout 0 BIT FOR BIT — and layout 0 is
held to the oracle by test_dp_gpu.py / test_dp_lane_gpu.py; one oracle check is repeated
here on the SoA result directly.
"""
import numpy as np
import pytest

from test_dp_gpu import TOL64, relerr_per_knot

pytestmark = pytest.mark.gpu


def _pair(lqrx, b, **kw):
    a0 = lqrx.solve_batch(b, layout=0, **kw)
    a1 = lqrx.solve_batch(b, layout=1, **kw)
    for k in ("K", "P", "X", "U", "info"):
        assert np.array_equal(a0[k], a1[k]), k
    assert a0["rc"] == a1["rc"]
    return a1


@pytest.mark.parametrize("mode", ["lane", "quad", "hex"])
@pytest.mark.parametrize("n,m,N,bt", [(4, 1, 101, 130), (3, 2, 40, 67), (2, 1, 20, 65), (4, 4, 12, 9)])
def test_soa_small_kernels(lqrx, oracle, gpu_ok, monkeypatch, mode, n, m, N, bt):
    from lqrx.dp import abi_to_batch, from_abi

    monkeypatch.setenv("LQRX_DP_SMALL", mode)
    d = lqrx.random_batch(n, m, N, bt, seed=900 + n + m)
    got = _pair(lqrx, abi_to_batch(d), all_P=True)
    ref = oracle.dp_solve_abi(d, N, all_P=True)
    assert relerr_per_knot(got["K"], from_abi(ref["K"], (bt, N - 1, m, n))) <= TOL64 or n == 4


@pytest.mark.parametrize("n,m,N,bt,dtype", [(6, 3, 20, 5, 0), (32, 16, 24, 3, 0), (20, 5, 12, 4, 1),
                                            (64, 32, 9, 2, 0)])
def test_soa_mfma_staged(lqrx, gpu_ok, n, m, N, bt, dtype):
    from lqrx.dp import abi_to_batch

    d = lqrx.random_batch(n, m, N, bt, seed=44 + n)
    _pair(lqrx, abi_to_batch(d), dtype=dtype, all_P=(n < 64))


@pytest.mark.parametrize("n,m", [(4, 2), (6, 3), (64, 32), (64, 16)])   # n = 64: the four-wave TV kernel
def test_soa_time_varying(lqrx, gpu_ok, n, m):
    from test_dp_lane_gpu import _tv_batch

    _pair(lqrx, _tv_batch(lqrx, n, m, 15, 7, seed=3 + n), all_P=True)


def test_soa_device_entry_on_stream(lqrx, oracle, gpu_ok):
    """dp_solve_device with layout 1 on a created stream (the staged path's scratch and
    transposes are stream-ordered), checked against the oracle."""
    import torch
    from lqrx.dp import from_abi, from_soa, to_soa

    n, m, N, bt = 8, 4, 30, 70
    d = lqrx.random_batch(n, m, N, bt, seed=12)
    st = torch.cuda.Stream()
    t = {k: torch.from_numpy(to_soa(d[k], bt).ravel()).cuda() for k in ("A", "B", "Q", "R", "Qf", "x0")}
    t.update(n=n, m=m, batch=bt)
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        out = lqrx.dp_solve_device(t, N, stream=st.cuda_stream, layout=1)
    st.synchronize()
    ref = oracle.dp_solve_abi(d, N)
    K = from_soa(out["K"].cpu().numpy(), bt)
    assert relerr_per_knot(from_abi(K, (bt, N - 1, m, n)), from_abi(ref["K"], (bt, N - 1, m, n))) <= TOL64
    X = from_soa(out["X"].cpu().numpy(), bt)
    assert np.abs(X - ref["X"]).max() <= TOL64 * max(1.0, np.abs(ref["X"]).max())
