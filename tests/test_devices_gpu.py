"""Multi-device solves through the C ABI (ABI 5, include/lqrx.h lqrx_*_host_devices) — VERDICT
r5 next #3, SURVEY §8(e): the batch split into contiguous shards, one thread + stream per entry
of devices[], each shard the single-device solve of its slice (dynamic_programming.jl:54-72 /
cholesky_solver.jl:166-182 per shard).  On the one-GPU box devices = [0, 0] (and [0, 0, 0])
runs two (three) shards concurrently on GPU 0; every trajectory's result must equal the
single-device call bit for bit, in both layouts, with info and the return code intact.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dp_batch(n, m, N, bt, seed, tv=False):
    import dataclasses
    from lqrx.dp import abi_to_batch, random_batch

    b = abi_to_batch(random_batch(n, m, N, bt, seed))
    if tv:
        rng = np.random.default_rng(seed)
        b = dataclasses.replace(b, A=b.A[:, None].repeat(N - 1, 1) * (1 + 0.01 * rng.standard_normal((bt, N - 1, 1, 1))),
                                B=b.B[:, None].repeat(N - 1, 1))
    return b


def _same(a, b):
    for k in ("K", "P", "X", "U", "info"):
        assert np.array_equal(a[k], b[k]), k
    assert a["rc"] == b["rc"]


@pytest.mark.parametrize("n,m,N,bt,layout,devices", [
    (32, 16, 64, 301, 0, [0, 0]),          # cfg4 shape, ragged shards (151 + 150)
    (32, 16, 64, 301, 1, [0, 0, 0]),       # layout 1: strided element rows per shard
    (64, 16, 12, 37, 0, [0, 0]),           # fp64 n = 64: the four-wave kernel per shard
    (64, 32, 10, 9, 0, [0, 0, 0]),         # m = 32: the four-wave kernel with the inverse on wave 3
    (6, 3, 40, 129, 0, [0, 0]),
    (4, 1, 101, 4096, 0, [0, 0]),          # cfg2 shape: both shards and the whole batch on the quad kernel
    (4, 1, 101, 1000, 1, [0, 0]),          # n ≤ 4 layout 1 (native SoA lane kernels)
])
def test_dp_devices_bit_identical(lqrx, gpu_ok, n, m, N, bt, layout, devices):
    from lqrx.dp import solve_batch

    b = _dp_batch(n, m, N, bt, seed=n * 7 + bt)
    one = solve_batch(b, layout=layout)
    many = solve_batch(b, layout=layout, devices=devices)
    _same(one, many)


def test_dp_devices_time_varying_linear_and_all_p(lqrx, gpu_ok):
    """Time-varying A, linear cost terms (lqrx_dp_solve_linear_host_devices) and p_mode 1."""
    import dataclasses
    from lqrx.dp import solve_batch

    b = _dp_batch(16, 4, 20, 65, seed=3, tv=True)
    rng = np.random.default_rng(5)
    bl = dataclasses.replace(b, q=rng.standard_normal((65, 16)), r=rng.standard_normal((65, 4)),
                             qf=rng.standard_normal((65, 16)))
    for bb, allp in ((b, True), (bl, False), (bl, True)):
        one = solve_batch(bb, all_P=allp)
        many = solve_batch(bb, all_P=allp, devices=[0, 0])
        _same(one, many)
        if bb.q is not None:
            assert np.array_equal(one["d"], many["d"]) and np.array_equal(one["p"], many["p"])


def test_dp_devices_info_and_more_shards_than_trajectories(lqrx, gpu_ok):
    """A non-SPD R in one trajectory: info lands at its global index (shard offset applied), the
    call returns 1; ndev > batch leaves the extra shards empty."""
    from lqrx.dp import solve_batch

    b = _dp_batch(8, 2, 10, 5, seed=9)
    b.R[3] = -np.eye(2)
    one = solve_batch(b)
    many = solve_batch(b, devices=[0] * 7)
    _same(one, many)
    assert one["rc"] == 1 and one["info"][3] != 0 and (np.delete(one["info"], 3) == 0).all()


def test_devices_invalid_ordinal(lqrx, gpu_ok):
    """An ordinal past hipGetDeviceCount returns the devices argument's index."""
    from lqrx import _lib
    from lqrx.dp import solve_batch

    b = _dp_batch(8, 2, 10, 4, seed=1)
    with pytest.raises(_lib.LqrxError) as e:
        solve_batch(b, devices=[0, 4096])
    assert e.value.code == -13 and "devices[1]" in str(e.value)
    with pytest.raises(_lib.LqrxError) as e:
        solve_batch(b, devices=[-1])
    assert e.value.code == -13


@pytest.mark.parametrize("layout,h_mode,dtype", [(0, 2, 0), (1, 2, 0), (0, 0, 0), (0, 2, 1)])
def test_kkt_devices_bit_identical(lqrx, gpu_ok, layout, h_mode, dtype):
    """lqrx_kkt_solve_host_devices: Dubins (the FIL kernel, native layout 1), dense H, and an
    fp32 large-block structure, sharded over [0, 0, 0]."""
    import lqrx.kkt as K

    if dtype == 1:
        st = K.trajectory_structure(16, 8, 12)
        pb = K.random_kkt(st, 77, seed=4, h_mode=h_mode, dyn="dense")
    else:
        st = K.dubins_structure(101)
        pb = K.random_kkt(st, 1001, seed=2 + h_mode, h_mode=h_mode)
    one = K.kkt_solve(pb, layout=layout, dtype=dtype)
    many = K.kkt_solve(pb, layout=layout, dtype=dtype, devices=[0, 0, 0])
    for k in ("dz", "lam", "info"):
        assert np.array_equal(one[k], many[k]), k
    assert one["rc"] == many["rc"] == 0
