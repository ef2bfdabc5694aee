"""CPU tests of the C ABI boundary (no GPU needed): the library loads, exports every
symbol include/lqrx.h declares, validates arguments (LAPACK-style −i codes) before touching
a device, and the synthetic generator is deterministic."""
import ctypes as C

import numpy as np
import pytest


def test_exports_every_header_symbol(lqrx):
    from lqrx import _lib

    lib = _lib.load()
    names = _lib.header_functions()
    assert len(names) >= 9
    for nm in names:
        assert hasattr(lib, nm), nm


def test_abi_version(lqrx):
    assert lqrx.load().lqrx_abi_version() == 5


def test_scratch_trim_without_pools(lqrx):
    """lqrx_scratch_trim before any pool exists (no GPU call made) is a no-op success."""
    assert lqrx.load().lqrx_scratch_trim(-1, 0) == 0


def test_header_kkt_dtype_comment_matches_validation(lqrx):
    """The header's lqrx_kkt_desc.dtype comment names exactly the dtypes the validation accepts
    (it said "LQRX_F64 only" after fp32 KKT shipped)."""
    import os
    import re

    import lqrx.kkt as K
    from lqrx import _lib

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "lqrx.h")).read()
    body = hdr[hdr.index("typedef struct lqrx_kkt_desc"):hdr.index("} lqrx_kkt_desc;")]
    m = re.search(r"int32_t dtype;\s*/\*(.*?)\*/", body, re.S)
    named = set(re.findall(r"LQRX_F(?:32|64)", m.group(1)))
    lib = lqrx.load()
    st = K.trajectory_structure(64, 32, 9)
    accepted = set()
    for name, code in (("LQRX_F64", _lib.F64), ("LQRX_F32", _lib.F32)):
        n = C.c_size_t(0)
        if lib.lqrx_kkt_workspace_size(C.byref(st.desc(8, K.H_DIAG, 1, 0, code)), C.byref(n)) == 0 and n.value > 0:
            accepted.add(name)
    assert named == accepted == {"LQRX_F64", "LQRX_F32"}, (named, accepted)
    n = C.c_size_t(0)
    assert lib.lqrx_kkt_workspace_size(C.byref(st.desc(8, K.H_DIAG, 1, 0, 7)), C.byref(n)) == -1


@pytest.mark.parametrize("field,val,code", [("n", 0, -1), ("m", 0, -1), ("N", 1, -1),
                                            ("dtype", 7, -1), ("p_mode", 3, -1),
                                            ("layout", 2, -1), ("knot_stride_AB", 5, -1),
                                            ("layout", 1, -2),     # SoA is valid: first NULL is A
                                            ("knot_stride_QR", 2, -1),
                                            ("knot_stride_QR", 1, -2)])   # valid: first NULL is A
def test_dp_validation(lqrx, field, val, code):
    from lqrx import _lib

    d = _lib.DpDesc(32, 16, 10, 0, 4, 0, 0, 0, 0)
    setattr(d, field, val)
    rc = lqrx.load().lqrx_dp_solve(C.byref(d), *([None] * 10), None, None)
    assert rc == code
    assert len(lqrx.load().lqrx_last_error()) > 0


def test_dp_time_varying_small_n_accepted(lqrx):
    """Per-knot A_k/B_k (knot_stride 1) is served by the n ≤ 4 lane kernel: validation
    passes and the first NULL pointer is what gets reported."""
    from lqrx import _lib

    d = _lib.DpDesc(4, 1, 10, 0, 4, 0, 0, 1, 1)
    rc = lqrx.load().lqrx_dp_solve(C.byref(d), *([None] * 10), None, None)
    assert rc == -2


def test_dp_null_pointer_codes(lqrx):
    from lqrx import _lib

    d = _lib.DpDesc(8, 4, 10, 0, 4, 0, 0, 0, 0)
    buf = np.zeros(16)
    p = buf.ctypes.data_as(C.c_void_p)
    rc = lqrx.load().lqrx_dp_solve(C.byref(d), None, p, p, p, p, p, p, p, p, p, None, None)
    assert rc == -2          # A is argument 2
    rc = lqrx.load().lqrx_dp_solve(C.byref(d), p, p, p, p, p, p, p, None, p, p, None, None)
    assert rc == -9          # P is argument 9


def test_dp_linear_null_pointer_codes(lqrx):
    """lqrx_dp_solve_linear: lin (argument 8) and each of its pointers are checked, the
    outputs K, P, X, U are arguments 9..12."""
    from lqrx import _lib

    d = _lib.DpDesc(8, 4, 10, 0, 4, 0, 0, 0, 0)
    buf = np.zeros(16)
    p = buf.ctypes.data_as(C.c_void_p)
    lib = lqrx.load()
    assert lib.lqrx_dp_solve_linear(C.byref(d), p, p, p, p, p, p, None, p, p, p, p, None, None) == -8
    for k in ("q", "r", "qf", "d", "p"):
        ln = _lib.DpLinear(p.value, p.value, p.value, p.value, p.value)
        setattr(ln, k, None)
        rc = lib.lqrx_dp_solve_linear(C.byref(d), p, p, p, p, p, p, C.byref(ln), p, p, p, p, None, None)
        assert rc == -8 and k in lib.lqrx_last_error().decode()
    ln = _lib.DpLinear(p.value, p.value, p.value, p.value, p.value)
    rc = lib.lqrx_dp_solve_linear(C.byref(d), p, p, p, p, p, p, C.byref(ln), p, None, p, p, None, None)
    assert rc == -10         # P is argument 10 of the linear entry point
    d.n = 0
    assert lib.lqrx_dp_solve_linear(C.byref(d), p, p, p, p, p, p, C.byref(ln), p, p, p, p, None, None) == -1


def test_kkt_validation(lqrx):
    import lqrx.kkt as K

    st = K.dubins_structure(5)
    d = st.desc(4, 2, 1)
    d.h_mode = 9
    assert lqrx.load().lqrx_kkt_solve(C.byref(d), *([None] * 7), None) == -1
    st2 = K.dubins_structure(5)
    st2.n1[2] = 2            # breaks the A ≡ previous-C aliasing (n1[k] == n2[k-1])
    d2 = st2.desc(4, 2, 1)
    assert lqrx.load().lqrx_kkt_solve(C.byref(d2), *([None] * 7), None) == -1
    d3 = st.desc(4, 2, 1, layout=2)                      # layouts: 0, 1
    assert lqrx.load().lqrx_kkt_solve(C.byref(d3), *([None] * 7), None) == -1
    d4 = st.desc(4, 2, 1, layout=1)                      # SoA is valid: first NULL is Y
    assert lqrx.load().lqrx_kkt_solve(C.byref(d4), *([None] * 7), None) == -2
    big = K.dubins_structure(101).desc(1 << 20, 2, 1, layout=1)   # Y rows past 2 GiB
    assert lqrx.load().lqrx_kkt_solve(C.byref(big), *([None] * 7), None) == lqrx._lib.ERR_UNSUPPORTED


def test_kkt_sizes(lqrx):
    import lqrx.kkt as K

    st = K.dubins_structure(101)
    d = st.desc(1, 2, 1)
    out = [C.c_int64() for _ in range(5)]
    assert lqrx.load().lqrx_kkt_sizes(C.byref(d), *[C.byref(o) for o in out]) == 0
    sY, sy, sH, sg = st.sizes(2)
    assert [o.value for o in out] == [sY, sy, sH, sg, sy]
    assert sg == 101 * 3 + 100 * 2 and sy == 306        # NN = 503, P = (N+1)·n


def test_kkt_workspace_size(lqrx):
    """lqrx_kkt_workspace_size: the FIL slab (wave-major, batch padded to 64, +1 KiB DMA
    overrun) for the Dubins structure; 0 for an empty batch; argument codes."""
    import lqrx.kkt as K

    st = K.dubins_structure(101)
    n = K.workspace_size(st, 16384, K.H_DIAG, 1)
    slot = 27                                            # first-knot slab: B̃ 6, C̃ 6, Ẽ 9, μ 3, λ 3
    assert n == 16384 * 101 * slot * 8 + 1024
    assert K.workspace_size(st, 100, K.H_DIAG, 1) == 128 * 101 * slot * 8 + 1024
    assert K.workspace_size(st, 0, K.H_DIAG, 1) == 0
    assert K.workspace_size(K.double_integrator_structure(3, 11), 64, K.H_DIAG, 1) > 0
    d = st.desc(4, 2, 1)
    assert lqrx.load().lqrx_kkt_workspace_size(C.byref(d), None) == -2


def test_generator_deterministic_and_sharded(lqrx):
    a = lqrx.random_batch(6, 3, 10, 8, seed=99)
    b = lqrx.random_batch(6, 3, 10, 8, seed=99)
    c = lqrx.random_batch(6, 3, 10, 4, seed=99, traj0=4)   # a shard of the same batch
    for k in ("A", "B", "Q", "R", "Qf", "x0"):
        assert np.array_equal(a[k], b[k])
        assert np.array_equal(a[k][len(a[k]) // 2:], c[k])
    from lqrx.dp import abi_to_batch

    bb = abi_to_batch(a)
    assert np.allclose(bb.Q, np.swapaxes(bb.Q, 1, 2))
    assert (np.linalg.eigvalsh(bb.R) > 0).all()


def test_get_last_error_copies(lqrx):
    from lqrx import _lib

    lib = lqrx.load()
    d = _lib.DpDesc(32, 16, 0, 0, 4, 0, 0, 0, 0)          # N = 0 is invalid
    assert lib.lqrx_dp_solve(C.byref(d), *([None] * 10), None, None) < 0
    full = lib.lqrx_last_error()
    buf = C.create_string_buffer(8)
    n = lib.lqrx_get_last_error(buf, 8)
    assert n == len(full) and buf.value == full[:7]
    big = C.create_string_buffer(1024)
    assert lib.lqrx_get_last_error(big, 1024) == len(full) and big.value == full


def test_ls_validation(lqrx):
    """lqrx_ls_solve argument checks (no compute): bad desc fields, NULL pointers, LDS limit."""
    import ctypes as C

    from lqrx import _lib

    lib = _lib.load()
    buf = (C.c_double * 4)()
    ptrs = [C.cast(buf, C.c_void_p)] * 9
    ok = dict(n=4, m=1, N=101, hu_mode=0, batch=2)
    for field, val, code in [("n", 0, -1), ("N", 1, -1), ("hu_mode", 3, -1), ("batch", -1, -1),
                             ("N", 1100, _lib.ERR_UNSUPPORTED)]:
        d = _lib.LsDesc(**{**ok, field: val})
        assert lib.lqrx_ls_solve(C.byref(d), *ptrs, None, None, None) == code, (field, val)
    d = _lib.LsDesc(**ok)
    assert lib.lqrx_ls_solve(C.byref(d), None, *ptrs[1:], None, None, None) == -2
    assert lib.lqrx_ls_solve(C.byref(d), *ptrs[:6], None, ptrs[7], ptrs[8], None, None, None) == -8
    assert lib.lqrx_ls_solve(C.byref(_lib.LsDesc(**{**ok, "batch": 0})), *ptrs, None, None, None) == 0
    assert lib.lqrx_ls_lds_bytes(4, 1, 101) > 0 and lib.lqrx_ls_lds_bytes(0, 1, 5) == 0


def test_constraint_block_dims(lqrx):
    """test/constraint_blocks.jl:25-32 — with dynamics on 1:N-1, an initial-condition
    constraint at knot 1 and a goal at N, block 1 is 2n×(n+m), interior blocks n̄+p+n̄ rows,
    block N is 2n×n (conblocks.jl:79-93 sizing)."""
    import lqrx.kkt as K

    for st in (K.double_integrator_structure(3, 101), K.dubins_structure(11)):
        n, m, N = st.n, st.m, st.N
        rows, w = st.rows, st.w
        assert (rows[0], w[0]) == (2 * n, n + m)
        assert (rows[-1], w[-1]) == (2 * n, n)
        assert all(rows[k] == 2 * n + st.p[k] and w[k] == n + m for k in range(1, N - 1))


def test_kkt_blocks_past_64_accepted(lqrx):
    """Blocks past the large-block kernels (n = 96: 96-row blocks, w = 144) route to the
    workgroup-per-trajectory kernel in fp64 and fp32 (a positive workspace size, no GPU call);
    past 512 rows the validation returns LQRX_ERR_UNSUPPORTED."""
    import lqrx.kkt as K
    from lqrx import _lib

    lib = lqrx.load()
    st = K.trajectory_structure(96, 48, 64)
    for code in (_lib.F64, _lib.F32):
        n = C.c_size_t(0)
        assert lib.lqrx_kkt_workspace_size(C.byref(st.desc(8, K.H_DIAG, 1, 0, code)), C.byref(n)) == 0
        assert n.value > 0
    n = C.c_size_t(0)
    big = K.trajectory_structure(513, 4, 3)
    assert lib.lqrx_kkt_workspace_size(C.byref(big.desc(2, K.H_DIAG, 1, 0, _lib.F64)), C.byref(n)) == -101


def test_julia_shim_ccalls_resolve(lqrx):
    """Every `ccall((:sym, liblqrx), …)` in julia/LQRX.jl names a symbol the library exports
    (Julia is not in this image; this keeps the shim's bindings in step with the ABI)."""
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "julia", "LQRX.jl")).read()
    syms = set(re.findall(r"ccall\(\(:(\w+),\s*liblqrx\)", src))
    assert {"lqrx_dp_solve_host", "lqrx_dp_compute_ctg_host", "lqrx_kkt_solve_host"} <= syms
    lib = lqrx.load()
    for s in sorted(syms):
        assert hasattr(lib, s), s


def test_library_built_from_these_sources(lqrx):
    """Build provenance: the loaded liblqrx.so carries the SHA-256 of the
    sources it was compiled from (lqrx_build_info); it must equal the hash of the sources in
    this tree, so the binary that travels to the GPU box is the one these sources build."""
    from lqrx import _lib

    b = _lib.build_info()
    assert b["src_sha256"] and len(b["src_sha256"]) == 64, b
    assert b["matches_tree"], b


def test_compute_ctg_rejects_asymmetric_cost():
    """lqrx_dp_compute_ctg's precondition (include/lqrx.h): P and Q symmetric — the host
    wrapper refuses a clearly asymmetric one before any device call (no GPU needed)."""
    import numpy as np
    from lqrx.dp import compute_ctg_batch

    rng = np.random.default_rng(0)
    A, B = rng.standard_normal((2, 5, 5)), rng.standard_normal((2, 5, 2))
    Q, R = np.tile(np.eye(5), (2, 1, 1)), np.tile(np.eye(2), (2, 1, 1))
    P = np.tile(np.eye(5), (2, 1, 1))
    P[1, 0, 3] = 0.5                                  # asymmetric
    with pytest.raises(ValueError, match="P must be symmetric"):
        compute_ctg_batch(A, B, Q, R, P)
    Q2 = Q.copy()
    Q2[0, 4, 1] = 1e-3
    with pytest.raises(ValueError, match="Q must be symmetric"):
        compute_ctg_batch(A, B, Q2, R, np.tile(np.eye(5), (2, 1, 1)))


def test_compute_ctg_symmetry_tolerance_follows_dtype():
    """an fp32 P symmetric only to fp32 rounding (~1e-7 relative) passes the
    wrapper's check (tolerance max(1e-10, 100 ulp of the dtype)), the same P in fp64 does not;
    Q is not checked on a gain-only call.  The accepted calls reach the library (here, with no
    GPU, a device error rather than the symmetry ValueError)."""
    import numpy as np
    import lqrx
    from lqrx.dp import compute_ctg_batch

    rng = np.random.default_rng(1)
    A, B = rng.standard_normal((2, 5, 5)), rng.standard_normal((2, 5, 2))
    Q, R = np.tile(np.eye(5), (2, 1, 1)), np.tile(np.eye(2), (2, 1, 1))
    P = np.tile(np.eye(5), (2, 1, 1))
    P[1, 0, 3] += 3e-7

    def reached_library(**kw):
        try:
            compute_ctg_batch(A, B, kw.pop("Q", Q), R, P, **kw)
        except ValueError as e:
            assert "symmetric" not in str(e), e
        except lqrx.LqrxError:
            pass
        return True

    assert reached_library(dtype=lqrx.F32)
    with pytest.raises(ValueError, match="P must be symmetric"):
        compute_ctg_batch(A, B, Q, R, P, dtype=lqrx.F64)
    P[1, 0, 3] = 0.0
    Q2 = Q.copy()
    Q2[0, 4, 1] = 1e-3
    assert reached_library(Q=Q2, gain_only=True)


def test_host_devices_argument_codes(lqrx):
    """the multi-device host entries (ABI 5) validate devices / ndev before
    any device call — NULL devices and ndev < 1 give the negative argument index (dp: 13 / 14,
    dp linear: 14 / 15, kkt: 9 / 10); the descriptor is still argument 1.  (An ordinal that is
    not a device is checked against hipGetDeviceCount: the -m gpu test covers it.)"""
    from lqrx import _lib
    import lqrx.kkt as K

    lib = lqrx.load()
    d = _lib.DpDesc(8, 4, 10, 0, 4, 0, 0, 0, 0)
    buf = np.zeros(16)
    p = buf.ctypes.data_as(C.c_void_p)
    dv = np.zeros(2, np.int32)
    dp_ = dv.ctypes.data_as(C.c_void_p)
    assert lib.lqrx_dp_solve_host_devices(C.byref(d), p, p, p, p, p, p, p, p, p, p, None, None, 2) == -13
    assert lib.lqrx_dp_solve_host_devices(C.byref(d), p, p, p, p, p, p, p, p, p, p, None, dp_, 0) == -14
    ln = _lib.DpLinear(p.value, p.value, p.value, p.value, p.value)
    assert lib.lqrx_dp_solve_linear_host_devices(C.byref(d), p, p, p, p, p, p, C.byref(ln), p, p, p, p, None,
                                                 None, 2) == -14
    assert lib.lqrx_dp_solve_linear_host_devices(C.byref(d), p, p, p, p, p, p, C.byref(ln), p, p, p, p, None,
                                                 dp_, -1) == -15
    assert lib.lqrx_dp_solve_linear_host_devices(C.byref(d), p, p, p, p, p, p, None, p, p, p, p, None,
                                                 dp_, 2) == -8
    kd = K.dubins_structure(5).desc(4, 2, 1)
    assert lib.lqrx_kkt_solve_host_devices(C.byref(kd), p, p, p, p, p, p, None, None, 1) == -9
    assert lib.lqrx_kkt_solve_host_devices(C.byref(kd), p, p, p, p, p, p, None, dp_, 0) == -10
    d.n = 0
    assert lib.lqrx_dp_solve_host_devices(C.byref(d), p, p, p, p, p, p, p, p, p, p, None, dp_, 2) == -1
