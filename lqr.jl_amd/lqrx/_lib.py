"""ctypes binding of the lqrx C ABI (include/lqrx.h).

The shared library is built in-tree (``lqr.jl_amd/csrc/Makefile`` → ``lqrx/liblqrx.so``).
There is no fallback: if the library is missing, importing the compute entry points raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LQRX_LIB") or os.path.join(_HERE, "liblqrx.so")
HEADER_PATH = os.path.abspath(os.path.join(_HERE, "..", "..", "include", "lqrx.h"))

F64, F32 = 0, 1
ERR_HIP, ERR_UNSUPPORTED, ERR_NODEVICE = -100, -101, -102


class DpDesc(C.Structure):
    """Mirror of ``lqrx_dp_desc``."""

    _fields_ = [
        ("n", C.c_int32), ("m", C.c_int32), ("N", C.c_int32), ("dtype", C.c_int32),
        ("batch", C.c_int64), ("layout", C.c_int32), ("p_mode", C.c_int32),
        ("knot_stride_AB", C.c_int64), ("knot_stride_QR", C.c_int64),
    ]


class DpLinear(C.Structure):
    """Mirror of ``lqrx_dp_linear`` (linear cost terms q, r, qf in; d, p out)."""

    _fields_ = [("q", C.c_void_p), ("r", C.c_void_p), ("qf", C.c_void_p),
                ("d", C.c_void_p), ("p", C.c_void_p)]


class KktDesc(C.Structure):
    """Mirror of ``lqrx_kkt_desc``."""

    _fields_ = [
        ("N", C.c_int32), ("dtype", C.c_int32), ("batch", C.c_int64),
        ("n1", C.POINTER(C.c_int32)), ("p", C.POINTER(C.c_int32)),
        ("n2", C.POINTER(C.c_int32)), ("w", C.POINTER(C.c_int32)),
        ("h_mode", C.c_int32), ("ginv", C.c_int32), ("layout", C.c_int32),
        ("reserved", C.c_int32),
    ]


class SqpDesc(C.Structure):
    """Mirror of ``lqrx_dubins_sqp_desc``."""

    _fields_ = [
        ("N", C.c_int32), ("max_iters", C.c_int32), ("batch", C.c_int64), ("dt", C.c_double),
        ("Q", C.c_double * 3), ("R", C.c_double * 2), ("Qf", C.c_double * 3), ("mu", C.c_double),
        ("tol_p", C.c_double), ("tol_d", C.c_double),
    ]


class TrajSqpDesc(C.Structure):
    """Mirror of ``lqrx_sqp_desc``."""

    _fields_ = [
        ("model", C.c_int32), ("N", C.c_int32), ("max_iters", C.c_int32), ("stage_rows", C.c_int32),
        ("batch", C.c_int64), ("dt", C.c_double), ("Q", C.c_double * 8), ("R", C.c_double * 8),
        ("Qf", C.c_double * 8), ("params", C.c_double * 4), ("mu", C.c_double),
        ("tol_p", C.c_double), ("tol_d", C.c_double), ("stage_A", C.c_double * 32), ("stage_b", C.c_double * 4),
    ]


class LsDesc(C.Structure):
    """Mirror of ``lqrx_ls_desc``."""

    _fields_ = [("n", C.c_int32), ("m", C.c_int32), ("N", C.c_int32), ("hu_mode", C.c_int32),
                ("batch", C.c_int64)]


_VP = C.c_void_p
_SIGS = {
    "lqrx_abi_version": (C.c_int, []),
    "lqrx_build_info": (C.c_char_p, []),
    "lqrx_last_error": (C.c_char_p, []),
    "lqrx_get_last_error": (C.c_int, [C.c_char_p, C.c_size_t]),
    "lqrx_device_available": (C.c_int, []),
    "lqrx_scratch_trim": (C.c_int, [C.c_int32, C.c_size_t]),
    "lqrx_dp_solve": (C.c_int, [C.POINTER(DpDesc)] + [_VP] * 10 + [_VP, _VP]),
    "lqrx_dp_solve_host": (C.c_int, [C.POINTER(DpDesc)] + [_VP] * 10 + [_VP]),
    "lqrx_dp_compute_ctg": (C.c_int, [C.POINTER(DpDesc)] + [_VP] * 8 + [_VP]),
    "lqrx_dp_compute_ctg_host": (C.c_int, [C.POINTER(DpDesc)] + [_VP] * 8),
    "lqrx_dp_solve_linear": (C.c_int, [C.POINTER(DpDesc)] + [_VP] * 6 + [C.POINTER(DpLinear)]
                             + [_VP] * 4 + [_VP, _VP]),
    "lqrx_dp_solve_linear_host": (C.c_int, [C.POINTER(DpDesc)] + [_VP] * 6
                                  + [C.POINTER(DpLinear)] + [_VP] * 5),
    "lqrx_dp_solve_host_devices": (C.c_int, [C.POINTER(DpDesc)] + [_VP] * 10 + [_VP, _VP, C.c_int32]),
    "lqrx_dp_solve_linear_host_devices": (C.c_int, [C.POINTER(DpDesc)] + [_VP] * 6 + [C.POINTER(DpLinear)]
                                          + [_VP] * 5 + [_VP, C.c_int32]),
    "lqrx_kkt_solve_host_devices": (C.c_int, [C.POINTER(KktDesc)] + [_VP] * 7 + [_VP, C.c_int32]),
    "lqrx_kkt_solve": (C.c_int, [C.POINTER(KktDesc)] + [_VP] * 7 + [_VP]),
    "lqrx_kkt_solve_host": (C.c_int, [C.POINTER(KktDesc)] + [_VP] * 7),
    "lqrx_kkt_sizes": (C.c_int, [C.POINTER(KktDesc)] + [C.POINTER(C.c_int64)] * 5),
    "lqrx_kkt_workspace_size": (C.c_int, [C.POINTER(KktDesc), C.POINTER(C.c_size_t)]),
    "lqrx_kkt_solve_ws": (C.c_int, [C.POINTER(KktDesc)] + [_VP] * 7 + [_VP, C.c_size_t, _VP]),
    "lqrx_dubins_sqp_solve": (C.c_int, [C.POINTER(SqpDesc)] + [_VP] * 6 + [_VP]),
    "lqrx_dubins_sqp_solve_host": (C.c_int, [C.POINTER(SqpDesc)] + [_VP] * 6),
    "lqrx_sqp_model_dims": (C.c_int, [C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "lqrx_sqp_solve": (C.c_int, [C.POINTER(TrajSqpDesc)] + [_VP] * 6 + [_VP]),
    "lqrx_sqp_solve_host": (C.c_int, [C.POINTER(TrajSqpDesc)] + [_VP] * 6),
    "lqrx_ls_lds_bytes": (C.c_size_t, [C.c_int32, C.c_int32, C.c_int32]),
    "lqrx_ls_solve": (C.c_int, [C.POINTER(LsDesc)] + [_VP] * 11 + [_VP]),
    "lqrx_ls_solve_host": (C.c_int, [C.POINTER(LsDesc)] + [_VP] * 9),
    "lqrx_make_random_dp": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, C.c_int64, C.c_uint64,
                                      C.c_int32] + [_VP] * 6),
}

_lib = None


def load() -> C.CDLL:
    """Load liblqrx.so (once).  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"lqrx native library not built: {LIB_PATH} is missing "
            "(run `make -C lqr.jl_amd/csrc` or __graft_entry__.build())")
    # One HIP runtime per process: torch ships its own libamdhip64 (same soname as
    # /opt/rocm's, which liblqrx.so links).  Whichever loads first serves both, and torch
    # finds no GPU on a runtime other than its own — so let torch's load first when present.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def header_functions() -> list[str]:
    """Names of every function declared in include/lqrx.h."""
    src = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char \*)\s*(lqrx_\w+)\s*\(", src, re.M)))


class LqrxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"lqrx error {code}: {msg}")
        self.code = code


def check(code: int) -> int:
    """Raise LqrxError for negative return codes; return 0/1 otherwise."""
    if code < 0:
        raise LqrxError(code, load().lqrx_last_error().decode())
    return code


def source_hash(root: str | None = None) -> str:
    """SHA-256 of the library sources exactly as the Makefile hashes them (csrc/*.hip, *.h,
    *.cpp in sorted name order, then include/lqrx.h)."""
    import glob
    import hashlib

    root = root or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    csrc = os.path.join(root, "lqr.jl_amd", "csrc")
    names = sorted(os.path.basename(f) for pat in ("*.hip", "*.h", "*.cpp")
                   for f in glob.glob(os.path.join(csrc, pat)))
    h = hashlib.sha256()
    for f in [os.path.join(csrc, nm) for nm in names] + [os.path.join(root, "include", "lqrx.h")]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _code_digest(path: str) -> str:
    """SHA-256 (16 hex) of a C/C++/HIP source with its comments and blank space removed: an edit
    of the documentation keeps the digest, an edit of the code changes it."""
    import hashlib

    with open(path) as fh:
        src = fh.read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    src = re.sub(r"\s+", " ", src).strip()
    return hashlib.sha256(src.encode()).hexdigest()[:16]


def _root(root: str | None) -> str:
    return root or os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def kernel_unit(kernel: str, root: str | None = None) -> str | None:
    """The csrc/*.hip translation unit that defines the __global__ function `kernel` (its base
    name, e.g. ``kb_fuse_mid_kernel``), relative to the repository root, or None."""
    import glob

    root = _root(root)
    base = re.findall(r"(\w+)", kernel.split("<")[0])[-1]
    for f in sorted(glob.glob(os.path.join(root, "lqr.jl_amd", "csrc", "*.hip"))):
        with open(f) as fh:
            src = fh.read()
        if re.search(r"__global__[^;{}]*?\b" + re.escape(base) + r"\s*\(", src, re.S):
            return os.path.relpath(f, root)
    return None


def kernel_source_digest(units, root: str | None = None) -> dict:
    """{path: code digest} of the given translation units and every local header they include
    (recursively; ``lqrx.h`` resolves to include/) — the sources a measured kernel's code comes
    from.  Recorded with each PMC traffic figure (tools/traffic_json.py) and recomputed by
    bench.py, which drops a figure whose kernel's code has changed since."""
    root = _root(root)
    out, todo = {}, list(units)
    while todo:
        rel = todo.pop()
        if rel in out:
            continue
        path = os.path.join(root, rel)
        if not os.path.exists(path):
            out[rel] = None
            continue
        out[rel] = _code_digest(path)
        with open(path) as fh:
            for inc in re.findall(r'#\s*include\s*"([^"]+)"', fh.read()):
                cand = os.path.normpath(os.path.join(os.path.dirname(rel), inc))
                if os.path.basename(inc) == "lqrx.h":
                    cand = os.path.join("include", "lqrx.h")
                todo.append(cand)
    return dict(sorted(out.items()))


def build_info() -> dict:
    """The loaded library's build record and whether it matches the sources in this tree."""
    info = load().lqrx_build_info().decode()
    fields = dict(kv.split("=", 1) for kv in info.split(" ") if "=" in kv)
    tree = source_hash()
    return {"info": info, "src_sha256": fields.get("src_sha256"), "tree_sha256": tree,
            "matches_tree": fields.get("src_sha256") == tree}
