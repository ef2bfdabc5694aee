"""Host-side mirror of the reference's block-tridiagonal KKT surface (CholeskySolver._solve!).

Reference (Julia, /root/reference/src):
  ConstraintBlock(n1, p, n2, w): Y = [D2; C; D1], y = [c; d]       conblocks.jl:365-401
  ConstraintBlocks sizing (n1, p, n2, w per knot)                   conblocks.jl:403-425
  InvertedQuadratic / BlockCholesky (dense, block-diag, diagonal)   block_cholesky.jl:19-159
  _solve!(solver): Schur → block Cholesky → fwd/bwd → primals      cholesky_solver.jl:166-182
  second_order_correction! (Ginv = false)                           cholesky_solver.jl:254-273

`KktProblem` holds one batch in the ABI's packed per-trajectory layout (every knot block
column-major, concatenated over knots, batch slowest).  Compute goes through liblqrx.so
(lqrx_kkt_solve / lqrx_kkt_solve_host); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib

__all__ = ["KktStructure", "KktProblem", "ConstraintBlocks", "dubins_structure",
           "double_integrator_structure", "random_kkt", "kkt_solve", "kkt_solve_device", "workspace_size",
           "second_order_correction", "SparseSolver"]

H_DENSE, H_BLOCKDIAG, H_DIAG = 0, 1, 2


@dataclass
class KktStructure:
    """Per-knot block sizes shared by the batch (ConstraintBlocks, conblocks.jl:403-425)."""

    n: int
    m: int
    N: int
    n1: np.ndarray
    p: np.ndarray
    n2: np.ndarray
    w: np.ndarray

    @property
    def rows(self):
        return self.n1 + self.p + self.n2

    def sizes(self, h_mode):
        sY = int(np.sum(self.rows * self.w))
        sy = int(np.sum(self.p + self.n2))
        sH = int(np.sum(self.w)) if h_mode == H_DIAG else int(np.sum(self.w * self.w))
        sg = int(np.sum(self.w))
        return sY, sy, sH, sg

    def desc(self, batch, h_mode, ginv, layout=0, dtype=None):
        arrs = [np.ascontiguousarray(a, dtype=np.int32) for a in (self.n1, self.p, self.n2, self.w)]
        ptr = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))
        dtype = _lib.F64 if dtype is None else dtype
        d = _lib.KktDesc(self.N, dtype, batch, *[ptr(a) for a in arrs], h_mode, ginv, layout, 0)
        d._keep = arrs  # keep the arrays alive with the descriptor
        return d


def ConstraintBlocks(n, m, N, stage_p):
    """conblocks.jl:403-425 for a problem whose constraints are the dynamics on 1:N-1 plus
    stage constraints with stage_p[k] rows at knot k (0-based): n1 = n̄ if dynamics at k−1,
    n2 = n̄ if dynamics at k, w = n̄ + m·(k < N−1)."""
    p = np.broadcast_to(np.asarray(stage_p, dtype=np.int32), (N,)).copy()
    n1 = np.array([0] + [n] * (N - 1), np.int32)
    n2 = np.array([n] * (N - 1) + [0], np.int32)
    w = np.array([n + m] * (N - 1) + [n], np.int32)
    return KktStructure(n, m, N, n1, p, n2, w)


def trajectory_structure(n, m, N):
    """Initial-state constraint at knot 1, dynamics, goal at knot N (the SQP problems of
    test/dubins_sqp.jl and test/problems.jl Cartpole()) — block 1 (0,n,n), blocks 2..N-1
    (n,0,n), block N (n,n,0)."""
    return ConstraintBlocks(n, m, N, [n] + [0] * (N - 2) + [n])


def dubins_structure(N=101):
    """Dubins car n=3, m=2 (BASELINE cfg3)."""
    return trajectory_structure(3, 2, N)


def double_integrator_structure(D=3, N=101):
    """test/problems.jl DoubleIntegrator(D, N): n = 2D, m = D; initial condition (n rows) at
    knot 1, a planar LinearConstraint (max(D−2,1) rows) on 2:N−1, goal (n rows) at N."""
    n = 2 * D
    p = max(D - 2, 1)
    return ConstraintBlocks(n, D, N, [n] + [p] * (N - 2) + [n])


@dataclass
class KktProblem:
    st: KktStructure
    batch: int
    h_mode: int
    Y: np.ndarray
    y: np.ndarray
    H: np.ndarray
    g: np.ndarray


def random_kkt(st: KktStructure, batch: int, seed: int, h_mode: int = H_DIAG, dyn: str = "small") -> KktProblem:
    """Synthetic KKT data with the reference's Jacobian structure: D1_k = [A_k B_k],
    D2_{k+1} = [−I 0] (dynamics x_{k+1} = f(x_k, u_k)), stage rows C random (the initial
    condition / goal rows are [I 0]); H_k SPD (diagonal, block-diagonal or dense).
    dyn "small": A = I + 0.1·G, B = 0.1·G (the small shapes); "dense": the SURVEY §8(d)
    random-dense scaling A = I + (0.1/√n)·G, B = G/√n, which keeps large n (cfg5's 64)
    well conditioned."""
    rng = np.random.default_rng(seed)
    n, m, N = st.n, st.m, st.N
    sY, sy, sH, sg = st.sizes(h_mode)
    Y = np.zeros((batch, sY))
    y = np.zeros((batch, sy))
    H = np.zeros((batch, sH))
    g = rng.standard_normal((batch, sg))
    oY = oy = oH = 0
    for k in range(N):
        n1, p, n2, w = int(st.n1[k]), int(st.p[k]), int(st.n2[k]), int(st.w[k])
        rows = n1 + p + n2
        blk = np.zeros((batch, rows, w))
        if n1:
            blk[:, :n1, :n] = -np.eye(n)
        if p:
            if k == 0 or k == N - 1:
                blk[:, n1:n1 + p, :n] = np.eye(n)[:p] if p <= n else 0
                if p > n:
                    blk[:, n1:n1 + p, :] = rng.standard_normal((batch, p, w))
            else:
                blk[:, n1:n1 + p, :] = rng.standard_normal((batch, p, w))
        if n2:
            if dyn == "dense":
                A = np.eye(n) + (0.1 / np.sqrt(n)) * rng.standard_normal((batch, n, n))
                B = rng.standard_normal((batch, n, m)) / np.sqrt(n)
            else:
                A = np.eye(n) + 0.1 * rng.standard_normal((batch, n, n))
                B = 0.1 * rng.standard_normal((batch, n, m))
            blk[:, n1 + p:, :n] = A
            blk[:, n1 + p:, n:n + m] = B
        Y[:, oY:oY + rows * w] = np.swapaxes(blk, 1, 2).reshape(batch, -1)
        y[:, oy:oy + p + n2] = 0.1 * rng.standard_normal((batch, p + n2))
        if h_mode == H_DIAG:
            H[:, oH:oH + w] = 0.1 + rng.random((batch, w))
            oH += w
        else:
            M = rng.standard_normal((batch, w, w)) * 0.3
            Hk = np.einsum("bij,bkj->bik", M, M) + np.eye(w)
            if h_mode == H_BLOCKDIAG and w > n:
                Hk[:, :n, n:] = 0.0
                Hk[:, n:, :n] = 0.0
            H[:, oH:oH + w * w] = np.swapaxes(Hk, 1, 2).reshape(batch, -1)
            oH += w * w
        oY += rows * w
        oy += p + n2
    return KktProblem(st, batch, h_mode, Y, y, H, g)


def random_kkt_device(st: KktStructure, batch: int, seed: int, device, dtype=None):
    """random_kkt(…, h_mode=H_DIAG, dyn="dense") generated directly in HBM (torch, per knot),
    for batches whose Y does not fit host memory (BASELINE configs[4]: n=64 m=32 N=512
    B=8192 fp32 is 206 GB of Y).  Same block structure and distributions; a different
    random stream than the host generator.  Returns dict Y, y, H, g (flat), batch."""
    import torch

    dtype = dtype or torch.float64
    gen = torch.Generator(device=device)
    gen.manual_seed(int(seed))
    n, m, N = st.n, st.m, st.N
    sY, sy, sH, sg = st.sizes(H_DIAG)
    Y = torch.zeros(batch, sY, dtype=dtype, device=device)
    eye = torch.eye(n, dtype=dtype, device=device)
    oY = 0
    for k in range(N):
        n1, p, n2, w = int(st.n1[k]), int(st.p[k]), int(st.n2[k]), int(st.w[k])
        rows = n1 + p + n2
        blk = Y[:, oY:oY + rows * w].view(batch, w, rows)        # [b][column][row]: column-major block
        if n1:
            blk[:, :n, :n1] = -eye[:, :n1]
        if p:
            if k == 0 or k == N - 1:
                if p <= n:
                    blk[:, :n, n1:n1 + p] = eye[:, :p]
                else:
                    blk[:, :, n1:n1 + p] = torch.randn(batch, w, p, generator=gen, dtype=dtype, device=device)
            else:
                blk[:, :, n1:n1 + p] = torch.randn(batch, w, p, generator=gen, dtype=dtype, device=device)
        if n2:
            A = torch.randn(batch, n, n2, generator=gen, dtype=dtype, device=device) * (0.1 / np.sqrt(n))
            A += eye[:, :n2]
            blk[:, :n, n1 + p:] = A                               # column j of A_kᵀ… rows of D1 = [A B]
            blk[:, n:n + m, n1 + p:] = torch.randn(batch, m, n2, generator=gen, dtype=dtype,
                                                   device=device) / np.sqrt(n)
        oY += rows * w
    y = 0.1 * torch.randn(batch, sy, generator=gen, dtype=dtype, device=device)
    H = 0.1 + torch.rand(batch, sH, generator=gen, dtype=dtype, device=device)
    g = torch.randn(batch, sg, generator=gen, dtype=dtype, device=device)
    return dict(Y=Y.view(-1), y=y.view(-1), H=H.view(-1), g=g.view(-1), batch=batch)


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def kkt_solve(pb: KktProblem, ginv: int = 1, layout: int = 0, dtype: int | None = None,
              devices=None):
    """Batched _solve! via lqrx_kkt_solve_host.  Returns dict dz (batch, NN), lam
    (batch, P), info (batch,), rc.  layout=1 hands the library batch-fastest (SoA) copies
    ([element][batch]) and transposes the outputs back — same results.  dtype=F32 rounds the
    inputs to float32 and runs the fp32 (large-block) kernels; outputs come back as float32.
    devices = [d0, d1, …] shards the batch over those GPUs in one call
    (lqrx_kkt_solve_host_devices; repeats allowed)."""
    lib = _lib.load()
    st, bt = pb.st, pb.batch
    sY, sy, sH, sg = st.sizes(pb.h_mode)
    dtype = _lib.F64 if dtype is None else dtype
    npdt = np.float32 if dtype == _lib.F32 else np.float64
    d = st.desc(bt, pb.h_mode, ginv, layout, dtype)
    f = (lambda a: np.ascontiguousarray(np.asarray(a, dtype=npdt).T)) if layout == 1 else \
        (lambda a: np.ascontiguousarray(a, dtype=npdt))
    Y, y, H, g = f(pb.Y), f(pb.y), f(pb.H), f(pb.g)
    dz = np.zeros((sg, bt) if layout == 1 else (bt, sg), npdt)
    lam = np.zeros((sy, bt) if layout == 1 else (bt, sy), npdt)
    info = np.zeros(bt, np.int32)
    args = (C.byref(d), _ptr(Y), _ptr(y), _ptr(H), _ptr(g), _ptr(dz), _ptr(lam), _ptr(info))
    if devices is None:
        rc = _lib.check(lib.lqrx_kkt_solve_host(*args))
    else:
        dv = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
        rc = _lib.check(lib.lqrx_kkt_solve_host_devices(*args, dv.ctypes.data_as(C.c_void_p),
                                                        C.c_int32(len(dv))))
    if layout == 1:
        dz, lam = np.ascontiguousarray(dz.T), np.ascontiguousarray(lam.T)
    return dict(dz=dz, lam=lam, info=info, rc=rc)


def second_order_correction(pb: KktProblem):
    """second_order_correction! (cholesky_solver.jl:254-273): δẑ = −Dᵀ(DDᵀ)⁻¹d."""
    return kkt_solve(pb, ginv=0)


def workspace_size(st: KktStructure, batch: int, h_mode: int, ginv: int = 1, layout: int = 0,
                   dtype: int | None = None) -> int:
    """Bytes of device workspace lqrx_kkt_solve_ws needs (lqrx_kkt_workspace_size)."""
    lib = _lib.load()
    n = C.c_size_t(0)
    _lib.check(lib.lqrx_kkt_workspace_size(C.byref(st.desc(batch, h_mode, ginv, layout, dtype)), C.byref(n)))
    return n.value


def kkt_solve_device(st: KktStructure, t: dict, h_mode: int, ginv: int = 1,
                     stream: int | None = None, out: dict | None = None, workspace=None,
                     layout: int = 0) -> dict:
    """Device-pointer entry on torch tensors (flat, ABI layout `layout`): t has Y, y, H, g,
    batch; float32 tensors select dtype F32.  `workspace` (a device uint8 tensor of >=
    workspace_size() bytes) selects lqrx_kkt_solve_ws: no allocation inside the call."""
    import torch

    lib = _lib.load()
    bt = t["batch"]
    sY, sy, sH, sg = st.sizes(h_mode)
    dev = t["Y"].device
    tdt = t["Y"].dtype
    if any(t[k].dtype != tdt for k in ("y", "H", "g")):
        raise ValueError("Y, y, H, g must share one dtype")
    dtype = _lib.F32 if tdt == torch.float32 else _lib.F64
    if out is None:
        out = dict(dz=torch.empty(bt * sg, dtype=tdt, device=dev),
                   lam=torch.empty(bt * sy, dtype=tdt, device=dev),
                   info=torch.empty(bt, dtype=torch.int32, device=dev))
    d = st.desc(bt, h_mode, ginv, layout, dtype)
    p = lambda x: C.c_void_p(x.data_ptr())
    args = [C.byref(d), p(t["Y"]), p(t["y"]), p(t["H"]), p(t["g"]), p(out["dz"]), p(out["lam"]),
            p(out["info"])]
    sp = C.c_void_p(stream) if stream else None
    if workspace is None:
        rc = lib.lqrx_kkt_solve(*args, sp)
    else:
        rc = lib.lqrx_kkt_solve_ws(*args, p(workspace), workspace.numel() * workspace.element_size(), sp)
    _lib.check(rc)
    out["rc"] = rc
    return out


# ------------------------------------------------------------------ sparse formulation
class SparseSolver:
    """The SparseSolver formulation (/root/reference/src/sparse_solver.jl:120-246): one
    global sparse constraint Jacobian D (P×NN, SparseConstraintSet :17-43), violation d,
    block-diagonal cost Hessian G and gradient g over z = [x_1; u_1; …; x_N].  Its
    `_solve!` (:267-292: HD = G⁻¹Dᵀ, S = D·HD, λ = S⁻¹(d − D G⁻¹g), δZ = −HD·λ − G⁻¹g) is
    the same KKT system the block solver factors, so the device path gathers the per-knot
    blocks — Dblocks[k] = D[off_k + (1:rows_k), zinds[k]] (:156-160), G's diagonal blocks
    (Gblocks, :164) — into the packed layout and runs lqrx_kkt_solve.  Batched: D, d, G, g
    are lists (one per trajectory) sharing `st`'s structure."""

    def __init__(self, st: KktStructure, h_mode: int = H_DENSE):
        self.st, self.h_mode = st, h_mode

    def blocks(self, D, d, G, g) -> KktProblem:
        """Global (D, d, G, g) of each trajectory → packed Y, y, H, g (batch axis first)."""
        st, h_mode = self.st, self.h_mode
        Ds, ds, Gs, gs = (x if isinstance(x, (list, tuple)) else [x] for x in (D, d, G, g))
        bt = len(Ds)
        sY, sy, sH, sg = st.sizes(h_mode)
        Y = np.zeros((bt, sY)); y = np.zeros((bt, sy)); H = np.zeros((bt, sH)); gg = np.zeros((bt, sg))
        for b in range(bt):
            Db = Ds[b].tocsr() if hasattr(Ds[b], "tocsr") else np.asarray(Ds[b])
            Gb = Gs[b].tocsr() if hasattr(Gs[b], "tocsr") else np.asarray(Gs[b])
            dense = lambda M, r0, r1, c0, c1: (M[r0:r1, c0:c1].toarray() if hasattr(M, "toarray")
                                               else np.asarray(M[r0:r1, c0:c1]))
            oY = oy = oH = 0
            off1 = off2 = 0
            for k in range(st.N):
                n1, p, n2, w = int(st.n1[k]), int(st.p[k]), int(st.n2[k]), int(st.w[k])
                rows = n1 + p + n2
                Y[b, oY:oY + rows * w] = dense(Db, off1, off1 + rows, off2, off2 + w).T.reshape(-1)
                y[b, oy:oy + p + n2] = np.asarray(ds[b])[off1 + n1:off1 + rows]
                Gk = dense(Gb, off2, off2 + w, off2, off2 + w)
                if h_mode == H_DIAG:
                    H[b, oH:oH + w] = np.diag(Gk)
                    oH += w
                else:
                    H[b, oH:oH + w * w] = Gk.T.reshape(-1)
                    oH += w * w
                gg[b, off2:off2 + w] = np.asarray(gs[b])[off2:off2 + w]
                oY += rows * w
                oy += p + n2
                off1 += n1 + p
                off2 += w
        return KktProblem(st, bt, h_mode, Y, y, H, gg)

    def solve(self, D, d, G, g) -> dict:
        """_solve!(::SparseSolver) (sparse_solver.jl:267-292) on the device: δZ, λ."""
        return kkt_solve(self.blocks(D, d, G, g), ginv=1)

    def second_order_correction(self, D, d) -> dict:
        """second_order_correction!(::SparseSolver) (sparse_solver.jl:385-401):
        δx̂ = −Dᵀ(DDᵀ)⁻¹d — the block solver's Ginv = false variant."""
        st = self.st
        NN = int(np.sum(st.w))
        Ds = D if isinstance(D, (list, tuple)) else [D]
        eye = [np.eye(NN)] * len(Ds)
        zero = [np.zeros(NN)] * len(Ds)
        return kkt_solve(self.blocks(D, d, eye, zero), ginv=0)
