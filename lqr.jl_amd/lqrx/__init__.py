"""lqrx — MI355X-native batched LQR / block-tridiagonal-KKT solver.

Drop-in for the hot path of bjack205/LQR.jl: the Riccati pass (dynamic_programming.jl)
and the block-tridiagonal KKT Cholesky (block_cholesky.jl, jacobian_blocks.jl,
cholesky_solve.jl, cholesky_solver.jl, conblocks.jl).  Compute runs in liblqrx.so
(hand-written HIP for gfx950, C ABI in include/lqrx.h); this package is the host mirror of
the reference's Julia surface.
"""
from . import _lib
from ._lib import F32, F64, LqrxError, load
from .dp import (DPSolver, LQRBatch, LQRProblem, LQRSolution, compute_ctg, compute_gain,
                 dp_solve_device, random_batch, solve, solve_batch)
from .ls import LeastSquaresSolver, Primals

__all__ = ["F32", "F64", "LqrxError", "load", "DPSolver", "LQRBatch", "LQRProblem",
           "LQRSolution", "solve", "solve_batch", "random_batch", "dp_solve_device",
           "compute_gain", "compute_ctg",
           "LeastSquaresSolver", "Primals"]
