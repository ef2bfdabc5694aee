// lqrx_layout.hip — batch-layout conversion for the ABI's layout 1 (batch fastest, SoA).
//
// The n ≤ 4 DP kernels read and write layout 1 natively (lqrx_dp_lane.hip: one lane per
// trajectory, so the SoA element e of 64 consecutive trajectories is one coalesced load).
// The MFMA kernel (n ≥ 5) works on one trajectory per wave and wants each trajectory's
// blocks contiguous; for it lqrx_dp_solve converts the SoA inputs to layout 0 in
// stream-ordered scratch, solves, and converts the outputs back.  Both conversions are one
// batched transpose: an SoA array is a row-major [S][batch] matrix, its layout-0 form the
// row-major [batch][S] matrix.  HBM-bound: 64×64 tiles through LDS (row padded by one
// element, no bank conflicts), reads and writes coalesced along 64-element rows.
#include "lqrx_internal.h"

namespace lqrx {

namespace {

constexpr int TT = 64;        // tile edge
constexpr int TROWS = 4;      // 256 threads = 64 columns × 4 rows per pass

// out[c·rows + r] = in[r·cols + c] for the rows × cols row-major matrix `in`
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T *__restrict__ in, T *__restrict__ out, int64_t rows,
                                                        int64_t cols, int64_t tiles_c)
{
    __shared__ T tile[TT][TT + 1];
    const int64_t t = blockIdx.x;
    const int64_t r0 = (t / tiles_c) * TT, c0 = (t % tiles_c) * TT;
    const int tx = threadIdx.x & (TT - 1), ty = threadIdx.x >> 6;
    for (int i = ty; i < TT; i += TROWS) {
        const int64_t r = r0 + i, c = c0 + tx;
        if (r < rows && c < cols) tile[i][tx] = in[r * cols + c];
    }
    __syncthreads();
    for (int i = ty; i < TT; i += TROWS) {
        const int64_t c = c0 + i, r = r0 + tx;     // out row c, column r
        if (r < rows && c < cols) out[c * rows + r] = tile[tx][i];
    }
}

} // namespace

hipError_t batch_transpose(const void *in, void *out, int64_t rows, int64_t cols, int elem_bytes, hipStream_t s)
{
    if (rows <= 0 || cols <= 0) return hipSuccess;
    const int64_t tr = (rows + TT - 1) / TT, tc = (cols + TT - 1) / TT;
    if (tr * tc > 0xffffffffLL) return hipErrorInvalidValue;
    dim3 grid((unsigned)(tr * tc)), block(TT * TROWS);
    if (elem_bytes == 8)
        hipLaunchKernelGGL(transpose_kernel<double>, grid, block, 0, s, (const double *)in, (double *)out, rows, cols, tc);
    else
        hipLaunchKernelGGL(transpose_kernel<float>, grid, block, 0, s, (const float *)in, (float *)out, rows, cols, tc);
    return hipGetLastError();
}

} // namespace lqrx
