// lqrx_tile.h — register-tile primitives for gfx950 (CDNA4) MFMA, fp64 and fp32.
//
// One 16×16 tile lives in the MFMA accumulator ("C") layout of v_mfma_{f64,f32}_16x16x4:
//   f64 (v_mfma_f64_16x16x4_f64): lane l, reg r holds element (row (l>>4) + 4r, col l&15)
//   f32 (v_mfma_f32_16x16x4_f32): lane l, reg r holds element (row 4(l>>4) + r, col l&15)
// The A/B operand maps of both instructions are A[i=l&15][k=l>>4], B[k=l>>4][j=l&15].
// Consequence used everywhere below: register r of a C-layout tile M is, lane for lane,
//   * a valid B operand for k-slice r (rows of M are the contraction index), and
//   * a valid A operand for k-slice r giving Mᵀ (M's rows again the contraction index),
// with the SAME global k for both (k = kk + 4r for f64, 4kk + r for f32).  So
//   D += Mᵀ·Y  for C-layout M and Y  is 4 MFMAs with no data movement at all.
// Every product in the Riccati step is written in that "TN" form (see lqrx_dp.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lqrx {

template <typename T> struct Tile;

template <> struct Tile<double> {
    using acc = double __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc mma(double a, double b, acc c)
    {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};

template <> struct Tile<float> {
    using acc = float __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc mma(float a, float b, acc c)
    {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};

__device__ __forceinline__ int tcol(int lane) { return lane & 15; }

// wave-uniform broadcast of lane `src`'s value (v_readlane_b32; src must be a constant
// or wave-uniform value)
__device__ __forceinline__ double readlane(double v, int src)
{
    long long x = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), src);
    int hi = __builtin_amdgcn_readlane((int)(x >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float readlane(float v, int src)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}

// D[I][J] += Σ_k M[k][I]ᵀ Y[k][J]  over KT k-tiles; M is KT×I tiles, Y is KT×J tiles.
// Loop order (k-tile, k-slice outermost, output tiles innermost) keeps consecutive MFMAs
// on different accumulators wherever I·J > 1.
template <typename T, int KT, int I, int J>
__device__ __forceinline__ void mma_tn(typename Tile<T>::acc (&D)[I][J],
                                       const typename Tile<T>::acc (&M)[KT][I],
                                       const typename Tile<T>::acc (&Y)[KT][J])
{
#pragma unroll
    for (int k = 0; k < KT; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < I; ++i)
#pragma unroll
                for (int j = 0; j < J; ++j) D[i][j] = Tile<T>::mma(M[k][i][r], Y[k][j][r], D[i][j]);
}

template <typename T, int I, int J>
__device__ __forceinline__ void tiles_zero(typename Tile<T>::acc (&D)[I][J])
{
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) D[i][j] = typename Tile<T>::acc{0, 0, 0, 0};
}

// Load a rows×cols column-major matrix (leading dim ld) into C-layout tiles, zero padded.
// If diag_pad, padded diagonal entries are 1 (keeps a padded SPD block SPD).
template <typename T, int I, int J>
__device__ __forceinline__ void tiles_load(typename Tile<T>::acc (&D)[I][J], const T *__restrict__ src,
                                           int rows, int cols, int ld, int lane, bool diag_pad)
{
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int row = i * 16 + Tile<T>::row(lane, r), col = j * 16 + tcol(lane);
                T v = (T)0;
                if (row < rows && col < cols) v = src[(size_t)row + (size_t)col * ld];
                else if (diag_pad && row == col) v = (T)1;
                D[i][j][r] = v;
            }
}

template <typename T, int I, int J>
__device__ __forceinline__ void tiles_store(const typename Tile<T>::acc (&D)[I][J], T *__restrict__ dst,
                                            int rows, int cols, int ld, int lane)
{
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int row = i * 16 + Tile<T>::row(lane, r), col = j * 16 + tcol(lane);
                if (row < rows && col < cols) dst[(size_t)row + (size_t)col * ld] = D[i][j][r];
            }
}

// C-layout tiles → column-major LDS image (column stride cs), and back.
template <typename T, int I, int J>
__device__ __forceinline__ void tiles_to_lds(const typename Tile<T>::acc (&D)[I][J], T *lds, int cs,
                                             int lane)
{
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int row = i * 16 + Tile<T>::row(lane, r), col = j * 16 + tcol(lane);
                lds[row + col * cs] = D[i][j][r];
            }
}

template <typename T, int I, int J>
__device__ __forceinline__ void tiles_from_lds(typename Tile<T>::acc (&D)[I][J], const T *lds, int cs,
                                               int lane)
{
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int row = i * 16 + Tile<T>::row(lane, r), col = j * 16 + tcol(lane);
                D[i][j][r] = lds[row + col * cs];
            }
}

} // namespace lqrx
