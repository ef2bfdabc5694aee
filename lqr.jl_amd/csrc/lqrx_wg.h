// lqrx_wg.h — workgroup-per-trajectory dense building blocks for the shapes past the register
// tiles (lqrx_dp_big.hip, lqrx_kkt_wg.hip): one 256-thread workgroup owns one trajectory and
// its matrices live in a per-trajectory global scratch block (an L2-resident working set).
//
//   wg_mm      C = Cin ± M1ᵀ·Y1 ± M2ᵀ·Y2 on 16×16 MFMA tiles (strided operand views)
//   wg_potrf   upper Cholesky (LAPACK potrf 'U'), left-looking by 16-row blocks: the update
//              of a block row by the rows above it is one wg_mm, the block row itself is
//              factored unblocked with every thread owning columns
//   wg_trsm_ut X ← U⁻ᵀ·X    (trsm 'L','U','T','N': forward substitution by 16-row blocks)
//   wg_trsm_un X ← U⁻¹·X    (trsm 'L','U','N','N': backward substitution by 16-row blocks)
// The triangular kernels put the block updates on the MFMA pipe and solve the 16×16 diagonal
// triangles column-parallel with the 16 unknowns of a column in registers.  Every routine is
// entered and left by all threads of the workgroup (it synchronises internally and on exit).
#pragma once
#include "lqrx_tile.h"

namespace lqrx {
namespace wg {

constexpr int BT = 256;

// One 16×16 MFMA C-layout tile of a matrix with general strides: element (row, col) at
// src[row·rs + col·cs] (column-major: rs = 1, cs = ld; its transpose: rs = ld, cs = 1);
// zero outside rows × cols.
template <typename T>
__device__ __forceinline__ void tile_ld(typename Tile<T>::acc &t, const T *src, int rows, int cols, size_t rs,
                                        size_t cs, int lane)
{
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = Tile<T>::row(lane, r), col = tcol(lane);
        const bool ok = row < rows && col < cols;
        t[r] = ok ? src[(size_t)row * rs + (size_t)col * cs] : (T)0;
    }
}

// Strided operand view: element (i, j) at p[i·rs + j·cs]
template <typename T> struct Mat {
    const T *p;
    size_t rs, cs;
    __device__ const T *at(int i, int j) const { return p + (size_t)i * rs + (size_t)j * cs; }
};
// column-major r × c matrix with leading dimension ld, and its transpose
template <typename T> __device__ __forceinline__ Mat<T> cm(const T *p, int ld) { return Mat<T>{p, 1, (size_t)ld}; }
template <typename T> __device__ __forceinline__ Mat<T> cmt(const T *p, int ld) { return Mat<T>{p, (size_t)ld, 1}; }

// Workgroup product on the MFMA pipe: C (r×c, column-major, ldc) = [Cin] + S1·M1ᵀ·Y1 + S2·M2ᵀ·Y2
// (S1, S2 ∈ {+1, −1}), M1 kk1×r, Y1 kk1×c (M2 kk2×r, Y2 kk2×c; kk = 0 drops a product).  The 4
// waves take the 16×16 output tiles round-robin and stream the k-tiles of their operands from
// L2.  Cin may alias C (each tile is read, then written, by the wave that owns it).
template <typename T, int S1, int S2>
__device__ __forceinline__ void wg_mm(T *C, int ldc, int r, int c, const T *Cin, Mat<T> M1, Mat<T> Y1, int kk1,
                                      Mat<T> M2, Mat<T> Y2, int kk2, int tid)
{
    using acc = typename Tile<T>::acc;
    const int wave = tid >> 6, lane = tid & 63;
    const int RT = (r + 15) / 16, CT = (c + 15) / 16;
    for (int ot = wave; ot < RT * CT; ot += BT / 64) {
        const int it = ot % RT, jt = ot / RT;
        acc D;
        if (Cin) tile_ld<T>(D, Cin + it * 16 + (size_t)jt * 16 * ldc, r - it * 16, c - jt * 16, 1, ldc, lane);
        else D = acc{0, 0, 0, 0};
        for (int kt = 0; kt < (kk1 + 15) / 16; ++kt) {
            acc Mt, Yt;
            tile_ld<T>(Mt, M1.at(kt * 16, it * 16), kk1 - kt * 16, r - it * 16, M1.rs, M1.cs, lane);
            tile_ld<T>(Yt, Y1.at(kt * 16, jt * 16), kk1 - kt * 16, c - jt * 16, Y1.rs, Y1.cs, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) D = S1 > 0 ? Tile<T>::mma(Mt[q], Yt[q], D) : Tile<T>::mma_nega(Mt[q], Yt[q], D);
        }
        for (int kt = 0; kt < (kk2 + 15) / 16; ++kt) {
            acc Mt, Yt;
            tile_ld<T>(Mt, M2.at(kt * 16, it * 16), kk2 - kt * 16, r - it * 16, M2.rs, M2.cs, lane);
            tile_ld<T>(Yt, Y2.at(kt * 16, jt * 16), kk2 - kt * 16, c - jt * 16, Y2.rs, Y2.cs, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) D = S2 > 0 ? Tile<T>::mma(Mt[q], Yt[q], D) : Tile<T>::mma_nega(Mt[q], Yt[q], D);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = it * 16 + Tile<T>::row(lane, q), col = jt * 16 + tcol(lane);
            if (row < r && col < c) C[row + (size_t)col * ldc] = D[q];
        }
    }
}
// one product: C = [Cin] + S·M1ᵀ·Y1
template <typename T, int S>
__device__ __forceinline__ void wg_mm1(T *C, int ldc, int r, int c, const T *Cin, Mat<T> M1, Mat<T> Y1, int kk1,
                                       int tid)
{
    wg_mm<T, S, 1>(C, ldc, r, c, Cin, M1, Y1, kk1, M1, Y1, 0, tid);
}

template <typename T> __device__ __forceinline__ T wsqrt(T x) { return sqrt(x); }

// A ← U with A = UᵀU (p×p, column-major, ld; only the upper triangle is read or written).
// Returns 0, or j+1 for the first pivot j that is not positive (LAPACK's info; the factor
// stops there, as dpotrf does).  The return value is uniform over the workgroup.
template <typename T> __device__ int wg_potrf(T *A, int ld, int p, int tid)
{
    for (int jb = 0; jb < p; jb += 16) {
        const int nb = min(16, p - jb);
        if (jb) {   // block row jb: A[jb:jb+nb, jb:p] −= U[0:jb, jb:jb+nb]ᵀ · U[0:jb, jb:p]
            T *blk = A + jb + (size_t)jb * ld;
            wg_mm1<T, -1>(blk, ld, nb, p - jb, blk, cm(A + (size_t)jb * ld, ld), cm(A + (size_t)jb * ld, ld), jb, tid);
            __syncthreads();
        }
        for (int j = jb; j < jb + nb; ++j) {
            T dj = A[j + (size_t)j * ld];
            for (int q = jb; q < j; ++q) dj -= A[q + (size_t)j * ld] * A[q + (size_t)j * ld];
            if (!(dj > (T)0)) {                                 // uniform: every thread saw the same dj
                __syncthreads();
                return j + 1;
            }
            dj = wsqrt(dj);
            for (int c = j + 1 + tid; c < p; c += BT) {
                T s = A[j + (size_t)c * ld];
                for (int q = jb; q < j; ++q) s -= A[q + (size_t)j * ld] * A[q + (size_t)c * ld];
                A[j + (size_t)c * ld] = s / dj;
            }
            __syncthreads();
            if (tid == 0) A[j + (size_t)j * ld] = dj;
            __syncthreads();
        }
    }
    return 0;
}

// X ← U⁻ᵀ·X : U p×p upper (ldu), X p×c (ldx).  Forward substitution by 16-row blocks.
template <typename T> __device__ void wg_trsm_ut(const T *U, int ldu, int p, T *X, int ldx, int c, int tid)
{
    for (int ib = 0; ib < p; ib += 16) {
        const int nb = min(16, p - ib);
        if (ib) {   // X[ib:ib+nb, :] −= U[0:ib, ib:ib+nb]ᵀ · X[0:ib, :]
            wg_mm1<T, -1>(X + ib, ldx, nb, c, X + ib, cm(U + (size_t)ib * ldu, ldu), cm<T>(X, ldx), ib, tid);
            __syncthreads();
        }
        for (int col = tid; col < c; col += BT) {
            T *x = X + ib + (size_t)col * ldx;
            T v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (i < nb) {
                    const T *u = U + ib + (size_t)(ib + i) * ldu;   // column ib+i of U, from row ib
                    T s = x[i];
#pragma unroll
                    for (int q = 0; q < i; ++q) s -= u[q] * v[q];
                    v[i] = s / u[i];
                    x[i] = v[i];
                }
            }
        }
        __syncthreads();
    }
}

// X ← U⁻¹·X : U p×p upper (ldu), X p×c (ldx).  Backward substitution by 16-row blocks.
template <typename T> __device__ void wg_trsm_un(const T *U, int ldu, int p, T *X, int ldx, int c, int tid)
{
    for (int ib = ((p - 1) / 16) * 16; ib >= 0; ib -= 16) {
        const int nb = min(16, p - ib), tail = p - ib - nb;
        if (tail) { // X[ib:ib+nb, :] −= U[ib:ib+nb, ib+nb:p] · X[ib+nb:p, :]
            wg_mm1<T, -1>(X + ib, ldx, nb, c, X + ib, cmt(U + ib + (size_t)(ib + nb) * ldu, ldu),
                          cm<T>(X + ib + nb, ldx), tail, tid);
            __syncthreads();
        }
        for (int col = tid; col < c; col += BT) {
            T *x = X + ib + (size_t)col * ldx;
            T v[16];
#pragma unroll
            for (int i = 15; i >= 0; --i) {
                if (i < nb) {
                    T s = x[i];
#pragma unroll
                    for (int q = i + 1; q < 16; ++q)
                        if (q < nb) s -= U[ib + i + (size_t)(ib + q) * ldu] * v[q];
                    v[i] = s / U[ib + i + (size_t)(ib + i) * ldu];
                    x[i] = v[i];
                }
            }
        }
        __syncthreads();
    }
}

} // namespace wg
} // namespace lqrx
