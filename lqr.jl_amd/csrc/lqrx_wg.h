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

// D ±= Mᵀ·Y over kk contraction rows for output tile (it, jt): the operand tiles of k-step
// kt+1 are loaded before the MFMAs of step kt (their L2 latency overlaps the products)
template <typename T, int S>
__device__ __forceinline__ void wg_mm_k(typename Tile<T>::acc &D, Mat<T> M, Mat<T> Y, int kk, int r, int c, int it,
                                        int jt, int lane)
{
    using acc = typename Tile<T>::acc;
    const int nk = (kk + 15) / 16;
    if (nk == 0) return;
    acc Mt, Yt;
    tile_ld<T>(Mt, M.at(0, it * 16), kk, r - it * 16, M.rs, M.cs, lane);
    tile_ld<T>(Yt, Y.at(0, jt * 16), kk, c - jt * 16, Y.rs, Y.cs, lane);
    for (int kt = 0; kt < nk; ++kt) {
        acc Mn = Mt, Yn = Yt;
        if (kt + 1 < nk) {
            tile_ld<T>(Mn, M.at((kt + 1) * 16, it * 16), kk - (kt + 1) * 16, r - it * 16, M.rs, M.cs, lane);
            tile_ld<T>(Yn, Y.at((kt + 1) * 16, jt * 16), kk - (kt + 1) * 16, c - jt * 16, Y.rs, Y.cs, lane);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) D = S > 0 ? Tile<T>::mma(Mt[q], Yt[q], D) : Tile<T>::mma_nega(Mt[q], Yt[q], D);
        Mt = Mn;
        Yt = Yn;
    }
}

// D[a][b] ±= Mᵀ·Y for the 2×2 output tiles (it0 + a, jt0 + b): every k-step loads two M and two Y
// tiles and feeds four accumulators (half the operand loads of four single tiles); k-step kt+1's
// tiles are loaded before the MFMAs of step kt.  Tiles past the matrix read zeros.
template <typename T, int S>
__device__ __forceinline__ void wg_mm_k22(typename Tile<T>::acc (&D)[2][2], Mat<T> M, Mat<T> Y, int kk, int r, int c,
                                          int it0, int jt0, int lane)
{
    using acc = typename Tile<T>::acc;
    const int nk = (kk + 15) / 16;
    if (nk == 0) return;
    acc Mt[2], Yt[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        tile_ld<T>(Mt[a], M.at(0, (it0 + a) * 16), kk, r - (it0 + a) * 16, M.rs, M.cs, lane);
        tile_ld<T>(Yt[a], Y.at(0, (jt0 + a) * 16), kk, c - (jt0 + a) * 16, Y.rs, Y.cs, lane);
    }
    for (int kt = 0; kt < nk; ++kt) {
        acc Mn[2] = {Mt[0], Mt[1]}, Yn[2] = {Yt[0], Yt[1]};
        if (kt + 1 < nk) {
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                tile_ld<T>(Mn[a], M.at((kt + 1) * 16, (it0 + a) * 16), kk - (kt + 1) * 16, r - (it0 + a) * 16, M.rs,
                           M.cs, lane);
                tile_ld<T>(Yn[a], Y.at((kt + 1) * 16, (jt0 + a) * 16), kk - (kt + 1) * 16, c - (jt0 + a) * 16, Y.rs,
                           Y.cs, lane);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    D[a][b] = S > 0 ? Tile<T>::mma(Mt[a][q], Yt[b][q], D[a][b]) : Tile<T>::mma_nega(Mt[a][q], Yt[b][q], D[a][b]);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            Mt[a] = Mn[a];
            Yt[a] = Yn[a];
        }
    }
}

// Workgroup product on the MFMA pipe: C (r×c, column-major, ldc) = [Cin] + S1·M1ᵀ·Y1 + S2·M2ᵀ·Y2
// (S1, S2 ∈ {+1, −1}), M1 kk1×r, Y1 kk1×c (M2 kk2×r, Y2 kk2×c; kk = 0 drops a product).  The 4
// waves take the output tiles round-robin — 2×2 blocks of them (shared operand loads) when there
// are more than 8 tiles, single tiles otherwise (so a thin product still spreads over the waves)
// — and stream the k-tiles of their operands from L2.  UPPER: only the tiles on or above the
// diagonal (it ≤ jt) are computed and stored (a symmetric result whose consumers read the upper
// triangle).  Cin may alias C (each tile is read, then written, by the wave that owns it).
template <typename T, int S1, int S2>
__device__ __forceinline__ void wg_mm(T *C, int ldc, int r, int c, const T *Cin, Mat<T> M1, Mat<T> Y1, int kk1,
                                      Mat<T> M2, Mat<T> Y2, int kk2, int tid, bool upper = false)
{
    using acc = typename Tile<T>::acc;
    const int wave = tid >> 6, lane = tid & 63;
    const int RT = (r + 15) / 16, CT = (c + 15) / 16;
    auto store = [&](const acc &D, int it, int jt) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = it * 16 + Tile<T>::row(lane, q), col = jt * 16 + tcol(lane);
            if (row < r && col < c) C[row + (size_t)col * ldc] = D[q];
        }
    };
    auto init = [&](acc &D, int it, int jt) __attribute__((always_inline)) {
        if (Cin) tile_ld<T>(D, Cin + it * 16 + (size_t)jt * 16 * ldc, r - it * 16, c - jt * 16, 1, ldc, lane);
        else D = acc{0, 0, 0, 0};
    };
    if (RT * CT > 8) {
        const int RB = (RT + 1) / 2, CB = (CT + 1) / 2;
        for (int ob = wave; ob < RB * CB; ob += BT / 64) {
            const int it0 = 2 * (ob % RB), jt0 = 2 * (ob / RB);
            if (upper && it0 > jt0 + 1) continue;
            acc D[2][2];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) init(D[a][b], it0 + a, jt0 + b);
            wg_mm_k22<T, S1>(D, M1, Y1, kk1, r, c, it0, jt0, lane);
            wg_mm_k22<T, S2>(D, M2, Y2, kk2, r, c, it0, jt0, lane);
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    if (!upper || it0 + a <= jt0 + b) store(D[a][b], it0 + a, jt0 + b);
        }
        return;
    }
    for (int ot = wave; ot < RT * CT; ot += BT / 64) {
        const int it = ot % RT, jt = ot / RT;
        if (upper && it > jt) continue;
        acc D;
        init(D, it, jt);
        wg_mm_k<T, S1>(D, M1, Y1, kk1, r, c, it, jt, lane);
        wg_mm_k<T, S2>(D, M2, Y2, kk2, r, c, it, jt, lane);
        store(D, it, jt);
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
// Per 16-row block: the rows above are subtracted by one wg_mm, then the block row is factored
// with each thread holding its column's 16 entries in registers; the pivot column of each row
// is published in LDS (one barrier per row), columns past the first 256 follow without barriers.
template <typename T> __device__ int wg_potrf(T *A, int ld, int p, int tid)
{
    __shared__ T pcol[16 * 16];   // pcol[q + 16j] = U[jb+q][jb+j] (q < j), pcol[j + 16j] = U_jj
    for (int jb = 0; jb < p; jb += 16) {
        const int nb = min(16, p - jb);
        if (jb) {   // block row jb: A[jb:jb+nb, jb:p] −= U[0:jb, jb:jb+nb]ᵀ · U[0:jb, jb:p]
            T *blk = A + jb + (size_t)jb * ld;
            wg_mm1<T, -1>(blk, ld, nb, p - jb, blk, cm(A + (size_t)jb * ld, ld), cm(A + (size_t)jb * ld, ld), jb, tid);
        }
        __syncthreads();
        const int c0 = jb + tid;
        const bool own = c0 < p;
        T v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = (own && i < nb) ? A[jb + i + (size_t)c0 * ld] : (T)0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (j < nb) {
                if (tid == j) {                                 // owner of pivot column jb + j
                    T d = v[j];
#pragma unroll
                    for (int q = 0; q < j; ++q) d -= v[q] * v[q];
                    d = d > (T)0 ? wsqrt(d) : (T)0;             // 0 (or NaN) marks the failure
                    v[j] = d;
#pragma unroll
                    for (int q = 0; q < j; ++q) pcol[q + 16 * j] = v[q];
                    pcol[j + 16 * j] = d;
                }
                __syncthreads();
                const T dj = pcol[j + 16 * j];
                if (!(dj > (T)0)) return jb + j + 1;            // uniform: every thread read dj
                if (own && tid > j) {
                    T sv = v[j];
#pragma unroll
                    for (int q = 0; q < j; ++q) sv -= pcol[q + 16 * j] * v[q];
                    v[j] = sv / dj;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (own && i < nb) A[jb + i + (size_t)c0 * ld] = v[i];
        for (int c = c0 + BT; c < p; c += BT) {                 // columns past the first BT
            T u[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) u[i] = i < nb ? A[jb + i + (size_t)c * ld] : (T)0;
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (j < nb) {
                    T sv = u[j];
#pragma unroll
                    for (int q = 0; q < j; ++q) sv -= pcol[q + 16 * j] * u[q];
                    u[j] = sv / pcol[j + 16 * j];
                }
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (i < nb) A[jb + i + (size_t)c * ld] = u[i];
        }
        __syncthreads();
    }
    return 0;
}

// X ← U⁻ᵀ·X : U p×p upper (ldu), X p×c (ldx).  Forward substitution by 16-row blocks: the
// block update on MFMA, the block's 16×16 triangle staged in LDS, each column's 16 unknowns
// loaded up front into registers.
template <typename T> __device__ void wg_trsm_ut(const T *U, int ldu, int p, T *X, int ldx, int c, int tid)
{
    __shared__ T ub[16 * 16];     // ub[q + 16i] = U[ib+q][ib+i], q ≤ i
    for (int ib = 0; ib < p; ib += 16) {
        const int nb = min(16, p - ib);
        if (ib)     // X[ib:ib+nb, :] −= U[0:ib, ib:ib+nb]ᵀ · X[0:ib, :]
            wg_mm1<T, -1>(X + ib, ldx, nb, c, X + ib, cm(U + (size_t)ib * ldu, ldu), cm<T>(X, ldx), ib, tid);
        for (int e = tid; e < 256; e += BT) {
            const int q = e & 15, i = e >> 4;
            ub[e] = (q <= i && i < nb) ? U[ib + q + (size_t)(ib + i) * ldu] : (T)0;
        }
        __syncthreads();
        for (int col = tid; col < c; col += BT) {
            T *x = X + ib + (size_t)col * ldx;
            T v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = i < nb ? x[i] : (T)0;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (i < nb) {
                    T sv = v[i];
#pragma unroll
                    for (int q = 0; q < i; ++q) sv -= ub[q + 16 * i] * v[q];
                    v[i] = sv / ub[i + 16 * i];
                }
            }
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (i < nb) x[i] = v[i];
        }
        __syncthreads();
    }
}

// X ← U⁻¹·X : U p×p upper (ldu), X p×c (ldx).  Backward substitution by 16-row blocks.
template <typename T> __device__ void wg_trsm_un(const T *U, int ldu, int p, T *X, int ldx, int c, int tid)
{
    __shared__ T ub[16 * 16];     // ub[i + 16q] = U[ib+i][ib+q], i ≤ q
    for (int ib = ((p - 1) / 16) * 16; ib >= 0; ib -= 16) {
        const int nb = min(16, p - ib), tail = p - ib - nb;
        if (tail)   // X[ib:ib+nb, :] −= U[ib:ib+nb, ib+nb:p] · X[ib+nb:p, :]
            wg_mm1<T, -1>(X + ib, ldx, nb, c, X + ib, cmt(U + ib + (size_t)(ib + nb) * ldu, ldu),
                          cm<T>(X + ib + nb, ldx), tail, tid);
        for (int e = tid; e < 256; e += BT) {
            const int i = e & 15, q = e >> 4;
            ub[e] = (i <= q && q < nb) ? U[ib + i + (size_t)(ib + q) * ldu] : (T)0;
        }
        __syncthreads();
        for (int col = tid; col < c; col += BT) {
            T *x = X + ib + (size_t)col * ldx;
            T v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = i < nb ? x[i] : (T)0;
#pragma unroll
            for (int i = 15; i >= 0; --i) {
                if (i < nb) {
                    T sv = v[i];
#pragma unroll
                    for (int q = i + 1; q < 16; ++q)
                        if (q < nb) sv -= ub[i + 16 * q] * v[q];
                    v[i] = sv / ub[i + 16 * i];
                }
            }
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (i < nb) x[i] = v[i];
        }
        __syncthreads();
    }
}

} // namespace wg
} // namespace lqrx
