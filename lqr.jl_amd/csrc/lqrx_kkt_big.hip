// lqrx_kkt_big.hip — block-tridiagonal KKT solve for large blocks (any structure with every
// block dimension ≤ 64, padded Y rows ≤ 128, w ≤ 128), fp64 and fp32, on MFMA tiles.
//
// Reference: CholeskySolver._solve! (/root/reference/src/cholesky_solver.jl:166-182) =
//   calculate_shur_factors!  jacobian_blocks.jl:220-286   (shur! :231-242, copy_shur! :249-286)
//   cholesky!(chol, shur)    cholesky_solve.jl:47-67       (block upper Cholesky, LAPACK potrf/trsm)
//   forward_substitution!    cholesky_solve.jl:93-117
//   backward_substitution!   cholesky_solve.jl:119-143
//   calculate_primals!       cholesky_solver.jl:185-236
// with the diagonal BlockCholesky mode (block_cholesky.jl:82-91) and the SOC variant
// (Ginv = false, :254-273).  The reference handles any block size through LAPACK; the
// compile-time-shaped lane kernels (lqrx_kkt_fil.hip) stop at a few rows.
//
// Two kernels, one 256-thread workgroup (4 waves) per trajectory:
//
// kkt_big_fwd_kernel — the forward sweep.  At step k the workgroup
//   (1) forms the Schur pieces of knot k+1, YYt = Y H⁻¹ Yᵀ (upper 16×16 tiles only, on
//       v_mfma_{f32,f64}_16x16x4 with operands from a 16-column LDS slab of Y_{k+1} that the
//       256 threads stream in coalesced, one slab prefetched in registers ahead) and
//       r = Y H⁻¹ g; the A ≡ previous-C alias of copy_shur! (:166) is an add into C_k, the
//       `d .+= r_[1]` of :251 an add into d_k;
//   (2) factors knot k with explicit inverses of the diagonal factors, so every triangular
//       solve of the reference becomes an MFMA product:
//          D̃ = Ã⁻ᵀD, F̃ = Ã⁻ᵀF              (Ã⁻¹ = W_{k−1}, kept in LDS)       :49, :57
//          B̃ = chol(B − D̃ᵀD̃), Binv = B̃⁻¹                                     :50-53
//          Ẽ = B̃⁻ᵀ(E − D̃ᵀF̃)                                                  :59-60
//          C̃ = chol(C − F̃ᵀF̃ − ẼᵀẼ), W_k = C̃⁻¹                                 :61-62
//       chol+inverse is blocked by 16: a 16×16 leaf (potrf + triangular inverse in one
//       wave's registers, the pivot test → info), panel and trailing updates on MFMA, the
//       off-diagonal inverse blocks assembled on MFMA;
//   (3) runs the forward substitution (:93-117) with the inverses, and stores Binv, Ẽ, W_k
//       (packed upper triangles) and the forward μ, λ in a per-trajectory slab;
//   (4) writes knot k+1's Schur tiles (held in registers across (2)-(3)) into LDS.
//
// kkt_big_bwd_kernel — backward substitution (:119-143) fused with primal recovery
//   (cholesky_solver.jl:185-236), k = N−1 … 0, Y_k staged in LDS (coalesced), GEMVs only:
//   the reference's D̃_{k+1}μ_{k+1} + F̃_{k+1}λ_{k+1} = W_kᵀ·(D2 H⁻¹ t), t = [C; D1]ᵀ[μ; λ]
//   of knot k+1 — the same t that knot k+1's residual needs (no F̃ in the slab, no matrix
//   recompute);  λ_k = W_k(λ_k + ·), μ_k = Binv(μ_k − Ẽλ_k), negated;
//   δz = −H⁻¹(D1ᵀλ_k + Cᵀμ_k + D2ᵀλ_{k−1} + g).
//
// Everything is padded to 16 per block (zero rows, identity on padded pivots) so tiles never
// straddle block boundaries; the arithmetic on padding adds exact zeros.
#include "lqrx_internal.h"
#include "lqrx_tile.h"
#include <type_traits>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>

namespace lqrx {
namespace {

// timing ablations (tools/tv_ablate.sh builds; results are wrong by design): bit 1 the 16×16
// leaf returns at once, 2 no Schur MFMAs, 4 no forward substitution, 8 no slab stores,
// 16 no chol_inv at all
#ifndef KB_ABL
#define KB_ABL 0
#endif

// KB_PROF builds (timing only): per-phase shader-clock cycles of the forward sweep summed
// into KbArgs::prof[wave][phase] (0 prefactor, 1 factor wave, 2 Schur waves, 3 step barrier,
// 4 hand-over)
#ifdef KB_PROF
#define KB_T0() int64_t kb_t0 = clock64()
#define KB_T(i)                                                                                             \
    do {                                                                                                    \
        const int64_t kb_t1 = clock64();                                                                    \
        kb_acc[i] += kb_t1 - kb_t0;                                                                         \
        kb_t0 = kb_t1;                                                                                      \
    } while (0)
#define KB_F0() int64_t kb_f0 = clock64()
#define KB_F(i)                                                                                             \
    do {                                                                                                    \
        const int64_t kb_f1 = clock64();                                                                    \
        kb_acc[i] += kb_f1 - kb_f0;                                                                         \
        kb_f0 = kb_f1;                                                                                      \
    } while (0)
#define KB_FLUSH()                                                                                          \
    do {                                                                                                    \
        if (lane == 0 && a.prof)                                                                            \
            for (int i_ = 0; i_ < 10; ++i_) atomicAdd((unsigned long long *)&a.prof[wave * 16 + i_], (unsigned long long)kb_acc[i_]); \
    } while (0)
#else
#define KB_T0()
#define KB_T(i)
#define KB_F0()
#define KB_F(i)
#define KB_FLUSH()
#endif

constexpr int KB_THREADS = 256;
constexpr int KB_PMAX = 64;    // n1, p, n2 per knot
constexpr int KB_RMAX = 128;   // padded rows P1 + Ps + P2
constexpr int KB_WMAX = 128;   // width
constexpr int KB_MAXT = 9;     // Schur tiles per wave: 36 upper tiles of an 8×8 grid / 4 waves
constexpr int KB_F1T = 8;      // factor-phase tiles per wave (D̃ + F̃: 2·16 tiles / 4 waves)
constexpr int KB_LDY = 144;
constexpr int KB_BPRE = KB_RMAX * KB_WMAX / 256;   // backward: Y_k elements per thread (≤ 64)
constexpr int KB_WPRE = 9;                         // backward: packed W elements per thread (≤ 2080/256)    // Y-slab column stride: ≥ 128 rows, ≡ 16 (mod 64) floats / (mod 32) doubles

__host__ __device__ __forceinline__ int r16(int x) { return (x + 15) & ~15; }

template <typename T> using acc_t = typename Tile<T>::acc;

__device__ __forceinline__ double rcp_full(double a) { return rcp_nr2(a); }
__device__ __forceinline__ float rcp_full(float a) { return rcp_nr(a); }

// per-knot block sizes (actual and padded) and packed-input offsets (meta table, lqrx_api.cpp)
struct Kn {
    int p1, ps, p2, w, rows;
    int P1, Ps, P2, R, nsl;
    int oY, oy, oH, og;
};
__device__ __forceinline__ Kn kn_load(const int32_t *__restrict__ meta, int k)
{
    const int32_t *m = meta + 8 * k;
    Kn q;
    q.p1 = m[0]; q.ps = m[1]; q.p2 = m[2]; q.w = m[3];
    q.oY = m[4]; q.oy = m[5]; q.oH = m[6]; q.og = m[7];
    q.rows = q.p1 + q.ps + q.p2;
    q.P1 = r16(q.p1); q.Ps = r16(q.ps); q.P2 = r16(q.p2);
    q.R = q.P1 + q.Ps + q.P2;
    q.nsl = (q.w + 15) >> 4;
    return q;
}

// slab of one knot: [W packed P2(P2+1)/2][Binv packed Ps(Ps+1)/2][Ẽ Ps×P2][μ Ps][λ P2]
__host__ __device__ __forceinline__ int64_t slab_size(int Ps, int P2)
{
    return (int64_t)P2 * (P2 + 1) / 2 + (int64_t)Ps * (Ps + 1) / 2 + (int64_t)Ps * P2 + Ps + P2;
}

// LDS offsets of knot k's Schur blocks (leading dimension LD): C, F, E, B, D in that order,
// present blocks only (host: kb_lds_layout takes the max over knots)
struct Bo {
    int C, F, E, B, D, end;
};
__host__ __device__ __forceinline__ Bo blk_off(int P1, int Ps, int P2, int LD)
{
    Bo o;
    int x = 0;
    o.C = x; x += P2 ? LD * P2 : 0;
    o.F = x; x += (P1 && P2) ? LD * P2 : 0;
    o.E = x; x += (Ps && P2) ? LD * P2 : 0;
    o.B = x; x += Ps ? LD * Ps : 0;
    o.D = x; x += (P1 && Ps) ? LD * Ps : 0;
    o.end = x;
    return o;
}

// ---------------------------------------------------------------- tile primitives (LDS)
// c (+/−)= op(A)·op(B) for one 16×16 output tile over K (multiple of 16) contraction indices.
// op(A)[i][k] = TA ? A[k + i·lda] : A[i + k·lda];  op(B)[k][j] = TB ? B[j + k·ldb] : B[k + j·ldb]
template <typename T, bool TA, bool TB, bool NEG>
__device__ __forceinline__ acc_t<T> tmm(acc_t<T> c, const T *A, int lda, const T *B, int ldb, int K, int lane)
{
    const int i = lane & 15, g = lane >> 4;
    const T *pa = TA ? A + g + i * lda : A + i + g * lda;
    const T *pb = TB ? B + i + g * ldb : B + g + i * ldb;
    const int sa = TA ? 4 : 4 * lda, sb = TB ? 4 * ldb : 4;
    for (int k0 = 0; k0 < K; k0 += 16) {
        T a[4], b[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            a[s] = pa[s * sa];
            b[s] = pb[s * sb];
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) c = NEG ? Tile<T>::mma_nega(a[s], b[s], c) : Tile<T>::mma(a[s], b[s], c);
        pa += 4 * sa;
        pb += 4 * sb;
    }
    return c;
}

// the same with a compile-time contraction length KT·16: every operand load is issued before
// the MFMAs (the compiler can also interleave independent calls)
template <typename T, bool TA, bool TB, bool NEG, int KT>
__device__ __forceinline__ acc_t<T> tmmk(acc_t<T> c, const T *A, int lda, const T *B, int ldb, int lane)
{
    const int i = lane & 15, g = lane >> 4;
    const T *pa = TA ? A + g + i * lda : A + i + g * lda;
    const T *pb = TB ? B + i + g * ldb : B + g + i * ldb;
    const int sa = TA ? 4 : 4 * lda, sb = TB ? 4 * ldb : 4;
    T a[4 * KT], b[4 * KT];
#pragma unroll
    for (int s = 0; s < 4 * KT; ++s) {
        a[s] = pa[s * sa];
        b[s] = pb[s * sb];
    }
#pragma unroll
    for (int s = 0; s < 4 * KT; ++s) c = NEG ? Tile<T>::mma_nega(a[s], b[s], c) : Tile<T>::mma(a[s], b[s], c);
    return c;
}
// runtime KT (1..4) → compile-time instance
template <typename T, bool TA, bool TB, bool NEG>
__device__ __forceinline__ acc_t<T> tmm4(acc_t<T> c, const T *A, int lda, const T *B, int ldb, int kt, int lane)
{
    switch (kt) {
    case 1: return tmmk<T, TA, TB, NEG, 1>(c, A, lda, B, ldb, lane);
    case 2: return tmmk<T, TA, TB, NEG, 2>(c, A, lda, B, ldb, lane);
    case 3: return tmmk<T, TA, TB, NEG, 3>(c, A, lda, B, ldb, lane);
    default: return tmmk<T, TA, TB, NEG, 4>(c, A, lda, B, ldb, lane);
    }
}

template <typename T>
__device__ __forceinline__ acc_t<T> tload(const T *X, int ld, int lane)
{
    acc_t<T> c;
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] = X[Tile<T>::row(lane, r) + (lane & 15) * ld];
    return c;
}
template <typename T>
__device__ __forceinline__ void tstore(T *X, int ld, acc_t<T> c, int lane)
{
#pragma unroll
    for (int r = 0; r < 4; ++r) X[Tile<T>::row(lane, r) + (lane & 15) * ld] = c[r];
}
template <typename T>
__device__ __forceinline__ void tadd(T *X, int ld, acc_t<T> c, int lane)
{
#pragma unroll
    for (int r = 0; r < 4; ++r) X[Tile<T>::row(lane, r) + (lane & 15) * ld] += c[r];
}
template <typename T> __device__ __forceinline__ acc_t<T> tzero() { return acc_t<T>{0, 0, 0, 0}; }

// c (+/−)= A·M with M a C-layout register tile used as the B operand (register r = k-slice
// r, k = Tile<T>::row(lane, r)) and A[i][k] read from LDS (column-major, ld).
template <typename T, bool NEG>
__device__ __forceinline__ acc_t<T> tmm_reg(acc_t<T> c, const T *A, int ld, acc_t<T> M, int lane)
{
    const int i = lane & 15;
    T a[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] = A[i + Tile<T>::row(lane, r) * ld];
#pragma unroll
    for (int r = 0; r < 4; ++r) c = NEG ? Tile<T>::mma_nega(a[r], M[r], c) : Tile<T>::mma(a[r], M[r], c);
    return c;
}

// ---------------------------------------------------------------- 16×16 leaf (one wave)
// In place: X (upper triangle of an SPD 16×16 block, column-major, ld) → T = U⁻¹ with
// UᵀU = X (upper, strictly-lower part zeroed).  Lane c (< 16) holds column c in registers;
// pivot i broadcasts row i of U by v_readlane (uniform lane and register indices).  q = the
// block's real pivots; pivots ≥ q are identity padding.  Returns 1 + the first pivot that is
// not positive (potrf's info), else 0.  Mirrors dpotf2 'U' (dynamic_programming.jl:29,
// cholesky_solve.jl:2) up to the rsqrt-multiply instead of sqrt-divide.
template <typename T>
__device__ __forceinline__ int leaf_chol_inv(T *X, int ld, int q, int lane)
{
    const int c = lane & 15;
    if (KB_ABL & 1) return 0;
    T col[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) col[r] = X[r + c * ld];
    int bad = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const T d = readlane(col[i], i);
        if (!(d > (T)0) && i < q && !bad) bad = i + 1;
        const T s = rsqrt_nr(d);
        col[i] = c >= i ? col[i] * s : (T)0;
#pragma unroll
        for (int r = i + 1; r < 16; ++r) col[r] = fma(-readlane(col[i], r), col[i], col[r]);
    }
    // T = U⁻¹, column c: for k = 15 … 0, T[k][c] = (δ_kc − Σ_{j>k} U[k][j] T[j][c]) / U[k][k]
    T t[16];
#pragma unroll
    for (int k = 15; k >= 0; --k) {
        T acc = c == k ? (T)1 : (T)0;
#pragma unroll
        for (int j = k + 1; j < 16; ++j) acc = fma(-readlane(col[k], j), t[j], acc);
        t[k] = acc * rcp_full(readlane(col[k], k));
    }
    if (lane < 16) {
#pragma unroll
        for (int r = 0; r < 16; ++r) X[r + c * ld] = t[r];
    }
    return bad;
}

// ---------------------------------------------------------------- blocked chol + inverse
// In place on the LDS image X (leading dimension LD, upper 16×16 tiles of a P×P SPD matrix
// whose real size is p; P = 16·nb, nb ≤ NBM ≤ 8): X ← U⁻¹ with UᵀU = X (upper tiles; diagonal tiles
// have a zero strictly-lower part).  Right-looking by 16: leaf (wave 0) → panel
// U_{jb,J} = T_jjᵀ X_{jb,J} → trailing X_IJ −= U_{jb,I}ᵀ U_{jb,J} (MFMA, waves round-robin);
// then W_IJ = −T_I Σ_{L=I+1..J} U_IL W_LJ (inv_column), column J by wave (J−1) mod 4, every U
// read before any write.  Returns 0, or 1 + the first non-positive pivot (all threads).
// W_IJ = −T_I Σ_{L=I+1..J} U_IL W_LJ for one block column J, bottom-up; W_LJ (L < J) stay in
// registers (w[L]) and feed the next products as C-layout B operands; W_JJ = T_J is in LDS.
template <typename T, int NBM>
__device__ __forceinline__ void inv_column(const T *X, int LD, int J, int lane, acc_t<T> (&w)[NBM])
{
    const T *TJ = X + 16 * J * (1 + LD);
#pragma unroll
    for (int I = NBM - 2; I >= 0; --I) {
        if (I < J) {
            acc_t<T> s = tmm<T, false, false, false>(tzero<T>(), X + 16 * I + 16 * J * LD, LD, TJ, LD, 16, lane);
#pragma unroll
            for (int L = I + 1; L < NBM - 1; ++L)
                if (L < J) s = tmm_reg<T, false>(s, X + 16 * I + 16 * L * LD, LD, w[L], lane);
            w[I] = tmm_reg<T, true>(tzero<T>(), X + 16 * I * (1 + LD), LD, s, lane);
        }
    }
}

template <typename T, int NBM = 4>
__device__ int chol_inv(T *X, int LD, int p, int P, int *flag, int tid)
{
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), nb = P >> 4;
    if (KB_ABL & 16) return 0;
    for (int i = p + tid; i < P; i += KB_THREADS) X[i + i * LD] = (T)1;   // identity padding
    if (tid == 0) *flag = 0;
    __syncthreads();
    for (int jb = 0; jb < nb; ++jb) {
        T *Xjj = X + 16 * jb * (1 + LD);
        if (wave == 0) {
            const int bad = leaf_chol_inv<T>(Xjj, LD, min(16, p - 16 * jb), lane);
            if (lane == 0 && bad && !*flag) *flag = 16 * jb + bad;
        }
        __syncthreads();
        if (jb + 1 < nb) {
            for (int J = jb + 1 + wave; J < nb; J += 4) {
                T *Xj = X + 16 * jb + 16 * J * LD;
                const acc_t<T> c = tmm<T, true, false, false>(tzero<T>(), Xjj, LD, Xj, LD, 16, lane);
                tstore(Xj, LD, c, lane);
            }
            __syncthreads();
            const int m = nb - jb - 1;
            for (int qq = wave; qq < m * (m + 1) / 2; qq += 4) {
                int I = 0, rem = qq;
                while (rem >= m - I) {
                    rem -= m - I;
                    ++I;
                }
                const int gI = jb + 1 + I, gJ = gI + rem;
                T *Xij = X + 16 * gI + 16 * gJ * LD;
                acc_t<T> c = tload(Xij, LD, lane);
                c = tmm<T, true, false, true>(c, X + 16 * jb + 16 * gI * LD, LD, X + 16 * jb + 16 * gJ * LD, LD, 16,
                                              lane);
                tstore(Xij, LD, c, lane);
            }
            __syncthreads();
        }
    }
    if (nb > 1) {
        // column J by wave (J − 1) mod 4; a wave holds its columns' W tiles in registers until
        // every wave has read the U tiles it needs (the barrier), then writes them over U
        acc_t<T> wa[NBM], wb[NBM];
        const int Ja = wave + 1, Jb = wave + 5;
        if (Ja < nb) inv_column<T, NBM>(X, LD, Ja, lane, wa);
        if (NBM > 5 && Jb < nb) inv_column<T, NBM>(X, LD, Jb, lane, wb);
        __syncthreads();
#pragma unroll
        for (int I = 0; I < NBM - 1; ++I) {
            if (I < Ja && Ja < nb) tstore(X + 16 * I + 16 * Ja * LD, LD, wa[I], lane);
            if (NBM > 5 && I < Jb && Jb < nb) tstore(X + 16 * I + 16 * Jb * LD, LD, wb[I], lane);
        }
    }
    __syncthreads();
    return *flag;
}

// out[i] = init[i] (±) Σ_{k<K(i)} M[k + i·ld]·x[k] for i < n (column dots), 4 threads per
// output; TRI: K(i) = min(K, i + 1) (upper-triangular M, i.e. Mᵀx); n ≤ 64.
template <typename T, bool TRI, bool NEG>
__device__ __forceinline__ void coldot(T *out, const T *init, const T *M, int ld, const T *x, int K, int n, int tid)
{
    const int i = tid >> 2, part = tid & 3;
    T s = (T)0;
    if (i < n) {
        const int Ki = TRI ? min(K, i + 1) : K;
        for (int k = part; k < Ki; k += 4) s = fma(M[k + i * ld], x[k], s);
    }
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    if (i < n && part == 0) out[i] = init ? (NEG ? init[i] - s : init[i] + s) : (NEG ? -s : s);
}

template <typename T>
struct KbArgs {
    const T *Y, *y, *H, *g;
    T *dz, *lam, *slab;
    int32_t *info;
    const int32_t *meta;
    int N, ginv;
    int64_t b0;                    // first trajectory of this chunk
    int64_t sY, sy, sH, sg, sS;    // per-trajectory strides (elements); sS: slab
    int LD, LDY, LDB;              // LDS leading dims: blocks, Y slab (fwd), staged Y (bwd)
    int oWp, oBlk, oSl, oV;        // fwd LDS offsets (elements of T)
    int oYl, oWl, oV2;             // bwd LDS offsets
    // dense / block-diagonal H (kkt_big_hfac_kernel ran first): Y, g point at its Z = Y U⁻¹,
    // gz = U⁻ᵀg (chunk-relative, yrel = 1), the sweeps use H = I, the backward sweep applies
    // −U⁻¹ (packed per knot in Ui, per-trajectory stride sU) to the residual, and info already
    // holds −(k+1) for a non-SPD H_k
    int hfac, yrel;
    const T *Ui;
    int64_t sU;
    int64_t *prof;                 // KB_PROF builds: [4 waves][8] cycle sums
};

// padded row → row of Y (−1 for a padding row)
__device__ __forceinline__ int rowmap(const Kn &q, int pr)
{
    if (pr < q.P1) return pr < q.p1 ? pr : -1;
    pr -= q.P1;
    if (pr < q.Ps) return pr < q.ps ? q.p1 + pr : -1;
    pr -= q.Ps;
    return pr < q.p2 ? q.p1 + q.ps + pr : -1;
}
__device__ __forceinline__ int part_of(const Kn &q, int I)
{
    const int r = 16 * I;
    return r < q.P1 ? 0 : (r < q.P1 + q.Ps ? 1 : 2);
}

// ---------------------------------------------------------------- single-wave factor tools
// chol_inv on ONE wave (the factor wave of the forward sweep): the same blocked algorithm,
// wave-level ordering only (no workgroup barriers).  The inverse is assembled from the last
// block column down: column J reads U_IL (L ≤ J) of rows I < J and writes W_IJ, which the
// columns after it (smaller J) never read.  Returns 0 or 1 + the first non-positive pivot.
template <typename T>
__device__ int chol_inv_w(T *X, int LD, int p, int P, int lane)
{
    const int nb = P >> 4;
    for (int i = p + lane; i < P; i += 64) X[i + i * LD] = (T)1;
    int bad = 0;
    for (int jb = 0; jb < nb; ++jb) {
        T *Xjj = X + 16 * jb * (1 + LD);
        const int b = leaf_chol_inv<T>(Xjj, LD, min(16, p - 16 * jb), lane);
        if (b && !bad) bad = 16 * jb + b;
        for (int J = jb + 1; J < nb; ++J) {
            T *Xj = X + 16 * jb + 16 * J * LD;
            tstore(Xj, LD, tmm<T, true, false, false>(tzero<T>(), Xjj, LD, Xj, LD, 16, lane), lane);
        }
        for (int I = jb + 1; I < nb; ++I)
            for (int J = I; J < nb; ++J) {
                T *Xij = X + 16 * I + 16 * J * LD;
                tstore(Xij, LD,
                       tmm<T, true, false, true>(tload(Xij, LD, lane), X + 16 * jb + 16 * I * LD, LD,
                                                 X + 16 * jb + 16 * J * LD, LD, 16, lane),
                       lane);
            }
    }
    for (int J = nb - 1; J >= 1; --J) {
        acc_t<T> w[4];
        inv_column<T, 4>(X, LD, J, lane, w);
#pragma unroll
        for (int I = 0; I < 3; ++I)
            if (I < J) tstore(X + 16 * I + 16 * J * LD, LD, w[I], lane);
    }
    return bad;
}

// out[i] = init[i] ± Σ_{k<K(i)} M[k + i·ld]·x[k] for i < n ≤ 64, one lane per output
// (TRI: K(i) = min(K, i + 1): Mᵀx for upper-triangular M); in place (out == init) is fine
template <typename T, bool TRI, bool NEG>
__device__ __forceinline__ void coldot_w(T *out, const T *init, const T *M, int ld, const T *x, int K, int n, int lane)
{
    if (lane < n) {
        const int Ki = TRI ? min(K, lane + 1) : K;
        const T *mc = M + lane * ld;
        T s0 = (T)0, s1 = (T)0, s2 = (T)0, s3 = (T)0;
        int k = 0;
        for (; k + 3 < Ki; k += 4) {
            s0 = fma(mc[k], x[k], s0);
            s1 = fma(mc[k + 1], x[k + 1], s1);
            s2 = fma(mc[k + 2], x[k + 2], s2);
            s3 = fma(mc[k + 3], x[k + 3], s3);
        }
        for (; k < Ki; ++k) s0 = fma(mc[k], x[k], s0);
        const T sum = (s0 + s1) + (s2 + s3);
        out[lane] = init ? (NEG ? init[lane] - sum : init[lane] + sum) : (NEG ? -sum : sum);
    }
}

// ---------------------------------------------------------------- Schur pieces (3 waves)
// Upper 16×16 tiles of Y H⁻¹ Yᵀ over a knot's padded row blocks (NBT of them), tile q (row-
// major over I ≤ J) owned by Schur wave q mod 3; compile-time per (NBT, wave), so the row-block
// fragments a wave needs are registers with static indices.
__host__ __device__ constexpr int tm_I(int nbt, int q)
{
    int I = 0;
    while (q >= nbt - I) {
        q -= nbt - I;
        ++I;
    }
    return I;
}
__host__ __device__ constexpr int tm_J(int nbt, int q)
{
    int I = 0;
    while (q >= nbt - I) {
        q -= nbt - I;
        ++I;
    }
    return I + q;
}
constexpr int KB_ST = 12;      // Schur tiles per Schur wave: 36 / 3
__host__ __device__ constexpr bool tm_need(int nbt, int si, int v)
{
    if (v % 3 == si) return true;                       // r = Y H⁻¹ g rows of block v
    for (int q = si; q < nbt * (nbt + 1) / 2; q += 3)
        if (tm_I(nbt, q) == v || tm_J(nbt, q) == v) return true;
    return false;
}

// compile-time loop: f(std::integral_constant<int, i>) for i = 0 … N−1 (indices stay constant
// expressions, so register arrays indexed by them never go to scratch)
template <typename F, int... Is>
__device__ __forceinline__ void sfor_(F &&f, std::integer_sequence<int, Is...>)
{
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F &&f)
{
    sfor_(f, std::make_integer_sequence<int, N>{});
}

// shur! (jacobian_blocks.jl:231-242) for knot q by Schur wave SI: this wave's tiles of
// YYt = Y·(H⁻¹Yᵀ) into acc and its rows of r = Y H⁻¹ g into rn (padded row order), Y read
// column by column straight from HBM (each k-step: one 4-column slice, lane = (row i, column
// g) as the MFMA operand maps want), one slice prefetched ahead.
template <typename T, int NBT, int SI>
__device__ __forceinline__ void schur_part(const Kn &q, const T *Yt, const T *Ht, const T *gt, bool hinv, bool useg,
                                           acc_t<T> (&acc)[KB_ST], T *rn, int lane)
{
    const int i16 = lane & 15, g4 = lane >> 4;
    int rb[NBT], lim[NBT];
#pragma unroll
    for (int v = 0; v < NBT; ++v) {
        const int r0 = 16 * v;
        if (r0 < q.P1) {
            rb[v] = r0;
            lim[v] = q.p1 - r0;
        } else if (r0 < q.P1 + q.Ps) {
            rb[v] = q.p1 + r0 - q.P1;
            lim[v] = q.ps - (r0 - q.P1);
        } else {
            rb[v] = q.p1 + q.ps + r0 - q.P1 - q.Ps;
            lim[v] = q.p2 - (r0 - q.P1 - q.Ps);
        }
    }
#pragma unroll
    for (int t = 0; t < KB_ST; ++t) acc[t] = tzero<T>();
    T rp[NBT];
#pragma unroll
    for (int v = 0; v < NBT; ++v) rp[v] = (T)0;
    const int nks = (q.w + 3) >> 2;
    const T *base = Yt + q.oY + i16;
    auto load = [&](int s, T (&f)[NBT], T &h, T &gg) __attribute__((always_inline)) {
        const int c = 4 * s + g4;
        const bool ok = c < q.w;
        const T *src = base + (int64_t)(ok ? c : 0) * q.rows;
        sfor<NBT>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            if constexpr (tm_need(NBT, SI, v)) f[v] = (ok && i16 < lim[v]) ? src[rb[v]] : (T)0;
        });
        h = ok ? (hinv ? (T)1 / Ht[q.oH + c] : (T)1) : (T)0;
        gg = (ok && useg) ? gt[q.og + c] : (T)0;
    };
    auto step = [&](const T (&f)[NBT], T h, T gg) __attribute__((always_inline)) {
        sfor<KB_ST>([&](auto tc) {
            constexpr int t = decltype(tc)::value, qq = SI + 3 * t;
            if constexpr (qq < NBT * (NBT + 1) / 2) {
                constexpr int I = tm_I(NBT, qq), J = tm_J(NBT, qq);
                const T av = f[I];
                const T bv = f[J] * h;
                if (KB_ABL & 2) acc[t][0] += av * bv;
                else acc[t] = Tile<T>::mma(av, bv, acc[t]);
            }
        });
        sfor<NBT>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            if constexpr (v % 3 == SI) rp[v] = fma(f[v] * h, gg, rp[v]);
        });
    };
    T fa[NBT], fb[NBT], ha = (T)0, hb = (T)0, ga = (T)0, gb = (T)0;
#pragma unroll
    for (int v = 0; v < NBT; ++v) fa[v] = fb[v] = (T)0;
    load(0, fa, ha, ga);
    for (int s = 0; s < nks; s += 2) {
        if (s + 1 < nks) load(s + 1, fb, hb, gb);
        step(fa, ha, ga);
        if (s + 1 < nks) {
            if (s + 2 < nks) load(s + 2, fa, ha, ga);
            step(fb, hb, gb);
        }
    }
    sfor<NBT>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        if constexpr (v % 3 == SI) {
            T x = rp[v];
            x += __shfl_xor(x, 16);
            x += __shfl_xor(x, 32);
            if (lane < 16) rn[16 * v + lane] = x;
        }
    });
}

// copy_shur! (:271-286): this wave's non-alias tiles of knot q into its LDS blocks
template <typename T, int NBT, int SI>
__device__ __forceinline__ void schur_store(const Kn &q, T *blk, int LD, const acc_t<T> (&acc)[KB_ST], int lane)
{
    const Bo b = blk_off(q.P1, q.Ps, q.P2, LD);
    sfor<KB_ST>([&](auto tc) {
        constexpr int t = decltype(tc)::value, qq = SI + 3 * t;
        if constexpr (qq < NBT * (NBT + 1) / 2) {
            constexpr int I = tm_I(NBT, qq), J = tm_J(NBT, qq);
            const int pi = part_of(q, I), pj = part_of(q, J);
            if (!(pi == 0 && pj == 0)) {                             // A: added into C_{k−1}
                const int li = 16 * I - (pi == 0 ? 0 : pi == 1 ? q.P1 : q.P1 + q.Ps);
                const int lj = 16 * J - (pj == 0 ? 0 : pj == 1 ? q.P1 : q.P1 + q.Ps);
                const int o = pi == 0 ? (pj == 1 ? b.D : b.F) : pi == 1 ? (pj == 1 ? b.B : b.E) : b.C;
                tstore(blk + o + li + lj * LD, LD, acc[t], lane);
            }
        }
    });
}

// the A ≡ previous-C alias (:166, copy_shur! `A .+= YYt[p1, p1]`): knot q's D2 H⁻¹ D2ᵀ tiles
// add into C of the knot before it (at LDS offset oC)
template <typename T, int NBT, int SI>
__device__ __forceinline__ void schur_addA(const Kn &q, T *Cprev, int LD, const acc_t<T> (&acc)[KB_ST], int lane)
{
    sfor<KB_ST>([&](auto tc) {
        constexpr int t = decltype(tc)::value, qq = SI + 3 * t;
        if constexpr (qq < NBT * (NBT + 1) / 2) {
            constexpr int I = tm_I(NBT, qq), J = tm_J(NBT, qq);
            if (16 * J < q.P1) tadd(Cprev + 16 * I + 16 * J * LD, LD, acc[t], lane);
        }
    });
}

// runtime NBT (1..8) and Schur-wave index (0..2) → the compile-time instances
#define KB_NBT_SWITCH(nbt, CALL)                                                                            \
    switch (nbt) {                                                                                          \
    case 1: CALL(1); break;                                                                                 \
    case 2: CALL(2); break;                                                                                 \
    case 3: CALL(3); break;                                                                                 \
    case 4: CALL(4); break;                                                                                 \
    case 5: CALL(5); break;                                                                                 \
    case 6: CALL(6); break;                                                                                 \
    case 7: CALL(7); break;                                                                                 \
    default: CALL(8); break;                                                                                \
    }
template <typename T, int SI>
__device__ __forceinline__ void schur_part_d(const Kn &q, const T *Yt, const T *Ht, const T *gt, bool hinv, bool useg,
                             acc_t<T> (&acc)[KB_ST], T *rn, int lane)
{
#define KB_C(NB) schur_part<T, NB, SI>(q, Yt, Ht, gt, hinv, useg, acc, rn, lane)
    KB_NBT_SWITCH(q.R >> 4, KB_C)
#undef KB_C
}
template <typename T, int SI>
__device__ __forceinline__ void schur_store_d(const Kn &q, T *blk, int LD, const acc_t<T> (&acc)[KB_ST], int lane)
{
#define KB_C(NB) schur_store<T, NB, SI>(q, blk, LD, acc, lane)
    KB_NBT_SWITCH(q.R >> 4, KB_C)
#undef KB_C
}
template <typename T, int SI>
__device__ __forceinline__ void schur_addA_d(const Kn &q, T *Cprev, int LD, const acc_t<T> (&acc)[KB_ST], int lane)
{
#define KB_C(NB) schur_addA<T, NB, SI>(q, Cprev, LD, acc, lane)
    KB_NBT_SWITCH(q.R >> 4, KB_C)
#undef KB_C
}

// ---------------------------------------------------------------- forward sweep
// Per trajectory one workgroup of 4 waves.  At step k the "factor wave" (wave k mod 4, rotated
// so the serial work spreads over the SIMDs) factors knot k alone — potrf/inverse chain,
// forward substitution, slab stores — while the other three ("Schur waves") form the Schur
// pieces of knot k+2 from HBM.  Between steps (three barriers): the Schur tiles of knot k+1
// (computed one step earlier and held in registers, `pend`) go into the LDS blocks, knot k+2's
// A-tiles add into C_{k+1}, and all four waves run the products D̃ = Ã⁻ᵀD, F̃ = Ã⁻ᵀF and the
// updates B −= D̃ᵀD̃, E −= D̃ᵀF̃, C −= F̃ᵀF̃ of knot k+1.
template <typename T>
__global__ void __launch_bounds__(KB_THREADS, sizeof(T) == 4 ? 2 : 1) kkt_big_fwd_kernel(KbArgs<T> a)
{
    extern __shared__ __align__(16) unsigned char kb_lds_raw[];
    T *lds = (T *)kb_lds_raw;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t t = a.b0 + blockIdx.x;
    const int LD = a.LD;
    T *Wp = lds + a.oWp, *blk = lds + a.oBlk;
    T *vc = lds + a.oV, *vd = vc + 64, *vlp = vd + 64, *vmu = vlp + 64, *vla = vmu + 64, *vt1 = vla + 64,
      *vt2 = vt1 + 64, *rnb = vt2 + 64;                      // rnb: r of two knots, [2][KB_RMAX]
    int *infol = (int *)(rnb + 2 * KB_RMAX);
    const int64_t ty = a.yrel ? (int64_t)blockIdx.x : t;
    const T *Yt = a.Y + ty * a.sY, *yt = a.y + t * a.sy, *Ht = a.H + t * a.sH, *gt = a.g + ty * a.sg;
    T *St = a.slab + (int64_t)blockIdx.x * a.sS;
    const int N = a.N;
    const bool hinv = a.ginv && !a.hfac, useg = a.ginv;
    int64_t oS = 0;

    acc_t<T> acc[KB_ST], pend[KB_ST];
    int sip = -1;
#ifdef KB_PROF
    int64_t kb_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif                                           // Schur-wave index `pend` was made with
    auto schur = [&](const Kn &q, int si, T *rn) __attribute__((always_inline)) {
        if (si == 0) schur_part_d<T, 0>(q, Yt, Ht, gt, hinv, useg, acc, rn, lane);
        else if (si == 1) schur_part_d<T, 1>(q, Yt, Ht, gt, hinv, useg, acc, rn, lane);
        else if (si == 2) schur_part_d<T, 2>(q, Yt, Ht, gt, hinv, useg, acc, rn, lane);
    };
    // knot q (= k+1): its pending tiles → LDS blocks, c, d = r − y
    auto store_pending = [&](const Kn &q, const T *rn) __attribute__((always_inline)) {
        if (sip == 0) schur_store_d<T, 0>(q, blk, LD, pend, lane);
        else if (sip == 1) schur_store_d<T, 1>(q, blk, LD, pend, lane);
        else if (sip == 2) schur_store_d<T, 2>(q, blk, LD, pend, lane);
        if (tid < 64) {
            vc[tid] = tid < q.ps ? rn[q.P1 + tid] - yt[q.oy + tid] : (T)0;
            vd[tid] = tid < q.p2 ? rn[q.P1 + q.Ps + tid] - yt[q.oy + q.ps + tid] : (T)0;
        }
    };
    // knot q2 (= k+2): A-tiles into C of q (= k+1), d_{k+1} .+= r_[1] (:251); pend ← acc
    auto add_next = [&](const Kn &q, const Kn &q2, int si, const T *rn2) __attribute__((always_inline)) {
        const Bo b = blk_off(q.P1, q.Ps, q.P2, LD);
        if (si == 0) schur_addA_d<T, 0>(q2, blk + b.C, LD, acc, lane);
        else if (si == 1) schur_addA_d<T, 1>(q2, blk + b.C, LD, acc, lane);
        else if (si == 2) schur_addA_d<T, 2>(q2, blk + b.C, LD, acc, lane);
        if (tid < q2.p1) vd[tid] += rn2[tid];
    };
    auto keep = [&](int si) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < KB_ST; ++u) pend[u] = acc[u];
        sip = si;
    };
    // products of knot q needing every wave: D̃ = Ã⁻ᵀD (:49), F̃ = Ã⁻ᵀF (:57) with Ã⁻¹ = W_{k−1}
    // in Wp (in place: all results in registers before the barrier), then B −= D̃ᵀD̃ (:50-52),
    // E −= D̃ᵀF̃ (:59), C −= F̃ᵀF̃ (:61) on the upper tiles
    auto prefactor = [&](const Kn &q0) __attribute__((always_inline)) {
        if (!q0.P1) return;
        const Bo b0 = blk_off(q0.P1, q0.Ps, q0.P2, LD);
        const int n1t = q0.P1 >> 4, nst = q0.Ps >> 4, n2t = q0.P2 >> 4, nD = n1t * nst, nF = n1t * n2t;
        acc_t<T> f1[KB_F1T];
#pragma unroll
        for (int s2 = 0; s2 < KB_F1T; ++s2) {
            const int qq = wave + 4 * s2;
            if (qq < nD + nF) {
                const bool isD = qq < nD;
                const int r = isD ? qq : qq - nD, nc = isD ? nst : n2t, I = r / nc, J = r - I * nc;
                f1[s2] = tmm<T, true, false, false>(tzero<T>(), Wp + 16 * I * LD, LD,
                                                    blk + (isD ? b0.D : b0.F) + 16 * J * LD, LD, 16 * (I + 1), lane);
            }
        }
        __syncthreads();
#pragma unroll
        for (int s2 = 0; s2 < KB_F1T; ++s2) {
            const int qq = wave + 4 * s2;
            if (qq < nD + nF) {
                const bool isD = qq < nD;
                const int r = isD ? qq : qq - nD, nc = isD ? nst : n2t, I = r / nc, J = r - I * nc;
                tstore(blk + (isD ? b0.D : b0.F) + 16 * I + 16 * J * LD, LD, f1[s2], lane);
            }
        }
        __syncthreads();
        const int nB = nst * (nst + 1) / 2, nE = nst * n2t, nC = n2t * (n2t + 1) / 2;
        for (int qq = wave; qq < nB + nE + nC; qq += 4) {
            int I, J, o;
            const T *Aop, *Bop;
            if (qq < nB || qq >= nB + nE) {
                const bool isB = qq < nB;
                const int m = isB ? nst : n2t;
                int rem = isB ? qq : qq - nB - nE;
                I = 0;
                while (rem >= m - I) {
                    rem -= m - I;
                    ++I;
                }
                J = I + rem;
                o = isB ? b0.B : b0.C;
                Aop = blk + (isB ? b0.D : b0.F);
                Bop = Aop;
            } else {
                const int r = qq - nB;
                I = r / n2t;
                J = r - I * n2t;
                o = b0.E;
                Aop = blk + b0.D;
                Bop = blk + b0.F;
            }
            T *X = blk + o + 16 * I + 16 * J * LD;
            acc_t<T> c = tload(X, LD, lane);
            c = tmm<T, true, false, true>(c, Aop + 16 * I * LD, LD, Bop + 16 * J * LD, LD, q0.P1, lane);
            tstore(X, LD, c, lane);
        }
    };
    // the factor wave's part of knot q0 (cholesky_solve.jl:47-67 after the products above,
    // forward_substitution! :93-117, the slab): single wave, no barriers
    auto factor = [&](const Kn &q0, int k) __attribute__((always_inline)) {
        const Bo b0 = blk_off(q0.P1, q0.Ps, q0.P2, LD);
        const int nst = q0.Ps >> 4, n2t = q0.P2 >> 4;
        int bad = 0;
        KB_F0();
        for (int pass = 0; pass < 2; ++pass) {         // B̃ (:53) → Binv, then C̃ (:62) → W_k
            const bool isB = pass == 0;
            const int pp = isB ? q0.ps : q0.p2;
            if (!pp || (KB_ABL & 16)) continue;
            bad |= chol_inv_w<T>(blk + (isB ? b0.B : b0.C), LD, pp, isB ? q0.Ps : q0.P2, lane);
            if (isB && q0.P2) {
                for (int J = 0; J < n2t; ++J)                                  // Ẽ = B̃⁻ᵀE (:60)
                    for (int I = nst - 1; I >= 0; --I) {
                        T *X = blk + b0.E + 16 * I + 16 * J * LD;
                        tstore(X, LD,
                               tmm<T, true, false, false>(tzero<T>(), blk + b0.B + 16 * I * LD, LD,
                                                          blk + b0.E + 16 * J * LD, LD, 16 * (I + 1), lane),
                               lane);
                    }
                for (int I = 0; I < n2t; ++I)                                  // C −= ẼᵀẼ (:61)
                    for (int J = I; J < n2t; ++J) {
                        T *X = blk + b0.C + 16 * I + 16 * J * LD;
                        tstore(X, LD,
                               tmm<T, true, false, true>(tload(X, LD, lane), blk + b0.E + 16 * I * LD, LD,
                                                         blk + b0.E + 16 * J * LD, LD, q0.Ps, lane),
                               lane);
                    }
            }
            if (isB) KB_F(5);
        }
        if (bad && lane == 0 && *infol == 0) *infol = k + 1;
        KB_F(6);
        if (!(KB_ABL & 4)) {
            if (q0.ps) {       // μ = B̃⁻ᵀ(c − D̃ᵀλ_{k−1})
                if (q0.P1) coldot_w<T, false, true>(vt1, vc, blk + b0.D, LD, vlp, q0.P1, q0.Ps, lane);
                else vt1[lane] = vc[lane];
                coldot_w<T, true, false>(vmu, nullptr, blk + b0.B, LD, vt1, q0.Ps, q0.Ps, lane);
            }
            if (q0.p2) {       // λ = C̃⁻ᵀ(d − F̃ᵀλ_{k−1} − Ẽᵀμ)
                if (q0.P1) coldot_w<T, false, true>(vt2, vd, blk + b0.F, LD, vlp, q0.P1, q0.P2, lane);
                else vt2[lane] = vd[lane];
                if (q0.ps) coldot_w<T, false, true>(vt2, vt2, blk + b0.E, LD, vmu, q0.Ps, q0.P2, lane);
                coldot_w<T, true, false>(vla, nullptr, blk + b0.C, LD, vt2, q0.P2, q0.P2, lane);
            }
        }
        KB_F(7);
        if (!(KB_ABL & 8)) {  // slab: W_k, Binv (packed upper), Ẽ, μ, λ
            T *Sk = St + oS;
            const int oB = q0.P2 * (q0.P2 + 1) / 2, oE = oB + q0.Ps * (q0.Ps + 1) / 2, oM = oE + q0.Ps * q0.P2;
            for (int j = 0; j < q0.P2; ++j)
                if (lane <= j) Sk[j * (j + 1) / 2 + lane] = blk[b0.C + lane + j * LD];
            for (int j = 0; j < q0.Ps; ++j)
                if (lane <= j) Sk[oB + j * (j + 1) / 2 + lane] = blk[b0.B + lane + j * LD];
            if (q0.Ps)
                for (int j = 0; j < q0.P2; ++j)
                    if (lane < q0.Ps) Sk[oE + lane + j * q0.Ps] = blk[b0.E + lane + j * LD];
            if (lane < q0.Ps) Sk[oM + lane] = vmu[lane];
            if (lane < q0.P2) Sk[oM + q0.Ps + lane] = vla[lane];
        }
        KB_F(8);
        // W_k becomes Ã⁻¹ of knot k+1 (U[k+1].A ≡ U[k].C, :166); λ_k its λ_{k−1}
        for (int j = 0; j < q0.P2; ++j)
            if (lane < q0.P2) Wp[lane + j * LD] = blk[b0.C + lane + j * LD];
        vlp[lane] = lane < q0.P2 ? vla[lane] : (T)0;
        KB_F(9);
    };

    // steps k = −2, −1 form the Schur pieces of knots 0 and 1 (no factor work yet); every
    // helper has a single call site (each inlines its compile-time instances once)
    Kn qa = kn_load(a.meta, 0), qb = qa, qc = qa;          // knots k, k+1, k+2 of step k
    if (tid == 0) *infol = 0;
    if (tid < 64) vlp[tid] = (T)0;
    for (int k = -2; k < N; ++k) {
        KB_T0();
        const int fw = (k + 4) & 3, sic = wave == fw ? -1 : ((wave - fw - 1) & 3);
        const bool n1 = k + 1 < N, n2 = k + 2 < N;
        if (k >= 0) {
            prefactor(qa);
            __syncthreads();
        }
        KB_T(0);
        if (wave == fw) {
            if (k >= 0) factor(qa, k);
            KB_T(1);
        } else if (n2) {
            schur(qc, sic, rnb + ((k + 2) & 1) * KB_RMAX);
            KB_T(2);
        }
        if (k >= 0) oS += slab_size(qa.Ps, qa.P2);
        __syncthreads();
        KB_T(3);
        if (n1 && k >= -1) {
            store_pending(qb, rnb + ((k + 1) & 1) * KB_RMAX);
            __syncthreads();
        }
        if (n2) {
            if (k >= -1) add_next(qb, qc, sic, rnb + ((k + 2) & 1) * KB_RMAX);
            keep(sic);
        }
        __syncthreads();
        KB_T(4);
        qa = qb;                                              // advance
        qb = qc;
        if (k + 3 < N) qc = kn_load(a.meta, k + 3);
    }
    KB_FLUSH();
    if (tid == 0 && a.info) {
        const int info = *infol;
        if (a.hfac) {
            if (a.info[t] == 0) a.info[t] = info;   // a non-SPD H_k (−(k+1)) takes precedence
        } else {
            a.info[t] = info;
        }
    }
}

// ---------------------------------------------------------------- backward sweep + primals
template <typename T>
__global__ void __launch_bounds__(KB_THREADS) kkt_big_bwd_kernel(KbArgs<T> a)
{
    extern __shared__ __align__(16) unsigned char kb_lds_raw[];
    T *lds = (T *)kb_lds_raw;
    const int tid = threadIdx.x;
    const int64_t t = a.b0 + blockIdx.x;
    const int LDB = a.LDB, N = a.N;
    T *Yl = lds + a.oYl, *Wl = lds + a.oWl;
    const T *Bl = nullptr, *El = nullptr;   // Binv, Ẽ: read from the slab (end knots only)
    T *xm = lds + a.oV2, *xl = xm + 64, *tv = xl + 64, *hv = tv + KB_WMAX, *gv = hv + KB_WMAX, *vv = gv + KB_WMAX,
      *zv = vv + KB_WMAX, *nl = zv + 64, *ev = nl + 64, *nm = ev + 64, *fm = nm + 64, *fl = fm + 64;
    const int64_t ty = a.yrel ? (int64_t)blockIdx.x : t;
    const T *Yt = a.Y + ty * a.sY, *Ht = a.H + t * a.sH, *gt = a.g + ty * a.sg;
    T *dzt = a.dz + t * a.sg, *lat = a.lam + t * a.sy;
    const T *Ut = a.hfac ? a.Ui + (int64_t)blockIdx.x * a.sU : nullptr;
    int64_t oU = 0;
    if (a.hfac)
        for (int k = 0; k < N; ++k) {
            const int w = a.meta[8 * k + 3];
            oU += (int64_t)w * (w + 1) / 2;
        }
    const T *St = a.slab + (int64_t)blockIdx.x * a.sS;

    int64_t oS = 0;
    for (int k = 0; k < N; ++k) {
        const int32_t *m = a.meta + 8 * k;
        oS += slab_size(r16(m[1]), r16(m[2]));
    }
    // knot k's slab (W packed, Binv packed, Ẽ, μ, λ of the forward sweep): W and the two
    // vectors go through registers into LDS (prefetched one knot ahead); Binv, Ẽ (end knots
    // only) are read from the slab in place
    T wpre[KB_WPRE], fpre = (T)0;
    auto slab_fetch = [&](const Kn &q, int64_t o) {
        const T *Sk = St + o;
        const int nW = q.P2 * (q.P2 + 1) / 2, nBv = q.Ps * (q.Ps + 1) / 2, nE = q.Ps * q.P2;
#pragma unroll
        for (int u = 0; u < KB_WPRE; ++u) {
            const int e = tid + KB_THREADS * u;
            wpre[u] = e < nW ? Sk[e] : (T)0;
        }
        if (tid < 128) {
            const int i = tid & 63;
            fpre = tid < 64 ? (i < q.Ps ? Sk[nW + nBv + nE + i] : (T)0) : (i < q.P2 ? Sk[nW + nBv + nE + q.Ps + i] : (T)0);
        }
    };
    auto slab_commit = [&](const Kn &q, int64_t o) {
        const int nW = q.P2 * (q.P2 + 1) / 2, nBv = q.Ps * (q.Ps + 1) / 2;
#pragma unroll
        for (int u = 0; u < KB_WPRE; ++u) {
            const int e = tid + KB_THREADS * u;
            if (e < nW) Wl[e] = wpre[u];
        }
        if (tid < 128) (tid < 64 ? fm : fl)[tid & 63] = fpre;
        Bl = St + o + nW;
        El = St + o + nW + nBv;
    };
    // Y_k (rows × w, contiguous in the packed input): every load of a thread in flight at once
    T ypre[KB_BPRE], hpre = (T)0, gpre = (T)0;
    auto y_fetch = [&](const Kn &q) {
        const int tot = q.rows * q.w;
        const T *src = Yt + q.oY;
#pragma unroll
        for (int u = 0; u < KB_BPRE; ++u) {
            const int e = tid + KB_THREADS * u;
            ypre[u] = e < tot ? src[e] : (T)0;
        }
        if (tid < q.w) {
            hpre = (a.ginv && !a.hfac) ? (T)1 / Ht[q.oH + tid] : (T)1;
            gpre = a.ginv ? gt[q.og + tid] : (T)0;
        }
    };
    auto y_commit = [&](const Kn &q) {
        const int tot = q.rows * q.w, sr = KB_THREADS % q.rows, sc = KB_THREADS / q.rows;
        int r = tid % q.rows, c = tid / q.rows;
#pragma unroll
        for (int u = 0; u < KB_BPRE; ++u) {
            if (tid + KB_THREADS * u < tot) Yl[r + c * LDB] = ypre[u];
            r += sr;
            c += sc;
            if (r >= q.rows) {
                r -= q.rows;
                ++c;
            }
        }
        if (tid < q.w) {
            hv[tid] = hpre;
            gv[tid] = gpre;
        }
    };
    // x ← B̃⁻¹ x for packed upper Binv (row dots): out[i] = Σ_{c ≥ i} U⁻¹[i][c] x[c]
    auto rowdot_packed = [&](T *out, const T *P, const T *x, int n) {
        const int i = tid >> 2, part = tid & 3;
        T s = (T)0;
        if (i < n)
            for (int c = i + part; c < n; c += 4) s = fma(P[c * (c + 1) / 2 + i], x[c], s);
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        if (i < n && part == 0) out[i] = s;
    };

    // terminal knot (backward_substitution! :139-143): μ_N = −B̃⁻¹μ, λ_N as the forward gave it
    Kn qj = kn_load(a.meta, N - 1);
    y_fetch(qj);
    oS -= slab_size(qj.Ps, qj.P2);
    slab_fetch(qj, oS);
    slab_commit(qj, oS);
    __syncthreads();
    if (qj.ps) rowdot_packed(nm, Bl, fm, qj.ps);
    __syncthreads();
    if (tid < 64) {
        xm[tid] = tid < qj.ps ? -nm[tid] : (T)0;
        xl[tid] = tid < qj.p2 ? fl[tid] : (T)0;
    }
    __syncthreads();
    if (tid < qj.ps) lat[qj.oy + tid] = xm[tid];
    if (tid < qj.p2) lat[qj.oy + qj.ps + tid] = xl[tid];
    int64_t oSp = oS;
    if (N > 1) {                                   // knot N−2's slab, for step j = N−1
        const Kn q = kn_load(a.meta, N - 2);
        oSp -= slab_size(q.Ps, q.P2);
        slab_fetch(q, oSp);
    }

    for (int j = N - 1; j >= 0; --j) {
        y_commit(qj);
        Kn qp = qj;
        if (j > 0) {
            qp = kn_load(a.meta, j - 1);
            slab_commit(qp, oSp);
        }
        __syncthreads();
        // prefetch for step j−1: Y_{j−1} and knot j−2's slab
        if (j > 0) y_fetch(qp);
        if (j > 1) {
            const Kn q2 = kn_load(a.meta, j - 2);
            oSp -= slab_size(q2.Ps, q2.P2);
            slab_fetch(q2, oSp);
        }
        // t = [C; D1]ᵀ[μ_j; λ_j]  (calc_residual!'s Cᵀμ + D1ᵀλ, :219-231)
        {
            const int c = tid >> 1, h = tid & 1;
            T s = (T)0;
            if (c < qj.w) {
                for (int r = qj.p1 + h; r < qj.rows; r += 2) {
                    const int rr = r - qj.p1;
                    s = fma(Yl[r + c * LDB], rr < qj.ps ? xm[rr] : xl[rr - qj.ps], s);
                }
            }
            s += __shfl_xor(s, 1);
            if (c < qj.w && h == 0) tv[c] = s;
        }
        __syncthreads();
        if (j > 0) {
            // v = D2 H⁻¹ t = D_{k+1}μ_{k+1} + F_{k+1}λ_{k+1} (the Schur blocks of knot j)
            {
                const int i = tid >> 2, part = tid & 3;
                T s = (T)0;
                if (i < qj.p1)
                    for (int c = part; c < qj.w; c += 4) s = fma(Yl[i + c * LDB], tv[c] * hv[c], s);
                s += __shfl_xor(s, 1);
                s += __shfl_xor(s, 2);
                if (part == 0 && i < 64) vv[i] = i < qj.p1 ? s : (T)0;
            }
            __syncthreads();
            // λ_{j−1} = C̃⁻¹(λ + C̃⁻ᵀ v) = W(λ + Wᵀv)  (:128-135)
            {
                const int i = tid >> 2, part = tid & 3;
                T s = (T)0;
                if (i < qp.p2)
                    for (int kk = part; kk <= i; kk += 4) s = fma(Wl[i * (i + 1) / 2 + kk], vv[kk], s);
                s += __shfl_xor(s, 1);
                s += __shfl_xor(s, 2);
                if (part == 0 && i < 64) zv[i] = i < qp.p2 ? fl[i] + s : (T)0;
            }
            __syncthreads();
            rowdot_packed(nl, Wl, zv, qp.p2);
            __syncthreads();
            if (qp.ps) {
                // μ_{j−1} = B̃⁻¹(μ − Ẽλ)  (:136-137)
                {
                    const int i = tid >> 2, part = tid & 3;
                    T s = (T)0;
                    if (i < qp.ps)
                        for (int c = part; c < qp.p2; c += 4) s = fma(El[i + c * qp.Ps], nl[c], s);
                    s += __shfl_xor(s, 1);
                    s += __shfl_xor(s, 2);
                    if (part == 0 && i < qp.ps) ev[i] = fm[i] - s;
                }
                __syncthreads();
                rowdot_packed(nm, Bl, ev, qp.ps);
                __syncthreads();
            }
            // negate (:138) and hand over: x = [μ_{j−1}; λ_{j−1}] for knot j−1
            if (tid < 64) {
                xl[tid] = tid < qp.p2 ? -nl[tid] : (T)0;
                xm[tid] = tid < qp.ps ? -nm[tid] : (T)0;
            }
            __syncthreads();
            if (tid < qp.ps) lat[qp.oy + tid] = xm[tid];
            if (tid < qp.p2) lat[qp.oy + qp.ps + tid] = xl[tid];
        }
        // δz_j = −H⁻¹(t + D2ᵀλ_{j−1} + g)  (calc_residual! + calc_primals!, :195-236)
        {
            const int c = tid >> 1, h = tid & 1;
            T s = (T)0;
            if (c < qj.w && j > 0)
                for (int r = h; r < qj.p1; r += 2) s = fma(Yl[r + c * LDB], xl[r], s);
            s += __shfl_xor(s, 1);
            if (c < qj.w && h == 0) {
                const T res = tv[c] + s + gv[c];
                if (a.hfac) vv[c] = res;                 // δz = −U⁻¹(Zᵀλ + U⁻ᵀg) below
                else dzt[qj.og + c] = -(res * hv[c]);
            }
        }
        __syncthreads();
        if (a.hfac) {
            // δz = −H⁻¹ res = −U⁻¹ (U⁻ᵀ res'), res' already U⁻ᵀ-applied: row dots on packed U⁻¹
            oU -= (int64_t)qj.w * (qj.w + 1) / 2;
            const T *Uk = Ut + oU;
            const int i = tid >> 1, h = tid & 1;
            T s = (T)0;
            if (i < qj.w)
                for (int c = i + h; c < qj.w; c += 2) s = fma(Uk[c * (c + 1) / 2 + i], vv[c], s);
            s += __shfl_xor(s, 1);
            if (i < qj.w && h == 0) dzt[qj.og + i] = -s;
            __syncthreads();
        }
        qj = qp;
    }
}

// ---------------------------------------------------------------- dense / block-diagonal H
// kkt_big_hfac_kernel (BlockCholesky dense and block-diagonal modes, block_cholesky.jl:55-77,
// 145-153): per trajectory and knot, H_k = UᵀU (potrf 'U'; a non-positive pivot → info =
// −(k+1), as the oracle reports it) → U⁻¹ (chol_inv, up to 8 diagonal blocks), then
//   Z_k = Y_k U⁻¹   so that Z Zᵀ = Y H⁻¹ Yᵀ (shur!'s YYt, jacobian_blocks.jl:234-240),
//   gz_k = U⁻ᵀ g_k  so that Z gz = Y H⁻¹ g (:236) and the residual Zᵀλ + gz = U⁻ᵀ(Yᵀλ + g),
// with U⁻¹ kept (packed) for the backward sweep's δz = −U⁻¹(Zᵀλ + gz) (calc_primals!,
// cholesky_solver.jl:195-199).  The sweeps then run with H = I on (Z, gz).
template <typename T>
struct KhArgs {
    const T *Y, *H, *g;
    T *Z, *gz, *Ui;
    int32_t *info;
    const int32_t *meta;
    int N, LDH;
    int64_t b0, sY, sH, sg, sU;
};

template <typename T>
__global__ void __launch_bounds__(KB_THREADS, 1) kkt_big_hfac_kernel(KhArgs<T> a)
{
    extern __shared__ __align__(16) unsigned char kb_lds_raw[];
    T *X = (T *)kb_lds_raw;
    int *flag = (int *)(X + a.LDH * KB_WMAX);
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6),
              i16 = lane & 15, g4 = lane >> 4;
    const int64_t t = a.b0 + blockIdx.x, c = blockIdx.x;
    const int LDH = a.LDH;
    const T *Yt = a.Y + t * a.sY, *Ht = a.H + t * a.sH, *gt = a.g + t * a.sg;
    T *Zt = a.Z + c * a.sY, *gzt = a.gz + c * a.sg, *Ut = a.Ui + c * a.sU;
    int hfail = 0;
    int64_t oU = 0;
    for (int k = 0; k < a.N; ++k) {
        const Kn q = kn_load(a.meta, k);
        const int w = q.w, W16 = r16(w), rows = q.rows;
        for (int e = tid; e < W16 * W16; e += KB_THREADS) {
            const int j = e / W16, i = e - j * W16;
            X[i + j * LDH] = (i < w && j < w) ? Ht[q.oH + i + j * w] : (T)0;
        }
        __syncthreads();
        const int bad = chol_inv<T, 8>(X, LDH, w, W16, flag, tid);
        if (bad && !hfail) hfail = k + 1;
        {   // gz = U⁻ᵀ g
            const int i = tid >> 1, h = tid & 1;
            T s = (T)0;
            if (i < w)
                for (int kk = h; kk <= i; kk += 2) s = fma(X[kk + i * LDH], gt[q.og + kk], s);
            s += __shfl_xor(s, 1);
            if (i < w && h == 0) gzt[q.og + i] = s;
        }
        for (int j = wave; j < w; j += 4)
            for (int i = lane; i <= j; i += 64) Ut[oU + j * (j + 1) / 2 + i] = X[i + j * LDH];
        // Z = Y U⁻¹ (rows × w): A = Y from global (column-major, ld rows), B = U⁻¹ from LDS
        const int RT = (rows + 15) >> 4, WT = W16 >> 4;
        for (int qq = wave; qq < RT * WT; qq += 4) {
            const int I = qq / WT, J = qq - I * WT, row = 16 * I + i16;
            acc_t<T> cc = tzero<T>();
            for (int kt = 0; kt <= J; ++kt) {
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) {
                    const int kk = 16 * kt + 4 * s2 + g4;
                    const T av = (row < rows && kk < w) ? Yt[q.oY + row + kk * rows] : (T)0;
                    const T bv = X[kk + (16 * J + i16) * LDH];
                    cc = Tile<T>::mma(av, bv, cc);
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int rr = 16 * I + Tile<T>::row(lane, r), col = 16 * J + i16;
                if (rr < rows && col < w) Zt[q.oY + rr + col * rows] = cc[r];
            }
        }
        oU += (int64_t)w * (w + 1) / 2;
        __syncthreads();
    }
    if (tid == 0 && a.info) a.info[t] = hfail ? -hfail : 0;
}

// ================================================================ split forward sweep
// The fused forward kernel above keeps one trajectory per workgroup: its Schur waves wait on
// HBM behind a one-slice prefetch, its factor wave on a serial LDS chain, and two
// trajectories fit a CU (KB_PROF, configs[4]: ~107 k cycles per step for ~10 k cycles of
// MFMA work).  The split path runs the two halves as separate kernels:
//   kb_schur_kernel  — shur! (jacobian_blocks.jl:231-242) for every knot, in parallel over
//                      (trajectory, run of KS_L knots): Y H⁻¹ Yᵀ (upper tiles) and Y H⁻¹ g on
//                      MFMA, Y streamed from HBM through a KS_PF-deep register ring; writes a
//                      per-knot image of the Schur blocks with copy_shur!'s A ≡ previous-C
//                      alias (:166) and `d .+= r_[1]` (:251) already applied;
//   kb_factor_kernel — cholesky! + forward_substitution! (cholesky_solve.jl:47-117), one wave
//                      per trajectory, every block a register-tile array and every product
//                      in the TN form of lqrx_tile.h (D += MᵀY without data movement); LDS only
//                      for the 16×16 leaves and tile transposes.  Several trajectories per
//                      SIMD hide each other's chains.
// Served when every knot has at most two of (n1, p, n2) nonzero: the trajectory structure
// of conblocks.jl:403-425 (first (0,n,n), interior (n,0,n), last (n,n,0)) and any structure
// without stage constraints at interior knots.  The backward kernel is shared (same slab).

// tunables (tools/tv_ablate.sh A/B builds override them)
#ifndef KS_L_KNOTS
#define KS_L_KNOTS 64
#endif
#ifndef KS_PF_SLICES
#define KS_PF_SLICES 2
#endif
#ifndef KS_MIN_BLOCKS
#define KS_MIN_BLOCKS 4
#endif
#ifndef KS_MIN_BLOCKS_F64
#define KS_MIN_BLOCKS_F64 3          // fp64 tiles need ~1.5x the registers: 4 blocks spill (r03g)
#endif
constexpr int KS_L = KS_L_KNOTS;     // knots per Schur unit (one extra A-only pass per unit)
constexpr int KS_HG = KB_WMAX + 4;   // staged H⁻¹ / g row: w columns padded to the slice grid
constexpr int KS_PF = KS_PF_SLICES;  // k-slices in flight per Schur wave
constexpr int KF_W = 4;        // trajectories (waves) per factor workgroup
constexpr int KF_LU = 68;      // factor LDS image leading dimension
constexpr int KF_SCR = 4 * KS_HG;                     // per-wave leaf scratch (≥ 64 + 256 + 16)
constexpr int KF_LDS = 64 * KF_LU + 64 + KF_SCR;      // per wave: U image, vector, scratch
#ifndef KF_OLD_LEAF
#define KF_OLD_LEAF 0                                 // 1: the 16-lane readlane leaf (A/B builds)
#endif
#ifndef KF_INV_SWEEP
#define KF_INV_SWEEP 0                                // 1: the round-4 leaf inverse sweep (A/B builds)
#endif
#ifndef KF_RSQ_RAW
#define KF_RSQ_RAW 1         // fp32 leaf pivots: v_rsq_f32 without its Newton step (0: A/B)
#endif
#ifndef KF_RSQ1_F64
#define KF_RSQ1_F64 1        // fp64 leaf pivots: v_rsq_f64 + one Newton step instead of two (0: A/B)
#endif
#ifndef KU_ZERO_PEEL
#define KU_ZERO_PEEL 1       // the fused stream's first slice starts its accumulators from a zero C
                             // operand instead of zeroing 26 tiles by v_mov (0: A/B)
#endif
#ifndef KF_LEAF_UNSCALED
#define KF_LEAF_UNSCALED 0   // 1 (A/B builds): unscaled rows, 1/d and 1/√d formed during the LDS
                             // round trip — measured slower (fp32 157.4 vs 155.3 ms, fp64 169.1
                             // vs 167.7 ms configs[4] KKT, profiles r05p): the extra fp64 VALU
                             // costs more than the rsqrt latency it takes off the chain
#endif

// image of one knot (elements of T from the knot's base): tiles D, F, B, E, C (256 elements
// each, lane-major C layout: element 4·lane + r = register r of lane `lane`), then
// v = [c (Ps) | d (P2)]; block tile offsets in tiles, v and end in elements
struct Im {
    int D, F, B, E, C, v, end;
};
__host__ __device__ __forceinline__ Im img_off(int P1, int Ps, int P2)
{
    const int a = P1 >> 4, s = Ps >> 4, b = P2 >> 4;
    Im o;
    int x = 0;
    o.D = x; x += a * s;
    o.F = x; x += a * b;
    o.B = x; x += s * (s + 1) / 2;
    o.E = x; x += s * b;
    o.C = x; x += b * (b + 1) / 2;
    o.v = 256 * x;
    o.end = o.v + Ps + P2;
    return o;
}
// elements of knot k's image slot (64-aligned, so every tile starts 256-B aligned)
__host__ __device__ __forceinline__ int64_t img_len(const int32_t *meta, int k)
{
    const int32_t *m = meta + 8 * k;
    return (img_off(r16(m[0]), r16(m[1]), r16(m[2])).end + 63) & ~(int64_t)63;
}
// image offset of knot k: the knots of a fused interior run [fz0, fz1) have no image
__host__ __device__ __forceinline__ int64_t img_before(const int32_t *meta, int k, int fz0 = 0, int fz1 = 0)
{
    int64_t o = 0;
    for (int j = 0; j < k; ++j)
        if (j < fz0 || j >= fz1) o += img_len(meta, j);
    return o;
}
// index of the upper tile (i ≤ j) of an n×n tile grid, row-major over the upper triangle
__host__ __device__ constexpr int upn(int i, int j, int n) { return i * n - i * (i - 1) / 2 + (j - i); }
__host__ __device__ constexpr int up4(int i, int j) { return upn(i, j, 4); }
__device__ __forceinline__ void tri_ij(int nbt, int q, int &I, int &J)
{
    I = 0;
    while (q >= nbt - I) {
        q -= nbt - I;
        ++I;
    }
    J = I + q;
}

template <typename T>
__device__ __forceinline__ void gstore_tile(T *p, const acc_t<T> &c, int lane) { *(acc_t<T> *)(p + 4 * lane) = c; }
template <typename T>
__device__ __forceinline__ acc_t<T> gload_tile(const T *p, int lane) { return *(const acc_t<T> *)(p + 4 * lane); }
// the transpose of the column-major 16×16 block at X as a C-layout tile
template <typename T>
__device__ __forceinline__ acc_t<T> tload_t(const T *X, int ld, int lane)
{
    acc_t<T> c;
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] = X[(lane & 15) + Tile<T>::row(lane, r) * ld];
    return c;
}
// D (+/−)= Mᵀ·Y for single C-layout tiles
template <typename T, bool NEG = false>
__device__ __forceinline__ acc_t<T> mtn(const acc_t<T> &M, const acc_t<T> &Y, acc_t<T> D)
{
#pragma unroll
    for (int r = 0; r < 4; ++r) D = NEG ? Tile<T>::mma_nega(M[r], Y[r], D) : Tile<T>::mma(M[r], Y[r], D);
    return D;
}
// wave-level ordering of LDS traffic between lanes (in-order LDS per wave; compiler fence)
__device__ __forceinline__ void wsync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- Schur kernel
template <typename T>
struct KsArgs {
    const T *Y, *y, *H, *g;
    T *img;
    const int32_t *meta;
    int N, nruns, hinv, useg, yrel;
    // knot segments: runs [0, nr0) cover knots [0, kend0), the others [kbeg1, N) — with the
    // fused interior kernel the Schur images of the interior run [kend0, kbeg1) are never made
    int nr0, kend0, kbeg1;
    int64_t b0, sY, sy, sH, sg, IMGT;   // IMGT: image elements per trajectory
};

__host__ __device__ constexpr bool ks_need(int nbt, int si, int nw, int v)
{
    if (v % nw == si) return true;     // r = Y H⁻¹ g rows of block v
    for (int q = si; q < nbt * (nbt + 1) / 2; q += nw)
        if (tm_I(nbt, q) == v || tm_J(nbt, q) == v) return true;
    return false;
}

// raw buffer load of one element (voffset + soffset bytes; 0 past the descriptor's size)
template <typename T> __device__ __forceinline__ T bload(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so);
template <> __device__ __forceinline__ float bload<float>(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)vo, (int)so, 0));
}
template <> __device__ __forceinline__ double bload<double>(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so)
{
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)vo, (int)so, 0));
}

// this wave's upper tiles (q = SI + NW·t) of Y H⁻¹ Yᵀ over the knot's padded row blocks and
// its rows (v ≡ SI mod NW) of r = Y H⁻¹ g into rn; k-slices of 4 columns, KS_PF in flight
template <typename T, int NBT, int SI, int NW>
__device__ __forceinline__ void schur_tiles(const Kn &q, const T *Yt, const T *hgl, acc_t<T> (&acc)[(36 + NW - 1) / NW],
                                            T *rn, int lane)
{
    constexpr int ST = (36 + NW - 1) / NW, NTT = NBT * (NBT + 1) / 2;
    const int i16 = lane & 15, g4 = lane >> 4;
    int rb[NBT], lim[NBT];
#pragma unroll
    for (int v = 0; v < NBT; ++v) {
        const int r0 = 16 * v;
        if (r0 < q.P1) {
            rb[v] = r0;
            lim[v] = q.p1 - r0;
        } else if (r0 < q.P1 + q.Ps) {
            rb[v] = q.p1 + r0 - q.P1;
            lim[v] = q.ps - (r0 - q.P1);
        } else {
            rb[v] = q.p1 + q.ps + r0 - q.P1 - q.Ps;
            lim[v] = q.p2 - (r0 - q.P1 - q.Ps);
        }
    }
#pragma unroll
    for (int t = 0; t < ST; ++t) acc[t] = tzero<T>();
    T rp[NBT];
#pragma unroll
    for (int v = 0; v < NBT; ++v) rp[v] = (T)0;
    const int nks = (q.w + 3) >> 2;
    // raw buffer loads of the knot's Y block: per k-slice a descriptor starting at the slice
    // whose size is what is left of the block, so the hardware range check (which covers
    // the VGPR offset, not soffset) returns 0 for columns past w and for the slices past the
    // last one that the ring prefetches — nothing past the block is read, not even at the
    // batch's last knot (the end of the caller's Y).  The descriptor is rebuilt per slice on
    // the SALU; per lane one byte offset per row block, fixed for the knot (rows past a
    // block's real rows get an out-of-range offset).  No exec-mask branch per load.
    constexpr uint32_t TS = sizeof(T), OOB = 0x80000000u;
    const char *ybase = (const char *)(Yt + q.oY);
    const int ybytes = q.rows * q.w * (int)TS;
    uint32_t vo[NBT];
#pragma unroll
    for (int v = 0; v < NBT; ++v) vo[v] = i16 < lim[v] ? (uint32_t)((g4 * q.rows + rb[v] + i16) * (int)TS) : OOB;
    const int so_col = 4 * q.rows * (int)TS;
    T f[KS_PF][NBT], hh[KS_PF], gg[KS_PF];
    auto load = [&](int s, T (&fr)[NBT], T &h, T &g_) __attribute__((always_inline)) {
        const int so = s * so_col;
        const __amdgpu_buffer_rsrc_t ry =
            __builtin_amdgcn_make_buffer_rsrc((void *)(ybase + so), (short)0, max(ybytes - so, 0), 0x00020000);
        sfor<NBT>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            if constexpr (ks_need(NBT, SI, NW, v)) fr[v] = bload<T>(ry, vo[v], 0u);
        });
        // raw H and g: the reciprocal is taken in step(), so nothing here waits for a load
        h = hgl[4 * s + g4];                       // H⁻¹ (or 1; 0 past w) and g, staged per knot
        g_ = hgl[KS_HG + 4 * s + g4];
    };
    auto step = [&](const T (&fr)[NBT], T hx, T gx, int s) __attribute__((always_inline)) {
        const T h = hx, g_ = gx;
        T fh[NBT];
        sfor<NBT>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            if constexpr (ks_need(NBT, SI, NW, v)) fh[v] = fr[v] * h;
        });
        sfor<ST>([&](auto tc) {
            constexpr int t = decltype(tc)::value, qq = SI + NW * t;
            if constexpr (qq < NTT) {
                constexpr int I = tm_I(NBT, qq), J = tm_J(NBT, qq);
                acc[t] = Tile<T>::mma(fr[I], fh[J], acc[t]);
            }
        });
        sfor<NBT>([&](auto vc) {
            constexpr int v = decltype(vc)::value;
            if constexpr (v % NW == SI) rp[v] = fma(fh[v], g_, rp[v]);
        });
    };
    sfor<KS_PF>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        load(u, f[u], hh[u], gg[u]);
    });
    // branch-free body (slices past w read 0 through the descriptors' bounds and get h = 0),
    // so the wait-count pass sees the same loads in flight on every path: each step waits
    // only for its own slice, issued KS_PF steps earlier
    for (int s0 = 0; s0 < nks; s0 += KS_PF) {
        sfor<KS_PF>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            step(f[u], hh[u], gg[u], s0 + u);
            load(s0 + u + KS_PF, f[u], hh[u], gg[u]);
            __builtin_amdgcn_sched_barrier(0);       // keep the ring order (no load sinking)
        });
    }
    sfor<NBT>([&](auto vc) {
        constexpr int v = decltype(vc)::value;
        if constexpr (v % NW == SI) {
            T x = rp[v];
            x += __shfl_xor(x, 16);
            x += __shfl_xor(x, 32);
            if (lane < 16) rn[16 * v + lane] = x;
        }
    });
}

template <typename T, int NW, int NBT>
__device__ __forceinline__ void schur_tiles_d(const Kn &q, int si, const T *Yt, const T *hgl,
                                              acc_t<T> (&acc)[(36 + NW - 1) / NW], T *rn, int lane)
{
    if (si == 0) schur_tiles<T, NBT, 0, NW>(q, Yt, hgl, acc, rn, lane);
    else if (si == 1) schur_tiles<T, NBT, 1 % NW, NW>(q, Yt, hgl, acc, rn, lane);
    else if (NW > 2 && si == 2) schur_tiles<T, NBT, 2 % NW, NW>(q, Yt, hgl, acc, rn, lane);
    else if (NW > 3) schur_tiles<T, NBT, 3 % NW, NW>(q, Yt, hgl, acc, rn, lane);
}

// image tile of the global upper tile (I, J) of knot q (−1: an A tile, which belongs to the
// knot before)
__device__ __forceinline__ int img_tile(const Kn &q, const Im &o, int I, int J)
{
    const int a = q.P1 >> 4, s = q.Ps >> 4, b = q.P2 >> 4;
    const int pi = I < a ? 0 : (I < a + s ? 1 : 2), pj = J < a ? 0 : (J < a + s ? 1 : 2);
    const int li = I - (pi == 0 ? 0 : pi == 1 ? a : a + s), lj = J - (pj == 0 ? 0 : pj == 1 ? a : a + s);
    if (pi == 0) return pj == 0 ? -1 : (pj == 1 ? o.D + li * s + lj : o.F + li * b + lj);
    if (pi == 1) return pj == 1 ? o.B + upn(li, lj, s) : o.E + li * b + lj;
    return o.C + upn(li, lj, b);
}

// One workgroup of NW waves per (trajectory, run of KS_L knots).  Knot k's tiles are split
// over the waves and go to knot k's image as they are (C without the alias); once knot k+1's
// tiles exist, the waves owning its A tiles add them into knot k's C tiles in the image
// (read-modify-write, ordered by the workgroup barrier) and knot k's v = [c | d + r1_{k+1}] is
// written from the two knots' r (LDS).  The run's last pass forms only the A tiles (and r1)
// of the first knot of the next run.
template <typename T, int NW, int NBT>
__global__ void __launch_bounds__(64 * NW, sizeof(T) == 8 ? KS_MIN_BLOCKS_F64 : KS_MIN_BLOCKS)
kb_schur_kernel(KsArgs<T> a)
{
    constexpr int ST = (36 + NW - 1) / NW;
    __shared__ T rbuf[2][KB_RMAX];                 // r of two knots (padded row order)
    __shared__ T hgl[2 * KS_HG];                   // H⁻¹ (or 1) | g of the knot, 0 past w
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t u = blockIdx.x, tl = u / a.nruns;
    const int run = (int)(u - tl * a.nruns);
    const int64_t t = a.b0 + tl, ty = a.yrel ? tl : t;
    const T *Yt = a.Y + ty * a.sY, *yt = a.y + t * a.sy, *Ht = a.H + t * a.sH, *gt = a.g + ty * a.sg;
    T *img = a.img + tl * a.IMGT;
    const int k0 = run < a.nr0 ? run * KS_L : a.kbeg1 + (run - a.nr0) * KS_L;
    const int k1 = min(k0 + KS_L, run < a.nr0 ? a.kend0 : a.N);
    int64_t oI = 0, oIp = 0;                       // image offsets of knot k and knot k−1
    oI = img_before(a.meta, k0, a.kend0, a.kbeg1);
    acc_t<T> acc[ST];
    Kn qp = kn_load(a.meta, k0);                   // knot k−1
    // v of knot kk (= qp): [c | d + r1 of knot kk+1 (if nx)]
    auto write_v = [&](int kk, bool nx, int p1n) __attribute__((always_inline)) {
        const Im o = img_off(qp.P1, qp.Ps, qp.P2);
        T *ik = img + oIp;
        const T *rk = rbuf[kk & 1], *rx = rbuf[(kk + 1) & 1];
        for (int e = tid; e < qp.Ps + qp.P2; e += 64 * NW) {
            T v;
            if (e < qp.Ps) {
                v = e < qp.ps ? rk[qp.P1 + e] - yt[qp.oy + e] : (T)0;
            } else {
                const int j = e - qp.Ps;
                v = j < qp.p2 ? rk[qp.P1 + qp.Ps + j] - yt[qp.oy + qp.ps + j] : (T)0;
                if (nx && j < p1n) v += rx[j];
            }
            ik[o.v + e] = v;
        }
    };
    for (int k = k0; k <= k1 && k < a.N; ++k) {
        const Kn q = kn_load(a.meta, k);
        const bool aonly = k == k1;
        Kn qs = q;
        if (aonly) {
            qs.ps = qs.p2 = 0;
            qs.Ps = qs.P2 = 0;
            qs.R = qs.P1;
        }
        // tiles over the launch's NBT×NBT block grid (the largest knot); rows past this
        // knot's R are zero fragments and their tiles are not stored
        // H⁻¹ (one division per column and knot, not per slice and lane) and g into LDS; the
        // previous knot's readers are past the barriers that closed its iteration
        for (int c = tid; c < KS_HG; c += 64 * NW) {
            const bool in = c < q.w;
            hgl[c] = in ? (a.hinv ? (T)1 / Ht[q.oH + c] : (T)1) : (T)0;
            hgl[KS_HG + c] = (in && a.useg) ? gt[q.og + c] : (T)0;
        }
        __syncthreads();
        if (qs.R) schur_tiles_d<T, NW, NBT>(qs, wave, Yt, hgl, acc, rbuf[k & 1], lane);
        const int nbt = qs.R >> 4, n1t = qs.P1 >> 4;
        if (!aonly) {
            const Im o = img_off(q.P1, q.Ps, q.P2);
            T *ik = img + oI;
#pragma unroll
            for (int s = 0; s < ST; ++s) {
                const int qq = wave + NW * s;
                if (qq < NBT * (NBT + 1) / 2) {
                    int I, J;
                    tri_ij(NBT, qq, I, J);
                    const int it = J < nbt ? img_tile(q, o, I, J) : -1;
                    if (it >= 0) gstore_tile(ik + 256 * it, acc[s], lane);
                }
            }
        }
        __syncthreads();                           // knot k−1's C tiles stored; rbuf[k & 1] complete
        if (k > k0) {
            // copy_shur! alias: knot k's A tiles into knot k−1's C tiles
            const Im o = img_off(qp.P1, qp.Ps, qp.P2);
            T *ip = img + oIp;
            const int b = qp.P2 >> 4;
#pragma unroll
            for (int s = 0; s < ST; ++s) {
                const int qq = wave + NW * s;
                if (qq < NBT * (NBT + 1) / 2) {
                    int I, J;
                    tri_ij(NBT, qq, I, J);
                    if (J < n1t) {
                        T *pc = ip + 256 * (o.C + upn(I, J, b));
                        gstore_tile(pc, gload_tile(pc, lane) + acc[s], lane);
                    }
                }
            }
            write_v(k - 1, true, q.p1);
        }
        if (!aonly) {
            qp = q;
            oIp = oI;
            oI += img_len(a.meta, k);
        }
        __syncthreads();                           // rbuf reuse
    }
    if (k1 == a.N) write_v(a.N - 1, false, 0);     // the last knot: nothing to alias
}

// ---------------------------------------------------------------- factor kernel
template <typename T>
struct KfArgs {
    const T *img;
    T *slab;
    int32_t *info;
    const int32_t *meta;
    int N, hfac;
    int kb, ke;                    // knot range of this launch (the state at kb − 1 is in the slab)
    int fz0, fz1;                  // knots without an image (the fused interior run), or 0, 0
    int64_t b0, nb, IMGT, sS;
};

// W_{k} (packed upper, slab) → C-layout tiles of X (padded P = 16·nt), and λ_k → row layout
template <typename T>
__device__ __forceinline__ void kf_resume(acc_t<T> (&X)[10], T (&lam)[4][4], const T *Sk, int P2, int Ps, int nt, int lane)
{
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j)
            if (j < nt) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * i + Tile<T>::row(lane, r), col = 16 * j + (lane & 15);
                    X[up4(i, j)][r] = row <= col ? Sk[col * (col + 1) / 2 + row] : (T)0;
                }
            }
    const int oM = P2 * (P2 + 1) / 2 + Ps * (Ps + 1) / 2 + Ps * P2;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = 16 * i + Tile<T>::row(lane, r);
            lam[i][r] = e < P2 ? Sk[oM + Ps + e] : (T)0;
        }
}
__device__ __forceinline__ int64_t slab_before(const int32_t *meta, int k)
{
    int64_t o = 0;
    for (int j = 0; j < k; ++j) o += slab_size(r16(meta[8 * j + 1]), r16(meta[8 * j + 2]));
    return o;
}
// info of a launch over knots [kb, ke): the first launch sets it (a non-SPD H_k of the hfac
// pre-pass, −(k+1), takes precedence); later launches only fill a still-zero entry
__device__ __forceinline__ void kf_info(int32_t *info, int64_t t, int v, int kb, int hfac)
{
    if (!info) return;
    if (kb == 0 && !hfac) info[t] = v;
    else if (v && info[t] == 0) info[t] = v;
}

// 16×16 leaf on a C-layout register tile, all 64 lanes (4 elements each): X ← T = U⁻¹ with
// UᵀU = X (upper; T's strictly-lower part is zero).  potrf 'U' right-looking (dpotf2's order
// up to rsqrt-multiply; dynamic_programming.jl:29, cholesky_solve.jl:2): pivot i's scaled row
// U[i][·] (0 at and left of the diagonal) goes through a 64-element LDS row — every row group
// writes its register holding row i of ITS rows, readers take the group that holds row i — and
// every lane applies the rank-1 update to its 4 elements unmasked (the zeros confine it to the
// trailing block).  Then T = U⁻¹ right-looking from the bottom: row k of T = B_k / U_kk is
// broadcast the same way and B_R −= U[R][k]·T_k with U's strictly-upper columns from an LDS
// image.  Only the upper triangle of X is read.  q = real pivots (pivots ≥ q are identity
// padding); returns 1 + the first non-positive pivot, else 0.  scr: KF_SCR elements of LDS.
__device__ __forceinline__ float leaf_rsq(float d) { return __builtin_amdgcn_rsqf(d); }
// fp64: v_rsq_f64 (≈ 1e-8 relative, as v_rcp_f64's 4.6e-8) and ONE Newton step — quadratic, so
// ≈ 1e-16 — where rsqrt_nr takes two (KF_RSQ1_F64 = 0: A/B)
__device__ __forceinline__ double leaf_rsq(double a)
{
    if constexpr (!KF_RSQ1_F64) return rsqrt_nr(a);
    const double y = __builtin_amdgcn_rsq(a);
    const double h = 0.5 * a * y;
    return fma(y, fma(-h, y, 0.5), y);
}

template <typename T>
__device__ __forceinline__ int leaf_chol_inv_t(acc_t<T> &X, T *scr, int q, int lane)
{
    T *ub = scr, *ut = scr + 64, *ri = ut + 256;        // row buffer, Uᵀ image, 1/U_ii
    const int c = lane & 15, g = lane >> 4;
    constexpr bool F64 = sizeof(T) == 8;
    int bad = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int gi = F64 ? (i & 3) : (i >> 2), rgi = F64 ? (i >> 2) : (i & 3);
        const T d = readlane(X[rgi], 16 * gi + i);
        if (!(d > (T)0) && i < q && !bad) bad = i + 1;
        const T sc = rsqrt_nr(d);
        wsync();
        ub[16 * g + c] = c > i ? X[rgi] * sc : (T)0;
        if (lane == 0) ri[i] = sc;
        wsync();
        const T uc = ub[16 * gi + c];
        T ur[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ur[r] = ub[16 * gi + Tile<T>::row(lane, r)];
#pragma unroll
        for (int r = 0; r < 4; ++r) X[r] = fma(-ur[r], uc, X[r]);
        ut[16 * c + i] = uc;                             // U[i][c] (c > i) at [c][i]: Uᵀ, column c
    }
    // B = I; k = 15 … 0: T_k = B_k / U_kk (broadcast), B_R −= U[R][k] T_k for R < k
    acc_t<T> B;
#pragma unroll
    for (int r = 0; r < 4; ++r) B[r] = Tile<T>::row(lane, r) == c ? (T)1 : (T)0;
    T rr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) rr[r] = ri[Tile<T>::row(lane, r)];
#pragma unroll
    for (int k = 15; k >= 0; --k) {
        const int gk = F64 ? (k & 3) : (k >> 2), rgk = F64 ? (k >> 2) : (k & 3);
        const T rk = ri[k];
        wsync();
        ub[16 * g + c] = B[rgk] * rk;
        wsync();
        const T tk = ub[16 * gk + c];
        T uk[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) uk[r] = ut[16 * k + Tile<T>::row(lane, r)];   // U[R][k], 0 for R ≥ k
#pragma unroll
        for (int r = 0; r < 4; ++r) B[r] = fma(-uk[r], tk, B[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) X[r] = B[r] * rr[r];
    wsync();
    return bad;
}

// The same leaf with the inverse carried along (round 5): the factor's row operations — row i
// scaled by 1/U_ii, rows r > i minus U[i][r]·(scaled row i) — applied to E = I as well turn it
// into U⁻ᵀ (the operations compose to U⁻ᵀ, since U⁻ᵀ·X = U), so each of the 16 steps broadcasts
// the scaled row i of E beside the pivot row (one LDS round trip for both) and the separate
// 16-step back-substitution chain of leaf_chol_inv_t disappears.  T = U⁻¹ = Eᵀ goes through the
// caller's image Dg (column-major, KF_LU; where leaf_chol_inv_t's caller stored T): E is written
// transposed and read back as X.  Returns 1 + the first non-positive pivot (< q), else 0.
template <typename T>
__device__ __forceinline__ int leaf_chol_inv_e(acc_t<T> &X, T *scr, T *Dg, int q, int lane)
{
    T *ub = scr, *eb = scr + 64;                        // pivot row of U, scaled row of E
    const int c = lane & 15, g = lane >> 4;
    constexpr bool F64 = sizeof(T) == 8;
    int bad = 0;
    acc_t<T> E;
#pragma unroll
    for (int r = 0; r < 4; ++r) E[r] = Tile<T>::row(lane, r) == c ? (T)1 : (T)0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int gi = F64 ? (i & 3) : (i >> 2), rgi = F64 ? (i >> 2) : (i & 3);
        const T d = readlane(X[rgi], 16 * gi + i);
        if (!(d > (T)0) && i < q && !bad) bad = i + 1;
#if KF_LEAF_UNSCALED
        // the UNSCALED rows go out at once and 1/d, 1/√d are formed while they cross the LDS:
        // U[i][r]·U[i][c] = x_r·(x_c/d), the E rows below take (e_i/d), row i itself e_i/√d
        wsync();
        ub[16 * g + c] = c > i ? X[rgi] : (T)0;
        eb[16 * g + c] = E[rgi];
        wsync();
        const T id = rcp_full(d), sc = rsqrt_nr(d);
        const T uc = ub[16 * gi + c], ec = eb[16 * gi + c];
        T ur[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ur[r] = ub[16 * gi + Tile<T>::row(lane, r)];
        const T tu = uc * id, te = ec * id, es = ec * sc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            X[r] = fma(-ur[r], tu, X[r]);
            E[r] = Tile<T>::row(lane, r) == i ? es : fma(-ur[r], te, E[r]);
        }
#else
        // fp32 (KF_RSQ_RAW): v_rsq_f32 alone — the Newton step (4 VALU per pivot, 256 per knot of
        // the fused kernel) buys nothing at the fp32 solve's 1e-4 tolerance; fp64: one step (leaf_rsq)
        const T sc = (F64 || KF_RSQ_RAW) ? leaf_rsq(d) : rsqrt_nr(d);
        wsync();
        ub[16 * g + c] = c > i ? X[rgi] * sc : (T)0;
        eb[16 * g + c] = E[rgi] * sc;
        wsync();
        const T uc = ub[16 * gi + c], ec = eb[16 * gi + c];
        T ur[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ur[r] = ub[16 * gi + Tile<T>::row(lane, r)];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            X[r] = fma(-ur[r], uc, X[r]);
            E[r] = Tile<T>::row(lane, r) == i ? ec : fma(-ur[r], ec, E[r]);
        }
#endif
    }
    wsync();
#pragma unroll
    for (int r = 0; r < 4; ++r) Dg[c + Tile<T>::row(lane, r) * KF_LU] = E[r];   // T = Eᵀ, column-major
    wsync();
    X = tload(Dg, KF_LU, lane);
    return bad;
}

// In place on the upper tiles X (packed up4) of a P×P SPD matrix (nb ≤ 4 block rows, p real
// pivots): X ← U⁻¹ with UᵀU = X.  Right-looking by 16 as chol_inv: leaf (LDS, one wave) →
// panel U_{jb,J} = T_jjᵀ X_{jb,J} → trailing X_IJ −= U_{jb,I}ᵀ U_{jb,J}, all in registers;
// then W_IJ = −T_I Σ_{L=I+1..J} U_IL W_LJ with U_ILᵀ and T_Iᵀ read transposed from the LDS
// image U (leading dimension KF_LU) the factor phase left there.  Returns 0 or 1 + the
// first non-positive pivot.
// kbc (KB_PROF timing builds only, else null): cycles of the leaves, the panel / trailing
// updates and the inverse assembly added to kbc[0..2]
template <typename T>
__device__ int chol_inv_reg(acc_t<T> (&X)[10], int nb, int p, T *U, T *scr, int lane, int64_t *kbc = nullptr)
{
    int64_t kc0 = kbc ? clock64() : 0;
    auto kct = [&](int i) {
        if (kbc) {
            const int64_t t = clock64();
            kbc[i] += t - kc0;
            kc0 = t;
        }
    };
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
        if (jb < nb) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * jb + Tile<T>::row(lane, r), c = 16 * jb + (lane & 15);
                if (i == c && i >= p) X[up4(jb, jb)][r] = (T)1;     // identity padding
            }
        }
    int bad = 0;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
        if (jb < nb) {
            T *Dg = U + 16 * jb * (1 + KF_LU);
#if KF_OLD_LEAF
            tstore(Dg, KF_LU, X[up4(jb, jb)], lane);
            wsync();
            const int b = leaf_chol_inv<T>(Dg, KF_LU, min(16, p - 16 * jb), lane);
            if (b && !bad) bad = 16 * jb + b;
            wsync();
            X[up4(jb, jb)] = tload(Dg, KF_LU, lane);
            (void)scr;
#elif defined(KF_NOLEAF)
            const int b = 0;       // timing ablation only: no leaf factor (wrong results)
            (void)scr;
#elif KF_INV_SWEEP
            // A/B: the round-4 leaf (inverse by a second 16-step back-substitution sweep)
            const int b = leaf_chol_inv_t<T>(X[up4(jb, jb)], scr, min(16, p - 16 * jb), lane);
            if (b && !bad) bad = 16 * jb + b;
            tstore(Dg, KF_LU, X[up4(jb, jb)], lane);     // T_jj for the inverse assembly's reads
#else
            const int b = leaf_chol_inv_e<T>(X[up4(jb, jb)], scr, Dg, min(16, p - 16 * jb), lane);
            if (b && !bad) bad = 16 * jb + b;            // (T_jj is in Dg for the inverse assembly)
#endif
            kct(0);
#pragma unroll
            for (int J = jb + 1; J < 4; ++J)
                if (J < nb) {
                    X[up4(jb, J)] = mtn<T>(X[up4(jb, jb)], X[up4(jb, J)], tzero<T>());
                    tstore(U + 16 * jb + 16 * J * KF_LU, KF_LU, X[up4(jb, J)], lane);
                }
#pragma unroll
            for (int I = jb + 1; I < 4; ++I)
#pragma unroll
                for (int J = I; J < 4; ++J)
                    if (J < nb) X[up4(I, J)] = mtn<T, true>(X[up4(jb, I)], X[up4(jb, J)], X[up4(I, J)]);
            kct(1);
        }
    }
    wsync();
#pragma unroll
    for (int J = 1; J < 4; ++J)
        if (J < nb) {
#pragma unroll
            for (int I = J - 1; I >= 0; --I) {
                acc_t<T> s = tzero<T>();
#pragma unroll
                for (int L = I + 1; L <= J; ++L)
                    s = mtn<T>(tload_t(U + 16 * I + 16 * L * KF_LU, KF_LU, lane), X[up4(L, J)], s);
                X[up4(I, J)] = mtn<T, true>(tload_t(U + 16 * I * (1 + KF_LU), KF_LU, lane), s, tzero<T>());
            }
        }
    kct(2);
    return bad;
}

// y (column layout: lane holds y[16j + (lane & 15)]) = Mᵀx for x in row layout
// (x[i][r] = x[16i + row(lane, r)]); UP: M is upper (packed up4), else full [i·4 + j]
template <typename T, bool UP, int NM>
__device__ __forceinline__ void mtv(T (&y)[4], const acc_t<T> (&M)[NM], const T (&x)[4][4], int ni, int nj)
{
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        T s = (T)0;
        if (j < nj) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (i < ni && (!UP || i <= j)) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) s = fma(M[UP ? up4(i, j) : i * 4 + j][r], x[i][r], s);
                }
        }
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        y[j] = s;
    }
}
// column layout → row layout through the wave's LDS vector buffer
template <typename T>
__device__ __forceinline__ void col2row(T (&x)[4][4], const T (&y)[4], T *vb, int lane)
{
    if (lane < 16) {
#pragma unroll
        for (int j = 0; j < 4; ++j) vb[16 * j + lane] = y[j];
    }
    wsync();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) x[i][r] = vb[16 * i + Tile<T>::row(lane, r)];
    wsync();
}

// One wave per trajectory.  Registers: X (10 upper tiles) holds W_{k−1} = Ã⁻¹ at the start of
// knot k, then B → B̃⁻¹, then C → W_k; G (a 4×4 tile grid) holds D̃ or F̃ (knots with an n1
// block) or E → Ẽ (the first knot's shape, n1 = 0).  With at most two blocks per knot those
// lifetimes never overlap.
template <typename T>
__global__ void __launch_bounds__(64 * KF_W, sizeof(T) == 4 ? 2 : 1) kb_factor_kernel(KfArgs<T> a)
{
    extern __shared__ __align__(16) unsigned char kb_lds_raw[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t tl = (int64_t)blockIdx.x * KF_W + wave;
    if (tl >= a.nb) return;                          // whole wave; no workgroup barriers below
    T *U = (T *)kb_lds_raw + wave * KF_LDS, *vb = U + 64 * KF_LU, *scr = vb + 64;
    const int64_t t = a.b0 + tl;
    const T *imt = a.img + tl * a.IMGT;
    T *St = a.slab + tl * a.sS;
    int64_t oI = img_before(a.meta, a.kb, a.fz0, a.fz1), oS = slab_before(a.meta, a.kb);
    acc_t<T> X[10], G[16];
    T lam[4][4];                                     // λ_{k−1}, row layout
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) lam[i][r] = (T)0;
    if (a.kb > 0) {
        const int32_t *m = a.meta + 8 * (a.kb - 1);
        const int P2 = r16(m[2]), Ps = r16(m[1]);
        kf_resume<T>(X, lam, St + oS - slab_size(Ps, P2), P2, Ps, P2 >> 4, lane);
    }
    int info = 0;
    // the D or F tiles of knot kn (n1 > 0) into G, every load in flight at once
    auto prefetch_g = [&](int kn, int64_t oIn) __attribute__((always_inline)) {
        const Kn qn = kn_load(a.meta, kn);
        if (!(qn.P1 >> 4)) return;
        const Im on = img_off(qn.P1, qn.Ps, qn.P2);
        const int n1n = qn.P1 >> 4, gc = qn.Ps ? qn.Ps >> 4 : qn.P2 >> 4;
        const T *Yb = imt + oIn + 256 * (qn.Ps ? on.D : on.F);
#pragma unroll
        for (int L = 0; L < 4; ++L)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (L < n1n && j < gc) G[L * 4 + j] = gload_tile(Yb + 256 * (L * gc + j), lane);
    };
    for (int k = a.kb; k < a.ke; ++k) {
        const Kn q = kn_load(a.meta, k);
        const Im o = img_off(q.P1, q.Ps, q.P2);
        const T *ik = imt + oI;
        prefetch_g(k, oI);
        T *Sk = St + oS;
        oI += img_len(a.meta, k);
        oS += slab_size(q.Ps, q.P2);
        const int n1t = q.P1 >> 4, nst = q.Ps >> 4, n2t = q.P2 >> 4;
        const int oB = q.P2 * (q.P2 + 1) / 2, oE = oB + q.Ps * (q.Ps + 1) / 2, oM = oE + q.Ps * q.P2;
        T yv[4] = {(T)0, (T)0, (T)0, (T)0};
        int bad = 0;
        if (n1t) {
            // D̃ = Ã⁻ᵀD or F̃ = Ã⁻ᵀF with Ã⁻¹ = W_{k−1} (:49, :57), in place on the loaded
            // tiles, one column of tiles at a time
            const int gc = nst ? nst : n2t;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j < gc) {
                    acc_t<T> Yc[4];
#pragma unroll
                    for (int L = 0; L < 4; ++L) Yc[L] = G[L * 4 + j];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (i < n1t) {
                            acc_t<T> g = tzero<T>();
#pragma unroll
                            for (int L = 0; L <= i; ++L) g = mtn<T>(X[up4(L, i)], Yc[L], g);
                            G[i * 4 + j] = g;
                        }
                }
            mtv<T, false>(yv, G, lam, n1t, gc);      // D̃ᵀλ_{k−1} or F̃ᵀλ_{k−1}
        }
        T mur[4][4];                                 // μ, row layout (for Ẽᵀμ)
        if (nst) {
            // B̃ = chol(B − D̃ᵀD̃) (:50-53) → X = B̃⁻¹
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = i; j < 4; ++j)
                    if (j < nst) {
                        acc_t<T> c = gload_tile(ik + 256 * (o.B + upn(i, j, nst)), lane);
                        if (n1t) {
#pragma unroll
                            for (int L = 0; L < 4; ++L)
                                if (L < n1t) c = mtn<T, true>(G[L * 4 + i], G[L * 4 + j], c);
                        }
                        X[up4(i, j)] = c;
                    }
            bad |= chol_inv_reg<T>(X, nst, q.ps, U, scr, lane);
            // μ = B̃⁻ᵀ(c − D̃ᵀλ_{k−1})  (:101-107)
            T x[4], xr[4][4], mu[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = (j < nst ? ik[o.v + 16 * j + (lane & 15)] : (T)0) - yv[j];
            col2row<T>(xr, x, vb, lane);
            mtv<T, true>(mu, X, xr, nst, nst);
            col2row<T>(mur, mu, vb, lane);
            // slab: B̃⁻¹ packed upper, μ
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = i; j < 4; ++j)
                    if (j < nst) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = 16 * i + Tile<T>::row(lane, r), col = 16 * j + (lane & 15);
                            if (row <= col) Sk[oB + col * (col + 1) / 2 + row] = X[up4(i, j)][r];
                        }
                    }
            if (lane < 16) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < nst) Sk[oM + 16 * j + lane] = mu[j];
            }
            if (n2t) {
                // (n1 = 0 here) Ẽ = B̃⁻ᵀE (:59-60) into G, column by column
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < n2t) {
                        acc_t<T> Ec[4];
#pragma unroll
                        for (int L = 0; L < 4; ++L)
                            if (L < nst) Ec[L] = gload_tile(ik + 256 * (o.E + L * n2t + j), lane);
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            if (i < nst) {
                                acc_t<T> e = tzero<T>();
#pragma unroll
                                for (int L = 0; L <= i; ++L) e = mtn<T>(X[up4(L, i)], Ec[L], e);
                                G[i * 4 + j] = e;
#pragma unroll
                                for (int r = 0; r < 4; ++r)
                                    Sk[oE + 16 * i + Tile<T>::row(lane, r) + (16 * j + (lane & 15)) * q.Ps] = e[r];
                            }
                    }
            }
        }
        if (n2t) {
            // C̃ = chol(C − F̃ᵀF̃ − ẼᵀẼ) (:61-62) → X = W_k
            const int gr = n1t ? n1t : nst;          // G = F̃ (n1 rows) or Ẽ (p rows)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = i; j < 4; ++j)
                    if (j < n2t) {
                        acc_t<T> c = gload_tile(ik + 256 * (o.C + upn(i, j, n2t)), lane);
#pragma unroll
                        for (int L = 0; L < 4; ++L)
                            if (L < gr) c = mtn<T, true>(G[L * 4 + i], G[L * 4 + j], c);
                        X[up4(i, j)] = c;
                    }
            // Ẽᵀμ for λ while G still holds Ẽ
            T ey[4];
            if (nst) mtv<T, false>(ey, G, mur, nst, n2t);
            bad |= chol_inv_reg<T>(X, n2t, q.p2, U, scr, lane);
            // λ = C̃⁻ᵀ(d − F̃ᵀλ_{k−1} − Ẽᵀμ)  (:108-116)
            T x[4], xr[4][4], lc[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = (j < n2t ? ik[o.v + q.Ps + 16 * j + (lane & 15)] : (T)0) - (nst ? ey[j] : yv[j]);
            col2row<T>(xr, x, vb, lane);
            mtv<T, true>(lc, X, xr, n2t, n2t);
            col2row<T>(lam, lc, vb, lane);
            // slab: W_k packed upper, λ
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = i; j < 4; ++j)
                    if (j < n2t) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = 16 * i + Tile<T>::row(lane, r), col = 16 * j + (lane & 15);
                            if (row <= col) Sk[col * (col + 1) / 2 + row] = X[up4(i, j)][r];
                        }
                    }
            if (lane < 16) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < n2t) Sk[oM + q.Ps + 16 * j + lane] = lc[j];
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) lam[i][r] = (T)0;
        }
        if (bad && !info) info = k + 1;
    }
    if (lane == 0) kf_info(a.info, t, info, a.kb, a.hfac);
}

// The interior knots of a trajectory structure (n1 = n2 = 16·NT padded, p = 0) with compile-time
// tile counts: F̃ = Wᵀ F in place on the F tiles, C −= F̃ᵀF̃, chol + inverse, λ = Wᵀ(d − F̃ᵀλ).  The
// next knot's F and C tiles (and d) are requested as soon as this knot's copies are dead, so
// their latency runs under the factorisation.
template <typename T, int NT>
__global__ void __launch_bounds__(64 * KF_W, sizeof(T) == 4 ? 2 : 1) kb_factor_mid_kernel(KfArgs<T> a)
{
    extern __shared__ __align__(16) unsigned char kb_lds_raw[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t tl = (int64_t)blockIdx.x * KF_W + wave;
    if (tl >= a.nb) return;
    T *U = (T *)kb_lds_raw + wave * KF_LDS, *vb = U + 64 * KF_LU, *scr = vb + 64;
    const int64_t t = a.b0 + tl;
    const T *imt = a.img + tl * a.IMGT;
    T *St = a.slab + tl * a.sS;
    constexpr int NG = NT * NT, NX = NT * (NT + 1) / 2, PP = 16 * NT;   // X, Cn: up4-packed
    int64_t oI = img_before(a.meta, a.kb, a.fz0, a.fz1), oS = slab_before(a.meta, a.kb);
    acc_t<T> X[10], G[16], Cn[10];
    T lam[4][4], dd[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) lam[i][r] = (T)0;
    {
        const int32_t *m = a.meta + 8 * (a.kb - 1);
        kf_resume<T>(X, lam, St + oS - slab_size(r16(m[1]), r16(m[2])), r16(m[2]), r16(m[1]), NT, lane);
    }
    // the image of an interior knot: F (NT×NT tiles), C (upper), v = d (PP)
    constexpr Im o = {0, 0, NG, NG, NG, 256 * (NG + NX), 256 * (NG + NX) + PP};
    auto fetch = [&](const T *ik) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < NG; ++u) G[u] = gload_tile(ik + 256 * (o.F + u), lane);
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = i; j < NT; ++j) Cn[up4(i, j)] = gload_tile(ik + 256 * (o.C + upn(i, j, NT)), lane);
#pragma unroll
        for (int j = 0; j < NT; ++j) dd[j] = ik[o.v + 16 * j + (lane & 15)];
    };
    fetch(imt + oI);
    int info = 0;
    for (int k = a.kb; k < a.ke; ++k) {
        const int p2 = a.meta[8 * k + 2];
        T *Sk = St + oS;
        oI += img_len(a.meta, k);
        oS += slab_size(0, PP);
        // F̃ = Ã⁻ᵀF (:57) in place, column of tiles by column
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            acc_t<T> Yc[NT];
#pragma unroll
            for (int L = 0; L < NT; ++L) Yc[L] = G[L * NT + j];
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                acc_t<T> g = tzero<T>();
#pragma unroll
                for (int L = 0; L <= i; ++L) g = mtn<T>(X[up4(L, i)], Yc[L], g);
                G[i * NT + j] = g;
            }
        }
        // F̃ᵀλ_{k−1}, then x = d − F̃ᵀλ_{k−1} (column layout)
        T x[4];
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            T sacc = (T)0;
#pragma unroll
            for (int i = 0; i < NT; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) sacc = fma(G[i * NT + j][r], lam[i][r], sacc);
            sacc += __shfl_xor(sacc, 16);
            sacc += __shfl_xor(sacc, 32);
            x[j] = dd[j] - sacc;
        }
        // C − F̃ᵀF̃ (:61) → X
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = i; j < NT; ++j) {
                acc_t<T> c = Cn[up4(i, j)];
#pragma unroll
                for (int L = 0; L < NT; ++L) c = mtn<T, true>(G[L * NT + i], G[L * NT + j], c);
                X[up4(i, j)] = c;
            }
        // G, Cn, dd are dead: knot k+1's tiles land during the factorisation below
        if (k + 1 < a.ke) fetch(imt + oI);
        const int bad = chol_inv_reg<T>(X, NT, p2, U, scr, lane);
        // λ = C̃⁻ᵀ(d − F̃ᵀλ_{k−1}) (:108-116)
        T xr[4][4], lc[4];
        col2row<T>(xr, x, vb, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            T sacc = (T)0;
            if (j < NT) {
#pragma unroll
                for (int i = 0; i <= j; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) sacc = fma(X[up4(i, j)][r], xr[i][r], sacc);
            }
            sacc += __shfl_xor(sacc, 16);
            sacc += __shfl_xor(sacc, 32);
            lc[j] = sacc;
        }
        col2row<T>(lam, lc, vb, lane);
        // slab: W_k packed upper, λ
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = i; j < NT; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * i + Tile<T>::row(lane, r), col = 16 * j + (lane & 15);
                    if (row <= col) Sk[col * (col + 1) / 2 + row] = X[up4(i, j)][r];
                }
        if (lane < 16) {
#pragma unroll
            for (int j = 0; j < NT; ++j) Sk[PP * (PP + 1) / 2 + 16 * j + lane] = lc[j];
        }
        if (bad && !info) info = k + 1;
    }
    if (lane == 0) kf_info(a.info, t, info, a.kb, a.hfac);
}

// ---------------------------------------------------------------- fused interior-knot kernel
// The interior run [kb, ke) of a trajectory structure (p = 0, n1 = n2 padded to 16·NT) with
// BOTH halves of the forward sweep in ONE WAVE PER TRAJECTORY — no Schur image is written or
// read for these knots (the split path's per-knot images and copy_shur!'s read-modify-write
// alias were 2/3 of its HBM traffic).  Step k:
//   * cholesky! + forward_substitution! of knot k (cholesky_solve.jl:47-67, 93-117) on the
//     pivot tiles X = C_k + A_{k+1} − F̃_kᵀF̃_k: X → W_k = C̃_k⁻¹ (kept in LDS), λ_k, the slab;
//   * shur! (jacobian_blocks.jl:231-242) of knot k+1 — F = D2 H⁻¹ D1ᵀ into G, C = D1 H⁻¹ D1ᵀ
//     into Cn, r2 — and of knot k+2's D2 rows only: A = D2 H⁻¹ D2ᵀ accumulated straight into
//     Cn (copy_shur!'s A ≡ previous-C alias, :249-286, in registers) and r1;
//   * F̃_{k+1} = W_kᵀF_{k+1}, x_{k+1} = d_{k+1} − F̃ᵀλ_k, X ← Cn − F̃ᵀF̃ (:57, :61).
// Nothing but G and Cn (26 tiles at NT = 4) is live across the streaming, so fp32 runs at 2
// waves/SIMD; the D2 rows of each knot are streamed twice, one step apart (the second read is
// the cache's).
template <typename T>
struct KuArgs {
    const T *Y, *y, *H, *g;
    T *slab;
    int32_t *info;
    const int32_t *meta;
    int N, kb, ke, hinv, useg, yrel, hfac;
    int64_t b0, nb, sY, sy, sH, sg, sS;
    int64_t *prof;                           // KB_PROF builds: per-phase cycles (else unused)
};
#ifndef KU_PF_SLICES
#define KU_PF_SLICES 0       // 0: per precision (ku_pf)
#endif
#ifndef KU_LEAN
#define KU_LEAN 1            // H⁻¹/g read at use, λ carried in column layout (fewer live registers)
#endif
#ifndef KU_WAVES
#define KU_WAVES 4           // trajectories (waves) per fused workgroup: 4, or 8 (2 per SIMD in one WG)
#endif
#ifndef KU_STAGGER
#define KU_STAGGER 0         // > 0 (with KU_WAVES 8): waves 4–7 start this many s_sleep units late
#endif
#ifndef KU_HG_AHEAD
#define KU_HG_AHEAD 1        // (KU_LEAN) a slice's H⁻¹/g LDS reads issued one stream step ahead:
                             // 1 fp64 only, 2 fp32 as well, 0 off (A/B)
#endif
#ifndef KU_PP
#define KU_PP 1              // H⁻¹/g row areas ping-pong: each step stages only knot k+2's rows (0: A/B)
#endif
#ifndef KU_HGPF
#define KU_HGPF 1            // (KU_PP) knot k+2's H / g loads issued before knot k's factor (0: A/B)
#endif
#ifndef KU_PRIO
#define KU_PRIO 1            // the factor phase (latency-bound chain) runs at raised issue priority
#endif
// waves per fused workgroup: fp64 stays at 4 (one per SIMD: its LDS and registers)
template <typename T> constexpr int ku_w() { return sizeof(T) == 4 ? KU_WAVES : 4; }
// k-slices of Y (of both knots) in flight per wave: fp64 runs one wave per SIMD (512 registers),
// where a third slice fits and gains (stream 86 k → 82 k cycles per knot, profiles/r05/h; fp32's
// 2 waves/SIMD spill with three)
template <typename T> constexpr int ku_pf() { return KU_PF_SLICES ? KU_PF_SLICES : (sizeof(T) == 8 ? 3 : 2); }
constexpr int KU_LDS = KF_LDS;   // per wave: U / W image, vector, 2 H⁻¹|g rows (also the leaf scratch)

// H⁻¹ (or 1) and g of knot q into one of the wave's LDS rows (0 past w); earlier reads of the
// row are ordered before these writes by the wave's in-order LDS (wsync: compiler fence)
template <typename T>
__device__ __forceinline__ void fu_stage_hg(T *hgl, const Kn &q, const T *Ht, const T *gt, int hinv, int useg, int lane)
{
    wsync();
#pragma unroll
    for (int u = 0; u < (KS_HG + 63) / 64; ++u) {
        const int c = lane + 64 * u;
        if (c < KS_HG) {
            const bool in = c < q.w;
            hgl[c] = in ? (hinv ? (T)1 / Ht[q.oH + c] : (T)1) : (T)0;
            hgl[KS_HG + c] = (in && useg) ? gt[q.og + c] : (T)0;
        }
    }
    wsync();
}

// the same rows from values the caller loaded earlier (hv / gv: columns lane + 64u of H and g)
template <typename T>
__device__ __forceinline__ void fu_put_hg(T *hgl, const Kn &q, const T (&hv)[(KS_HG + 63) / 64], const T (&gv)[(KS_HG + 63) / 64],
                                          int hinv, int useg, int lane)
{
    wsync();
#pragma unroll
    for (int u = 0; u < (KS_HG + 63) / 64; ++u) {
        const int c = lane + 64 * u;
        if (c < KS_HG) {
            const bool in = c < q.w;
            hgl[c] = in ? (hinv ? (T)1 / hv[u] : (T)1) : (T)0;
            hgl[KS_HG + c] = (in && useg) ? gv[u] : (T)0;
        }
    }
    wsync();
}

// shur! pieces of two knots in one pass (one k-slice of each per loop step): of knot q1 the F
// tiles (D2 H⁻¹ D1ᵀ, into G) and the C tiles (D1 H⁻¹ D1ᵀ, into P) and r2 = D1 H⁻¹ g; of knot
// q2 = q1 + 1 only the D2 rows: the A tiles (D2 H⁻¹ D2ᵀ) into the SAME P tiles (copy_shur!'s A ≡
// previous-C alias: q1's pivot block needs C_{q1} + A_{q2}) and r1 = D2 H⁻¹ g.  Row blocks
// 0..NT−1 are the D2 rows, NT..2NT−1 the D1 rows (after the p stage rows).  G and P are zeroed
// here; r comes back in column layout (every lane holds r[16v + (lane & 15)]): rv[v] for v ≥ NT
// of q1, for v < NT of q2.  Y is read by raw buffer loads through per-slice descriptors bounded
// by each block's end (columns past w and slices past the last one read 0: nothing past a
// block is read), KU_PF slices in flight.  FULL: whole 16-row blocks and D1 at row 16·NT — the
// row-block offsets are immediates of one VGPR offset; otherwise one range-checked offset per
// row block (rows past a part read 0).
template <typename T, int NT, bool FULL>
__device__ __forceinline__ void fu_schur2(const Kn &q1, const T *Y1, const T *hg1, const Kn &q2, const T *Y2, const T *hg2,
                                          acc_t<T> (&G)[16], acc_t<T> (&P)[10], T (&rv)[2 * NT], int lane)
{
    constexpr int NB = 2 * NT;
    const int i16 = lane & 15, g4 = lane >> 4;
    constexpr uint32_t TS = sizeof(T), OOB = 0x80000000u;
    constexpr int NV1 = FULL ? 1 : NB, NV2 = FULL ? 1 : NT;
    uint32_t vo1[NV1], vo2[NV2];
    if constexpr (FULL) {
        vo1[0] = (uint32_t)((g4 * q1.rows + i16) * (int)TS);
        vo2[0] = (uint32_t)((g4 * q2.rows + i16) * (int)TS);
    } else {
#pragma unroll
        for (int v = 0; v < NB; ++v) {
            const int rb = v < NT ? 16 * v : q1.p1 + q1.ps + 16 * (v - NT);
            const int lim = v < NT ? q1.p1 - 16 * v : q1.p2 - 16 * (v - NT);
            vo1[v] = i16 < lim ? (uint32_t)((g4 * q1.rows + rb + i16) * (int)TS) : OOB;
        }
#pragma unroll
        for (int v = 0; v < NT; ++v)
            vo2[v] = i16 < q2.p1 - 16 * v ? (uint32_t)((g4 * q2.rows + 16 * v + i16) * (int)TS) : OOB;
    }
    if constexpr (!KU_ZERO_PEEL) {
#pragma unroll
        for (int u = 0; u < NT * NT; ++u) G[u] = tzero<T>();
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = i; j < NT; ++j) P[up4(i, j)] = tzero<T>();
    }
    T rp[NB];
#pragma unroll
    for (int v = 0; v < NB; ++v) rp[v] = (T)0;
    const char *yb1 = (const char *)Y1, *yb2 = (const char *)Y2;
    const int yn1 = q1.rows * q1.w * (int)TS, so1 = 4 * q1.rows * (int)TS;
    const int yn2 = q2.rows * q2.w * (int)TS, so2 = 4 * q2.rows * (int)TS;
    const int nks = max(q1.w + 3, q2.w + 3) >> 2;
    constexpr int KU_PF = ku_pf<T>();
    T f1[KU_PF][NB], f2[KU_PF][NT], h1[KU_PF], c1[KU_PF], h2[KU_PF], c2[KU_PF];
    // AHEAD: the step of slice s uses the H⁻¹/g values the previous step read and reads those of
    // slice s + 1, so the LDS round trip is not between a step's start and its first MFMA (rows
    // are KS_HG = KB_WMAX + 4 long; the read index is clamped to the row)
    constexpr bool AHEAD = KU_LEAN && (KU_HG_AHEAD == 2 || (KU_HG_AHEAD == 1 && sizeof(T) == 8));
    T nh1 = (T)0, ng1 = (T)0, nh2 = (T)0, ng2 = (T)0;
    if constexpr (AHEAD) {
        nh1 = hg1[g4];
        ng1 = hg1[KS_HG + g4];
        nh2 = hg2[g4];
        ng2 = hg2[KS_HG + g4];
    }
    auto load = [&](int s, T (&a1)[NB], T (&a2)[NT], T &hh1, T &gg1, T &hh2, T &gg2) __attribute__((always_inline)) {
        const int o1 = s * so1, o2 = s * so2;
        const __amdgpu_buffer_rsrc_t r1 =
            __builtin_amdgcn_make_buffer_rsrc((void *)(yb1 + o1), (short)0, max(yn1 - o1, 0), 0x00020000);
        const __amdgpu_buffer_rsrc_t r2 =
            __builtin_amdgcn_make_buffer_rsrc((void *)(yb2 + o2), (short)0, max(yn2 - o2, 0), 0x00020000);
#pragma unroll
        for (int v = 0; v < NB; ++v)
            a1[v] = bload<T>(r1, FULL ? vo1[0] + (uint32_t)(16 * v * (int)TS) : vo1[FULL ? 0 : v], 0u);
#pragma unroll
        for (int v = 0; v < NT; ++v)
            a2[v] = bload<T>(r2, FULL ? vo2[0] + (uint32_t)(16 * v * (int)TS) : vo2[FULL ? 0 : v], 0u);
        if constexpr (!KU_LEAN) {
            hh1 = hg1[4 * s + g4];
            gg1 = hg1[KS_HG + 4 * s + g4];
            hh2 = hg2[4 * s + g4];
            gg2 = hg2[KS_HG + 4 * s + g4];
        }
    };
    // FIRST (std::true_type, KU_ZERO_PEEL): the stream's first slice — the accumulators start from
    // a zero C operand (an MFMA inline constant) instead of 26 zeroed tiles
    auto step = [&](auto first, const T (&a1)[NB], const T (&a2)[NT], T hh1, T gg1, T hh2, T gg2, int s)
        __attribute__((always_inline)) {
        constexpr bool F0 = decltype(first)::value;
        if constexpr (AHEAD) {
            hh1 = nh1;
            gg1 = ng1;
            hh2 = nh2;
            gg2 = ng2;
            const int sn = min(s + 1, KS_HG / 4 - 1);      // (a slice past the last step: unused)
            nh1 = hg1[4 * sn + g4];
            ng1 = hg1[KS_HG + 4 * sn + g4];
            nh2 = hg2[4 * sn + g4];
            ng2 = hg2[KS_HG + 4 * sn + g4];
        } else if constexpr (KU_LEAN) {      // H⁻¹, g of the slice straight from LDS (no ring registers)
            hh1 = hg1[4 * s + g4];
            gg1 = hg1[KS_HG + 4 * s + g4];
            hh2 = hg2[4 * s + g4];
            gg2 = hg2[KS_HG + 4 * s + g4];
        }
        T fh1[NB], fh2[NT];
#pragma unroll
        for (int v = NT; v < NB; ++v) fh1[v] = a1[v] * hh1;
#pragma unroll
        for (int v = 0; v < NT; ++v) fh2[v] = a2[v] * hh2;
#ifndef KU_ABL_MM
#define KU_ABL_MM 0          // timing ablations only (wrong results): 1 no F (G) products, 2 no C / A
#endif
        if constexpr (KU_ABL_MM != 1) {
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
                G[i * NT + j] = Tile<T>::mma(a1[i], fh1[NT + j], F0 ? tzero<T>() : G[i * NT + j]);
        }
        if constexpr (KU_ABL_MM != 2) {
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = i; j < NT; ++j)
                P[up4(i, j)] = Tile<T>::mma(a1[NT + i], fh1[NT + j], F0 ? tzero<T>() : P[up4(i, j)]);
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = i; j < NT; ++j) P[up4(i, j)] = Tile<T>::mma(a2[i], fh2[j], P[up4(i, j)]);
        }
#pragma unroll
        for (int v = NT; v < NB; ++v) rp[v] = fma(fh1[v], gg1, rp[v]);
#pragma unroll
        for (int v = 0; v < NT; ++v) rp[v] = fma(fh2[v], gg2, rp[v]);
    };
#pragma unroll
    for (int u = 0; u < KU_PF; ++u) load(u, f1[u], f2[u], h1[u], c1[u], h2[u], c2[u]);
    // branch-free ring (slices past a block's last read 0 and carry h = 0): each step waits
    // only for its own slice, requested KU_PF steps earlier
    int s00 = 0;
    if constexpr (KU_ZERO_PEEL) {            // the first group of KU_PF slices, peeled
        step(std::true_type{}, f1[0], f2[0], h1[0], c1[0], h2[0], c2[0], 0);
        load(KU_PF, f1[0], f2[0], h1[0], c1[0], h2[0], c2[0]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 1; u < KU_PF; ++u) {
            step(std::false_type{}, f1[u], f2[u], h1[u], c1[u], h2[u], c2[u], u);
            load(u + KU_PF, f1[u], f2[u], h1[u], c1[u], h2[u], c2[u]);
            __builtin_amdgcn_sched_barrier(0);
        }
        s00 = KU_PF;
    }
    for (int s0 = s00; s0 < nks; s0 += KU_PF) {
#pragma unroll
        for (int u = 0; u < KU_PF; ++u) {
            step(std::false_type{}, f1[u], f2[u], h1[u], c1[u], h2[u], c2[u], s0 + u);
            load(s0 + u + KU_PF, f1[u], f2[u], h1[u], c1[u], h2[u], c2[u]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int v = 0; v < NB; ++v) {
        T x = rp[v];
        x += __shfl_xor(x, 16);
        x += __shfl_xor(x, 32);
        rv[v] = x;
    }
}

// F̃ = Wᵀ G in place (:57; W's upper tiles from the wave's LDS image, column-major with
// leading dimension KF_LU, each read once: block rows i from the bottom, so G[L] for L ≤ i is
// still F when row i is formed), x = xn − F̃ᵀλ (column layout), P ← P − F̃ᵀF̃ (:61)
template <typename T, int NT>
__device__ __forceinline__ void fu_reduce(acc_t<T> (&P)[10], acc_t<T> (&G)[16], const T *Wl, const T (&lam)[4][4],
                                          const T (&xn)[4], T (&x)[4], int lane)
{
    (void)lane;
#pragma unroll
    for (int i = NT - 1; i >= 0; --i) {
        acc_t<T> acc[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = tzero<T>();
#pragma unroll
        for (int L = 0; L <= i; ++L) {
            const acc_t<T> w = tload(Wl + 16 * L + 16 * i * KF_LU, KF_LU, lane);
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[j] = mtn<T>(w, G[L * NT + j], acc[j]);
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) G[i * NT + j] = acc[j];
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        T sacc = (T)0;
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) sacc = fma(G[i * NT + j][r], lam[i][r], sacc);
        sacc += __shfl_xor(sacc, 16);
        sacc += __shfl_xor(sacc, 32);
        x[j] = xn[j] - sacc;
    }
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = i; j < NT; ++j) {
#pragma unroll
            for (int L = 0; L < NT; ++L) P[up4(i, j)] = mtn<T, true>(G[L * NT + i], G[L * NT + j], P[up4(i, j)]);
        }
}

// shur! of knot kn (F, C, r2 → xn = r2 − y) and the D2 part of knot kn+1 (A into P, r1 added
// to xn: d_kn = r2 − y + r1 of the next knot, as the image's v)
template <typename T, int NT, bool FULL>
__device__ __forceinline__ void fu_stream(const int32_t *meta, int kn, const T *Yt, const T *yt, const T *Ht, const T *gt,
                                          int hinv, int useg, T *h1, T *h2, bool stage1, acc_t<T> (&G)[16],
                                          acc_t<T> (&P)[10], T (&xn)[4], int lane,
                                          const T (*hv)[(KS_HG + 63) / 64] = nullptr, const T (*gv)[(KS_HG + 63) / 64] = nullptr)
{
    const Kn q1 = kn_load(meta, kn), q2 = kn_load(meta, kn + 1);
    T rv[2 * NT];
    if (stage1) fu_stage_hg<T>(h1, q1, Ht, gt, hinv, useg, lane);
    if (hv) fu_put_hg<T>(h2, q2, *hv, *gv, hinv, useg, lane);      // q2's H / g loaded before the factor
    else fu_stage_hg<T>(h2, q2, Ht, gt, hinv, useg, lane);
    fu_schur2<T, NT, FULL>(q1, Yt + q1.oY, h1, q2, Yt + q2.oY, h2, G, P, rv, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int e = 16 * j + (lane & 15);
        xn[j] = (j < NT && e < q1.p2) ? (rv[NT + j] - yt[q1.oy + e]) + rv[j] : (T)0;
    }
}

template <typename T, int NT, bool FULL>
__global__ void __launch_bounds__(64 * ku_w<T>(), sizeof(T) == 4 ? 8 / ku_w<T>() : 1) kb_fuse_mid_kernel(KuArgs<T> a)
{
    extern __shared__ __align__(16) unsigned char kb_lds_raw[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int KU_W = ku_w<T>();
    const int64_t tl = (int64_t)blockIdx.x * KU_W + wave;
    if (tl >= a.nb) return;                          // whole wave; no workgroup barriers below
    if constexpr (KU_W == 8 && KU_STAGGER > 0) {
        // the two waves sharing a SIMD (w, w + 4) run the same program; offset them so that
        // one's MFMA-dense streaming overlaps the other's latency-bound factorisation
        if (wave >= 4)
            for (int i = 0; i < KU_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
    }
    T *U = (T *)kb_lds_raw + wave * KU_LDS, *vb = U + 64 * KF_LU, *hgl = vb + 64;
    const int64_t t = a.b0 + tl, ty = a.yrel ? tl : t;
    const T *Yt = a.Y + ty * a.sY, *yt = a.y + t * a.sy, *Ht = a.H + t * a.sH, *gt = a.g + ty * a.sg;
    T *St = a.slab + tl * a.sS;
    constexpr int PP = 16 * NT;
    int64_t oS = slab_before(a.meta, a.kb);
    acc_t<T> G[16], P[10];                           // P: pivot tiles; W_k after the factor
    T lam[4][4], x[4], xn[4], lcol[4];               // λ in row layout, or (KU_LEAN) column layout
    {
        // the state at kb − 1 (W_{kb−1}, λ_{kb−1}, left in the slab by the general kernel)
        // into the LDS W image the reduction reads
        const int32_t *m = a.meta + 8 * (a.kb - 1);
        kf_resume<T>(P, lam, St + oS - slab_size(r16(m[1]), r16(m[2])), r16(m[2]), r16(m[1]), NT, lane);
        if constexpr (KU_LEAN) {
            const T *Sk = St + oS - slab_size(r16(m[1]), r16(m[2]));
            const int P2 = r16(m[2]), Ps = r16(m[1]);
            const int oM = P2 * (P2 + 1) / 2 + Ps * (Ps + 1) / 2 + Ps * P2;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int e = 16 * j + (lane & 15);
                lcol[j] = e < P2 ? Sk[oM + Ps + e] : (T)0;
            }
        }
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = i; j < NT; ++j) tstore(U + 16 * i + 16 * j * KF_LU, KF_LU, P[up4(i, j)], lane);
    }
    // prologue: knot kb's F, C, d and knot kb+1's A; then F̃_kb, x_kb, P = C_kb + A_{kb+1} − F̃ᵀF̃
    // H⁻¹/g rows: knot k+1's were staged by the previous stream (as its q2) — KU_PP: the two row
    // areas ping-pong (hcur: knot k+1's rows, kept through the factor; hoth: the leaf scratch, then
    // knot k+2's rows) instead of re-staging both knots every step
    T *hcur = hgl + 2 * KS_HG, *hoth = hgl;
    fu_stream<T, NT, FULL>(a.meta, a.kb, Yt, yt, Ht, gt, a.hinv, a.useg, hgl, hgl + 2 * KS_HG, true, G, P, xn, lane);
    wsync();
    if constexpr (KU_LEAN) col2row<T>(lam, lcol, vb, lane);
    fu_reduce<T, NT>(P, G, U, lam, xn, x, lane);
    int info = 0;
#ifdef KB_PROF
    int64_t kb_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    KB_T0();
#endif
    constexpr bool HGPF = KU_PP && KU_HGPF;
    constexpr int NHG = (KS_HG + 63) / 64;
    for (int k = a.kb; k < a.ke; ++k) {
        const int p2 = a.meta[8 * k + 2];
        // HGPF: knot k+2's H and g requested before the factor (they land under it; the stream
        // after it only forms H⁻¹ and writes the LDS rows)
        T hv[NHG], gv[NHG];
        if constexpr (HGPF) {
            if (k + 1 < a.ke) {
                const Kn q2 = kn_load(a.meta, k + 2);
#pragma unroll
                for (int u = 0; u < NHG; ++u) {
                    const int c = lane + 64 * u;
                    const bool in = c < q2.w;
                    hv[u] = (in && a.hinv) ? Ht[q2.oH + c] : (T)1;
                    gv[u] = (in && a.useg) ? gt[q2.og + c] : (T)0;
                }
            }
        }
        // C̃_k = chol(P) → P = W_k (:61-62)
        if constexpr (KU_PRIO) __builtin_amdgcn_s_setprio(2);
#ifdef KU_NOCHOL
        const int bad = 0;         // timing ablation only: no factorisation (wrong results)
        (void)p2;
#else
#ifdef KB_PROF
        const int bad = chol_inv_reg<T>(P, NT, p2, U, KU_PP ? hoth : hgl, lane, kb_acc + 4);
#else
        const int bad = chol_inv_reg<T>(P, NT, p2, U, KU_PP ? hoth : hgl, lane);
#endif
#endif
        KB_T(0);
        // λ_k = W_kᵀ x_k (:108-116)
        T xr[4][4], lc[4];
        col2row<T>(xr, x, vb, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            T sacc = (T)0;
            if (j < NT) {
#pragma unroll
                for (int i = 0; i <= j; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) sacc = fma(P[up4(i, j)][r], xr[i][r], sacc);
            }
            sacc += __shfl_xor(sacc, 16);
            sacc += __shfl_xor(sacc, 32);
            lc[j] = sacc;
        }
        if constexpr (KU_LEAN) {
#pragma unroll
            for (int j = 0; j < 4; ++j) lcol[j] = lc[j];
        } else {
            col2row<T>(lam, lc, vb, lane);
        }
        // slab: W_k packed upper (column col at col(col+1)/2: the off-diagonal tiles store
        // unpredicated at a per-lane column base plus immediates; only the diagonal tiles test
        // row ≤ col, the same four lane masks for every tile), λ_k
        T *Sk = St + oS;
        oS += slab_size(0, PP);
        {
            const int c = lane & 15;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                T *cb = Sk + (16 * j + c) * (16 * j + c + 1) / 2;
#pragma unroll
                for (int i = 0; i < j; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) cb[16 * i + Tile<T>::row(lane, r)] = P[up4(i, j)][r];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (Tile<T>::row(lane, r) <= c) cb[16 * j + Tile<T>::row(lane, r)] = P[up4(j, j)][r];
            }
        }
        if (lane < 16) {
#pragma unroll
            for (int j = 0; j < NT; ++j) Sk[PP * (PP + 1) / 2 + 16 * j + lane] = lc[j];
        }
        if (bad && !info) info = k + 1;
        if constexpr (KU_PRIO) __builtin_amdgcn_s_setprio(0);
        KB_T(1);
        if (k + 1 < a.ke) {
            // W_k to the LDS image (chol_inv_reg's scratch is free again): no tile is live
            // across the streaming but G and P (zeroed there)
            wsync();
#pragma unroll
            for (int i = 0; i < NT; ++i)
#pragma unroll
                for (int j = i; j < NT; ++j) tstore(U + 16 * i + 16 * j * KF_LU, KF_LU, P[up4(i, j)], lane);
            if constexpr (KU_PP) {
                fu_stream<T, NT, FULL>(a.meta, k + 1, Yt, yt, Ht, gt, a.hinv, a.useg, hcur, hoth, false, G, P, xn, lane,
                                       HGPF ? &hv : nullptr, HGPF ? &gv : nullptr);
                T *const h = hcur;
                hcur = hoth;
                hoth = h;
            } else {
                fu_stream<T, NT, FULL>(a.meta, k + 1, Yt, yt, Ht, gt, a.hinv, a.useg, hgl, hgl + 2 * KS_HG, true, G, P,
                                       xn, lane);
            }
            wsync();
            KB_T(2);
            if constexpr (KU_LEAN) col2row<T>(lam, lcol, vb, lane);
            fu_reduce<T, NT>(P, G, U, lam, xn, x, lane);
            KB_T(3);
        }
    }
    KB_FLUSH();
    if (lane == 0) kf_info(a.info, t, info, a.kb, a.hfac);
}

// ---------------------------------------------------------------- backward sweep (split path)
// backward_substitution! (cholesky_solve.jl:119-143) fused with calculate_primals!
// (cholesky_solver.jl:185-236), one wave per trajectory — the same operations as
// kkt_big_bwd_kernel without its workgroup barriers and LDS staging of Y: every GEMV over Y_j
// reads HBM/L2 directly, lane = column for Yᵀ-products (t, D2ᵀλ: each lane a contiguous run
// of its column) and lane = row for Y-products (v: coalesced columns); the multipliers pass
// between lanes through a small per-wave LDS vector area.  Bound by the bytes of Y (read
// once per knot; the D2 rows a second time, from L2).
// per-wave LDS: vectors x (128), t (128), v, z (= e), λ (64 each), then the packed W image
// (≤ 64×65/2).  2528 elements: four waves per 40 KB (fp32) workgroup, 4 workgroups (16 waves)
// per CU; fp64 2 workgroups per CU.  (At 2656 elements LDS held fp32 to 12 waves per CU —
// configs[4]'s 8192 waves took 3 rounds instead of 2 — and fp64 to 4.)
constexpr int KBW_V = 7 * 64;
constexpr int KBW_W = 2080;
#ifndef KBW_VC_COLS
#define KBW_VC_COLS 16
#endif
#ifndef KBW_RUN
#define KBW_RUN 32
#endif
// D2 columns the backward kernel holds in registers between its two uses (fp32 96, fp64 32:
// wider knots hold their first columns and read the rest twice; 2 = off, the array is then a
// dummy).  KBW_NOHOLD=1 restores the second pass over every D2 column (A/B).
#ifndef KBW_NOHOLD
#define KBW_NOHOLD 0
#endif
__device__ __forceinline__ float rdlane(float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l)); }
__device__ __forceinline__ double rdlane(double v, int l)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
#ifndef KBW_HOLD64
#define KBW_HOLD64 32        // fp64 D2 columns held (A/B: 64, 96 take the kernel to one wave per SIMD)
#endif
template <typename T> constexpr int kbw_hold() { return KBW_NOHOLD ? 2 : sizeof(T) == 4 ? 96 : KBW_HOLD64; }
constexpr int KBW_VC = KBW_VC_COLS;  // columns of Y in flight per lane in the v product
constexpr int KBW_R = KBW_RUN;       // column-run elements in flight per lane (t, D2ᵀλ)

// Σ_{r<n} p[r]·x[r] for a contiguous run p (global) and x (LDS, broadcast reads), n ≤ 128:
// every load of a 32-element chunk issued before its FMAs (16-B vector loads when `vec`)
template <typename T>
__device__ __forceinline__ T dot_run(const T *p, const T *x, int n, bool vec)
{
    constexpr int V = 16 / sizeof(T);
    typedef T tv __attribute__((ext_vector_type(V)));
    T s0 = (T)0, s1 = (T)0;
    for (int r0 = 0; r0 < n; r0 += KBW_R) {
        T y[KBW_R];
        if (vec && r0 + KBW_R <= n) {
#pragma unroll
            for (int j = 0; j < KBW_R / V; ++j) {
                const tv w = *(const tv *)(p + r0 + V * j);
#pragma unroll
                for (int e = 0; e < V; ++e) y[V * j + e] = w[e];
            }
        } else {
#pragma unroll
            for (int j = 0; j < KBW_R; ++j) y[j] = r0 + j < n ? p[r0 + j] : (T)0;
        }
        // x past n is not data (stale LDS, possibly NaN): never multiply it, even by 0
        if (r0 + KBW_R <= n) {
#pragma unroll
            for (int j = 0; j < KBW_R; j += 2) {
                s0 = fma(y[j], x[r0 + j], s0);
                s1 = fma(y[j + 1], x[r0 + j + 1], s1);
            }
        } else {
#pragma unroll
            for (int j = 0; j < KBW_R; ++j)
                if (r0 + j < n) s0 = fma(y[j], x[r0 + j], s0);
        }
    }
    return s0 + s1;
}

template <typename T>
__global__ void __launch_bounds__(64 * KF_W) kb_bwd_kernel(KbArgs<T> a, int64_t nb)
{
    extern __shared__ __align__(16) unsigned char kb_lds_raw[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t tl = (int64_t)blockIdx.x * KF_W + wave;
    if (tl >= nb) return;
    constexpr int V = 16 / sizeof(T);
    T *xb = (T *)kb_lds_raw + wave * (KBW_V + KBW_W);  // x = [μ_j; λ_j] in Y's row order past D2
    // eb (μ − Ẽλ) reuses zb: z is dead once λ = W z is formed (a wave barrier between)
    T *tb = xb + 128, *vb = tb + 128, *zb = vb + 64, *lb = zb + 64, *eb = zb, *wl = xb + KBW_V;
    const int64_t t = a.b0 + tl, ty = a.yrel ? tl : t;
    const T *Yt = a.Y + ty * a.sY, *Ht = a.H + t * a.sH, *gt = a.g + ty * a.sg;
    T *dzt = a.dz + t * a.sg, *lat = a.lam + t * a.sy;
    const T *Ut = a.hfac ? a.Ui + tl * a.sU : nullptr;
    const T *St = a.slab + tl * a.sS;
    const int N = a.N;
    int64_t oS = 0, oU = 0;
    for (int k = 0; k < N; ++k) {
        const int32_t *m = a.meta + 8 * k;
        oS += slab_size(r16(m[1]), r16(m[2]));
        if (a.hfac) oU += (int64_t)m[3] * (m[3] + 1) / 2;
    }
    // out_i = Σ_{c ≥ i} P[c(c+1)/2 + i]·x[c] for packed upper P (row dots), lane = row
    auto rowdot = [&](const T *P, const T *x, int n) __attribute__((always_inline)) {
        T s0 = (T)0, s1 = (T)0;
        if (lane < n) {
            int c = lane;
            for (; c + 1 < n; c += 2) {
                s0 = fma(P[c * (c + 1) / 2 + lane], x[c], s0);
                s1 = fma(P[(c + 1) * (c + 2) / 2 + lane], x[c + 1], s1);
            }
            if (c < n) s0 = fma(P[c * (c + 1) / 2 + lane], x[c], s0);
        }
        return s0 + s1;
    };
    // terminal knot (:139-143): μ_N = −B̃⁻¹μ, λ_N as the forward sweep left it
    Kn qj = kn_load(a.meta, N - 1);
    oS -= slab_size(qj.Ps, qj.P2);
    {
        const T *Sk = St + oS;
        const int nW = qj.P2 * (qj.P2 + 1) / 2, nBv = qj.Ps * (qj.Ps + 1) / 2, nE = qj.Ps * qj.P2;
        const T *fm = Sk + nW + nBv + nE, *fl = fm + qj.Ps;
        const T nm = rowdot(Sk + nW, fm, qj.ps);
        const T xm = -nm, xl = lane < qj.p2 ? fl[lane] : (T)0;
        if (lane < qj.ps) {
            xb[lane] = xm;
            lat[qj.oy + lane] = xm;
        }
        if (lane < qj.p2) {
            xb[qj.ps + lane] = xl;
            lat[qj.oy + qj.ps + lane] = xl;
        }
    }
    wsync();
    const bool ybase16 = ((uintptr_t)Yt % 16) == 0;
    for (int j = N - 1; j >= 0; --j) {
        const T *Yk = Yt + qj.oY;
        const int nr = qj.rows - qj.p1;
        // 16-B loads of column runs need every column start 16-B aligned
        const bool vt = ybase16 && (qj.oY % V) == 0 && (qj.rows % V) == 0 && (qj.p1 % V) == 0;
        const bool vs = ybase16 && (qj.oY % V) == 0 && (qj.rows % V) == 0;
        T hraw[2], graw[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = lane + 64 * u;
            hraw[u] = (c < qj.w && a.ginv && !a.hfac) ? Ht[qj.oH + c] : (T)1;
            graw[u] = (c < qj.w && a.ginv) ? gt[qj.og + c] : (T)0;
        }
        // t = [C; D1]ᵀ[μ_j; λ_j] (calc_residual!'s Cᵀμ + D1ᵀλ, :219-231), lane = column
        T tc[2], hc[2], tbv[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = lane + 64 * u;
            T tt = (T)0, h = (T)0;
            if (c < qj.w) {
                tt = dot_run<T>(Yk + (int64_t)c * qj.rows + qj.p1, xb, nr, vt);
                h = (a.ginv && !a.hfac) ? (T)1 / hraw[u] : (T)1;
                tb[c] = tt * h;
            } else {
                tb[c] = (T)0;
            }
            tbv[u] = c < qj.w ? tt * h : (T)0;          // column c's t·h in lane c (held-D2 path)
            tc[u] = tt;
            hc[u] = h;
        }
        wsync();
        // fp32, w ≤ KBW_HOLD: knot j's D2 rows stay in registers (lane = row) from the v product
        // to D2ᵀλ_{j−1}, so D2 is read once per knot instead of twice
        T d2[kbw_hold<T>()];
        constexpr int KH = kbw_hold<T>();
        const bool hold = KH > 2;                  // columns [0, min(w, KH)) held
        Kn qp = qj;
        if (j > 0) {
            qp = kn_load(a.meta, j - 1);
            oS -= slab_size(qp.Ps, qp.P2);
            const T *Sk = St + oS;
            const int nW = qp.P2 * (qp.P2 + 1) / 2, nBv = qp.Ps * (qp.Ps + 1) / 2, nE = qp.Ps * qp.P2;
            const T *Bl = Sk + nW, *El = Bl + nBv, *fm = El + nE, *fl = fm + qp.Ps;
            // W_{j−1} (packed) → LDS, all loads in flight at once
            {
                const int nv = nW / V;
                const bool wv = ((uintptr_t)Sk % 16) == 0;
                if (wv) {
                    typedef T tv __attribute__((ext_vector_type(V)));
                    for (int e0 = 0; e0 < nv; e0 += 64 * 8) {
                        tv w8[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            const int e = e0 + lane + 64 * u;
                            if (e < nv) w8[u] = *(const tv *)(Sk + V * e);
                        }
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            const int e = e0 + lane + 64 * u;
                            if (e < nv) *(tv *)(wl + V * e) = w8[u];
                        }
                    }
                    for (int e = V * nv + lane; e < nW; e += 64) wl[e] = Sk[e];
                } else {
                    for (int e = lane; e < nW; e += 64) wl[e] = Sk[e];
                }
            }
            // v = D2 H⁻¹ t = D_{k+1}μ_{k+1} + F_{k+1}λ_{k+1}, lane = row (coalesced columns, 16 in flight)
            if (hold) {
                // every D2 column in flight at once, and kept in registers for D2ᵀλ_{j−1} below
                // (the second pass over D2 was ~30 % of this kernel's fabric traffic)
                const int rl = lane < qj.p1 ? lane : 0;
                const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
                    (void *)Yk, (short)0, (int)(qj.rows * qj.w * sizeof(T)), 0x00020000);
                __builtin_amdgcn_sched_barrier(0);       // not hoisted over the W staging above
#pragma unroll
                for (int c = 0; c < kbw_hold<T>(); ++c)      // uniform column offset in soffset
                    d2[c] = bload<T>(yrs, (uint32_t)rl * sizeof(T), (uint32_t)((c < qj.w ? c : 0) * qj.rows * sizeof(T)));
                T s0 = (T)0, s1 = (T)0;
#pragma unroll
                for (int c = 0; c < kbw_hold<T>(); c += 2) {  // tbv is 0 past w (set above)
                    s0 = fma(d2[c], rdlane(tbv[c >> 6], c & 63), s0);
                    s1 = fma(d2[c + 1], rdlane(tbv[(c + 1) >> 6], (c + 1) & 63), s1);
                }
                for (int c0 = KH; c0 < qj.w; c0 += KBW_VC) {    // columns past the held ones
                    T y[KBW_VC];
#pragma unroll
                    for (int u = 0; u < KBW_VC; ++u) y[u] = c0 + u < qj.w ? Yk[rl + (int64_t)(c0 + u) * qj.rows] : (T)0;
#pragma unroll
                    for (int u = 0; u < KBW_VC; ++u)
                        if (c0 + u < qj.w) s0 = fma(y[u], tb[c0 + u], s0);
                }
                vb[lane] = lane < qj.p1 ? s0 + s1 : (T)0;
            } else {
                T s0 = (T)0, s1 = (T)0;
                const int rl = lane < qj.p1 ? lane : 0;
                for (int c0 = 0; c0 < qj.w; c0 += KBW_VC) {
                    T y[KBW_VC];
#pragma unroll
                    for (int u = 0; u < KBW_VC; ++u) y[u] = c0 + u < qj.w ? Yk[rl + (int64_t)(c0 + u) * qj.rows] : (T)0;
                    if (c0 + KBW_VC <= qj.w) {
#pragma unroll
                        for (int u = 0; u < KBW_VC; u += 2) {
                            s0 = fma(y[u], tb[c0 + u], s0);
                            s1 = fma(y[u + 1], tb[c0 + u + 1], s1);
                        }
                    } else {
#pragma unroll
                        for (int u = 0; u < KBW_VC; ++u)
                            if (c0 + u < qj.w) s0 = fma(y[u], tb[c0 + u], s0);
                    }
                }
                vb[lane] = lane < qj.p1 ? s0 + s1 : (T)0;
            }
            wsync();
            // λ_{j−1} = C̃⁻¹(λ + C̃⁻ᵀv) = W(λ + Wᵀv)  (:128-135): z = fl + Wᵀv (lane = column)
            {
                T s0 = (T)0, s1 = (T)0;
                if (lane < qp.P2) {
                    const T *wc = wl + lane * (lane + 1) / 2;
                    int i = 0;
                    for (; i + 1 <= lane; i += 2) {
                        s0 = fma(wc[i], vb[i], s0);
                        s1 = fma(wc[i + 1], vb[i + 1], s1);
                    }
                    if (i <= lane) s0 = fma(wc[i], vb[i], s0);
                    zb[lane] = fl[lane] + (s0 + s1);
                }
            }
            wsync();
            const T nl = rowdot(wl, zb, qp.P2);
            lb[lane] = nl;
            T nm = (T)0;
            if (qp.ps) {
                // μ_{j−1} = B̃⁻¹(μ − Ẽλ)  (:136-137)
                wsync();
                T s = (T)0;
                if (lane < qp.Ps)
                    for (int c = 0; c < qp.P2; ++c) s = fma(El[lane + c * qp.Ps], lb[c], s);
                eb[lane] = lane < qp.Ps ? fm[lane] - s : (T)0;
                wsync();
                nm = rowdot(Bl, eb, qp.Ps);
            }
            wsync();
            // negate (:138) and hand over: x = [μ_{j−1}; λ_{j−1}] for knot j−1
            if (lane < qp.ps) {
                xb[lane] = -nm;
                lat[qp.oy + lane] = -nm;
            }
            if (lane < qp.p2) {
                xb[qp.ps + lane] = -nl;
                lat[qp.oy + qp.ps + lane] = -nl;
            }
            lb[lane] = -nl;
            wsync();
        }
        if (hold && j > 0) {
            // D2ᵀλ_{j−1} from the held rows: per-lane products, column sums by a 16-column LDS
            // transpose (row stride 17: conflict-free both ways) and two lane exchanges; the sums
            // land in tb (dead since the v product).  W_{j−1} (wl) is dead once λ_{j−1} is formed.
            const T lr = lane < qj.p1 ? lb[lane] : (T)0;
            T *red = wl;
            const int cc = lane & 15, q4 = lane >> 4;
#pragma unroll
            for (int c0 = 0; c0 < kbw_hold<T>(); c0 += 16) {
                if (c0 < qj.w) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) red[lane * 17 + i] = d2[c0 + i] * lr;
                    wsync();
                    T s0 = (T)0, s1 = (T)0;
#pragma unroll
                    for (int i = 0; i < 16; i += 2) {
                        s0 += red[(q4 * 16 + i) * 17 + cc];
                        s1 += red[(q4 * 16 + i + 1) * 17 + cc];
                    }
                    T s = s0 + s1;
                    s += __shfl_xor(s, 16);
                    s += __shfl_xor(s, 32);
                    wsync();
                    if (lane < 16) tb[c0 + lane] = s;
                }
            }
            wsync();
        }
        // δz_j = −H⁻¹(t + D2ᵀλ_{j−1} + g)  (calc_residual! + calc_primals!, :195-236), lane = column
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = lane + 64 * u;
            if (c < qj.w) {
                const T sd = j > 0 ? ((hold && c < KH) ? tb[c] : dot_run<T>(Yk + (int64_t)c * qj.rows, lb, qj.p1, vs)) : (T)0;
                const T res = tc[u] + sd + graw[u];
                if (a.hfac) tb[c] = res;
                else dzt[qj.og + c] = -(res * hc[u]);
            }
        }
        if (a.hfac) {
            // δz = −U⁻¹ res (res already U⁻ᵀ-applied), row dots on the packed U⁻¹
            wsync();
            oU -= (int64_t)qj.w * (qj.w + 1) / 2;
            const T *Uk = Ut + oU;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int i = lane + 64 * u;
                if (i < qj.w) {
                    T s = (T)0;
                    for (int c = i; c < qj.w; ++c) s = fma(Uk[c * (c + 1) / 2 + i], tb[c], s);
                    dzt[qj.og + i] = -s;
                }
            }
        }
        wsync();
        qj = qp;
    }
}

// ---------------------------------------------------------------- host: plan and launch
struct KbPlan {
    int PM, LD, LDY, LDB, maxrows, maxw, blk;
    int64_t S;                      // slab elements per trajectory
    bool hfac;                      // dense / block-diagonal H with ginv: the hfac pre-pass
    int LDH, nh;                    // its LDS leading dimension and size (elements)
    int64_t sU;                     // packed U⁻¹ elements per trajectory
    int oWp, oBlk, oSl, oV, nf;     // fwd LDS (elements)
    int oYl, oWl, oV2, nb;          // bwd LDS (elements)
    bool split;                     // the split forward sweep (Schur kernel + factor kernel)
    int64_t IMGT;                   // split: image elements per trajectory
    int nruns;                      // split: Schur units per trajectory
    int nbt;                        // split: the Schur kernel's block grid (max R / 16)
    int mid0, mid1, midnt;          // split: knots [mid0, mid1) run on kb_factor_mid_kernel<midnt>
    bool fuse;                      // … or on kb_fuse_mid_kernel<midnt> (no Schur images there)
    bool midfull;                   // fused: n2 of the run a multiple of 16 (whole row blocks)
    int nr0;                        // Schur runs over knots [0, mid0) (fused) or all runs
};

// LQRX_KKT_MID=0 keeps the interior knots on the general factor kernel (A/B checks)
int kb_mid_env()
{
    static const int v = [] { const char *e = std::getenv("LQRX_KKT_MID"); return e && *e ? std::atoi(e) : 1; }();
    return v;
}
// LQRX_KKT_FUSE=0 runs the interior knots as Schur kernel + kb_factor_mid_kernel (A/B checks)
int kb_fuse_env()
{
    static const int v = [] { const char *e = std::getenv("LQRX_KKT_FUSE"); return e && *e ? std::atoi(e) : 1; }();
    return v;
}
// LQRX_KKT_SPLIT=0 keeps every structure on the fused forward kernel (A/B checks)
int kb_split_env()
{
    static const int v = [] { const char *e = std::getenv("LQRX_KKT_SPLIT"); return e && *e ? std::atoi(e) : 1; }();
    return v;
}

// the big kernels' block limits and LDS plan for this structure; false = not served
bool kb_plan(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2, const int32_t *w, int tsize,
             KbPlan &P)
{
    if (a.layout != 0 || a.N < 1) return false;
    P.hfac = a.ginv && a.h_mode != 2;
    int PM = 16, RM = 16, maxrows = 1, maxw = 1, PMW = 0;
    int64_t S = 0, sU = 0;
    for (int k = 0; k < a.N; ++k) {
        if (n1[k] > KB_PMAX || p[k] > KB_PMAX || n2[k] > KB_PMAX || w[k] > KB_WMAX) return false;
        const int P1 = r16(n1[k]), Ps = r16(p[k]), P2 = r16(n2[k]), R = P1 + Ps + P2;
        if (R > KB_RMAX) return false;
        PM = std::max(PM, std::max(P1, std::max(Ps, P2)));
        RM = std::max(RM, R);
        maxrows = std::max(maxrows, n1[k] + p[k] + n2[k]);
        maxw = std::max(maxw, w[k]);
        PMW = std::max(PMW, P2);
        S += slab_size(Ps, P2);
        sU += (int64_t)w[k] * (w[k] + 1) / 2;
    }
    // bank-conflict pads (MI355X LDS: 64 banks × 4 B): tile operands read as (lane·ld + group)
    P.PM = PM;
    P.LD = PM + 4;
    P.LDY = KB_LDY;
    P.LDB = maxrows | 1;
    P.maxrows = maxrows;
    P.maxw = maxw;
    int blk = 0;
    for (int k = 0; k < a.N; ++k) blk = std::max(blk, blk_off(r16(n1[k]), r16(p[k]), r16(n2[k]), P.LD).end);
    P.blk = blk;
    P.S = S;
    int o = 0;
    P.oWp = o; o += P.LD * PM;
    P.oBlk = o; o += blk;
    P.oSl = o;                              // (the forward sweep reads Y straight from HBM)
    o = (o + 3) & ~3;
    P.oV = o; o += 7 * 64 + 2 * KB_RMAX + 4;   // vectors, r of two knots, the info int
    P.nf = o;
    o = 0;
    P.oYl = o; o += P.LDB * maxw;
    o = (o + 3) & ~3;
    P.oWl = o; o += std::max(1, PMW * (PMW + 1) / 2);
    o = (o + 3) & ~3;
    P.oV2 = o; o += 2 * 64 + 4 * KB_WMAX + 6 * 64;
    P.nb = o;
    P.sU = P.hfac ? sU : 0;
    P.LDH = r16(maxw) + 4;
    P.nh = P.hfac ? P.LDH * KB_WMAX + 4 : 0;
    // split path: at most two of (n1, p, n2) nonzero at every knot (register tile budget of
    // the factor kernel: one 4×4 grid of Ã⁻ᵀ[D|F] or Ẽ, plus B and C)
    P.split = kb_split_env() != 0;
    int64_t IMGT = 0;
    for (int k = 0; k < a.N; ++k) {
        if ((n1[k] > 0) + (p[k] > 0) + (n2[k] > 0) > 2) P.split = false;
        if (k + 1 < a.N && n2[k] != n1[k + 1]) P.split = false;
        IMGT += (img_off(r16(n1[k]), r16(p[k]), r16(n2[k])).end + 63) & ~(int64_t)63;
    }
    P.IMGT = IMGT;
    P.nruns = (a.N + KS_L - 1) / KS_L;
    P.nbt = RM >> 4;
    // the longest run of interior knots (p = 0, n1 = n2 = one padded size, knot 0 excluded:
    // the mid kernel resumes from the slab state of the knot before)
    P.mid0 = P.mid1 = 0;
    P.midnt = 0;
    if (P.split && kb_mid_env()) {
        int best0 = 0, best1 = 0;
        for (int k = 1; k < a.N;) {
            const int P2 = r16(n2[k]);
            if (p[k] == 0 && P2 > 0 && r16(n1[k]) == P2) {
                int e = k;
                while (e < a.N && p[e] == 0 && r16(n2[e]) == P2 && r16(n1[e]) == P2) ++e;
                if (e - k > best1 - best0) {
                    best0 = k;
                    best1 = e;
                }
                k = e;
            } else {
                ++k;
            }
        }
        if (best1 - best0 >= 2) {
            P.mid0 = best0;
            P.mid1 = best1;
            P.midnt = r16(n2[best0]) >> 4;
        }
    }
    // fused interior run: the Schur kernel covers [0, mid0) and [mid1, N) only, and the
    // interior knots get no image
    P.fuse = P.midnt > 0 && P.mid1 < a.N && kb_fuse_env() != 0;
    P.midfull = P.fuse && n2[P.mid0] == 16 * P.midnt;
    P.nr0 = P.nruns;
    if (P.fuse) {
        P.nr0 = (P.mid0 + KS_L - 1) / KS_L;
        P.nruns = P.nr0 + (a.N - P.mid1 + KS_L - 1) / KS_L;
        for (int k = P.mid0; k < P.mid1; ++k) P.IMGT -= (img_off(r16(n1[k]), r16(p[k]), r16(n2[k])).end + 63) & ~(int64_t)63;
    }
    constexpr size_t LDS_CAP = 160 * 1024;
    return (size_t)P.nf * tsize <= LDS_CAP && (size_t)P.nb * tsize <= LDS_CAP && (size_t)P.nh * tsize <= LDS_CAP;
}

size_t kb_slab_cap()    // LQRX_KKT_BIG_SLAB_MB bounds the stream-ordered scratch (default 40 GiB)
{
    static const size_t v = [] {
        const char *e = std::getenv("LQRX_KKT_BIG_SLAB_MB");
        return e ? (size_t)std::strtoull(e, nullptr, 10) << 20 : (size_t)40 << 30;
    }();
    return v;
}

// scratch elements per trajectory: the slab, plus Z, gz and packed U⁻¹ for a dense H, plus
// the Schur images of the split path
int64_t kb_per_traj(const KktArgs &a, const KbPlan &P)
{
    return P.S + (P.hfac ? a.sY + a.sg + P.sU : 0) + (P.split ? P.IMGT : 0);
}

// trajectories per chunk: as many as `avail` holds, then evened out over the chunks (a
// short last chunk would leave most of the GPU idle in the factor kernel)
int64_t kb_chunk(const KktArgs &a, const KbPlan &P, int tsize, size_t avail)
{
    const size_t per = (size_t)kb_per_traj(a, P) * tsize;
    const int64_t most = std::max<int64_t>(1, std::min<int64_t>(a.batch, (int64_t)(avail / std::max<size_t>(per, 1))));
    const int64_t nch = (a.batch + most - 1) / most;
    return std::max<int64_t>(1, (a.batch + nch - 1) / nch);
}

template <typename T>
hipError_t kb_launch_t(const KktArgs &a, const KbPlan &P, hipStream_t s)
{
    const size_t per = (size_t)kb_per_traj(a, P) * sizeof(T);
    int64_t chunk = kb_chunk(a, P, sizeof(T), a.ws ? a.ws_bytes : kb_slab_cap());
    Scratch sc;
    hipError_t e = sc.get(a, (size_t)chunk * per, s);
    // library scratch (no caller workspace): when the pool cannot hold the cap's chunk, run the
    // batch in smaller chunks instead of failing — halve until it fits or one trajectory fails
    while (e == hipErrorOutOfMemory && !a.ws && chunk > 1) {
        (void)hipGetLastError();
        chunk = kb_chunk(a, P, sizeof(T), (size_t)((chunk + 1) / 2) * per);
        e = sc.get(a, (size_t)chunk * per, s);
    }
    if (e != hipSuccess) return e;
    const size_t lf = (size_t)P.nf * sizeof(T), lb = (size_t)P.nb * sizeof(T);
    const size_t lh = (size_t)P.nh * sizeof(T);
    if ((e = hipFuncSetAttribute((const void *)kkt_big_fwd_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lf)) != hipSuccess ||
        (e = hipFuncSetAttribute((const void *)kkt_big_bwd_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)lb)) != hipSuccess ||
        (P.hfac && (e = hipFuncSetAttribute((const void *)kkt_big_hfac_kernel<T>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lh)) != hipSuccess)) {
        (void)sc.release(s);
        return e;
    }
    // scratch: [slab chunk·S][Z chunk·sY][gz chunk·sg][U⁻¹ chunk·sU] (dense H) [images chunk·IMGT] (split)
    T *slab = (T *)sc.p, *Z = slab + chunk * P.S, *gz = Z + chunk * a.sY, *Ui = gz + chunk * a.sg;
    T *img = P.hfac ? Ui + chunk * P.sU : Z;
    constexpr int KS_NW = 4;
    const size_t lfac = (size_t)KF_W * KF_LDS * sizeof(T);
    if (P.split && ((e = hipFuncSetAttribute((const void *)kb_factor_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lfac)) != hipSuccess ||
                    (e = hipFuncSetAttribute((const void *)kb_factor_mid_kernel<T, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lfac)) != hipSuccess ||
                    (e = hipFuncSetAttribute((const void *)kb_factor_mid_kernel<T, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lfac)) != hipSuccess ||
                    (e = hipFuncSetAttribute((const void *)kb_factor_mid_kernel<T, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lfac)) != hipSuccess ||
                    (e = hipFuncSetAttribute((const void *)kb_factor_mid_kernel<T, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lfac)) != hipSuccess ||
                    (e = hipFuncSetAttribute((const void *)kb_bwd_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)((size_t)KF_W * (KBW_V + KBW_W) * sizeof(T)))) != hipSuccess)) {
        (void)sc.release(s);
        return e;
    }
    KsArgs<T> ks{};
    KfArgs<T> kf{};
    if (P.split) {
        ks.Y = P.hfac ? Z : (const T *)a.Y; ks.y = (const T *)a.y; ks.H = (const T *)a.H;
        ks.g = P.hfac ? gz : (const T *)a.g;
        ks.img = img; ks.meta = a.meta; ks.N = a.N; ks.nruns = P.nruns;
        ks.hinv = a.ginv && !P.hfac; ks.useg = a.ginv; ks.yrel = P.hfac;
        ks.sY = a.sY; ks.sy = a.sy; ks.sH = a.sH; ks.sg = a.sg; ks.IMGT = P.IMGT;
        ks.nr0 = P.nr0;
        ks.kend0 = P.fuse ? P.mid0 : a.N;
        ks.kbeg1 = P.fuse ? P.mid1 : a.N;
        kf.img = img; kf.slab = slab; kf.info = a.info; kf.meta = a.meta; kf.N = a.N; kf.hfac = P.hfac;
        kf.IMGT = P.IMGT; kf.sS = P.S;
        kf.fz0 = P.fuse ? P.mid0 : 0;
        kf.fz1 = P.fuse ? P.mid1 : 0;
    }
    KuArgs<T> ku{};
    constexpr int KU_W = ku_w<T>();
#ifdef KU_SOLO
    const size_t lfu = std::max((size_t)KU_W * KU_LDS * sizeof(T), (size_t)96 * 1024);   // 1 WG per CU (A/B only)
#else
    const size_t lfu = (size_t)KU_W * KU_LDS * sizeof(T);
#endif
    if (P.fuse) {
        ku.Y = P.hfac ? Z : (const T *)a.Y; ku.y = (const T *)a.y; ku.H = (const T *)a.H;
        ku.g = P.hfac ? gz : (const T *)a.g;
        ku.slab = slab; ku.info = a.info; ku.meta = a.meta; ku.N = a.N; ku.kb = P.mid0; ku.ke = P.mid1;
        ku.hinv = a.ginv && !P.hfac; ku.useg = a.ginv; ku.yrel = P.hfac; ku.hfac = P.hfac;
        ku.sY = a.sY; ku.sy = a.sy; ku.sH = a.sH; ku.sg = a.sg; ku.sS = P.S;
        const void *fk[8] = {(const void *)kb_fuse_mid_kernel<T, 1, false>, (const void *)kb_fuse_mid_kernel<T, 1, true>,
                             (const void *)kb_fuse_mid_kernel<T, 2, false>, (const void *)kb_fuse_mid_kernel<T, 2, true>,
                             (const void *)kb_fuse_mid_kernel<T, 3, false>, (const void *)kb_fuse_mid_kernel<T, 3, true>,
                             (const void *)kb_fuse_mid_kernel<T, 4, false>, (const void *)kb_fuse_mid_kernel<T, 4, true>};
        for (int i = 0; i < 8 && e == hipSuccess; ++i)
            e = hipFuncSetAttribute(fk[i], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lfu);
        if (e != hipSuccess) {
            (void)sc.release(s);
            return e;
        }
    }
    KhArgs<T> h{};
    if (P.hfac) {
        h.Y = (const T *)a.Y; h.H = (const T *)a.H; h.g = (const T *)a.g;
        h.Z = Z; h.gz = gz; h.Ui = Ui; h.info = a.info; h.meta = a.meta; h.N = a.N; h.LDH = P.LDH;
        h.sY = a.sY; h.sH = a.sH; h.sg = a.sg; h.sU = P.sU;
    }
    KbArgs<T> k{};
    k.Y = (const T *)a.Y; k.y = (const T *)a.y; k.H = (const T *)a.H; k.g = (const T *)a.g;
    k.dz = (T *)a.dz; k.lam = (T *)a.lam; k.slab = (T *)sc.p; k.info = a.info; k.meta = a.meta;
    k.N = a.N; k.ginv = a.ginv;
    k.sY = a.sY; k.sy = a.sy; k.sH = a.sH; k.sg = a.sg; k.sS = P.S;
    k.LD = P.LD; k.LDY = P.LDY; k.LDB = P.LDB;
    k.oWp = P.oWp; k.oBlk = P.oBlk; k.oSl = P.oSl; k.oV = P.oV;
    k.oYl = P.oYl; k.oWl = P.oWl; k.oV2 = P.oV2;
    k.slab = slab;
    if (P.hfac) {
        k.hfac = 1; k.yrel = 1; k.Y = Z; k.g = gz; k.Ui = Ui; k.sU = P.sU;
    }
#ifdef KB_PROF
    static int64_t *prof = nullptr;
    if (!prof) (void)hipMalloc((void **)&prof, 128 * sizeof(int64_t));   // ≤ 8 waves × 16 phases
    (void)hipMemsetAsync(prof, 0, 128 * sizeof(int64_t), s);
    k.prof = prof;
    ku.prof = prof;
#endif
    for (int64_t b0 = 0; b0 < a.batch && e == hipSuccess; b0 += chunk) {
        const int64_t nb = std::min<int64_t>(chunk, a.batch - b0);
        k.b0 = b0;
        if (P.hfac) {
            h.b0 = b0;
            hipLaunchKernelGGL(kkt_big_hfac_kernel<T>, dim3((unsigned)nb), dim3(KB_THREADS), lh, s, h);
        }
        if (P.split) {
            ks.b0 = b0;
            kf.b0 = b0;
            kf.nb = nb;
            const dim3 gs((unsigned)(nb * P.nruns)), bs(64 * KS_NW);
            switch (P.nbt) {
#define KS_L_(NB) case NB: hipLaunchKernelGGL((kb_schur_kernel<T, KS_NW, NB>), gs, bs, 0, s, ks); break;
            KS_L_(1) KS_L_(2) KS_L_(3) KS_L_(4) KS_L_(5) KS_L_(6) KS_L_(7)
            default: hipLaunchKernelGGL((kb_schur_kernel<T, KS_NW, 8>), gs, bs, 0, s, ks); break;
#undef KS_L_
            }
            const dim3 gf((unsigned)((nb + KF_W - 1) / KF_W)), bf(64 * KF_W);
            auto generic = [&](int k0_, int k1_) {
                if (k0_ >= k1_) return;
                kf.kb = k0_;
                kf.ke = k1_;
                hipLaunchKernelGGL(kb_factor_kernel<T>, gf, bf, lfac, s, kf);
            };
            if (P.fuse) {
                generic(0, P.mid0);
                ku.b0 = b0;
                ku.nb = nb;
                const dim3 gu((unsigned)((nb + KU_W - 1) / KU_W)), bu(64 * KU_W);
                switch (P.midnt * 2 + (P.midfull ? 1 : 0)) {
#define KU_L_(NT_, F_) case NT_ * 2 + F_: hipLaunchKernelGGL((kb_fuse_mid_kernel<T, NT_, F_ != 0>), gu, bu, lfu, s, ku); break;
                KU_L_(1, 0) KU_L_(1, 1) KU_L_(2, 0) KU_L_(2, 1) KU_L_(3, 0) KU_L_(3, 1) KU_L_(4, 0)
                default: hipLaunchKernelGGL((kb_fuse_mid_kernel<T, 4, true>), gu, bu, lfu, s, ku); break;
#undef KU_L_
                }
                generic(P.mid1, a.N);
            } else if (P.mid1 > P.mid0) {
                generic(0, P.mid0);
                kf.kb = P.mid0;
                kf.ke = P.mid1;
                switch (P.midnt) {
                case 1: hipLaunchKernelGGL((kb_factor_mid_kernel<T, 1>), gf, bf, lfac, s, kf); break;
                case 2: hipLaunchKernelGGL((kb_factor_mid_kernel<T, 2>), gf, bf, lfac, s, kf); break;
                case 3: hipLaunchKernelGGL((kb_factor_mid_kernel<T, 3>), gf, bf, lfac, s, kf); break;
                default: hipLaunchKernelGGL((kb_factor_mid_kernel<T, 4>), gf, bf, lfac, s, kf); break;
                }
                generic(P.mid1, a.N);
            } else {
                generic(0, a.N);
            }
        } else
            hipLaunchKernelGGL(kkt_big_fwd_kernel<T>, dim3((unsigned)nb), dim3(KB_THREADS), lf, s, k);
        if (P.split)
            hipLaunchKernelGGL(kb_bwd_kernel<T>, dim3((unsigned)((nb + KF_W - 1) / KF_W)), dim3(64 * KF_W),
                               (size_t)KF_W * (KBW_V + KBW_W) * sizeof(T), s, k, nb);
        else
            hipLaunchKernelGGL(kkt_big_bwd_kernel<T>, dim3((unsigned)nb), dim3(KB_THREADS), lb, s, k);
        e = hipGetLastError();
    }
#ifdef KB_PROF
    {
        int64_t h[128];
        (void)hipStreamSynchronize(s);
        (void)hipMemcpy(h, prof, sizeof h, hipMemcpyDeviceToHost);
        const double steps = (double)a.batch * (a.N + 2);
        if (P.fuse) {
            const double kn = (double)a.batch * (P.mid1 - P.mid0);   // wave-knots
            std::fprintf(stderr, "KB_PROF fused kernel, cycles per knot and wave [chol+inv | lambda+slab | stream | reduce"
                                 " || chol: leaves | panel+trailing | inverse assembly]:");
            for (int i = 0; i < 7; ++i) {
                double sum = 0;
                for (int w = 0; w < 8; ++w) sum += (double)h[16 * w + i];
                std::fprintf(stderr, " %9.0f", sum / kn);
            }
            std::fprintf(stderr, "\n");
        }
        std::fprintf(stderr, "KB_PROF cycles per step and wave [prefactor factor schur barrier handover | "
                             "F: cholB+E cholC fwdsubst slab Wcopy]:\n");
        for (int w = 0; w < 4; ++w) {
            std::fprintf(stderr, "  wave %d:", w);
            for (int i = 0; i < 10; ++i) std::fprintf(stderr, " %8.0f", h[16 * w + i] / steps);
            std::fprintf(stderr, "\n");
        }
    }
#endif
    const hipError_t ef = sc.release(s);
    return e != hipSuccess ? e : ef;
}

} // namespace

bool kkt_big_supported(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2, const int32_t *w)
{
    KbPlan P;
    return kb_plan(a, n1, p, n2, w, a.dtype == 1 ? 4 : 8, P);
}

size_t kkt_big_scratch_bytes(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                             const int32_t *w)
{
    KbPlan P;
    const int ts = a.dtype == 1 ? 4 : 8;
    if (!kb_plan(a, n1, p, n2, w, ts, P)) return 0;
    return (size_t)kb_chunk(a, P, ts, kb_slab_cap()) * (size_t)kb_per_traj(a, P) * ts;
}

hipError_t kkt_big_launch(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                          const int32_t *w, hipStream_t s)
{
    KbPlan P;
    const int ts = a.dtype == 1 ? 4 : 8;
    if (!kb_plan(a, n1, p, n2, w, ts, P)) return hipErrorNotSupported;
    return a.dtype == 1 ? kb_launch_t<float>(a, P, s) : kb_launch_t<double>(a, P, s);
}

} // namespace lqrx
