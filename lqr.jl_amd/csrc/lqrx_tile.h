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
    // D = −A·B + C  (f64 MFMA neg modifier on A: blgp bit 0 → "neg:[1,0,0]")
    static __device__ __forceinline__ acc mma_nega(double a, double b, acc c)
    {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 1);
    }
    static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};

template <> struct Tile<float> {
    using acc = float __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc mma(float a, float b, acc c)
    {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // f32 MFMA has no neg modifier (blgp is a broadcast control): negate the operand
    static __device__ __forceinline__ acc mma_nega(float a, float b, acc c)
    {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(-a, b, c, 0, 0, 0);
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
template <typename T, int KT, int I, int J, bool NEG = false>
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
                for (int j = 0; j < J; ++j)
                    D[i][j] = NEG ? Tile<T>::mma_nega(M[k][i][r], Y[k][j][r], D[i][j])
                                  : Tile<T>::mma(M[k][i][r], Y[k][j][r], D[i][j]);
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
// If diag_pad, padded diagonal entries are 1 (keeps a padded SPD block SPD).  Loads are
// unconditional (out-of-range lanes read element 0 and select the pad value) so the tile
// load is one straight run of global loads; FULL = dimensions are exact multiples of 16.
template <typename T, int I, int J, bool FULL = false>
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
                bool ok = FULL || (row < rows && col < cols);
                T v = src[ok ? (size_t)row + (size_t)col * ld : 0];
                if (!FULL) v = ok ? v : ((diag_pad && row == col) ? (T)1 : (T)0);
                D[i][j][r] = v;
            }
}

template <typename T, int I, int J, bool FULL = false>
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
                if (FULL || (row < rows && col < cols)) dst[(size_t)row + (size_t)col * ld] = D[i][j][r];
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

// D[i][j] += Σ_k M[k][i]ᵀ Y[k][j] for the lower tiles i >= j only (symmetric results).
template <typename T, int KT, int NT, bool NEG = false>
__device__ __forceinline__ void mma_tn_lower(typename Tile<T>::acc (&D)[NT][NT],
                                             const typename Tile<T>::acc (&M)[KT][NT],
                                             const typename Tile<T>::acc (&Y)[KT][NT])
{
#pragma unroll
    for (int k = 0; k < KT; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < NT; ++i)
#pragma unroll
                for (int j = 0; j <= i; ++j)
                    D[i][j] = NEG ? Tile<T>::mma_nega(M[k][i][r], Y[k][j][r], D[i][j])
                                  : Tile<T>::mma(M[k][i][r], Y[k][j][r], D[i][j]);
}

// Load the lower tiles (i >= j) of a rows×cols column-major matrix; upper tiles zeroed.
template <typename T, int NT, bool FULL = false>
__device__ __forceinline__ void tiles_load_lower(typename Tile<T>::acc (&D)[NT][NT], const T *__restrict__ src,
                                                 int rows, int cols, int lane)
{
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int row = i * 16 + Tile<T>::row(lane, r), col = j * 16 + tcol(lane);
                if (j > i) { D[i][j][r] = (T)0; continue; }
                bool ok = FULL || (row < rows && col < cols);
                T v = src[ok ? (size_t)row + (size_t)col * rows : 0];
                D[i][j][r] = (FULL || ok) ? v : (T)0;
            }
}

// Make a tile matrix exactly symmetric from its lower triangle: every element above the
// diagonal (upper tiles AND the upper half of diagonal tiles) is replaced by its mirror.
// Needed for the fast form P_ = Q + AᵀPA − GᵀK, whose accuracy relies on P staying
// symmetric (GᵀK equals the reference's APB·K only for symmetric P).  Goes through an
// NT·16 × NT·16 column-major LDS image with column stride NT·16 + 2.  Every LDS read is
// unconditional and the diagonal tiles blend with a bit mask (no exec-mask branches: a
// predicated read costs ~6 scalar/VALU instructions plus an SGPR-spill readlane).
__device__ __forceinline__ double blend_upper(double keep, double mirror, bool take)
{
    const long long m = -(long long)take;                       // all-ones when take
    return __longlong_as_double((__double_as_longlong(mirror) & m) | (__double_as_longlong(keep) & ~m));
}
__device__ __forceinline__ float blend_upper(float keep, float mirror, bool take)
{
    const int m = -(int)take;
    return __int_as_float((__float_as_int(mirror) & m) | (__float_as_int(keep) & ~m));
}

template <typename T, int NT>
__device__ __forceinline__ void tiles_symmetrize_lower(typename Tile<T>::acc (&D)[NT][NT], T *lds,
                                                       int lane)
{
    constexpr int S = NT * 16 + 2;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                lds[(i * 16 + Tile<T>::row(lane, r)) + (j * 16 + tcol(lane)) * S] = D[i][j][r];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = i; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = i * 16 + Tile<T>::row(lane, r), col = j * 16 + tcol(lane);
                const T v = lds[col + row * S];
                if (j > i) D[i][j][r] = v;                       // strictly upper tile: all mirrored
                else D[i][j][r] = blend_upper(D[i][j][r], v, row < col);
            }
    __syncthreads();
}

// Load the lower tiles (i >= j) of an LDS-resident column-major image (column stride cs);
// upper tiles zeroed.
template <typename T, int NT>
__device__ __forceinline__ void tiles_lower_from_lds(typename Tile<T>::acc (&D)[NT][NT], const T *lds, int cs,
                                                     int lane)
{
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                D[i][j][r] = (j > i) ? (T)0 : lds[(i * 16 + Tile<T>::row(lane, r)) + (j * 16 + tcol(lane)) * cs];
}

// wave-wide max (xor butterfly; every lane gets the result)
__device__ __forceinline__ double wave_max(double v)
{
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v)
{
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// Wave-wide max of a NON-NEGATIVE value as a wave-uniform scalar (lands in an SGPR, so a
// branch on it is uniform): integer max on the float bit pattern (order-preserving for
// x ≥ 0) through DPP row shifts and row broadcasts (gfx9 DPP), then v_readlane of lane 63.
// 6 VALU + 1 readlane, no LDS (the xor-butterfly above costs 12 ds_bpermute for a double).
__device__ __forceinline__ int wave_max_uniform_i(int v)
{
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ float wave_max_uniform(float x)
{
    return __int_as_float(wave_max_uniform_i(__float_as_int(x)));
}

// 1/a: hardware estimate (v_rcp_f64: max rel err 4.6e-8 measured on gfx950, see
// profiles/r01/lat_probe.txt) + one Newton step → ~2e-15 relative.
__device__ __forceinline__ double rcp_nr(double a)
{
    double y = __builtin_amdgcn_rcp(a);
#pragma unroll
    for (int it = 0; it < 1; ++it) {
        double e = fma(-a, y, 1.0);
        y = fma(y, e, y);
    }
    return y;
}
__device__ __forceinline__ float rcp_nr(float a)
{
    float y = __builtin_amdgcn_rcpf(a);
    float e = fmaf(-a, y, 1.0f);
    return fmaf(y, e, y);
}

// 1/a to full fp64 precision (two Newton steps) — replaces IEEE division (~10 instrs)
__device__ __forceinline__ double rcp_nr2(double a)
{
    double y = __builtin_amdgcn_rcp(a);
    double e = fma(-a, y, 1.0);
    y = fma(y, e, y);
    e = fma(-a, y, 1.0);
    return fma(y, e, y);
}

// 1/sqrt(a): hardware estimate + Newton steps to full precision.
__device__ __forceinline__ double rsqrt_nr(double a)
{
    double y = __builtin_amdgcn_rsq(a);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        double h = 0.5 * a * y;
        double r = fma(-h, y, 0.5);
        y = fma(y, r, y);
    }
    return y;
}
__device__ __forceinline__ float rsqrt_nr(float a)
{
    float y = __builtin_amdgcn_rsqf(a);
    float h = 0.5f * a * y;
    float r = fmaf(-h, y, 0.5f);
    return fmaf(y, r, y);
}

} // namespace lqrx
