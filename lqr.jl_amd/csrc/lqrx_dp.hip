// lqrx_dp.hip — batched finite-horizon LQR (Riccati backward pass + forward rollout) on
// gfx950.  Replaces, for a whole batch per launch, the reference's per-knot LAPACK/BLAS
// calls in solve!(sol, ::DPSolver, ::LQRProblem)  /root/reference/src/dynamic_programming.jl:54-72.
//
// Mapping: ONE WAVEFRONT PER TRAJECTORY (64-thread workgroup).  The wave walks the
// horizon k = N-1 … 1 sequentially (the Riccati recurrence is serial in k); parallelism is
// the batch.  All n×n / n×m products of a knot are fp64 MFMA (v_mfma_f64_16x16x4_f64) on
// register-resident C-layout tiles, each written as a "Mᵀ·Y" product (lqrx_tile.h) so that
// no operand ever moves between lanes:
//
//   reference (dynamic_programming.jl)      here (all tiles C-layout, P symmetric)
//   :38  PB  = P*B                          PB   = Pᵀ·B
//   :39  E   = R + B'PB                     E    = R + Bᵀ·PB
//   :40  PA  = P*A                          PA   = Pᵀ·A
//   :41  K   = B'PA                         G    = Bᵀ·PA
//   :29-30 potrf!/potrs!(E, K)              K    = E⁻¹G   (lane-per-column Cholesky, VALU)
//   :50  APB = A'PB                         APBᵀ = PBᵀ·A   (the transpose is what is needed)
//   :51  P_  = Q + A'PA - APB*K             P_   = Q + Aᵀ·PA + (APBᵀ)ᵀ·(−K)
//
// The time-invariant A, B, Q, R (lqr_problem.jl:1-11) stay in registers for the whole
// horizon; HBM traffic is the K stream (written per knot, re-read by the rollout) plus X, U.
// The m×m Cholesky + two triangular solves run on the VALU in a lane-per-column layout of
// the augmented matrix [E | G] (wave-uniform broadcasts via v_readlane), overlapping the
// MFMA work of the other wave resident on the same SIMD (launch bounds: 2 waves/SIMD).
#include <cstdlib>
#include "lqrx_tile.h"
#include "lqrx_internal.h"

#ifndef LQRX_DP_WAVES
#define LQRX_DP_WAVES 2
#endif
#ifndef LQRX_DP_BCAST
#define LQRX_DP_BCAST 0
#endif
#ifndef LQRX_DP_VAR
#define LQRX_DP_VAR 0
#endif
#ifndef LQRX_DP_TVWAVES
#define LQRX_DP_TVWAVES 0   // 0: per tile grid (launch_dp_tv); 1 or 2 forces waves/SIMD (A/B builds)
#endif
#ifndef LQRX_DP_TVEXTRA
#define LQRX_DP_TVEXTRA 0   // extra VAR bits for the time-varying launch (ablations, tools only)
#endif
#ifndef LQRX_DP_TVABL
#define LQRX_DP_TVABL 0     // ablation (tools only): re-read knot-1 inputs, see the kernel
#endif
#ifndef LQRX_DP_TVAD
#define LQRX_DP_TVAD 1      // time-varying rollout: knots of A_k/B_k row prefetch (A/B builds)
#endif
#ifndef LQRX_DP_KD
#define LQRX_DP_KD 4        // rollout: knots of K_k prefetch (A/B builds)
#endif
#ifndef LQRX_DP_TVKD
#define LQRX_DP_TVKD 4      // time-varying rollout: knots of K_k prefetch (A/B builds)
#endif
#ifndef LQRX_DP_TVWAIT
#define LQRX_DP_TVWAIT 0
#endif
#ifndef LQRX_DP_WG4
#define LQRX_DP_WG4 1         // fp64 n = 64: the four-wave kernel (A/B builds: 0 = one wave)
#endif
#ifndef LQRX_DP_ROLL_FULL
#define LQRX_DP_ROLL_FULL 1   // exact tile grids: the register-streamed rollout (A/B builds: 0)
#endif

namespace lqrx {

// wave-level ordering of LDS traffic between the lanes of a one-wave workgroup (the LDS is in
// order per wave; this is the compiler fence + wave barrier, no s_barrier)
__device__ __forceinline__ void wsync_w()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// v of lane (lane ^ o): one ds_bpermute per dword with the lane address precomputed (the
// generic __shfl_xor adds a width test and a select per call)
__device__ __forceinline__ double xor_shfl(double v, int addr)
{
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)(x & 0xffffffffll));
    const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(x >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ float xor_shfl(float v, int addr)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
}

// Forward LDLᵀ sweep on the augmented matrix [E | G | I] — the factor/solve of
// chol_solve! (dynamic_programming.jl:28-31: potrf 'U' + potrs 'U'), reorganised so that
// it costs the fewest VALU instructions (fp64 VALU does not overlap fp64 MFMA on gfx950).
//
// E = L D Lᵀ (unit-lower L; D_ii are exactly potrf's squared pivots U_ii², so the
// potrf failure test "pivot ≤ 0" is unchanged).  One column of [E | G | I] per lane
// (columns lane + 64q).  Step i:  piv = E'[i][i] (v_readlane of lane i), t = x[i]/piv,
// x[p] −= E'[i][p]·t for p > i, where the unscaled pivot row E'[i][p] reaches every lane
// as a uniform LDS read (BCAST = 1) or v_readlane (BCAST = 0).  Afterwards
//   G columns hold Y = L⁻¹G,  I columns hold W = L⁻¹,  and rinv[i] = 1/piv_i,
// so  K = E⁻¹G = Wᵀ·(D⁻¹Y)  — finished by the caller as one TN MFMA product.
// Column images written back to LDS: aug[MP..MP+NP) ← Y, aug[MP+NP..2MP+NP) ← W,
// rinv (MP values) at aug + (2MP+NP)·CS.  Returns false if a pivot was not > 0.
template <typename T, int MP, int NP, int CS, int BCAST>
__device__ __forceinline__ bool aug_ldl_forward(T *aug, int lane)
{
    constexpr int NC = MP + NP + MP;
    constexpr int CPL = (NC + 63) / 64;
    T *rowbuf = aug + NC * CS;        // 64-wide broadcast row (reused every step)
    T *rinv = rowbuf + 64;            // 1/pivot per row
    T x[CPL][MP];
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
        int c = lane + 64 * q;
        if (c < MP + NP) {
#pragma unroll
            for (int i = 0; i < MP; ++i) x[q][i] = aug[c * CS + i];
        } else {
#pragma unroll
            for (int i = 0; i < MP; ++i) x[q][i] = (c - MP - NP == i) ? (T)1 : (T)0;
        }
    }
    bool ok = true;
#pragma unroll
    for (int i = 0; i < MP; ++i) {
        if constexpr (BCAST == 1) {
            // publish row i of E' (final after step i-1) for the uniform reads below
            rowbuf[lane] = x[0][i];   // 64-wide row buffer: no exec mask
        }
        T piv = readlane(x[i / 64][i], i % 64);
        ok = ok && (piv > (T)0);
        T ri = rcp_nr(piv);
        if (lane == 0) rinv[i] = ri;
        T t[CPL];
#pragma unroll
        for (int q = 0; q < CPL; ++q) t[q] = x[q][i] * ri;
        if constexpr (BCAST == 1) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
        for (int p = i + 1; p < MP; ++p) {
            T e;
            if constexpr (BCAST == 1) e = rowbuf[p];
            else e = readlane(x[p / 64][i], p % 64);
#pragma unroll
            for (int q = 0; q < CPL; ++q) x[q][p] = fma(-e, t[q], x[q][p]);
        }
        if constexpr (BCAST == 1) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
        int c = lane + 64 * q;
        if (c >= MP && c < NC) {
#pragma unroll
            for (int i = 0; i < MP; ++i) aug[c * CS + i] = x[q][i];
        }
    }
    return ok;
}

// Newton–Schulz refinement of X ≈ E⁻¹ (E SPD, MT×MT tiles), warm-started from the previous
// knot's inverse.  One step: R = I − EᵀX (4·MT³ MFMAs, neg-A with C = I), X ← X + XᵀR.
// Returns true once the step just taken is converged to working precision: with
// ρ = 16·MT·max|R| ≥ ‖R‖∞ the new residual is ≤ cond(E)·ρ², so ρ ≤ tol (1e-11 in fp64:
// cond·1e-22, far below the rounding floor) accepts.  Not converged after `it` steps
// (e.g. a cold or poor start) → false, and the caller runs the exact sweep.
template <typename T> struct NsTol;
template <> struct NsTol<double> {
    static constexpr double v = 1e-11, one_step = 1e-9; static constexpr int it = 6;
};
template <> struct NsTol<float> {
    static constexpr float v = 3e-4f, one_step = 1e-5f; static constexpr int it = 6;
};

// NaN-propagating magnitude key: the high word of |v| (sign cleared) — order-preserving
// for magnitudes, and every NaN key exceeds +inf's.  (fmax() would silently DROP a NaN
// element — IEEE maxNum — and let a diverged iterate pass the convergence test.)
// key_bound(k) is the largest double with that high word: an upper bound of the magnitude.
__device__ __forceinline__ int mag_key(double v) { return __double2hiint(v) & 0x7fffffff; }
__device__ __forceinline__ double key_bound(int k, double) { return __hiloint2double(k, -1); }
__device__ __forceinline__ int mag_key(float v) { return __float_as_int(v) & 0x7fffffff; }
__device__ __forceinline__ float key_bound(int k, float) { return __int_as_float(k); }

template <typename T, int MT>
__device__ __forceinline__ bool ns_refine(typename Tile<T>::acc (&X)[MT][MT],
                                          const typename Tile<T>::acc (&E)[MT][MT],
                                          const typename Tile<T>::acc (&Id)[MT][MT], int lane)
{
    using acc = typename Tile<T>::acc;
    for (int it = 0; it < NsTol<T>::it; ++it) {
        acc R[MT][MT];
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < MT; ++j) R[i][j] = Id[i][j];
        mma_tn<T, MT, MT, MT, true>(R, E, X);                   // R = I − EᵀX
        int key = 0;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < MT; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) key = max(key, mag_key(R[i][j][r]));
        // uniform (SGPR) residual bound ρ ≥ ‖R‖∞ (NaN if any element is NaN)
        const T rho = (T)(16 * MT) * key_bound(wave_max_uniform_i(key), (T)0);
        if (rho <= NsTol<T>::v) return true;                    // X already at working precision
        if (!(rho < (T)1)) return false;                        // no contraction (or NaN): exact sweep
        mma_tn<T, MT, MT, MT>(X, X, R);                         // X ← X + XᵀR
        if (rho <= NsTol<T>::one_step) return true;             // new residual ≤ cond·ρ² ≪ eps
    }
    (void)lane;
    return false;
}

template <typename T, int NT, int MT> struct DpCfg {
    static constexpr int NP = NT * 16, MP = MT * 16;
    static constexpr int CS = MP + 2;                       // padded LDS column stride
    static constexpr int AUG = (MP + NP + MP) * CS + 64 + MP; // [E | G | I] image + row/rinv
    static constexpr int ROLL = MP * NP + NP + MP;          // K_k + x + u (rollout)
    static constexpr int SYM = NP * (NP + 2);                // symmetrize image
    static constexpr int LDS_ELEMS = (AUG > ROLL ? AUG : ROLL) > SYM ? (AUG > ROLL ? AUG : ROLL) : SYM;
    static constexpr int QCS = NP + 2;                      // LDS-resident Q image: column stride
    static constexpr int QIMG = NP * QCS;
    static constexpr int KPL = (MP * NP + 63) / 64;         // K elements per lane (rollout)
};

// Forward rollout  dynamic_programming.jl:66-70 :  u_k = −K_k x_k ; x_{k+1} = A x_k + B u_k.
// K_k is streamed back from global (written by the backward sweep of this same wave),
// DEPTH knots ahead, 64 lanes × KPL coalesced elements per knot, staged through LDS.
// Dot products are split over the wave: u_i by SU = 64/MP lanes (i = lane % MP), x'_i by
// SX = 64/NP lanes (i = lane % NP), partial sums combined with xor-shuffles.
template <typename T, int NT, int MT, int DEPTH, bool TV = false, bool LIN = false>
__device__ __forceinline__ void dp_rollout(const DpArgs &a, int64_t b, T *lds, int lane)
{
    using C = DpCfg<T, NT, MT>;
    constexpr int NP = C::NP, MP = C::MP, KPL = C::KPL;
    constexpr int SU = 64 / MP > 0 ? 64 / MP : 1, SX = 64 / NP > 0 ? 64 / NP : 1;
    constexpr int JU = NP / SU, JX = NP / SX, PX = MP / SX; // per-lane slice lengths
    static_assert(MP <= 64 && NP <= 64, "rollout assumes n, m <= 64");
    const int n = a.n, m = a.m, N = a.N;
    const size_t mn = (size_t)m * n;
    const T *__restrict__ Kg = (const T *)a.K + (size_t)b * (size_t)(N - 1) * mn;
    // time-varying (TV): knot k's A_k, B_k at knot stride sA, sB (0 for a time-invariant field)
    const int64_t sA = (TV && a.tv_AB) ? (int64_t)n * n : 0, sB = (TV && a.tv_AB) ? (int64_t)n * m : 0;
    const T *__restrict__ Ag = (const T *)a.A + (size_t)b * n * n * (TV && a.tv_AB ? N - 1 : 1);
    const T *__restrict__ Bg = (const T *)a.B + (size_t)b * n * m * (TV && a.tv_AB ? N - 1 : 1);
    T *__restrict__ Xg = (T *)a.X + (size_t)b * (size_t)N * n;
    T *__restrict__ Ug = (T *)a.U + (size_t)b * (size_t)(N - 1) * m;
    T *Ks = lds, *xs = lds + MP * NP, *us = xs + NP;

    const int iu = lane % MP, hu = lane / MP;   // u row, column part
    const int ix = lane % NP, hx = lane / NP;   // x row, column part
    // TV: A_k, B_k rows are prefetched AD knots ahead (a ring rotated by register moves)
    constexpr int AD = TV ? LQRX_DP_TVAD : 1;
    T arow[JX], brow[PX], arow_n[AD][TV ? JX : 1], brow_n[AD][TV ? PX : 1];
    auto load_rows = [&](int kk, T *ar, T *br) {   // row ix of A_kk, B_kk (this lane's part)
        const T *Ak = Ag + (int64_t)(kk - 1) * sA, *Bk = Bg + (int64_t)(kk - 1) * sB;
        // per-knot (TV) loads: lane-derived offsets are laundered and kept 32-bit, so they
        // are recomputed per call instead of hoisted out of the knot loop as 24 live
        // 64-bit addresses (which spilled the whole time-varying kernel at 2 waves/SIMD)
        int lx = ix, lh = hx;
        if constexpr (TV) asm volatile("" : "+v"(lx), "+v"(lh));
#pragma unroll
        for (int t = 0; t < JX; ++t) {
            int j = lh * JX + t;
            ar[t] = (lx < n && j < n) ? Ak[lx + j * n] : (T)0;
        }
#pragma unroll
        for (int t = 0; t < PX; ++t) {
            int p = lh * PX + t;
            br[t] = (lx < n && p < m) ? Bk[lx + p * n] : (T)0;
        }
    };
    load_rows(1, arow, brow);
    if constexpr (TV) {
#pragma unroll
        for (int d = 0; d + 1 < AD; ++d)
            if (2 + d <= N - 1) load_rows(2 + d, arow_n[d], brow_n[d]);
    }
    const T *x0 = (const T *)a.x0 + (size_t)b * n;
    if (lane < NP) xs[lane] = (lane < n) ? x0[lane] : (T)0;
    if (lane < MP) us[lane] = (T)0;
    if (lane < n) Xg[lane] = x0[lane];

    T ring[DEPTH][KPL], dring[LIN ? DEPTH : 1];   // K_k (+ the feedforward d_k, lane < m)
    const T *Dg = LIN ? (const T *)a.d + (size_t)b * (size_t)(N - 1) * m : nullptr;
    auto issue = [&](int kk, T(&dst)[KPL]) {
#pragma unroll
        for (int s = 0; s < KPL; ++s) {
            size_t e = (size_t)lane + 64 * s;
            dst[s] = (kk <= N - 1 && e < mn) ? Kg[(size_t)(kk - 1) * mn + e] : (T)0;
        }
    };
    auto issue_d = [&](int kk, T &dst) {
        if constexpr (LIN) dst = (kk <= N - 1 && lane < m) ? Dg[(size_t)(kk - 1) * m + lane] : (T)0;
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        issue(1 + d, ring[d]);
        issue_d(1 + d, dring[LIN ? d : 0]);
    }
    __syncthreads();

    for (int k0 = 1; k0 <= N - 1; k0 += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int k = k0 + d;
            if (k <= N - 1) {
#pragma unroll
                for (int s = 0; s < KPL; ++s) {
                    size_t e = (size_t)lane + 64 * s;
                    if (e < mn) Ks[e] = ring[d][s];
                }
                issue(k + DEPTH, ring[d]);
                T dcur = (T)0;
                if constexpr (LIN) {
                    dcur = dring[d];
                    issue_d(k + DEPTH, dring[d]);
                }
                if constexpr (TV) {
                    if (k + AD <= N - 1) load_rows(k + AD, arow_n[AD - 1], brow_n[AD - 1]);   // AD knots ahead
                }
                __syncthreads();
                // u_i = −Σ_j K[i][j] x_j   (dynamic_programming.jl:68)
                T s0 = 0, s1 = 0;
#pragma unroll
                for (int t = 0; t < JU; t += 2) {
                    int j0 = hu * JU + t, j1 = j0 + 1;
                    if (j0 < n) s0 = fma(Ks[iu + j0 * m], xs[j0], s0);
                    if (t + 1 < JU && j1 < n) s1 = fma(Ks[iu + j1 * m], xs[j1], s1);
                }
                T su = s0 + s1;
#pragma unroll
                for (int o = MP; o < 64; o <<= 1) su += xor_shfl(su, (lane ^ o) << 2);
                if (lane < m) {
                    const T u = LIN ? -(su + dcur) : -su;   // u = −K x (− d)
                    us[lane] = u;
                    Ug[(size_t)(k - 1) * m + lane] = u;
                }
                __syncthreads();
                // x_{k+1} = A x_k + B u_k   (:69)
                T t0 = 0, t1 = 0;
#pragma unroll
                for (int t = 0; t < JX; t += 2) {
                    t0 = fma(arow[t], xs[hx * JX + t], t0);
                    if (t + 1 < JX) t1 = fma(arow[t + 1], xs[hx * JX + t + 1], t1);
                }
#pragma unroll
                for (int t = 0; t < PX; ++t) t1 = fma(brow[t], us[hx * PX + t], t1);
                T xn = t0 + t1;
#pragma unroll
                for (int o = NP; o < 64; o <<= 1) xn += __shfl_xor(xn, o);
                __syncthreads();
                if (lane < n) {
                    xs[lane] = xn;
                    Xg[(size_t)k * n + lane] = xn;
                }
                if constexpr (TV) {
#pragma unroll
                    for (int t = 0; t < JX; ++t) arow[t] = arow_n[0][t];
#pragma unroll
                    for (int t = 0; t < PX; ++t) brow[t] = brow_n[0][t];
#pragma unroll
                    for (int d = 0; d + 1 < AD; ++d) {
#pragma unroll
                        for (int t = 0; t < JX; ++t) arow_n[d][t] = arow_n[d + 1][t];
#pragma unroll
                        for (int t = 0; t < PX; ++t) brow_n[d][t] = brow_n[d + 1][t];
                    }
                }
                __syncthreads();
            }
        }
    }
}

// one global load the compiler's wait-count pass does not track (the caller waits by hand)
template <typename T, int OFF> __device__ __forceinline__ T gload_asm(const T *p);
template <> __device__ __forceinline__ double gload_asm<double, 0>(const double *p)
{
    double v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p));
    return v;
}
template <typename T, int OFF> __device__ __forceinline__ T gload_asm(const T *p)
{
    T v;
    if constexpr (sizeof(T) == 8)
        asm volatile("global_load_dwordx2 %0, %1, off offset:%2" : "=v"(v) : "v"(p), "n"(OFF));
    else
        asm volatile("global_load_dword %0, %1, off offset:%2" : "=v"(v) : "v"(p), "n"(OFF));
    return v;
}
template <> __device__ __forceinline__ float gload_asm<float, 0>(const float *p)
{
    float v;
    asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p));
    return v;
}
// dst[c] = p[c·STR bytes] for c < C (compile-time immediate offsets)
template <typename T, int C, int STR>
__device__ __forceinline__ void gload_run(T *dst, const T *p)
{
    if constexpr (C > 0) {
        gload_run<T, C - 1, STR>(dst, p);
        dst[C - 1] = gload_asm<T, (C - 1) * STR>(p);
    }
}
// s_waitcnt vmcnt(N) that the values r (and d) depend on: their consumers stay after it
template <int N, typename T, int C>
__device__ __forceinline__ void vm_wait_regs(T (&r)[C], T &d)
{
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(d) : "n"(N) : "memory");
#pragma unroll
    for (int c = 0; c < C; ++c) asm volatile("" : "+v"(r[c]));
}

// The same rollout for exact tile grids (n = 16·NT ∈ {16, 32, 64}, m = 16·MT; time-invariant A,
// B), restructured so that nothing but its arithmetic is left per knot: K_k goes from HBM
// straight into registers DEPTH knots ahead (no LDS staging, no exec-mask branches), in a lane
// map where lane l owns row iu = l mod MP of K_k and a contiguous run of CU columns, so
// u_i = −Σ K[i][j] x_j is one FMA chain per lane plus xor-shuffles over the SU = 64/MP lanes of
// the row; x_{k+1} = A x + B u with A, B rows in registers (lane l: row l mod NP, a
// contiguous column run); x and u pass between lanes through LDS, read as contiguous runs;
// the wave is its own workgroup, so wave-level ordering (wsync) replaces barriers.
template <typename T, int NT, int MT, int DEPTH, bool LIN>
__device__ __forceinline__ void dp_rollout_full(const DpArgs &a, int64_t b, T *lds, int lane)
{
    constexpr int NP = 16 * NT, MP = 16 * MT;
    constexpr int SU = 64 / MP, CU = NP / SU;          // lanes per K row, K columns per lane
    constexpr int SX = 64 / NP, CX = NP / SX, CB = MP / SX;   // lanes per x row; A, B columns per lane
    static_assert(64 % NP == 0 && 64 % MP == 0, "exact tile grids with 64 % n == 0");
    const int N = a.N;
    constexpr size_t mn = (size_t)MP * NP;
    const T *__restrict__ Kg = (const T *)a.K + (size_t)b * (size_t)(N - 1) * mn;
    const T *__restrict__ Ag = (const T *)a.A + (size_t)b * NP * NP;
    const T *__restrict__ Bg = (const T *)a.B + (size_t)b * NP * MP;
    T *__restrict__ Xg = (T *)a.X + (size_t)b * (size_t)N * NP;
    T *__restrict__ Ug = (T *)a.U + (size_t)b * (size_t)(N - 1) * MP;
    const T *Dg = LIN ? (const T *)a.d + (size_t)b * (size_t)(N - 1) * MP : nullptr;
    T *xs = lds, *us = lds + NP;
    const int iu = lane % MP, hu = lane / MP, ix = lane % NP, hx = lane / NP;
    T arow[CX], brow[CB];
#pragma unroll
    for (int c = 0; c < CX; ++c) arow[c] = Ag[ix + (size_t)(hx * CX + c) * NP];
#pragma unroll
    for (int c = 0; c < CB; ++c) brow[c] = Bg[ix + (size_t)(hx * CB + c) * NP];
    const T *x0 = (const T *)a.x0 + (size_t)b * NP;
    if (lane < NP) {
        const T v = x0[lane];
        xs[lane] = v;
        Xg[lane] = v;
    }
    // K_kk (knot kk = 1 … N−1; past the end: the last knot again, never used).  The loads are
    // inline asm, invisible to the compiler's wait-count pass, which would otherwise wait at
    // the loop header for the loads issued one knot earlier instead of DEPTH knots earlier;
    // the wait is placed by hand: per knot the wave issues KOPS memory ops (CU loads of K
    // (+1 of d), then the U and X stores), so knot k's slot is complete once at most
    // KOPS·(DEPTH−1) are outstanding (fewer in the first DEPTH knots: the bound below is the
    // smallest such count, i.e. a slight over-wait in the steady state)
    // (A K slot too large for the 6-bit vmcnt — n = 64, m = 32 — takes compiler-tracked loads.)
    // Not with linear terms: there the compiler copied an in-flight d register (the asm load's
    // destination, which it sees as already written) into another register before the hand
    // wait, so u_k now and then used the load's address bits (an intermittent wrong X/U in
    // tests/test_dp_linear_gpu.py::test_dp_linear_device_stream; the copy is visible in the
    // gfx950 assembly of dp_riccati_kernel<double,2,1,2,64,true>).  The LIN variants take
    // compiler-tracked loads, whose waits the compiler places itself.
    constexpr int VMW = (CU + (LIN ? 1 : 0)) * (DEPTH - 1);
    constexpr bool HAND = !LIN && VMW <= 63 && CU * MP * (int)sizeof(T) <= 4096;
    T ring[DEPTH][CU], dring[DEPTH];
    auto issue = [&](int kk, T (&dst)[CU], T &dd) __attribute__((always_inline)) {
        const T *Kk = Kg + (size_t)(min(kk, N - 1) - 1) * mn + iu + (size_t)hu * CU * MP;
        const T *Dk = LIN ? Dg + (size_t)(min(kk, N - 1) - 1) * MP + iu : nullptr;
        if constexpr (HAND) {
            gload_run<T, CU, MP * (int)sizeof(T)>(dst, Kk);
            if constexpr (LIN) dd = gload_asm<T, 0>(Dk);
        } else {
#pragma unroll
            for (int c = 0; c < CU; ++c) dst[c] = Kk[(size_t)c * MP];
            if constexpr (LIN) dd = *Dk;
        }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        dring[d] = (T)0;
        issue(1 + d, ring[d], dring[d]);
    }
    wsync_w();
    // one knot: slot d holds K_k (issued DEPTH knots earlier); NEXT: refill the slot with knot
    // k + DEPTH (the main loop) or not (the tail)
    auto knot = [&](int k, T (&rk)[CU], T &dk, bool next) __attribute__((always_inline)) {
        // u = −K_k x_k (− d_k)   (dynamic_programming.jl:68)
        T xu[CU];
#pragma unroll
        for (int c = 0; c < CU; ++c) xu[c] = xs[hu * CU + c];
        T s0 = (T)0, s1 = (T)0;
#pragma unroll
        for (int c = 0; c < CU; c += 2) {
            s0 = fma(rk[c], xu[c], s0);
            if (c + 1 < CU) s1 = fma(rk[c + 1], xu[c + 1], s1);
        }
        T su = s0 + s1;
#pragma unroll
        for (int o = MP; o < 64; o <<= 1) su += __shfl_xor(su, o);
        const T u = LIN ? -(su + dk) : -su;
        T dn = (T)0;
        if (next) issue(k + DEPTH, rk, LIN ? dk : dn);
        if (hu == 0) {
            us[iu] = u;
            Ug[(size_t)(k - 1) * MP + iu] = u;
        }
        wsync_w();
        // x_{k+1} = A x_k + B u_k   (:69)
        T t0 = (T)0, t1 = (T)0;
#pragma unroll
        for (int c = 0; c < CX; c += 2) {
            t0 = fma(arow[c], xs[hx * CX + c], t0);
            if (c + 1 < CX) t1 = fma(arow[c + 1], xs[hx * CX + c + 1], t1);
        }
#pragma unroll
        for (int c = 0; c < CB; ++c) t1 = fma(brow[c], us[hx * CB + c], t1);
        T xn = t0 + t1;
#pragma unroll
        for (int o = NP; o < 64; o <<= 1) xn += xor_shfl(xn, (lane ^ o) << 2);
        wsync_w();
        if (hx == 0) {
            xs[ix] = xn;
            Xg[(size_t)k * NP + ix] = xn;
        }
        wsync_w();
    };
    // Whole groups of DEPTH knots: every slot is waited for, consumed and refilled on every
    // path through the loop body, so the hand bound VMW holds on every path the compiled code
    // has (tests/isa_vmcnt.py checks it on the gfx950 assembly; a body that skipped knots past
    // N−1 had compiled paths with fewer loads between a slot's issue and its wait).
    int k0 = 1;
    for (; k0 + DEPTH - 1 <= N - 1; k0 += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            if constexpr (HAND) vm_wait_regs<VMW>(ring[d], dring[d]);
            knot(k0 + d, ring[d], dring[d], true);
        }
    }
    // the last < DEPTH knots: their K is in the ring already; drain every load first (also
    // the clamped refills past N−1, so no load is in flight when the rollout returns)
    if constexpr (HAND) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) vm_wait_regs<0>(ring[d], dring[d]);
    }
#pragma unroll
    for (int d = 0; d < DEPTH - 1; ++d)
        if (k0 + d <= N - 1) knot(k0 + d, ring[d], dring[d], false);
}

// Kernel variants (compile-time VAR bits):
//   (0)        : the symmetric fast form: APBᵀ = PBᵀA equals G = BᵀPA for symmetric P,
//                so P_ = Q + AᵀPA − GᵀK; P_ is symmetric, so only its lower tiles are
//                computed and the upper ones mirrored (LDS transpose); Q lives in an LDS
//                image and is read into the P_ accumulators each knot.  (The reference op
//                order — explicit APB, all n×n tiles — was a round-1 A/B variant; it was
//                never selectable through the ABI and is gone: parity is checked against
//                the oracle, which keeps the reference order.)
//   VAR_NOSOLVE / VAR_NOROLL / VAR_NOKSTORE : diagnostic ablations (tools/dp_ablate).
//   VAR_TV     : time-varying A_k, B_k, Q_k, R_k (ABI knot strides 1):
//                knot k-1's A, B, R are loaded into the same registers right after knot k's
//                last product that reads them (the load hides behind the rest of the knot);
//                Q_k is loaded from global straight into the P_ accumulators.
//   VAR_LIN    : linear cost terms (lqrx_dp_solve_linear), alone (time-invariant problem) or
//                with VAR_TV: K = XᵀG's companion d = Xᵀ(r + Bᵀp) and p ← q + Aᵀp − Gᵀd
//                (Gᵀ = APB for symmetric P) on the VALU — the vectors are exchanged through
//                a small LDS image (lin_* helpers below).
enum : int { VAR_NOSOLVE = 2, VAR_NOROLL = 4, VAR_NOKSTORE = 8, VAR_SWEEPONLY = 16, VAR_TV = 32,
             VAR_LIN = 64 };

// Vector products with register tiles (VAR_LIN).  A vector v is read from its LDS image in
// "row layout" (lane l, slot [i][r] = v[16i + Tile::row(l, r)], the rows a C-layout tile's
// lane holds); Mᵀv is then a per-lane FMA chain over those rows, summed over the four row
// groups (lanes l, l^16, l^32, l^48), and lands in "column layout": lane l holds
// (Mᵀv)[16j + (l & 15)] for output tile j.
template <typename T, int RT>
__device__ __forceinline__ void lin_rows(T (&v)[RT][4], const T *img, int lane)
{
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[i][r] = img[16 * i + Tile<T>::row(lane, r)];
}
template <typename T, int RT, int CT>
__device__ __forceinline__ void lin_tn(T (&y)[CT], const typename Tile<T>::acc (&M)[RT][CT], const T (&v)[RT][4])
{
#pragma unroll
    for (int j = 0; j < CT; ++j)
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) y[j] = fma(M[i][j][r], v[i][r], y[j]);
}
template <typename T>
__device__ __forceinline__ T lin_rowsum(T x)
{
    x += __shfl_xor(x, 16);
    return x + __shfl_xor(x, 32);
}

template <typename T, int NT, int MT, int WAVES, int VAR, bool FULL>
__global__ __launch_bounds__(64, WAVES) void dp_riccati_kernel(const DpArgs a)
{
    using C = DpCfg<T, NT, MT>;
    using acc = typename Tile<T>::acc;
    constexpr int MP = C::MP, CS = C::CS;
    constexpr bool TV = (VAR & VAR_TV) != 0, LIN = (VAR & VAR_LIN) != 0;
    constexpr int NP = C::NP;
    __shared__ T lds[C::LDS_ELEMS];
    // p (NP), then w / d (MP); time-invariant q (NP), r (MP) images after them
    __shared__ T vimg[LIN ? (TV ? NP + MP : 2 * (NP + MP)) : 1];
    // Q (time-invariant, read every knot as the P_ accumulator start) lives in LDS for the
    // horizon: an LDS read per element instead of an L2 round trip per knot
    __shared__ T qimg[TV ? 1 : C::QIMG];

    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    if (b >= a.batch) return;
    const int n = a.n, m = a.m, N = a.N;
    const size_t nn = (size_t)n * n, nm = (size_t)n * m, mm = (size_t)m * m;
    // per-trajectory bases; time-varying fields hold N-1 knots (knot k at index k-1)
    const size_t kAB = (TV && a.tv_AB) ? (size_t)(N - 1) : 1, kQR = (TV && a.tv_QR) ? (size_t)(N - 1) : 1;
    size_t sA = kAB > 1 ? nn : 0, sB = kAB > 1 ? nm : 0, sQ = kQR > 1 ? nn : 0, sR = kQR > 1 ? mm : 0;
#if LQRX_DP_TVABL
    // ablation (tools only): bit 1 = Q_k, bit 2 = A_k/B_k/R_k re-read from knot 1 (cache-resident)
    if (LQRX_DP_TVABL & 1) sQ = 0;
    if (LQRX_DP_TVABL & 2) sA = sB = sR = 0;
#endif
    const T *Ab = (const T *)a.A + b * nn * kAB, *Bb = (const T *)a.B + b * nm * kAB;
    const T *Qb = (const T *)a.Q + b * nn * kQR, *Rb = (const T *)a.R + b * mm * kQR;
    const T *Qg = Qb;

    acc At[NT][NT], Bt[NT][MT], Rt[MT][MT], P[NT][NT];
    const size_t k0 = TV ? (size_t)(N - 2) : 0;                 // first backward knot k = N-1
    tiles_load<T, NT, NT, FULL>(At, Ab + k0 * sA, n, n, n, lane, false);
    tiles_load<T, NT, MT, FULL>(Bt, Bb + k0 * sB, n, m, n, lane, false);
    tiles_load<T, MT, MT, FULL>(Rt, Rb + k0 * sR, m, m, m, lane, true);
    tiles_load<T, NT, NT, FULL>(P, (const T *)a.Qf + b * nn, n, n, n, lane, false); // :58 P = Qf
    if constexpr (!TV) {
        // zero-padded NP×NP image of Q (padding rows/cols 0, as tiles_load_lower)
        for (int e = lane; e < C::NP * C::NP; e += 64) {
            const int i = e % C::NP, j = e / C::NP;
            qimg[i + j * C::QCS] = (i < n && j < n) ? Qg[i + (size_t)j * n] : (T)0;
        }
        __syncthreads();
    }

    T *Pall = a.p_all ? (T *)a.P + (size_t)b * nn * N : nullptr;
    if (Pall) tiles_store<T, NT, NT>(P, Pall + (size_t)(N - 1) * nn, n, n, n, lane);
    T *Kb = (T *)a.K + (size_t)b * (size_t)(N - 1) * nm;
    int info = 0;
    // linear terms: q_k, r_k (knot stride with Q, R), outputs d_k and p (p_1 or every p_k)
    const size_t sq = (LIN && a.tv_QR) ? (size_t)n : 0, sr = (LIN && a.tv_QR) ? (size_t)m : 0;
    const T *qg = LIN ? (const T *)a.q + (size_t)b * n * kQR : nullptr;
    const T *rg = LIN ? (const T *)a.r + (size_t)b * m * kQR : nullptr;
    T *dg = LIN ? (T *)a.d + (size_t)b * (size_t)(N - 1) * m : nullptr;
    T *pallv = (LIN && a.p_all) ? (T *)a.p + (size_t)b * (size_t)N * n : nullptr;
    if constexpr (LIN) {
        const T *qf = (const T *)a.qf + (size_t)b * n;
        for (int i = lane; i < NP; i += 64) {
            const T v = i < n ? qf[i] : (T)0;        // p = qf
            vimg[i] = v;
            if (pallv && i < n) pallv[(size_t)(N - 1) * n + i] = v;
            if constexpr (!TV) vimg[NP + MP + i] = i < n ? qg[i] : (T)0;
        }
        if constexpr (!TV) {
            for (int i = lane; i < MP; i += 64) vimg[2 * NP + MP + i] = i < m ? rg[i] : (T)0;
        }
        __syncthreads();
    }
    acc Xi[MT][MT], Xp[MT][MT], Id[MT][MT];     // E⁻¹ of the last two knots, identity tiles
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                Id[i][j][r] = (i == j && Tile<T>::row(lane, r) == tcol(lane)) ? (T)1 : (T)0;
                Xi[i][j][r] = (T)0;
                Xp[i][j][r] = (T)0;
            }

    for (int k = N - 1; k >= 1; --k) { // :61
        acc PB[NT][MT], E[MT][MT], PA[NT][NT], G[MT][NT], Pn[NT][NT];
        // column layout; time-varying: issued ahead of the MFMAs, time-invariant: read from
        // the LDS images where they are used (no registers held across the knot)
        T qv[LIN ? NT : 1], rv[LIN ? MT : 1];
        auto lin_qr_lds = [&]() {
            if constexpr (LIN && !TV) {
#pragma unroll
                for (int j = 0; j < NT; ++j) qv[j] = vimg[NP + MP + 16 * j + tcol(lane)];
#pragma unroll
                for (int j = 0; j < MT; ++j) rv[j] = vimg[2 * NP + MP + 16 * j + tcol(lane)];
            }
        };
        if constexpr (LIN && TV) {
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int i = 16 * j + tcol(lane);
                qv[j] = i < n ? qg[(size_t)(k - 1) * sq + i] : (T)0;
            }
#pragma unroll
            for (int j = 0; j < MT; ++j) {
                const int i = 16 * j + tcol(lane);
                rv[j] = i < m ? rg[(size_t)(k - 1) * sr + i] : (T)0;
            }
        }
        tiles_zero<T, NT, MT>(PB);
        mma_tn<T, NT, NT, MT>(PB, P, Bt);                          // :38 PB = P B
        tiles_zero<T, NT, NT>(PA);
        mma_tn<T, NT, NT, NT>(PA, P, At);                          // :40 PA = P A
        if constexpr (TV) {
            tiles_load_lower<T, NT, FULL>(Pn, Qb + (size_t)(k - 1) * sQ, n, n, lane);
#if LQRX_DP_TVWAIT
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        }
        else tiles_lower_from_lds<T, NT>(Pn, qimg, C::QCS, lane);       // P_ ← Q (lower tiles)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < MT; ++j) E[i][j] = Rt[i][j];
        mma_tn<T, NT, MT, MT>(E, Bt, PB);                          // :39 E = R + B'PB
        tiles_zero<T, MT, NT>(G);
        mma_tn<T, NT, MT, NT>(G, Bt, PA);                          // :41 K = B'PA
        mma_tn_lower<T, NT, NT>(Pn, At, PA);                       // :51 Q + A'PA (lower)
        // linear terms, first half (time-varying: before A_k, B_k leave the tiles; time-
        // invariant: after the solve, where fewer registers are live): w = r + Bᵀp, Aᵀp partials
        T w[LIN ? MT : 1], ap[LIN ? NT : 1];
        auto lin_first = [&]() {
            if constexpr (LIN) {
                T prow[NT][4];
                lin_rows<T, NT>(prow, vimg, lane);
#pragma unroll
                for (int j = 0; j < MT; ++j) w[j] = (T)0;
#pragma unroll
                for (int j = 0; j < NT; ++j) ap[j] = (T)0;
                lin_tn<T, NT, MT>(w, Bt, prow);
                lin_tn<T, NT, NT>(ap, At, prow);
#pragma unroll
                for (int j = 0; j < MT; ++j) w[j] = rv[j] + lin_rowsum(w[j]);
            }
        };
        if constexpr (LIN && TV) lin_first();
        if constexpr (TV) {
            // knot k's A, B, R are consumed: bring in knot k-1's (lands during the solve)
            if (k > 1) {
                tiles_load<T, NT, NT, FULL>(At, Ab + (size_t)(k - 2) * sA, n, n, n, lane, false);
                tiles_load<T, NT, MT, FULL>(Bt, Bb + (size_t)(k - 2) * sB, n, m, n, lane, false);
                tiles_load<T, MT, MT, FULL>(Rt, Rb + (size_t)(k - 2) * sR, m, m, m, lane, true);
            }
        }

        // :42 chol_solve!(E, K) — potrf 'U' + potrs 'U', as K = E⁻¹G with X ≈ E⁻¹:
        //  * warm start: Newton–Schulz from the previous knot's inverse, all MFMA
        //      R = I − EᵀX (neg-A modifier, C = I),  X ← X + XᵀR   (quadratic; no symmetry
        //      needed: X⁺ − E⁻¹ = −ΔᵀEΔ), accepted at working precision (see NsTol)
        //  * the first knot, and any knot whose iteration does not converge, run the exact
        //    LDLᵀ sweep of [E | I] (potrf's pivot test → info) and X = Wᵀ D⁻¹ W.
        acc Kt[MT][NT];
        if constexpr ((VAR & VAR_NOSOLVE) != 0) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j) Kt[i][j] = G[i][j] * (T)1e-3 + E[0][0] * (T)1e-9;
        } else {
            bool have = false;
            if constexpr ((VAR & VAR_SWEEPONLY) == 0) {
                if (k < N - 1) {
                    // warm start: linear extrapolation 2X_{k+1} − X_{k+2} once both exist
                    acc X0[MT][MT];
#pragma unroll
                    for (int i = 0; i < MT; ++i)
#pragma unroll
                        for (int j = 0; j < MT; ++j) {
                            X0[i][j] = Xi[i][j];
                            Xi[i][j] = (T)2 * Xi[i][j] - Xp[i][j];   // = X_{k+1} at k = N−2 (Xp = Xi there)
                        }
                    have = !a.ns_off && ns_refine<T, MT>(Xi, E, Id, lane);
#pragma unroll
                    for (int i = 0; i < MT; ++i)
#pragma unroll
                        for (int j = 0; j < MT; ++j) Xp[i][j] = X0[i][j];
                }
            }
            if (!have) {
                tiles_to_lds<T, MT, MT>(E, lds, CS, lane);
                __syncthreads();
                bool ok = aug_ldl_forward<T, MP, 0, CS, LQRX_DP_BCAST>(lds, lane);
                if (!ok && info == 0) info = k;
                __syncthreads();
                acc Wt[MT][MT], DW[MT][MT];
                tiles_from_lds<T, MT, MT>(Wt, lds + MP * CS, CS, lane);
                const T *rinv = lds + (2 * MP) * CS + 64;
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        T sc = rinv[i * 16 + Tile<T>::row(lane, r)];         // D⁻¹ row scale
#pragma unroll
                        for (int j = 0; j < MT; ++j) DW[i][j][r] = Wt[i][j][r] * sc;
                    }
                __syncthreads();
                tiles_zero<T, MT, MT>(Xi);
                mma_tn<T, MT, MT, MT>(Xi, Wt, DW);                      // X = Wᵀ D⁻¹ W = E⁻¹
                if (k == N - 1) {
                    // no extrapolation into knot N−2 (only one inverse exists): 2X − Xp = X
#pragma unroll
                    for (int i = 0; i < MT; ++i)
#pragma unroll
                        for (int j = 0; j < MT; ++j) Xp[i][j] = Xi[i][j];
                }
            }
            tiles_zero<T, MT, NT>(Kt);
            mma_tn<T, MT, MT, NT>(Kt, Xi, G);                          // K = XᵀG = E⁻¹G
            if constexpr ((VAR & VAR_NOKSTORE) == 0)
                tiles_store<T, MT, NT, FULL>(Kt, Kb + (size_t)(k - 1) * nm, m, n, m, lane);
            if constexpr (LIN) {
                if constexpr (!TV) {
                    lin_qr_lds();
                    lin_first();
                }
                // second half: d = Xᵀw (the companion of K = XᵀG) ;  p ← q + Aᵀp − Gᵀd
                T dv[MT], gd[NT];
#pragma unroll
                for (int j = 0; j < MT; ++j) dv[j] = (T)0;
#pragma unroll
                for (int j = 0; j < NT; ++j) gd[j] = (T)0;
#pragma unroll
                for (int j = 0; j < MT; ++j)
                    if (lane < 16) vimg[NP + 16 * j + lane] = w[j];
                __syncthreads();
                T wrow[MT][4];
                lin_rows<T, MT>(wrow, vimg + NP, lane);
                lin_tn<T, MT, MT>(dv, Xi, wrow);
                __syncthreads();                       // w read by every lane before d lands
#pragma unroll
                for (int j = 0; j < MT; ++j) {
                    dv[j] = lin_rowsum(dv[j]);
                    const int i = 16 * j + lane;
                    if (lane < 16) {
                        vimg[NP + i] = dv[j];
                        if (i < m) dg[(size_t)(k - 1) * m + i] = dv[j];
                    }
                }
                __syncthreads();
                T drow[MT][4];
                lin_rows<T, MT>(drow, vimg + NP, lane);
                lin_tn<T, MT, NT>(gd, G, drow);
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const T pn = qv[j] + lin_rowsum(ap[j]) - lin_rowsum(gd[j]);
                    const int i = 16 * j + lane;
                    if (lane < 16) {
                        vimg[i] = pn;
                        if (pallv && i < n) pallv[(size_t)(k - 1) * n + i] = pn;
                    }
                }
                __syncthreads();
            }
        }
        mma_tn_lower<T, MT, NT, true>(Pn, G, Kt);                  // :50-51 − GᵀK (= APB K)
        tiles_symmetrize_lower<T, NT>(Pn, lds, lane);              // P_ exactly symmetric
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) P[i][j] = Pn[i][j];
        if (Pall) tiles_store<T, NT, NT>(P, Pall + (size_t)(k - 1) * nn, n, n, n, lane);
    }
    if (!a.p_all) tiles_store<T, NT, NT>(P, (T *)a.P + (size_t)b * nn, n, n, n, lane);
    if (a.info && lane == 0) a.info[b] = info;
    if constexpr (LIN) {
        if (!a.p_all && lane < n) ((T *)a.p)[(size_t)b * n + lane] = vimg[lane];   // p_1
    }

    if constexpr ((VAR & VAR_NOROLL) == 0) {
        // make this wave's K stores visible to its own (other-lane) rollout loads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#if LQRX_DP_ROLL_FULL
        if constexpr (FULL && !TV && (64 % (16 * NT)) == 0 && (64 % (16 * MT)) == 0)
            dp_rollout_full<T, NT, MT, LQRX_DP_KD, LIN>(a, b, lds, lane);
        else
#endif
            dp_rollout<T, NT, MT, TV ? LQRX_DP_TVKD : LQRX_DP_KD, TV, LIN>(a, b, lds, lane);
    }
}

// ------------------------------------------------------------------ four waves per trajectory
// dp_wg4_kernel<T, MT, VAR> — fp64 n = 64, m = 16·MT: the shape whose tile grid does not fit one
// wave (A alone is 128 fp64 registers; the one-wave kernel spills ~2–3 KB per lane there).  One
// 256-thread workgroup per trajectory, one wave per SIMD, the same fast form and the same
// Newton–Schulz / exact-sweep inverse as dp_riccati_kernel, with the knot's products split by the
// n-dimension's 16-column tiles (wave w ↔ tile column w):
//   :38  PB[w][:] = P[:, w]ᵀ·B            (P tiles from the LDS image, B from its image)
//   :40  PA[:, w] = Pᵀ·A[:, w]             (all of P from LDS, A[:, w] in registers)
//   :39  E tile (w mod MT, w / MT) = R + BᵀPB   (PB from its LDS image; one tile per wave)
//   :41  G[:, w] = Bᵀ·PA[:, w]             (registers only; also to an LDS image)
//   :42  X ≈ E⁻¹ — m = 32, time-invariant: on wave 3 alone, published with its verdict through
//        the PB image while waves 0–2 form the K-independent half Q + A[:, i]ᵀPA[:, w] of their P_
//        tiles; otherwise in every wave, the four verdicts AND-ed — then K[:, w] = XᵀG[:, w] to sol.K
//   :51  P_ tiles (i, w), i from wave w's row list — the ten tiles of the symmetric 4×4 grid
//        as 3, 3, 3, 1 (inverse on wave 3) or 3, 3, 2, 2 per wave: Q + A[:, i]ᵀPA[:, w] −
//        G[:, i]ᵀK[:, w], written to the P image at (i, w) and mirrored to (w, i) (diagonal tiles
//        from their lower triangle), so the image stays exactly symmetric as
//        tiles_symmetrize_lower keeps the one-wave P.
// Four workgroup barriers per knot (after PB/PA, after E/G, the inverse's verdict (and X), after
// P_).  A lives in an LDS image (the P_ rows' A columns are read from it), A[:, w] also in
// registers; B, Q in images; R's E tile in registers.
// VAR_TV (constrained_problem.jl:3-4: per-knot A_k, B_k, Q_k, R_k): A is double-buffered in LDS
// (the time-invariant Q image's space — Q_k's P_ tiles come straight from HBM into the P_
// accumulators); knot k−1's A, B and R are requested at the top of knot k and land in LDS after
// the last reader of their buffer (A: the other buffer, after PB/PA; B: after B2; R: registers).
// VAR_LIN (lqrx_dp_solve_linear): w = r + Bᵀp (every wave, beside PB), d = Xᵀw (every wave, its
// own X), p ← q + Aᵀp − Gᵀd for rows 16w…16w+15 (A[:, w], G[:, w] are the wave's own tiles);
// p is double-buffered in LDS, w and d pass from column to row layout through per-wave slots.
// The rollout (:66-70): dp_rollout_wg4 on all four waves (an LQRX_WG4_ROLL4=0 build runs the
// time-invariant one as dp_rollout_full on wave 0: 234.1 vs 224.4 ms at n=64 m=32 N=512 B=8192).
// The Newton–Schulz step split over the waves (wg4_ns_split, LQRX_WG4_NS_SPLIT=1) measured
// slower (247.5 vs 234.1 ms: one more barrier per step and 224 B of spills) and is off.
#ifndef LQRX_WG4_NS_SPLIT
#define LQRX_WG4_NS_SPLIT 0   // 1: the Newton–Schulz step split over the four waves (m = 32; A/B — measured slower)
#endif
#ifndef LQRX_WG4_NS_ONE
#define LQRX_WG4_NS_ONE 1     // m = 32, time-invariant: the inverse on wave 3, the others' P_ A-parts meanwhile (0: A/B)
#endif
#ifndef LQRX_WG4_ROLL4
#define LQRX_WG4_ROLL4 1      // time-invariant four-wave kernel: the four-wave rollout (0: wave 0 alone, A/B)
#endif
template <typename T, int MT, int VAR>
struct Wg4Cfg {
    static constexpr bool TV = (VAR & VAR_TV) != 0, LIN = (VAR & VAR_LIN) != 0;
    static constexpr int NT = 4, NP = 64, MP = 16 * MT;
    // odd column strides: the compiler pairs a tile's rows into ds_read2_b64 / ds_write_b64, whose
    // 16-lane groups bank by (a/4) mod 32 — at an even stride (NP + 2) columns c and c + 8 of a tile
    // shared banks (2-way; SQ_LDS_BANK_CONFLICT ≈ a quarter of the kernel's cycles)
    static constexpr int PL = NP + 1;                    // P, Q, A, B images
    static constexpr int CS = MP + 1;                    // PB / E / G images, aug sweep
    static constexpr int P_EL = NP * PL;
    static constexpr int AUG = 2 * MP * CS + 64 + MP;   // [E | I] sweep image + row/rinv
    static constexpr int PB_EL = (MP * PL > AUG ? MP * PL : AUG);   // PB (NP × MP, stride PL) | the sweep image
    static constexpr int E_EL = MP * CS, G_EL = NP * CS;
    static constexpr int B_EL = MP * PL;                                 // B image (NP × MP)
    static constexpr int V_EL = LIN ? 2 * NP + 8 * MP : 0;               // p (×2), per-wave w, d
    static constexpr int LDS = 3 * P_EL + B_EL + PB_EL + E_EL + G_EL + V_EL + 8;   // P, Q | A₂, A, B images
    static_assert(LDS * sizeof(T) <= 160 * 1024, "dp_wg4_kernel LDS");
};
// row tile of wave w's t-th P_ tile (column tile w), −1: none
__host__ __device__ constexpr int wg4_pn_row(int w, int t)
{
    constexpr int tab[4][3] = {{0, 1, 2}, {1, 2, 3}, {2, 3, -1}, {3, 0, -1}};
    return tab[w][t];
}
// the same ten tiles when wave 3 runs the knot's Newton–Schulz inverse alone (wg4 "NS on one
// wave", m = 32): 3, 3, 3, 1 — each pair {i, j} is formed by one of its two column waves
__host__ __device__ constexpr int wg4_pn_row1(int w, int t)
{
    constexpr int tab[4][3] = {{0, 1, 3}, {1, 2, 3}, {2, 0, 3}, {3, -1, -1}};
    return tab[w][t];
}

template <typename T>
__device__ __forceinline__ typename Tile<T>::acc wg4_tload(const T *X, int ld, int lane)
{
    typename Tile<T>::acc c;
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] = X[Tile<T>::row(lane, r) + tcol(lane) * ld];
    return c;
}
template <typename T>
__device__ __forceinline__ void wg4_tstore(T *X, int ld, const typename Tile<T>::acc &c, int lane)
{
#pragma unroll
    for (int r = 0; r < 4; ++r) X[Tile<T>::row(lane, r) + tcol(lane) * ld] = c[r];
}
// D += Mᵀ·Y (one 16×16×16 tile product, 4 MFMAs)
template <typename T, bool NEG = false>
__device__ __forceinline__ void wg4_mtn(typename Tile<T>::acc &D, const typename Tile<T>::acc &M,
                                        const typename Tile<T>::acc &Y)
{
#pragma unroll
    for (int r = 0; r < 4; ++r) D = NEG ? Tile<T>::mma_nega(M[r], Y[r], D) : Tile<T>::mma(M[r], Y[r], D);
}
// y += Mᵀv for one tile M (rows 16i…, this lane's column) and v in row layout (lin_rows)
template <typename T>
__device__ __forceinline__ T wg4_vtn(T y, const typename Tile<T>::acc &M, const T (&v)[4])
{
#pragma unroll
    for (int r = 0; r < 4; ++r) y = fma(M[r], v[r], y);
    return y;
}

// Forward rollout (dynamic_programming.jl:66-70) on the four waves of dp_wg4_kernel: wave w owns
// rows 16w…16w+15 of x_{k+1} = A_k x_k + B_k u_k (lane l: row 16w + (l & 15), column quarter l >> 4
// of A's and B's columns, summed by two xor-shuffles); every wave forms the whole
// u_k = −K_k x_k (− d_k) itself (lane l: row l mod MP of K_k, a contiguous run of its columns), so
// the only workgroup barrier per knot publishes x_{k+1} (a double-buffered LDS vector).  K_k, d_k
// and — time-varying — the wave's rows of A_k, B_k are requested one knot ahead.
template <typename T, int MT, bool TV, bool LIN>
__device__ __forceinline__ void dp_rollout_wg4(const DpArgs &a, int64_t b, T *lds, int w, int lane)
{
    constexpr int NP = 64, MP = 16 * MT;
    constexpr int SU = 64 / MP, CU = NP / SU;        // lanes per K row, K columns per lane
    constexpr int CA = NP / 4, CB = MP / 4;          // A, B columns per lane
    const int N = a.N;
    constexpr size_t mn = (size_t)MP * NP;
    const bool tvab = TV && a.tv_AB;
    const int64_t sA = tvab ? (int64_t)NP * NP : 0, sB = tvab ? (int64_t)NP * MP : 0;
    const T *__restrict__ Kg = (const T *)a.K + (size_t)b * (size_t)(N - 1) * mn;
    const T *__restrict__ Ag = (const T *)a.A + (size_t)b * NP * NP * (tvab ? (size_t)(N - 1) : 1);
    const T *__restrict__ Bg = (const T *)a.B + (size_t)b * NP * MP * (tvab ? (size_t)(N - 1) : 1);
    T *__restrict__ Xg = (T *)a.X + (size_t)b * (size_t)N * NP;
    T *__restrict__ Ug = (T *)a.U + (size_t)b * (size_t)(N - 1) * MP;
    const T *Dg = LIN ? (const T *)a.d + (size_t)b * (size_t)(N - 1) * MP : nullptr;
    T *xs = lds, *us = lds + 2 * NP + w * MP;        // x_k double-buffered; this wave's u_k
    const int iu = lane % MP, hu = lane / MP;
    const int ix = 16 * w + (lane & 15), hx = lane >> 4;
    T ar[CA], br[CB], arn[TV ? CA : 1], brn[TV ? CB : 1];
    auto load_ab = [&](int kk, T *ra, T *rb) __attribute__((always_inline)) {
        const T *Ak = Ag + (int64_t)(kk - 1) * sA + ix + (size_t)hx * CA * NP;
        const T *Bk = Bg + (int64_t)(kk - 1) * sB + ix + (size_t)hx * CB * NP;
#pragma unroll
        for (int c = 0; c < CA; ++c) ra[c] = Ak[(size_t)c * NP];
#pragma unroll
        for (int c = 0; c < CB; ++c) rb[c] = Bk[(size_t)c * NP];
    };
    T kr[CU], krn[CU], dr = (T)0, drn = (T)0;
    auto load_k = [&](int kk, T *rk, T &dd) __attribute__((always_inline)) {
        const T *Kk = Kg + (size_t)(kk - 1) * mn + iu + (size_t)hu * CU * MP;
#pragma unroll
        for (int c = 0; c < CU; ++c) rk[c] = Kk[(size_t)c * MP];
        if constexpr (LIN) dd = Dg[(size_t)(kk - 1) * MP + iu];
    };
    load_ab(1, ar, br);
    load_k(1, kr, dr);
    if (N - 1 >= 2) {
        load_k(2, krn, drn);
        if constexpr (TV) load_ab(2, arn, brn);
    }
    const T *x0 = (const T *)a.x0 + (size_t)b * NP;
    if (w == 0) {
        const T v = x0[lane];
        xs[NP + lane] = v;                           // x_1 in buffer 1 (knot k reads buffer k & 1)
        Xg[lane] = v;
    }
    __syncthreads();
    for (int k = 1; k <= N - 1; ++k) {
        const T *xc = xs + (k & 1) * NP;
        // u = −K_k x_k (− d_k)   (dynamic_programming.jl:68)
        T s0 = (T)0, s1 = (T)0;
#pragma unroll
        for (int c = 0; c < CU; c += 2) {
            s0 = fma(kr[c], xc[hu * CU + c], s0);
            s1 = fma(kr[c + 1], xc[hu * CU + c + 1], s1);
        }
        T su = s0 + s1;
#pragma unroll
        for (int o = MP; o < 64; o <<= 1) su += xor_shfl(su, (lane ^ o) << 2);
        const T u = LIN ? -(su + dr) : -su;
#pragma unroll
        for (int c = 0; c < CU; ++c) kr[c] = krn[c];
        dr = drn;
        if (k + 2 <= N - 1) load_k(k + 2, krn, drn);
        if (hu == 0) {
            us[iu] = u;
            if (w == 0) Ug[(size_t)(k - 1) * MP + iu] = u;
        }
        wsync_w();
        // x_{k+1} = A_k x_k + B_k u_k   (:69), rows 16w…16w+15
        T t0 = (T)0, t1 = (T)0;
#pragma unroll
        for (int c = 0; c < CA; c += 2) {
            t0 = fma(ar[c], xc[hx * CA + c], t0);
            t1 = fma(ar[c + 1], xc[hx * CA + c + 1], t1);
        }
#pragma unroll
        for (int c = 0; c < CB; ++c) t1 = fma(br[c], us[hx * CB + c], t1);
        T xn = t0 + t1;
        xn += xor_shfl(xn, (lane ^ 16) << 2);
        xn += xor_shfl(xn, (lane ^ 32) << 2);
        if constexpr (TV) {
#pragma unroll
            for (int c = 0; c < CA; ++c) ar[c] = arn[c];
#pragma unroll
            for (int c = 0; c < CB; ++c) br[c] = brn[c];
            if (k + 2 <= N - 1) load_ab(k + 2, arn, brn);
        }
        if (lane < 16) {
            xs[((k + 1) & 1) * NP + ix] = xn;
            Xg[(size_t)k * NP + ix] = xn;
        }
        __syncthreads();
    }
}

// Newton–Schulz on the four waves (MT = 2, ns_refine's step split by output tile): wave w owns
// tile (w & 1, w >> 1) of R = I − EᵀX and of X + XᵀR; the residual tiles and their magnitude keys
// meet in LDS (rimg, keys), the new X in ximg — every wave reads the same four keys, so the
// verdict is workgroup-uniform by construction, and each wave issues a quarter of the refinement
// (16 instead of 64 MFMAs per step).  X: the full inverse in every wave, in and out.
template <typename T, int MT>
__device__ __forceinline__ bool wg4_ns_split(typename Tile<T>::acc (&X)[MT][MT], const T *eimg,
                                             T *rimg, T *ximg, int *keys, int ld, int w, int lane)
{
    static_assert(MT == 2, "one output tile per wave");
    using acc = typename Tile<T>::acc;
    const int ti = w & 1, tj = w >> 1;
    for (int it = 0; it < NsTol<T>::it; ++it) {
        acc R;
#pragma unroll
        for (int r = 0; r < 4; ++r) R[r] = (ti == tj && Tile<T>::row(lane, r) == tcol(lane)) ? (T)1 : (T)0;
#pragma unroll
        for (int l = 0; l < MT; ++l)                                               // R = I − EᵀX
            wg4_mtn<T, true>(R, wg4_tload(eimg + 16 * l + 16 * ti * ld, ld, lane), X[l][tj]);
        int key = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) key = max(key, mag_key(R[r]));
        key = wave_max_uniform_i(key);
        wg4_tstore(rimg + 16 * ti + 16 * tj * ld, ld, R, lane);
        if (lane == 0) keys[w] = key;
        __syncthreads();
        key = max(max(keys[0], keys[1]), max(keys[2], keys[3]));
        const T rho = (T)(16 * MT) * key_bound(key, (T)0);
        if (rho <= NsTol<T>::v) return true;                    // X already at working precision
        if (!(rho < (T)1)) return false;                        // no contraction (or NaN): exact sweep
        acc Xn = X[ti][tj];
#pragma unroll
        for (int l = 0; l < MT; ++l) wg4_mtn<T>(Xn, X[l][ti], wg4_tload(rimg + 16 * l + 16 * tj * ld, ld, lane));
        wg4_tstore(ximg + 16 * ti + 16 * tj * ld, ld, Xn, lane);   // X + XᵀR
        __syncthreads();
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < MT; ++j) X[i][j] = wg4_tload(ximg + 16 * i + 16 * j * ld, ld, lane);
        if (rho <= NsTol<T>::one_step) return true;             // new residual ≤ cond·ρ² ≪ eps
    }
    return false;
}

template <typename T, int MT, int VAR>
__global__ __launch_bounds__(256, 1) void dp_wg4_kernel(const DpArgs a)
{
    using C = Wg4Cfg<T, MT, VAR>;
    using acc = typename Tile<T>::acc;
    constexpr bool TV = C::TV, LIN = C::LIN;
    constexpr int NT = C::NT, NP = C::NP, MP = C::MP, PL = C::PL, CS = C::CS;
    constexpr int BPT = NP * MP / 256;           // B elements per thread (TV staging)
    __shared__ T lds[C::LDS];
    T *Pim = lds, *Q2 = Pim + C::P_EL, *Bim = Q2 + C::P_EL, *PBim = Bim + C::B_EL, *Eim = PBim + C::PB_EL;
    T *Gim = Eim + C::E_EL, *Aim = Gim + C::G_EL, *vec = Aim + C::P_EL;
    int *flag = (int *)(vec + C::V_EL);
    T *Qim = Q2;                         // time-invariant Q; time-varying: A's second buffer
    T *aug = PBim;                       // the exact sweep reuses the PB image (read before it)
    int *vote = flag + 4;                // per-wave Newton–Schulz verdicts (flag[0]: the sweep's)
    T *pimg = vec, *wslot = vec + 2 * NP, *dslot = wslot + 4 * MP;   // VAR_LIN vectors

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t b = blockIdx.x;
    if (b >= a.batch) return;            // whole workgroup
    const int N = a.N;
    constexpr size_t nn = (size_t)NP * NP, nm = (size_t)NP * MP, mm = (size_t)MP * MP;
    // per-trajectory bases; time-varying fields hold N−1 knots (knot k at index k−1)
    const size_t kAB = (TV && a.tv_AB) ? (size_t)(N - 1) : 1, kQR = (TV && a.tv_QR) ? (size_t)(N - 1) : 1;
    const size_t sA = kAB > 1 ? nn : 0, sB = kAB > 1 ? nm : 0, sQ = kQR > 1 ? nn : 0, sR = kQR > 1 ? mm : 0;
    const T *Ab = (const T *)a.A + b * nn * kAB, *Bb = (const T *)a.B + b * nm * kAB;
    const T *Qb = (const T *)a.Q + b * nn * kQR, *Rb = (const T *)a.R + b * mm * kQR;
    auto abuf = [&](int k) { return (TV && (k & 1)) ? Q2 : Aim; };   // knot k's A image
    const size_t k0 = TV ? (size_t)(N - 2) : 0;                     // first backward knot k = N − 1
    // linear terms: q_k, r_k (knot stride with Q, R), outputs d_k and p (p_1 or every p_k)
    const size_t sq = (LIN && kQR > 1) ? (size_t)NP : 0, sr = (LIN && kQR > 1) ? (size_t)MP : 0;
    const T *qg = LIN ? (const T *)a.q + (size_t)b * NP * kQR : nullptr;
    const T *rg = LIN ? (const T *)a.r + (size_t)b * MP * kQR : nullptr;
    T *dg = LIN ? (T *)a.d + (size_t)b * (size_t)(N - 1) * MP : nullptr;
    T *pallv = (LIN && a.p_all) ? (T *)a.p + (size_t)b * (size_t)N * NP : nullptr;

    acc Ar[NT], Rw = acc{0, 0, 0, 0};
    auto Bt = [&](int kk, int j) { return wg4_tload(Bim + 16 * kk + 16 * j * PL, PL, lane); };   // B[kk][j]
    const int ei = w % MT, ej = w / MT;          // this wave's E tile (w < MT²)
    if (w < MT * MT) Rw = wg4_tload(Rb + k0 * sR + 16 * ei + (size_t)16 * ej * MP, MP, lane);
    if constexpr (!TV) {
#pragma unroll
        for (int kk = 0; kk < NT; ++kk) Ar[kk] = wg4_tload(Ab + 16 * kk + (size_t)16 * w * NP, NP, lane);  // A[kk][w]
    }
    // P = Qf (:58) into the image; Q (the P_ accumulators' start) into its own; A, B of knot N−1
    {
        T *A0 = abuf(N - 1);
        for (int e = tid; e < NP * NP; e += 256) {
            Pim[(e % NP) + (e / NP) * PL] = ((const T *)a.Qf)[b * nn + e];
            if constexpr (!TV) Qim[(e % NP) + (e / NP) * PL] = Qb[e];
            A0[(e % NP) + (e / NP) * PL] = Ab[k0 * sA + e];
        }
    }
    for (int e = tid; e < NP * MP; e += 256) Bim[(e % NP) + (e / NP) * PL] = Bb[k0 * sB + e];
    if constexpr (LIN) {
        if (tid < NP) {
            const T v = ((const T *)a.qf)[(size_t)b * NP + tid];          // p = qf
            pimg[(N & 1) * NP + tid] = v;                                // p_k in buffer k & 1
            if (pallv) pallv[(size_t)(N - 1) * NP + tid] = v;
        }
    }
    T *Pall = a.p_all ? (T *)a.P + (size_t)b * nn * N : nullptr;
    T *Kb = (T *)a.K + (size_t)b * (size_t)(N - 1) * nm;
    int info = 0;
    acc Xi[MT][MT], Xp[MT][MT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) Xi[i][j] = Xp[i][j] = acc{0, 0, 0, 0};
    __syncthreads();
    if (Pall)
        for (int e = tid; e < NP * NP; e += 256) Pall[(size_t)(N - 1) * nn + e] = Pim[(e % NP) + (e / NP) * PL];

    for (int k = N - 1; k >= 1; --k) {           // :61
        T *Acur = abuf(k);
        // time-varying: knot k−1's A, B (this thread's elements) and R tile, requested now
        T An[TV ? 16 : 1], Bn[TV ? BPT : 1];
        acc Rn = Rw;
        if constexpr (TV) {
#pragma unroll
            for (int kk = 0; kk < NT; ++kk) Ar[kk] = wg4_tload(Acur + 16 * kk + 16 * w * PL, PL, lane);
            if (k > 1) {
                const T *Ak = Ab + (size_t)(k - 2) * sA, *Bk = Bb + (size_t)(k - 2) * sB;
#pragma unroll
                for (int s = 0; s < 16; ++s) An[s] = Ak[tid + 256 * s];
#pragma unroll
                for (int s = 0; s < BPT; ++s) Bn[s] = Bk[tid + 256 * s];
                if (w < MT * MT) Rn = wg4_tload(Rb + (size_t)(k - 2) * sR + 16 * ei + (size_t)16 * ej * MP, MP, lane);
            }
        }
        // linear terms: w = Bᵀp_{k+1} partials (p_{k+1} read per row tile, in row layout)
        const T *pk1 = pimg + ((k + 1) & 1) * NP;
        T wv[LIN ? MT : 1];
        if constexpr (LIN) {
#pragma unroll
            for (int j = 0; j < MT; ++j) wv[j] = (T)0;
        }
        // :38, :40 — one pass over the P image: PA[:, w] and PB[w][:]
        acc PA[NT], PB[MT];
#pragma unroll
        for (int i = 0; i < NT; ++i) PA[i] = acc{0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < MT; ++j) PB[j] = acc{0, 0, 0, 0};
#pragma unroll
        for (int kk = 0; kk < NT; ++kk) {
            acc Pt[NT];
#pragma unroll
            for (int i = 0; i < NT; ++i) Pt[i] = wg4_tload(Pim + 16 * kk + 16 * i * PL, PL, lane);   // P[kk][i]
#pragma unroll
            for (int i = 0; i < NT; ++i) wg4_mtn<T>(PA[i], Pt[i], Ar[kk]);
            const acc Pw = wg4_tload(Pim + 16 * kk + 16 * w * PL, PL, lane);                     // P[kk][w]
            T prow[4];
            if constexpr (LIN) {
#pragma unroll
                for (int r = 0; r < 4; ++r) prow[r] = pk1[16 * kk + Tile<T>::row(lane, r)];
            }
#pragma unroll
            for (int j = 0; j < MT; ++j) {
                const acc Bkj = Bt(kk, j);
                wg4_mtn<T>(PB[j], Pw, Bkj);
                if constexpr (LIN) wv[j] = wg4_vtn<T>(wv[j], Bkj, prow);                          // Bᵀp
            }
        }
#pragma unroll
        for (int j = 0; j < MT; ++j) wg4_tstore(PBim + 16 * w + 16 * j * PL, PL, PB[j], lane);
        if constexpr (TV) {
            if (k > 1) {                                   // knot k−1's A into the other buffer
                T *An_img = abuf(k - 1);
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    const int e = tid + 256 * s;
                    An_img[(e % NP) + (e / NP) * PL] = An[s];
                }
            }
        }
        __syncthreads();                                   // B1: PB image complete, P image read
        // :39 E tile, :41 G[:, w]
        if (w < MT * MT) {
            acc Et = Rw;
#pragma unroll
            for (int kk = 0; kk < NT; ++kk) {
                const acc Y = wg4_tload(PBim + 16 * kk + 16 * ej * PL, PL, lane);               // PB[kk][ej]
                wg4_mtn<T>(Et, Bt(kk, ei), Y);
            }
            wg4_tstore(Eim + 16 * ei + 16 * ej * CS, CS, Et, lane);
        }
        acc G[MT];
#pragma unroll
        for (int c = 0; c < MT; ++c) {
            G[c] = acc{0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < NT; ++kk) wg4_mtn<T>(G[c], Bt(kk, c), PA[kk]);
            wg4_tstore(Gim + 16 * c + 16 * w * CS, CS, G[c], lane);
        }
        __syncthreads();                                   // B2: E and G images complete, B read
        acc Qt[TV ? 3 : 1];
        if constexpr (TV) {
            if (k > 1) {                                   // knot k−1's B (B's last reader was G)
#pragma unroll
                for (int s = 0; s < BPT; ++s) {
                    const int e = tid + 256 * s;
                    Bim[(e % NP) + (e / NP) * PL] = Bn[s];
                }
            }
#pragma unroll
            for (int t = 0; t < 3; ++t) {                  // Q_k's P_ tiles straight from HBM
                const int i = wg4_pn_row(w, t) < 0 ? w : wg4_pn_row(w, t);
                Qt[t] = wg4_tload(Qb + (size_t)(k - 1) * sQ + 16 * i + (size_t)16 * w * NP, NP, lane);
            }
        }
        // m = 32, time-invariant (NS1): wave 3 alone refines X ≈ E⁻¹ and publishes it through the free
        // PB image while waves 0–2 form the K-independent part Q + A[:, i]ᵀPA[:, w] of their three
        // P_ tiles — the knot's critical path drops from 16 + 4 + 18 tile products (inverse in every
        // wave, 3/3/2/2 P_ tiles) to 16 + 4 + 6 (3/3/3/1 tiles, wg4_pn_row1)
        // (time-varying problems keep the inverse in every wave: with Q_k's tiles from HBM added
        // after the barrier the TV / TV+LIN variants measured 73.2 vs 72.7 and 159.5 vs 121.1 ms,
        // profiles/r06/u)
        constexpr bool NS1 = MT == 2 && !TV && LQRX_WG4_NS_ONE;
        acc PnA[NS1 ? 3 : 1];
        if constexpr (NS1) {
            if (w != 3) {
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const int i = wg4_pn_row1(w, t);
                    PnA[t] = wg4_tload(Qim + 16 * i + 16 * w * PL, PL, lane);                     // Q[i][w]
#pragma unroll
                    for (int kk = 0; kk < NT; ++kk) {
                        const acc At = t == 0 ? Ar[kk] : wg4_tload(Acur + 16 * kk + 16 * i * PL, PL, lane);
                        wg4_mtn<T>(PnA[t], At, PA[kk]);
                    }
                }
            }
        }
        // :42 X ≈ E⁻¹ (warm-started Newton–Schulz; the exact sweep on wave 0 otherwise)
        bool have = false;
        if (NS1 && k < N - 1) {
            T *Ximg = PBim;                              // free after B2 (the sweep reuses it only when !have)
            if (w == 3) {
                acc Id[MT][MT], E[MT][MT];
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) Id[i][j][r] = (i == j && Tile<T>::row(lane, r) == tcol(lane)) ? (T)1 : (T)0;
                        E[i][j] = wg4_tload(Eim + 16 * i + 16 * j * CS, CS, lane);
                        const acc x1 = Xi[i][j];
                        Xi[i][j] = (T)2 * x1 - Xp[i][j];
                        Xp[i][j] = x1;
                    }
                have = !a.ns_off && ns_refine<T, MT>(Xi, E, Id, lane);
                if (have) {
#pragma unroll
                    for (int i = 0; i < MT; ++i)
#pragma unroll
                        for (int j = 0; j < MT; ++j) wg4_tstore(Ximg + 16 * i + 16 * j * CS, CS, Xi[i][j], lane);
                }
                if (lane == 0) vote[0] = have ? 1 : 0;
            }
            __syncthreads();                             // wave 3's verdict (uniform by construction) and X
            have = vote[0] != 0;
            if (have && w != 3) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j) Xi[i][j] = wg4_tload(Ximg + 16 * i + 16 * j * CS, CS, lane);
            }
        } else if (k < N - 1) {
            // warm start 2X_{k+1} − X_{k+2}; Xp takes X_{k+1} before the refinement
            acc Id[MT][MT];
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < MT; ++j) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) Id[i][j][r] = (i == j && Tile<T>::row(lane, r) == tcol(lane)) ? (T)1 : (T)0;
                    const acc x1 = Xi[i][j];
                    Xi[i][j] = (T)2 * x1 - Xp[i][j];
                    Xp[i][j] = x1;
                }
            if constexpr (MT == 2 && LQRX_WG4_NS_SPLIT) {
                // split over the waves; the PB image is free after B2 (the exact sweep below, which
                // reuses it, starts only once every wave has left the refinement)
                have = wg4_ns_split<T, MT>(Xi, Eim, PBim, PBim + MP * CS, vote, CS, w, lane);
            } else {
                acc E[MT][MT];
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j) E[i][j] = wg4_tload(Eim + 16 * i + 16 * j * CS, CS, lane);
                have = !a.ns_off && ns_refine<T, MT>(Xi, E, Id, lane);
                // workgroup-uniform verdict by construction (the branch below holds a barrier): each
                // wave posts its own Newton–Schulz verdict, every wave takes the AND of all four — no
                // reliance on the four refinements agreeing bitwise.  (The slots are rewritten only
                // after this knot's B3, which every wave reaches after reading them.)
                if (lane == 0) vote[w] = have ? 1 : 0;
                __syncthreads();
                have = (vote[0] & vote[1] & vote[2] & vote[3]) != 0;
            }
        }
        if (!have) {                                       // uniform (k == N − 1, or the vote above)
            if (w == 0) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j)
                        wg4_tstore(aug + 16 * i + 16 * j * CS, CS, wg4_tload(Eim + 16 * i + 16 * j * CS, CS, lane), lane);
                wsync_w();
                const bool ok = aug_ldl_forward<T, MP, 0, CS, 0>(aug, lane);
                if (lane == 0) *flag = ok ? 1 : 0;
            }
            __syncthreads();
            if (!*flag && info == 0) info = k;
            acc Wt[MT][MT], DW[MT][MT];
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < MT; ++j) Wt[i][j] = wg4_tload(aug + MP * CS + 16 * i + 16 * j * CS, CS, lane);
            const T *rinv = aug + 2 * MP * CS + 64;
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const T sc = rinv[i * 16 + Tile<T>::row(lane, r)];
#pragma unroll
                    for (int j = 0; j < MT; ++j) DW[i][j][r] = Wt[i][j][r] * sc;
                }
            tiles_zero<T, MT, MT>(Xi);
            mma_tn<T, MT, MT, MT>(Xi, Wt, DW);             // X = Wᵀ D⁻¹ W = E⁻¹
            if (k == N - 1) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j) Xp[i][j] = Xi[i][j];
            }
        }
        // K[:, w] = XᵀG[:, w]  → sol.K[k−1] columns 16w…16w+15
        acc Kt[MT];
#pragma unroll
        for (int c = 0; c < MT; ++c) {
            Kt[c] = acc{0, 0, 0, 0};
#pragma unroll
            for (int i = 0; i < MT; ++i) wg4_mtn<T>(Kt[c], Xi[i][c], G[i]);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                Kb[(size_t)(k - 1) * nm + 16 * c + Tile<T>::row(lane, r) + (size_t)(16 * w + tcol(lane)) * MP] = Kt[c][r];
        }
        if constexpr (LIN) {
            // d = Xᵀw (w = r + Bᵀp, the companion of K = XᵀG); p_k rows 16w… = q + Aᵀp − Gᵀd
            T *ws_ = wslot + w * MP, *ds_ = dslot + w * MP;
#pragma unroll
            for (int j = 0; j < MT; ++j) {
                const T wj = rg[(size_t)(k - 1) * sr + 16 * j + tcol(lane)] + lin_rowsum(wv[j]);   // r + Bᵀp
                if (lane < 16) ws_[16 * j + lane] = wj;
            }
            wsync_w();
            T wrow[MT][4], dv[MT];
            lin_rows<T, MT>(wrow, ws_, lane);
#pragma unroll
            for (int j = 0; j < MT; ++j) {
                dv[j] = (T)0;
#pragma unroll
                for (int i = 0; i < MT; ++i) dv[j] = wg4_vtn<T>(dv[j], Xi[i][j], wrow[i]);
                dv[j] = lin_rowsum(dv[j]);
                if (lane < 16) {
                    ds_[16 * j + lane] = dv[j];
                    if (w == 0) dg[(size_t)(k - 1) * MP + 16 * j + lane] = dv[j];
                }
            }
            wsync_w();
            T drow[MT][4];
            lin_rows<T, MT>(drow, ds_, lane);
            T ap = (T)0, gd = (T)0, prow[NT][4];
            lin_rows<T, NT>(prow, pk1, lane);
#pragma unroll
            for (int kk = 0; kk < NT; ++kk) ap = wg4_vtn<T>(ap, Ar[kk], prow[kk]);
#pragma unroll
            for (int c = 0; c < MT; ++c) gd = wg4_vtn<T>(gd, G[c], drow[c]);
            const T pn = qg[(size_t)(k - 1) * sq + 16 * w + tcol(lane)] + lin_rowsum(ap) - lin_rowsum(gd);
            if (lane < 16) {
                pimg[(k & 1) * NP + 16 * w + lane] = pn;
                if (pallv) pallv[(size_t)(k - 1) * NP + 16 * w + lane] = pn;
            }
        }
        // :51 P_ tiles (i, w) = Q + A[:, i]ᵀPA[:, w] − G[:, i]ᵀK[:, w] → the P image, mirrored
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int i = NS1 ? wg4_pn_row1(w, t) : wg4_pn_row(w, t);
            if (i < 0) continue;
            acc Pn;
            if (NS1 && w != 3) {
                Pn = PnA[NS1 ? t : 0];                   // Q + A[:, i]ᵀPA[:, w] formed beside the inverse
            } else {
                if constexpr (TV) Pn = Qt[t];
                else Pn = wg4_tload(Qim + 16 * i + 16 * w * PL, PL, lane);                       // Q[i][w]
#pragma unroll
                for (int kk = 0; kk < NT; ++kk) {
                    const acc At = t == 0 ? Ar[kk] : wg4_tload(Acur + 16 * kk + 16 * i * PL, PL, lane);  // A[kk][i]
                    wg4_mtn<T>(Pn, At, PA[kk]);
                }
            }
#pragma unroll
            for (int c = 0; c < MT; ++c)
                wg4_mtn<T, true>(Pn, wg4_tload(Gim + 16 * c + 16 * i * CS, CS, lane), Kt[c]);
            T *at = Pim + 16 * i + 16 * w * PL, *mr = Pim + 16 * w + 16 * i * PL;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int rr = Tile<T>::row(lane, r), cc = tcol(lane);
                if (i != w) {
                    at[rr + cc * PL] = Pn[r];
                    mr[cc + rr * PL] = Pn[r];
                } else if (rr >= cc) {                     // diagonal tile: its lower triangle
                    at[rr + cc * PL] = Pn[r];
                    at[cc + rr * PL] = Pn[r];
                }
            }
        }
        if constexpr (TV) Rw = Rn;
        __syncthreads();                                   // B3: P_ image complete
        if (Pall)
            for (int e = tid; e < NP * NP; e += 256) Pall[(size_t)(k - 1) * nn + e] = Pim[(e % NP) + (e / NP) * PL];
    }
    if (!a.p_all)
        for (int e = tid; e < NP * NP; e += 256) ((T *)a.P)[b * nn + e] = Pim[(e % NP) + (e / NP) * PL];
    if constexpr (LIN) {
        if (!a.p_all && tid < NP) ((T *)a.p)[(size_t)b * NP + tid] = pimg[NP + tid];   // p_1 (buffer 1)
    }
    if (a.info && tid == 0) a.info[b] = info;
    // rollout once every wave's K (and d) stores are visible to the waves that read them
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (TV || LQRX_WG4_ROLL4) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        dp_rollout_wg4<T, MT, TV, LIN>(a, b, lds, w, lane);
    } else if (w == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        dp_rollout_full<T, NT, MT, LQRX_DP_KD, LIN>(a, b, lds, lane);
    }
}

template <int MT>
static hipError_t launch_wg4(const DpArgs &a, hipStream_t s)
{
    dim3 grid((unsigned)a.batch), block(256);
    const bool tv = a.tv_AB || a.tv_QR;
    if (a.lin && tv) hipLaunchKernelGGL((dp_wg4_kernel<double, MT, VAR_TV | VAR_LIN>), grid, block, 0, s, a);
    else if (a.lin) hipLaunchKernelGGL((dp_wg4_kernel<double, MT, VAR_LIN>), grid, block, 0, s, a);
    else if (tv) hipLaunchKernelGGL((dp_wg4_kernel<double, MT, VAR_TV>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((dp_wg4_kernel<double, MT, 0>), grid, block, 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------ launcher
template <typename T, int NT, int MT, int WAVES = 2, int VAR = 0>
static hipError_t launch_dp(const DpArgs &a, hipStream_t s);

// time-varying problems take the VAR_TV variant of the same tile grid
template <typename T, int NT, int MT, int WAVES = 2, int VAR = 0>
static hipError_t launch_dp_tv(const DpArgs &a, hipStream_t s)
{
    // 2 waves/SIMD where the time-varying kernel fits 256 registers without spills (tile
    // grids up to 2×1, i.e. n ≤ 32, m ≤ 16 — cfg4's shape), else 1
    constexpr int TVW = LQRX_DP_TVWAVES ? LQRX_DP_TVWAVES : ((NT <= 2 && MT <= 1) ? 2 : 1);
    // linear cost terms.  Time-varying: the extra vectors tip cfg4's 2×1 double grid over 256
    // VGPRs (72–91 spilled at 2 waves/SIMD), so VAR_TV|VAR_LIN runs 2 waves/SIMD only on the
    // 1×1 (double) and up to 2×1 (float) grids; time-invariant LIN keeps the plain kernel's
    // occupancy (its vector work sits after the solve, where fewer tiles are live)
    constexpr int LW = (NT * MT <= (sizeof(T) == 4 ? 2 : 1)) ? 2 : 1;
    if (a.lin && (a.tv_AB || a.tv_QR)) return launch_dp<T, NT, MT, LW, VAR_TV | VAR_LIN>(a, s);
    if (a.lin) return launch_dp<T, NT, MT, WAVES, VAR_LIN>(a, s);
    if (a.tv_AB || a.tv_QR) return launch_dp<T, NT, MT, TVW, VAR_TV | LQRX_DP_TVEXTRA>(a, s);
    return launch_dp<T, NT, MT, WAVES, VAR>(a, s);
}

template <typename T, int NT, int MT, int WAVES, int VAR>
static hipError_t launch_dp(const DpArgs &a, hipStream_t s)
{
    dim3 grid((unsigned)a.batch), block(64);
    if (a.n == NT * 16 && a.m == MT * 16)
        hipLaunchKernelGGL((dp_riccati_kernel<T, NT, MT, WAVES, VAR, true>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((dp_riccati_kernel<T, NT, MT, WAVES, VAR, false>), grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t dp_launch(const DpArgs &a_in, hipStream_t s)
{
    static const int ns_off = [] { const char *e = std::getenv("LQRX_DP_NS_OFF"); return e && *e == '1' ? 1 : 0; }();
    DpArgs a = a_in;
    a.ns_off = ns_off;
    // n ≤ 4: one lane per trajectory (a 16×16 MFMA tile would be mostly padding)
    if (dp_lane_supported(a.n, a.m)) return dp_lane_launch(a, s);
    // smallest instantiated tile grid that covers (n, m); padding is exact (zero rows /
    // columns, unit diagonal in R), see tiles_load
    const int nt = (a.n + 15) / 16, mt = (a.m + 15) / 16;
    // LQRX_DP_BIG=1 sends every shape past the lane kernel to dp_big_kernel (A/B checks)
    static const bool force_big = [] { const char *e = std::getenv("LQRX_DP_BIG"); return e && *e == '1'; }();
    if (force_big && dp_big_supported(a.n, a.m)) return dp_big_launch(a, s);
    if (a.dtype == 0) {
        if (nt <= 1 && mt <= 1) return launch_dp_tv<double, 1, 1>(a, s);
        if (nt <= 2 && mt <= 1) return launch_dp_tv<double, 2, 1, LQRX_DP_WAVES, LQRX_DP_VAR>(a, s);
        // 2×2 fp64 tiles do not fit 256 registers (≈ 450 live): the 2-wave launch bound compiles
        // to occupancy 1 (hipcc: "desired occupancy 2, final occupancy 1"; 44–60 B of spills).
        // Declaring one wave per SIMD instead (launch_dp_tv<double, 2, 2, 1>) gave an allocation
        // with 124 B of spills whose launch ended the process with SIGABRT on the box (round 6,
        // profiles/r06/d) — kept at the launch bound that passes, see DESIGN §3.1
        if (nt <= 2 && mt <= 2) return launch_dp_tv<double, 2, 2>(a, s);
        // n = 64, m ∈ {16, 32}: four waves per trajectory — time-invariant or time-varying, with
        // or without linear terms (LQRX_DP_WG4=0 in the environment: the one-wave kernel, for A/B
        // runs and tests)
        static const bool wg4 = [] { const char *e = std::getenv("LQRX_DP_WG4"); return LQRX_DP_WG4 && !(e && *e == '0'); }();
        if (wg4 && a.n == 64 && (a.m == 16 || a.m == 32))
            return a.m == 16 ? launch_wg4<1>(a, s) : launch_wg4<2>(a, s);
        if (nt <= 4 && mt <= 2) return launch_dp_tv<double, 4, 2, 1>(a, s);   // n ≤ 64: 1 wave/SIMD
    } else {
        if (nt <= 1 && mt <= 1) return launch_dp_tv<float, 1, 1>(a, s);
        if (nt <= 2 && mt <= 1) return launch_dp_tv<float, 2, 1>(a, s);
        if (nt <= 2 && mt <= 2) return launch_dp_tv<float, 2, 2>(a, s);
        if (nt <= 4 && mt <= 2) return launch_dp_tv<float, 4, 2, 1>(a, s);    // cfg5: n=64 m=32
    }
    return dp_big_launch(a, s);     // past the register tiles: workgroup per trajectory
}

bool dp_supported(int dtype, int n, int m, bool tv)
{
    (void)dtype;
    (void)tv;
    if (dp_lane_supported(n, m)) return true;
    const int nt = (n + 15) / 16, mt = (m + 15) / 16;
    return (n >= 1 && m >= 1 && nt <= 4 && mt <= 2) || dp_big_supported(n, m);
}

} // namespace lqrx
