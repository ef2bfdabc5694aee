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
#include "lqrx_tile.h"
#include "lqrx_internal.h"

namespace lqrx {

// Augmented upper Cholesky solve.  aug (LDS, column-major, column stride CS) holds
// [E | G] with E MP×MP (upper triangle used, as potrf 'U' does) and G MP×NP.  On return
// the G columns hold K = E⁻¹G (potrs 'U': Uᵀ Y = G, then U K = Y).  Each lane owns the
// columns lane + 64q.  Returns false (wave-uniform) if a pivot was not > 0.
// Also streams K (true m×n part) to global `Kout` (column-major, ld m) when Kout != null.
template <typename T, int MP, int NP, int CS>
__device__ __forceinline__ bool aug_chol_solve(T *aug, int lane, int m, int n, T *__restrict__ Kout)
{
    constexpr int NC = MP + NP;
    constexpr int CPL = (NC + 63) / 64;
    T x[CPL][MP];
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
        int c = lane + 64 * q;
#pragma unroll
        for (int i = 0; i < MP; ++i) x[q][i] = (c < NC) ? aug[c * CS + i] : (T)0;
    }
    bool ok = true;
    T dinv[MP];
    // forward: upper Cholesky of E and Uᵀ Y = G in one elimination sweep
#pragma unroll
    for (int i = 0; i < MP; ++i) {
        T piv = readlane(x[i / 64][i], i % 64);
        ok = ok && (piv > (T)0);
        T d = sqrt(piv);
        T di = (T)1 / d;
        dinv[i] = di;
#pragma unroll
        for (int q = 0; q < CPL; ++q) x[q][i] *= di;
#pragma unroll
        for (int p = i + 1; p < MP; ++p) {
            T u = readlane(x[p / 64][i], p % 64); // U[i][p], held by the owner of column p
#pragma unroll
            for (int q = 0; q < CPL; ++q) x[q][p] = fma(-u, x[q][i], x[q][p]);
        }
    }
    // backward: U K = Y on the G columns only (E columns keep U for the broadcasts)
#pragma unroll
    for (int j = MP - 1; j >= 0; --j) {
        T kj[CPL];
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
            bool rhs = (lane + 64 * q) >= MP;
            kj[q] = rhs ? x[q][j] * dinv[j] : (T)0;
            x[q][j] = rhs ? kj[q] : x[q][j];
        }
#pragma unroll
        for (int p = 0; p < j; ++p) {
            T u = readlane(x[j / 64][p], j % 64); // U[p][j]
#pragma unroll
            for (int q = 0; q < CPL; ++q) x[q][p] = fma(-u, kj[q], x[q][p]);
        }
    }
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
        int c = lane + 64 * q;
        if (c >= MP && c < NC) {
#pragma unroll
            for (int i = 0; i < MP; ++i) aug[c * CS + i] = x[q][i];
            int j = c - MP;
            if (Kout && j < n) {
#pragma unroll
                for (int i = 0; i < MP; ++i)
                    if (i < m) Kout[(size_t)i + (size_t)j * m] = x[q][i];
            }
        }
    }
    return ok;
}

template <typename T, int NT, int MT> struct DpCfg {
    static constexpr int NP = NT * 16, MP = MT * 16;
    static constexpr int CS = MP + 2;                       // padded LDS column stride
    static constexpr int AUG = (MP + NP) * CS;              // [E | G] image
    static constexpr int ROLL = MP * NP + NP + MP;          // K_k + x + u (rollout)
    static constexpr int LDS_ELEMS = AUG > ROLL ? AUG : ROLL;
    static constexpr int KPL = (MP * NP + 63) / 64;         // K elements per lane (rollout)
};

// Forward rollout  dynamic_programming.jl:66-70 :  u_k = −K_k x_k ; x_{k+1} = A x_k + B u_k.
// K_k is streamed back from global (written by the backward sweep of this same wave),
// DEPTH knots ahead, 64 lanes × KPL coalesced elements per knot.
template <typename T, int NT, int MT, int DEPTH>
__device__ __forceinline__ void dp_rollout(const DpArgs &a, int64_t b, T *lds, int lane)
{
    using C = DpCfg<T, NT, MT>;
    constexpr int NP = C::NP, MP = C::MP, KPL = C::KPL;
    const int n = a.n, m = a.m, N = a.N;
    const size_t mn = (size_t)m * n;
    const T *__restrict__ Kg = (const T *)a.K + (size_t)b * (size_t)(N - 1) * mn;
    const T *__restrict__ Ag = (const T *)a.A + (size_t)b * n * n;
    const T *__restrict__ Bg = (const T *)a.B + (size_t)b * n * m;
    T *__restrict__ Xg = (T *)a.X + (size_t)b * (size_t)N * n;
    T *__restrict__ Ug = (T *)a.U + (size_t)b * (size_t)(N - 1) * m;
    T *Ks = lds, *xs = lds + MP * NP, *us = xs + NP;

    // rows of A and B for the x-update (lane i < n owns row i)
    T arow[NP], brow[MP];
#pragma unroll
    for (int j = 0; j < NP; ++j) arow[j] = (lane < n && j < n) ? Ag[lane + (size_t)j * n] : (T)0;
#pragma unroll
    for (int p = 0; p < MP; ++p) brow[p] = (lane < n && p < m) ? Bg[lane + (size_t)p * n] : (T)0;

    const T *x0 = (const T *)a.x0 + (size_t)b * n;
    if (lane < NP) xs[lane] = (lane < n) ? x0[lane] : (T)0;
    if (lane < MP) us[lane] = (T)0;
    if (lane < n) Xg[lane] = x0[lane];

    // ring of DEPTH prefetched K knots
    T ring[DEPTH][KPL];
    auto issue = [&](int kk, T(&dst)[KPL]) {
#pragma unroll
        for (int s = 0; s < KPL; ++s) {
            size_t e = (size_t)lane + 64 * s;
            dst[s] = (kk <= N - 1 && e < mn) ? Kg[(size_t)(kk - 1) * mn + e] : (T)0;
        }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) issue(1 + d, ring[d]);
    __syncthreads();

    for (int k0 = 1; k0 <= N - 1; k0 += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int k = k0 + d;
            if (k <= N - 1) {
                // stage K_k into LDS (col-major m×n), refill this ring slot with K_{k+DEPTH}
#pragma unroll
                for (int s = 0; s < KPL; ++s) {
                    size_t e = (size_t)lane + 64 * s;
                    if (e < mn) Ks[e] = ring[d][s];
                }
                issue(k + DEPTH, ring[d]);
                __syncthreads();
                if (lane < m) {
                    T s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
                    for (int j = 0; j < NP; j += 4) {
                        if (j + 0 < n) s0 = fma(Ks[lane + (j + 0) * m], xs[j + 0], s0);
                        if (j + 1 < n) s1 = fma(Ks[lane + (j + 1) * m], xs[j + 1], s1);
                        if (j + 2 < n) s2 = fma(Ks[lane + (j + 2) * m], xs[j + 2], s2);
                        if (j + 3 < n) s3 = fma(Ks[lane + (j + 3) * m], xs[j + 3], s3);
                    }
                    T u = -((s0 + s1) + (s2 + s3));
                    us[lane] = u;
                    Ug[(size_t)(k - 1) * m + lane] = u;
                }
                __syncthreads();
                T xn = 0;
                if (lane < n) {
                    T s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
                    for (int j = 0; j < NP; j += 4) {
                        s0 = fma(arow[j + 0], xs[j + 0], s0);
                        s1 = fma(arow[j + 1], xs[j + 1], s1);
                        s2 = fma(arow[j + 2], xs[j + 2], s2);
                        s3 = fma(arow[j + 3], xs[j + 3], s3);
                    }
                    T t0 = 0, t1 = 0;
#pragma unroll
                    for (int p = 0; p < MP; p += 2) {
                        t0 = fma(brow[p + 0], us[p + 0], t0);
                        t1 = fma(brow[p + 1], us[p + 1], t1);
                    }
                    xn = ((s0 + s1) + (s2 + s3)) + (t0 + t1);
                    Xg[(size_t)k * n + lane] = xn;
                }
                __syncthreads();
                if (lane < n) xs[lane] = xn;
                __syncthreads();
            }
        }
    }
}

template <typename T, int NT, int MT>
__global__ __launch_bounds__(64, 2) void dp_riccati_kernel(const DpArgs a)
{
    using C = DpCfg<T, NT, MT>;
    using acc = typename Tile<T>::acc;
    constexpr int NP = C::NP, MP = C::MP, CS = C::CS;
    __shared__ T lds[C::LDS_ELEMS];

    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    if (b >= a.batch) return;
    const int n = a.n, m = a.m, N = a.N;
    const size_t nn = (size_t)n * n, nm = (size_t)n * m, mm = (size_t)m * m;

    acc At[NT][NT], Bt[NT][MT], Qt[NT][NT], Rt[MT][MT], P[NT][NT];
    tiles_load<T, NT, NT>(At, (const T *)a.A + b * nn, n, n, n, lane, false);
    tiles_load<T, NT, MT>(Bt, (const T *)a.B + b * nm, n, m, n, lane, false);
    tiles_load<T, NT, NT>(Qt, (const T *)a.Q + b * nn, n, n, n, lane, false);
    tiles_load<T, MT, MT>(Rt, (const T *)a.R + b * mm, m, m, m, lane, true);
    tiles_load<T, NT, NT>(P, (const T *)a.Qf + b * nn, n, n, n, lane, false); // :58 P = Qf

    T *Pall = a.p_all ? (T *)a.P + (size_t)b * nn * N : nullptr;
    if (Pall) tiles_store<T, NT, NT>(P, Pall + (size_t)(N - 1) * nn, n, n, n, lane);
    T *Kb = (T *)a.K + (size_t)b * (size_t)(N - 1) * nm;
    int info = 0;

    for (int k = N - 1; k >= 1; --k) { // :61
        acc PB[NT][MT], E[MT][MT], PA[NT][NT], G[MT][NT];
        tiles_zero<T, NT, MT>(PB);
        mma_tn<T, NT, NT, MT>(PB, P, Bt);                          // :38 PB = P B
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < MT; ++j) E[i][j] = Rt[i][j];
        mma_tn<T, NT, MT, MT>(E, Bt, PB);                          // :39 E = R + B'PB
        tiles_zero<T, NT, NT>(PA);
        mma_tn<T, NT, NT, NT>(PA, P, At);                          // :40 PA = P A
        tiles_zero<T, MT, NT>(G);
        mma_tn<T, NT, MT, NT>(G, Bt, PA);                          // :41 K = B'PA

        // :42 chol_solve!(E, K) — potrf 'U' + potrs 'U'
        tiles_to_lds<T, MT, MT>(E, lds, CS, lane);
        tiles_to_lds<T, MT, NT>(G, lds + MP * CS, CS, lane);
        __syncthreads();
        bool ok = aug_chol_solve<T, MP, NP, CS>(lds, lane, m, n, Kb + (size_t)(k - 1) * nm);
        if (!ok && info == 0) info = k;
        __syncthreads();
        acc Kt[MT][NT];
        tiles_from_lds<T, MT, NT>(Kt, lds + MP * CS, CS, lane);
        __syncthreads();

        acc APBt[MT][NT];
        tiles_zero<T, MT, NT>(APBt);
        mma_tn<T, NT, MT, NT>(APBt, PB, At);                       // :50 APBᵀ = PBᵀ A
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) Kt[i][j] = -Kt[i][j];
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) P[i][j] = Qt[i][j];
        mma_tn<T, NT, NT, NT>(P, At, PA);                          // :51 Q + A'PA
        mma_tn<T, MT, NT, NT>(P, APBt, Kt);                        //     − APB K
        if (Pall) tiles_store<T, NT, NT>(P, Pall + (size_t)(k - 1) * nn, n, n, n, lane);
    }
    if (!a.p_all) tiles_store<T, NT, NT>(P, (T *)a.P + (size_t)b * nn, n, n, n, lane);
    if (a.info && lane == 0) a.info[b] = info;

    // make this wave's K stores visible to its own (other-lane) rollout loads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    dp_rollout<T, NT, MT, 4>(a, b, lds, lane);
}

// ------------------------------------------------------------------ launcher
template <typename T, int NT, int MT> static hipError_t launch_dp(const DpArgs &a, hipStream_t s)
{
    dim3 grid((unsigned)a.batch), block(64);
    hipLaunchKernelGGL((dp_riccati_kernel<T, NT, MT>), grid, block, 0, s, a);
    return hipGetLastError();
}

hipError_t dp_launch(const DpArgs &a, hipStream_t s)
{
    const int nt = (a.n + 15) / 16, mt = (a.m + 15) / 16;
    if (a.dtype == 0) {
        if (nt == 1 && mt == 1) return launch_dp<double, 1, 1>(a, s);
        if (nt == 2 && mt == 1) return launch_dp<double, 2, 1>(a, s);
        if (nt == 2 && mt == 2) return launch_dp<double, 2, 2>(a, s);
    } else {
        if (nt == 1 && mt == 1) return launch_dp<float, 1, 1>(a, s);
        if (nt == 2 && mt == 1) return launch_dp<float, 2, 1>(a, s);
        if (nt == 2 && mt == 2) return launch_dp<float, 2, 2>(a, s);
    }
    return hipErrorNotSupported;
}

bool dp_supported(int dtype, int n, int m)
{
    const int nt = (n + 15) / 16, mt = (m + 15) / 16;
    if (n < 1 || m < 1) return false;
    return (nt == 1 && mt == 1) || (nt == 2 && mt == 1) || (nt == 2 && mt == 2);
}

} // namespace lqrx
