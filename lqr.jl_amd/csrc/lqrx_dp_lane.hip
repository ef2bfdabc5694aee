// lqrx_dp_lane.hip — batched Riccati backward pass + forward rollout for SMALL state
// dimensions (n ≤ 4, m ≤ 4): the reference's test problems (cartpole n=4 m=1,
// test/cartpole.jl; Dubins n=3 m=2; double integrators), BASELINE configs[0..1].
// Replaces solve!(sol, ::DPSolver, ::LQRProblem), /root/reference/src/dynamic_programming.jl:54-72.
//
// Mapping: ONE LANE PER TRAJECTORY (64 trajectories per wave).  At n = 4 a 16×16 fp64 MFMA
// tile would be 94 % padding; here every flop is useful: the whole knot (≈160 fp64 FMAs at
// n=4, m=1) is straight-line scalar code on registers, all dimensions compile-time padded
// (NP, MP) with exact zero padding (A, B, Q padded with zeros, R with a unit diagonal: the
// padded rows/columns of P, E, K stay exactly 0/identity, so real entries see only +0·x
// terms).  The horizon walk is serial per lane; the batch is the parallelism.
//
// Per knot (fast symmetric form, as the MFMA kernel; reference lines of dynamic_programming.jl):
//   :38  PB = P·B           :39  E = R + BᵀPB         :40  PA = P·A       :41  G = BᵀPA
//   :29-30 potrf 'U' of E (pivot ≤ 0 → info = k) and K = E⁻¹G by two triangular solves
//   :50-51 P_ = Q + AᵀPA − GᵀK  (GᵀK ≡ APB·K for symmetric P), lower triangle, mirrored.
// Time-varying problems (per-knot A_k, B_k, Q_k, R_k) reload the knot's
// matrices instead of keeping them in registers.
#include "lqrx_internal.h"
#include "lqrx_tile.h"
#include <cstdlib>

namespace lqrx {

namespace {

template <typename T> __device__ __forceinline__ T lane_rsqrt(T a);
template <> __device__ __forceinline__ double lane_rsqrt<double>(double a) { return rsqrt_nr(a); }
template <> __device__ __forceinline__ float lane_rsqrt<float>(float a) { return rsqrt_nr(a); }

// load an r×c column-major block (ld = r) into a padded RP×CP register array; pad value
// `dpad` on the padded diagonal (1 for R so the padded E stays SPD), 0 elsewhere.  `es` is
// the element stride: 1 in layout 0, the batch in layout 1 (SoA: consecutive lanes read
// consecutive words — one coalesced load per element across the wave)
template <typename T, int RP, int CP>
__device__ __forceinline__ void lane_load(T (&D)[RP][CP], const T *__restrict__ src, int r, int c, T dpad,
                                          int64_t es)
{
#pragma unroll
    for (int j = 0; j < CP; ++j)
#pragma unroll
        for (int i = 0; i < RP; ++i) {
            const bool ok = i < r && j < c;
            D[i][j] = ok ? src[(i + j * r) * es] : (i == j ? dpad : (T)0);
        }
}

} // namespace

// LIN (linear cost terms, lqrx_dp_solve_linear; q, r follow Q, R: per knot with TV,
// loaded once otherwise): p = qf, then per knot
//   d = E⁻¹(r + Bᵀp)  (the same potrf factor, one more potrs column),
//   p ← q + Aᵀp − APB·d  (APB = AᵀPB = Gᵀ for symmetric P),
// and the rollout applies u = −(K x + d).  Reference op order: oracle_dp_solve_one_lin.
template <typename T, int NP, int MP, bool TV, bool SOA, bool LIN = false>
__global__ __launch_bounds__(64) void dp_lane_kernel(const DpArgs a)
{
    const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (b >= a.batch) return;   // no barriers / cross-lane ops below
    const int n = a.n, m = a.m, N = a.N;
    const int64_t nn = (int64_t)n * n, nm = (int64_t)n * m, mm = (int64_t)m * m;
    // layout: trajectory base offset of an array with S elements per trajectory, and the
    // element stride (layout 0: b·S, 1; layout 1 / SoA: b, batch)
    const int64_t es = SOA ? a.batch : 1;
    auto tb = [&](int64_t S) { return SOA ? b : b * S; };
    // TV (template): matrices are re-read every knot; a time-invariant field of a
    // time-varying problem simply has knot stride 0 (it stays cache-resident)
    constexpr bool tvAB = TV, tvQR = TV;
    const int64_t kAB = a.tv_AB ? N - 1 : 1, kQR = a.tv_QR ? N - 1 : 1;    // knots stored
    const int64_t sA = a.tv_AB ? nn : 0, sB = a.tv_AB ? nm : 0;            // knot strides
    const int64_t sQ = a.tv_QR ? nn : 0, sR = a.tv_QR ? mm : 0;
    const T *Ab = (const T *)a.A + tb(nn * kAB);
    const T *Bb = (const T *)a.B + tb(nm * kAB);
    const T *Qb = (const T *)a.Q + tb(nn * kQR);
    const T *Rb = (const T *)a.R + tb(mm * kQR);

    T A[NP][NP], B[NP][MP], Q[NP][NP], R[MP][MP], P[NP][NP];
    lane_load<T, NP, NP>(P, (const T *)a.Qf + tb(nn), n, n, (T)0, es);   // :58 P = Qf
    if constexpr (!tvAB) {
        lane_load<T, NP, NP>(A, Ab, n, n, (T)0, es);
        lane_load<T, NP, MP>(B, Bb, n, m, (T)0, es);
    }
    if constexpr (!tvQR) {
        lane_load<T, NP, NP>(Q, Qb, n, n, (T)0, es);
        lane_load<T, MP, MP>(R, Rb, m, m, (T)1, es);
    }
    T *Kb = (T *)a.K + tb((int64_t)(N - 1) * nm);
    T *Pall = a.p_all ? (T *)a.P + tb(nn * N) : nullptr;
    auto store_P = [&](T *dst) {
#pragma unroll
        for (int j = 0; j < NP; ++j)
#pragma unroll
            for (int i = 0; i < NP; ++i)
                if (i < n && j < n) dst[(i + j * n) * es] = (i >= j) ? P[i][j] : P[j][i];
    };
    if (Pall) store_P(Pall + (int64_t)(N - 1) * nn * es);
    int info = 0;
    // linear terms: p (cost-to-go gradient), knot vectors q_k, r_k (stride with Q, R)
    constexpr int LN = LIN ? NP : 1, LM = LIN ? MP : 1;
    const int64_t sq = a.tv_QR ? n : 0, sr = a.tv_QR ? m : 0;
    const T *qb = LIN ? (const T *)a.q + tb(n * kQR) : nullptr;
    const T *rb = LIN ? (const T *)a.r + tb(m * kQR) : nullptr;
    T *db = LIN ? (T *)a.d + tb((int64_t)(N - 1) * m) : nullptr;
    T *pall = (LIN && a.p_all) ? (T *)a.p + tb((int64_t)N * n) : nullptr;
    T pv[LN], qv[LN], rv[LM], qn[LN], rn[LM];
    if constexpr (LIN) {
        const T *qf = (const T *)a.qf + tb(n);
#pragma unroll
        for (int i = 0; i < NP; ++i) pv[i] = i < n ? qf[i * es] : (T)0;
        if (pall) {
#pragma unroll
            for (int i = 0; i < NP; ++i)
                if (i < n) pall[((int64_t)(N - 1) * n + i) * es] = pv[i];
        }
        if constexpr (!TV) {   // time-invariant q, r: loaded once
#pragma unroll
            for (int i = 0; i < NP; ++i) qv[i] = i < n ? qb[i * es] : (T)0;
#pragma unroll
            for (int i = 0; i < MP; ++i) rv[i] = i < m ? rb[i * es] : (T)0;
        }
    }
    // time-varying: knot k's matrices are prefetched during knot k+1
    constexpr int TN = TV ? NP : 1, TM = TV ? MP : 1;
    T An[TN][TN], Bn[TN][TM], Qn[TN][TN], Rn[TM][TM];
    auto fetch_tv = [&](int k) {
        if (k < 1) return;
        if constexpr (LIN) {
#pragma unroll
            for (int i = 0; i < NP; ++i) qn[i] = i < n ? qb[((int64_t)(k - 1) * sq + i) * es] : (T)0;
#pragma unroll
            for (int i = 0; i < MP; ++i) rn[i] = i < m ? rb[((int64_t)(k - 1) * sr + i) * es] : (T)0;
        }
        if constexpr (tvAB) {
            lane_load<T, NP, NP>(An, Ab + (int64_t)(k - 1) * sA * es, n, n, (T)0, es);
            lane_load<T, NP, MP>(Bn, Bb + (int64_t)(k - 1) * sB * es, n, m, (T)0, es);
        }
        if constexpr (tvQR) {
            lane_load<T, NP, NP>(Qn, Qb + (int64_t)(k - 1) * sQ * es, n, n, (T)0, es);
            lane_load<T, MP, MP>(Rn, Rb + (int64_t)(k - 1) * sR * es, m, m, (T)1, es);
        }
    };
    if constexpr (TV) fetch_tv(N - 1);

    for (int k = N - 1; k >= 1; --k) {   // :61
        if constexpr (tvAB) {
#pragma unroll
            for (int i = 0; i < NP; ++i) {
#pragma unroll
                for (int j = 0; j < NP; ++j) A[i][j] = An[i][j];
#pragma unroll
                for (int c = 0; c < MP; ++c) B[i][c] = Bn[i][c];
            }
        }
        if constexpr (tvQR) {
#pragma unroll
            for (int i = 0; i < NP; ++i)
#pragma unroll
                for (int j = 0; j < NP; ++j) Q[i][j] = Qn[i][j];
#pragma unroll
            for (int i = 0; i < MP; ++i)
#pragma unroll
                for (int j = 0; j < MP; ++j) R[i][j] = Rn[i][j];
        }
        if constexpr (LIN && TV) {
#pragma unroll
            for (int i = 0; i < NP; ++i) qv[i] = qn[i];
#pragma unroll
            for (int i = 0; i < MP; ++i) rv[i] = rn[i];
        }
        if constexpr (TV) fetch_tv(k - 1);
        // P is symmetric: only P[i][j], i ≥ j, is maintained
#define PS(i, j) ((i) >= (j) ? P[i][j] : P[j][i])
        T PB[NP][MP], PA[NP][NP];
#pragma unroll
        for (int i = 0; i < NP; ++i) {
#pragma unroll
            for (int c = 0; c < MP; ++c) {                       // :38 PB = P B
                T s = (T)0;
#pragma unroll
                for (int l = 0; l < NP; ++l) s = fma(PS(i, l), B[l][c], s);
                PB[i][c] = s;
            }
#pragma unroll
            for (int j = 0; j < NP; ++j) {                       // :40 PA = P A
                T s = (T)0;
#pragma unroll
                for (int l = 0; l < NP; ++l) s = fma(PS(i, l), A[l][j], s);
                PA[i][j] = s;
            }
        }
#undef PS
        T E[MP][MP], G[MP][NP];
#pragma unroll
        for (int c = 0; c < MP; ++c) {
#pragma unroll
            for (int d = 0; d <= c; ++d) {                       // :39 E = R + BᵀPB (lower)
                T s = R[c][d];
#pragma unroll
                for (int i = 0; i < NP; ++i) s = fma(B[i][c], PB[i][d], s);
                E[c][d] = s;
            }
#pragma unroll
            for (int j = 0; j < NP; ++j) {                       // :41 G = BᵀPA
                T s = (T)0;
#pragma unroll
                for (int i = 0; i < NP; ++i) s = fma(B[i][c], PA[i][j], s);
                G[c][j] = s;
            }
        }
        // :29 potrf 'U' (E = UᵀU; here the lower storage holds Uᵀ = L): column by column
        T L[MP][MP], Linv[MP];
#pragma unroll
        for (int j = 0; j < MP; ++j) {
            T d = E[j][j];
#pragma unroll
            for (int p = 0; p < j; ++p) d = fma(-L[j][p], L[j][p], d);
            if (!(d > (T)0) && info == 0) info = k;
            const T ri = lane_rsqrt<T>(d);
            Linv[j] = ri;
#pragma unroll
            for (int i = j + 1; i < MP; ++i) {
                T s = E[i][j];
#pragma unroll
                for (int p = 0; p < j; ++p) s = fma(-L[i][p], L[j][p], s);
                L[i][j] = s * ri;
            }
            L[j][j] = d * ri;
        }
        // :30 potrs: L y = G (forward), Lᵀ K = y (backward), column by column of G
        T K[MP][NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            T y[MP];
#pragma unroll
            for (int i = 0; i < MP; ++i) {
                T s = G[i][j];
#pragma unroll
                for (int p = 0; p < i; ++p) s = fma(-L[i][p], y[p], s);
                y[i] = s * Linv[i];
            }
#pragma unroll
            for (int i = MP - 1; i >= 0; --i) {
                T s = y[i];
#pragma unroll
                for (int p = i + 1; p < MP; ++p) s = fma(-L[p][i], K[p][j], s);
                K[i][j] = s * Linv[i];
            }
        }
        T *Kk = Kb + (int64_t)(k - 1) * nm * es;                 // sol.K[k], m×n col-major
#pragma unroll
        for (int j = 0; j < NP; ++j)
#pragma unroll
            for (int i = 0; i < MP; ++i)
                if (i < m && j < n) Kk[(i + j * m) * es] = K[i][j];
        if constexpr (LIN) {
            // d = E⁻¹(r + Bᵀp): the potrs of :30 on one more column
            T y[MP], dv[MP];
#pragma unroll
            for (int i = 0; i < MP; ++i) {
                T s = (T)0;
#pragma unroll
                for (int l = 0; l < NP; ++l) s = fma(B[l][i], pv[l], s);
                s = rv[i] + s;
#pragma unroll
                for (int c = 0; c < i; ++c) s = fma(-L[i][c], y[c], s);
                y[i] = s * Linv[i];
            }
#pragma unroll
            for (int i = MP - 1; i >= 0; --i) {
                T s = y[i];
#pragma unroll
                for (int c = i + 1; c < MP; ++c) s = fma(-L[c][i], dv[c], s);
                dv[i] = s * Linv[i];
            }
#pragma unroll
            for (int i = 0; i < MP; ++i)
                if (i < m) db[((int64_t)(k - 1) * m + i) * es] = dv[i];
            // p ← q + Aᵀp − APB·d  (APB[i][c] = G[c][i])
            T pn[NP];
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                T s = (T)0, t = (T)0;
#pragma unroll
                for (int l = 0; l < NP; ++l) s = fma(A[l][i], pv[l], s);
#pragma unroll
                for (int c = 0; c < MP; ++c) t = fma(G[c][i], dv[c], t);
                pn[i] = qv[i] + s - t;
            }
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                pv[i] = pn[i];
                if (pall && i < n) pall[((int64_t)(k - 1) * n + i) * es] = pv[i];
            }
        }
        // :51 P_ = Q + AᵀPA − GᵀK   (lower triangle)
#pragma unroll
        for (int i = 0; i < NP; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) {
                T s = Q[i][j];
#pragma unroll
                for (int l = 0; l < NP; ++l) s = fma(A[l][i], PA[l][j], s);
#pragma unroll
                for (int c = 0; c < MP; ++c) s = fma(-G[c][i], K[c][j], s);
                P[i][j] = s;
            }
        if (Pall) store_P(Pall + (int64_t)(k - 1) * nn * es);
    }
    if (!a.p_all) store_P((T *)a.P + tb(nn));
    if (a.info) a.info[b] = info;
    if constexpr (LIN) {
        if (!a.p_all) {
            T *p1 = (T *)a.p + tb(n);
#pragma unroll
            for (int i = 0; i < NP; ++i)
                if (i < n) p1[i * es] = pv[i];
        }
    }

    // forward rollout  :66-70  u_k = −K_k x_k ; x_{k+1} = A_k x_k + B_k u_k
    T *Xb = (T *)a.X + tb((int64_t)N * n), *Ub = (T *)a.U + tb((int64_t)(N - 1) * m);
    const T *x0 = (const T *)a.x0 + tb(n);
    T x[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) x[i] = i < n ? x0[i * es] : (T)0;
#pragma unroll
    for (int i = 0; i < NP; ++i)
        if (i < n) Xb[i * es] = x[i];
    // K_k (and A_k, B_k when time-varying) were written / live in HBM; the x-recurrence is a
    // short dependent chain per knot, so the loads are issued RD knots ahead from a
    // register ring (unrolled by RD so every ring index is static).
    constexpr int RD = TV ? 4 : ((MP * NP <= 8) ? 8 : 4);
    struct Knot {
        T K[MP][NP], A[TV ? NP : 1][TV ? NP : 1], B[TV ? NP : 1][TV ? MP : 1], d[LM];
    };
    Knot ring[RD];
    auto fetch = [&](int k, Knot &d) {
        if (k > N - 1) return;
        const T *Kk = Kb + (int64_t)(k - 1) * nm * es;
#pragma unroll
        for (int j = 0; j < NP; ++j)
#pragma unroll
            for (int i = 0; i < MP; ++i) d.K[i][j] = (i < m && j < n) ? Kk[(i + j * m) * es] : (T)0;
        if constexpr (LIN) {
#pragma unroll
            for (int i = 0; i < MP; ++i) d.d[i] = i < m ? db[((int64_t)(k - 1) * m + i) * es] : (T)0;
        }
        if constexpr (tvAB) {
            lane_load<T, NP, NP>(d.A, Ab + (int64_t)(k - 1) * sA * es, n, n, (T)0, es);
            lane_load<T, NP, MP>(d.B, Bb + (int64_t)(k - 1) * sB * es, n, m, (T)0, es);
        }
    };
#pragma unroll
    for (int d = 0; d < RD; ++d) fetch(1 + d, ring[d]);
    for (int k0 = 1; k0 <= N - 1; k0 += RD) {
#pragma unroll
        for (int d = 0; d < RD; ++d) {
            const int k = k0 + d;
            if (k > N - 1) break;
            T Kc[MP][NP], dc[LM];
#pragma unroll
            for (int j = 0; j < NP; ++j)
#pragma unroll
                for (int i = 0; i < MP; ++i) Kc[i][j] = ring[d].K[i][j];
#pragma unroll
            for (int i = 0; i < LM; ++i) dc[i] = ring[d].d[i];
            if constexpr (tvAB) {
#pragma unroll
                for (int i = 0; i < NP; ++i) {
#pragma unroll
                    for (int j = 0; j < NP; ++j) A[i][j] = ring[d].A[i][j];
#pragma unroll
                    for (int c = 0; c < MP; ++c) B[i][c] = ring[d].B[i][c];
                }
            }
            fetch(k + RD, ring[d]);
            T u[MP];
#pragma unroll
            for (int i = 0; i < MP; ++i) {
                T s = (T)0;
#pragma unroll
                for (int j = 0; j < NP; ++j) s = fma(Kc[i][j], x[j], s);
                if constexpr (LIN) u[i] = -(s + dc[i]);   // u = −(K x + d)
                else u[i] = -s;
                if (i < m) Ub[((int64_t)(k - 1) * m + i) * es] = u[i];
            }
            T xn[NP];
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                T s = (T)0;
#pragma unroll
                for (int j = 0; j < NP; ++j) s = fma(A[i][j], x[j], s);
#pragma unroll
                for (int c = 0; c < MP; ++c) s = fma(B[i][c], u[c], s);
                xn[i] = s;
            }
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                x[i] = xn[i];
                if (i < n) Xb[((int64_t)k * n + i) * es] = x[i];
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// dp_quad_kernel: FOUR LANES PER TRAJECTORY (a DPP quad), n ∈ {3, 4}, time-invariant.
// With one lane per trajectory a B = 4096 batch is 64 waves — one per CU on a quarter of
// the chip, each a serial ~160-FMA-per-knot chain.  Here lane q of the quad owns column q
// of everything that splits by columns and the small m-sized work is replicated:
//   replicated: PB = P·B, E = R + BᵀPB, potrf of E
//   column q:   PA[:,q] = P·A[:,q]; G[:,q] = PBᵀA[:,q] (= BᵀPA for symmetric P);
//               Kq = E⁻¹G[:,q]; P_[:,q] = Q[:,q] + Aᵀ(PA[:,q] − PB·Kq)  (= AᵀPA − GᵀK)
// then P_ is re-replicated by four DPP quad broadcasts of the lower-triangle columns (lane r
// supplies column r).  Rollout: x replicated, lane q computes x_{k+1}[q] = A[q,:]x + B[q,:]u
// and the quad broadcasts re-assemble x.  Same reference lines as dp_lane_kernel.
// LIN (linear cost terms): w = r + Bᵀp and d = E⁻¹w replicated (the quad holds the potrf
// factor anyway), lane q forms p_new[q] = q[q] + A[:,q]ᵀp − G[:,q]ᵀd and the four quad
// broadcasts re-replicate p; the rollout adds d_k (lane c < m loads d_k[c], broadcast).
template <int CTRL>
__device__ __forceinline__ double qbcast(double v)
{
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(x >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL>
__device__ __forceinline__ float qbcast(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
// quad_perm [r,r,r,r]: every lane of the quad reads lane r
template <int R, typename T>
__device__ __forceinline__ T qfrom(T v) { return qbcast<R | (R << 2) | (R << 4) | (R << 6)>(v); }

#ifndef LQRX_QUAD_RCP
#define LQRX_QUAD_RCP 1         // m = 1: K = G·rcp(E) instead of the two potrs scalings by rsq(E) (0: A/B)
#endif
#ifndef LQRX_QUAD_PB_REPL
#define LQRX_QUAD_PB_REPL 0     // A/B: 1 = PB = P·B replicated in every lane of the quad (round 4)
#endif
// EX (exact shape: n = 4, m = MP, trajectory-contiguous layout): every stride and padding test
// is a compile-time constant — the rollout's K loads become immediate offsets of one pointer
template <typename T, int MP, bool SOA, bool LIN = false, bool EX = false>
__global__ __launch_bounds__(64) void dp_quad_kernel(const DpArgs a)
{
    constexpr int NP = 4;
    static_assert(!EX || !SOA, "EX: trajectory-contiguous layout only");
    const int64_t b = ((int64_t)blockIdx.x * 64 + threadIdx.x) >> 2;
    const int q = threadIdx.x & 3;
    if (b >= a.batch) return;   // whole quads retire together; DPP stays inside the quad
    const int n = EX ? NP : a.n, m = EX ? MP : a.m, N = a.N;
    const int64_t nn = (int64_t)n * n, nm = (int64_t)n * m, mm = (int64_t)m * m;
    const int64_t es = SOA ? a.batch : 1;                      // as dp_lane_kernel
    auto tb = [&](int64_t S) { return SOA ? b : b * S; };
    const T *Ag = (const T *)a.A + tb(nn), *Bg = (const T *)a.B + tb(nm);
    const T *Qg = (const T *)a.Q + tb(nn), *Rg = (const T *)a.R + tb(mm);

    T A[NP][NP], B[NP][MP], R[MP][MP], P[NP][NP];
    lane_load<T, NP, NP>(P, (const T *)a.Qf + tb(nn), n, n, (T)0, es);   // :58 P = Qf
    lane_load<T, NP, NP>(A, Ag, n, n, (T)0, es);
    lane_load<T, NP, MP>(B, Bg, n, m, (T)0, es);
    lane_load<T, MP, MP>(R, Rg, m, m, (T)1, es);
    // this lane's column of A and Q, row of A and B (dynamic q → loaded, not indexed)
    T Acol[NP], Qcol[NP], Arow[NP], Brow[MP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const bool ok = i < n && q < n;
        Acol[i] = ok ? Ag[(i + q * n) * es] : (T)0;
        Qcol[i] = ok ? Qg[(i + q * n) * es] : (T)0;
        Arow[i] = ok ? Ag[(q + i * n) * es] : (T)0;
    }
#pragma unroll
    for (int c = 0; c < MP; ++c) Brow[c] = (q < n && c < m) ? Bg[(q + c * n) * es] : (T)0;

    T *Kb = (T *)a.K + tb((int64_t)(N - 1) * nm);
    T *Pall = a.p_all ? (T *)a.P + tb(nn * N) : nullptr;
#define PS(i, j) ((i) >= (j) ? P[i][j] : P[j][i])
    auto store_Pcol = [&](T *dst) {   // lane q writes column q
        if (q >= n) return;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            T v = P[i][0];
#pragma unroll
            for (int r = 1; r < NP; ++r) v = q == r ? PS(i, r) : v;
            if (q == 0) v = PS(i, 0);
            if (i < n) dst[(i + q * n) * es] = v;
        }
    };
    if (Pall) store_Pcol(Pall + (int64_t)(N - 1) * nn * es);
    int info = 0;
    // linear terms (time-invariant q, r): p replicated, this lane's q[q], r replicated
    constexpr int LN = LIN ? NP : 1, LM = LIN ? MP : 1;
    T pv[LN], rv[LM], qq = (T)0;
    T *db = LIN ? (T *)a.d + tb((int64_t)(N - 1) * m) : nullptr;
    T *pall = (LIN && a.p_all) ? (T *)a.p + tb((int64_t)N * n) : nullptr;
    if constexpr (LIN) {
        const T *qg = (const T *)a.q + tb(n), *rg = (const T *)a.r + tb(m), *qf = (const T *)a.qf + tb(n);
#pragma unroll
        for (int i = 0; i < NP; ++i) pv[i] = i < n ? qf[i * es] : (T)0;
#pragma unroll
        for (int i = 0; i < MP; ++i) rv[i] = i < m ? rg[i * es] : (T)0;
        qq = q < n ? qg[q * es] : (T)0;
        if (pall && q < n) pall[((int64_t)(N - 1) * n + q) * es] = qf[q * es];
    }
    // this lane's column of P (row q by symmetry): P_N = Qf, then the P_[:,q] the knot forms
    T Pcol[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) Pcol[i] = (i < n && q < n) ? ((const T *)a.Qf + tb(nn))[(i + q * n) * es] : (T)0;
    for (int k = N - 1; k >= 1; --k) {   // :61
        T PB[NP][MP];
        if constexpr (LQRX_QUAD_PB_REPL || sizeof(T) == 4) {
#pragma unroll
            for (int i = 0; i < NP; ++i)
#pragma unroll
                for (int c = 0; c < MP; ++c) {                       // :38 PB = P B
                    T s = (T)0;
#pragma unroll
                    for (int l = 0; l < NP; ++l) s = fma(PS(i, l), B[l][c], s);
                    PB[i][c] = s;
                }
        } else {
            // :38 PB = P B split by rows (fp64): lane q forms row q from its own column P_[:,q] (the
            // upper-triangle part of that row differs from the symmetrised P by rounding only), the
            // quad broadcasts hand every lane the same PB — NP·MP FMAs per lane instead of NP²·MP.
            // fp32 keeps the replicated form: there the mixed-triangle row measurably loosens the
            // random-problem parity bound (tests/test_dp_lane_gpu.py::test_lane_parity_f32)
#pragma unroll
            for (int c = 0; c < MP; ++c) {
                T s = (T)0;
#pragma unroll
                for (int l = 0; l < NP; ++l) s = fma(Pcol[l], B[l][c], s);
                PB[0][c] = qfrom<0>(s);
                PB[1][c] = qfrom<1>(s);
                PB[2][c] = qfrom<2>(s);
                PB[3][c] = qfrom<3>(s);
            }
        }
        T PAc[NP];
#pragma unroll
        for (int i = 0; i < NP; ++i) {                           // :40 PA[:,q] = P A[:,q]
            T s = (T)0;
#pragma unroll
            for (int l = 0; l < NP; ++l) s = fma(PS(i, l), Acol[l], s);
            PAc[i] = s;
        }
        T E[MP][MP], Gq[MP];
#pragma unroll
        for (int c = 0; c < MP; ++c) {
#pragma unroll
            for (int d = 0; d <= c; ++d) {                       // :39 E = R + BᵀPB (lower)
                T s = R[c][d];
#pragma unroll
                for (int i = 0; i < NP; ++i) s = fma(B[i][c], PB[i][d], s);
                E[c][d] = s;
            }
            T s = (T)0;                                          // :41 G[:,q] = PBᵀA[:,q]
#pragma unroll
            for (int l = 0; l < NP; ++l) s = fma(PB[l][c], Acol[l], s);
            Gq[c] = s;
        }
        // :29 potrf 'U' of E (replicated), :30 potrs for this lane's column Kq = E⁻¹G[:,q]
        T L[MP][MP], Linv[MP];
#pragma unroll
        for (int j = 0; j < MP; ++j) {
            T d = E[j][j];
#pragma unroll
            for (int p = 0; p < j; ++p) d = fma(-L[j][p], L[j][p], d);
            if (!(d > (T)0) && info == 0) info = k;
            const T ri = lane_rsqrt<T>(d);
            Linv[j] = ri;
#pragma unroll
            for (int i = j + 1; i < MP; ++i) {
                T s = E[i][j];
#pragma unroll
                for (int p = 0; p < j; ++p) s = fma(-L[i][p], L[j][p], s);
                L[i][j] = s * ri;
            }
            L[j][j] = d * ri;
        }
        T y[MP], Kq[MP];
#pragma unroll
        for (int i = 0; i < MP; ++i) {
            T s = Gq[i];
#pragma unroll
            for (int p = 0; p < i; ++p) s = fma(-L[i][p], y[p], s);
            y[i] = s * Linv[i];
        }
#pragma unroll
        for (int i = MP - 1; i >= 0; --i) {
            T s = y[i];
#pragma unroll
            for (int p = i + 1; p < MP; ++p) s = fma(-L[p][i], Kq[p], s);
            Kq[i] = s * Linv[i];
        }
        if constexpr (MP == 1 && sizeof(T) == 8 && LQRX_QUAD_RCP) {
            // m = 1: potrs is K = G/E.  1/E as v_rcp + one Newton step (≈ 2e-15 relative, rcp_nr)
            // is 3 fp64 instructions where 1/√E (v_rsq + two Newton steps) and the two scalings
            // by it took 9: the backward knot is VALU-issue-bound (≈ 80 VALU per knot on one wave
            // per SIMD, tools/chain_len.py), so the 6 instructions are what it saves.  The pivot
            // test and the L used by the linear terms are unchanged.  fp64 only: in fp32 the
            // random-problem parity bound of test_lane_parity_f32 is conditioning-tight and the
            // float rcp step moved it past its limit.
            Kq[0] = Gq[0] * rcp_nr(E[0][0]);
        }
        if (q < n) {
            T *Kk = Kb + ((int64_t)(k - 1) * nm + q * m) * es;    // sol.K[k] column q
#pragma unroll
            for (int c = 0; c < MP; ++c)
                if (c < m) Kk[c * es] = Kq[c];
        }
        if constexpr (LIN) {
            // d = E⁻¹(r + Bᵀp) (replicated), p_new[q] = q[q] + A[:,q]ᵀp − G[:,q]ᵀd
            T yl[MP], dv[MP];
#pragma unroll
            for (int i = 0; i < MP; ++i) {
                T s = (T)0;
#pragma unroll
                for (int l = 0; l < NP; ++l) s = fma(B[l][i], pv[l], s);
                s = rv[i] + s;
#pragma unroll
                for (int c = 0; c < i; ++c) s = fma(-L[i][c], yl[c], s);
                yl[i] = s * Linv[i];
            }
#pragma unroll
            for (int i = MP - 1; i >= 0; --i) {
                T s = yl[i];
#pragma unroll
                for (int c = i + 1; c < MP; ++c) s = fma(-L[c][i], dv[c], s);
                dv[i] = s * Linv[i];
            }
            if (q < m) {   // lane q stores d_k[q]
                T v = dv[0];
#pragma unroll
                for (int c = 1; c < MP; ++c) v = q == c ? dv[c] : v;
                db[((int64_t)(k - 1) * m + q) * es] = v;
            }
            T s = (T)0, t = (T)0;
#pragma unroll
            for (int l = 0; l < NP; ++l) s = fma(Acol[l], pv[l], s);
#pragma unroll
            for (int c = 0; c < MP; ++c) t = fma(Gq[c], dv[c], t);
            const T pn = qq + s - t;
            if (pall && q < n) pall[((int64_t)(k - 1) * n + q) * es] = pn;
            pv[0] = qfrom<0>(pn);
            pv[1] = qfrom<1>(pn);
            pv[2] = qfrom<2>(pn);
            pv[3] = qfrom<3>(pn);
        }
        // :51 P_[:,q] = Q[:,q] + AᵀPA[:,q] − Gᵀ Kq = Q[:,q] + Aᵀ(PA[:,q] − PB·Kq)
        // (G = PBᵀA, so GᵀKq = Aᵀ(PB Kq): no full G)
        T wv[NP], Pn[NP];
#pragma unroll
        for (int l = 0; l < NP; ++l) {
            T s = PAc[l];
#pragma unroll
            for (int c = 0; c < MP; ++c) s = fma(-PB[l][c], Kq[c], s);
            wv[l] = s;
        }
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            T s = Qcol[i];
#pragma unroll
            for (int l = 0; l < NP; ++l) s = fma(A[l][i], wv[l], s);
            Pn[i] = s;
        }
#pragma unroll
        for (int i = 0; i < NP; ++i) Pcol[i] = Pn[i];
        // re-replicate the lower triangle: P[i][r] (i ≥ r) from lane r
#pragma unroll
        for (int i = 0; i < NP; ++i) P[i][0] = qfrom<0>(Pn[i]);
#pragma unroll
        for (int i = 1; i < NP; ++i) P[i][1] = qfrom<1>(Pn[i]);
#pragma unroll
        for (int i = 2; i < NP; ++i) P[i][2] = qfrom<2>(Pn[i]);
        P[3][3] = qfrom<3>(Pn[3]);
        if (Pall) store_Pcol(Pall + (int64_t)(k - 1) * nn * es);
    }
    if (!a.p_all) store_Pcol((T *)a.P + tb(nn));
    if (a.info && q == 0) a.info[b] = info;
    if constexpr (LIN) {
        if (!a.p_all && q < n) {
            T v = pv[0];
#pragma unroll
            for (int i = 1; i < NP; ++i) v = q == i ? pv[i] : v;
            ((T *)a.p)[tb(n) + q * es] = v;
        }
    }

    // forward rollout :66-70 — x replicated; lane q forms x_{k+1}[q]
    T *Xb = (T *)a.X + tb((int64_t)N * n), *Ub = (T *)a.U + tb((int64_t)(N - 1) * m);
    const T *x0 = (const T *)a.x0 + tb(n);
    T x[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) x[i] = i < n ? x0[i * es] : (T)0;
    if (q < n) Xb[q * es] = q == 0 ? x[0] : (q == 1 ? x[1] : (q == 2 ? x[2] : x[3]));
    if (N < 2) return;                 // no controls (the clamped fetches below need knot 1)
    constexpr int RD = 8;
    T ring[RD][MP][NP], dring[LIN ? RD : 1];
    const int64_t kst = nm * es, dst = (int64_t)m * es;     // knot strides of K and d
    // The ring: slot d of a group holds knot k0 + d; its refill fetches knot k0 + d + RD from
    // the group's base pointer (scalar offsets d·stride, no per-knot index arithmetic), or —
    // in the one group whose refills run past the last knot — from knot min(k, N − 1).
    // Unconditional loads with nothing applied to them until the knot uses them, so the
    // compiler's waits count the ring instead of draining it at every knot: a padding entry
    // (i ≥ m or j ≥ n) reads another element of K_k (an index clamp, not a select the compiler
    // could turn into a branch) — finite — and only ever meets a zero (x[j ≥ n] = 0;
    // u[i ≥ m] meets Brow[i] = 0 and is not stored).
    auto fetch = [&](const T *Kk, T (&d)[MP][NP]) {
#pragma unroll
        for (int j = 0; j < NP; ++j)
#pragma unroll
            for (int i = 0; i < MP; ++i) d[i][j] = Kk[min(i + j * m, (int)nm - 1) * es];
    };
    auto fetch_d = [&](const T *dk, T &d) {   // lane q < m: d_k[q] (q ≥ m: unused)
        if constexpr (LIN) d = dk[min(q, m - 1) * es];
    };
    auto kat = [&](int k) { return Kb + (int64_t)(min(k, N - 1) - 1) * kst; };
    auto dat = [&](int k) { return db + (int64_t)(min(k, N - 1) - 1) * dst; };
    // K_k was written by this quad's own lanes above; make those stores visible to the
    // quad's loads (other lanes' stores: complete them and drop any stale L1 line, once)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
    for (int d = 0; d < RD; ++d) {
        fetch(kat(1 + d), ring[d]);
        if constexpr (LIN) fetch_d(dat(1 + d), dring[d]);
    }
    // knot k from ring slot d; REFILL 1: the slot then fetches knot k + RD at (Kr, Dr)
    auto knot = [&](int k, T (&slot)[MP][NP], T &dslot, bool refill, const T *Kr, const T *Dr)
        __attribute__((always_inline)) {
        T Kc[MP][NP], dq = (T)0;
#pragma unroll
        for (int j = 0; j < NP; ++j)
#pragma unroll
            for (int i = 0; i < MP; ++i) Kc[i][j] = slot[i][j];
        if constexpr (LIN) dq = dslot;
        if (refill) {
            fetch(Kr, slot);
            fetch_d(Dr, dslot);
        }
        T u[MP];
#pragma unroll
        for (int i = 0; i < MP; ++i) {
            T s = (T)0;
#pragma unroll
            for (int j = 0; j < NP; ++j) s = fma(Kc[i][j], x[j], s);
            if constexpr (LIN) {   // u = −(K x + d), d_k[i] from lane i
                const T di = i == 0 ? qfrom<0>(dq) : i == 1 ? qfrom<1>(dq) : i == 2 ? qfrom<2>(dq) : qfrom<3>(dq);
                u[i] = -(s + di);
            } else {
                u[i] = -s;
            }
            if (q == 0 && i < m) Ub[((int64_t)(k - 1) * m + i) * es] = u[i];
        }
        T s = (T)0;
#pragma unroll
        for (int j = 0; j < NP; ++j) s = fma(Arow[j], x[j], s);
#pragma unroll
        for (int c = 0; c < MP; ++c) s = fma(Brow[c], u[c], s);
        if (q < n) Xb[((int64_t)k * n + q) * es] = s;
        x[0] = qfrom<0>(s);
        x[1] = qfrom<1>(s);
        x[2] = qfrom<2>(s);
        x[3] = qfrom<3>(s);
    };
    // whole groups of RD knots (no per-knot exit test) whose refills stay inside the horizon,
    // then at most one group with clamped refills, then the < RD remaining knots
    int k0 = 1;
    for (; k0 + 2 * RD - 1 <= N - 1; k0 += RD) {
        const T *Kg = Kb + (int64_t)(k0 + RD - 1) * kst;
        const T *Dg = LIN ? db + (int64_t)(k0 + RD - 1) * dst : nullptr;
#pragma unroll
        for (int d = 0; d < RD; ++d)
            knot(k0 + d, ring[d], dring[LIN ? d : 0], true, Kg + d * kst, LIN ? Dg + d * dst : nullptr);
    }
    if (k0 + RD - 1 <= N - 1) {
#pragma unroll
        for (int d = 0; d < RD; ++d)
            knot(k0 + d, ring[d], dring[LIN ? d : 0], true, kat(k0 + d + RD), LIN ? dat(k0 + d + RD) : nullptr);
        k0 += RD;
    }
#pragma unroll
    for (int d = 0; d < RD - 1; ++d)
        if (k0 + d <= N - 1) knot(k0 + d, ring[d], dring[LIN ? d : 0], false, nullptr, nullptr);
#undef PS
}

// ---------------------------------------------------------------------------------------
// dp_hex_kernel: SIXTEEN LANES PER TRAJECTORY (one DPP row), n ≤ 4, m ≤ 4, time-invariant.
// BASELINE cfg2 (cartpole B = 4096) is a 101-knot serial chain per trajectory: with four lanes
// per trajectory the whole batch is 256 waves, one SIMD in four busy, and each knot a ~100-op
// dependent chain per lane.  Here lane (i, j) = 4i + j of the row owns ONE element of every
// n×n quantity, so the per-knot chain is a handful of FMAs between DPP reductions, and the
// 1024 waves fill every SIMD:
//   PA[i][j] = Σ_l P[i][l]A[l][j]         P[i][l] by quad broadcast (the 4 lanes of row i
//                                          are a DPP quad)
//   PB[i][c] = Σ_l P[i][l]B[l][c]         the same broadcasts, every lane of the quad
//   E[c][d]  = R[c][d] + Σ_t B[t][c]PB[t][d]   PB[t] by row_newbcast from quad t
//   G[c][j]  = Σ_t PB[t][c]A[t][j]         (= BᵀPA for symmetric P)
//   potrf E (replicated), K[:, j] = E⁻¹G[:, j]  (every lane, its column j)
//   P_[i][j] = Q[i][j] + Σ_l A[l][i](PA[l][j] − Σ_c PB[l][c]K[c][j])   (W from quad l by
//              row_ror 4s: the same AᵀPA − GᵀK as the quad kernel); the upper triangle then
//              takes the lower one's values (one bpermute), the symmetric form of the others
// Rollout: lane (i, j) holds x[j]; x and K_k's rows reach every lane of the quad by
// broadcasts, u = −Kx and (Ax + Bu)[i] are the quad kernel's FMA chains (the same value in
// every lane of the quad), and x_{k+1}[j] comes back from quad j by the same rotations.  The rotation direction is
// probed once (the quad index itself rotated), so no lane map is assumed.
template <int CTRL> __device__ __forceinline__ int dppi(int v)
{
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
template <typename T, int MP, bool SOA>
__global__ __launch_bounds__(64) void dp_hex_kernel(const DpArgs a)
{
    constexpr int NP = 4;
    const int64_t b = ((int64_t)blockIdx.x * 64 + threadIdx.x) >> 4;
    const int r16 = threadIdx.x & 15, i = r16 >> 2, j = r16 & 3;
    if (b >= a.batch) return;   // whole rows retire together; DPP stays inside the row
    const int n = a.n, m = a.m, N = a.N;
    const int64_t nn = (int64_t)n * n, nm = (int64_t)n * m, mm = (int64_t)m * m;
    const int64_t es = SOA ? a.batch : 1;
    auto tb = [&](int64_t S) { return SOA ? b : b * S; };
    const T *Ag = (const T *)a.A + tb(nn), *Bg = (const T *)a.B + tb(nm);
    const T *Qg = (const T *)a.Q + tb(nn), *Rg = (const T *)a.R + tb(mm);
    // the quads whose values row_ror 4s delivers to this lane (s = 1, 2, 3)
    const int q1 = dppi<0x124>(i), q2 = dppi<0x128>(i), q3 = dppi<0x12C>(i);
    const int qs[4] = {i, q1, q2, q3};
    auto Ael = [&](int r, int c) { return (r < n && c < n) ? Ag[(r + c * n) * es] : (T)0; };
    T p = (i < n && j < n) ? ((const T *)a.Qf + tb(nn))[(i + j * n) * es] : (T)0;   // :58 P = Qf
    const T qij = (i < n && j < n) ? Qg[(i + j * n) * es] : (T)0;
    T Acolj[NP], Acoef[NP];
#pragma unroll
    for (int l = 0; l < NP; ++l) {
        Acolj[l] = Ael(l, j);          // A[l][j]       (PA)
        Acoef[l] = Ael(qs[l], i);      // A[q_s][i]     (P_, W from quad q_s)
    }
    T Bl[NP][MP], Bi[MP], R[MP][MP], Arow[NP];
#pragma unroll
    for (int l = 0; l < NP; ++l) {
        Arow[l] = Ael(i, l);           // A[i][l]       (rollout)
#pragma unroll
        for (int c = 0; c < MP; ++c) Bl[l][c] = (l < n && c < m) ? Bg[(l + c * n) * es] : (T)0;
    }
#pragma unroll
    for (int c = 0; c < MP; ++c) {
        Bi[c] = (i < n && c < m) ? Bg[(i + c * n) * es] : (T)0;
#pragma unroll
        for (int d = 0; d < MP; ++d)
            R[c][d] = (c < m && d < m) ? Rg[(c + d * m) * es] : (c == d ? (T)1 : (T)0);
    }
    T *Kb = (T *)a.K + tb((int64_t)(N - 1) * nm);
    T *Pall = a.p_all ? (T *)a.P + tb(nn * N) : nullptr;
    const bool own = i < n && j < n;
    if (Pall && own) Pall[((int64_t)(N - 1) * nn + i + j * n) * es] = p;
    int info = 0;
    for (int k = N - 1; k >= 1; --k) {   // :61
        const T P0 = qfrom<0>(p), P1 = qfrom<1>(p), P2 = qfrom<2>(p), P3 = qfrom<3>(p);
        T PB[MP];
#pragma unroll
        for (int c = 0; c < MP; ++c) {                              // :38 PB[i][c] (same in the quad)
            T sv = P0 * Bl[0][c];
            sv = fma(P1, Bl[1][c], sv);
            sv = fma(P2, Bl[2][c], sv);
            PB[c] = fma(P3, Bl[3][c], sv);
        }
        T pa = P0 * Acolj[0];                                       // :40 PA[i][j]
        pa = fma(P1, Acolj[1], pa);
        pa = fma(P2, Acolj[2], pa);
        pa = fma(P3, Acolj[3], pa);
        // PB[t][·] of every row t (lane 4t of the DPP row holds it) → E, G by the quad kernel's
        // FMA chains, the same value in every lane of the row
        T PBt[NP][MP];
#pragma unroll
        for (int c = 0; c < MP; ++c) {
            PBt[0][c] = qbcast<0x150>(PB[c]);                       // row_newbcast:0
            PBt[1][c] = qbcast<0x154>(PB[c]);                       // row_newbcast:4
            PBt[2][c] = qbcast<0x158>(PB[c]);                       // row_newbcast:8
            PBt[3][c] = qbcast<0x15C>(PB[c]);                       // row_newbcast:12
        }
        T E[MP][MP], G[MP];
#pragma unroll
        for (int c = 0; c < MP; ++c) {
#pragma unroll
            for (int d = 0; d <= c; ++d) {                          // :39 E = R + BᵀPB
                T sv = R[c][d];
#pragma unroll
                for (int t = 0; t < NP; ++t) sv = fma(Bl[t][c], PBt[t][d], sv);
                E[c][d] = sv;
            }
            T sv = PBt[0][c] * Acolj[0];                            // :41 G[c][j] = Σ_t PB[t][c]A[t][j]
#pragma unroll
            for (int t = 1; t < NP; ++t) sv = fma(PBt[t][c], Acolj[t], sv);
            G[c] = sv;
        }
        // :29 potrf 'U' of E (replicated), :30 potrs for column j: K[:, j] = E⁻¹G[:, j]
        T L[MP][MP], Linv[MP];
#pragma unroll
        for (int jj = 0; jj < MP; ++jj) {
            T d = E[jj][jj];
#pragma unroll
            for (int pp = 0; pp < jj; ++pp) d = fma(-L[jj][pp], L[jj][pp], d);
            if (!(d > (T)0) && info == 0) info = k;
            const T ri = lane_rsqrt<T>(d);
            Linv[jj] = ri;
#pragma unroll
            for (int ii = jj + 1; ii < MP; ++ii) {
                T sv = E[ii][jj];
#pragma unroll
                for (int pp = 0; pp < jj; ++pp) sv = fma(-L[ii][pp], L[jj][pp], sv);
                L[ii][jj] = sv * ri;
            }
            L[jj][jj] = d * ri;
        }
        T y[MP], Kc[MP];
#pragma unroll
        for (int ii = 0; ii < MP; ++ii) {
            T sv = G[ii];
#pragma unroll
            for (int pp = 0; pp < ii; ++pp) sv = fma(-L[ii][pp], y[pp], sv);
            y[ii] = sv * Linv[ii];
        }
#pragma unroll
        for (int ii = MP - 1; ii >= 0; --ii) {
            T sv = y[ii];
#pragma unroll
            for (int pp = ii + 1; pp < MP; ++pp) sv = fma(-L[pp][ii], Kc[pp], sv);
            Kc[ii] = sv * Linv[ii];
        }
        if (i == 0 && j < n) {                                      // sol.K[k] column j
            T *Kk = Kb + ((int64_t)(k - 1) * nm + j * m) * es;
#pragma unroll
            for (int c = 0; c < MP; ++c)
                if (c < m) Kk[c * es] = Kc[c];
        }
        // :51 P_[i][j] = Q[i][j] + Σ_l A[l][i]·W[l][j],  W = PA − PB·K (row l, column j)
        T wv = pa;
#pragma unroll
        for (int c = 0; c < MP; ++c) wv = fma(-PB[c], Kc[c], wv);
        const T w1 = qbcast<0x124>(wv), w2 = qbcast<0x128>(wv), w3 = qbcast<0x12C>(wv);
        T pn = fma(Acoef[0], wv, qij);
        pn = fma(Acoef[1], w1, pn);
        pn = fma(Acoef[2], w2, pn);
        pn = fma(Acoef[3], w3, pn);
        // symmetric form, as the quad / MFMA kernels: the upper triangle mirrors the lower
        // (left unsymmetrised, rounding asymmetry grows along ill-conditioned horizons)
        const T pt = __shfl(pn, (int)(threadIdx.x & ~15u) | (4 * j + i), 64);
        p = own ? (i >= j ? pn : pt) : (T)0;
        if (Pall && own) Pall[((int64_t)(k - 1) * nn + i + j * n) * es] = p;
    }
    if (!a.p_all && own) ((T *)a.P + tb(nn))[(i + j * n) * es] = p;
    if (a.info && r16 == 0) a.info[b] = info;

    // forward rollout :66-70 — lane (i, j) holds x[j]
    T *Xb = (T *)a.X + tb((int64_t)N * n), *Ub = (T *)a.U + tb((int64_t)(N - 1) * m);
    const T *x0 = (const T *)a.x0 + tb(n);
    T xj = j < n ? x0[j * es] : (T)0;
    if (i == 0 && j < n) Xb[j * es] = xj;
    constexpr int RD = 8;
    T ring[RD][MP];
    auto fetch = [&](int k, T (&d)[MP]) {   // K_k[:, j]
        if (k > N - 1) return;
        const T *Kk = Kb + (int64_t)(k - 1) * nm * es;
#pragma unroll
        for (int c = 0; c < MP; ++c) d[c] = (c < m && j < n) ? Kk[(c + j * m) * es] : (T)0;
    };
    // K_k was written by lanes (0, j) of this row above: make those stores visible
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
    for (int d = 0; d < RD; ++d) fetch(1 + d, ring[d]);
    const int s_of_j = j == qs[0] ? 0 : j == qs[1] ? 1 : j == qs[2] ? 2 : 3;
    for (int k0 = 1; k0 <= N - 1; k0 += RD) {
#pragma unroll
        for (int d = 0; d < RD; ++d) {
            const int k = k0 + d;
            if (k > N - 1) break;
            T Kc[MP];
#pragma unroll
            for (int c = 0; c < MP; ++c) Kc[c] = ring[d][c];
            fetch(k + RD, ring[d]);
            // x and K_k's rows by quad broadcasts, then the quad kernel's FMA chains: every lane
            // of the quad forms the same u and (Ax + Bu)[i]
            const T x0v = qfrom<0>(xj), x1v = qfrom<1>(xj), x2v = qfrom<2>(xj), x3v = qfrom<3>(xj);
            T u[MP];
#pragma unroll
            for (int c = 0; c < MP; ++c) {
                T sv = qfrom<0>(Kc[c]) * x0v;                       // u = −K x
                sv = fma(qfrom<1>(Kc[c]), x1v, sv);
                sv = fma(qfrom<2>(Kc[c]), x2v, sv);
                sv = fma(qfrom<3>(Kc[c]), x3v, sv);
                u[c] = -sv;
                if (r16 == c && c < m) Ub[((int64_t)(k - 1) * m + c) * es] = u[c];
            }
            T xi = Arow[0] * x0v;                                   // (A x)[i]
            xi = fma(Arow[1], x1v, xi);
            xi = fma(Arow[2], x2v, xi);
            xi = fma(Arow[3], x3v, xi);
#pragma unroll
            for (int c = 0; c < MP; ++c) xi = fma(Bi[c], u[c], xi); // + (B u)[i]
            if (j == 0 && i < n) Xb[((int64_t)k * n + i) * es] = xi;
            const T x1 = qbcast<0x124>(xi), x2 = qbcast<0x128>(xi), x3 = qbcast<0x12C>(xi);
            xj = s_of_j == 0 ? xi : s_of_j == 1 ? x1 : s_of_j == 2 ? x2 : x3;
        }
    }
}

template <typename T, int MP>
static hipError_t launch_hex(const DpArgs &a, hipStream_t s)
{
    dim3 grid((unsigned)((a.batch * 16 + 63) / 64)), block(64);
    if (a.layout == 1) hipLaunchKernelGGL((dp_hex_kernel<T, MP, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((dp_hex_kernel<T, MP, false>), grid, block, 0, s, a);
    return hipGetLastError();
}

template <typename T, int NP, int MP>
static hipError_t launch_lane(const DpArgs &a, hipStream_t s)
{
    dim3 grid((unsigned)((a.batch + 63) / 64)), block(64);
    const bool tv = a.tv_AB || a.tv_QR, soa = a.layout == 1;
    if (a.lin && tv && soa) hipLaunchKernelGGL((dp_lane_kernel<T, NP, MP, true, true, true>), grid, block, 0, s, a);
    else if (a.lin && tv) hipLaunchKernelGGL((dp_lane_kernel<T, NP, MP, true, false, true>), grid, block, 0, s, a);
    else if (a.lin && soa) hipLaunchKernelGGL((dp_lane_kernel<T, NP, MP, false, true, true>), grid, block, 0, s, a);
    else if (a.lin) hipLaunchKernelGGL((dp_lane_kernel<T, NP, MP, false, false, true>), grid, block, 0, s, a);
    else if (tv && soa) hipLaunchKernelGGL((dp_lane_kernel<T, NP, MP, true, true>), grid, block, 0, s, a);
    else if (tv) hipLaunchKernelGGL((dp_lane_kernel<T, NP, MP, true, false>), grid, block, 0, s, a);
    else if (soa) hipLaunchKernelGGL((dp_lane_kernel<T, NP, MP, false, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((dp_lane_kernel<T, NP, MP, false, false>), grid, block, 0, s, a);
    return hipGetLastError();
}

bool dp_lane_supported(int n, int m) { return n >= 1 && m >= 1 && n <= 4 && m <= 4; }

// quad kernel for small batches: 4·batch lanes still fit ≤ 4 waves per CU, where the
// lane kernel would leave most CUs idle.  LQRX_DP_SMALL=lane|quad overrides (tests).
static bool use_quad(const DpArgs &a)
{
    if (a.tv_AB || a.tv_QR || a.n < 3 || a.n > 4) return false;
    const char *e = std::getenv("LQRX_DP_SMALL");
    if (e && e[0] == 'l') return false;
    if (e && e[0] == 'q') return true;
    return a.batch <= 16384;
}

template <typename T, int MP>
static hipError_t launch_quad(const DpArgs &a, hipStream_t s)
{
    dim3 grid((unsigned)((a.batch * 4 + 63) / 64)), block(64);
    if (a.lin && a.layout == 1) hipLaunchKernelGGL((dp_quad_kernel<T, MP, true, true>), grid, block, 0, s, a);
    else if (a.lin) hipLaunchKernelGGL((dp_quad_kernel<T, MP, false, true>), grid, block, 0, s, a);
    else if (a.layout == 1) hipLaunchKernelGGL((dp_quad_kernel<T, MP, true>), grid, block, 0, s, a);
    else if (a.n == 4 && a.m == MP) hipLaunchKernelGGL((dp_quad_kernel<T, MP, false, false, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((dp_quad_kernel<T, MP, false>), grid, block, 0, s, a);
    return hipGetLastError();
}

// hex kernel (16 lanes per trajectory; n ≤ 4, m ≤ 4, time-invariant, no linear terms): an
// A/B alternative selected by LQRX_DP_SMALL=hex only — measured slower than the quad kernel
// on cfg2 (0.082 vs 0.055 ms): the replicated m-sized work and the broadcasts
// leave each lane about as many dependent instructions per knot as the quad's lane has.
static bool use_hex(const DpArgs &a)
{
    if (a.tv_AB || a.tv_QR || a.lin || a.n > 4 || a.m > 4) return false;
    const char *e = std::getenv("LQRX_DP_SMALL");
    return e && e[0] == 'h';
}

hipError_t dp_lane_launch(const DpArgs &a, hipStream_t s)
{
    const int np = a.n <= 2 ? 2 : 4, mp = a.m <= 1 ? 1 : (a.m <= 2 ? 2 : 4);
    if (use_hex(a)) {
        if (a.dtype == 0) {
            if (mp == 1) return launch_hex<double, 1>(a, s);
            if (mp == 2) return launch_hex<double, 2>(a, s);
            return launch_hex<double, 4>(a, s);
        }
        if (mp == 1) return launch_hex<float, 1>(a, s);
        if (mp == 2) return launch_hex<float, 2>(a, s);
        return launch_hex<float, 4>(a, s);
    }
    if (use_quad(a)) {
        if (a.dtype == 0) {
            if (mp == 1) return launch_quad<double, 1>(a, s);
            if (mp == 2) return launch_quad<double, 2>(a, s);
            return launch_quad<double, 4>(a, s);
        }
        if (mp == 1) return launch_quad<float, 1>(a, s);
        if (mp == 2) return launch_quad<float, 2>(a, s);
        return launch_quad<float, 4>(a, s);
    }
    if (a.dtype == 0) {
        if (np == 2 && mp == 1) return launch_lane<double, 2, 1>(a, s);
        if (np == 2 && mp == 2) return launch_lane<double, 2, 2>(a, s);
        if (np == 4 && mp == 1) return launch_lane<double, 4, 1>(a, s);
        if (np == 4 && mp == 2) return launch_lane<double, 4, 2>(a, s);
        if (np == 4 && mp == 4) return launch_lane<double, 4, 4>(a, s);
    } else {
        if (np == 2 && mp == 1) return launch_lane<float, 2, 1>(a, s);
        if (np == 2 && mp == 2) return launch_lane<float, 2, 2>(a, s);
        if (np == 4 && mp == 1) return launch_lane<float, 4, 1>(a, s);
        if (np == 4 && mp == 2) return launch_lane<float, 4, 2>(a, s);
        if (np == 4 && mp == 4) return launch_lane<float, 4, 4>(a, s);
    }
    return hipErrorNotSupported;
}

} // namespace lqrx
