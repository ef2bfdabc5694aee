// lqrx_kkt.hip — batched block-tridiagonal KKT solve on gfx950: one inner solve of
// CholeskySolver._solve! (/root/reference/src/cholesky_solver.jl:166-182) per trajectory.
//
// Mapping (small blocks, e.g. Dubins n=3 m=2): ONE LANE PER TRAJECTORY, 64 trajectories
// per wave.  The reference's five phases are fused into two sweeps over the horizon:
//
//   forward  k = 0 … N-1  (one-knot lookahead for the aliased A ≡ previous-C block):
//     shur!/copy_shur!  (jacobian_blocks.jl:231-286) for knot k+1 — YYt = Y H⁻¹ Yᵀ and
//       r = Y H⁻¹ g streamed column by column from HBM (H diagonal: h_mode 2, or dense /
//       block-diagonal factored by a w×w Cholesky, block_cholesky.jl:55-101);
//     cholesky!(U[k], F[k])  (cholesky_solve.jl:47-67);
//     forward_substitution!  (cholesky_solve.jl:93-117);
//     the factor blocks B, C, D, E, F and the forward μ, λ go to a scratch slab.
//   backward k = N-1 … 0:
//     backward_substitution!  (cholesky_solve.jl:119-143), and with a one-knot lag
//     calc_residual! + calc_primals!  (cholesky_solver.jl:195-236): δz_k = −H_k⁻¹ res_k.
//
// Every per-knot operation is the oracle's (oracle/lqr_oracle.c) scalar loop, executed by
// each lane on its own trajectory; register arrays are sized by compile-time maxima of the
// block dimensions (template), loops run to the runtime sizes.
#include "lqrx_internal.h"
#include "lqrx_tile.h"
#include "lqrx_stage.h"
#include <hip/hip_runtime.h>

namespace lqrx {

#define KIDX(i, j, ld) ((i) + (j) * (ld))

// upper Cholesky of an n×n (n ≤ NM) column-major array, potrf 'U'; returns false on a
// non-positive pivot (the factorisation continues with garbage, like LAPACK's caller here)
template <int NM>
__device__ __forceinline__ bool potrf_u(double *A, int n)
{
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NM; ++j) {
        if (j < n) {
            double d = A[KIDX(j, j, NM)];
#pragma unroll
            for (int p = 0; p < NM; ++p)
                if (p < j) d -= A[KIDX(p, j, NM)] * A[KIDX(p, j, NM)];
            ok = ok && (d > 0.0);
            double s = sqrt(d);
            double si = rcp_nr2(s);
            A[KIDX(j, j, NM)] = s;
#pragma unroll
            for (int c = 0; c < NM; ++c)
                if (c > j && c < n) {
                    double v = A[KIDX(j, c, NM)];
#pragma unroll
                    for (int p = 0; p < NM; ++p)
                        if (p < j) v -= A[KIDX(p, j, NM)] * A[KIDX(p, c, NM)];
                    A[KIDX(j, c, NM)] = v * si;
                }
        }
    }
    return ok;
}

// X (n×nr, ld XM) ← U⁻ᵀ X   (trsm 'L','U','T','N'); U n×n with ld UM
template <int UM, int XM, int NRM>
__device__ __forceinline__ void trsm_ut(const double *U, int n, double *X, int nr)
{
#pragma unroll
    for (int c = 0; c < NRM; ++c)
        if (c < nr) {
#pragma unroll
            for (int i = 0; i < UM; ++i)
                if (i < n) {
                    double s = X[KIDX(i, c, XM)];
#pragma unroll
                    for (int p = 0; p < UM; ++p)
                        if (p < i) s -= U[KIDX(p, i, UM)] * X[KIDX(p, c, XM)];
                    X[KIDX(i, c, XM)] = s * rcp_nr2(U[KIDX(i, i, UM)]);
                }
        }
}

// x ← U⁻¹ x  (trsv 'U','N')
template <int UM>
__device__ __forceinline__ void trsv_un(const double *U, int n, double *x)
{
#pragma unroll
    for (int ii = UM - 1; ii >= 0; --ii)
        if (ii < n) {
            double s = x[ii];
#pragma unroll
            for (int p = 0; p < UM; ++p)
                if (p > ii && p < n) s -= U[KIDX(ii, p, UM)] * x[p];
            x[ii] = s * rcp_nr2(U[KIDX(ii, ii, UM)]);
        }
}

// knot metadata (lqrx_api.cpp kkt_layout): n1, p, n2, w, oY, oy, oH, og
struct KMeta {
    int n1, p, n2, w, oY, oy, oH, og;
};
__device__ __forceinline__ KMeta kmeta(const int32_t *m, int k)
{
    const int32_t *q = m + 8 * k;
    return KMeta{q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]};
}

// H_k⁻¹ application data for one knot: diagonal inverse, or the w×w upper factor.
template <int WM> struct HFac {
    double f[WM * WM]; // dense: upper factor (ld WM);  diag: f[i] = 1/h_i
};

template <int WM>
__device__ __forceinline__ bool load_hfac(HFac<WM> &hf, const double *H, int w, int hmode)
{
    if (hmode == 2) {
#pragma unroll
        for (int i = 0; i < WM; ++i) hf.f[i] = (i < w) ? rcp_nr2(H[i]) : 0.0; // block_cholesky.jl:86 inv
        return true;
    }
#pragma unroll
    for (int j = 0; j < WM; ++j)
#pragma unroll
        for (int i = 0; i < WM; ++i) hf.f[KIDX(i, j, WM)] = (i < w && j < w) ? H[i + j * w] : 0.0;
    return potrf_u<WM>(hf.f, w); // block_cholesky.jl:63 potrf!
}

template <int WM>
__device__ __forceinline__ void hinv_apply(const HFac<WM> &hf, double *x, int w, int hmode)
{
    if (hmode == 2) {
#pragma unroll
        for (int i = 0; i < WM; ++i)
            if (i < w) x[i] *= hf.f[i];
        return;
    }
    // potrs: Uᵀ y = x, U z = y
#pragma unroll
    for (int i = 0; i < WM; ++i)
        if (i < w) {
            double s = x[i];
#pragma unroll
            for (int p = 0; p < WM; ++p)
                if (p < i) s -= hf.f[KIDX(p, i, WM)] * x[p];
            x[i] = s * rcp_nr2(hf.f[KIDX(i, i, WM)]);
        }
    trsv_un<WM>(hf.f, w, x);
}

// Schur pieces of one knot in block form (shur! + copy_shur!, jacobian_blocks.jl:231-286):
// with Y = [D2; C; D1] (segments 1, s, 2 of p1, ps, p2 rows) and YYt = Y H⁻¹ Yᵀ:
//   A = YYt[1,1] (added to the previous knot's C),  B = YYt[s,s],  C = YYt[2,2],
//   D = YYt[1,s],  E = YYt[s,2],  F = YYt[1,2];   r = Y H⁻¹ g split as r1, rs, r2.
// All register arrays are indexed statically (the segment offsets are runtime values, so
// they only ever enter global addresses).
template <int P1M, int PSM, int P2M> struct ShurBlk {
    double A[P1M * P1M], B[PSM * PSM], C[P2M * P2M], D[P1M * PSM], E[PSM * P2M], F[P1M * P2M];
    double r1[P1M], rs[PSM], r2[P2M];
};

template <int M1, int M2>
__device__ __forceinline__ void outer_acc(double *X, const double *u, const double *v, double s)
{
#pragma unroll
    for (int j = 0; j < M2; ++j)
#pragma unroll
        for (int i = 0; i < M1; ++i) X[KIDX(i, j, M1)] += u[i] * v[j] * s;
}

template <int M>
__device__ __forceinline__ void sym_acc(double *X, const double *u, double s)
{
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const double uj = u[j] * s;
#pragma unroll
        for (int i = 0; i <= j; ++i) X[KIDX(i, j, M)] = fma(u[i], uj, X[KIDX(i, j, M)]);
    }
}

template <int M> __device__ __forceinline__ void sym_mirror(double *X)
{
#pragma unroll
    for (int j = 0; j < M; ++j)
#pragma unroll
        for (int i = j + 1; i < M; ++i) X[KIDX(i, j, M)] = X[KIDX(j, i, M)];
}

template <int P1M, int PSM, int P2M, int WM>
__device__ __forceinline__ bool compute_shur(ShurBlk<P1M, PSM, P2M> &s, const double *Yk,
                                             const double *Hk, const double *gk, const KMeta &km,
                                             int hmode, int ginv)
{
    const int p1 = km.n1, ps = km.p, p2 = km.n2, rows = p1 + ps + p2, w = km.w;
    HFac<WM> hf;
    bool ok = true;
    if (ginv) ok = load_hfac<WM>(hf, Hk, w, hmode);
#pragma unroll
    for (int i = 0; i < P1M * P1M; ++i) s.A[i] = 0.0;
#pragma unroll
    for (int i = 0; i < PSM * PSM; ++i) s.B[i] = 0.0;
#pragma unroll
    for (int i = 0; i < P2M * P2M; ++i) s.C[i] = 0.0;
#pragma unroll
    for (int i = 0; i < P1M * PSM; ++i) s.D[i] = 0.0;
#pragma unroll
    for (int i = 0; i < PSM * P2M; ++i) s.E[i] = 0.0;
#pragma unroll
    for (int i = 0; i < P1M * P2M; ++i) s.F[i] = 0.0;
#pragma unroll
    for (int i = 0; i < P1M; ++i) s.r1[i] = 0.0;
#pragma unroll
    for (int i = 0; i < PSM; ++i) s.rs[i] = 0.0;
#pragma unroll
    for (int i = 0; i < P2M; ++i) s.r2[i] = 0.0;
    auto seg = [&](double *dst, int M, int off, int cnt, int j) {
        for (int a = 0; a < M; ++a) dst[a] = (a < cnt) ? Yk[(off + a) + j * rows] : 0.0;
    };
    if (!ginv || hmode == 2) {
        // stream Y column by column:  YYt += y_j h_j y_jᵀ,  r += y_j h_j g_j
#pragma unroll
        for (int j = 0; j < WM; ++j)
            if (j < w) {
                const double hj = ginv ? hf.f[j] : 1.0, gj = ginv ? gk[j] * hj : 0.0;
                double c1[P1M], cs[PSM], c2[P2M];
#pragma unroll
                for (int a = 0; a < P1M; ++a) c1[a] = (a < p1) ? Yk[a + j * rows] : 0.0;
#pragma unroll
                for (int a = 0; a < PSM; ++a) cs[a] = (a < ps) ? Yk[(p1 + a) + j * rows] : 0.0;
#pragma unroll
                for (int a = 0; a < P2M; ++a) c2[a] = (a < p2) ? Yk[(p1 + ps + a) + j * rows] : 0.0;
                // block sizes are wave-uniform (shared structure): empty blocks are skipped
                // by scalar branches; symmetric blocks accumulate the upper triangle only
                if (p1) sym_acc<P1M>(s.A, c1, hj);
                if (ps) sym_acc<PSM>(s.B, cs, hj);
                if (p2) sym_acc<P2M>(s.C, c2, hj);
                if (p1 && ps) outer_acc<P1M, PSM>(s.D, c1, cs, hj);
                if (ps && p2) outer_acc<PSM, P2M>(s.E, cs, c2, hj);
                if (p1 && p2) outer_acc<P1M, P2M>(s.F, c1, c2, hj);
#pragma unroll
                for (int a = 0; a < P1M; ++a) s.r1[a] += c1[a] * gj;
#pragma unroll
                for (int a = 0; a < PSM; ++a) s.rs[a] += cs[a] * gj;
#pragma unroll
                for (int a = 0; a < P2M; ++a) s.r2[a] += c2[a] * gj;
            }
        sym_mirror<P1M>(s.A);
        sym_mirror<PSM>(s.B);
        sym_mirror<P2M>(s.C);
    } else {
        // dense / block-diagonal H: W = H⁻¹Yᵀ one row of Y at a time, per segment
        double W1[P1M * WM], Ws[PSM * WM], W2[P2M * WM];
        auto hrow = [&](double *Wr, int off, int cnt, int M) {
#pragma unroll
            for (int a = 0; a < M; ++a) {
                double v[WM];
#pragma unroll
                for (int j = 0; j < WM; ++j) v[j] = (a < cnt && j < w) ? Yk[(off + a) + j * rows] : 0.0;
                hinv_apply<WM>(hf, v, w, hmode);
#pragma unroll
                for (int j = 0; j < WM; ++j) Wr[a * WM + j] = v[j];
            }
        };
        hrow(W1, 0, p1, P1M);
        hrow(Ws, p1, ps, PSM);
        hrow(W2, p1 + ps, p2, P2M);
#pragma unroll
        for (int j = 0; j < WM; ++j)
            if (j < w) {
                double c1[P1M], cs[PSM], c2[P2M];
#pragma unroll
                for (int a = 0; a < P1M; ++a) c1[a] = (a < p1) ? Yk[a + j * rows] : 0.0;
#pragma unroll
                for (int a = 0; a < PSM; ++a) cs[a] = (a < ps) ? Yk[(p1 + a) + j * rows] : 0.0;
#pragma unroll
                for (int a = 0; a < P2M; ++a) c2[a] = (a < p2) ? Yk[(p1 + ps + a) + j * rows] : 0.0;
                double w1[P1M], ws[PSM], w2[P2M];
#pragma unroll
                for (int a = 0; a < P1M; ++a) w1[a] = W1[a * WM + j];
#pragma unroll
                for (int a = 0; a < PSM; ++a) ws[a] = Ws[a * WM + j];
#pragma unroll
                for (int a = 0; a < P2M; ++a) w2[a] = W2[a * WM + j];
                outer_acc<P1M, P1M>(s.A, c1, w1, 1.0);
                outer_acc<PSM, PSM>(s.B, cs, ws, 1.0);
                outer_acc<P2M, P2M>(s.C, c2, w2, 1.0);
                outer_acc<P1M, PSM>(s.D, c1, ws, 1.0);
                outer_acc<PSM, P2M>(s.E, cs, w2, 1.0);
                outer_acc<P1M, P2M>(s.F, c1, w2, 1.0);
                const double gj = gk[j];
#pragma unroll
                for (int a = 0; a < P1M; ++a) s.r1[a] += w1[a] * gj;
#pragma unroll
                for (int a = 0; a < PSM; ++a) s.rs[a] += ws[a] * gj;
#pragma unroll
                for (int a = 0; a < P2M; ++a) s.r2[a] += w2[a] * gj;
            }
    }
    (void)seg;
    return ok;
}

// per-knot scratch slab layout (doubles): B ps×ps | C p2×p2 | D p1×ps | E ps×p2 | F p1×p2 | μ | λ
template <int P1M, int PSM, int P2M> struct Slab {
    static constexpr int B = 0, C = B + PSM * PSM, D = C + P2M * P2M, E = D + P1M * PSM,
                         F = E + PSM * P2M, MU = F + P1M * P2M, LAM = MU + PSM,
                         SIZE = LAM + P2M;
};

template <int P1M, int PSM, int P2M, int WM, int RM>
__global__ __launch_bounds__(64) void kkt_lane_kernel(const KktArgs a, double *__restrict__ scratch)
{
    using SL = Slab<P1M, PSM, P2M>;
    constexpr int PM = (P1M > P2M ? P1M : P2M); // λ blocks (p1 of k+1 == p2 of k)
    const int64_t t = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (t >= a.batch) return;
    const int N = a.N, hmode = a.h_mode, ginv = a.ginv;
    const double *Y = a.Y + t * a.sY, *yv = a.y + t * a.sy, *H = a.H + t * a.sH, *g = a.g + t * a.sg;
    double *dz = a.dz + t * a.sg, *lam = a.lam + t * a.sl;
    double *sc = scratch + t * (int64_t)N * SL::SIZE;
    int info = 0;

    // ---------------- forward sweep ----------------
    ShurBlk<P1M, PSM, P2M> cur, nxt;
    KMeta km = kmeta(a.meta, 0);
    if (!compute_shur<P1M, PSM, P2M, WM>(cur, Y + km.oY, H + km.oH, g + km.og, km, hmode, ginv) && !info) info = -1;
    double Ua[PM * PM];      // factor of the previous C block (A ≡ previous C)
    double lprev[PM];        // forward λ of the previous knot
#pragma unroll
    for (int i = 0; i < PM * PM; ++i) Ua[i] = 0.0;
#pragma unroll
    for (int i = 0; i < PM; ++i) lprev[i] = 0.0;

    for (int k = 0; k < N; ++k) {
        const int p1 = km.n1, ps = km.p, p2 = km.n2;
        const int o1 = 0, os = p1, o2 = p1 + ps;
        KMeta kn{};
        if (k + 1 < N) {
            kn = kmeta(a.meta, k + 1);
            if (!compute_shur<P1M, PSM, P2M, WM>(nxt, Y + kn.oY, H + kn.oH, g + kn.og, kn, hmode, ginv) && !info)
                info = -(k + 2);
        }
        // copy_shur!(F[k], block[k], block[k+1])  (:249-286): C gets knot k+1's A-part
        // (A_{k+1} ≡ C_k, jacobian_blocks.jl:166), d gets knot k+1's r_[1] (:251)
        double FB[PSM * PSM], FC[P2M * P2M], FD[P1M * PSM], FE[PSM * P2M], FF[P1M * P2M], c[PSM], d[P2M];
#pragma unroll
        for (int i = 0; i < PSM * PSM; ++i) FB[i] = cur.B[i];
#pragma unroll
        for (int j = 0; j < P2M; ++j)
#pragma unroll
            for (int i = 0; i < P2M; ++i)
                FC[KIDX(i, j, P2M)] = cur.C[KIDX(i, j, P2M)] +
                    ((k + 1 < N && i < P1M && j < P1M) ? nxt.A[KIDX(i < P1M ? i : 0, j < P1M ? j : 0, P1M)] : 0.0);
#pragma unroll
        for (int i = 0; i < P1M * PSM; ++i) FD[i] = cur.D[i];
#pragma unroll
        for (int i = 0; i < PSM * P2M; ++i) FE[i] = cur.E[i];
#pragma unroll
        for (int i = 0; i < P1M * P2M; ++i) FF[i] = cur.F[i];
#pragma unroll
        for (int i = 0; i < PSM; ++i) c[i] = (i < ps) ? cur.rs[i] - yv[km.oy + i] : 0.0;
#pragma unroll
        for (int i = 0; i < P2M; ++i) {
            double v = (i < p2) ? cur.r2[i] - yv[km.oy + ps + i] : 0.0;
            if (k + 1 < N && i < P1M) v += nxt.r1[i < P1M ? i : 0];
            d[i] = v;
        }
        (void)o1; (void)os; (void)o2;

        // cholesky!(U[k], F[k])  (cholesky_solve.jl:47-67)
        if (p1 > 0) {
            trsm_ut<PM, P1M, PSM>(Ua, p1, FD, ps);                             // D = A⁻ᵀ F.D
            trsm_ut<PM, P1M, P2M>(Ua, p1, FF, p2);                             // F = A⁻ᵀ F.F
        }
#pragma unroll
        for (int j = 0; j < PSM; ++j)                                           // B − DᵀD
#pragma unroll
            for (int i = 0; i < PSM; ++i) {
                double s = FB[KIDX(i, j, PSM)];
#pragma unroll
                for (int q = 0; q < P1M; ++q) s -= FD[KIDX(q, i, P1M)] * FD[KIDX(q, j, P1M)];
                FB[KIDX(i, j, PSM)] = s;
            }
        if (ps > 0 && !potrf_u<PSM>(FB, ps) && !info) info = k + 1;
#pragma unroll
        for (int j = 0; j < P2M; ++j)                                           // E − DᵀF
#pragma unroll
            for (int i = 0; i < PSM; ++i) {
                double s = FE[KIDX(i, j, PSM)];
#pragma unroll
                for (int q = 0; q < P1M; ++q) s -= FD[KIDX(q, i, P1M)] * FF[KIDX(q, j, P1M)];
                FE[KIDX(i, j, PSM)] = s;
            }
        if (ps > 0) trsm_ut<PSM, PSM, P2M>(FB, ps, FE, p2);                     // B⁻ᵀ(…)
#pragma unroll
        for (int j = 0; j < P2M; ++j)                                           // C − FᵀF − EᵀE
#pragma unroll
            for (int i = 0; i < P2M; ++i) {
                double s = FC[KIDX(i, j, P2M)];
#pragma unroll
                for (int q = 0; q < P1M; ++q) s -= FF[KIDX(q, i, P1M)] * FF[KIDX(q, j, P1M)];
#pragma unroll
                for (int q = 0; q < PSM; ++q) s -= FE[KIDX(q, i, PSM)] * FE[KIDX(q, j, PSM)];
                FC[KIDX(i, j, P2M)] = s;
            }
        if (p2 > 0 && !potrf_u<P2M>(FC, p2) && !info) info = k + 1;

        // forward_substitution!  (:93-117)
        double mu[PSM], la[P2M];
#pragma unroll
        for (int i = 0; i < PSM; ++i) {
            double s = c[i];
#pragma unroll
            for (int q = 0; q < P1M; ++q)
                if (q < p1) s -= FD[KIDX(q, i, P1M)] * lprev[q];
            mu[i] = s;
        }
        if (ps > 0) trsm_ut<PSM, PSM, 1>(FB, ps, mu, 1);
#pragma unroll
        for (int i = 0; i < P2M; ++i) {
            double s = d[i];
#pragma unroll
            for (int q = 0; q < P1M; ++q)
                if (q < p1) s -= FF[KIDX(q, i, P1M)] * lprev[q];
#pragma unroll
            for (int q = 0; q < PSM; ++q)
                if (q < ps) s -= FE[KIDX(q, i, PSM)] * mu[q];
            la[i] = s;
        }
        if (p2 > 0) trsm_ut<P2M, P2M, 1>(FC, p2, la, 1);

        // spill the factor blocks + forward vectors for the backward sweep
        double *s = sc + (int64_t)k * SL::SIZE;
#pragma unroll
        for (int i = 0; i < PSM * PSM; ++i) s[SL::B + i] = FB[i];
#pragma unroll
        for (int i = 0; i < P2M * P2M; ++i) s[SL::C + i] = FC[i];
#pragma unroll
        for (int i = 0; i < P1M * PSM; ++i) s[SL::D + i] = FD[i];
#pragma unroll
        for (int i = 0; i < PSM * P2M; ++i) s[SL::E + i] = FE[i];
#pragma unroll
        for (int i = 0; i < P1M * P2M; ++i) s[SL::F + i] = FF[i];
#pragma unroll
        for (int i = 0; i < PSM; ++i) s[SL::MU + i] = mu[i];
#pragma unroll
        for (int i = 0; i < P2M; ++i) s[SL::LAM + i] = la[i];

        // next knot: A ≡ this C
#pragma unroll
        for (int j = 0; j < PM; ++j)
#pragma unroll
            for (int i = 0; i < PM; ++i) Ua[KIDX(i, j, PM)] = (i < P2M && j < P2M) ? FC[KIDX(i, j, P2M)] : 0.0;
#pragma unroll
        for (int i = 0; i < PM; ++i) lprev[i] = (i < P2M) ? la[i] : 0.0;
        if (k + 1 < N) {
            cur = nxt;
            km = kn;
        }
    }

    // ---------------- backward sweep + primal recovery ----------------
    double nD[P1M * PSM], nF[P1M * P2M], nmu[PSM], nla[P2M]; // knot k+1 (final μ, λ)
    int nps = 0, np2 = 0;
#pragma unroll
    for (int i = 0; i < P1M * PSM; ++i) nD[i] = 0.0;
#pragma unroll
    for (int i = 0; i < P1M * P2M; ++i) nF[i] = 0.0;
#pragma unroll
    for (int i = 0; i < PSM; ++i) nmu[i] = 0.0;
#pragma unroll
    for (int i = 0; i < P2M; ++i) nla[i] = 0.0;

    for (int k = N - 1; k >= -1; --k) {
        double mu[PSM] = {}, la[P2M] = {};
        KMeta kk{};
        if (k >= 0) {
            kk = kmeta(a.meta, k);
            const int ps = kk.p, p2 = kk.n2;
            const double *s = sc + (int64_t)k * SL::SIZE;
            double FB[PSM * PSM], FC[P2M * P2M], FE[PSM * P2M];
#pragma unroll
            for (int i = 0; i < PSM * PSM; ++i) FB[i] = s[SL::B + i];
#pragma unroll
            for (int i = 0; i < P2M * P2M; ++i) FC[i] = s[SL::C + i];
#pragma unroll
            for (int i = 0; i < PSM * P2M; ++i) FE[i] = s[SL::E + i];
#pragma unroll
            for (int i = 0; i < PSM; ++i) mu[i] = s[SL::MU + i];
#pragma unroll
            for (int i = 0; i < P2M; ++i) la[i] = s[SL::LAM + i];
            if (k < N - 1) {
#pragma unroll
                for (int i = 0; i < P2M; ++i) {                                 // λ += Dμ' + Fλ'
                    double v = la[i];
#pragma unroll
                    for (int q = 0; q < PSM; ++q)
                        if (q < nps) v += nD[KIDX(i, q, P1M)] * nmu[q];
#pragma unroll
                    for (int q = 0; q < P2M; ++q)
                        if (q < np2) v += nF[KIDX(i, q, P1M)] * nla[q];
                    la[i] = v;
                }
                if (p2 > 0) trsv_un<P2M>(FC, p2, la);
#pragma unroll
                for (int i = 0; i < PSM; ++i) {                                 // μ −= E λ
                    double v = mu[i];
#pragma unroll
                    for (int q = 0; q < P2M; ++q)
                        if (q < p2) v -= FE[KIDX(i, q, PSM)] * la[q];
                    mu[i] = v;
                }
                if (ps > 0) trsv_un<PSM>(FB, ps, mu);
#pragma unroll
                for (int i = 0; i < P2M; ++i) la[i] = -la[i];
#pragma unroll
                for (int i = 0; i < PSM; ++i) mu[i] = -mu[i];
            } else {                                                            // terminal
                if (ps > 0) trsv_un<PSM>(FB, ps, mu);
#pragma unroll
                for (int i = 0; i < PSM; ++i) mu[i] = -mu[i];
            }
            // multipliers out: [μ_k; λ_k]  (get_multipliers ordering)
#pragma unroll
            for (int i = 0; i < PSM; ++i)
                if (i < ps) lam[kk.oy + i] = mu[i];
#pragma unroll
            for (int i = 0; i < P2M; ++i)
                if (i < p2) lam[kk.oy + ps + i] = la[i];
        }
        // primal for knot k+1 (all of λ_{k+1}, μ_{k+1}, λ_k are final now)
        if (k + 1 <= N - 1) {
            const int kp = k + 1;
            KMeta m1 = kmeta(a.meta, kp);
            const int rows = m1.n1 + m1.p + m1.n2, w = m1.w;
            const double *Yk = Y + m1.oY;
            double z[WM];
#pragma unroll
            for (int j = 0; j < WM; ++j)
                if (j < w) {
                    double v = 0.0;
#pragma unroll
                    for (int i = 0; i < P2M; ++i)                               // D1ᵀλ_{k+1}
                        if (i < m1.n2) v += Yk[(m1.n1 + m1.p + i) + j * rows] * nla[i];
#pragma unroll
                    for (int i = 0; i < PSM; ++i)                               // Cᵀμ_{k+1}
                        if (i < m1.p) v += Yk[(m1.n1 + i) + j * rows] * nmu[i];
                    if (kp > 0) {
#pragma unroll
                        for (int i = 0; i < P1M; ++i)                           // D2ᵀλ_k
                            if (i < m1.n1) v += Yk[i + j * rows] * la[i];
                    }
                    if (ginv) v += g[m1.og + j];                                 // add_gradient!
                    z[j] = v;
                } else {
                    z[j] = 0.0;
                }
            if (ginv) {
                HFac<WM> hf;
                load_hfac<WM>(hf, H + m1.oH, w, hmode);
                hinv_apply<WM>(hf, z, w, hmode);                                 // :197 ldiv!
            }
#pragma unroll
            for (int j = 0; j < WM; ++j)
                if (j < w) dz[m1.og + j] = -z[j];                               // :198 z .*= -1
        }
        if (k >= 0) {
            // this knot becomes "k+1" for the next (lower) knot
            const double *s = sc + (int64_t)k * SL::SIZE;
#pragma unroll
            for (int i = 0; i < P1M * PSM; ++i) nD[i] = s[SL::D + i];
#pragma unroll
            for (int i = 0; i < P1M * P2M; ++i) nF[i] = s[SL::F + i];
#pragma unroll
            for (int i = 0; i < PSM; ++i) nmu[i] = mu[i];
#pragma unroll
            for (int i = 0; i < P2M; ++i) nla[i] = la[i];
            nps = kk.p;
            np2 = kk.n2;
        }
    }
    if (a.info) a.info[t] = info;
}

// ---------------------------------------------------------------------------------------
// Staged variant: identical arithmetic, but every per-knot input (Y_k, y_k, H_k, g_k of the
// wave's 64 trajectories) is brought into LDS by coalesced LDS-DMA (global_load_lds), one
// knot ahead in a double buffer, and the factor slab is batch-fastest (coalesced).  The
// per-trajectory packed layout keeps each trajectory's knot block contiguous, so the wave
// reads 64 contiguous chunks (dense, lane-linear [t][L] image in LDS).
template <int WM, int RM, int YM> struct StageCfg {
    static constexpr int LY = RM * WM, Ly = YM, LH = WM * WM, Lg = WM;
    static constexpr int SIZE = 64 * (LY + Ly + LH + Lg); // doubles per buffer
};

__device__ __forceinline__ void stage_knot(const KktArgs &a, const KMeta &km, int64_t t0, double *buf,
                                           int LYm, int Lym, int LHm, int lane)
{
    const int rows = km.n1 + km.p + km.n2;
    const int LH = a.h_mode == 2 ? km.w : km.w * km.w;
    dma_group();                                                 // one knot: one DMA group
    stage_chunk(a.Y, a.sY, km.oY, rows * km.w, t0, a.batch, buf, lane);
    stage_chunk(a.y, a.sy, km.oy, km.p + km.n2, t0, a.batch, buf + 64 * LYm, lane);
    stage_chunk(a.H, a.sH, km.oH, LH, t0, a.batch, buf + 64 * (LYm + Lym), lane);
    stage_chunk(a.g, a.sg, km.og, km.w, t0, a.batch, buf + 64 * (LYm + Lym + LHm), lane);
}

// LDS-DMA completion is ordered for ds_read only by vmcnt; and a ds_read still in flight
// when a DMA is issued into its buffer may return the new bytes, so every wait that
// precedes a restage also drains lgkmcnt.
__device__ __forceinline__ void dma_wait()
{
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}
// wait for everything but the N most recent vector-memory ops (the previous knot's slab
// stores, issued after the DMA being waited for: the most recent DMA group, g=1 — checked on
// the compiled instruction stream by tests/isa_vmcnt.py)
template <int NST> __device__ __forceinline__ void dma_wait_but()
{
    static_assert(NST >= 0 && NST < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0) ; lqrx.wait g=1" ::"n"(NST) : "memory");
}

#ifndef LQRX_KKT_DMACHECK
#define LQRX_KKT_DMACHECK 0
#endif
// Debug build only (-DLQRX_KKT_DMACHECK=1): compare a staged knot image against a plain
// global read of the same bytes; a mismatch means a staging/wait bug.  Returns 0 if clean.
__device__ __noinline__ int dma_verify(const KktArgs &a, const KMeta &km, int64_t t, bool live,
                                       const double *Yl, const double *yl, const double *Hl,
                                       const double *gl, int k, int where)
{
    if (!live) return 0;
    const int rows = km.n1 + km.p + km.n2;
    const int LH = a.h_mode == 2 ? km.w : km.w * km.w;
    const double *src[4] = {a.Y + t * a.sY + km.oY, a.y + t * a.sy + km.oy, a.H + t * a.sH + km.oH,
                            a.g + t * a.sg + km.og};
    const double *lds[4] = {Yl, yl, Hl, gl};
    const int L[4] = {rows * km.w, km.p + km.n2, LH, km.w};
    int bad = 0;
    for (int f = 0; f < 4; ++f)
        for (int e = 0; e < L[f]; ++e)
            if (__double_as_longlong(src[f][e]) != __double_as_longlong(lds[f][e])) {
                if (!bad)
                    printf("DMACHECK where=%d knot=%d t=%ld field=%d e=%d lds=%g glob=%g\n", where, k,
                           (long)t, f, e, lds[f][e], src[f][e]);
                bad = 1;
            }
    return bad;
}

template <int P1M, int PSM, int P2M, int WM, int RM>
__global__ __launch_bounds__(64) void kkt_staged_kernel(const KktArgs a, const int32_t *__restrict__ meta,
                                                        double *__restrict__ scratch)
{
    using SL = Slab<P1M, PSM, P2M>;
    constexpr int PM = (P1M > P2M ? P1M : P2M);
    using SC = StageCfg<WM, RM, PSM + P2M>;
    constexpr int LYm = SC::LY, Lym = SC::Ly, LHm = SC::LH;
    __shared__ double stg[2 * SC::SIZE];
    const int lane = threadIdx.x;
    const int64_t t0 = (int64_t)blockIdx.x * 64, t = t0 + lane;
    const bool live = t < a.batch;
    const int N = a.N, hmode = a.h_mode, ginv = a.ginv;
    const int64_t Bp = (a.batch + 63) & ~(int64_t)63;           // slab batch stride
    double *dz = a.dz + t * a.sg, *lam = a.lam + t * a.sl;
    auto slab = [&](int k, int f) -> double & { return scratch[((int64_t)k * SL::SIZE + f) * Bp + t]; };
    auto Yb = [&](int b, const KMeta &km) { return stg + b * SC::SIZE + lane * ((km.n1 + km.p + km.n2) * km.w); };
    auto yb = [&](int b, const KMeta &km) { return stg + b * SC::SIZE + 64 * LYm + lane * (km.p + km.n2); };
    auto Hb = [&](int b, const KMeta &km) {
        return stg + b * SC::SIZE + 64 * (LYm + Lym) + lane * (hmode == 2 ? km.w : km.w * km.w);
    };
    auto gb = [&](int b, const KMeta &km) { return stg + b * SC::SIZE + 64 * (LYm + Lym + LHm) + lane * km.w; };
    int info = 0;

    // ---------------- forward sweep ----------------
    ShurBlk<P1M, PSM, P2M> cur, nxt;
    KMeta km = kmeta(meta, 0);
    double ycur[PSM + P2M];                                     // y_k of the current knot
    stage_knot(a, km, t0, stg, LYm, Lym, LHm, lane);
    dma_wait();
    if (N > 1) stage_knot(a, kmeta(meta, 1), t0, stg + SC::SIZE, LYm, Lym, LHm, lane);
    if (LQRX_KKT_DMACHECK && dma_verify(a, km, t, live, Yb(0, km), yb(0, km), Hb(0, km), gb(0, km), 0, 0))
        info = 9999;
    if (!compute_shur<P1M, PSM, P2M, WM>(cur, Yb(0, km), Hb(0, km), gb(0, km), km, hmode, ginv) && !info)
        info = -1;
    {
        const double *yk = yb(0, km);
#pragma unroll
        for (int i = 0; i < PSM + P2M; ++i) ycur[i] = (i < km.p + km.n2) ? yk[i] : 0.0;
    }
    double Ua[PM * PM], lprev[PM];
#pragma unroll
    for (int i = 0; i < PM * PM; ++i) Ua[i] = 0.0;
#pragma unroll
    for (int i = 0; i < PM; ++i) lprev[i] = 0.0;
    // knot 1 landed (its DMA ran under knot 0's Schur pieces) — here rather than at the loop's
    // k = 0 step, so the loop's hand bound below holds on every compiled path
    dma_wait();

    for (int k = 0; k < N; ++k) {
        const int p1 = km.n1, ps = km.p, p2 = km.n2;
        KMeta kn{};
        double ynxt[PSM + P2M];
        if (k + 1 < N) {
            kn = kmeta(meta, k + 1);
            // knot k+1 has landed (the previous knot's slab stores may still fly) and every
            // ds_read of the buffer about to be restaged has returned (WAR vs the DMA); at k = 0
            // everything already has (the wait before the loop)
            dma_wait_but<SL::SIZE>();
            if (k + 2 < N) stage_knot(a, kmeta(meta, k + 2), t0, stg + (k & 1) * SC::SIZE, LYm, Lym, LHm, lane);
            asm volatile("" ::: "memory");                      // keep the DMAs before the stores
            const int b = (k + 1) & 1;
            if (LQRX_KKT_DMACHECK && dma_verify(a, kn, t, live, Yb(b, kn), yb(b, kn), Hb(b, kn), gb(b, kn), k + 1, 1))
                info = 9999;
            if (!compute_shur<P1M, PSM, P2M, WM>(nxt, Yb(b, kn), Hb(b, kn), gb(b, kn), kn, hmode, ginv) && !info)
                info = -(k + 2);
            const double *yk = yb(b, kn);
#pragma unroll
            for (int i = 0; i < PSM + P2M; ++i) ynxt[i] = (i < kn.p + kn.n2) ? yk[i] : 0.0;
        }
        double FB[PSM * PSM], FC[P2M * P2M], FD[P1M * PSM], FE[PSM * P2M], FF[P1M * P2M], c[PSM], d[P2M];
#pragma unroll
        for (int i = 0; i < PSM * PSM; ++i) FB[i] = cur.B[i];
#pragma unroll
        for (int j = 0; j < P2M; ++j)
#pragma unroll
            for (int i = 0; i < P2M; ++i)
                FC[KIDX(i, j, P2M)] = cur.C[KIDX(i, j, P2M)] +
                    ((k + 1 < N && i < P1M && j < P1M) ? nxt.A[KIDX(i < P1M ? i : 0, j < P1M ? j : 0, P1M)] : 0.0);
#pragma unroll
        for (int i = 0; i < P1M * PSM; ++i) FD[i] = cur.D[i];
#pragma unroll
        for (int i = 0; i < PSM * P2M; ++i) FE[i] = cur.E[i];
#pragma unroll
        for (int i = 0; i < P1M * P2M; ++i) FF[i] = cur.F[i];
#pragma unroll
        for (int i = 0; i < PSM; ++i) c[i] = (i < ps) ? cur.rs[i] - ycur[i] : 0.0;
        // y_d starts at index ps (runtime): select statically
#pragma unroll
        for (int i = 0; i < P2M; ++i) {
            double yd = 0.0;
#pragma unroll
            for (int q = 0; q < PSM + P2M; ++q)
                if (q == ps + i) yd = ycur[q];
            d[i] = (i < p2) ? cur.r2[i] - yd : 0.0;
            if (k + 1 < N && i < P1M) d[i] += nxt.r1[i < P1M ? i : 0];
        }
        // cholesky!(U[k], F[k])
        if (p1 > 0) {
            if (ps) trsm_ut<PM, P1M, PSM>(Ua, p1, FD, ps);
            if (p2) trsm_ut<PM, P1M, P2M>(Ua, p1, FF, p2);
        }
        if (ps) {
#pragma unroll
            for (int j = 0; j < PSM; ++j)
#pragma unroll
                for (int i = 0; i < PSM; ++i) {
                    double s = FB[KIDX(i, j, PSM)];
#pragma unroll
                    for (int q = 0; q < P1M; ++q) s -= FD[KIDX(q, i, P1M)] * FD[KIDX(q, j, P1M)];
                    FB[KIDX(i, j, PSM)] = s;
                }
            if (!potrf_u<PSM>(FB, ps) && !info) info = k + 1;
#pragma unroll
            for (int j = 0; j < P2M; ++j)
#pragma unroll
                for (int i = 0; i < PSM; ++i) {
                    double s = FE[KIDX(i, j, PSM)];
#pragma unroll
                    for (int q = 0; q < P1M; ++q) s -= FD[KIDX(q, i, P1M)] * FF[KIDX(q, j, P1M)];
                    FE[KIDX(i, j, PSM)] = s;
                }
            if (p2) trsm_ut<PSM, PSM, P2M>(FB, ps, FE, p2);
        }
        if (p2) {
#pragma unroll
            for (int j = 0; j < P2M; ++j)
#pragma unroll
                for (int i = 0; i <= j; ++i) {
                    double s = FC[KIDX(i, j, P2M)];
#pragma unroll
                    for (int q = 0; q < P1M; ++q) s -= FF[KIDX(q, i, P1M)] * FF[KIDX(q, j, P1M)];
#pragma unroll
                    for (int q = 0; q < PSM; ++q) s -= FE[KIDX(q, i, PSM)] * FE[KIDX(q, j, PSM)];
                    FC[KIDX(i, j, P2M)] = s;
                }
            if (!potrf_u<P2M>(FC, p2) && !info) info = k + 1;
        }
        // forward_substitution!
        double mu[PSM], la[P2M];
#pragma unroll
        for (int i = 0; i < PSM; ++i) {
            double s = c[i];
#pragma unroll
            for (int q = 0; q < P1M; ++q)
                if (q < p1) s -= FD[KIDX(q, i, P1M)] * lprev[q < PM ? q : 0];
            mu[i] = s;
        }
        if (ps > 0) trsm_ut<PSM, PSM, 1>(FB, ps, mu, 1);
#pragma unroll
        for (int i = 0; i < P2M; ++i) {
            double s = d[i];
#pragma unroll
            for (int q = 0; q < P1M; ++q)
                if (q < p1) s -= FF[KIDX(q, i, P1M)] * lprev[q < PM ? q : 0];
#pragma unroll
            for (int q = 0; q < PSM; ++q)
                if (q < ps) s -= FE[KIDX(q, i, PSM)] * mu[q];
            la[i] = s;
        }
        if (p2 > 0) trsm_ut<P2M, P2M, 1>(FC, p2, la, 1);
        // factor slab (batch-fastest → coalesced)
#pragma unroll
        for (int i = 0; i < PSM * PSM; ++i) slab(k, SL::B + i) = FB[i];
#pragma unroll
        for (int i = 0; i < P2M * P2M; ++i) slab(k, SL::C + i) = FC[i];
#pragma unroll
        for (int i = 0; i < P1M * PSM; ++i) slab(k, SL::D + i) = FD[i];
#pragma unroll
        for (int i = 0; i < PSM * P2M; ++i) slab(k, SL::E + i) = FE[i];
#pragma unroll
        for (int i = 0; i < P1M * P2M; ++i) slab(k, SL::F + i) = FF[i];
#pragma unroll
        for (int i = 0; i < PSM; ++i) slab(k, SL::MU + i) = mu[i];
#pragma unroll
        for (int i = 0; i < P2M; ++i) slab(k, SL::LAM + i) = la[i];
#pragma unroll
        for (int j = 0; j < PM; ++j)
#pragma unroll
            for (int i = 0; i < PM; ++i) Ua[KIDX(i, j, PM)] = (i < P2M && j < P2M) ? FC[KIDX(i < P2M ? i : 0, j < P2M ? j : 0, P2M)] : 0.0;
#pragma unroll
        for (int i = 0; i < PM; ++i) lprev[i] = (i < P2M) ? la[i < P2M ? i : 0] : 0.0;
        if (k + 1 < N) {
            cur = nxt;
            km = kn;
#pragma unroll
            for (int i = 0; i < PSM + P2M; ++i) ycur[i] = ynxt[i];
        }
    }

    // ---------------- backward sweep + primal recovery ----------------
    double nD[P1M * PSM], nF[P1M * P2M], nmu[PSM], nla[P2M];
    int nps = 0, np2 = 0;
#pragma unroll
    for (int i = 0; i < P1M * PSM; ++i) nD[i] = 0.0;
#pragma unroll
    for (int i = 0; i < P1M * P2M; ++i) nF[i] = 0.0;
#pragma unroll
    for (int i = 0; i < PSM; ++i) nmu[i] = 0.0;
#pragma unroll
    for (int i = 0; i < P2M; ++i) nla[i] = 0.0;
    dma_wait();
    __syncthreads();
    stage_knot(a, kmeta(meta, N - 1), t0, stg + ((N - 1) & 1) * SC::SIZE, LYm, Lym, LHm, lane);

    for (int k = N - 1; k >= -1; --k) {
        double mu[PSM] = {}, la[P2M] = {};
        KMeta kk{};
        if (k >= 0) {
            kk = kmeta(meta, k);
            const int ps = kk.p, p2 = kk.n2;
            double FB[PSM * PSM], FC[P2M * P2M], FE[PSM * P2M];
#pragma unroll
            for (int i = 0; i < PSM * PSM; ++i) FB[i] = slab(k, SL::B + i);
#pragma unroll
            for (int i = 0; i < P2M * P2M; ++i) FC[i] = slab(k, SL::C + i);
#pragma unroll
            for (int i = 0; i < PSM * P2M; ++i) FE[i] = slab(k, SL::E + i);
#pragma unroll
            for (int i = 0; i < PSM; ++i) mu[i] = slab(k, SL::MU + i);
#pragma unroll
            for (int i = 0; i < P2M; ++i) la[i] = slab(k, SL::LAM + i);
            if (k < N - 1) {
#pragma unroll
                for (int i = 0; i < P2M; ++i) {
                    double v = la[i];
#pragma unroll
                    for (int q = 0; q < PSM; ++q)
                        if (q < nps) v += nD[KIDX(i < P1M ? i : 0, q, P1M)] * nmu[q];
#pragma unroll
                    for (int q = 0; q < P2M; ++q)
                        if (q < np2) v += nF[KIDX(i < P1M ? i : 0, q, P1M)] * nla[q];
                    la[i] = v;
                }
                if (p2 > 0) trsv_un<P2M>(FC, p2, la);
#pragma unroll
                for (int i = 0; i < PSM; ++i) {
                    double v = mu[i];
#pragma unroll
                    for (int q = 0; q < P2M; ++q)
                        if (q < p2) v -= FE[KIDX(i, q, PSM)] * la[q];
                    mu[i] = v;
                }
                if (ps > 0) trsv_un<PSM>(FB, ps, mu);
#pragma unroll
                for (int i = 0; i < P2M; ++i) la[i] = -la[i];
#pragma unroll
                for (int i = 0; i < PSM; ++i) mu[i] = -mu[i];
            } else {
                if (ps > 0) trsv_un<PSM>(FB, ps, mu);
#pragma unroll
                for (int i = 0; i < PSM; ++i) mu[i] = -mu[i];
            }
            if (live) {
#pragma unroll
                for (int i = 0; i < PSM; ++i)
                    if (i < ps) lam[kk.oy + i] = mu[i];
#pragma unroll
                for (int i = 0; i < P2M; ++i)
                    if (i < p2) lam[kk.oy + ps + i] = la[i];
            }
        }
        if (k + 1 <= N - 1) {
            const int kp = k + 1;
            KMeta m1 = kmeta(meta, kp);
            dma_wait();                                          // knot k+1 landed, reads retired
            if (k >= 0) stage_knot(a, kk, t0, stg + (k & 1) * SC::SIZE, LYm, Lym, LHm, lane);
            const int b = kp & 1;
            const int rows = m1.n1 + m1.p + m1.n2, w = m1.w;
            const double *Yk = Yb(b, m1), *Hk = Hb(b, m1), *gk = gb(b, m1);
            if (LQRX_KKT_DMACHECK && dma_verify(a, m1, t, live, Yk, yb(b, m1), Hk, gk, kp, 2)) info = 9999;
            double z[WM];
#pragma unroll
            for (int j = 0; j < WM; ++j)
                if (j < w) {
                    double v = 0.0;
#pragma unroll
                    for (int i = 0; i < P2M; ++i)
                        if (i < m1.n2) v += Yk[(m1.n1 + m1.p + i) + j * rows] * nla[i];
#pragma unroll
                    for (int i = 0; i < PSM; ++i)
                        if (i < m1.p) v += Yk[(m1.n1 + i) + j * rows] * nmu[i];
                    if (kp > 0) {
#pragma unroll
                        for (int i = 0; i < P1M; ++i)
                            if (i < m1.n1) v += Yk[i + j * rows] * la[i < P2M ? i : 0];
                    }
                    if (ginv) v += gk[j];
                    z[j] = v;
                } else {
                    z[j] = 0.0;
                }
            if (ginv) {
                HFac<WM> hf;
                load_hfac<WM>(hf, Hk, w, hmode);
                hinv_apply<WM>(hf, z, w, hmode);
            }
            if (live) {
#pragma unroll
                for (int j = 0; j < WM; ++j)
                    if (j < w) dz[m1.og + j] = -z[j];
            }
        }
        if (k >= 0) {
#pragma unroll
            for (int i = 0; i < P1M * PSM; ++i) nD[i] = slab(k, SL::D + i);
#pragma unroll
            for (int i = 0; i < P1M * P2M; ++i) nF[i] = slab(k, SL::F + i);
#pragma unroll
            for (int i = 0; i < PSM; ++i) nmu[i] = mu[i];
#pragma unroll
            for (int i = 0; i < P2M; ++i) nla[i] = la[i];
            nps = kk.p;
            np2 = kk.n2;
        }
    }
    dma_wait();
    if (a.info && live) a.info[t] = info;
}

template <int P1M, int PSM, int P2M>
static size_t staged_bytes(const KktArgs &a)
{
    const size_t Bp = ((size_t)a.batch + 63) & ~(size_t)63;      // batch-fastest slab
    return Bp * (size_t)a.N * Slab<P1M, PSM, P2M>::SIZE * sizeof(double);
}
template <int P1M, int PSM, int P2M>
static size_t lane_bytes(const KktArgs &a)
{
    return (size_t)a.batch * (size_t)a.N * Slab<P1M, PSM, P2M>::SIZE * sizeof(double);
}

template <int P1M, int PSM, int P2M, int WM, int RM>
static hipError_t launch_staged(const KktArgs &a, hipStream_t s)
{
    Scratch sc;
    hipError_t e = sc.get(a, staged_bytes<P1M, PSM, P2M>(a), s);
    if (e != hipSuccess) return e;
    dim3 grid((unsigned)((a.batch + 63) / 64)), block(64);
    hipLaunchKernelGGL((kkt_staged_kernel<P1M, PSM, P2M, WM, RM>), grid, block, 0, s, a, a.meta, (double *)sc.p);
    e = hipGetLastError();
    hipError_t ef = sc.release(s);
    return e != hipSuccess ? e : ef;
}

template <int P1M, int PSM, int P2M, int WM, int RM>
static hipError_t launch_lane(const KktArgs &a, hipStream_t s)
{
    Scratch sc;
    hipError_t e = sc.get(a, lane_bytes<P1M, PSM, P2M>(a), s);
    if (e != hipSuccess) return e;
    dim3 grid((unsigned)((a.batch + 63) / 64)), block(64);
    hipLaunchKernelGGL((kkt_lane_kernel<P1M, PSM, P2M, WM, RM>), grid, block, 0, s, a, (double *)sc.p);
    e = hipGetLastError();
    hipError_t ef = sc.release(s);
    return e != hipSuccess ? e : ef;
}

size_t kkt_scratch_bytes(const KktArgs &a)
{
    const int P1 = a.max_p1, PS = a.max_ps, P2 = a.max_p2, W = a.maxw, R = a.maxrows;
    if (!a.force_lane && P1 <= 3 && PS <= 3 && P2 <= 3 && W <= 5 && R <= 6) return staged_bytes<3, 3, 3>(a);
    if (P1 <= 4 && PS <= 4 && P2 <= 4 && W <= 8 && R <= 8) return lane_bytes<4, 4, 4>(a);
    if (P1 <= 8 && PS <= 8 && P2 <= 8 && W <= 12 && R <= 16) return lane_bytes<8, 8, 8>(a);
    return 0;
}

int kkt_generic_class(const KktArgs &a)
{
    const int P1 = a.max_p1, PS = a.max_ps, P2 = a.max_p2, W = a.maxw, R = a.maxrows;
    if (!a.force_lane && P1 <= 3 && PS <= 3 && P2 <= 3 && W <= 5 && R <= 6) return 1;
    if (P1 <= 4 && PS <= 4 && P2 <= 4 && W <= 8 && R <= 8) return 2;
    if (P1 <= 8 && PS <= 8 && P2 <= 8 && W <= 12 && R <= 16) return 3;
    return 0;
}

hipError_t kkt_launch(const KktArgs &a, hipStream_t s)
{
    // block-size maxima from the structure (host copy in a.hmeta)
    const int P1 = a.max_p1, PS = a.max_ps, P2 = a.max_p2, W = a.maxw, R = a.maxrows;
    if (!a.force_lane && P1 <= 3 && PS <= 3 && P2 <= 3 && W <= 5 && R <= 6) return launch_staged<3, 3, 3, 5, 6>(a, s);
    if (P1 <= 4 && PS <= 4 && P2 <= 4 && W <= 8 && R <= 8) return launch_lane<4, 4, 4, 8, 8>(a, s);
    if (P1 <= 8 && PS <= 8 && P2 <= 8 && W <= 12 && R <= 16) return launch_lane<8, 8, 8, 12, 16>(a, s);
    return hipErrorNotSupported;
}

} // namespace lqrx
