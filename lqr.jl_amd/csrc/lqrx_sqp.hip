// lqrx_sqp.hip — batched trajectory-optimisation SQP on the device (SURVEY.md §8(f) ranks 2–3)
// for the reference's test models: the Dubins car (test/dubins_sqp.jl, BASELINE cfg3) and the
// cartpole (test/cartpole.jl, test/problems.jl:58-88).
//
// Around the block-tridiagonal KKT kernel this adds the two steps the reference runs on
// either side of _solve! (cholesky_solver.jl:166-182):
//   before — KKT input assembly (CholeskySolver.update!, cholesky_solver.jl:155-164, which
//            calls TrajOptCore): constraint Jacobian blocks Y_k = [D2; C; D1] from the RK3
//            model dynamics (forward-mode dual numbers through the three RK3 stages, as
//            ForwardDiff differentiates RobotDynamics.discrete_dynamics in the reference),
//            constraint values y_k, the diagonal cost Hessian H_k and gradient g_k of the
//            LQRObjective;
//   after  — the L1-merit backtracking line search with a second-order correction
//            (test/dubins_sqp.jl:58-97; the SOC step −Dᵀ(DDᵀ)⁻¹c(z+dz) is the ginv = 0 KKT
//            variant, second_order_correction!, cholesky_solver.jl:254-273), inside the outer
//            loop of CholeskySolver.solve!/step! (:109-153: ≤ max_iters steps, stop when
//            ‖c‖∞ < tol_p and ‖∇f + ∇cᵀλ‖₂ < tol_d, checked before each step).
// Variables z = [x₁; u₁; …; x_{N-1}; u_{N-1}; x_N] per trajectory (the KKT δz ordering);
// multipliers in the KKT λ ordering ([μ_init; λ₁] | λ_k | μ_goal).
//
// Work split: one wave per trajectory, lanes over knots (k = lane, lane + 64, …) for the
// assembly, the merit evaluations and the residual; wave reductions (fixed butterfly order,
// lane 0's result broadcast) make every accept/reject decision wave-uniform and
// deterministic.
#include "lqrx_internal.h"

#include <cmath>
#include <vector>

#ifndef LQRX_SQP_YSTAGE
#define LQRX_SQP_YSTAGE 1   // stage the expand kernel's Y blocks through LDS (0: direct stores, A/B)
#endif
#ifndef LQRX_SQP_ETPB
#define LQRX_SQP_ETPB 1     // expand kernel: waves (trajectories) per workgroup (A/B: 1 ≥ 2 > 4)
#endif
#ifndef LQRX_SQP_EWAVES
#define LQRX_SQP_EWAVES 1   // expand kernel: minimum waves per SIMD the register allocation targets
#endif

namespace lqrx {
namespace sqp {

constexpr double ETA = 1e-4, RHO = 0.5;   // dubins_sqp.jl:76-77
constexpr int LS_TRIES = 10;              // :78
enum : int32_t { ACTIVE = -1, CONVERGED = 0, LIMIT = 1, LS_FAILED = 2 };

using Args = SqpArgs;

// ---------------------------------------------------------------- forward-mode dual numbers
// value + D directional derivatives (seeded with the unit vectors of [x u]): the dynamics are
// written once, generic in the scalar, and their RK3 Jacobian falls out exactly (to rounding)
template <int D> struct Dual {
    double v, d[D];
};
template <int D> __device__ __forceinline__ Dual<D> operator+(const Dual<D> &a, const Dual<D> &b)
{
    Dual<D> r{a.v + b.v, {}};
    for (int i = 0; i < D; ++i) r.d[i] = a.d[i] + b.d[i];
    return r;
}
template <int D> __device__ __forceinline__ Dual<D> operator-(const Dual<D> &a, const Dual<D> &b)
{
    Dual<D> r{a.v - b.v, {}};
    for (int i = 0; i < D; ++i) r.d[i] = a.d[i] - b.d[i];
    return r;
}
template <int D> __device__ __forceinline__ Dual<D> operator-(const Dual<D> &a)
{
    Dual<D> r{-a.v, {}};
    for (int i = 0; i < D; ++i) r.d[i] = -a.d[i];
    return r;
}
template <int D> __device__ __forceinline__ Dual<D> operator*(const Dual<D> &a, const Dual<D> &b)
{
    Dual<D> r{a.v * b.v, {}};
    for (int i = 0; i < D; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
    return r;
}
template <int D> __device__ __forceinline__ Dual<D> operator*(double a, const Dual<D> &b)
{
    Dual<D> r{a * b.v, {}};
    for (int i = 0; i < D; ++i) r.d[i] = a * b.d[i];
    return r;
}
template <int D> __device__ __forceinline__ Dual<D> operator/(const Dual<D> &a, const Dual<D> &b)
{
    const double q = a.v / b.v;
    Dual<D> r{q, {}};
    for (int i = 0; i < D; ++i) r.d[i] = (a.d[i] - q * b.d[i]) / b.v;
    return r;
}
template <int D> __device__ __forceinline__ void dsincos(const Dual<D> &a, Dual<D> *sn, Dual<D> *cs)
{
    double s, c;
    sincos(a.v, &s, &c);
    sn->v = s;
    cs->v = c;
    for (int i = 0; i < D; ++i) sn->d[i] = c * a.d[i], cs->d[i] = -s * a.d[i];
}
__device__ __forceinline__ void dsincos(double a, double *sn, double *cs) { sincos(a, sn, cs); }
// mixed Dual / double arithmetic the models use
template <int D> __device__ __forceinline__ Dual<D> operator+(const Dual<D> &a, double b)
{
    Dual<D> r = a;
    r.v += b;
    return r;
}
template <int D> __device__ __forceinline__ Dual<D> operator-(double a, const Dual<D> &b) { return -(b + (-a)); }


// ---------------------------------------------------------------- models (continuous dynamics)
// RobotZoo.DubinsCar: ẋ = [v cosθ, v sinθ, ω]
struct Dubins {
    static constexpr int NX = 3, NU = 2;
    template <class T> __device__ static void f(const T *x, const T *u, T *out, const double *)
    {
        T s, c;
        dsincos(x[2], &s, &c);
        out[0] = u[0] * c;
        out[1] = u[0] * s;
        out[2] = u[1];
    }
};
// RobotZoo.Cartpole (test/problems.jl:58-88; SURVEY §8(c) constants mc, mp, l, g in par[0..3]):
// q = [x, θ], q̈ = −H⁻¹(C q̇ + G − B u), H = [mc+mp, mp·l·cθ; mp·l·cθ, mp·l²],
// C q̇ = [−mp·l·sθ·θ̇², 0], G = [0, mp·g·l·sθ], B = [1, 0]
struct Cartpole {
    static constexpr int NX = 4, NU = 1;
    template <class T> __device__ static void f(const T *x, const T *u, T *out, const double *par)
    {
        const double mc = par[0], mp = par[1], l = par[2], g = par[3];
        T s, c;
        dsincos(x[1], &s, &c);
        const T h01 = (mp * l) * c;
        const T r0 = (mp * l) * (s * (x[3] * x[3])) + u[0];      // −(C q̇ + G − B u), row 0
        const T r1 = -((mp * g * l) * s);                       //                    row 1
        const T det = (mc + mp) * (mp * l * l) - h01 * h01;
        out[0] = x[2];
        out[1] = x[3];
        out[2] = ((mp * l * l) * r0 - h01 * r1) / det;
        out[3] = ((mc + mp) * r1 - h01 * r0) / det;
    }
};

// RobotZoo.DoubleIntegrator(D) (test/problems.jl:14-56): x = [q; q̇] ∈ R^{2D}, ẋ = [q̇; u]
template <int D> struct DoubleIntegrator {
    static constexpr int NX = 2 * D, NU = D;
    template <class T> __device__ static void f(const T *x, const T *u, T *out, const double *)
    {
        for (int i = 0; i < D; ++i) out[i] = x[D + i], out[D + i] = u[i];
    }
};

// a model + the number of rows PK of the linear stage constraint A_s·x_k = b_s on the interior
// knots 1..N−2 (the LinearConstraint DoubleIntegrator() adds on 2:N−1, problems.jl:40-44;
// 0 = none).  A_s (PK × NX, column-major) and b_s are shared by the batch.
template <class Dyn, int PK_> struct Prob : Dyn {
    static constexpr int PK = PK_;
};

// RobotDynamics RK3: k1 = f(x)dt, k2 = f(x + k1/2)dt, k3 = f(x − k1 + 2k2)dt,
// x⁺ = x + (k1 + 4k2 + k3)/6 — generic in the scalar type
template <class M, class T>
__device__ __forceinline__ void rk3_t(const T *x, const T *u, double dt, T *xn, const double *par)
{
    constexpr int NX = M::NX;
    T k1[NX], k2[NX], k3[NX], t[NX];
    M::f(x, u, k1, par);
    for (int i = 0; i < NX; ++i) k1[i] = dt * k1[i], t[i] = x[i] + 0.5 * k1[i];
    M::f(t, u, k2, par);
    for (int i = 0; i < NX; ++i) k2[i] = dt * k2[i], t[i] = (x[i] - k1[i]) + 2.0 * k2[i];
    M::f(t, u, k3, par);
    for (int i = 0; i < NX; ++i) k3[i] = dt * k3[i], xn[i] = x[i] + (1.0 / 6.0) * ((k1[i] + 4.0 * k2[i]) + k3[i]);
}
template <class M> __device__ __forceinline__ void rk3(const double *x, const double *u, double dt, double *xn, const double *par)
{
    rk3_t<M, double>(x, u, dt, xn, par);
}
// the same with J = ∂x⁺/∂[x u] (NX × (NX+NU)) by forward-mode duals
template <class M>
__device__ __forceinline__ void rk3_jac(const double *x, const double *u, double dt, double *xn, double (*J)[M::NX + M::NU],
                                        const double *par)
{
    constexpr int NX = M::NX, NU = M::NU, W = NX + NU;
    Dual<W> xd[NX], ud[NU], xo[NX];
    for (int i = 0; i < NX; ++i) {
        xd[i].v = x[i];
        for (int j = 0; j < W; ++j) xd[i].d[j] = (i == j) ? 1.0 : 0.0;
    }
    for (int i = 0; i < NU; ++i) {
        ud[i].v = u[i];
        for (int j = 0; j < W; ++j) ud[i].d[j] = (NX + i == j) ? 1.0 : 0.0;
    }
    rk3_t<M, Dual<W>>(xd, ud, dt, xo, par);
    for (int i = 0; i < NX; ++i) {
        xn[i] = xo[i].v;
        for (int j = 0; j < W; ++j) J[i][j] = xo[i].d[j];
    }
}

template <class M> struct Dims {
    static constexpr int NX = M::NX, NU = M::NU, W = NX + NU, PK = M::PK;
    // KKT block rows of knot k: first [C = initial state; D1], interior [D2; C = stage; D1],
    // last [D2; C = goal]
    __host__ __device__ static constexpr int rows(int k, int N) { return k == 0 || k == N - 1 ? 2 * NX : 2 * NX + PK; }
    __host__ __device__ static constexpr int64_t nn(int N) { return (int64_t)N * NX + (int64_t)(N - 1) * NU; }
    // multipliers = constraint rows: init NX, per interior knot PK + NX, dynamics 0 NX, goal NX
    __host__ __device__ static constexpr int64_t np_(int N) { return (int64_t)(N + 1) * NX + (int64_t)(N - 2) * PK; }
    __host__ __device__ static constexpr int64_t ny_(int N)
    {
        return 2 * NX * W + (int64_t)(N - 2) * (2 * NX + PK) * W + 2 * NX * NX;
    }
    __device__ static int64_t oY(int k) { return k == 0 ? 0 : 2 * NX * W + (int64_t)(k - 1) * (2 * NX + PK) * W; }
    __device__ static int64_t oy(int k) { return k == 0 ? 0 : 2 * NX + (int64_t)(k - 1) * (PK + NX); }   // y / λ blocks
    __device__ static int64_t om(int k) { return k == 0 ? 0 : oy(k) - NX; }        // [λ_{k-1}; μ_k; λ_k]
};

// the stage constraint values A_s·x − b_s (PK rows)
template <class M> __device__ __forceinline__ void stage_con(const Args &A, const double *x, double *c)
{
    for (int r = 0; r < M::PK; ++r) {
        double v = -A.Sb[r];
        for (int j = 0; j < M::NX; ++j) v += A.SA[r + M::PK * j] * x[j];
        c[r] = v;
    }
}

// merit pieces of knot k at the point zk (+ a·dk + b·ek): cost and Σ|c| of the constraint
// values the knot owns (knot 0: initial state + dynamics 0; knot k: dynamics k; last: goal)
struct KnotPt {
    const double *z, *d, *e;   // z, dz, SOC step (e may be null)
    double a, b;
    __device__ double at(int64_t i) const
    {
        double v = z[i];
        if (d) v += a * d[i];
        if (e) v += b * e[i];
        return v;
    }
};

template <class M>
__device__ __forceinline__ void knot_merit(const Args &A, int t, int k, const KnotPt &p, double &cost, double &c1)
{
    constexpr int NX = M::NX, NU = M::NU, W = NX + NU;
    const int N = A.N;
    const int64_t o = (int64_t)W * k;
    double x[NX], u[NU];
    for (int i = 0; i < NX; ++i) x[i] = p.at(o + i);
    const double *xf = A.xf + (int64_t)t * NX;
    cost = 0.0;
    c1 = 0.0;
    if (k < N - 1) {
        for (int i = 0; i < NU; ++i) u[i] = p.at(o + NX + i);
        for (int i = 0; i < NX; ++i) cost += 0.5 * (x[i] - xf[i]) * A.Q[i] * (x[i] - xf[i]);
        for (int i = 0; i < NU; ++i) cost += 0.5 * u[i] * A.R[i] * u[i];
        double xn[NX];
        rk3<M>(x, u, A.dt, xn, A.par);
        if (k == 0)
            for (int i = 0; i < NX; ++i) c1 += fabs(x[i] - A.x0[(int64_t)t * NX + i]);
        if constexpr (M::PK > 0)
            if (k > 0) {
                double cs[M::PK > 0 ? M::PK : 1];
                stage_con<M>(A, x, cs);
                for (int r = 0; r < M::PK; ++r) c1 += fabs(cs[r]);
            }
        for (int i = 0; i < NX; ++i) c1 += fabs(xn[i] - p.at(o + W + i));
    } else {
        for (int i = 0; i < NX; ++i) cost += 0.5 * (x[i] - xf[i]) * A.Qf[i] * (x[i] - xf[i]);
        for (int i = 0; i < NX; ++i) c1 += fabs(x[i] - xf[i]);
    }
}

// ---------------------------------------------------------------- wave-per-trajectory helpers
// One wave per trajectory: lane l takes knots l, l+64, …; per-knot sums are reduced across
// the wave and lane 0's value is broadcast, so every decision is wave-uniform.
constexpr int TPB = 4;                                    // trajectories (waves) per workgroup

__device__ __forceinline__ double wave_sum(double v)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return __shfl(v, 0, 64);
}
__device__ __forceinline__ double wave_max(double v)
{
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return __shfl(v, 0, 64);
}

// ϕ = f + μ‖c‖₁ at the point p (dubins_sqp.jl:60)
template <class M> __device__ double merit(const Args &A, int t, const KnotPt &p, int lane)
{
    double f = 0.0, c = 0.0;
    for (int k = lane; k < A.N; k += 64) {
        double ck, c1;
        knot_merit<M>(A, t, k, p, ck, c1);
        f += ck;
        c += c1;
    }
    return wave_sum(f) + A.mu * wave_sum(c);
}

// z ← p, λ ← λ of the Newton solve, one more accepted step (wave-cooperative, coalesced)
template <class M> __device__ void accept(const Args &A, int64_t t, const KnotPt &p, int lane)
{
    const int64_t NN = Dims<M>::nn(A.N), P = Dims<M>::np_(A.N);
    double *z = A.Z + t * NN;
    for (int64_t i = lane; i < NN; i += 64) z[i] = p.at(i);
    for (int64_t i = lane; i < P; i += 64) A.lam[t * P + i] = A.lamn[t * P + i];
    if (lane == 0) A.iters[t] += 1;
}

// ---------------------------------------------------------------- assembly (update!) + check
// Knot k: Y_k, y_k, H_k, g_k of the trajectory structure (knot 0: (n1 0, p NX, n2 NX, w W),
// interior (NX, 0, NX, W), last (NX, NX, 0, NX)) and its share of the convergence check: cost,
// Σ|c|, max|c|, ‖g_k + Y_kᵀ m_k‖² with m_k = [λ_{k-1}; μ_k; λ_k] the multipliers of the
// last Newton step (calc_residual!, cholesky_solver.jl:201-236).  Then the wave's check:
// ‖c‖∞ < tol_p and ‖∇f + ∇cᵀλ‖₂ < tol_d → converged (cholesky_solver.jl:129-137).
// Y_k goes to `Y` (the wave's LDS image of its 64 knots' blocks when staged, else HBM)
template <class M>
__device__ __forceinline__ void expand_knot(const Args &A, int t, int k, double *Y, double &cost, double &c1,
                                            double &cinf, double &r2)
{
    using D = Dims<M>;
    constexpr int NX = M::NX, NU = M::NU, W = NX + NU, PK = M::PK, RM = 2 * NX + PK;
    const int N = A.N;
    const int64_t NN = D::nn(N), P = D::np_(N);
    const double *z = A.Z + t * NN + (int64_t)W * k;
    const double *xf = A.xf + (int64_t)t * NX;
    double *y = A.y + t * P + D::oy(k);
    double *H = A.H + t * NN + (int64_t)W * k;
    double *g = A.g + t * NN + (int64_t)W * k;
    const double *m = A.lam + t * P + D::om(k);
    double x[NX];
    for (int i = 0; i < NX; ++i) x[i] = z[i];
    auto con = [&](double v, int i) {
        y[i] = v;
        c1 += fabs(v);
        cinf = fmax(cinf, fabs(v));
    };
    if (k < N - 1) {
        double u[NU];
        for (int i = 0; i < NU; ++i) u[i] = z[NX + i];
        double xn[NX], J[NX][W];
        rk3_jac<M>(x, u, A.dt, xn, J, A.par);
        // rows: k == 0: [C = [I 0] (initial state); D1 = J]                   (2NX rows)
        //       else    [D2 = [−I 0]; C = [A_s 0] (stage, PK rows); D1 = J]   (2NX + PK rows)
        const bool first = (k == 0);
        const int R = first ? 2 * NX : RM, o1 = first ? NX : NX + PK;   // o1: first row of D1
        for (int j = 0; j < W; ++j) {
            double *Yj = Y + (int64_t)R * j;
            for (int i = 0; i < NX; ++i) Yj[i] = (i == j) ? (first ? 1.0 : -1.0) : 0.0;
            if constexpr (PK > 0)
                if (!first)
                    for (int q = 0; q < PK; ++q) Yj[NX + q] = j < NX ? A.SA[q + PK * j] : 0.0;
            for (int i = 0; i < NX; ++i) Yj[o1 + i] = J[i][j];
        }
        int r = 0;
        if (k == 0)
            for (int i = 0; i < NX; ++i) con(x[i] - A.x0[(int64_t)t * NX + i], r++);
        if constexpr (PK > 0)
            if (k > 0) {
                double cs[PK > 0 ? PK : 1];
                stage_con<M>(A, x, cs);
                for (int q = 0; q < PK; ++q) con(cs[q], r++);
            }
        for (int i = 0; i < NX; ++i) con(xn[i] - z[W + i], r++);
        double gk[W];
        for (int i = 0; i < NX; ++i) {
            const double e = x[i] - xf[i];
            gk[i] = A.Q[i] * e;
            H[i] = A.Q[i];
            cost += 0.5 * (x[i] - xf[i]) * A.Q[i] * (x[i] - xf[i]);
        }
        for (int i = 0; i < NU; ++i) {
            gk[NX + i] = A.R[i] * u[i];
            H[NX + i] = A.R[i];
            cost += 0.5 * u[i] * A.R[i] * u[i];
        }
        // ∇f + ∇cᵀλ restricted to z_k: g_k + Y_kᵀ m_k, from the block structure
        for (int j = 0; j < W; ++j) {
            g[j] = gk[j];
            double sres = gk[j];
            if (j < NX) sres += first ? m[j] : -m[j];
            if constexpr (PK > 0)
                if (!first && j < NX)
                    for (int q = 0; q < PK; ++q) sres += A.SA[q + PK * j] * m[NX + q];
            for (int i = 0; i < NX; ++i) sres += J[i][j] * m[o1 + i];
            r2 += sres * sres;
        }
    } else {
        // last knot: [D2 = −I; C = I (goal)], 2NX × NX
        for (int j = 0; j < NX; ++j)
            for (int i = 0; i < NX; ++i) {
                Y[i + 2 * NX * j] = (i == j) ? -1.0 : 0.0;
                Y[NX + i + 2 * NX * j] = (i == j) ? 1.0 : 0.0;
            }
        for (int i = 0; i < NX; ++i) con(x[i] - xf[i], i);
        for (int i = 0; i < NX; ++i) {
            const double e = x[i] - xf[i];
            g[i] = A.Qf[i] * e;
            H[i] = A.Qf[i];
            cost += 0.5 * (x[i] - xf[i]) * A.Qf[i] * (x[i] - xf[i]);
            const double sres = g[i] - m[i] + m[NX + i];
            r2 += sres * sres;
        }
    }
}

// The 64 knots a wave expands at once own one contiguous run of Y (consecutive knot blocks,
// Dims::oY).  Written lane-per-knot, every store instruction touches 64 blocks RM·W·8 bytes
// apart; staged, the blocks are built in the wave's LDS image and the run is copied out in
// 512-B rows.  Staged when the image fits 20 KB per wave.
template <class M> constexpr int yimg_doubles() { return 64 * (2 * M::NX + M::PK) * (M::NX + M::NU); }
template <class M> constexpr bool y_staged() { return LQRX_SQP_YSTAGE && yimg_doubles<M>() * 8 <= 20480; }
constexpr int ETPB = LQRX_SQP_ETPB;                       // trajectories (waves) per expand workgroup

__device__ inline void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <class M> __global__ __launch_bounds__(64 * ETPB, LQRX_SQP_EWAVES) void sqp_expand_kernel(const Args A)
{
    using D = Dims<M>;
    constexpr bool ST = y_staged<M>();
    __shared__ double yimg[ST ? ETPB * yimg_doubles<M>() : 1];
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * ETPB + (threadIdx.x >> 6);
    if (t >= A.B || A.status[t] != ACTIVE) return;                 // wave-uniform
    double cost = 0.0, c1 = 0.0, cinf = 0.0, r2 = 0.0;
    const int N = A.N;
    double *Yt = A.Y + t * D::ny_(N);
    double *yw = yimg + (ST ? (threadIdx.x >> 6) * yimg_doubles<M>() : 0);
    for (int kb = 0; kb < N; kb += 64) {
        const int k = kb + lane;
        const int64_t e0 = D::oY(kb);
        if (k < N) expand_knot<M>(A, (int)t, k, ST ? yw + (D::oY(k) - e0) : Yt + D::oY(k), cost, c1, cinf, r2);
        if constexpr (ST) {
            const int64_t e1 = kb + 64 < N ? D::oY(kb + 64) : D::ny_(N);
            wave_sync();
            for (int64_t i = lane; i < e1 - e0; i += 64) Yt[e0 + i] = yw[i];
            wave_sync();
        }
    }
    const double f = wave_sum(cost), cs = wave_sum(c1), cm = wave_max(cinf), rs = wave_sum(r2);
    if (lane != 0) return;
    if (cm < A.tol_p && sqrt(rs) < A.tol_d) {
        A.status[t] = CONVERGED;
        return;
    }
    A.phi0[t] = f + A.mu * cs;
    A.dphi[t] = -A.mu * cs;          // + ∇fᵀdz once the step is known (sqp_ls1_kernel)
    atomicAdd(A.n_active, 1);
}

// ---------------------------------------------------------------- line search, full step
// ϕ′ = ∇fᵀdz − μ‖c‖₁ (dubins_sqp.jl:61); Armijo at α = 1 (:79); otherwise the constraint
// values at z + dz go to y for the second-order-correction solve.
template <class M> __global__ __launch_bounds__(64 * TPB) void sqp_ls1_kernel(const Args A)
{
    using D = Dims<M>;
    constexpr int NX = M::NX, NU = M::NU, W = NX + NU;
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * TPB + (threadIdx.x >> 6);
    if (t >= A.B) return;
    if (lane == 0) A.need_soc[t] = 0;
    if (A.status[t] != ACTIVE) return;
    const int N = A.N;
    const int64_t NN = D::nn(N), P = D::np_(N);
    const double *z = A.Z + t * NN, *dz = A.dz + t * NN, *g = A.g + t * NN;
    double gd = 0.0;
    for (int64_t i = lane; i < NN; i += 64) gd += g[i] * dz[i];
    const double dphi = wave_sum(gd) + A.dphi[t];
    const KnotPt p1{z, dz, nullptr, 1.0, 0.0};
    const double phi1 = merit<M>(A, (int)t, p1, lane);
    if (lane == 0) A.dphi[t] = dphi;
    if (phi1 <= A.phi0[t] + ETA * dphi) {
        accept<M>(A, t, p1, lane);
        return;
    }
    if (lane == 0) A.need_soc[t] = 1;
    double *y = A.y + t * P;
    for (int k = lane; k < N; k += 64) {
        const int64_t o = (int64_t)W * k;
        double x[NX];
        for (int i = 0; i < NX; ++i) x[i] = p1.at(o + i);
        double *yk = y + D::oy(k);
        if (k < N - 1) {
            double u[NU];
            for (int i = 0; i < NU; ++i) u[i] = p1.at(o + NX + i);
            double xn[NX];
            rk3<M>(x, u, A.dt, xn, A.par);
            int r = 0;
            if (k == 0)
                for (int i = 0; i < NX; ++i) yk[r++] = x[i] - A.x0[t * NX + i];
            if constexpr (M::PK > 0)
                if (k > 0) {
                    stage_con<M>(A, x, yk);
                    r += M::PK;
                }
            for (int i = 0; i < NX; ++i) yk[r++] = xn[i] - p1.at(o + W + i);
        } else {
            for (int i = 0; i < NX; ++i) yk[i] = x[i] - A.xf[t * NX + i];
        }
    }
}

// ---------------------------------------------------------------- line search, SOC + backtracking
// dubins_sqp.jl:82-94: z + dz + dẑ accepted on strict decrease below ϕ + ηϕ′; else α = ρ, ρ², …
template <class M> __global__ __launch_bounds__(64 * TPB) void sqp_ls2_kernel(const Args A)
{
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * TPB + (threadIdx.x >> 6);
    if (t >= A.B || !A.need_soc[t]) return;
    const int64_t NN = Dims<M>::nn(A.N);
    const double *z = A.Z + t * NN, *dz = A.dz + t * NN, *ds = A.dzs + t * NN;
    const double phi0 = A.phi0[t], dphi = A.dphi[t];
    const KnotPt ps{z, dz, ds, 1.0, 1.0};
    if (merit<M>(A, (int)t, ps, lane) < phi0 + ETA * dphi) {
        accept<M>(A, t, ps, lane);
        return;
    }
    double a = RHO;
    for (int i = 1; i < LS_TRIES; ++i, a *= RHO) {
        const KnotPt pa{z, dz, nullptr, a, 0.0};
        if (merit<M>(A, (int)t, pa, lane) <= phi0 + ETA * a * dphi) {
            accept<M>(A, t, pa, lane);
            return;
        }
    }
    if (lane == 0) A.status[t] = LS_FAILED;
}

__global__ __launch_bounds__(256) void sqp_init_kernel(const Args A, int64_t P)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < A.B * P) A.lam[i] = 0.0;
    if (i < A.B) {
        A.status[i] = ACTIVE;
        A.iters[i] = 0;
    }
}

// sel ← the trajectories with gate[t] == val (any order: every trajectory's KKT solve is
// independent of which wave runs it), *nsel ← their count; one atomic per wave
__global__ __launch_bounds__(256) void sqp_select_kernel(const int32_t *gate, int32_t val, int64_t B, int32_t *sel,
                                                         int32_t *nsel)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool on = t < B && gate[t] == val;
    const uint64_t m = __ballot(on);
    const int lane = threadIdx.x & 63;
    int32_t base = 0;
    if (lane == 0 && m) base = atomicAdd(nsel, (int32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (on) sel[base + (int32_t)__popcll(m & ((1ull << lane) - 1))] = (int32_t)t;
}

__global__ __launch_bounds__(256) void sqp_finish_kernel(const Args A)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < A.B && A.status[t] == ACTIVE) A.status[t] = LIMIT;
}

static dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

using KktFn = int (*)(void *ctx, int ginv, double *dz, const int32_t *sel, const int32_t *nsel);

// sel ← {t : gate[t] == val}
static hipError_t select(const SqpArgs &A, const int32_t *gate, int32_t val, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(A.nsel, 0, sizeof(int32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sqp_select_kernel, grid_for(A.B), dim3(256), 0, s, gate, val, A.B, A.sel, A.nsel);
    return hipGetLastError();
}

template <class M>
hipError_t run(const SqpArgs &A, int max_iters, hipStream_t s, KktFn kkt, void *ctx, int *kkt_rc)
{
    const int64_t BP = A.B * Dims<M>::np_(A.N);
    hipLaunchKernelGGL(sqp_init_kernel, grid_for(BP > A.B ? BP : A.B), dim3(256), 0, s, A, Dims<M>::np_(A.N));
    int32_t h_active = 0;
    for (int it = 0; it < max_iters; ++it) {
        hipError_t e = hipMemsetAsync(A.n_active, 0, sizeof(int32_t), s);
        if (e != hipSuccess) return e;
        const dim3 ge((unsigned)((A.B + ETPB - 1) / ETPB)), be(64 * ETPB);
        const dim3 gw((unsigned)((A.B + TPB - 1) / TPB)), bw(64 * TPB);
        hipLaunchKernelGGL(sqp_expand_kernel<M>, ge, be, 0, s, A);
        if ((e = hipMemcpyAsync(&h_active, A.n_active, sizeof(int32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return e;
        if (h_active == 0) break;
        // Newton step for the still-active trajectories, SOC for those whose full step failed
        // the Armijo test (usually a few): the KKT kernel runs the selected subset only
        if ((e = select(A, A.status, ACTIVE, s)) != hipSuccess) return e;
        if ((*kkt_rc = kkt(ctx, 1, A.dz, A.sel, A.nsel)) < 0) return hipSuccess;
        hipLaunchKernelGGL(sqp_ls1_kernel<M>, gw, bw, 0, s, A);
        if ((e = select(A, A.need_soc, 1, s)) != hipSuccess) return e;
        if ((*kkt_rc = kkt(ctx, 0, A.dzs, A.sel, A.nsel)) < 0) return hipSuccess;
        hipLaunchKernelGGL(sqp_ls2_kernel<M>, gw, bw, 0, s, A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(sqp_finish_kernel, grid_for(A.B), dim3(256), 0, s, A);
    return hipGetLastError();
}

} // namespace sqp

bool sqp_model_dims(int model, int *nx, int *nu)
{
    switch (model) {
    case SQP_DUBINS: *nx = sqp::Dubins::NX, *nu = sqp::Dubins::NU; return true;
    case SQP_CARTPOLE: *nx = sqp::Cartpole::NX, *nu = sqp::Cartpole::NU; return true;
    case SQP_DI1: *nx = 2, *nu = 1; return true;
    case SQP_DI2: *nx = 4, *nu = 2; return true;
    case SQP_DI3: *nx = 6, *nu = 3; return true;
    default: return false;
    }
}

// the structure tables of the trajectory KKT (ConstraintBlocks, conblocks.jl:403-425):
// knot 0 (0, NX, NX, NX+NU), interior (NX, PK, NX, NX+NU), last (NX, NX, 0, NX)
void sqp_structure(int nx, int nu, int pk, int N, std::vector<int32_t> &n1, std::vector<int32_t> &p,
                   std::vector<int32_t> &n2, std::vector<int32_t> &w)
{
    n1.assign(N, nx);
    p.assign(N, pk);
    n2.assign(N, nx);
    w.assign(N, nx + nu);
    n1[0] = 0;
    p[0] = nx;
    p[N - 1] = nx;
    n2[N - 1] = 0;
    w[N - 1] = nx;
}

namespace {
template <class Dyn>
hipError_t run_pk(const SqpArgs &A, int max_iters, hipStream_t s, sqp::KktFn kkt, void *ctx, int *kkt_rc)
{
    switch (A.stage_rows) {
    case 0: return sqp::run<sqp::Prob<Dyn, 0>>(A, max_iters, s, kkt, ctx, kkt_rc);
    case 1: return sqp::run<sqp::Prob<Dyn, 1>>(A, max_iters, s, kkt, ctx, kkt_rc);
    case 2: return sqp::run<sqp::Prob<Dyn, 2>>(A, max_iters, s, kkt, ctx, kkt_rc);
    default: return hipErrorInvalidValue;
    }
}
} // namespace

// Device driver (lqrx_api.cpp validates and calls this).  kkt(ctx, ginv, dz) runs one KKT
// solve of the trajectory structure on Y, y, H, g → dz, lamn; a negative return stops the loop.
hipError_t sqp_run(const SqpArgs &A, int max_iters, hipStream_t s, sqp::KktFn kkt, void *ctx, int *kkt_rc)
{
    switch (A.model) {
    case SQP_DUBINS: return run_pk<sqp::Dubins>(A, max_iters, s, kkt, ctx, kkt_rc);
    case SQP_CARTPOLE: return run_pk<sqp::Cartpole>(A, max_iters, s, kkt, ctx, kkt_rc);
    case SQP_DI1: return run_pk<sqp::DoubleIntegrator<1>>(A, max_iters, s, kkt, ctx, kkt_rc);
    case SQP_DI2: return run_pk<sqp::DoubleIntegrator<2>>(A, max_iters, s, kkt, ctx, kkt_rc);
    case SQP_DI3: return run_pk<sqp::DoubleIntegrator<3>>(A, max_iters, s, kkt, ctx, kkt_rc);
    default: return hipErrorInvalidValue;
    }
}

} // namespace lqrx
