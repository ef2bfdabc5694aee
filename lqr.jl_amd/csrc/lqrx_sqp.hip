// lqrx_sqp.hip — batched Dubins-car SQP on the device (SURVEY.md §8(f) ranks 2–3).
//
// Around the block-tridiagonal KKT kernel this adds the two steps the reference runs on
// either side of _solve! (cholesky_solver.jl:166-182):
//   before — KKT input assembly (CholeskySolver.update!, cholesky_solver.jl:155-164, which
//            calls TrajOptCore): constraint Jacobian blocks Y_k = [D2; C; D1] from the RK3
//            Dubins dynamics (analytic chain rule), constraint values y_k, the diagonal cost
//            Hessian H_k and gradient g_k of the LQRObjective;
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

namespace lqrx {
namespace sqp {

constexpr int NX = 3, NU = 2, W = NX + NU;
constexpr double ETA = 1e-4, RHO = 0.5;   // dubins_sqp.jl:76-77
constexpr int LS_TRIES = 10;              // :78
enum : int32_t { ACTIVE = -1, CONVERGED = 0, LIMIT = 1, LS_FAILED = 2 };

using Args = SqpArgs;

__host__ __device__ constexpr int64_t nn(int N) { return (int64_t)N * NX + (int64_t)(N - 1) * NU; }
__host__ __device__ constexpr int64_t np_(int N) { return (int64_t)(N + 1) * NX; }
__host__ __device__ constexpr int64_t ny_(int N) { return 30 * (int64_t)(N - 1) + 18; }
__device__ __forceinline__ int64_t oy(int k) { return k == 0 ? 0 : 3 * (int64_t)k + 3; }   // y / λ blocks
__device__ __forceinline__ int64_t om(int k) { return k == 0 ? 0 : 3 * (int64_t)k; }       // [λ_{k-1}; μ_k; λ_k]

// RobotZoo.DubinsCar: ẋ = [v cosθ, v sinθ, ω]
__device__ __forceinline__ void dubins(const double x[NX], const double u[NU], double f[NX])
{
    double s, c;
    sincos(x[2], &s, &c);
    f[0] = u[0] * c;
    f[1] = u[0] * s;
    f[2] = u[1];
}

// RobotDynamics RK3: k1 = f(x)dt, k2 = f(x + k1/2)dt, k3 = f(x − k1 + 2k2)dt,
// x⁺ = x + (k1 + 4k2 + k3)/6
__device__ __forceinline__ void rk3(const double x[NX], const double u[NU], double dt, double xn[NX])
{
    double k1[NX], k2[NX], k3[NX], t[NX];
    dubins(x, u, k1);
    for (int i = 0; i < NX; ++i) k1[i] *= dt, t[i] = x[i] + 0.5 * k1[i];
    dubins(t, u, k2);
    for (int i = 0; i < NX; ++i) k2[i] *= dt, t[i] = x[i] - k1[i] + 2.0 * k2[i];
    dubins(t, u, k3);
    for (int i = 0; i < NX; ++i) k3[i] *= dt, xn[i] = x[i] + (k1[i] + 4.0 * k2[i] + k3[i]) / 6.0;
}

// the same with J = ∂x⁺/∂[x u] (3×5) by the chain rule through the three stages.  The only
// state dependence of f is through θ: ∂f/∂x = e_θᵀ ⊗ [−v sinθ, v cosθ, 0]ᵀ.
__device__ __forceinline__ void rk3_jac(const double x[NX], const double u[NU], double dt, double xn[NX],
                                        double J[NX][W])
{
    double k[3][NX], Jk[3][NX][W], t[NX], Jt[NX][W];
    for (int st = 0; st < 3; ++st) {
        // stage input t = x (+ combination of previous stages) and its Jacobian Jt
        for (int i = 0; i < NX; ++i) {
            double v = x[i];
            if (st == 1) v += 0.5 * k[0][i];
            if (st == 2) v += -k[0][i] + 2.0 * k[1][i];
            t[i] = v;
            for (int j = 0; j < W; ++j) {
                double a = (i == j) ? 1.0 : 0.0;
                if (st == 1) a += 0.5 * Jk[0][i][j];
                if (st == 2) a += -Jk[0][i][j] + 2.0 * Jk[1][i][j];
                Jt[i][j] = a;
            }
        }
        double s, c;
        sincos(t[2], &s, &c);
        const double v = u[0];
        k[st][0] = dt * v * c;
        k[st][1] = dt * v * s;
        k[st][2] = dt * u[1];
        // Jk = dt·(fθ ⊗ row θ of Jt + [0 | fu])
        const double fth[NX] = {-v * s, v * c, 0.0};
        for (int i = 0; i < NX; ++i)
            for (int j = 0; j < W; ++j) Jk[st][i][j] = dt * fth[i] * Jt[2][j];
        Jk[st][0][NX] += dt * c;
        Jk[st][1][NX] += dt * s;
        Jk[st][2][NX + 1] += dt;
    }
    for (int i = 0; i < NX; ++i) {
        xn[i] = x[i] + (k[0][i] + 4.0 * k[1][i] + k[2][i]) / 6.0;
        for (int j = 0; j < W; ++j) J[i][j] = ((i == j) ? 1.0 : 0.0) + (Jk[0][i][j] + 4.0 * Jk[1][i][j] + Jk[2][i][j]) / 6.0;
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

__device__ __forceinline__ void knot_merit(const Args &A, int t, int k, const KnotPt &p, double &cost, double &c1)
{
    const int N = A.N;
    const int64_t o = (int64_t)W * k;
    double x[NX], u[NU] = {0.0, 0.0};
    for (int i = 0; i < NX; ++i) x[i] = p.at(o + i);
    const double *xf = A.xf + (int64_t)t * NX;
    cost = 0.0;
    c1 = 0.0;
    if (k < N - 1) {
        for (int i = 0; i < NU; ++i) u[i] = p.at(o + NX + i);
        for (int i = 0; i < NX; ++i) cost += 0.5 * (x[i] - xf[i]) * A.Q[i] * (x[i] - xf[i]);
        for (int i = 0; i < NU; ++i) cost += 0.5 * u[i] * A.R[i] * u[i];
        double xn[NX];
        rk3(x, u, A.dt, xn);
        if (k == 0)
            for (int i = 0; i < NX; ++i) c1 += fabs(x[i] - A.x0[(int64_t)t * NX + i]);
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
__device__ double merit(const Args &A, int t, const KnotPt &p, int lane)
{
    double f = 0.0, c = 0.0;
    for (int k = lane; k < A.N; k += 64) {
        double ck, c1;
        knot_merit(A, t, k, p, ck, c1);
        f += ck;
        c += c1;
    }
    return wave_sum(f) + A.mu * wave_sum(c);
}

// z ← p, λ ← λ of the Newton solve, one more accepted step (wave-cooperative, coalesced)
__device__ void accept(const Args &A, int64_t t, const KnotPt &p, int lane)
{
    const int64_t NN = nn(A.N), P = np_(A.N);
    double *z = A.Z + t * NN;
    for (int64_t i = lane; i < NN; i += 64) z[i] = p.at(i);
    for (int64_t i = lane; i < P; i += 64) A.lam[t * P + i] = A.lamn[t * P + i];
    if (lane == 0) A.iters[t] += 1;
}

// ---------------------------------------------------------------- assembly (update!) + check
// Knot k: Y_k, y_k, H_k, g_k of the Dubins structure (knot 0: (n1 0, p 3, n2 3, w 5),
// interior (3, 0, 3, 5), last (3, 3, 0, 3)) and its share of the convergence check: cost,
// Σ|c|, max|c|, ‖g_k + Y_kᵀ m_k‖² with m_k = [λ_{k-1}; μ_k; λ_k] the multipliers of the
// last Newton step (calc_residual!, cholesky_solver.jl:201-236).  Then the wave's check:
// ‖c‖∞ < tol_p and ‖∇f + ∇cᵀλ‖₂ < tol_d → converged (cholesky_solver.jl:129-137).
__device__ void expand_knot(const Args &A, int t, int k, double &cost, double &c1, double &cinf, double &r2)
{
    const int N = A.N;
    const int64_t NN = nn(N), P = np_(N);
    const double *z = A.Z + t * NN + (int64_t)W * k;
    const double *xf = A.xf + (int64_t)t * NX;
    double *Y = A.Y + t * ny_(N) + 30 * (int64_t)k;
    double *y = A.y + t * P + oy(k);
    double *H = A.H + t * NN + (int64_t)W * k;
    double *g = A.g + t * NN + (int64_t)W * k;
    const double *m = A.lam + t * P + om(k);
    double x[NX];
    for (int i = 0; i < NX; ++i) x[i] = z[i];
    auto con = [&](double v, int i) {
        y[i] = v;
        c1 += fabs(v);
        cinf = fmax(cinf, fabs(v));
    };
    if (k < N - 1) {
        const double u[NU] = {z[NX], z[NX + 1]};
        double xn[NX], J[NX][W];
        rk3_jac(x, u, A.dt, xn, J);
        // rows: k == 0: [C = [I 0] (initial state); D1 = J]; else [D2 = [−I 0]; D1 = J]
        double Yk[6][W];
        for (int i = 0; i < NX; ++i)
            for (int j = 0; j < W; ++j) {
                Yk[i][j] = (i == j) ? (k == 0 ? 1.0 : -1.0) : 0.0;
                Yk[NX + i][j] = J[i][j];
            }
        for (int j = 0; j < W; ++j)
            for (int i = 0; i < 6; ++i) Y[i + 6 * j] = Yk[i][j];
        int r = 0;
        if (k == 0)
            for (int i = 0; i < NX; ++i) con(x[i] - A.x0[(int64_t)t * NX + i], r++);
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
        for (int j = 0; j < W; ++j) {
            g[j] = gk[j];
            double sres = gk[j];
            for (int i = 0; i < 6; ++i) sres += Yk[i][j] * m[i];
            r2 += sres * sres;
        }
    } else {
        // last knot: [D2 = −I; C = I (goal)], 6×3
        for (int j = 0; j < NX; ++j)
            for (int i = 0; i < NX; ++i) {
                Y[i + 6 * j] = (i == j) ? -1.0 : 0.0;
                Y[NX + i + 6 * j] = (i == j) ? 1.0 : 0.0;
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

__global__ __launch_bounds__(64 * TPB) void sqp_expand_kernel(const Args A)
{
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * TPB + (threadIdx.x >> 6);
    if (t >= A.B || A.status[t] != ACTIVE) return;                 // wave-uniform
    double cost = 0.0, c1 = 0.0, cinf = 0.0, r2 = 0.0;
    for (int k = lane; k < A.N; k += 64) expand_knot(A, (int)t, k, cost, c1, cinf, r2);
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
__global__ __launch_bounds__(64 * TPB) void sqp_ls1_kernel(const Args A)
{
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * TPB + (threadIdx.x >> 6);
    if (t >= A.B) return;
    if (lane == 0) A.need_soc[t] = 0;
    if (A.status[t] != ACTIVE) return;
    const int N = A.N;
    const int64_t NN = nn(N), P = np_(N);
    const double *z = A.Z + t * NN, *dz = A.dz + t * NN, *g = A.g + t * NN;
    double gd = 0.0;
    for (int64_t i = lane; i < NN; i += 64) gd += g[i] * dz[i];
    const double dphi = wave_sum(gd) + A.dphi[t];
    const KnotPt p1{z, dz, nullptr, 1.0, 0.0};
    const double phi1 = merit(A, (int)t, p1, lane);
    if (lane == 0) A.dphi[t] = dphi;
    if (phi1 <= A.phi0[t] + ETA * dphi) {
        accept(A, t, p1, lane);
        return;
    }
    if (lane == 0) A.need_soc[t] = 1;
    double *y = A.y + t * P;
    for (int k = lane; k < N; k += 64) {
        const int64_t o = (int64_t)W * k;
        double x[NX];
        for (int i = 0; i < NX; ++i) x[i] = p1.at(o + i);
        double *yk = y + oy(k);
        if (k < N - 1) {
            const double u[NU] = {p1.at(o + NX), p1.at(o + NX + 1)};
            double xn[NX];
            rk3(x, u, A.dt, xn);
            int r = 0;
            if (k == 0)
                for (int i = 0; i < NX; ++i) yk[r++] = x[i] - A.x0[t * NX + i];
            for (int i = 0; i < NX; ++i) yk[r++] = xn[i] - p1.at(o + W + i);
        } else {
            for (int i = 0; i < NX; ++i) yk[i] = x[i] - A.xf[t * NX + i];
        }
    }
}

// ---------------------------------------------------------------- line search, SOC + backtracking
// dubins_sqp.jl:82-94: z + dz + dẑ accepted on strict decrease below ϕ + ηϕ′; else α = ρ, ρ², …
__global__ __launch_bounds__(64 * TPB) void sqp_ls2_kernel(const Args A)
{
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * TPB + (threadIdx.x >> 6);
    if (t >= A.B || !A.need_soc[t]) return;
    const int64_t NN = nn(A.N);
    const double *z = A.Z + t * NN, *dz = A.dz + t * NN, *ds = A.dzs + t * NN;
    const double phi0 = A.phi0[t], dphi = A.dphi[t];
    const KnotPt ps{z, dz, ds, 1.0, 1.0};
    if (merit(A, (int)t, ps, lane) < phi0 + ETA * dphi) {
        accept(A, t, ps, lane);
        return;
    }
    double a = RHO;
    for (int i = 1; i < LS_TRIES; ++i, a *= RHO) {
        const KnotPt pa{z, dz, nullptr, a, 0.0};
        if (merit(A, (int)t, pa, lane) <= phi0 + ETA * a * dphi) {
            accept(A, t, pa, lane);
            return;
        }
    }
    if (lane == 0) A.status[t] = LS_FAILED;
}

__global__ __launch_bounds__(256) void sqp_init_kernel(const Args A)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t P = np_(A.N);
    if (i < A.B * P) A.lam[i] = 0.0;
    if (i < A.B) {
        A.status[i] = ACTIVE;
        A.iters[i] = 0;
    }
}

__global__ __launch_bounds__(256) void sqp_finish_kernel(const Args A)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < A.B && A.status[t] == ACTIVE) A.status[t] = LIMIT;
}

static dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

} // namespace sqp

// the structure tables of the Dubins KKT (ConstraintBlocks, conblocks.jl:403-425)
void sqp_structure(int N, std::vector<int32_t> &n1, std::vector<int32_t> &p, std::vector<int32_t> &n2,
                   std::vector<int32_t> &w)
{
    using namespace sqp;
    n1.assign(N, NX);
    p.assign(N, 0);
    n2.assign(N, NX);
    w.assign(N, W);
    n1[0] = 0;
    p[0] = NX;
    p[N - 1] = NX;
    n2[N - 1] = 0;
    w[N - 1] = NX;
}

// Device driver (lqrx_api.cpp validates and calls this).  kkt(ctx, ginv, dz) runs one KKT
// solve of the Dubins structure on Y, y, H, g → dz, lamn; a negative return stops the loop.
hipError_t sqp_run(const SqpArgs &A0, int max_iters, hipStream_t s, int (*kkt)(void *ctx, int ginv, double *dz),
                   void *ctx, int *kkt_rc)
{
    using namespace sqp;
    SqpArgs A = A0;
    const int64_t BP = A.B * np_(A.N);
    hipLaunchKernelGGL(sqp_init_kernel, grid_for(BP > A.B ? BP : A.B), dim3(256), 0, s, A);
    int32_t h_active = 0;
    for (int it = 0; it < max_iters; ++it) {
        hipError_t e = hipMemsetAsync(A.n_active, 0, sizeof(int32_t), s);
        if (e != hipSuccess) return e;
        const dim3 gw((unsigned)((A.B + TPB - 1) / TPB)), bw(64 * TPB);
        hipLaunchKernelGGL(sqp_expand_kernel, gw, bw, 0, s, A);
        if ((e = hipMemcpyAsync(&h_active, A.n_active, sizeof(int32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return e;
        if (h_active == 0) break;
        if ((*kkt_rc = kkt(ctx, 1, A.dz)) < 0) return hipSuccess;
        hipLaunchKernelGGL(sqp_ls1_kernel, gw, bw, 0, s, A);
        if ((*kkt_rc = kkt(ctx, 0, A.dzs)) < 0) return hipSuccess;
        hipLaunchKernelGGL(sqp_ls2_kernel, gw, bw, 0, s, A);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(sqp_finish_kernel, grid_for(A.B), dim3(256), 0, s, A);
    return hipGetLastError();
}

} // namespace lqrx
