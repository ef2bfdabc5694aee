/*
 * lqr_oracle.c — CPU ORACLE for the lqrx hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the reported CPU baseline.  The product path
 * (lqr.jl_amd/csrc → liblqrx.so) never links, loads or calls anything in oracle/.
 *
 * What it is: a plain-C, fp64, op-for-op restatement of the reference's algorithms:
 *
 *   DP (Riccati backward pass + forward rollout)
 *     /root/reference/src/dynamic_programming.jl:28-31  chol_solve!  (potrf 'U' + potrs 'U')
 *     /root/reference/src/dynamic_programming.jl:37-43  compute_gain!
 *     /root/reference/src/dynamic_programming.jl:48-52  compute_ctg!
 *     /root/reference/src/dynamic_programming.jl:54-72  solve!
 *
 *   KKT (block-tridiagonal Schur complement + block upper Cholesky + substitutions)
 *     /root/reference/src/jacobian_blocks.jl:220-286   calculate_shur_factors!/shur!/copy_shur!
 *     /root/reference/src/cholesky_solve.jl:47-67     cholesky!(U, F)   (block upper recurrence)
 *     /root/reference/src/cholesky_solve.jl:93-143     forward_/backward_substitution!
 *     /root/reference/src/cholesky_solver.jl:185-236    calculate_primals!/calc_residual!
 *     /root/reference/src/block_cholesky.jl:55-101      H_k factor modes (dense / block-diag / diag)
 *
 * Pinning: the reference is Julia and cannot run here (no julia binary, unvendored deps,
 * SURVEY.md §8(c)); it ships no golden vectors.  The KKT restatement is pinned by
 * re-running the reference's own known-answer identities (test/cholesky_solve.jl:18-44)
 * in tests/test_oracle.py; the DP restatement is pinned by identities (dense-KKT optimum,
 * DARE limit) because the reference's DP test (test/dp.jl) holds no assertion.
 *
 * LAPACK/BLAS semantics restated (Julia's OpenBLAS, version unpinned):
 *   dpotrf('U'): A = UᵀU, U in the upper triangle, lower triangle untouched; info = order
 *                of the first non-positive leading minor (the reference DISCARDS info).
 *   dpotrs('U'): solve A X = B as Uᵀ Y = B then U X = Y.
 *   dtrsm/dtrsv('U','T') / ('U','N'): triangular solves with U.
 * Layout: column-major (Julia), element (i,j) of an r×c matrix at [i + j*r].
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define IDX(i, j, ld) ((size_t)(i) + (size_t)(j) * (size_t)(ld))

/* ---------------------------------------------------------------- dense helpers */

/* C(r×c) = op(A) op(B), column-major.  ta/tb: 0 = as-is, 1 = transposed. */
static void gemm(int r, int c, int kk, int ta, const double *A, int lda, int tb,
                 const double *B, int ldb, double *C, int ldc)
{
    for (int j = 0; j < c; ++j)
        for (int i = 0; i < r; ++i) {
            double s = 0.0;
            for (int p = 0; p < kk; ++p) {
                double a = ta ? A[IDX(p, i, lda)] : A[IDX(i, p, lda)];
                double b = tb ? B[IDX(j, p, ldb)] : B[IDX(p, j, ldb)];
                s += a * b;
            }
            C[IDX(i, j, ldc)] = s;
        }
}

/* Unblocked upper Cholesky (dpotf2 'U' semantics).  Returns LAPACK info. */
int oracle_potrf_upper(int n, double *A, int lda)
{
    for (int j = 0; j < n; ++j) {
        double d = A[IDX(j, j, lda)];
        for (int p = 0; p < j; ++p) d -= A[IDX(p, j, lda)] * A[IDX(p, j, lda)];
        if (!(d > 0.0)) { A[IDX(j, j, lda)] = d; return j + 1; }
        d = sqrt(d);
        A[IDX(j, j, lda)] = d;
        for (int c = j + 1; c < n; ++c) {
            double s = A[IDX(j, c, lda)];
            for (int p = 0; p < j; ++p) s -= A[IDX(p, j, lda)] * A[IDX(p, c, lda)];
            A[IDX(j, c, lda)] = s / d;
        }
    }
    return 0;
}

/* X ← U⁻ᵀ X  (dtrsm 'L','U','T','N'), X is n×nrhs */
static void trsm_ut(int n, int nrhs, const double *U, int ldu, double *X, int ldx)
{
    for (int c = 0; c < nrhs; ++c)
        for (int i = 0; i < n; ++i) {
            double s = X[IDX(i, c, ldx)];
            for (int p = 0; p < i; ++p) s -= U[IDX(p, i, ldu)] * X[IDX(p, c, ldx)];
            X[IDX(i, c, ldx)] = s / U[IDX(i, i, ldu)];
        }
}

/* X ← U⁻¹ X  (dtrsm 'L','U','N','N') */
static void trsm_un(int n, int nrhs, const double *U, int ldu, double *X, int ldx)
{
    for (int c = 0; c < nrhs; ++c)
        for (int i = n - 1; i >= 0; --i) {
            double s = X[IDX(i, c, ldx)];
            for (int p = i + 1; p < n; ++p) s -= U[IDX(i, p, ldu)] * X[IDX(p, c, ldx)];
            X[IDX(i, c, ldx)] = s / U[IDX(i, i, ldu)];
        }
}

/* dpotrs('U') */
static void potrs_upper(int n, int nrhs, const double *U, int ldu, double *X, int ldx)
{
    trsm_ut(n, nrhs, U, ldu, X, ldx);
    trsm_un(n, nrhs, U, ldu, X, ldx);
}

/* ======================================================================== DP */

/*
 * One trajectory of solve!(sol, ::DPSolver, ::LQRProblem), dynamic_programming.jl:54-72.
 *   A n×n, B n×m, Q n×n, R m×m, Qf n×n, x0 n  (time-invariant, lqr_problem.jl:1-11)
 *   K  m×n×(N-1)   K[k] for k = 1..N-1 (Julia index) stored at slot k-1
 *   P  n×n         P_1 (p_all == 0, what solver.P holds on return, :63)
 *      n×n×N       P_k for k = 1..N (p_all != 0; P_N = Qf)
 *   X  n×N, U m×(N-1)
 * Returns info: 0, or the (1-based) knot k whose E = R + BᵀPB was not SPD (first met in
 * the backward sweep).  The sweep continues either way, as the reference does.
 */
/*
 * Linear cost terms (SURVEY §8(f) rank 1 "cost linear terms"; an extension — the reference
 * LQRProblem has none): stage cost ½xᵀQx + qᵀx + ½uᵀRu + rᵀu, terminal ½xᵀQf x + qfᵀx.
 * The value function gains a linear part, V_k(x) = ½xᵀP_k x + p_kᵀx, and the policy a
 * feedforward, u_k = −K_k x_k − d_k.  Restated in the reference's own op order: d is one
 * more right-hand side of the same chol_solve! (:42, potrs on [B'PA | r + B'p]), and p
 * follows compute_ctg!'s P_ .= Q + A'PA − APB*K (:51) as p_ .= q + A'p − APB*d.
 *   q  n (per knot with tvQR: n×(N-1), knot k at slot k-1), r m (idem), qf n
 *   d  m×(N-1)   d[k] for k = 1..N-1 at slot k-1
 *   p  n (p_all == 0: p_1) or n×N (p_all: p_k for k = 1..N, p_N = qf)
 * q == NULL runs the plain reference recursion (r, qf, d, p unused).
 */
int oracle_dp_solve_one_lin(int n, int m, int N, const double *A0, const double *B0,
                            const double *Q0, const double *R0, const double *Qf,
                            const double *x0, double *K, double *P, int p_all, double *X,
                            double *U, int tvAB, int tvQR, const double *q0,
                            const double *r0, const double *qf, double *d, double *p)
{
    size_t nn = (size_t)n * n, nm = (size_t)n * m, mm = (size_t)m * m;
    double *Pc = malloc(nn * sizeof(double)), *P_ = malloc(nn * sizeof(double));
    double *PA = malloc(nn * sizeof(double)), *PB = malloc(nm * sizeof(double));
    double *APB = malloc(nm * sizeof(double)), *E = malloc(mm * sizeof(double));
    double *T1 = malloc(nn * sizeof(double)), *T2 = malloc(nn * sizeof(double));
    const int lin = q0 != NULL;
    double *pc = malloc((size_t)n * sizeof(double)), *p_ = malloc((size_t)n * sizeof(double));
    double *t1 = malloc((size_t)n * sizeof(double)), *t2 = malloc((size_t)n * sizeof(double));
    int info = 0;

    memcpy(Pc, Qf, nn * sizeof(double));                       /* :58  P .= Qf */
    if (p_all) memcpy(P + (size_t)(N - 1) * nn, Qf, nn * sizeof(double));
    if (lin) {                                                 /* p .= qf */
        memcpy(pc, qf, (size_t)n * sizeof(double));
        if (p_all) memcpy(p + (size_t)(N - 1) * n, qf, (size_t)n * sizeof(double));
    }

    for (int k = N - 1; k >= 1; --k) {                        /* :61  k = N-1:-1:1 */
        double *Kk = K + (size_t)(k - 1) * nm;
        /* time-varying extension (LCRProblem.A[k]/B[k]): knot k's
         * matrices; the time-invariant reference is tvAB = tvQR = 0 */
        const double *A = A0 + (tvAB ? (size_t)(k - 1) * nn : 0);
        const double *B = B0 + (tvAB ? (size_t)(k - 1) * nm : 0);
        const double *Q = Q0 + (tvQR ? (size_t)(k - 1) * nn : 0);
        const double *R = R0 + (tvQR ? (size_t)(k - 1) * mm : 0);
        /* compute_gain!  :37-43 */
        gemm(n, m, n, 0, Pc, n, 0, B, n, PB, n);               /* :38  PB .= P*B */
        gemm(m, m, n, 1, B, n, 0, PB, n, E, m);                /* :39  E .= R .+ B'PB */
        for (size_t i = 0; i < mm; ++i) E[i] = R[i] + E[i];
        gemm(n, n, n, 0, Pc, n, 0, A, n, PA, n);               /* :40  PA .= P*A */
        gemm(m, n, n, 1, B, n, 0, PA, n, Kk, m);               /* :41  K .= B'PA */
        int st = oracle_potrf_upper(m, E, m);                  /* :29  potrf!('U',E) */
        if (st && !info) info = k;
        potrs_upper(m, n, E, m, Kk, m);                        /* :30  potrs!('U',E,K) */
        double *dk = lin ? d + (size_t)(k - 1) * m : NULL;
        if (lin) {                                             /* d = E⁻¹(r + B'p) */
            const double *r = r0 + (tvQR ? (size_t)(k - 1) * m : 0);
            gemm(m, 1, n, 1, B, n, 0, pc, n, dk, m);
            for (int i = 0; i < m; ++i) dk[i] = r[i] + dk[i];
            potrs_upper(m, 1, E, m, dk, m);
        }
        /* compute_ctg!  :50-51 */
        gemm(n, m, n, 1, A, n, 0, PB, n, APB, n);              /* :50  APB .= A'PB */
        gemm(n, n, n, 1, A, n, 0, PA, n, T1, n);               /*      A'PA         */
        gemm(n, n, m, 0, APB, n, 0, Kk, m, T2, n);             /*      APB*K        */
        for (size_t i = 0; i < nn; ++i) P_[i] = Q[i] + T1[i] - T2[i]; /* :51 */
        memcpy(Pc, P_, nn * sizeof(double));                   /* :63  P .= P_ */
        if (p_all) memcpy(P + (size_t)(k - 1) * nn, Pc, nn * sizeof(double));
        if (lin) {                                             /* p_ .= q + A'p − APB*d */
            const double *q = q0 + (tvQR ? (size_t)(k - 1) * n : 0);
            gemm(n, 1, n, 1, A, n, 0, pc, n, t1, n);
            gemm(n, 1, m, 0, APB, n, 0, dk, m, t2, n);
            for (int i = 0; i < n; ++i) p_[i] = q[i] + t1[i] - t2[i];
            memcpy(pc, p_, (size_t)n * sizeof(double));
            if (p_all) memcpy(p + (size_t)(k - 1) * n, pc, (size_t)n * sizeof(double));
        }
    }
    if (!p_all) memcpy(P, Pc, nn * sizeof(double));
    if (lin && !p_all) memcpy(p, pc, (size_t)n * sizeof(double));

    memcpy(X, x0, (size_t)n * sizeof(double));                 /* :66 */
    for (int k = 1; k <= N - 1; ++k) {                         /* :67-70 */
        const double *Kk = K + (size_t)(k - 1) * nm;
        const double *xk = X + (size_t)(k - 1) * n;
        double *uk = U + (size_t)(k - 1) * m, *xn = X + (size_t)k * n;
        const double *A = A0 + (tvAB ? (size_t)(k - 1) * nn : 0);
        const double *B = B0 + (tvAB ? (size_t)(k - 1) * nm : 0);
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            for (int j = 0; j < n; ++j) s += Kk[IDX(i, j, m)] * xk[j];
            uk[i] = lin ? -(s + d[(size_t)(k - 1) * m + i]) : -s;   /* u = −Kx (− d) */
        }
        for (int i = 0; i < n; ++i) {
            double s = 0.0, t = 0.0;
            for (int j = 0; j < n; ++j) s += A[IDX(i, j, n)] * xk[j];
            for (int j = 0; j < m; ++j) t += B[IDX(i, j, n)] * uk[j];
            xn[i] = s + t;
        }
    }
    free(Pc); free(P_); free(PA); free(PB); free(APB); free(E); free(T1); free(T2);
    free(pc); free(p_); free(t1); free(t2);
    return info;
}

int oracle_dp_solve_one_tv(int n, int m, int N, const double *A0, const double *B0,
                           const double *Q0, const double *R0, const double *Qf,
                           const double *x0, double *K, double *P, int p_all, double *X,
                           double *U, int tvAB, int tvQR)
{
    return oracle_dp_solve_one_lin(n, m, N, A0, B0, Q0, R0, Qf, x0, K, P, p_all, X, U, tvAB,
                                   tvQR, NULL, NULL, NULL, NULL, NULL);
}

int oracle_dp_solve_one(int n, int m, int N, const double *A, const double *B,
                        const double *Q, const double *R, const double *Qf,
                        const double *x0, double *K, double *P, int p_all, double *X,
                        double *U)
{
    return oracle_dp_solve_one_tv(n, m, N, A, B, Q, R, Qf, x0, K, P, p_all, X, U, 0, 0);
}

/*
 * Batched driver, Julia layout (batch slowest).  `nthreads` > 1 uses OpenMP when the
 * library is built with -fopenmp (the CPU baseline); returns the number of trajectories
 * with info != 0.  Inputs may be time-invariant only (the reference LQRProblem).
 */
int64_t oracle_dp_solve_batch_tv(int n, int m, int N, int64_t batch, const double *A,
                                 const double *B, const double *Q, const double *R,
                                 const double *Qf, const double *x0, double *K, double *P,
                                 int p_all, double *X, double *U, int32_t *info, int nthreads,
                                 int tvAB, int tvQR)
{
    size_t nn = (size_t)n * n, nm = (size_t)n * m, mm = (size_t)m * m;
    size_t kAB = tvAB ? (size_t)(N - 1) : 1, kQR = tvQR ? (size_t)(N - 1) : 1;
    size_t pstride = p_all ? nn * (size_t)N : nn;
    int64_t bad = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads) reduction(+ : bad)
#endif
    for (int64_t b = 0; b < batch; ++b) {
        int st = oracle_dp_solve_one_tv(n, m, N, A + b * nn * kAB, B + b * nm * kAB,
                                        Q + b * nn * kQR, R + b * mm * kQR,
                                        Qf + b * nn, x0 + b * (size_t)n,
                                        K + b * nm * (size_t)(N - 1), P + b * pstride, p_all,
                                        X + b * (size_t)n * N, U + b * (size_t)m * (N - 1),
                                        tvAB, tvQR);
        if (info) info[b] = st;
        bad += (st != 0);
    }
    (void)nthreads;
    return bad;
}

/* batched driver of oracle_dp_solve_one_lin (q, r follow tvQR's knot layout) */
int64_t oracle_dp_solve_batch_lin(int n, int m, int N, int64_t batch, const double *A,
                                  const double *B, const double *Q, const double *R,
                                  const double *Qf, const double *x0, double *K, double *P,
                                  int p_all, double *X, double *U, int32_t *info, int nthreads,
                                  int tvAB, int tvQR, const double *q, const double *r,
                                  const double *qf, double *d, double *p)
{
    size_t nn = (size_t)n * n, nm = (size_t)n * m, mm = (size_t)m * m;
    size_t kAB = tvAB ? (size_t)(N - 1) : 1, kQR = tvQR ? (size_t)(N - 1) : 1;
    size_t pstride = p_all ? nn * (size_t)N : nn, vstride = p_all ? (size_t)n * N : (size_t)n;
    int64_t bad = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads) reduction(+ : bad)
#endif
    for (int64_t b = 0; b < batch; ++b) {
        int st = oracle_dp_solve_one_lin(n, m, N, A + b * nn * kAB, B + b * nm * kAB,
                                         Q + b * nn * kQR, R + b * mm * kQR,
                                         Qf + b * nn, x0 + b * (size_t)n,
                                         K + b * nm * (size_t)(N - 1), P + b * pstride, p_all,
                                         X + b * (size_t)n * N, U + b * (size_t)m * (N - 1),
                                         tvAB, tvQR, q + b * (size_t)n * kQR,
                                         r + b * (size_t)m * kQR, qf + b * (size_t)n,
                                         d + b * (size_t)m * (N - 1), p + b * vstride);
        if (info) info[b] = st;
        bad += (st != 0);
    }
    (void)nthreads;
    return bad;
}

int64_t oracle_dp_solve_batch(int n, int m, int N, int64_t batch, const double *A,
                              const double *B, const double *Q, const double *R,
                              const double *Qf, const double *x0, double *K, double *P,
                              int p_all, double *X, double *U, int32_t *info, int nthreads)
{
    return oracle_dp_solve_batch_tv(n, m, N, batch, A, B, Q, R, Qf, x0, K, P, p_all, X, U,
                                    info, nthreads, 0, 0);
}

int oracle_num_threads_max(void)
{
#ifdef _OPENMP
    extern int omp_get_max_threads(void);
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ======================================================================== KKT */

/*
 * Per-knot block sizes follow ConstraintBlocks (conblocks.jl:403-425): block k has
 *   n1[k] rows of D2 (previous dynamics), p[k] stage rows C, n2[k] rows of D1 (dynamics
 *   at k), width w[k] = n̄ + m·(k<N).  n1[k] == n2[k-1] (the aliased A ≡ previous C block,
 *   jacobian_blocks.jl:166).
 * Per-trajectory packed inputs (concatenated over k = 1..N, each block column-major):
 *   Y  : rows_k × w_k,  rows_k = n1+p+n2   Y = [D2; C; D1]     (conblocks.jl:365-401)
 *   y  : p_k + n2_k                         y = [c; d]
 *   H  : h_mode 0/1 → w_k × w_k cost Hessian (dense / block-diag: same storage);
 *        h_mode 2 → w_k diagonal                                  (block_cholesky.jl:55-91)
 *   g  : w_k                                 gradient [q; r]      (block_cholesky.jl:126-132)
 * Outputs:
 *   dz : w_k per knot  (δz = -H⁻¹(Dᵀλ + g), or −Dᵀλ for the SOC variant ginv == 0)
 *   lam: p_k + n2_k per knot, [μ_k; λ_k]  (get_multipliers ordering, jacobian_blocks.jl:197-211)
 * Optional dense debug outputs (NULL to skip), P = Σ (p_k + n2_k):
 *   S (P×P, upper blocks as copy_shur_factors! writes them), U (P×P, block Cholesky
 *   factor, strictly-lower part zero), r (P)
 */
typedef struct {
    int p1, ps, p2;
    double *A, *B, *C, *D, *E, *F; /* p1×p1 (aliases prev C), ps×ps, p2×p2, p1×ps, ps×p2, p1×p2 */
    double *mu, *lam, *c, *d;
} oblk;

static void alloc_blocks(int N, const int *n1, const int *p, const int *n2, oblk *F)
{
    for (int k = 0; k < N; ++k) {
        oblk *b = &F[k];
        b->p1 = n1[k]; b->ps = p[k]; b->p2 = n2[k];
        b->A = (k == 0) ? calloc((size_t)b->p1 * b->p1 + 1, sizeof(double)) : F[k - 1].C;
        b->B = calloc((size_t)b->ps * b->ps + 1, sizeof(double));
        b->C = calloc((size_t)b->p2 * b->p2 + 1, sizeof(double));
        b->D = calloc((size_t)b->p1 * b->ps + 1, sizeof(double));
        b->E = calloc((size_t)b->ps * b->p2 + 1, sizeof(double));
        b->F = calloc((size_t)b->p1 * b->p2 + 1, sizeof(double));
        b->mu = calloc((size_t)b->ps + 1, sizeof(double));
        b->lam = calloc((size_t)b->p2 + 1, sizeof(double));
        b->c = calloc((size_t)b->ps + 1, sizeof(double));
        b->d = calloc((size_t)b->p2 + 1, sizeof(double));
    }
}

static void free_blocks(int N, oblk *F)
{
    for (int k = 0; k < N; ++k) {
        if (k == 0) free(F[k].A);
        free(F[k].B); free(F[k].C); free(F[k].D); free(F[k].E); free(F[k].F);
        free(F[k].mu); free(F[k].lam); free(F[k].c); free(F[k].d);
    }
}

/* X ← H⁻¹ X for one knot; X is w×nc.  Dense/block-diag: the factor Hf (upper Cholesky in
 * place, block_cholesky.jl:63/74-75) applied as potrs; diag: multiply by 1/h
 * (block_cholesky.jl:85-96). */
static void hinv_apply(int hm, int w, const double *Hf, double *X, int nc)
{
    if (hm == 2) {
        for (int c = 0; c < nc; ++c)
            for (int i = 0; i < w; ++i) X[IDX(i, c, w)] *= Hf[i];
    } else {
        potrs_upper(w, nc, Hf, w, X, w);
    }
}

/* Shared by the upper solve and the lower-variant factor: per-knot offsets into the
 * packed inputs, the H_k factors and the Schur pieces r_k. */
typedef struct {
    size_t *oY, *oy, *oH, *og;
    double *Hf;
    double **rk;
} kkt_work;

static void kkt_work_free(int N, kkt_work *wk)
{
    for (int k = 0; k < N; ++k) free(wk->rk[k]);
    free(wk->rk); free(wk->Hf); free(wk->oY); free(wk->oy); free(wk->oH); free(wk->og);
}

/* H_k factors (block_cholesky.jl:55-91,145-153) and calculate_shur_factors!
 * (jacobian_blocks.jl:220-286) into F, stored as copy_shur!(::BlockUpperTriangular3)
 * writes it (:271-286).  Returns −(k+1) for the first H_k that is not SPD, else 0. */
static int kkt_schur(int N, const int *n1, const int *p, const int *n2, const int *w,
                     const double *Y, const double *y, int h_mode, const double *H,
                     const double *g, int ginv, oblk *F, kkt_work *wkp)
{
    int info = 0;
    size_t *oY = malloc(N * sizeof(size_t)), *oy = malloc(N * sizeof(size_t));
    size_t *oH = malloc(N * sizeof(size_t)), *og = malloc(N * sizeof(size_t));
    size_t aY = 0, ay = 0, aH = 0, ag = 0;
    for (int k = 0; k < N; ++k) {
        int rows = n1[k] + p[k] + n2[k];
        oY[k] = aY; aY += (size_t)rows * w[k];
        oy[k] = ay; ay += (size_t)p[k] + n2[k];
        oH[k] = aH; aH += (h_mode == 2) ? (size_t)w[k] : (size_t)w[k] * w[k];
        og[k] = ag; ag += (size_t)w[k];
    }

    /* H_k factors (InvertedQuadratic / update_cost!, block_cholesky.jl:145-153) */
    double *Hf = malloc((aH + 1) * sizeof(double));
    for (int k = 0; k < N; ++k) {
        if (h_mode == 2) {
            for (int i = 0; i < w[k]; ++i) Hf[oH[k] + i] = 1.0 / H[oH[k] + i]; /* :86,:89 inv */
        } else {
            memcpy(Hf + oH[k], H + oH[k], (size_t)w[k] * w[k] * sizeof(double));
            int st = oracle_potrf_upper(w[k], Hf + oH[k], w[k]);          /* :63 potrf! */
            if (st && !info) info = -(k + 1);
        }
    }

    /* KKT-3/4/5: calculate_shur_factors!  (jacobian_blocks.jl:220-286) */
    double **rk = malloc(N * sizeof(double *));
    for (int k = 0; k < N; ++k) {
        int rows = n1[k] + p[k] + n2[k], wk = w[k];
        const double *Yk = Y + oY[k];
        double *JYt = malloc(((size_t)wk * rows + 1) * sizeof(double));
        double *YYt = malloc(((size_t)rows * rows + 1) * sizeof(double));
        rk[k] = calloc((size_t)rows + 1, sizeof(double));
        for (int i = 0; i < rows; ++i)                                    /* :232 transpose! */
            for (int j = 0; j < wk; ++j) JYt[IDX(j, i, wk)] = Yk[IDX(i, j, rows)];
        if (ginv) {
            hinv_apply(h_mode, wk, Hf + oH[k], JYt, rows);                /* :234 ldiv! */
            for (int i = 0; i < rows; ++i) {                              /* :236 r = YJ*g */
                double s = 0.0;
                for (int j = 0; j < wk; ++j) s += JYt[IDX(j, i, wk)] * g[og[k] + j];
                rk[k][i] = s;
            }
        }                                                                 /* else r .*= 0 */
        gemm(rows, rows, wk, 0, Yk, rows, 0, JYt, wk, YYt, rows);         /* :240 Y*JYt */
        /* copy_shur!(F[k], block)  :271-286 */
        oblk *b = &F[k];
        int o1 = 0, os = b->p1, o2 = b->p1 + b->ps;
        for (int j = 0; j < b->p1; ++j)
            for (int i = 0; i < b->p1; ++i) b->A[IDX(i, j, b->p1)] += YYt[IDX(o1 + i, o1 + j, rows)];
        for (int j = 0; j < b->ps; ++j)
            for (int i = 0; i < b->ps; ++i) b->B[IDX(i, j, b->ps)] = YYt[IDX(os + i, os + j, rows)];
        for (int j = 0; j < b->p2; ++j)
            for (int i = 0; i < b->p2; ++i) b->C[IDX(i, j, b->p2)] = YYt[IDX(o2 + i, o2 + j, rows)];
        for (int j = 0; j < b->ps; ++j)
            for (int i = 0; i < b->p1; ++i) b->D[IDX(i, j, b->p1)] = YYt[IDX(o1 + i, os + j, rows)];
        for (int j = 0; j < b->p2; ++j)
            for (int i = 0; i < b->ps; ++i) b->E[IDX(i, j, b->ps)] = YYt[IDX(os + i, o2 + j, rows)];
        for (int j = 0; j < b->p2; ++j)
            for (int i = 0; i < b->p1; ++i) b->F[IDX(i, j, b->p1)] = YYt[IDX(o1 + i, o2 + j, rows)];
        for (int i = 0; i < b->ps; ++i) b->c[i] = rk[k][os + i] - y[oy[k] + i];
        for (int i = 0; i < b->p2; ++i) b->d[i] = rk[k][o2 + i] - y[oy[k] + b->ps + i];
        if (k > 0)                                                        /* :251 d .+= r_[1] */
            for (int i = 0; i < F[k - 1].p2; ++i) F[k - 1].d[i] += rk[k][i];
        free(JYt); free(YYt);
    }
    wkp->oY = oY; wkp->oy = oy; wkp->oH = oH; wkp->og = og; wkp->Hf = Hf; wkp->rk = rk;
    return info;
}

int oracle_kkt_solve_one(int N, const int *n1, const int *p, const int *n2, const int *w,
                         const double *Y, const double *y, int h_mode, const double *H,
                         const double *g, int ginv, double *dz, double *lam, double *Sd,
                         double *Ud, double *rd)
{
    oblk *F = calloc((size_t)N, sizeof(oblk)), *U = calloc((size_t)N, sizeof(oblk));
    alloc_blocks(N, n1, p, n2, F);
    alloc_blocks(N, n1, p, n2, U);
    kkt_work kw;
    int info = kkt_schur(N, n1, p, n2, w, Y, y, h_mode, H, g, ginv, F, &kw);
    const size_t *oY = kw.oY, *oH = kw.oH, *og = kw.og;
    const double *Hf = kw.Hf;

    /* dense S and r (copy_shur_factors!, jacobian_blocks.jl:173-211) */
    size_t Ptot = 0;
    for (int k = 0; k < N; ++k) Ptot += (size_t)p[k] + n2[k];
    if (Sd) memset(Sd, 0, Ptot * Ptot * sizeof(double));
    if (Ud) memset(Ud, 0, Ptot * Ptot * sizeof(double));

    /* KKT-7: cholesky!(U, F)  (cholesky_solve.jl:47-67) */
    for (int k = 0; k < N; ++k) {
        oblk *u = &U[k], *f = &F[k];
        int p1 = u->p1, ps = u->ps, p2 = u->p2;
        memcpy(u->D, f->D, (size_t)p1 * ps * sizeof(double));            /* :48 */
        if (p1) trsm_ut(p1, ps, u->A, p1, u->D, p1);                      /* :49 A⁻ᵀD */
        for (int j = 0; j < ps; ++j)                                      /* :50-53 B - D'D */
            for (int i = 0; i < ps; ++i) {
                double s = f->B[IDX(i, j, ps)];
                for (int q = 0; q < p1; ++q) s -= u->D[IDX(q, i, p1)] * u->D[IDX(q, j, p1)];
                u->B[IDX(i, j, ps)] = s;
            }
        if (ps) { int st = oracle_potrf_upper(ps, u->B, ps); if (st && !info) info = k + 1; }
        memcpy(u->F, f->F, (size_t)p1 * p2 * sizeof(double));            /* :56 */
        if (p1) trsm_ut(p1, p2, u->A, p1, u->F, p1);                      /* :57 */
        for (int j = 0; j < p2; ++j)                                      /* :59 E - D'F */
            for (int i = 0; i < ps; ++i) {
                double s = f->E[IDX(i, j, ps)];
                for (int q = 0; q < p1; ++q) s -= u->D[IDX(q, i, p1)] * u->F[IDX(q, j, p1)];
                u->E[IDX(i, j, ps)] = s;
            }
        if (ps) trsm_ut(ps, p2, u->B, ps, u->E, ps);                      /* :60 */
        for (int j = 0; j < p2; ++j)                                      /* :61-62 C - F'F - E'E */
            for (int i = 0; i < p2; ++i) {
                double s = f->C[IDX(i, j, p2)];
                for (int q = 0; q < p1; ++q) s -= u->F[IDX(q, i, p1)] * u->F[IDX(q, j, p1)];
                for (int q = 0; q < ps; ++q) s -= u->E[IDX(q, i, ps)] * u->E[IDX(q, j, ps)];
                u->C[IDX(i, j, p2)] = s;
            }
        if (p2) { int st = oracle_potrf_upper(p2, u->C, p2); if (st && !info) info = k + 1; }
        memcpy(u->c, f->c, (size_t)ps * sizeof(double));                 /* :64-65 */
        memcpy(u->d, f->d, (size_t)p2 * sizeof(double));
    }

    /* KKT-8: forward_substitution!  (cholesky_solve.jl:93-117) */
    for (int k = 0; k < N; ++k) {
        oblk *u = &U[k];
        int p1 = u->p1, ps = u->ps, p2 = u->p2;
        const double *lp = k ? U[k - 1].lam : NULL;
        for (int i = 0; i < ps; ++i) {                                    /* μ = c - D'λ_{k-1} */
            double s = u->c[i];
            for (int q = 0; q < p1 && k; ++q) s -= u->D[IDX(q, i, p1)] * lp[q];
            u->mu[i] = s;
        }
        if (ps) trsm_ut(ps, 1, u->B, ps, u->mu, ps);                      /* B⁻ᵀ */
        for (int i = 0; i < p2; ++i) {                                    /* λ = d - F'λ - E'μ */
            double s = u->d[i];
            for (int q = 0; q < p1 && k; ++q) s -= u->F[IDX(q, i, p1)] * lp[q];
            for (int q = 0; q < ps; ++q) s -= u->E[IDX(q, i, ps)] * u->mu[q];
            u->lam[i] = s;
        }
        if (p2) trsm_ut(p2, 1, u->C, p2, u->lam, p2);                     /* C⁻ᵀ */
    }
    /* KKT-9: backward_substitution!  (cholesky_solve.jl:119-143) */
    for (int k = N - 1; k >= 0; --k) {
        oblk *u = &U[k];
        int ps = u->ps, p2 = u->p2;
        if (k < N - 1) {
            oblk *nx = &U[k + 1];                                         /* Lprev = L[k+1] */
            for (int i = 0; i < p2; ++i) {                                /* λ += D μ' + F λ' */
                double s = u->lam[i];
                for (int q = 0; q < nx->ps; ++q) s += nx->D[IDX(i, q, nx->p1)] * nx->mu[q];
                for (int q = 0; q < nx->p2; ++q) s += nx->F[IDX(i, q, nx->p1)] * nx->lam[q];
                u->lam[i] = s;
            }
            if (p2) trsm_un(p2, 1, u->C, p2, u->lam, p2);
            for (int i = 0; i < ps; ++i) {                                /* μ -= E λ */
                double s = u->mu[i];
                for (int q = 0; q < p2; ++q) s -= u->E[IDX(i, q, ps)] * u->lam[q];
                u->mu[i] = s;
            }
            if (ps) trsm_un(ps, 1, u->B, ps, u->mu, ps);
            for (int i = 0; i < p2; ++i) u->lam[i] = -u->lam[i];
            for (int i = 0; i < ps; ++i) u->mu[i] = -u->mu[i];
        } else {                                                          /* terminal :139-143 */
            if (ps) trsm_un(ps, 1, u->B, ps, u->mu, ps);
            for (int i = 0; i < ps; ++i) u->mu[i] = -u->mu[i];
            /* λ_N (p2 == 0 for the reference's terminal block) is left as forward gave it */
        }
    }

    /* multipliers out, dense S / U / r (copy_block!, Upper, :197-211) */
    size_t off = 0, ol = 0;
    for (int k = 0; k < N; ++k) {
        oblk *u = &U[k], *f = &F[k];
        int p1 = u->p1, ps = u->ps, p2 = u->p2;
        for (int i = 0; i < ps; ++i) lam[ol + i] = u->mu[i];
        for (int i = 0; i < p2; ++i) lam[ol + ps + i] = u->lam[i];
        ol += (size_t)ps + p2;
        size_t b1 = off, bs = off + p1, b2 = off + p1 + ps;
#define PUT(M, blk, r0, c0, nr, nc, upper)                                              \
    for (int j = 0; j < (nc); ++j)                                                      \
        for (int i = 0; i < (nr); ++i)                                                  \
            if (!(upper) || i <= j) M[IDX((r0) + i, (c0) + j, Ptot)] = (blk)[IDX(i, j, (nr))];
        if (Sd) {
            if (k == 0) PUT(Sd, f->A, b1, b1, p1, p1, 0);
            PUT(Sd, f->B, bs, bs, ps, ps, 0); PUT(Sd, f->C, b2, b2, p2, p2, 0);
            PUT(Sd, f->D, b1, bs, p1, ps, 0); PUT(Sd, f->E, bs, b2, ps, p2, 0);
            PUT(Sd, f->F, b1, b2, p1, p2, 0);
        }
        if (Ud) {
            PUT(Ud, u->B, bs, bs, ps, ps, 1); PUT(Ud, u->C, b2, b2, p2, p2, 1);
            PUT(Ud, u->D, b1, bs, p1, ps, 0); PUT(Ud, u->E, bs, b2, ps, p2, 0);
            PUT(Ud, u->F, b1, b2, p1, p2, 0);
        }
#undef PUT
        if (rd) {
            for (int i = 0; i < ps; ++i) rd[bs + i] = f->c[i];
            for (int i = 0; i < p2; ++i) rd[b2 + i] = f->d[i];
        }
        off += (size_t)p1 + ps;
    }

    /* KKT-10: calc_residual! + calc_primals!  (cholesky_solver.jl:185-236) */
    size_t oz = 0;
    for (int k = 0; k < N; ++k) {
        int rows = n1[k] + p[k] + n2[k], wk = w[k];
        const double *Yk = Y + oY[k];
        double *z = dz + oz;
        for (int j = 0; j < wk; ++j) {
            double s = 0.0;
            for (int i = 0; i < n2[k]; ++i) s += Yk[IDX(n1[k] + p[k] + i, j, rows)] * U[k].lam[i]; /* D1'λ */
            for (int i = 0; i < p[k]; ++i) s += Yk[IDX(n1[k] + i, j, rows)] * U[k].mu[i];          /* C'μ */
            if (k > 0)
                for (int i = 0; i < n1[k]; ++i) s += Yk[IDX(i, j, rows)] * U[k - 1].lam[i];      /* D2'λ */
            if (ginv) s += g[og[k] + j];                                  /* add_gradient! */
            z[j] = s;
        }
        if (ginv) {
            hinv_apply(h_mode, wk, Hf + oH[k], z, 1);                     /* :197 ldiv! */
        }
        for (int j = 0; j < wk; ++j) z[j] = -z[j];                        /* :198 / SOC :266 */
        oz += (size_t)wk;
    }

    kkt_work_free(N, &kw);
    free_blocks(N, F); free_blocks(N, U); free(F); free(U);
    return info;
}

/* ------------------------------------------------ KKT-12: lower-storage block Cholesky */

/* Lower Cholesky A = L Lᵀ in place (Julia cholesky(A).L), strict upper part zeroed.
 * Returns LAPACK-style info (cholesky() throws PosDefException there). */
static int potrf_lower(int n, double *A, int lda)
{
    for (int j = 0; j < n; ++j) {
        double d = A[IDX(j, j, lda)];
        for (int q = 0; q < j; ++q) d -= A[IDX(j, q, lda)] * A[IDX(j, q, lda)];
        if (!(d > 0.0)) return j + 1;
        d = sqrt(d);
        A[IDX(j, j, lda)] = d;
        for (int i = j + 1; i < n; ++i) {
            double s = A[IDX(i, j, lda)];
            for (int q = 0; q < j; ++q) s -= A[IDX(i, q, lda)] * A[IDX(j, q, lda)];
            A[IDX(i, j, lda)] = s / d;
        }
        for (int i = 0; i < j; ++i) A[IDX(i, j, lda)] = 0.0;
    }
    return 0;
}

/* X ← X / Lᵀ  (Julia X / chol.U with chol.U = Lᵀ): X is r×c, L lower c×c. */
static void rdiv_lt(int r, int c, double *X, int ldx, const double *L, int ldl)
{
    for (int i = 0; i < r; ++i)
        for (int j = 0; j < c; ++j) {
            double s = X[IDX(i, j, ldx)];
            for (int q = 0; q < j; ++q) s -= X[IDX(i, q, ldx)] * L[IDX(j, q, ldl)];
            X[IDX(i, j, ldx)] = s / L[IDX(j, j, ldl)];
        }
}

/* x ← L⁻¹ x (trans = 0) or L⁻ᵀ x (trans = 1), L lower n×n */
static void trsv_l(int n, const double *L, int ldl, double *x, int trans)
{
    if (!trans) {
        for (int i = 0; i < n; ++i) {
            double s = x[i];
            for (int q = 0; q < i; ++q) s -= L[IDX(i, q, ldl)] * x[q];
            x[i] = s / L[IDX(i, i, ldl)];
        }
    } else {
        for (int i = n - 1; i >= 0; --i) {
            double s = x[i];
            for (int q = i + 1; q < n; ++q) s -= L[IDX(q, i, ldl)] * x[q];
            x[i] = s / L[IDX(i, i, ldl)];
        }
    }
}

/*
 * KKT-12: the reference's lower-storage variant, used only as a cross-check
 * of the upper factor (test/constraint_blocks.jl:96-133).
 *   Schur blocks in BlockLowerTriangular3 storage (copy_shur!(::BlockTriangular3),
 *     jacobian_blocks.jl:254-269: D = YYt[ps,p1], E = YYt[p2,ps], F = YYt[p2,p1]),
 *   cholesky!(L, F)  cholesky_solve.jl:5-26 (A = previous C factor, D/A.U, B = chol(.).L,
 *     F/A.U, E = (F.E − L.F L.Dᵀ)/B.U, C = chol(.).L),
 *   the lower forward/backward substitutions kept (commented out) at cholesky_solve.jl:
 *     146-168 — in the reference the live forward_substitution! has no method for lower
 *     blocks, so these follow the commented text: y = L⁻¹h, then x = L⁻ᵀy = S⁻¹h with
 *     h = [c; d] (= r, the Schur residual).
 * Outputs (P = Σ p_k + n2_k; NULL to skip): Ld (P×P, copy_block! placement :181-195),
 * yv (P, after the forward sweep), xv (P, after the backward sweep).  Returns the
 * 1-based block whose B or C factor failed (cholesky() throws), −(k+1) for a non-SPD
 * H_k, else 0.
 */
int oracle_kkt_lower_one(int N, const int *n1, const int *p, const int *n2, const int *w,
                         const double *Y, const double *y, int h_mode, const double *H,
                         const double *g, int ginv, double *Ld, double *yv, double *xv)
{
    oblk *F = calloc((size_t)N, sizeof(oblk)), *L = calloc((size_t)N, sizeof(oblk));
    alloc_blocks(N, n1, p, n2, F);
    alloc_blocks(N, n1, p, n2, L);   /* D/E/F buffers hold the transposed shapes */
    kkt_work kw;
    int info = kkt_schur(N, n1, p, n2, w, Y, y, h_mode, H, g, ginv, F, &kw);
    size_t Ptot = 0;
    for (int k = 0; k < N; ++k) Ptot += (size_t)p[k] + n2[k];

    /* cholesky!(L, F)  :5-26;  `A` = the previous block's C factor (0×0 at k = 1, :7) */
    for (int k = 0; k < N; ++k) {
        oblk *l = &L[k], *f = &F[k];
        int p1 = l->p1, ps = l->ps, p2 = l->p2;
        const double *Af = k ? L[k - 1].C : NULL;
        for (int j = 0; j < p1; ++j)                                      /* :16 D = F.D/A.U */
            for (int i = 0; i < ps; ++i) l->D[IDX(i, j, ps)] = f->D[IDX(j, i, p1)];
        if (p1) rdiv_lt(ps, p1, l->D, ps, Af, p1);
        for (int j = 0; j < ps; ++j)                                      /* :17 B − D Dᵀ */
            for (int i = 0; i < ps; ++i) {
                double s = f->B[IDX(i, j, ps)];
                for (int q = 0; q < p1; ++q) s -= l->D[IDX(i, q, ps)] * l->D[IDX(j, q, ps)];
                l->B[IDX(i, j, ps)] = s;
            }
        if (ps) { int st = potrf_lower(ps, l->B, ps); if (st && !info) info = k + 1; } /* :17-18 */
        for (int j = 0; j < p1; ++j)                                      /* :19 F = F.F/A.U */
            for (int i = 0; i < p2; ++i) l->F[IDX(i, j, p2)] = f->F[IDX(j, i, p1)];
        if (p1) rdiv_lt(p2, p1, l->F, p2, Af, p1);
        for (int j = 0; j < ps; ++j)                                      /* :20 (E − F Dᵀ)/B.U */
            for (int i = 0; i < p2; ++i) {
                double s = f->E[IDX(j, i, ps)];
                for (int q = 0; q < p1; ++q) s -= l->F[IDX(i, q, p2)] * l->D[IDX(j, q, ps)];
                l->E[IDX(i, j, p2)] = s;
            }
        if (ps) rdiv_lt(p2, ps, l->E, p2, l->B, ps);
        for (int j = 0; j < p2; ++j)                                      /* :21 C − FFᵀ − EEᵀ */
            for (int i = 0; i < p2; ++i) {
                double s = f->C[IDX(i, j, p2)];
                for (int q = 0; q < p1; ++q) s -= l->F[IDX(i, q, p2)] * l->F[IDX(j, q, p2)];
                for (int q = 0; q < ps; ++q) s -= l->E[IDX(i, q, p2)] * l->E[IDX(j, q, p2)];
                l->C[IDX(i, j, p2)] = s;
            }
        if (p2) { int st = potrf_lower(p2, l->C, p2); if (st && !info) info = k + 1; } /* :21-22 */
        memcpy(l->c, f->c, (size_t)ps * sizeof(double));                 /* :23-24 */
        memcpy(l->d, f->d, (size_t)p2 * sizeof(double));
    }

    /* forward substitution, lower blocks (commented text :146-156) */
    for (int k = 0; k < N; ++k) {
        oblk *l = &L[k];
        int p1 = l->p1, ps = l->ps, p2 = l->p2;
        const double *lp = k ? L[k - 1].lam : NULL;
        for (int i = 0; i < ps; ++i) {                                    /* μ = B\(c − Dλ) */
            double s = l->c[i];
            for (int q = 0; q < p1 && k; ++q) s -= l->D[IDX(i, q, ps)] * lp[q];
            l->mu[i] = s;
        }
        if (ps) trsv_l(ps, l->B, ps, l->mu, 0);
        for (int i = 0; i < p2; ++i) {                                    /* λ = C\(d − Fλ − Eμ) */
            double s = l->d[i];
            for (int q = 0; q < p1 && k; ++q) s -= l->F[IDX(i, q, p2)] * lp[q];
            for (int q = 0; q < ps; ++q) s -= l->E[IDX(i, q, p2)] * l->mu[q];
            l->lam[i] = s;
        }
        if (p2) trsv_l(p2, l->C, p2, l->lam, 0);
    }
    size_t ol = 0;
    for (int k = 0; k < N; ++k) {
        if (yv) {
            for (int i = 0; i < L[k].ps; ++i) yv[ol + i] = L[k].mu[i];
            for (int i = 0; i < L[k].p2; ++i) yv[ol + L[k].ps + i] = L[k].lam[i];
        }
        ol += (size_t)L[k].ps + L[k].p2;
    }
    /* backward substitution, lower blocks (commented text :158-168) */
    for (int k = N - 1; k >= 0; --k) {
        oblk *l = &L[k];
        int ps = l->ps, p2 = l->p2;
        if (k < N - 1) {
            oblk *nx = &L[k + 1];                                         /* Lprev = L[k+1] */
            for (int i = 0; i < p2; ++i) {                                /* λ −= D'μ' + F'λ' */
                double s = l->lam[i];
                for (int q = 0; q < nx->ps; ++q) s -= nx->D[IDX(q, i, nx->ps)] * nx->mu[q];
                for (int q = 0; q < nx->p2; ++q) s -= nx->F[IDX(q, i, nx->p2)] * nx->lam[q];
                l->lam[i] = s;
            }
            if (p2) trsv_l(p2, l->C, p2, l->lam, 1);
            for (int i = 0; i < ps; ++i) {                                /* μ −= E'λ */
                double s = l->mu[i];
                for (int q = 0; q < p2; ++q) s -= l->E[IDX(q, i, p2)] * l->lam[q];
                l->mu[i] = s;
            }
        } else if (p2) {
            trsv_l(p2, l->C, p2, l->lam, 1);       /* a terminal p2 > 0 (not a reference shape) */
            for (int i = 0; i < ps; ++i) {
                double s = l->mu[i];
                for (int q = 0; q < p2; ++q) s -= l->E[IDX(q, i, p2)] * l->lam[q];
                l->mu[i] = s;
            }
        }
        if (ps) trsv_l(ps, l->B, ps, l->mu, 1);
    }

    /* dense L and x (copy_block!, lower storage :181-195) */
    if (Ld) memset(Ld, 0, Ptot * Ptot * sizeof(double));
    size_t off = 0;
    ol = 0;
    for (int k = 0; k < N; ++k) {
        oblk *l = &L[k];
        int p1 = l->p1, ps = l->ps, p2 = l->p2;
        size_t b1 = off, bs = off + p1, b2 = off + p1 + ps;
        if (Ld) {
#define PUTL(blk, r0, c0, nr, nc)                                                        \
    for (int j = 0; j < (nc); ++j)                                                      \
        for (int i = 0; i < (nr); ++i) Ld[IDX((r0) + i, (c0) + j, Ptot)] = (blk)[IDX(i, j, (nr))];
            PUTL(l->B, bs, bs, ps, ps); PUTL(l->C, b2, b2, p2, p2);
            PUTL(l->D, bs, b1, ps, p1); PUTL(l->E, b2, bs, p2, ps); PUTL(l->F, b2, b1, p2, p1);
#undef PUTL
        }
        if (xv) {
            for (int i = 0; i < ps; ++i) xv[ol + i] = l->mu[i];
            for (int i = 0; i < p2; ++i) xv[ol + ps + i] = l->lam[i];
        }
        ol += (size_t)ps + p2;
        off += (size_t)p1 + ps;
    }
    kkt_work_free(N, &kw);
    free_blocks(N, F); free_blocks(N, L); free(F); free(L);
    return info;
}

/* Batched KKT driver: every trajectory has the same block structure. */
int64_t oracle_kkt_solve_batch(int N, const int *n1, const int *p, const int *n2, const int *w,
                               int64_t batch, const double *Y, const double *y, int h_mode,
                               const double *H, const double *g, int ginv, double *dz,
                               double *lam, int32_t *info, int nthreads)
{
    size_t sY = 0, sy = 0, sH = 0, sg = 0, sl = 0;
    for (int k = 0; k < N; ++k) {
        sY += (size_t)(n1[k] + p[k] + n2[k]) * w[k];
        sy += (size_t)p[k] + n2[k];
        sH += (h_mode == 2) ? (size_t)w[k] : (size_t)w[k] * w[k];
        sg += (size_t)w[k];
        sl += (size_t)p[k] + n2[k];
    }
    int64_t bad = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads) reduction(+ : bad)
#endif
    for (int64_t b = 0; b < batch; ++b) {
        int st = oracle_kkt_solve_one(N, n1, p, n2, w, Y + b * sY, y + b * sy, h_mode,
                                      H + b * sH, g + b * sg, ginv, dz + b * sg, lam + b * sl,
                                      NULL, NULL, NULL);
        if (info) info[b] = st;
        bad += (st != 0);
    }
    (void)nthreads;
    return bad;
}
