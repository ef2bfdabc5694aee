/*
 * san_main.c — sanitizer driver for the CPU oracle (TEST INFRASTRUCTURE ONLY; SURVEY §5
 * "race detection / sanitizers").  Built by `make -C oracle asan` with
 * -fsanitize=address,undefined together with lqr_oracle.c and run by
 * tests/test_sanitizers.py: every oracle entry point is driven over small problems (DP
 * time-invariant / time-varying, P_1 / all P_k; KKT upper solve in the three H modes, both
 * Ginv variants, with the dense debug outputs; the lower-storage variant), so an
 * out-of-bounds access, use-after-free, leak or undefined operation aborts the run.
 * A numerical self-check (lower solve x = −λ of the upper solve) guards against a
 * sanitizer build that silently computes garbage.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int64_t oracle_dp_solve_batch_tv(int n, int m, int N, int64_t batch, const double *A,
                                 const double *B, const double *Q, const double *R,
                                 const double *Qf, const double *x0, double *K, double *P,
                                 int p_all, double *X, double *U, int32_t *info, int nthreads,
                                 int tvAB, int tvQR);
int oracle_kkt_solve_one(int N, const int *n1, const int *p, const int *n2, const int *w,
                         const double *Y, const double *y, int h_mode, const double *H,
                         const double *g, int ginv, double *dz, double *lam, double *Sd,
                         double *Ud, double *rd);
int oracle_kkt_lower_one(int N, const int *n1, const int *p, const int *n2, const int *w,
                         const double *Y, const double *y, int h_mode, const double *H,
                         const double *g, int ginv, double *Ld, double *yv, double *xv);

static uint64_t rs = 0x9e3779b97f4a7c15ull;
static double urand(void)
{
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return (double)(rs >> 11) * (1.0 / 9007199254740992.0) - 0.5;
}
static double *vec(size_t k)
{
    double *v = malloc((k ? k : 1) * sizeof(double));
    for (size_t i = 0; i < k; ++i) v[i] = urand();
    return v;
}
/* SPD n×n (col-major) = I·s + GᵀG/n */
static void spd(int n, double s, double *M)
{
    double *G = vec((size_t)n * n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double a = 0.0;
            for (int q = 0; q < n; ++q) a += G[q + i * n] * G[q + j * n];
            M[i + j * n] = a / n + (i == j ? s : 0.0);
        }
    free(G);
}

static int run_dp(int n, int m, int N, int bt, int tv, int p_all)
{
    const size_t kk = tv ? (size_t)(N - 1) : 1, nn = (size_t)n * n;
    double *A = vec(nn * kk * bt), *B = vec((size_t)n * m * kk * bt);
    double *Q = malloc(nn * kk * bt * sizeof(double)), *R = malloc((size_t)m * m * kk * bt * sizeof(double));
    double *Qf = malloc(nn * bt * sizeof(double)), *x0 = vec((size_t)n * bt);
    for (size_t i = 0; i < nn * kk * bt; ++i) A[i] = 0.2 * A[i] + ((i % nn) % (n + 1) == 0 ? 1.0 : 0.0);
    for (size_t t = 0; t < kk * bt; ++t) { spd(n, 1.0, Q + t * nn); spd(m, 1.0, R + t * m * m); }
    for (int t = 0; t < bt; ++t) spd(n, 10.0, Qf + t * nn);
    double *K = calloc((size_t)m * n * (N - 1) * bt, sizeof(double));
    double *P = calloc(nn * (p_all ? N : 1) * bt, sizeof(double));
    double *X = calloc((size_t)n * N * bt, sizeof(double)), *U = calloc((size_t)m * (N - 1) * bt, sizeof(double));
    int32_t *info = calloc(bt, sizeof(int32_t));
    int64_t bad = oracle_dp_solve_batch_tv(n, m, N, bt, A, B, Q, R, Qf, x0, K, P, p_all, X, U, info, 2,
                                           tv, tv);
    int fin = 1;
    for (size_t i = 0; i < (size_t)n * N * bt; ++i) fin &= isfinite(X[i]) != 0;
    free(A); free(B); free(Q); free(R); free(Qf); free(x0); free(K); free(P); free(X); free(U); free(info);
    if (bad || !fin) { fprintf(stderr, "dp n=%d m=%d N=%d tv=%d: bad=%ld finite=%d\n", n, m, N, tv, (long)bad, fin); return 1; }
    return 0;
}

static int run_kkt(int nx, int nu, int N, int h_mode)
{
    int *n1 = malloc(N * sizeof(int)), *p = malloc(N * sizeof(int)), *n2 = malloc(N * sizeof(int)),
        *w = malloc(N * sizeof(int));
    size_t sY = 0, sy = 0, sH = 0, sg = 0, P = 0;
    for (int k = 0; k < N; ++k) {
        n1[k] = k ? nx : 0;
        n2[k] = k < N - 1 ? nx : 0;
        p[k] = (k == 0 || k == N - 1) ? nx : (k % 3 == 1);      /* a stage row on some knots */
        w[k] = k < N - 1 ? nx + nu : nx;
        const int rows = n1[k] + p[k] + n2[k];
        sY += (size_t)rows * w[k]; sy += (size_t)p[k] + n2[k];
        sH += h_mode == 2 ? (size_t)w[k] : (size_t)w[k] * w[k]; sg += (size_t)w[k];
    }
    P = sy;
    double *Y = vec(sY), *y = vec(sy), *g = vec(sg), *H = malloc(sH * sizeof(double));
    size_t oH = 0;
    for (int k = 0; k < N; ++k) {
        if (h_mode == 2) { for (int i = 0; i < w[k]; ++i) H[oH + i] = 1.0 + fabs(urand()); oH += w[k]; }
        else {
            spd(w[k], 1.0, H + oH);
            if (h_mode == 1)                                    /* block-diagonal Q, R */
                for (int j = 0; j < w[k]; ++j)
                    for (int i = 0; i < w[k]; ++i)
                        if ((i < nx) != (j < nx)) H[oH + i + (size_t)j * w[k]] = 0.0;
            oH += (size_t)w[k] * w[k];
        }
    }
    int err = 0;
    for (int ginv = 0; ginv <= 1; ++ginv) {
        double *dz = calloc(sg, sizeof(double)), *lam = calloc(P, sizeof(double));
        double *S = calloc(P * P, sizeof(double)), *Ud = calloc(P * P, sizeof(double)), *r = calloc(P, sizeof(double));
        double *L = calloc(P * P, sizeof(double)), *yv = calloc(P, sizeof(double)), *xv = calloc(P, sizeof(double));
        int iu = oracle_kkt_solve_one(N, n1, p, n2, w, Y, y, h_mode, H, g, ginv, dz, lam, S, Ud, r);
        int il = oracle_kkt_lower_one(N, n1, p, n2, w, Y, y, h_mode, H, g, ginv, L, yv, xv);
        double e = 0.0, sc = 1e-300;
        for (size_t i = 0; i < P; ++i) { e = fmax(e, fabs(xv[i] + lam[i])); sc = fmax(sc, fabs(lam[i])); }
        if (iu || il || !(e <= 1e-9 * sc)) {
            fprintf(stderr, "kkt N=%d h=%d ginv=%d: info %d/%d, lower-vs-upper %.3e\n", N, h_mode, ginv, iu, il, e / sc);
            err = 1;
        }
        free(dz); free(lam); free(S); free(Ud); free(r); free(L); free(yv); free(xv);
    }
    free(Y); free(y); free(g); free(H); free(n1); free(p); free(n2); free(w);
    return err;
}

int main(void)
{
    int err = 0;
    err |= run_dp(4, 1, 12, 3, 0, 0);
    err |= run_dp(6, 3, 9, 2, 0, 1);
    err |= run_dp(5, 2, 7, 3, 1, 1);
    err |= run_dp(1, 1, 2, 1, 0, 0);
    for (int h = 0; h <= 2; ++h) {
        err |= run_kkt(3, 2, 11, h);
        err |= run_kkt(2, 1, 4, h);
    }
    printf(err ? "oracle sanitizer run: FAILED\n" : "oracle sanitizer run: ok\n");
    return err;
}
