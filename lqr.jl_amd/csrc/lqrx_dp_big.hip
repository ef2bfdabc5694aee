// lqrx_dp_big.hip — batched Riccati backward pass + rollout for shapes past the register-tiled
// kernels (n > 64 or m > 32, up to 512 each): the reference's DP handles any (n, m)
// (/root/reference/src/dynamic_programming.jl:54-72), so the drop-in does too.
//
// Mapping: ONE 256-THREAD WORKGROUP PER TRAJECTORY; the knot's matrices live in a per-
// trajectory global scratch block (L2-resident working set: 3n² + 2nm + m² elements) and every
// product is spread over the workgroup one output element per thread-iteration (column-major
// order, so consecutive threads touch consecutive rows).  The reference's own op order is kept
// step for step — PB = P·B, E = R + BᵀPB, PA = P·A, K = BᵀPA, potrf 'U' (left-looking, as
// dpotf2), potrs, APB = AᵀPB, P_ = Q + AᵀPA − APB·K — so the results track the oracle to
// rounding (no symmetric fast form).  fp64 VALU has the MFMA peak on gfx950; this path is
// bandwidth/latency-bound on L2 and exists for coverage, not speed.
// Time-varying knot strides, all-P output, linear cost terms (d, p) as in the other kernels.
#include "lqrx_internal.h"
#include <cmath>

namespace lqrx {

namespace {

constexpr int BT = 256;

template <typename T> __device__ __forceinline__ T dsqrt(T x) { return sqrt(x); }

template <typename T>
__global__ __launch_bounds__(BT) void dp_big_kernel(const DpArgs a, T *__restrict__ ws, size_t ws_elems)
{
    const int64_t b = blockIdx.x;
    if (b >= a.batch) return;
    const int tid = threadIdx.x;
    const int n = a.n, m = a.m, N = a.N;
    const size_t nn = (size_t)n * n, nm = (size_t)n * m, mm = (size_t)m * m;
    const size_t kAB = a.tv_AB ? (size_t)(N - 1) : 1, kQR = a.tv_QR ? (size_t)(N - 1) : 1;
    const size_t sA = a.tv_AB ? nn : 0, sB = a.tv_AB ? nm : 0, sQ = a.tv_QR ? nn : 0, sR = a.tv_QR ? mm : 0;
    const T *A0 = (const T *)a.A + b * nn * kAB, *B0 = (const T *)a.B + b * nm * kAB;
    const T *Q0 = (const T *)a.Q + b * nn * kQR, *R0 = (const T *)a.R + b * mm * kQR;
    const bool lin = a.lin != 0;
    const size_t sq = a.tv_QR ? (size_t)n : 0, sr = a.tv_QR ? (size_t)m : 0;

    T *w0 = ws + (size_t)b * ws_elems;
    T *P = w0, *Pn = P + nn, *PA = Pn + nn, *PB = PA + nn, *APB = PB + nm, *E = APB + nm;
    T *pv = E + mm, *pn = pv + n, *wv = pn + n;
    T *Kb = (T *)a.K + (size_t)b * (size_t)(N - 1) * nm;
    T *Pall = a.p_all ? (T *)a.P + (size_t)b * nn * N : nullptr;
    T *db = lin ? (T *)a.d + (size_t)b * (size_t)(N - 1) * m : nullptr;
    T *pall = (lin && a.p_all) ? (T *)a.p + (size_t)b * (size_t)N * n : nullptr;
    __shared__ int s_info;

    const T *Qf = (const T *)a.Qf + b * nn;
    for (size_t e = tid; e < nn; e += BT) {                     // :58 P .= Qf
        P[e] = Qf[e];
        if (Pall) Pall[(size_t)(N - 1) * nn + e] = Qf[e];
    }
    if (lin) {
        const T *qf = (const T *)a.qf + b * n;
        for (int i = tid; i < n; i += BT) {
            pv[i] = qf[i];
            if (pall) pall[(size_t)(N - 1) * n + i] = qf[i];
        }
    }
    if (tid == 0) s_info = 0;
    __syncthreads();

    for (int k = N - 1; k >= 1; --k) {                          // :61
        const T *A = A0 + (size_t)(k - 1) * sA, *B = B0 + (size_t)(k - 1) * sB;
        const T *Q = Q0 + (size_t)(k - 1) * sQ, *R = R0 + (size_t)(k - 1) * sR;
        T *K = Kb + (size_t)(k - 1) * nm;
        // :38 PB = P*B
        for (size_t e = tid; e < nm; e += BT) {
            const int i = (int)(e % n), c = (int)(e / n);
            T s = 0;
            for (int l = 0; l < n; ++l) s += P[i + (size_t)l * n] * B[l + (size_t)c * n];
            PB[e] = s;
        }
        // :40 PA = P*A
        for (size_t e = tid; e < nn; e += BT) {
            const int i = (int)(e % n), j = (int)(e / n);
            T s = 0;
            for (int l = 0; l < n; ++l) s += P[i + (size_t)l * n] * A[l + (size_t)j * n];
            PA[e] = s;
        }
        if (lin) {                                              // w = r + B'p
            const T *r = (const T *)a.r + b * m * kQR + (size_t)(k - 1) * sr;
            for (int c = tid; c < m; c += BT) {
                T s = 0;
                for (int l = 0; l < n; ++l) s += B[l + (size_t)c * n] * pv[l];
                wv[c] = r[c] + s;
            }
        }
        __syncthreads();
        // :39 E = R + B'PB ; :41 K = B'PA ; :50 APB = A'PB
        for (size_t e = tid; e < mm; e += BT) {
            const int c = (int)(e % m), d = (int)(e / m);
            T s = 0;
            for (int l = 0; l < n; ++l) s += B[l + (size_t)c * n] * PB[l + (size_t)d * n];
            E[e] = R[e] + s;
        }
        for (size_t e = tid; e < nm; e += BT) {
            const int c = (int)(e % m), j = (int)(e / m);
            T s = 0;
            for (int l = 0; l < n; ++l) s += B[l + (size_t)c * n] * PA[l + (size_t)j * n];
            K[e] = s;
        }
        for (size_t e = tid; e < nm; e += BT) {
            const int i = (int)(e % n), c = (int)(e / n);
            T s = 0;
            for (int l = 0; l < n; ++l) s += A[l + (size_t)i * n] * PB[l + (size_t)c * n];
            APB[e] = s;
        }
        __syncthreads();
        // :29 potrf!('U', E) — left-looking dpotf2; a failed pivot stops the factor (as LAPACK)
        bool failed = false;
        for (int j = 0; j < m; ++j) {
            T dj = E[j + (size_t)j * m];
            for (int p = 0; p < j; ++p) dj -= E[p + (size_t)j * m] * E[p + (size_t)j * m];
            if (!(dj > (T)0)) {
                failed = true;                                  // uniform: every thread saw the same dj
                if (tid == 0) {
                    E[j + (size_t)j * m] = dj;
                    if (s_info == 0) s_info = k;
                }
                break;
            }
            dj = dsqrt(dj);
            for (int c = j + 1 + tid; c < m; c += BT) {
                T s = E[j + (size_t)c * m];
                for (int p = 0; p < j; ++p) s -= E[p + (size_t)j * m] * E[p + (size_t)c * m];
                E[j + (size_t)c * m] = s / dj;
            }
            __syncthreads();
            if (tid == 0) E[j + (size_t)j * m] = dj;
            __syncthreads();
        }
        (void)failed;
        __syncthreads();
        // :30 potrs!('U', E, K) — one column per thread (Uᵀy = K[:,j], then U x = y); the linear
        // terms' w is one more column (d, written to its output)
        for (int j = tid; j < n + (lin ? 1 : 0); j += BT) {
            T *x = j < n ? K + (size_t)j * m : db + (size_t)(k - 1) * m;
            if (j == n) {
                for (int i = 0; i < m; ++i) x[i] = wv[i];
            }
            for (int i = 0; i < m; ++i) {
                T s = x[i];
                for (int p = 0; p < i; ++p) s -= E[p + (size_t)i * m] * x[p];
                x[i] = s / E[i + (size_t)i * m];
            }
            for (int i = m - 1; i >= 0; --i) {
                T s = x[i];
                for (int p = i + 1; p < m; ++p) s -= E[i + (size_t)p * m] * x[p];
                x[i] = s / E[i + (size_t)i * m];
            }
        }
        __syncthreads();
        // :51 P_ = Q + A'PA − APB*K   (and p_ = q + A'p − APB*d)
        for (size_t e = tid; e < nn; e += BT) {
            const int i = (int)(e % n), j = (int)(e / n);
            T s1 = 0, s2 = 0;
            for (int l = 0; l < n; ++l) s1 += A[l + (size_t)i * n] * PA[l + (size_t)j * n];
            for (int c = 0; c < m; ++c) s2 += APB[i + (size_t)c * n] * K[c + (size_t)j * m];
            Pn[e] = Q[e] + s1 - s2;
        }
        if (lin) {
            const T *q = (const T *)a.q + b * n * kQR + (size_t)(k - 1) * sq;
            const T *dk = db + (size_t)(k - 1) * m;
            for (int i = tid; i < n; i += BT) {
                T s1 = 0, s2 = 0;
                for (int l = 0; l < n; ++l) s1 += A[l + (size_t)i * n] * pv[l];
                for (int c = 0; c < m; ++c) s2 += APB[i + (size_t)c * n] * dk[c];
                pn[i] = q[i] + s1 - s2;
            }
        }
        __syncthreads();
        // :63 P .= P_
        { T *t = P; P = Pn; Pn = t; }
        if (lin) { T *t = pv; pv = pn; pn = t; }
        if (Pall) {
            for (size_t e = tid; e < nn; e += BT) Pall[(size_t)(k - 1) * nn + e] = P[e];
        }
        if (pall) {
            for (int i = tid; i < n; i += BT) pall[(size_t)(k - 1) * n + i] = pv[i];
        }
    }
    if (!a.p_all) {
        for (size_t e = tid; e < nn; e += BT) ((T *)a.P)[(size_t)b * nn + e] = P[e];
        if (lin) {
            for (int i = tid; i < n; i += BT) ((T *)a.p)[(size_t)b * n + i] = pv[i];
        }
    }
    __syncthreads();
    if (tid == 0 && a.info) a.info[b] = s_info;

    // :66-70 rollout  u_k = −K_k x_k (− d_k),  x_{k+1} = A x_k + B u_k
    T *X = (T *)a.X + (size_t)b * (size_t)N * n, *U = (T *)a.U + (size_t)b * (size_t)(N - 1) * m;
    const T *x0 = (const T *)a.x0 + b * n;
    for (int i = tid; i < n; i += BT) X[i] = x0[i];
    __syncthreads();
    for (int k = 1; k <= N - 1; ++k) {
        const T *A = A0 + (size_t)(k - 1) * sA, *B = B0 + (size_t)(k - 1) * sB;
        const T *K = Kb + (size_t)(k - 1) * nm, *x = X + (size_t)(k - 1) * n;
        T *u = U + (size_t)(k - 1) * m;
        for (int c = tid; c < m; c += BT) {
            T s = 0;
            for (int j = 0; j < n; ++j) s += K[c + (size_t)j * m] * x[j];
            u[c] = lin ? -(s + db[(size_t)(k - 1) * m + c]) : -s;
        }
        __syncthreads();
        T *xn = X + (size_t)k * n;
        for (int i = tid; i < n; i += BT) {
            T s = 0, t = 0;
            for (int j = 0; j < n; ++j) s += A[i + (size_t)j * n] * x[j];
            for (int j = 0; j < m; ++j) t += B[i + (size_t)j * n] * u[j];
            xn[i] = s + t;
        }
        __syncthreads();
    }
}

} // namespace

bool dp_big_supported(int n, int m) { return n >= 1 && m >= 1 && n <= 512 && m <= 512; }

hipError_t dp_big_launch(const DpArgs &a, hipStream_t s)
{
    if (!dp_big_supported(a.n, a.m)) return hipErrorNotSupported;
    const size_t n = a.n, m = a.m;
    const size_t elems = 3 * n * n + 2 * n * m + m * m + 2 * n + m;   // P, P_, PA, PB, APB, E, p, p_, w
    const size_t es = a.dtype == 0 ? 8 : 4;
    void *ws = nullptr;
    hipError_t e = scratch_alloc(&ws, elems * es * (size_t)a.batch, s);
    if (e != hipSuccess) return e;
    dim3 grid((unsigned)a.batch), block(BT);
    if (a.dtype == 0)
        hipLaunchKernelGGL((dp_big_kernel<double>), grid, block, 0, s, a, (double *)ws, elems);
    else
        hipLaunchKernelGGL((dp_big_kernel<float>), grid, block, 0, s, a, (float *)ws, elems);
    e = hipGetLastError();
    hipError_t ef = scratch_free(ws, s);
    return e != hipSuccess ? e : ef;
}

} // namespace lqrx
