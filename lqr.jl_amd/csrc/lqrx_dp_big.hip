// lqrx_dp_big.hip — batched Riccati backward pass + rollout for shapes past the register-tiled
// kernels (n > 64 or m > 32, up to 512 each): the reference's DP handles any (n, m)
// (/root/reference/src/dynamic_programming.jl:54-72), so the drop-in does too.
//
// Mapping: ONE 256-THREAD WORKGROUP PER TRAJECTORY; the knot's matrices live in a per-
// trajectory global scratch block (L2-resident working set: 3n² + 2nm + m² elements); the
// element-wise parts are spread over the workgroup one element per thread-iteration (column-major
// order, so consecutive threads touch consecutive rows).  The reference's own sequence of
// products is kept — PB = P·B, E = R + BᵀPB, PA = P·A, K = BᵀPA, potrf 'U', potrs, APB = AᵀPB,
// P_ = Q + AᵀPA − APB·K (no symmetric fast form) — the products on fp64/fp32 MFMA tiles (wg_mm:
// the 4 waves take output tiles round-robin and stream strided operand tiles from L2), the factor
// and the triangular solves blocked by 16 with their updates on MFMA too (lqrx_wg.h), the rollout
// on the VALU.
// Time-varying knot strides, all-P output, linear cost terms (d, p) as in the other kernels.
#include "lqrx_internal.h"
#include "lqrx_tile.h"
#include "lqrx_wg.h"
#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace lqrx {

namespace {

using wg::BT;
using wg::Mat;


template <typename T>
__global__ __launch_bounds__(BT) void dp_big_kernel(const DpArgs a, T *__restrict__ ws, size_t ws_elems, int64_t b0)
{
    const int64_t b = b0 + blockIdx.x;                          // trajectory; scratch slot blockIdx.x
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

    T *w0 = ws + (size_t)blockIdx.x * ws_elems;
    T *P = w0, *Pn = P + nn, *PA = Pn + nn, *PB = PA + nn, *APB = PB + nm, *E = APB + nm;
    T *pv = E + mm, *pn = pv + n, *wv = pn + n;
    T *Kb = (T *)a.K + (size_t)b * (size_t)(N - 1) * nm;
    T *Pall = a.p_all ? (T *)a.P + (size_t)b * nn * N : nullptr;
    T *db = lin ? (T *)a.d + (size_t)b * (size_t)(N - 1) * m : nullptr;
    T *pall = (lin && a.p_all) ? (T *)a.p + (size_t)b * (size_t)N * n : nullptr;
    __shared__ int s_info;
    // E (m×m) lives in LDS when it fits (m ≤ 64): the factor's pivot chain and the triangular
    // solves read it m² times in dependent order — L2 latency per read otherwise
    constexpr int EL = 64;
    __shared__ T Es[EL * EL];
    if (m <= EL) E = Es;

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
        const Mat<T> Pt{P, (size_t)n, 1}, Am{A, 1, (size_t)n}, Bm{B, 1, (size_t)n}, none{nullptr, 0, 0};
        // :38 PB = P*B  (= (Pᵀ)ᵀ·B) ; :40 PA = P*A
        wg::wg_mm<T, 1, 1>(PB, n, n, m, nullptr, Pt, Bm, n, none, none, 0, tid);
        wg::wg_mm<T, 1, 1>(PA, n, n, n, nullptr, Pt, Am, n, none, none, 0, tid);
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
        const Mat<T> PBm{PB, 1, (size_t)n}, PAm{PA, 1, (size_t)n};
        wg::wg_mm<T, 1, 1>(E, m, m, m, R, Bm, PBm, n, none, none, 0, tid);
        wg::wg_mm<T, 1, 1>(K, m, m, n, nullptr, Bm, PAm, n, none, none, 0, tid);
        wg::wg_mm<T, 1, 1>(APB, n, n, m, nullptr, Am, PBm, n, none, none, 0, tid);
        __syncthreads();
        // :29 potrf!('U', E) — blocked left-looking (lqrx_wg.h); a failed pivot stops the factor
        // (as LAPACK) and reports this knot
        const int f = wg::wg_potrf<T>(E, m, m, tid);
        if (f && tid == 0 && s_info == 0) s_info = k;
        // :30 potrs!('U', E, K): K ← E⁻¹K by two blocked triangular solves; the linear terms'
        // w is one more right-hand side (d, written to its output)
        if (lin)
            for (int i = tid; i < m; i += BT) db[(size_t)(k - 1) * m + i] = wv[i];
        __syncthreads();
        wg::wg_trsm_ut<T>(E, m, m, K, m, n, tid);
        wg::wg_trsm_un<T>(E, m, m, K, m, n, tid);
        if (lin) {
            T *x = db + (size_t)(k - 1) * m;
            wg::wg_trsm_ut<T>(E, m, m, x, m, 1, tid);
            wg::wg_trsm_un<T>(E, m, m, x, m, 1, tid);
        }
        // :51 P_ = Q + A'PA − APB*K  (APB·K = (APBᵀ)ᵀ·K)   (and p_ = q + A'p − APB*d)
        {
            const Mat<T> APBt{APB, (size_t)n, 1}, Km{K, 1, (size_t)m};
            wg::wg_mm<T, 1, -1>(Pn, n, n, n, Q, Am, PAm, n, APBt, Km, m, tid);
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
    // the batch in chunks whose scratch stays ≤ 4 GiB (n = m = 512: 12.6 MB per trajectory);
    // the chunks reuse one stream-ordered block, in stream order
    const int64_t per = (int64_t)(elems * es);
    int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(a.batch, ((int64_t)4 << 30) / per));
    if (const char *ev = std::getenv("LQRX_DP_BIG_CHUNK"))   // tests: force the multi-chunk path
        chunk = std::max<int64_t>(1, std::min<int64_t>(chunk, std::atoll(ev)));
    void *ws = nullptr;
    hipError_t e = scratch_alloc(&ws, (size_t)per * (size_t)chunk, s);
    if (e != hipSuccess) return e;
    for (int64_t b0 = 0; b0 < a.batch && e == hipSuccess; b0 += chunk) {
        dim3 grid((unsigned)std::min<int64_t>(chunk, a.batch - b0)), block(BT);
        if (a.dtype == 0)
            hipLaunchKernelGGL((dp_big_kernel<double>), grid, block, 0, s, a, (double *)ws, elems, b0);
        else
            hipLaunchKernelGGL((dp_big_kernel<float>), grid, block, 0, s, a, (float *)ws, elems, b0);
        e = hipGetLastError();
    }
    hipError_t ef = scratch_free(ws, s);
    return e != hipSuccess ? e : ef;
}

} // namespace lqrx
