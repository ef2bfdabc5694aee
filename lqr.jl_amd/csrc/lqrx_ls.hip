// lqrx_ls.hip — batched condensed least-squares LQR.
//
// Restates LeastSquaresSolver (/root/reference/src/least_squares.jl) on the device, one
// 256-thread workgroup per trajectory with the whole per-trajectory problem in LDS:
//   LeastSquaresSolver(prob) :30-56   Sq = chol(Q).U, Sf = chol(Qf).U, Sr = chol(R).U
//   buildAb!(solver, prob)   :58-103  Ā[block r, block c] = S_r A^{r−1−c} B (r > c),
//                                     b̄[block r] = S_r A^r x0 (S_r = Sf for the last row)
//   solve!                   :158-183 H = ĀᵀĀ + Hu, y = −Āᵀb̄, potrf 'U' + potrs 'U'
//   rollout!                 :197-202 X_1 = x0, X_{k+1} = A X_k + B U_k
// Hu (hu_mode): 0 = zero (a fresh solver, matbuild :Ab — no control cost), 1 = chol(R).U
// blocks (after build_least_squares!, :121), 2 = R blocks (the LQR cost; extension).
//
// Ā is never materialised: with V_q[l] = Sq·A^l·B (l ≤ K−2) and V_f[l] = Sf·A^l·B
// (l ≤ K−1), K = N−1 controls,
//   H[(c1,a),(c2,b)] = Σ_{r=max(c1,c2)+1}^{K−1} (V_q[r−1−c1]ᵀ V_q[r−1−c2])_{ab}
//                      + (V_f[K−1−c1]ᵀ V_f[K−1−c2])_{ab}
// which is ĀᵀĀ summed by row blocks, one element of H's upper triangle per thread-iteration;
// the Cholesky is right-looking over LDS columns, the triangular solves one column per
// barrier.  Bound: LDS bandwidth of the
// O(K³n m²/3) ĀᵀĀ sum; one workgroup per CU when H is large.  Ā and b̄ can be written out
// (optional) for a direct buildAb! parity check.
#include "lqrx_internal.h"
#include <math.h>

namespace lqrx {

namespace {

constexpr int LS_THREADS = 256;

struct LsLayout {
    int n, m, N, K, Nm, Nn;
    // LDS offsets in doubles
    int oSq, oSf, oHu, oA, oB, oPl, oW, oVq, oVf, obb, oH, oy, oX, oFlag, total;
};

__host__ __device__ inline LsLayout ls_layout(int n, int m, int N)
{
    LsLayout L;
    L.n = n; L.m = m; L.N = N; L.K = N - 1; L.Nm = L.K * m; L.Nn = N * n;
    int o = 0;
    L.oSq = o; o += n * n;
    L.oSf = o; o += n * n;
    L.oHu = o; o += m * m;
    L.oA = o; o += n * n;
    L.oB = o; o += n * m;
    L.oPl = o; o += 2 * n * m;              // ping-pong A^l B
    L.oW = o; o += 2 * n;                   // ping-pong A^l x0
    L.oVq = o; o += (L.K > 1 ? L.K - 1 : 1) * n * m;
    L.oVf = o; o += L.K * n * m;
    L.obb = o; o += N * n;
    L.oH = o;  // also stages Q, Qf, R for the small factorisations
    o += L.Nm * L.Nm > 2 * n * n + m * m ? L.Nm * L.Nm : 2 * n * n + m * m;
    L.oy = o; o += L.Nm;
    L.oX = o; o += N * n;
    L.oFlag = o; o += 1;
    L.total = o;
    return L;
}

// upper Cholesky of a small s×s column-major matrix in LDS (thread 0 only); returns false
// when a pivot is not positive (cholesky() throws PosDefException there, :50-52)
__device__ bool small_chol_u(const double *M, double *U, int s)
{
    for (int j = 0; j < s; ++j)
        for (int i = 0; i < s; ++i) U[i + j * s] = i <= j ? M[i + j * s] : 0.0;
    for (int j = 0; j < s; ++j) {
        double d = U[j + j * s];
        for (int k = 0; k < j; ++k) d -= U[k + j * s] * U[k + j * s];
        if (!(d > 0.0)) return false;
        d = sqrt(d);
        U[j + j * s] = d;
        for (int c = j + 1; c < s; ++c) {
            double v = U[j + c * s];
            for (int k = 0; k < j; ++k) v -= U[k + j * s] * U[k + c * s];
            U[j + c * s] = v / d;
        }
    }
    return true;
}

__global__ void __launch_bounds__(LS_THREADS)
ls_condensed_kernel(const double *__restrict__ gA, const double *__restrict__ gB, const double *__restrict__ gQ,
                    const double *__restrict__ gR, const double *__restrict__ gQf, const double *__restrict__ gx0,
                    double *__restrict__ gU, double *__restrict__ gX, int32_t *__restrict__ ginfo,
                    double *__restrict__ gAb, double *__restrict__ gbb, int n, int m, int N, int hu_mode)
{
    extern __shared__ double lds[];
    const LsLayout L = ls_layout(n, m, N);
    const int K = L.K, Nm = L.Nm, tid = threadIdx.x;
    const int64_t b = blockIdx.x;
    double *Sq = lds + L.oSq, *Sf = lds + L.oSf, *Hu = lds + L.oHu, *A = lds + L.oA, *B = lds + L.oB;
    double *Pl = lds + L.oPl, *W = lds + L.oW, *Vq = lds + L.oVq, *Vf = lds + L.oVf, *bb = lds + L.obb;
    double *H = lds + L.oH, *y = lds + L.oy, *X = lds + L.oX;
    int *flag = (int *)(lds + L.oFlag);
    const int nn = n * n, nm = n * m, mm = m * m;

    // ---- inputs: A, B, x0 into LDS; Q, Qf, R staged in H's space for the factorisations
    double *tQ = H, *tQf = H + nn, *tR = H + 2 * nn;
    for (int i = tid; i < nn; i += LS_THREADS) {
        A[i] = gA[b * nn + i];
        tQ[i] = gQ[b * nn + i];
        tQf[i] = gQf[b * nn + i];
    }
    for (int i = tid; i < nm; i += LS_THREADS) B[i] = gB[b * nm + i];
    for (int i = tid; i < mm; i += LS_THREADS) tR[i] = gR[b * mm + i];
    for (int i = tid; i < n; i += LS_THREADS) W[i] = gx0[b * n + i];
    __syncthreads();
    // ---- LeastSquaresSolver(prob) :50-52: Sq, Sf (and Sr) by cholesky(·).U
    if (tid == 0) {
        bool ok = small_chol_u(tQ, Sq, n) && small_chol_u(tQf, Sf, n);
        if (hu_mode == 1) ok = ok && small_chol_u(tR, Hu, m);
        else if (hu_mode == 2) for (int i = 0; i < mm; ++i) Hu[i] = tR[i];
        else for (int i = 0; i < mm; ++i) Hu[i] = 0.0;
        *flag = ok ? 0 : -1;
    }
    __syncthreads();
    if (*flag) {
        if (tid == 0 && ginfo) ginfo[b] = -1;
        return;
    }

    // ---- buildAb! :70-101: powers P_l = A^l B, w_r = A^r x0; V_q, V_f and b̄ = S_r w_r
    for (int i = tid; i < nm; i += LS_THREADS) Pl[i] = B[i];
    __syncthreads();
    for (int l = 0; l <= K; ++l) {
        const double *P = Pl + (l & 1) * nm, *w = W + (l & 1) * n;
        double *Pn = Pl + ((l + 1) & 1) * nm, *wn = W + ((l + 1) & 1) * n;
        // b̄ row block l: S_l·A^l·x0 (S = Sf for the last block, :71-75)
        const double *S = l < K ? Sq : Sf;
        for (int i = tid; i < n; i += LS_THREADS) {
            double v = 0.0;
            for (int j = i; j < n; ++j) v = fma(S[i + j * n], w[j], v);
            bb[l * n + i] = v;
        }
        for (int e = tid; e < 2 * nm; e += LS_THREADS) {
            const int which = e / nm, ea = e - which * nm, i = ea % n, a = ea / n;
            if (l >= K || (which == 0 && l >= K - 1)) continue;
            const double *S2 = which ? Sf : Sq;
            double v = 0.0;
            for (int j = i; j < n; ++j) v = fma(S2[i + j * n], P[j + a * n], v);
            (which ? Vf : Vq)[l * nm + ea] = v;
        }
        // next powers (:101): P_{l+1} = A·P_l, w_{l+1} = A·w_l
        for (int e = tid; e < nm + n; e += LS_THREADS) {
            const bool isw = e >= nm;
            const int ea = isw ? e - nm : e, i = ea % n, a = ea / n;
            const double *src = isw ? w : P + a * n;
            double v = 0.0;
            for (int j = 0; j < n; ++j) v = fma(A[i + j * n], src[j], v);
            if (isw) wn[i] = v; else Pn[ea] = v;
        }
        __syncthreads();
    }

    // optional outputs: Ā (Nn×Nm col-major) and b̄, as buildAb! leaves them
    if (gAb) {
        const int64_t sz = (int64_t)L.Nn * Nm;
        double *dst = gAb + b * sz;
        for (int64_t e = tid; e < sz; e += LS_THREADS) {
            const int row = (int)(e % L.Nn), col = (int)(e / L.Nn);
            const int r = row / n, i = row - r * n, c = col / m, a = col - c * m;
            double v = 0.0;
            if (r > c) {
                const int l = r - 1 - c;
                v = r < K ? Vq[l * nm + i + a * n] : Vf[l * nm + i + a * n];
            }
            dst[e] = v;
        }
    }
    if (gbb)
        for (int e = tid; e < L.Nn; e += LS_THREADS) gbb[b * L.Nn + e] = bb[e];

    // ---- H = ĀᵀĀ + Hu (:171-172), upper triangle (potrf 'U' reads no other), one element
    // per thread-iteration, consecutive threads down a column
    const int ntri = Nm * (Nm + 1) / 2;
    for (int t = tid; t < ntri; t += LS_THREADS) {
        int q = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
        while (q * (q + 1) / 2 > t) --q;
        while ((q + 1) * (q + 2) / 2 <= t) ++q;
        const int p = t - q * (q + 1) / 2;
        const int c1 = p / m, a1 = p - c1 * m, c2 = q / m, a2 = q - c2 * m;
        const int r0 = (c1 > c2 ? c1 : c2) + 1;
        double v = 0.0;
        for (int r = r0; r < K; ++r) {
            const double *v1 = Vq + (r - 1 - c1) * nm + a1 * n;
            const double *v2 = Vq + (r - 1 - c2) * nm + a2 * n;
            for (int i = 0; i < n; ++i) v = fma(v1[i], v2[i], v);
        }
        const double *f1 = Vf + (K - 1 - c1) * nm + a1 * n;
        const double *f2 = Vf + (K - 1 - c2) * nm + a2 * n;
        for (int i = 0; i < n; ++i) v = fma(f1[i], f2[i], v);
        if (c1 == c2) v += Hu[a1 + a2 * m];
        H[p + q * Nm] = v;
    }
    // y = −Āᵀb̄ (:173): y[(c,a)] = −Σ_{r>c} (S_r A^{r−1−c} B)ᵀ_a · b̄_r
    for (int pidx = tid; pidx < Nm; pidx += LS_THREADS) {
        const int c = pidx / m, a = pidx - c * m;
        double v = 0.0;
        for (int r = c + 1; r <= K; ++r) {
            const double *vv = (r < K ? Vq : Vf) + (r - 1 - c) * nm + a * n;
            const double *br = bb + r * n;
            for (int i = 0; i < n; ++i) v = fma(vv[i], br[i], v);
        }
        y[pidx] = -v;
    }
    if (tid == 0) *flag = 0;
    __syncthreads();

    // ---- potrf 'U' (:181): right-looking over columns; info = first non-positive pivot
    for (int j = 0; j < Nm; ++j) {
        const double d = H[j + j * Nm];
        if (!(d > 0.0)) {   // uniform: every thread reads the same LDS word
            if (tid == 0 && ginfo) ginfo[b] = j + 1;
            return;
        }
        const double rd = 1.0 / sqrt(d);
        // scale row j right of the diagonal, then the trailing update of the upper triangle
        for (int k = j + 1 + tid; k < Nm; k += LS_THREADS) H[j + k * Nm] *= rd;
        __syncthreads();
        if (tid == 0) H[j + j * Nm] = d * rd;
        const int tr = Nm - j - 1, ntr = tr * (tr + 1) / 2;
        for (int t = tid; t < ntr; t += LS_THREADS) {
            int kk = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
            while (kk * (kk + 1) / 2 > t) --kk;
            while ((kk + 1) * (kk + 2) / 2 <= t) ++kk;
            const int ii = t - kk * (kk + 1) / 2;
            const int i = j + 1 + ii, k = j + 1 + kk;
            H[i + k * Nm] = fma(-H[j + i * Nm], H[j + k * Nm], H[i + k * Nm]);
        }
        __syncthreads();
    }
    // ---- potrs 'U' (:182): Uᵀz = y, then U x = z
    for (int j = 0; j < Nm; ++j) {
        const double zj = y[j] / H[j + j * Nm];
        for (int k = j + 1 + tid; k < Nm; k += LS_THREADS) y[k] = fma(-H[j + k * Nm], zj, y[k]);
        __syncthreads();
        if (tid == 0) y[j] = zj;
    }
    __syncthreads();
    for (int j = Nm - 1; j >= 0; --j) {
        const double xj = y[j] / H[j + j * Nm];
        for (int i = tid; i < j; i += LS_THREADS) y[i] = fma(-H[i + j * Nm], xj, y[i]);
        __syncthreads();
        if (tid == 0) y[j] = xj;
    }
    __syncthreads();
    // ---- rollout! (:197-202), one wave (n ≤ 64 lanes per row sweep)
    if (tid < 64) {
        for (int i = tid; i < n; i += 64) X[i] = gx0[b * n + i];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        for (int k = 0; k < K; ++k) {
            const double *xk = X + k * n, *uk = y + k * m;
            for (int i = tid; i < n; i += 64) {
                double v = 0.0;
                for (int j = 0; j < n; ++j) v = fma(A[i + j * n], xk[j], v);
                for (int a = 0; a < m; ++a) v = fma(B[i + a * n], uk[a], v);
                X[(k + 1) * n + i] = v;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
    }
    __syncthreads();
    for (int i = tid; i < Nm; i += LS_THREADS) gU[b * Nm + i] = y[i];
    for (int i = tid; i < L.Nn; i += LS_THREADS) gX[b * L.Nn + i] = X[i];
    if (tid == 0 && ginfo) ginfo[b] = 0;
}

} // namespace

size_t ls_lds_bytes(int n, int m, int N)
{
    return (size_t)ls_layout(n, m, N).total * sizeof(double);
}

hipError_t ls_launch(const LsArgs &a, hipStream_t s)
{
    const size_t lds = ls_lds_bytes(a.n, a.m, a.N);
    hipError_t e = hipFuncSetAttribute((const void *)ls_condensed_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // one workgroup per trajectory; the grid dimension is capped at 2^31−1 by the ABI check
    hipLaunchKernelGGL(ls_condensed_kernel, dim3((unsigned)a.batch), dim3(LS_THREADS), lds, s, a.A, a.B, a.Q,
                       a.R, a.Qf, a.x0, a.U, a.X, a.info, a.Ab, a.bb, a.n, a.m, a.N, a.hu_mode);
    return hipGetLastError();
}

} // namespace lqrx
