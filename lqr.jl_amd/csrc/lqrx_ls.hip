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
// which is ĀᵀĀ summed by row blocks (a prefix sum along each block diagonal, below);
// H is stored packed (upper triangle); the Cholesky is right-looking over LDS columns, the triangular solves one column per
// barrier.  Bound: the Nm-step
// Cholesky / substitution barrier chain; one workgroup per CU when H is large.  Ā and b̄ can be written out
// (optional) for a direct buildAb! parity check.
#include "lqrx_internal.h"
#include "lqrx_tile.h"
#include <math.h>
#include <algorithm>

namespace lqrx {

namespace {

constexpr int LS_THREADS = 256;
constexpr int LS_REG = 16;     // register fast paths (buildAb!, rollout!) for n, m ≤ 16, nm + n ≤ 64
constexpr int LS_MAX_NM = 192; // (N−1)·m with H in LDS: a packed triangle (Nm(Nm+1)/2 doubles);
                               // the LDS budget (≤ 163840 B, validate_ls) binds at Nm = 192
constexpr int LS_BIG_MAX_NM = 1024; // H in global scratch (the "big" path): blocked factor
constexpr int LS_PB = 16;           // big path: max panel rows factored in LDS per pass (the host
                                    // halves it until the panel fits the LDS budget)
constexpr size_t LS_LDS_CAP = 163840;
#ifndef LQRX_LS_PNL
#define LQRX_LS_PNL 4
#endif
constexpr int LS_PNL = LQRX_LS_PNL;  // LDS path: potrf panel rows per barrier pair

// order one wave's LDS accesses across lanes (a wave executes LDS ops in order; this stops
// the compiler from moving them across and waits for the writes)
__device__ inline void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// element j of a wave-distributed vector (lane l, slot s ↔ index l + 64 s), j wave-uniform.
// Every slot is read out by readlane and the scalar results selected: selecting the slot
// first made the compiler index the array dynamically (through scratch).
__device__ inline double readlane_d(double v, int lane)
{
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)bits, lane);
    const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int S>
__device__ inline double bcast_slot(const double (&v)[S], int j)
{
    double sel = readlane_d(v[0], j & 63);
#pragma unroll
    for (int s = 1; s < S; ++s) {
        const double r = readlane_d(v[s], j & 63);
        sel = (j >> 6) == s ? r : sel;
    }
    return sel;
}

struct LsLayout {
    int n, m, N, K, Nm, Nn;
    // LDS offsets in doubles
    int oSq, oSf, oHu, oA, oB, oPl, oW, oVq, oVf, obb, oH, oy, odi, oX, oFlag, oPan, total;
};

// big = H in global scratch: the LDS keeps only the staging space for Q, Qf, R in place of
// H, plus a panel of LS_PB rows for the blocked factor
__host__ __device__ inline LsLayout ls_layout(int n, int m, int N, bool big = false, int pb = LS_PB)
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
    L.oX = L.obb;   // X (rollout) reuses b̄'s space: b̄ is dead once y = −Āᵀb̄ is formed
    L.oH = o;  // also stages Q, Qf, R for the small factorisations
    const int hp = big ? 0 : L.Nm * (L.Nm + 1) / 2;   // packed upper triangle, rows contiguous
    o += hp > 2 * n * n + m * m ? hp : 2 * n * n + m * m;
    L.oy = o; o += L.Nm;
    L.odi = o; o += L.Nm;   // 1/U_jj of the factor (potrs multiplies instead of dividing)
    L.oFlag = o; o += 1;
    L.oPan = o; o += big ? pb * L.Nm : 0;
    L.total = o;
    return L;
}

// packed upper-triangular index of (i, k), i ≤ k, rows stored contiguously (row i holds
// columns i..Nm−1 and starts at Σ_{r<i} (Nm − r))
__device__ inline int rbase(int i, int Nm) { return i * Nm - ((i * (i - 1)) >> 1) - i; }  // + k
__device__ inline int up(int i, int k, int Nm) { return rbase(i, Nm) + k; }

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

// A failed trajectory (Q/Qf/R not SPD, or a non-positive pivot of H) gets NaN in U and X
// — never uninitialised memory — and its info code; the reference throws there
// (cholesky / potrf!).  Called by every thread of the workgroup (uniform early return).
__device__ void ls_fail(double *gU, double *gX, int32_t *ginfo, int64_t b, int n, int m, int N, int code)
{
    const double qnan = __builtin_nan("");
    const int nu = (N - 1) * m, nx = N * n;
    for (int i = threadIdx.x; i < nu; i += LS_THREADS) gU[b * nu + i] = qnan;
    for (int i = threadIdx.x; i < nx; i += LS_THREADS) gX[b * nx + i] = qnan;
    if (threadIdx.x == 0 && ginfo) ginfo[b] = code;
}

// BIG = false: the whole problem in LDS (Nm ≤ 192).  BIG = true: H = ĀᵀĀ + Hu lives in a
// per-trajectory global scratch block (packed, rows contiguous: gH + b·Nm(Nm+1)/2), built by
// the same code, factored by a blocked right-looking Cholesky (LS_PB-row panels factored in
// LDS, one trailing update of the remaining rows per panel), solved by the same potrs —
// the reference's own LS test problem (test/least_squares.jl: DoubleIntegrator(), Nm = 300)
// takes this path.
template <bool BIG>
__global__ void __launch_bounds__(LS_THREADS)
ls_condensed_kernel(const double *__restrict__ gA, const double *__restrict__ gB, const double *__restrict__ gQ,
                    const double *__restrict__ gR, const double *__restrict__ gQf, const double *__restrict__ gx0,
                    double *__restrict__ gU, double *__restrict__ gX, int32_t *__restrict__ ginfo,
                    double *__restrict__ gAb, double *__restrict__ gbb, int n, int m, int N, int hu_mode,
                    double *__restrict__ gH, int pb, int64_t b0)
{
    extern __shared__ double lds[];
    const LsLayout L = ls_layout(n, m, N, BIG, pb);
    const int K = L.K, Nm = L.Nm, tid = threadIdx.x;
    const int64_t b = b0 + blockIdx.x;
    double *Sq = lds + L.oSq, *Sf = lds + L.oSf, *Hu = lds + L.oHu, *A = lds + L.oA, *B = lds + L.oB;
    double *Pl = lds + L.oPl, *W = lds + L.oW, *Vq = lds + L.oVq, *Vf = lds + L.oVf, *bb = lds + L.obb;
    double *y = lds + L.oy, *X = lds + L.oX, *dinv = lds + L.odi;
    // big path: the scratch holds one chunk of the batch (blocks b0 .. b0 + gridDim.x − 1)
    double *H = BIG ? gH + (b - b0) * ((int64_t)Nm * (Nm + 1) / 2) : lds + L.oH;
    int *flag = (int *)(lds + L.oFlag);
    const int nn = n * n, nm = n * m, mm = m * m;

    // ---- inputs: A, B, x0 into LDS; Q, Qf, R staged in H's LDS space for the factorisations
    double *tQ = lds + L.oH, *tQf = tQ + nn, *tR = tQ + 2 * nn;
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
        ls_fail(gU, gX, ginfo, b, n, m, N, -1);
        return;
    }

    // ---- buildAb! :70-101: powers P_l = A^l B, w_r = A^r x0; V_q, V_f and b̄ = S_r w_r
    // a serial chain of K+1 tiny steps: wave 0 alone, wave-level ordering instead of barriers
    const bool regpath = n <= LS_REG && m <= LS_REG && nm + n <= 64;
    if (tid < 64 && regpath) {
        // register form: lane e < nm holds P_l[i,a] (e = i + a·n), lane nm + i holds w_l[i];
        // each step gathers the lane's column by n shuffles, no LDS round trips or fences
        const int e = tid;
        const bool isP = e < nm, isW = e >= nm && e < nm + n;
        const int ea = isP ? e : (isW ? e - nm : 0), i = ea % n, a = isP ? ea / n : 0;
        const int src0 = isP ? a * n : nm;
        double Ar[LS_REG], Sqr[LS_REG], Sfr[LS_REG];
#pragma unroll
        for (int j = 0; j < LS_REG; ++j) {
            const bool ok = (isP || isW) && j < n;
            Ar[j] = ok ? A[i + j * n] : 0.0;
            Sqr[j] = ok && j >= i ? Sq[i + j * n] : 0.0;
            Sfr[j] = ok && j >= i ? Sf[i + j * n] : 0.0;
        }
        double v = isP ? B[ea] : (isW ? W[ea] : 0.0);
        for (int l = 0; l <= K; ++l) {
            double col[LS_REG];
#pragma unroll
            for (int j = 0; j < LS_REG; ++j) col[j] = j < n ? __shfl(v, src0 + j) : 0.0;
            double vq = 0.0, vf = 0.0, nx = 0.0;
#pragma unroll
            for (int j = 0; j < LS_REG; ++j) {
                vq = fma(Sqr[j], col[j], vq);
                vf = fma(Sfr[j], col[j], vf);
                nx = fma(Ar[j], col[j], nx);
            }
            if (isW) bb[l * n + i] = l < K ? vq : vf;          // b̄ block l (:71-80)
            if (isP) {                                        // Ā blocks (:90-96)
                if (l < K - 1) Vq[l * nm + ea] = vq;
                if (l < K) Vf[l * nm + ea] = vf;
            }
            v = nx;                                           // next power (:101)
        }
    }
    if (tid < 64 && !regpath) {
        for (int i = tid; i < nm; i += 64) Pl[i] = B[i];
        wave_sync();
        for (int l = 0; l <= K; ++l) {
            const double *P = Pl + (l & 1) * nm, *w = W + (l & 1) * n;
            double *Pn = Pl + ((l + 1) & 1) * nm, *wn = W + ((l + 1) & 1) * n;
            // b̄ row block l: S_l·A^l·x0 (S = Sf for the last block, :71-75)
            const double *S = l < K ? Sq : Sf;
            for (int i = tid; i < n; i += 64) {
                double v = 0.0;
                for (int j = i; j < n; ++j) v = fma(S[i + j * n], w[j], v);
                bb[l * n + i] = v;
            }
            for (int e = tid; e < 2 * nm; e += 64) {
                const int which = e / nm, ea = e - which * nm, i = ea % n, a = ea / n;
                if (l >= K || (which == 0 && l >= K - 1)) continue;
                const double *S2 = which ? Sf : Sq;
                double v = 0.0;
                for (int j = i; j < n; ++j) v = fma(S2[i + j * n], P[j + a * n], v);
                (which ? Vf : Vq)[l * nm + ea] = v;
            }
            // next powers (:101): P_{l+1} = A·P_l, w_{l+1} = A·w_l
            for (int e = tid; e < nm + n; e += 64) {
                const bool isw = e >= nm;
                const int ea = isw ? e - nm : e, i = ea % n, a = ea / n;
                const double *src = isw ? w : P + a * n;
                double v = 0.0;
                for (int j = 0; j < n; ++j) v = fma(A[i + j * n], src[j], v);
                if (isw) wn[i] = v; else Pn[ea] = v;
            }
            wave_sync();
        }
    }
    __syncthreads();

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

    // ---- H = ĀᵀĀ + Hu (:171-172), upper triangle (potrf 'U' reads no other).  Along a block
    // diagonal d = c2 − c1 the Q-rows part is a prefix sum: with s = r−1−c2,
    //   H_q(c1, c2) = Σ_{s=0}^{K−2−c2} V_q[s+d]ᵀ V_q[s]
    // so one thread per (d, a1, a2) scans s upward and emits H(c2−d, c2) for c2 = K−2−s —
    // O(K²nm²) instead of the O(K³nm²) of a dense ĀᵀĀ (same sum, accumulated in s order).
    for (int e = tid; e < K * mm; e += LS_THREADS) {
        const int d = e / mm, a12 = e - d * mm, a1 = a12 % m, a2 = a12 / m;
        if (d == 0 && a1 > a2) continue;
        const double hu = d == 0 ? Hu[a1 + a2 * m] : 0.0;
        auto emit = [&](int c2, double q) {
            const int c1 = c2 - d;
            const double *f1 = Vf + (K - 1 - c1) * nm + a1 * n, *f2 = Vf + (K - 1 - c2) * nm + a2 * n;
            double v = q;
            for (int i = 0; i < n; ++i) v = fma(f1[i], f2[i], v);
            H[up(c1 * m + a1, c2 * m + a2, Nm)] = v + hu;
        };
        if (K - 1 - d >= 0) emit(K - 1, 0.0);          // last control: Qf row only
        double acc = 0.0;
        for (int s2 = 0; s2 <= K - 2 - d; ++s2) {
            const double *v1 = Vq + (s2 + d) * nm + a1 * n, *v2 = Vq + s2 * nm + a2 * n;
            for (int i = 0; i < n; ++i) acc = fma(v1[i], v2[i], acc);
            emit(K - 2 - s2, acc);
        }
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

    const int wave = tid >> 6, lane = tid & 63;
    if constexpr (BIG) {
    // ---- potrf 'U' (:181), big path: blocked right-looking over LS_PB-row panels.  A panel
    // (rows r0..r0+pr−1, columns r0..Nm−1 of the upper triangle) is brought to LDS, factored
    // there (one barrier per pivot, rows scaled to U as each pivot completes), written back,
    // and the trailing rows get one update H[i,k] −= Σ_u U[u,i]·U[u,k] per panel — global
    // read-modify-writes once per panel instead of once per pivot.
    double *Pn = lds + L.oPan;
    for (int r0 = 0; r0 < Nm; r0 += pb) {
        const int pr = Nm - r0 < pb ? Nm - r0 : pb, w = Nm - r0;
        for (int e = tid; e < pr * w; e += LS_THREADS) {
            const int u = e / w, c = e - u * w;
            Pn[e] = c >= u ? H[rbase(r0 + u, Nm) + r0 + c] : 0.0;
        }
        __syncthreads();
        for (int u = 0; u < pr; ++u) {
            const double d = Pn[u * w + u];
            if (!(d > 0.0)) {   // uniform: every thread reads the same LDS word
                ls_fail(gU, gX, ginfo, b, n, m, N, r0 + u + 1);
                return;
            }
            const double ri = rsqrt_nr(d);
            // every thread has read the pivot before tid 0 overwrites it with sqrt(d): a lagging
            // wave (columns u + 64 and up) must not see the scaled value
            __syncthreads();
            for (int c = u + tid; c < w; c += LS_THREADS) Pn[u * w + c] = c == u ? d * ri : Pn[u * w + c] * ri;
            if (tid == 0) dinv[r0 + u] = ri;
            __syncthreads();
            for (int v = u + 1 + wave; v < pr; v += LS_THREADS / 64) {
                const double uv = Pn[u * w + v];
                for (int c = v + lane; c < w; c += 64) Pn[v * w + c] = fma(-uv, Pn[u * w + c], Pn[v * w + c]);
            }
            __syncthreads();
        }
        for (int e = tid; e < pr * w; e += LS_THREADS) {
            const int u = e / w, c = e - u * w;
            if (c >= u) H[rbase(r0 + u, Nm) + r0 + c] = Pn[e];
        }
        for (int i = r0 + pr + wave; i < Nm; i += LS_THREADS / 64) {
            double ui[LS_PB];
#pragma unroll
            for (int u = 0; u < LS_PB; ++u) ui[u] = u < pr ? Pn[u * w + (i - r0)] : 0.0;
            const int ri0 = rbase(i, Nm);
            for (int k = i + lane; k < Nm; k += 64) {
                double v = H[ri0 + k];
#pragma unroll
                for (int u = 0; u < LS_PB; ++u)
                    if (u < pr) v = fma(-ui[u], Pn[u * w + (k - r0)], v);
                H[ri0 + k] = v;
            }
        }
        __syncthreads();
    }
    } else {
    // ---- potrf 'U' (:181): blocked right-looking with LS_PNL-row panels and one-panel
    // lookahead, one barrier per panel instead of one per pivot.  While waves 1..3 apply panel
    // p's rank-pr update H[i,k] −= Σ_u U[u,i]·U[u,k] (u in pivot order) to the trailing rows
    // past panel p+1 (4 rows per wave pass sharing each loaded panel column, lanes over
    // columns), wave 0 applies it to panel p+1's rows and factors that panel (pivot by pivot,
    // rows scaled to U at once, in-panel updates; wave-level ordering only).  info = first
    // non-positive pivot.
    auto factor_panel = [&](int j0, int pr) {           // wave 0 only
        for (int u = 0; u < pr; ++u) {
            const int j = j0 + u, rj = rbase(j, Nm);
            const double d = H[rj + j];
            if (!(d > 0.0)) {      // wave-uniform: every lane reads the same LDS word
                if (lane == 0) *flag = j + 1;
                return;
            }
            const double rd = rsqrt_nr(d);
            for (int k = j + 1 + lane; k < Nm; k += 64) H[rj + k] *= rd;
            if (lane == 0) {
                H[rj + j] = d * rd;
                dinv[j] = rd;
            }
            wave_sync();
            for (int v = j + 1; v < j0 + pr; ++v) {
                const double ujv = H[rj + v];
                const int rv = rbase(v, Nm);
                for (int k = v + lane; k < Nm; k += 64) H[rv + k] = fma(-ujv, H[rj + k], H[rv + k]);
            }
            wave_sync();
        }
    };
    // rows [ia, Nm) −= panel (rows j0..j0+pr−1), by nw waves starting at wave w0; rows ≥ ib skipped
    auto rank_update = [&](int j0, int pr, int ia, int ib, int w0, int nw) {
        int rp[LS_PNL];
#pragma unroll
        for (int u = 0; u < LS_PNL; ++u) rp[u] = u < pr ? rbase(j0 + u, Nm) : 0;
        for (int i0 = ia + 4 * (wave - w0); i0 < ib; i0 += 4 * nw) {
            double ui[4][LS_PNL];
            int rb[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool ok = i0 + q < ib;
                rb[q] = ok ? rbase(i0 + q, Nm) : 0;
#pragma unroll
                for (int u = 0; u < LS_PNL; ++u) ui[q][u] = (ok && u < pr) ? H[rp[u] + i0 + q] : 0.0;
            }
            for (int k = i0 + lane; k < Nm; k += 64) {
                double hp[LS_PNL];
#pragma unroll
                for (int u = 0; u < LS_PNL; ++u) hp[u] = u < pr ? H[rp[u] + k] : 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (i0 + q < ib && i0 + q <= k) {
                        double v = H[rb[q] + k];
#pragma unroll
                        for (int u = 0; u < LS_PNL; ++u) v = fma(-ui[q][u], hp[u], v);
                        H[rb[q] + k] = v;
                    }
            }
        }
    };
    if (wave == 0) factor_panel(0, Nm < LS_PNL ? Nm : LS_PNL);
    __syncthreads();
    for (int j0 = 0; j0 < Nm; j0 += LS_PNL) {
        if (*flag) {            // uniform
            ls_fail(gU, gX, ginfo, b, n, m, N, *flag);
            return;
        }
        const int pr = Nm - j0 < LS_PNL ? Nm - j0 : LS_PNL, n0 = j0 + pr;
        if (n0 >= Nm) break;
        const int pr2 = Nm - n0 < LS_PNL ? Nm - n0 : LS_PNL;
        if (wave == 0) {
            rank_update(j0, pr, n0, n0 + pr2, 0, 1);
            wave_sync();
            factor_panel(n0, pr2);
        } else {
            rank_update(j0, pr, n0 + pr2, Nm, 1, LS_THREADS / 64 - 1);
        }
        __syncthreads();
    }
    }
    // ---- potrs 'U' (:182): Uᵀz = y, then U x = z — wave 0, y held in registers (lane l owns
    // y[l + 64 s]), the pivot broadcast by readlane: no barriers in the 2·Nm-step chain
    if (tid < 64) {
        constexpr int S = (BIG ? LS_BIG_MAX_NM : LS_MAX_NM) / 64;
        double yr[S];
#pragma unroll
        for (int s2 = 0; s2 < S; ++s2) {
            const int idx = lane + 64 * s2;
            yr[s2] = idx < Nm ? y[idx] : 0.0;
        }
        for (int j = 0; j < Nm; ++j) {
            const double zj = bcast_slot<S>(yr, j) * dinv[j];
#pragma unroll
            for (int s2 = 0; s2 < S; ++s2) {
                const int idx = lane + 64 * s2;
                if (idx > j && idx < Nm) yr[s2] = fma(-H[up(j, idx, Nm)], zj, yr[s2]);
                else if (idx == j) yr[s2] = zj;
            }
        }
        for (int j = Nm - 1; j >= 0; --j) {
            const double xj = bcast_slot<S>(yr, j) * dinv[j];
#pragma unroll
            for (int s2 = 0; s2 < S; ++s2) {
                const int idx = lane + 64 * s2;
                if (idx < j) yr[s2] = fma(-H[up(idx, j, Nm)], xj, yr[s2]);
                else if (idx == j) yr[s2] = xj;
            }
        }
#pragma unroll
        for (int s2 = 0; s2 < S; ++s2) {
            const int idx = lane + 64 * s2;
            if (idx < Nm) y[idx] = yr[s2];
        }
        wave_sync();
    }
    // ---- rollout! (:197-202), one wave (n ≤ 64 lanes per row sweep)
    if (tid < 64 && regpath) {
        // lane i < n holds x_k[i]; x_k gathered by readlane (uniform j), u_k read from LDS
        const bool ok = tid < n;
        double Ar[LS_REG], Br[LS_REG];
#pragma unroll
        for (int j = 0; j < LS_REG; ++j) {
            Ar[j] = ok && j < n ? A[tid + j * n] : 0.0;
            Br[j] = ok && j < m ? B[tid + j * n] : 0.0;
        }
        double x = ok ? gx0[b * n + tid] : 0.0;
        if (ok) X[tid] = x;
        for (int k = 0; k < K; ++k) {
            double v = 0.0;
#pragma unroll
            for (int j = 0; j < LS_REG; ++j)
                if (j < n) v = fma(Ar[j], readlane_d(x, j), v);
#pragma unroll
            for (int c = 0; c < LS_REG; ++c)
                if (c < m) v = fma(Br[c], y[k * m + c], v);
            x = v;
            if (ok) X[(k + 1) * n + tid] = x;
        }
    }
    if (tid < 64 && !regpath) {
        for (int i = tid; i < n; i += 64) X[i] = gx0[b * n + i];
        wave_sync();
        for (int k = 0; k < K; ++k) {
            const double *xk = X + k * n, *uk = y + k * m;
            for (int i = tid; i < n; i += 64) {
                double v = 0.0;
                for (int j = 0; j < n; ++j) v = fma(A[i + j * n], xk[j], v);
                for (int a = 0; a < m; ++a) v = fma(B[i + a * n], uk[a], v);
                X[(k + 1) * n + i] = v;
            }
            wave_sync();
        }
    }
    __syncthreads();
    for (int i = tid; i < Nm; i += LS_THREADS) gU[b * Nm + i] = y[i];
    for (int i = tid; i < L.Nn; i += LS_THREADS) gX[b * L.Nn + i] = X[i];
    if (tid == 0 && ginfo) ginfo[b] = 0;
}

} // namespace

// the big path (H in global scratch) serves what the LDS-resident kernel cannot hold
bool ls_big(int n, int m, int N)
{
    const LsLayout L = ls_layout(n, m, N);
    return L.Nm > LS_MAX_NM || (size_t)L.total * sizeof(double) > LS_LDS_CAP;
}
// big path panel rows: the widest of 16, 8, 4, 2 whose panel fits the LDS budget
int ls_panel(int n, int m, int N)
{
    int pb = LS_PB;
    while (pb > 2 && (size_t)ls_layout(n, m, N, true, pb).total * sizeof(double) > LS_LDS_CAP) pb /= 2;
    return pb;
}

size_t ls_lds_bytes(int n, int m, int N)
{
    const bool big = ls_big(n, m, N);
    return (size_t)ls_layout(n, m, N, big, big ? ls_panel(n, m, N) : LS_PB).total * sizeof(double);
}

int ls_max_nm() { return LS_BIG_MAX_NM; }

hipError_t ls_launch(const LsArgs &a, hipStream_t s)
{
    const bool big = ls_big(a.n, a.m, a.N);
    const size_t lds = ls_lds_bytes(a.n, a.m, a.N);
    const void *fn = big ? (const void *)ls_condensed_kernel<true> : (const void *)ls_condensed_kernel<false>;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // one workgroup per trajectory; the grid dimension is capped at 2^31−1 by the ABI check
    if (!big) {
        hipLaunchKernelGGL(ls_condensed_kernel<false>, dim3((unsigned)a.batch), dim3(LS_THREADS), lds, s, a.A, a.B,
                           a.Q, a.R, a.Qf, a.x0, a.U, a.X, a.info, a.Ab, a.bb, a.n, a.m, a.N, a.hu_mode, nullptr, LS_PB,
                           (int64_t)0);
        return hipGetLastError();
    }
    // big path: packed H per trajectory in one stream-ordered scratch block of at most 4 GiB,
    // reused by consecutive chunks of the batch in stream order (as dp_big_launch does)
    const int Nm = (a.N - 1) * a.m;
    const size_t per = ((size_t)Nm * (Nm + 1) / 2) * sizeof(double);
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(a.batch, (int64_t)((size_t(4) << 30) / per)));
    Scratch sc;
    e = scratch_alloc(&sc.p, (size_t)chunk * per, s);
    if (e != hipSuccess) return e;
    sc.owned = true;
    const int pb = ls_panel(a.n, a.m, a.N);
    for (int64_t b0 = 0; b0 < a.batch && e == hipSuccess; b0 += chunk) {
        const int64_t nb = std::min<int64_t>(chunk, a.batch - b0);
        hipLaunchKernelGGL(ls_condensed_kernel<true>, dim3((unsigned)nb), dim3(LS_THREADS), lds, s, a.A, a.B, a.Q,
                           a.R, a.Qf, a.x0, a.U, a.X, a.info, a.Ab, a.bb, a.n, a.m, a.N, a.hu_mode, (double *)sc.p, pb,
                           b0);
        e = hipGetLastError();
    }
    hipError_t ef = sc.release(s);
    return e != hipSuccess ? e : ef;
}

} // namespace lqrx
