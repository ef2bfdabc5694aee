// lqrx_kkt_wg.hip — batched block-tridiagonal KKT solve for block sizes past the large-block
// register tiles (any n1, p, n2 > 64 or w > 128, up to KW_MAX_BLOCK / KW_MAX_W): the
// reference's block Cholesky takes any block size through LAPACK/BLAS
// (/root/reference/src/cholesky_solve.jl:47-143, jacobian_blocks.jl:220-286,
// cholesky_solver.jl:166-236), so the drop-in does too.
//
// Mapping: ONE 256-THREAD WORKGROUP PER TRAJECTORY (as lqrx_dp_big.hip).  The knot's Schur
// pieces, its block-Cholesky factor and its multipliers live in a per-trajectory global
// scratch block (an L2-resident working set); products and the blocked factor / triangular
// solves run on the MFMA pipe through lqrx_wg.h.  The reference's sequence is kept:
//   forward, knot k:  H_k factor (potrf, block_cholesky.jl:55-91 — or 1/h for a diagonal H),
//                     JYt = H_k⁻¹·Y_kᵀ, r = JYtᵀ·g (jacobian_blocks.jl:231-242),
//                     the Schur pieces B C D E F and A (added into knot k−1's C, the
//                     copy_shur! alias, :249-286), c = r_C − y_c, d = r_D1 − y_d, d_{k−1} += r_D2;
//                     then knot k−1 — now complete — is factored (cholesky_solve.jl:47-67) and
//                     its forward substitution run (:93-117);
//   backward:         cholesky_solve.jl:119-143;
//   primal recovery:  δz_k = −H_k⁻¹(Y_kᵀ[λ_{k−1}; μ_k; λ_k] + g)   (cholesky_solver.jl:185-236;
//                     −Y_kᵀ[…] for the second-order correction, ginv = 0, :254-273).
// info: −(k+1) for the first knot whose H_k is not SPD, else k+1 for the first knot whose B̃
// or C̃ pivot fails (the oracle's convention, oracle/lqr_oracle.c).
//
// Scratch per knot (column-major): [D | F] (p1 × (ps+p2)), B (ps²), [E | μ] (ps × (p2+1)),
// C (p2²), λ (p2), H factor (w² or w).  Contiguous [D | F] and [E | μ] let one triangular solve
// serve both members.  Transients: JYt (maxw × maxrows) and a vector of max(maxw, maxrows).
#include "lqrx_internal.h"
#include "lqrx_tile.h"
#include "lqrx_wg.h"
#include <algorithm>
#include <cstdlib>

namespace lqrx {

namespace {

using wg::BT;
using wg::Mat;
using wg::cm;
using wg::cmt;

template <typename T> struct Knot {
    int p1, ps, p2, w, rows, oY, oy, oH, og;
    T *DF, *B, *Emu, *C, *lam, *Hf;
    __device__ T *mu() const { return Emu + (size_t)ps * p2; }
};

__device__ __forceinline__ size_t kw_knot_elems(const int32_t *m, int hm)
{
    const size_t p1 = m[0], ps = m[1], p2 = m[2], w = m[3];
    return p1 * (ps + p2) + ps * ps + ps * (p2 + 1) + p2 * p2 + p2 + (hm == 2 ? w : w * w);
}

template <typename T> __device__ __forceinline__ Knot<T> kw_knot(const int32_t *meta, int k, T *base, int hm)
{
    const int32_t *m = meta + (size_t)k * 8;
    Knot<T> K;
    K.p1 = m[0]; K.ps = m[1]; K.p2 = m[2]; K.w = m[3];
    K.rows = K.p1 + K.ps + K.p2;
    K.oY = m[4]; K.oy = m[5]; K.oH = m[6]; K.og = m[7];
    K.DF = base;
    K.B = K.DF + (size_t)K.p1 * (K.ps + K.p2);
    K.Emu = K.B + (size_t)K.ps * K.ps;
    K.C = K.Emu + (size_t)K.ps * (K.p2 + 1);
    K.lam = K.C + (size_t)K.p2 * K.p2;
    K.Hf = K.lam + K.p2;
    (void)hm;
    return K;
}

// cholesky_solve.jl:47-67 and :93-117 for knot j (its Schur pieces complete), Kp = knot j−1
// (its C factored: the A factor of this knot; its λ final from the forward sweep)
template <typename T>
__device__ void kw_factor_fwd(const Knot<T> &K, const Knot<T> *Kp, int j, int *s_finfo, int tid)
{
    const int p1 = K.p1, ps = K.ps, p2 = K.p2;
    T *mu = K.mu();
    const Mat<T> Dm = cm<T>(K.DF, p1), Fm = cm<T>(K.DF + (size_t)p1 * ps, p1);
    if (p1) {
        // :49, :57  [D | F] ← Ã⁻ᵀ[D | F]
        wg::wg_trsm_ut<T>(Kp->C, p1, p1, K.DF, p1, ps + p2, tid);
        const Mat<T> lp = cm<T>(Kp->lam, p1);
        // :50-53 B − DᵀD ; :59 E − DᵀF ; :100-105 c − Dᵀλ_{j−1}, d − Fᵀλ_{j−1}
        wg::wg_mm1<T, -1>(K.B, ps, ps, ps, K.B, Dm, Dm, p1, tid);
        wg::wg_mm1<T, -1>(K.Emu, ps, ps, p2, K.Emu, Dm, Fm, p1, tid);
        wg::wg_mm1<T, -1>(mu, ps, ps, 1, mu, Dm, lp, p1, tid);
        wg::wg_mm1<T, -1>(K.lam, p2, p2, 1, K.lam, Fm, lp, p1, tid);
        __syncthreads();
    }
    if (ps) {
        const int f = wg::wg_potrf<T>(K.B, ps, ps, tid);                // :53
        if (f && tid == 0 && *s_finfo == 0) *s_finfo = j + 1;
        wg::wg_trsm_ut<T>(K.B, ps, ps, K.Emu, ps, p2 + 1, tid);         // :60, :106 [Ẽ | μ]
    }
    if (p2) {
        // :61-62 C − FᵀF − ẼᵀẼ ; :108-112 d − Ẽᵀμ
        const Mat<T> Em = cm<T>(K.Emu, ps), mum = cm<T>(mu, ps);
        wg::wg_mm<T, -1, -1>(K.C, p2, p2, p2, K.C, Fm, Fm, p1, Em, Em, ps, tid);
        wg::wg_mm1<T, -1>(K.lam, p2, p2, 1, K.lam, Em, mum, ps, tid);
        __syncthreads();
        const int f = wg::wg_potrf<T>(K.C, p2, p2, tid);                // :62
        if (f && tid == 0 && *s_finfo == 0) *s_finfo = j + 1;
        wg::wg_trsm_ut<T>(K.C, p2, p2, K.lam, p2, 1, tid);              // :113 C̃⁻ᵀ
    }
}

template <typename T>
__global__ __launch_bounds__(BT) void kkt_wg_kernel(const KktArgs a, T *__restrict__ ws, size_t ws_elems, int64_t b0)
{
    const int64_t b = b0 + blockIdx.x;          // trajectory; scratch slot blockIdx.x
    if (b >= a.batch) return;
    const int tid = threadIdx.x, N = a.N, hm = a.h_mode;
    const bool ginv = a.ginv != 0;
    const T *Yb = (const T *)a.Y + b * a.sY, *yb = (const T *)a.y + b * a.sy;
    const T *Hb = (const T *)a.H + b * a.sH, *gb = (const T *)a.g + b * a.sg;
    T *dzb = (T *)a.dz + b * a.sg, *lamb = (T *)a.lam + b * a.sl;
    T *w0 = ws + (size_t)blockIdx.x * ws_elems;
    T *JYt = w0, *vt = JYt + (size_t)a.maxw * a.maxrows, *per = vt + std::max(a.maxw, a.maxrows);
    __shared__ int s_hinfo, s_finfo;
    if (tid == 0) { s_hinfo = 0; s_finfo = 0; }
    __syncthreads();

    // ---- forward: Schur pieces of knot k, then factor + forward substitution of knot k−1
    size_t off = 0, offp = 0, offpp = 0;   // bases of knots k, k−1, k−2
    for (int k = 0; k <= N; ++k) {
        Knot<T> K{}, Kp{};
        if (k > 0) Kp = kw_knot<T>(a.meta, k - 1, per + offp, hm);
        if (k < N) {
            K = kw_knot<T>(a.meta, k, per + off, hm);
            const int w = K.w, rows = K.rows;
            // H_k factor (block_cholesky.jl:55-91,145-153): potrf, or 1/h for a diagonal H
            const T *Hk = Hb + K.oH;
            if (hm == 2) {
                for (int i = tid; i < w; i += BT) K.Hf[i] = (T)1 / Hk[i];
                __syncthreads();                                         // JYt below reads all of it
            } else {
                for (int e = tid; e < w * w; e += BT) K.Hf[e] = Hk[e];
                __syncthreads();
                const int f = wg::wg_potrf<T>(K.Hf, w, w, tid);
                if (f && tid == 0 && s_hinfo == 0) s_hinfo = -(k + 1);
            }
            // jacobian_blocks.jl:232-236  JYt = H⁻¹Yᵀ (w × rows), r = JYtᵀg
            const T *Yk = Yb + K.oY;
            for (int e = tid; e < w * rows; e += BT) {
                const int i = e / w, j = e - i * w;
                T v = Yk[i + (size_t)j * rows];
                if (ginv && hm == 2) v *= K.Hf[j];
                JYt[j + (size_t)i * w] = v;
            }
            __syncthreads();
            if (ginv && hm != 2) {                                       // potrs
                wg::wg_trsm_ut<T>(K.Hf, w, w, JYt, w, rows, tid);
                wg::wg_trsm_un<T>(K.Hf, w, w, JYt, w, rows, tid);
            }
            if (ginv) {
                wg::wg_mm1<T, 1>(vt, rows, rows, 1, nullptr, cm<T>(JYt, w), cm<T>(gb + K.og, w), w, tid);
                __syncthreads();
            }
            // :240 Y·JYt by blocks, copy_shur! (:271-286): rows [0,p1) D2, [p1,p1+ps) C, [p1+ps,rows) D1
            const int p1 = K.p1, ps = K.ps, p2 = K.p2, o2 = p1 + ps;
            auto Ym = [&](int i0) { return cmt<T>(Yk + i0, rows); };      // (q, i) → Y[i0+i, q]
            auto Jm = [&](int j0) { return cm<T>(JYt + (size_t)j0 * w, w); };
            if (k > 0 && p1) wg::wg_mm1<T, 1>(Kp.C, p1, p1, p1, Kp.C, Ym(0), Jm(0), w, tid);   // A ≡ prev C
            wg::wg_mm1<T, 1>(K.B, ps, ps, ps, nullptr, Ym(p1), Jm(p1), w, tid);
            wg::wg_mm1<T, 1>(K.C, p2, p2, p2, nullptr, Ym(o2), Jm(o2), w, tid);
            wg::wg_mm1<T, 1>(K.DF, p1, p1, ps, nullptr, Ym(0), Jm(p1), w, tid);
            wg::wg_mm1<T, 1>(K.DF + (size_t)p1 * ps, p1, p1, p2, nullptr, Ym(0), Jm(o2), w, tid);
            wg::wg_mm1<T, 1>(K.Emu, ps, ps, p2, nullptr, Ym(p1), Jm(o2), w, tid);
            // c = r_C − y_c, d = r_D1 − y_d ; d_{k−1} += r_D2 (:251)
            const T *yk = yb + K.oy;
            T *mu = K.mu();
            for (int i = tid; i < ps; i += BT) mu[i] = (ginv ? vt[p1 + i] : (T)0) - yk[i];
            for (int i = tid; i < p2; i += BT) K.lam[i] = (ginv ? vt[o2 + i] : (T)0) - yk[ps + i];
            if (k > 0 && ginv)
                for (int i = tid; i < p1; i += BT) Kp.lam[i] += vt[i];
            __syncthreads();
        }
        if (k > 0) {
            if (k > 1) {
                const Knot<T> K2 = kw_knot<T>(a.meta, k - 2, per + offpp, hm);
                kw_factor_fwd<T>(Kp, &K2, k - 1, &s_finfo, tid);
            } else {
                kw_factor_fwd<T>(Kp, nullptr, k - 1, &s_finfo, tid);
            }
        }
        if (k < N) {
            offpp = offp;
            offp = off;
            off += kw_knot_elems(a.meta + (size_t)k * 8, hm);
        }
    }

    // ---- backward substitution (cholesky_solve.jl:119-143); offp = knot N−1's base
    size_t oc = offp, on = 0;                  // knot k's base, knot k+1's base
    for (int k = N - 1; k >= 0; --k) {
        const Knot<T> K = kw_knot<T>(a.meta, k, per + oc, hm);
        T *mu = K.mu();
        if (k < N - 1) {
            const Knot<T> Kn = kw_knot<T>(a.meta, k + 1, per + on, hm);
            // λ_k += D_{k+1}μ_{k+1} + F_{k+1}λ_{k+1}
            wg::wg_mm<T, 1, 1>(K.lam, K.p2, K.p2, 1, K.lam, cmt<T>(Kn.DF, Kn.p1), cm<T>(Kn.mu(), Kn.ps), Kn.ps,
                               cmt<T>(Kn.DF + (size_t)Kn.p1 * Kn.ps, Kn.p1), cm<T>(Kn.lam, Kn.p2), Kn.p2, tid);
            __syncthreads();
            if (K.p2) wg::wg_trsm_un<T>(K.C, K.p2, K.p2, K.lam, K.p2, 1, tid);
            // μ_k −= Ẽλ_k
            wg::wg_mm1<T, -1>(mu, K.ps, K.ps, 1, mu, cmt<T>(K.Emu, K.ps), cm<T>(K.lam, K.p2), K.p2, tid);
            __syncthreads();
        }
        if (K.ps) wg::wg_trsm_un<T>(K.B, K.ps, K.ps, mu, K.ps, 1, tid);
        for (int i = tid; i < K.ps; i += BT) {
            mu[i] = -mu[i];
            lamb[K.oy + i] = mu[i];
        }
        if (k < N - 1)
            for (int i = tid; i < K.p2; i += BT) {
                K.lam[i] = -K.lam[i];
                lamb[K.oy + K.ps + i] = K.lam[i];
            }
        else
            for (int i = tid; i < K.p2; i += BT) lamb[K.oy + K.ps + i] = K.lam[i];
        __syncthreads();
        if (k > 0) {
            on = oc;
            oc -= kw_knot_elems(a.meta + (size_t)(k - 1) * 8, hm);
        }
    }

    // ---- primal recovery (cholesky_solver.jl:185-236, SOC :254-273)
    off = 0;
    offp = 0;
    for (int k = 0; k < N; ++k) {
        const Knot<T> K = kw_knot<T>(a.meta, k, per + off, hm);
        const int w = K.w, rows = K.rows;
        const T *Yk = Yb + K.oY;
        // v = [λ_{k−1}; μ_k; λ_k]
        if (k > 0) {
            const Knot<T> Kp = kw_knot<T>(a.meta, k - 1, per + offp, hm);
            for (int i = tid; i < K.p1; i += BT) vt[i] = Kp.lam[i];
        }
        for (int i = tid; i < K.ps; i += BT) vt[K.p1 + i] = K.mu()[i];
        for (int i = tid; i < K.p2; i += BT) vt[K.p1 + K.ps + i] = K.lam[i];
        __syncthreads();
        T *z = dzb + K.og;
        wg::wg_mm1<T, 1>(z, w, w, 1, ginv ? gb + K.og : nullptr, cm<T>(Yk, rows), cm<T>(vt, rows), rows, tid);
        __syncthreads();
        if (ginv && hm != 2) {
            wg::wg_trsm_ut<T>(K.Hf, w, w, z, w, 1, tid);
            wg::wg_trsm_un<T>(K.Hf, w, w, z, w, 1, tid);
        }
        for (int j = tid; j < w; j += BT) z[j] = (ginv && hm == 2) ? -(z[j] * K.Hf[j]) : -z[j];
        __syncthreads();
        offp = off;
        off += kw_knot_elems(a.meta + (size_t)k * 8, hm);
    }
    if (tid == 0 && a.info) a.info[b] = s_hinfo ? s_hinfo : s_finfo;
}

// per-trajectory scratch elements
size_t kw_elems(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2, const int32_t *w)
{
    size_t e = (size_t)a.maxw * a.maxrows + std::max(a.maxw, a.maxrows);
    for (int k = 0; k < a.N; ++k) {
        const size_t P1 = n1[k], PS = p[k], P2 = n2[k], W = w[k];
        e += P1 * (PS + P2) + PS * PS + PS * (P2 + 1) + P2 * P2 + P2 + (a.h_mode == 2 ? W : W * W);
    }
    return e;
}

int64_t kw_chunk(const KktArgs &a, size_t per_bytes)
{
    int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(a.batch, ((int64_t)4 << 30) / (int64_t)per_bytes));
    if (const char *ev = std::getenv("LQRX_KKT_WG_CHUNK"))   // tests: force the multi-chunk path
        chunk = std::max<int64_t>(1, std::min<int64_t>(chunk, std::atoll(ev)));
    return chunk;
}

} // namespace

bool kkt_wg_supported(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2, const int32_t *w)
{
    if (a.layout != 0 || a.N < 1) return false;
    for (int k = 0; k < a.N; ++k)
        if (n1[k] > KW_MAX_BLOCK || p[k] > KW_MAX_BLOCK || n2[k] > KW_MAX_BLOCK || w[k] > KW_MAX_W) return false;
    return true;
}

size_t kkt_wg_scratch_bytes(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                            const int32_t *w)
{
    if (a.batch == 0 || !kkt_wg_supported(a, n1, p, n2, w)) return 0;
    const size_t per = kw_elems(a, n1, p, n2, w) * (a.dtype == 0 ? 8 : 4);
    return per * (size_t)kw_chunk(a, per);
}

hipError_t kkt_wg_launch(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2, const int32_t *w,
                         hipStream_t s)
{
    if (!kkt_wg_supported(a, n1, p, n2, w)) return hipErrorNotSupported;
    const size_t elems = kw_elems(a, n1, p, n2, w), per = elems * (a.dtype == 0 ? 8 : 4);
    int64_t chunk = kw_chunk(a, per);
    if (a.ws) chunk = std::min<int64_t>(chunk, (int64_t)(a.ws_bytes / per));
    if (chunk < 1) return hipErrorInvalidValue;
    Scratch sc;
    hipError_t e = sc.get(a, per * (size_t)chunk, s);
    if (e != hipSuccess) return e;
    for (int64_t b0 = 0; b0 < a.batch && e == hipSuccess; b0 += chunk) {
        dim3 grid((unsigned)std::min<int64_t>(chunk, a.batch - b0)), block(BT);
        if (a.dtype == 0)
            hipLaunchKernelGGL((kkt_wg_kernel<double>), grid, block, 0, s, a, (double *)sc.p, elems, b0);
        else
            hipLaunchKernelGGL((kkt_wg_kernel<float>), grid, block, 0, s, a, (float *)sc.p, elems, b0);
        e = hipGetLastError();
    }
    hipError_t ef = sc.release(s);
    return e != hipSuccess ? e : ef;
}

} // namespace lqrx
