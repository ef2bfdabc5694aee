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

// ---- diagonal H (and the SOC, where H⁻¹ → I): the Schur pieces straight from Y ----------------
// shur!/copy_shur! (jacobian_blocks.jl:231-286) need Y·H⁻¹·Yᵀ by blocks of Y = [D2; C; D1]: A = D2
// H⁻¹D2ᵀ (added into knot k−1's C), D, F = D2 H⁻¹[Cᵀ | D1ᵀ], B, E = C H⁻¹[Cᵀ | D1ᵀ], C = D1 H⁻¹D1ᵀ —
// the upper block triangle of one Gram matrix over the rows in segment order.  With a diagonal
// H it is formed with no H⁻¹Yᵀ transient: Y is streamed in 4-column k-slices, every lane holds
// one element of each of a super-tile's row blocks (16 rows), the column side scaled by h⁻¹ on
// the fly; each wave owns 4×4 super-tiles of 16×16 output tiles (round-robin), so one slice of
// ≤ 8 row blocks feeds ≤ 16 MFMAs.  The k order (16-column k-tiles, Tile<T>::row's k index per
// MFMA) is wg_mm_k's, so the results equal the transient path's bit for bit.
template <typename T> __device__ __forceinline__ T kw_bload(__amdgpu_buffer_rsrc_t r, uint32_t vo)
{
    if constexpr (sizeof(T) == 8)
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)vo, 0, 0));
    else
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)vo, 0, 0));
}
struct KwBlk {
    int seg, r0, nv, off;          // segment (0 D2, 1 C, 2 D1), first Y row, valid rows, row offset in the segment
};
template <typename T> __device__ __forceinline__ KwBlk kw_blk(const Knot<T> &K, int b)
{
    const int n0 = (K.p1 + 15) >> 4, n1 = (K.ps + 15) >> 4;
    if (b < n0) return KwBlk{0, 16 * b, min(16, K.p1 - 16 * b), 16 * b};
    if (b < n0 + n1) return KwBlk{1, K.p1 + 16 * (b - n0), min(16, K.ps - 16 * (b - n0)), 16 * (b - n0)};
    const int c = b - n0 - n1;
    return KwBlk{2, K.p1 + K.ps + 16 * c, min(16, K.p2 - 16 * c), 16 * c};
}
// destination of the (si, sj) block of the Gram matrix (si ≤ sj); null: not needed
template <typename T>
__device__ __forceinline__ T *kw_dst(const Knot<T> &K, const Knot<T> *Kp, int si, int sj, int &ld, bool &add)
{
    add = false;
    if (si == 0 && sj == 0) { ld = K.p1; add = true; return Kp ? Kp->C : nullptr; }   // A ≡ prev C (+=)
    if (si == 0 && sj == 1) { ld = K.p1; return K.DF; }                                // D
    if (si == 0) { ld = K.p1; return K.DF + (size_t)K.p1 * K.ps; }                     // F
    if (si == 1 && sj == 1) { ld = K.ps; return K.B; }
    if (si == 1) { ld = K.ps; return K.Emu; }                                          // E
    ld = K.p2;
    return K.C;
}

// one super-tile: row blocks 4·GI … 4·GI+3 × column blocks RJ·GJ … (all RJ·4 tiles are
// accumulated; only the upper ones, bi ≤ bj, are stored)
template <typename T> constexpr int kw_rj() { return sizeof(T) == 8 ? 2 : 4; }
template <typename T>
__device__ __forceinline__ void kw_gram_st(const Knot<T> &K, const Knot<T> *Kp, const T *Yk, const T *hs, int GI,
                                           int GJ, int NB, int lane)
{
    using acc = typename Tile<T>::acc;
    constexpr int RJ = kw_rj<T>();
    constexpr uint32_t TS = sizeof(T), OOB = 0x80000000u;
    const int i16 = lane & 15, rows = K.rows, w = K.w;
    // this lane's k index within a 16-column k-tile for the slice q = s mod 4: Tile<T>::row(lane, q)
    const int kl = Tile<T>::row(lane, 0), kq = Tile<T>::row(lane, 1) - kl;   // row(lane, q) = kl + q·kq
    KwBlk bI[4], bJ[RJ];
    uint32_t vI[4], vJ[RJ];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int b = 4 * GI + i;
        bI[i] = b < NB ? kw_blk<T>(K, b) : KwBlk{-1, 0, 0, 0};
        vI[i] = i16 < bI[i].nv ? (uint32_t)((bI[i].r0 + i16 + kl * rows) * (int)TS) : OOB;
    }
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        const int c = RJ * GJ + j;
        bJ[j] = c < NB ? kw_blk<T>(K, c) : KwBlk{-1, 0, 0, 0};
        vJ[j] = i16 < bJ[j].nv ? (uint32_t)((bJ[j].r0 + i16 + kl * rows) * (int)TS) : OOB;
    }
    acc D[4][RJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < RJ; ++j) {
            D[i][j] = acc{0, 0, 0, 0};
            // the A tiles (D2·D2ᵀ) add into knot k−1's C: start from it
            if (Kp && bI[i].seg == 0 && bJ[j].seg == 0 && 4 * GI + i <= RJ * GJ + j)
                wg::tile_ld<T>(D[i][j], Kp->C + bI[i].off + (size_t)bJ[j].off * K.p1, bI[i].nv, bJ[j].nv, 1, K.p1, lane);
        }
    const char *yb = (const char *)Yk;
    // fp64: one slice = 4 consecutive columns (kq = 4); fp32: kq = 1, so a 16-column k-tile takes
    // all 4 of its slices even when only part of it lies below w (the rest read 0)
    const int yn = rows * w * (int)TS, nks = kq == 1 ? 4 * ((w + 15) >> 4) : (w + 3) >> 2;
    // slice s: columns 16(s/4) + row(lane, s mod 4) — descriptor base at the slice's first column
    auto base = [&](int s) { return 16 * (s >> 2) + kq * (s & 3); };
    constexpr int PF = 2;
    T aI[PF][4], aJ[PF][RJ];
    auto load = [&](int s, T (&xi)[4], T (&xj)[RJ]) __attribute__((always_inline)) {
        const int o = base(s) * rows * (int)TS;
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc((void *)(yb + o), (short)0, max(yn - o, 0), 0x00020000);
#pragma unroll
        for (int i = 0; i < 4; ++i) xi[i] = kw_bload<T>(r, vI[i]);
#pragma unroll
        for (int j = 0; j < RJ; ++j) xj[j] = kw_bload<T>(r, vJ[j]);
    };
#pragma unroll
    for (int u = 0; u < PF; ++u) load(u, aI[u], aJ[u]);
    for (int s0 = 0; s0 < nks; s0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int s = s0 + u;
            const T h = hs[base(s) + kl];             // 0 past w (and the loads read 0 there)
            T fj[RJ];
#pragma unroll
            for (int j = 0; j < RJ; ++j) fj[j] = aJ[u][j] * h;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < RJ; ++j) D[i][j] = Tile<T>::mma(aI[u][i], fj[j], D[i][j]);
            load(s + PF, aI[u], aJ[u]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // store: the upper tiles (bi ≤ bj) into their block's destination; a same-segment off-
    // diagonal tile also transposed (the symmetric blocks stay full, as the transient path left them)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < RJ; ++j) {
            const KwBlk &P = bI[i], &Q = bJ[j];
            if (P.seg < 0 || Q.seg < 0 || 4 * GI + i > RJ * GJ + j) continue;
            int ld;
            bool add;
            T *dst = kw_dst<T>(K, Kp, P.seg, Q.seg, ld, add);
            if (!dst) continue;
            const bool mirror = P.seg == Q.seg && P.off != Q.off;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = Tile<T>::row(lane, r), col = tcol(lane);
                if (row < P.nv && col < Q.nv) {
                    dst[P.off + row + (size_t)(Q.off + col) * ld] = D[i][j][r];
                    if (mirror) dst[Q.off + col + (size_t)(P.off + row) * ld] = D[i][j][r];
                }
            }
        }
}

// the Schur pieces of knot k from Y with column scale hs (LDS, ≥ w + 16 entries, 0 past w):
// the waves take the super-tiles that hold an upper tile round-robin
template <typename T>
__device__ void kw_gram(const Knot<T> &K, const Knot<T> *Kp, const T *Yk, const T *hs, int tid)
{
    constexpr int RJ = kw_rj<T>();
    const int NB = ((K.p1 + 15) >> 4) + ((K.ps + 15) >> 4) + ((K.p2 + 15) >> 4);
    const int GR = (NB + 3) >> 2, GC = (NB + RJ - 1) / RJ, wave = tid >> 6, lane = tid & 63;
    int idx = 0;
    for (int GI = 0; GI < GR; ++GI)
        for (int GJ = (4 * GI) / RJ; GJ < GC; ++GJ, ++idx)       // first column group with a tile bj ≥ 4·GI
            if (idx % (BT / 64) == wave) kw_gram_st<T>(K, Kp, Yk, hs, GI, GJ, NB, lane);
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
        wg::wg_mm<T, -1, 1>(K.B, ps, ps, ps, K.B, Dm, Dm, p1, Dm, Dm, 0, tid, true);   // (upper, as C)
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
        // (upper tiles only: potrf and the triangular solves read C's upper triangle)
        wg::wg_mm<T, -1, -1>(K.C, p2, p2, p2, K.C, Fm, Fm, p1, Em, Em, ps, tid, true);
        wg::wg_mm1<T, -1>(K.lam, p2, p2, 1, K.lam, Em, mum, ps, tid);
        __syncthreads();
        const int f = wg::wg_potrf<T>(K.C, p2, p2, tid);                // :62
        if (f && tid == 0 && *s_finfo == 0) *s_finfo = j + 1;
        wg::wg_trsm_ut<T>(K.C, p2, p2, K.lam, p2, 1, tid);              // :113 C̃⁻ᵀ
    }
}

template <typename T>
__global__ __launch_bounds__(BT, 2) void kkt_wg_kernel(const KktArgs a, T *__restrict__ ws, size_t ws_elems, int64_t b0)
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
    __shared__ T hs_l[KW_MAX_W + 16], hg_l[KW_MAX_W];      // diagonal H: h⁻¹ (or 1), h⁻¹·g
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
            const T *Yk = Yb + K.oY;
            const int p1 = K.p1, ps = K.ps, p2 = K.p2, o2 = p1 + ps;
            if (hm == 2) {
                // no H⁻¹Yᵀ transient: the Schur pieces straight from Y (kw_gram), r = Y·(h⁻¹g)
                const T *gk = gb + K.og;
                for (int i = tid; i < w + 16; i += BT) {
                    const T hi = i < w ? (T)1 / Hk[i] : (T)0;
                    if (i < w) K.Hf[i] = hi;
                    hs_l[i] = i < w ? (ginv ? hi : (T)1) : (T)0;
                    if (ginv && i < w) hg_l[i] = hi * gk[i];
                }
                __syncthreads();
                kw_gram<T>(K, k > 0 ? &Kp : nullptr, Yk, hs_l, tid);
                if (ginv) {
                    for (int i = tid; i < rows; i += BT) {
                        T s0 = (T)0, s1 = (T)0;
                        int q = 0;
                        for (; q + 1 < w; q += 2) {
                            s0 = fma(Yk[i + (size_t)q * rows], hg_l[q], s0);
                            s1 = fma(Yk[i + (size_t)(q + 1) * rows], hg_l[q + 1], s1);
                        }
                        if (q < w) s0 = fma(Yk[i + (size_t)q * rows], hg_l[q], s0);
                        vt[i] = s0 + s1;
                    }
                }
                __syncthreads();
            } else {
                for (int e = tid; e < w * w; e += BT) K.Hf[e] = Hk[e];
                __syncthreads();
                const int f = wg::wg_potrf<T>(K.Hf, w, w, tid);
                if (f && tid == 0 && s_hinfo == 0) s_hinfo = -(k + 1);
                // jacobian_blocks.jl:232-236  JYt = H⁻¹Yᵀ (w × rows), r = JYtᵀg
                for (int e = tid; e < w * rows; e += BT) {
                    const int i = e / w, j = e - i * w;
                    JYt[j + (size_t)i * w] = Yk[i + (size_t)j * rows];
                }
                __syncthreads();
                if (ginv) {                                              // potrs
                    wg::wg_trsm_ut<T>(K.Hf, w, w, JYt, w, rows, tid);
                    wg::wg_trsm_un<T>(K.Hf, w, w, JYt, w, rows, tid);
                    wg::wg_mm1<T, 1>(vt, rows, rows, 1, nullptr, cm<T>(JYt, w), cm<T>(gb + K.og, w), w, tid);
                    __syncthreads();
                }
                // :240 Y·JYt by blocks, copy_shur! (:271-286): rows [0,p1) D2, [p1,p1+ps) C, [p1+ps,rows) D1
                auto Ym = [&](int i0) { return cmt<T>(Yk + i0, rows); };  // (q, i) → Y[i0+i, q]
                auto Jm = [&](int j0) { return cm<T>(JYt + (size_t)j0 * w, w); };
                if (k > 0 && p1) wg::wg_mm1<T, 1>(Kp.C, p1, p1, p1, Kp.C, Ym(0), Jm(0), w, tid);   // A ≡ prev C
                wg::wg_mm1<T, 1>(K.B, ps, ps, ps, nullptr, Ym(p1), Jm(p1), w, tid);
                wg::wg_mm1<T, 1>(K.C, p2, p2, p2, nullptr, Ym(o2), Jm(o2), w, tid);
                wg::wg_mm1<T, 1>(K.DF, p1, p1, ps, nullptr, Ym(0), Jm(p1), w, tid);
                wg::wg_mm1<T, 1>(K.DF + (size_t)p1 * ps, p1, p1, p2, nullptr, Ym(0), Jm(o2), w, tid);
                wg::wg_mm1<T, 1>(K.Emu, ps, ps, p2, nullptr, Ym(p1), Jm(o2), w, tid);
            }
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

// per-launch scratch caps: the library's own pool takes up to 24 GiB (n = 96: ~10 MB per
// trajectory — the B = 2048 batch in one launch instead of five under-filled ones) and halves
// on an out-of-memory; lqrx_kkt_workspace_size quotes the round-4 4 GiB, so a caller-owned
// workspace stays modest (the launch then runs the batch in more chunks) — but never less than
// one full residency of the device (kw_resident: 2 workgroups per CU): a chunk below that leaves
// CUs idle in every launch (round 6: 4 GiB = 410 trajectories of n = 96 per launch on 512 slots
// took the B = 2048 line 131 → 162 ms, profiles/r06/m)
constexpr int64_t KW_POOL_CAP = (int64_t)24 << 30, KW_WS_CAP = (int64_t)4 << 30;

// workgroups of kkt_wg_kernel the current device holds at once (launch bounds: 2 per CU)
int64_t kw_resident()
{
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    (void)hipGetLastError();
    return 2 * (int64_t)std::max(cus, 1);
}

int64_t kw_chunk(const KktArgs &a, size_t per_bytes, int64_t cap_bytes, bool full = false)
{
    // chunks of at most cap_bytes of per-trajectory scratch (full: at least one device residency),
    // evened out over the launches
    int64_t cap = std::max<int64_t>(1, cap_bytes / (int64_t)per_bytes);
    if (full) cap = std::max(cap, kw_resident());
    const int64_t nl = (a.batch + cap - 1) / cap;
    int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(a.batch, (a.batch + nl - 1) / nl));
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
    return per * (size_t)kw_chunk(a, per, KW_WS_CAP, true);
}

hipError_t kkt_wg_launch(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2, const int32_t *w,
                         hipStream_t s)
{
    if (!kkt_wg_supported(a, n1, p, n2, w)) return hipErrorNotSupported;
    const size_t elems = kw_elems(a, n1, p, n2, w), per = elems * (a.dtype == 0 ? 8 : 4);
    int64_t chunk = kw_chunk(a, per, a.ws ? (int64_t)std::min<size_t>(a.ws_bytes, (size_t)KW_POOL_CAP) : KW_POOL_CAP);
    if (a.ws) chunk = std::min<int64_t>(chunk, (int64_t)(a.ws_bytes / per));
    if (chunk < 1) return hipErrorInvalidValue;
    Scratch sc;
    hipError_t e = sc.get(a, per * (size_t)chunk, s);
    // library scratch: when the pool cannot hold the chunk (the device partly in use by torch or
    // another rank), halve until it fits or one trajectory fails — as kb_launch_t does
    while (e == hipErrorOutOfMemory && !a.ws && chunk > 1) {
        (void)hipGetLastError();
        chunk = kw_chunk(a, per, (int64_t)per * ((chunk + 1) / 2));
        e = sc.get(a, per * (size_t)chunk, s);
    }
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
