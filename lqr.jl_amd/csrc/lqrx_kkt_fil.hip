// lqrx_kkt_fil.hip — batched block-tridiagonal KKT solve (CholeskySolver._solve!,
// /root/reference/src/cholesky_solver.jl:166-182) for block structures of the
// "first / interior / last" form that ConstraintBlocks produces for trajectory problems
// (conblocks.jl:403-425): knot 0 = (n1 0, p P0, n2 n̄, w n̄+m), knots 1..N-2 = (n̄, PK, n̄,
// n̄+m), knot N-1 = (n̄, PN, 0, n̄).  Dubins (BASELINE cfg3: n̄=3, m=2, P0=3, PK=0, PN=3) and
// the double integrators of test/problems.jl have this form.
//
// Why a separate kernel: with every block size a compile-time constant, each knot's work is
// straight-line register code (no runtime-size predication, no selects), which is ~5× fewer
// VALU instructions per knot than the generic kernel (lqrx_kkt.hip) — and the per-wave
// instruction stream IS the cost here: one lane per trajectory, the horizon serial.
//
// Mapping: ONE LANE PER TRAJECTORY, 64 per wave (one wave per workgroup).  Per-knot inputs
// (Y_k, y_k, H_k, g_k of the wave's 64 trajectories, packed per trajectory in the ABI) are
// brought to LDS by coalesced LDS-DMA (lqrx_stage.h) two knots ahead into a ring of three
// buffers; the factor slab is batch-fastest (coalesced stores/loads).
//
//   forward  k = 0..N-1: shur!/copy_shur! of knot k+1 (jacobian_blocks.jl:231-286; its
//            A block and r1 fold into knot k's C and d — the aliasing of :166/:251),
//            cholesky! of knot k (cholesky_solve.jl:47-67), forward_substitution!
//            (:93-117); factor blocks + forward μ, λ → slab.
//   backward k = N-1..0: backward_substitution! (:119-143) and, one knot behind,
//            calc_residual!/calc_primals! (cholesky_solver.jl:195-236) from re-staged
//            Y, H, g: δz_k = −H_k⁻¹(D2ᵀλ_{k-1} + Cᵀμ_k + D1ᵀλ_k + g_k).
// Triangular factors keep 1/U_ii on the diagonal (multiplies instead of divides).
#include "lqrx_internal.h"
#include "lqrx_stage.h"
#include "lqrx_tile.h"
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <type_traits>

namespace lqrx {
namespace fil {

#ifndef LQRX_FIL_ABL
#define LQRX_FIL_ABL 0   // ablation builds for tools/ only (bits: 1 forward sweep alone, 2 Schur
                         // from one column, 4 no F̃ recompute, 8 primal without Yᵀm, 16 no
                         // hand-placed VMEM waits, 32 no forward slab stores, 64 no δz/λ
                         // stores — timing bounds only, results wrong)
#endif
#ifndef LQRX_FIL_RING
#define LQRX_FIL_RING 1  // layout-0 δz/λ of interior knots through the LDS output ring (0: direct stores)
#endif
#ifndef LQRX_FIL_N12
#define LQRX_FIL_N12 1   // 12-byte LDS-DMA pieces for the short chunks (0: dwords only)
#endif
constexpr int Z(int x) { return x > 0 ? x : 1; }
constexpr int tri(int x) { return x * (x + 1) / 2; }

template <int P1_, int PS_, int P2_, int W_> struct Cls {
    static constexpr int P1 = P1_, PS = PS_, P2 = P2_, W = W_, R = P1_ + PS_ + P2_;
    static constexpr int O1 = 0, OS = P1_, O2 = P1_ + PS_;     // row segments of Y = [D2; C; D1]
    static constexpr bool none = (W_ == 0);
};
using NoCls = Cls<0, 0, 0, 0>;

// SOA = ABI layout 1 (batch fastest): element e of a trajectory's packed array at [e·batch + t],
// so the 64 trajectories of a wave read one element as a contiguous 512-B row
// PAD (direct kernel, layout 0): the compile-time sizes are MAXIMA and the structure's own
// (n̄, m, P0, PK, PN) come at run time (KktArgs::rt, struct Rt below): every block is zero-padded
// in registers — padded Y rows/columns and g read as 0, padded H as 1, a padded constraint row
// gets a unit Schur pivot (decoupled: its off-diagonal entries are exact zeros), padded δz/λ
// entries are never stored.  The real entries see the same operations in the same order as on
// the exact shape (the padding only adds exact zeros), so one instantiation serves every
// smaller trajectory structure.
template <int NX_, int M_, int P0_, int PK_, int PN_, bool HDIAG_, bool GINV_, bool SOA_ = false, bool PAD_ = false>
struct Shape {
    static constexpr int NX = NX_, M = M_;
    static constexpr bool HDIAG = HDIAG_, GINV = GINV_, SOA = SOA_, PAD = PAD_;
    static_assert(!PAD_ || !SOA_, "padded shapes read layout 0");
    using F = Cls<0, P0_, NX_, NX_ + M_>;
    using I = Cls<NX_, PK_, NX_, NX_ + M_>;
    using L = Cls<NX_, PN_, 0, NX_>;
    template <class C> static constexpr int LY() { return C::R * C::W; }
    template <class C> static constexpr int Ly() { return C::PS + C::P2; }
    template <class C> static constexpr int LH() { return HDIAG ? C::W : C::W * C::W; }
    template <class C> static constexpr int Lg() { return C::W; }
    // Y goes in 16-byte pieces when every knot's Y block has an even length (then every
    // knot offset and the trajectory stride are even); the short y/H/g chunks in dwords
    static constexpr bool WIDE_Y = (LY<F>() % 2 == 0) && (LY<I>() % 2 == 0) && (LY<L>() % 2 == 0);
    static constexpr int nsplit(int L) { return LQRX_FIL_N12 ? (8 * L) / 12 + ((8 * L) % 12) / 4 : 2 * L; }   // = Split<L>::instrs
    // SOA: one 16-B-per-lane DMA moves two element rows (2 × 64 doubles)
    static constexpr int rows2(int L) { return (L + 1) / 2; }
    template <class C> static constexpr int Dmin()   // DMA instructions of a forward restage
    {
        if constexpr (SOA)
            return C::none ? 0 : rows2(LY<C>()) + rows2(Ly<C>()) + (GINV ? rows2(LH<C>()) + rows2(Lg<C>()) : 0);
        return C::none ? 0 : (WIDE_Y ? LY<C>() / 2 : 2 * LY<C>()) + nsplit(Ly<C>()) +
                                 (GINV ? nsplit(LH<C>()) + nsplit(Lg<C>()) : 0);
    }
    template <class C> static constexpr int Dbwd()   // … of a backward restage (no y)
    {
        if constexpr (SOA)
            return C::none ? 0 : rows2(LY<C>()) + (GINV ? rows2(LH<C>()) + rows2(Lg<C>()) : 0);
        return C::none ? 0 : (WIDE_Y ? LY<C>() / 2 : 2 * LY<C>()) + (GINV ? nsplit(LH<C>()) + nsplit(Lg<C>()) : 0);
    }
    template <int A, int B, int C> static constexpr int mx3() { return A > B ? (A > C ? A : C) : (B > C ? B : C); }
    static constexpr int LYm = mx3<LY<F>(), LY<I>(), LY<L>()>();
    static constexpr int Lym = mx3<Ly<F>(), Ly<I>(), Ly<L>()>();
    static constexpr int LHm = mx3<LH<F>(), LH<I>(), LH<L>()>();
    static constexpr int Lgm = mx3<Lg<F>(), Lg<I>(), Lg<L>()>();
    // staging buffer (bytes): Y image (16-B pieces, dense) | y | H | g split images
    // (SOA: [element row][64 lanes] images, rows rounded up to even — the DMA moves row pairs)
    static constexpr int sb(int L)
    {
        return SOA ? 8 * (2 * rows2(L)) : LQRX_FIL_N12 ? 16 * ((8 * L) / 12) + 4 * (((8 * L) % 12) / 4) : 8 * L;
    }
    static constexpr int OFF_y = 64 * (SOA ? sb(LYm) : 8 * LYm);
    static constexpr int OFF_H = OFF_y + 64 * mx3<sb(Ly<F>()), sb(Ly<I>()), sb(Ly<L>())>();
    static constexpr int OFF_g = OFF_H + 64 * mx3<sb(LH<F>()), sb(LH<I>()), sb(LH<L>())>();
    static constexpr int BUF_BYTES = OFF_g + 64 * mx3<sb(Lg<F>()), sb(Lg<I>()), sb(Lg<L>())>();
    static constexpr int BUF = (BUF_BYTES + 15) / 16 * 2;       // doubles per staging buffer
    // slab slot: B̃ (tri) | C̃ (tri) | D̃ | Ẽ | μ | λ  (max over the classes).  F̃ (p1×p2, non-
    // empty only for interior knots) is NOT stored: the backward sweep recomputes
    // F̃_{k+1} = C̃_k⁻ᵀ·D2_{k+1}H⁻¹D1_{k+1}ᵀ from knot k+1's Y/H, which it re-stages for the
    // primal recovery anyway — 9 fewer doubles written and read back per interior knot
    template <class C> static constexpr int slab()
    {
        return tri(C::PS) + tri(C::P2) + C::P1 * C::PS + C::PS * C::P2 + C::PS + C::P2;
    }
    static constexpr int SLOT = mx3<slab<F>(), slab<I>(), slab<L>()>();
    // layout-0 output images (doubles per lane): δz chunk, then [μ; λ] chunk
    static constexpr int WOUT = mx3<F::W, I::W, L::W>();
    static constexpr int LOUT = mx3<F::PS + F::P2, I::PS + I::P2, L::PS + L::P2>();
};

// per-knot offsets (elements) in the packed per-trajectory arrays: knot 0 is class F,
// knots 1.. follow with class I sizes (the last knot starts where an I knot would)
template <class S> struct Off {
    __device__ static int64_t Y(int k) { return k == 0 ? 0 : S::template LY<typename S::F>() + (int64_t)(k - 1) * S::template LY<typename S::I>(); }
    __device__ static int64_t y(int k) { return k == 0 ? 0 : S::template Ly<typename S::F>() + (int64_t)(k - 1) * S::template Ly<typename S::I>(); }
    __device__ static int64_t H(int k) { return k == 0 ? 0 : S::template LH<typename S::F>() + (int64_t)(k - 1) * S::template LH<typename S::I>(); }
    __device__ static int64_t g(int k) { return k == 0 ? 0 : S::template Lg<typename S::F>() + (int64_t)(k - 1) * S::template Lg<typename S::I>(); }
};

// runtime block sizes of a padded shape (S::PAD): packed offsets of the real structure and the
// padded → real row / column maps of each knot class (uniform values: scalar registers)
struct Rt {
    int nx = 0, m = 0, p0 = 0, pk = 0, pn = 0;
    int64_t LYF = 0, LYI = 0, LyF = 0, LyI = 0, Lg = 0;
    // the wave's array bases (trajectory t0) and this lane's byte offsets from them: inputs are
    // buffer loads with the element offset in the scalar soffset (no per-element address math;
    // host-checked: 64 trajectories of any array span < 2 GiB)
    const double *bY = nullptr, *bH = nullptr, *bg = nullptr, *by = nullptr;
    uint32_t vY = 0, vH = 0, vg = 0, vy = 0;
    __device__ __forceinline__ void lanes(const KktArgs &a, int64_t t0, int64_t t)
    {
        bY = a.Y + t0 * a.sY; bH = a.H + t0 * a.sH; bg = a.g + t0 * a.sg; by = a.y + t0 * a.sy;
        vY = (uint32_t)((t - t0) * a.sY * 8); vH = (uint32_t)((t - t0) * a.sH * 8);
        vg = (uint32_t)((t - t0) * a.sg * 8); vy = (uint32_t)((t - t0) * a.sy * 8);
    }
    __device__ __forceinline__ void init(const KktArgs &a)
    {
        nx = a.rt[0]; m = a.rt[1]; p0 = a.rt[2]; pk = a.rt[3]; pn = a.rt[4];
        LYF = (int64_t)(p0 + nx) * (nx + m);
        LYI = (int64_t)(2 * nx + pk) * (nx + m);
        LyF = p0 + nx;
        LyI = pk + nx;
        Lg = nx + m;
    }
    // a copy whose sizes the compiler cannot see through: every offset / map derived from it is
    // recomputed where it is used (scalar ALU, cheap) instead of being hoisted out of the knot
    // loop into hundreds of live scalar registers (which spilled)
    __device__ __forceinline__ Rt fresh() const
    {
        Rt r = *this;
        asm volatile("" : "+s"(r.nx), "+s"(r.m), "+s"(r.p0), "+s"(r.pk), "+s"(r.pn));
        r.LYF = (int64_t)(r.p0 + r.nx) * (r.nx + r.m);
        r.LYI = (int64_t)(2 * r.nx + r.pk) * (r.nx + r.m);
        r.LyF = r.p0 + r.nx;
        r.LyI = r.pk + r.nx;
        r.Lg = r.nx + r.m;
        return r;
    }
    __device__ __forceinline__ int64_t oY(int k) const { return k == 0 ? 0 : LYF + (int64_t)(k - 1) * LYI; }
    __device__ __forceinline__ int64_t oy(int k) const { return k == 0 ? 0 : LyF + (int64_t)(k - 1) * LyI; }
    __device__ __forceinline__ int64_t og(int k) const { return (int64_t)k * Lg; }   // diag H: oH = og
    // real (p1, ps, p2) of class C of shape S: first (0, P0, n̄), interior (n̄, PK, n̄), last (n̄, PN, 0)
    template <class S, class C> __device__ __forceinline__ void cls(int &p1, int &ps, int &p2) const
    {
        if constexpr (std::is_same<C, typename S::F>::value) { p1 = 0; ps = p0; p2 = nx; }
        else if constexpr (std::is_same<C, typename S::I>::value) { p1 = nx; ps = pk; p2 = nx; }
        else { p1 = nx; ps = pn; p2 = 0; }
    }
    template <class S, class C> __device__ __forceinline__ int R() const
    {
        int p1, ps, p2;
        cls<S, C>(p1, ps, p2);
        return p1 + ps + p2;
    }
    // padded row i of Y = [D2; C; D1] (class C) → real row, or −1
    template <class S, class C> __device__ __forceinline__ int row(int i) const
    {
        int p1, ps, p2;
        cls<S, C>(p1, ps, p2);
        if (i < C::P1) return i < p1 ? i : -1;
        if (i < C::P1 + C::PS) return i - C::P1 < ps ? p1 + (i - C::P1) : -1;
        return i - C::P1 - C::PS < p2 ? p1 + ps + (i - C::P1 - C::PS) : -1;
    }
    // padded row i of the [μ; λ] chunk (PS + P2 rows) → real row, or −1
    template <class S, class C> __device__ __forceinline__ int lrow(int i) const
    {
        int p1, ps, p2;
        cls<S, C>(p1, ps, p2);
        if (i < C::PS) return i < ps ? i : -1;
        return i - C::PS < p2 ? ps + (i - C::PS) : -1;
    }
    // padded column j ([x; u]: NX state then M input columns; the last knot has states only)
    template <class S, class C> __device__ __forceinline__ int col(int j) const
    {
        if (j < S::NX) return j < nx ? j : -1;
        return j - S::NX < m ? nx + (j - S::NX) : -1;
    }
};

using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void *base)
{
    // raw buffer (stride 0), full 31-bit range; gfx9 dword-3 format bits
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000);
}
// (u4_t, make_rsrc4, dma_lds, lds_addr: the inline-asm LDS-DMA issue, lqrx_stage.h)

// DMA pattern of one packed array for a chunk of L doubles per trajectory: the wave's 64
// chunks form a dense [t][L] image of `per` pieces per trajectory (16 B pieces when WIDE,
// else dwords); instruction i moves pieces 64i .. 64i+63, lane l piece 64i + l.  The per-lane
// byte offsets are knot-invariant (only the scalar soffset changes per knot), so once
// initialised an issue costs no VALU work.  Lanes past the batch end read the last live
// trajectory (clamped) so no out-of-range access is ever issued.
template <int L, bool WIDE> struct Pat {
    static constexpr int unit = WIDE ? 16 : 4;
    static constexpr int per = L * 8 / unit;
    uint32_t vo[per > 0 ? per : 1];
    // sel (optional): the wave's trajectories are sel[0..nlive) instead of 0..nlive-1
    __device__ __forceinline__ void init(int64_t s, int lane, int nlive, const int32_t *sel = nullptr)
    {
#pragma unroll
        for (int i = 0; i < per; ++i) {
            const uint32_t p = 64u * (uint32_t)i + (uint32_t)lane;
            uint32_t tr = p / (uint32_t)per;
            const uint32_t e = p - tr * (uint32_t)per;
            tr = tr < (uint32_t)nlive ? tr : (uint32_t)(nlive - 1);
            if (sel) tr = (uint32_t)sel[tr];
            vo[i] = tr * (uint32_t)(s * 8) + e * (uint32_t)unit;
        }
    }
    __device__ __forceinline__ void issue(u4_t r, int64_t off_elems, double *lds) const
    {
        const uint32_t so = (uint32_t)(off_elems * 8), l0 = lds_addr(lds);
#pragma unroll
        for (int i = 0; i < per; ++i) dma_lds<unit>(r, vo[i], so, l0 + i * 64 * unit);
    }
};

// Short chunks (y, H, g: odd numbers of doubles, so 16-B alignment is impossible) go as
// 12-byte pieces (buffer_load_dwordx3 … lds, gfx950) plus a dword tail: L doubles = 8L bytes
// = n12·12 + n4·4.  A 12-byte LDS-DMA lands each lane's piece in a 16-byte LDS slot
// (measured: tools/dma12_probe.hip, profiles/r01/dma12_probe.txt), so the images are
// A = [t][n12][16 B] (12 valid) and B = [t][n4][4 B].  The reader (SImg) reassembles a
// double from its two dwords.  5 doubles cost 3 + 1 instructions instead of 10 dwords.
template <int L> struct Split {
    static constexpr int B = 8 * L, n12 = LQRX_FIL_N12 ? B / 12 : 0, n4 = (B - 12 * n12) / 4;
    static constexpr int bytesA = 64 * 16 * n12;
    static constexpr int lane_bytes = 16 * n12 + 4 * n4;       // LDS bytes per trajectory
    static constexpr int instrs = n12 + n4;
};
template <int L> struct PatS {
    using SP = Split<L>;
    uint32_t voA[SP::n12 > 0 ? SP::n12 : 1], voB[SP::n4 > 0 ? SP::n4 : 1];
    __device__ __forceinline__ void init(int64_t s, int lane, int nlive, const int32_t *sel = nullptr)
    {
        const uint32_t sb = (uint32_t)(s * 8);
#pragma unroll
        for (int i = 0; i < SP::n12; ++i) {
            const uint32_t p = 64u * (uint32_t)i + (uint32_t)lane;
            uint32_t tr = p / (uint32_t)(SP::n12 > 0 ? SP::n12 : 1);
            const uint32_t e = p - tr * (uint32_t)(SP::n12 > 0 ? SP::n12 : 1);
            tr = tr < (uint32_t)nlive ? tr : (uint32_t)(nlive - 1);
            if (sel) tr = (uint32_t)sel[tr];
            voA[i] = tr * sb + 12u * e;
        }
#pragma unroll
        for (int i = 0; i < SP::n4; ++i) {
            const uint32_t p = 64u * (uint32_t)i + (uint32_t)lane;
            uint32_t tr = p / (uint32_t)(SP::n4 > 0 ? SP::n4 : 1);
            const uint32_t e = p - tr * (uint32_t)(SP::n4 > 0 ? SP::n4 : 1);
            tr = tr < (uint32_t)nlive ? tr : (uint32_t)(nlive - 1);
            if (sel) tr = (uint32_t)sel[tr];
            voB[i] = tr * sb + 12u * SP::n12 + 4u * e;
        }
    }
    __device__ __forceinline__ void issue(u4_t r, int64_t off_elems, double *lds) const
    {
        const uint32_t so = (uint32_t)(off_elems * 8), l0 = lds_addr(lds);
#pragma unroll
        for (int i = 0; i < SP::n12; ++i) dma_lds<12>(r, voA[i], so, l0 + i * 64 * 16);
#pragma unroll
        for (int i = 0; i < SP::n4; ++i) dma_lds<4>(r, voB[i], so, l0 + SP::bytesA + i * 64 * 4);
    }
};
// reader of a split image: element j of this lane's chunk
typedef const __attribute__((address_space(3))) uint32_t lds_u32;
typedef const __attribute__((address_space(3))) u4_t lds_u4;
template <int L> struct SImg {
    using SP = Split<L>;
    uint32_t base;                                                  // LDS byte address
    int lane;
    __device__ __forceinline__ uint32_t dw(int x) const
    {
        // explicit LDS (address-space 3) access: a generic-pointer form of this read trips
        // an instruction-selection bug in this compiler (src_shared_base compare)
        const uint32_t a = x < 12 * SP::n12 ? base + (lane * SP::n12 + x / 12) * 16 + x % 12
                                            : base + SP::bytesA + lane * (4 * SP::n4) + (x - 12 * SP::n12);
        return *(lds_u32 *)(size_t)a;
    }
    __device__ __forceinline__ double operator[](int j) const
    {
        const uint64_t lo = dw(8 * j), hi = dw(8 * j + 4);
        return __builtin_bit_cast(double, lo | (hi << 32));
    }
    // the whole chunk into registers: one 16-byte LDS read per 12-byte piece (the image's
    // 16-B slots of 16 consecutive lanes are distinct mod 16 — bank-conflict free, where
    // dword reads at the 48/32-B lane stride conflicted 4–8 ways) plus the dword tail
    __device__ __forceinline__ void load(double (&out)[L]) const
    {
        uint32_t w[2 * L];
#pragma unroll
        for (int s = 0; s < SP::n12; ++s) {
            const u4_t q = *(lds_u4 *)(size_t)(base + (lane * SP::n12 + s) * 16);
            w[3 * s] = q.x;
            w[3 * s + 1] = q.y;
            w[3 * s + 2] = q.z;
        }
#pragma unroll
        for (int t = 0; t < SP::n4; ++t) w[3 * SP::n12 + t] = *(lds_u32 *)(size_t)(base + SP::bytesA + lane * (4 * SP::n4) + 4 * t);
#pragma unroll
        for (int j = 0; j < L; ++j) out[j] = __builtin_bit_cast(double, (uint64_t)w[2 * j] | ((uint64_t)w[2 * j + 1] << 32));
    }
};
// a lane's Y chunk (L doubles at lane·L in the dense image) into registers: 16-byte reads
// when L is even (chunks 16-B aligned), doubles otherwise
typedef double d2_t __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(3))) d2_t lds_d2;
typedef const __attribute__((address_space(3))) double lds_d;
template <int L, bool WIDE> __device__ __forceinline__ void load_Y(uint32_t lds_base, int lane, double (&v)[L])
{
    if constexpr (WIDE && L % 2 == 0) {
#pragma unroll
        for (int p = 0; p < L / 2; ++p) {
            const d2_t q = *(lds_d2 *)(size_t)(lds_base + (lane * L + 2 * p) * 8);
            v[2 * p] = q.x;
            v[2 * p + 1] = q.y;
        }
    } else {
#pragma unroll
        for (int e = 0; e < L; ++e) v[e] = *(lds_d *)(size_t)(lds_base + (lane * L + e) * 8);
    }
}

// reader of an SOA image ([element][64 lanes]): element j of this lane's chunk — consecutive
// lanes read consecutive doubles (no bank conflicts)
template <int L> struct SImgS {
    uint32_t base;
    int lane;
    __device__ __forceinline__ double operator[](int j) const { return *(lds_d *)(size_t)(base + (j * 64 + lane) * 8); }
    __device__ __forceinline__ void load(double (&out)[L]) const
    {
#pragma unroll
        for (int j = 0; j < L; ++j) out[j] = (*this)[j];
    }
};

typedef unsigned int u2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void bstore(double v, rsrc_t r, uint32_t vo, uint32_t so)
{
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2_t, v), r, vo, so, 0);
}
typedef __attribute__((address_space(3))) double lds_dw;
// Layout-0 output stores (δz, λ): a wave's 64 chunks of L doubles are first written to an LDS
// image [t][L] (lane t's chunk at t·L), then stored as L instructions, instruction i moving
// the image's doubles 64i .. 64i+63 — consecutive lanes write consecutive doubles of one
// trajectory's chunk (≈ 64/L trajectories per instruction) instead of one double of each of
// 64 trajectories (64 cache lines per instruction; measured: dropping the layout-0 δz/λ
// stores altogether cut cfg3 from 0.356 to 0.262 ms).  Same instruction count as the
// per-lane stores, so the hand-placed vmcnt bounds are unchanged; doubles of dead
// trajectories get an offset past the buffer range (the store drops them — no exec branch).
template <int L> struct StPat {
    uint32_t vo[L];
    __device__ __forceinline__ void init(int64_t s, int lane, int nlive, const int32_t *sel)
    {
#pragma unroll
        for (int i = 0; i < L; ++i) {
            const uint32_t p = 64u * (uint32_t)i + (uint32_t)lane;
            const uint32_t tr = p / (uint32_t)L, e = p - tr * (uint32_t)L;
            const uint32_t tg = tr < (uint32_t)nlive ? (sel ? (uint32_t)sel[tr] : tr) : 0u;
            vo[i] = tr < (uint32_t)nlive ? tg * (uint32_t)(s * 8) + 8u * e : 0xFFFFFF00u;
        }
    }
    // padded shapes: a runtime chunk length lr ≤ L (image [t][lr]); instructions past the
    // image's 64·lr doubles store nothing (out-of-range offset)
    __device__ __forceinline__ void init_rt(int64_t s, int lane, int nlive, int lr)
    {
        const uint32_t l = (uint32_t)(lr > 0 ? lr : 1);
#pragma unroll
        for (int i = 0; i < L; ++i) {
            const uint32_t p = 64u * (uint32_t)i + (uint32_t)lane;
            const uint32_t tr = p / l, e = p - tr * l;
            vo[i] = (lr > 0 && tr < (uint32_t)nlive) ? tr * (uint32_t)(s * 8) + 8u * e : 0xFFFFFF00u;
        }
    }
};
template <int L>
__device__ __forceinline__ void dense_store(const double (&v)[Z(L)], double *img, const StPat<L> &pat, rsrc_t r,
                                            uint32_t so, int lane);
// staging buffer views (lane-linear [t][L] images; SOA: [element][64] images)
template <class S> struct Buf {
    double *base;
    __device__ const double *Y(int lane, int L) const { return base + lane * L; }
    __device__ uint32_t lds() const { return (uint32_t)(size_t)(lptr_t)base; }
    template <int L> using Img = typename std::conditional<S::SOA, SImgS<L>, SImg<L>>::type;
    template <int L> __device__ Img<L> y(int lane) const { return Img<L>{lds() + S::OFF_y, lane}; }
    template <int L> __device__ Img<L> H(int lane) const { return Img<L>{lds() + S::OFF_H, lane}; }
    template <int L> __device__ Img<L> g(int lane) const { return Img<L>{lds() + S::OFF_g, lane}; }
    template <class C> __device__ void ld_Y(int lane, double (&v)[S::template LY<C>()]) const
    {
        if constexpr (S::SOA)
            SImgS<S::template LY<C>()>{lds(), lane}.load(v);
        else
            load_Y<S::template LY<C>(), S::WIDE_Y>(lds(), lane, v);
    }
    template <class C> __device__ void ld_H(int lane, double (&v)[S::template LH<C>()]) const { H<S::template LH<C>()>(lane).load(v); }
    template <class C> __device__ void ld_g(int lane, double (&v)[S::template Lg<C>()]) const { g<S::template Lg<C>()>(lane).load(v); }
};

// per-wave context: buffer resources, lane facts, the DMA patterns of interior knots
template <class S> struct Ctx {
    using I = typename S::I;
    const double *bY, *by, *bH, *bg;              // wave bases (→ buffer resources at use)
    double *bS, *bdz, *blam;
    int lane, nlive;
    bool live;
    uint32_t vS, vdz, vlam;                        // per-lane byte offsets: slab, dz, lam
    const int32_t *sel = nullptr;                  // layout 0, selected trajectories (a.sel + t0) or null
    uint32_t vsoa = 0, rowb = 0;                   // SOA: lane's row-pair offset, bytes per element row
    uint32_t limY = 0, limy = 0, limH = 0, limg = 0; // SOA: bytes from the wave base to each array's end
    uint32_t lpad = 0;                             // LDS byte address of the DMA filler's 256-B target
    // layout 0: LDS images of the coalesced δz / λ stores (dense_store), interior patterns
    double *ozi = nullptr, *oli = nullptr;
    int64_t sgz = 0, slz = 0;                      // per-trajectory strides of dz, lam
    StPat<S::I::W> pz;
    StPat<Z(S::I::PS + S::I::P2)> pl;
    Rt rt;                                         // S::PAD: the structure's real block sizes
    __device__ __forceinline__ void init_out(const KktArgs &a, double *ost)
    {
        ozi = ost;
        oli = ost + 64 * S::WOUT;
        sgz = a.sg;
        slz = a.sl;
        if constexpr (S::PAD) {
            ozb = (uint32_t)(size_t)(lptr_t)ost;
            olb = ozb + 64 * S::WOUT * 8;
            pz.init_rt(a.sg, lane, nlive, (int)rt.Lg);
            pl.init_rt(a.sl, lane, nlive, (int)rt.LyI);
        } else {
            pz.init(a.sg, lane, nlive, sel);
            pl.init(a.sl, lane, nlive, sel);
        }
    }
    // padded shapes: a chunk of L padded doubles, real length lr, element j at real position
    // map(j) (−1: padding, not stored); INTERIOR: the precomputed interior pattern applies
    uint32_t ozb = 0, olb = 0;                     // LDS byte addresses of ozi / oli
    template <int L, bool INTERIOR, class Map>
    __device__ __forceinline__ void out_store_pad(const double (&v)[Z(L)], uint32_t b, const StPat<L> *pi,
                                                  int64_t stride, const double *base, int64_t off, int lr,
                                                  Map &&map) const
    {
#pragma unroll
        for (int j = 0; j < L; ++j) {
            const int cj = map(j);
            if (cj >= 0) *(lds_dw *)(size_t)(b + (lane * lr + cj) * 8) = v[j];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        StPat<L> q;
        if constexpr (!INTERIOR) q.init_rt(stride, lane, nlive, lr);
        const StPat<L> &pat = INTERIOR ? *pi : q;
        const rsrc_t r = make_rsrc(base);
#pragma unroll
        for (int i = 0; i < L; ++i) bstore(*(lds_dw *)(size_t)(b + (64 * i + lane) * 8), r, pat.vo[i], (uint32_t)(off * 8));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    // a chunk of L doubles per trajectory at element offset off: the interior pattern when the
    // length matches, else a one-off pattern (first / last knot)
    template <int L, int LI>
    __device__ __forceinline__ void out_store(const double (&v)[Z(L)], double *img, const StPat<LI> &pi,
                                              int64_t stride, const double *base, int64_t off) const
    {
        if constexpr (L == LI) {
            dense_store<L>(v, img, pi, make_rsrc(base), (uint32_t)(off * 8), lane);
        } else {
            StPat<L> q;
            q.init(stride, lane, nlive, sel);
            dense_store<L>(v, img, q, make_rsrc(base), (uint32_t)(off * 8), lane);
        }
    }
    // SOA: L element rows from row r0 of one array, as (L+1)/2 row-pair DMAs (lane l → row
    // 2i + l/32, trajectories 2(l mod 32), +1).  Reads past the array's end (dead lanes of the
    // last wave, the odd row of the last pair) are out of the resource's range and return 0.
    template <int L>
    __device__ __forceinline__ void soa_issue(const double *base, uint32_t lim, int64_t r0, double *lds) const
    {
        const u4_t r = make_rsrc4n(base, lim);
        const uint32_t l0 = lds_addr(lds), v0 = vsoa + (uint32_t)r0 * rowb;
        // (the row offset rides in the VGPR offset: the buffer range check does not cover soffset)
#pragma unroll
        for (int i = 0; i < S::rows2(L); ++i) dma_lds<16>(r, v0 + 2u * (uint32_t)i * rowb, 0u, l0 + 1024u * i);
    }
    Pat<S::template LY<I>(), S::WIDE_Y> pY;
    PatS<S::template Ly<I>()> py;
    PatS<S::template LH<I>()> pH;
    PatS<S::template Lg<I>()> pg;

    // interior knot k: the precomputed patterns
    __device__ __forceinline__ void stage_I(int k, double *buf, bool fwd) const
    {
        using O = Off<S>;
        if constexpr (S::SOA) {
            soa_issue<S::template LY<I>()>(bY, limY, O::Y(k), buf);
            if (fwd) soa_issue<S::template Ly<I>()>(by, limy, O::y(k), buf + S::OFF_y / 8);
            if constexpr (S::GINV) {
                soa_issue<S::template LH<I>()>(bH, limH, O::H(k), buf + S::OFF_H / 8);
                soa_issue<S::template Lg<I>()>(bg, limg, O::g(k), buf + S::OFF_g / 8);
            }
            return;
        }
        pY.issue(make_rsrc4(bY), O::Y(k), buf);
        if (fwd) py.issue(make_rsrc4(by), O::y(k), buf + S::OFF_y / 8);
        if constexpr (S::GINV) {
            pH.issue(make_rsrc4(bH), O::H(k), buf + S::OFF_H / 8);
            pg.issue(make_rsrc4(bg), O::g(k), buf + S::OFF_g / 8);
        }
    }
    // first / last knot (class C): one-off patterns
    template <class C>
    __device__ __forceinline__ void stage(const KktArgs &a, int k, double *buf, bool fwd) const
    {
        using O = Off<S>;
        if constexpr (S::SOA) {
            soa_issue<S::template LY<C>()>(bY, limY, O::Y(k), buf);
            if (fwd) soa_issue<S::template Ly<C>()>(by, limy, O::y(k), buf + S::OFF_y / 8);
            if constexpr (S::GINV) {
                soa_issue<S::template LH<C>()>(bH, limH, O::H(k), buf + S::OFF_H / 8);
                soa_issue<S::template Lg<C>()>(bg, limg, O::g(k), buf + S::OFF_g / 8);
            }
            return;
        }
        Pat<S::template LY<C>(), S::WIDE_Y> qY;
        qY.init(a.sY, lane, nlive, sel);
        qY.issue(make_rsrc4(bY), O::Y(k), buf);
        if (fwd) {
            PatS<S::template Ly<C>()> qy;
            qy.init(a.sy, lane, nlive, sel);
            qy.issue(make_rsrc4(by), O::y(k), buf + S::OFF_y / 8);
        }
        if constexpr (S::GINV) {
            PatS<S::template LH<C>()> qH;
            qH.init(a.sH, lane, nlive, sel);
            qH.issue(make_rsrc4(bH), O::H(k), buf + S::OFF_H / 8);
            PatS<S::template Lg<C>()> qg;
            qg.init(a.sg, lane, nlive, sel);
            qg.issue(make_rsrc4(bg), O::g(k), buf + S::OFF_g / 8);
        }
    }
    // A first / last knot stages fewer DMA instructions than an interior one when its blocks
    // are smaller: it then issues filler DMAs (an out-of-range source — nothing is read — into
    // a 256-B LDS area nothing reads) up to the interior count.  Every staging group then issues
    // at least the interior count on every path, so the hand-counted vmcnt bounds, which count
    // interior groups, hold also on the compiled paths a static check cannot rule out (a last-
    // knot stage followed by an interior step's wait).
    template <class C>
    __device__ __forceinline__ void stage_fill(bool fwd) const
    {
        constexpr int nf = S::template Dmin<I>() - S::template Dmin<C>();
        constexpr int nb = S::template Dbwd<I>() - S::template Dbwd<C>();
        const u4_t r = make_rsrc4(bY);
        if (fwd) {
#pragma unroll
            for (int i = 0; i < nf; ++i) dma_lds<4>(r, 0xFFFFFF00u, 0u, lpad);
        } else {
#pragma unroll
            for (int i = 0; i < nb; ++i) dma_lds<4>(r, 0xFFFFFF00u, 0u, lpad);
        }
    }
    // any knot into its ring buffer (stg + (k mod 3)·BUF)
    __device__ __forceinline__ void stage_any(const KktArgs &a, int k, double *stg, bool fwd) const
    {
        double *buf = stg + (k % 3) * S::BUF;
        if (k == 0) {
            stage<typename S::F>(a, 0, buf, fwd);
            stage_fill<typename S::F>(fwd);
        } else if (k == a.N - 1) {
            stage<typename S::L>(a, k, buf, fwd);
            stage_fill<typename S::L>(fwd);
        } else {
            stage_I(k, buf, fwd);
        }
    }
};

template <int L>
__device__ __forceinline__ void dense_store(const double (&v)[Z(L)], double *img, const StPat<L> &pat, rsrc_t r,
                                            uint32_t so, int lane)
{
    const uint32_t b = (uint32_t)(size_t)(lptr_t)img;
#pragma unroll
    for (int j = 0; j < L; ++j) *(lds_dw *)(size_t)(b + (lane * L + j) * 8) = v[j];
    // one wave: its LDS ops execute in order — only keep the compiler from reordering
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < L; ++i) bstore(*(lds_dw *)(size_t)(b + (64 * i + lane) * 8), r, pat.vo[i], so);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // reads done before the next writes
    __builtin_amdgcn_wave_barrier();
}

// the forward sweep's slab stores (an ablation build can drop them)
__device__ __forceinline__ void sstore(double v, rsrc_t r, uint32_t vo, uint32_t so)
{
#if LQRX_FIL_ABL & 32
    (void)v, (void)r, (void)vo, (void)so;
#else
    bstore(v, r, vo, so);
#endif
}
__device__ __forceinline__ double bload(rsrc_t r, uint32_t vo, uint32_t so)
{
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
}

// wait until at most N vector-memory ops are outstanding (N ≤ 63) and all LDS ops are done.
// G names the DMA group the wait is for — the G-th most recent `dma_group()` — so that
// tests/isa_vmcnt.py can check N against the compiled instruction stream (N > 0 needs a G).
// LQRX_FIL_WAIT_SLACK (test-only negative control, never in the library build) loosens every
// bound by that many ops.
#ifndef LQRX_FIL_WAIT_SLACK
#define LQRX_FIL_WAIT_SLACK 0
#endif
template <int N, int G = 0> __device__ __forceinline__ void vm_wait()
{
    static_assert(N <= 0 || G > 0, "a hand vmcnt bound names its target DMA group");
    constexpr int n0 = N > 0 ? N + LQRX_FIL_WAIT_SLACK : N;
    constexpr int n = n0 > 63 ? 63 : (n0 < 0 ? 0 : n0);
#if LQRX_FIL_ABL & 16
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // ablation: no VMEM waits (wrong results)
    (void)n;
#else
    if constexpr (G > 0)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0) ; lqrx.wait g=%1" ::"n"(n), "n"(G) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(n) : "memory");
#endif
}

// ------------------------------------------------------------------ small dense kernels
// upper Cholesky X = UᵀU in place (upper triangle, i ≤ j); diagonal replaced by 1/U_ii.
// Returns false on a non-positive pivot (potrf info; the sweep continues like the caller).
template <int M>
__device__ __forceinline__ bool potrf_inv(double (&X)[Z(M)][Z(M)])
{
    bool ok = true;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        double d = X[j][j];
#pragma unroll
        for (int p = 0; p < j; ++p) d = fma(-X[p][j], X[p][j], d);
        ok = ok && (d > 0.0);
        const double ri = rsqrt_nr(d);
        X[j][j] = ri;
#pragma unroll
        for (int c = j + 1; c < M; ++c) {
            double v = X[j][c];
#pragma unroll
            for (int p = 0; p < j; ++p) v = fma(-X[p][j], X[p][c], v);
            X[j][c] = v * ri;
        }
    }
    return ok;
}

// X ← U⁻ᵀX (X is M×NR); U from potrf_inv (inverse diagonal)
template <int M, int NR>
__device__ __forceinline__ void trsm_t(const double (&U)[Z(M)][Z(M)], double (&X)[Z(M)][Z(NR)])
{
#pragma unroll
    for (int c = 0; c < NR; ++c)
#pragma unroll
        for (int i = 0; i < M; ++i) {
            double s = X[i][c];
#pragma unroll
            for (int p = 0; p < i; ++p) s = fma(-U[p][i], X[p][c], s);
            X[i][c] = s * U[i][i];
        }
}
// x ← U⁻ᵀx
template <int M> __device__ __forceinline__ void trsv_t(const double (&U)[Z(M)][Z(M)], double (&x)[Z(M)])
{
#pragma unroll
    for (int i = 0; i < M; ++i) {
        double s = x[i];
#pragma unroll
        for (int p = 0; p < i; ++p) s = fma(-U[p][i], x[p], s);
        x[i] = s * U[i][i];
    }
}
// x ← U⁻¹x
template <int M> __device__ __forceinline__ void trsv_n(const double (&U)[Z(M)][Z(M)], double (&x)[Z(M)])
{
#pragma unroll
    for (int i = M - 1; i >= 0; --i) {
        double s = x[i];
#pragma unroll
        for (int p = i + 1; p < M; ++p) s = fma(-U[i][p], x[p], s);
        x[i] = s * U[i][i];
    }
}

// ------------------------------------------------------------------ Schur pieces
// shur! (jacobian_blocks.jl:231-242): S = Y H⁻¹ Yᵀ (upper triangle), r = Y H⁻¹ g;
// Ginv = false (SOC variant): S = Y Yᵀ, r = 0.  Y is R×W column-major in LDS.
template <class C> struct Shur {
    double S[Z(C::R)][Z(C::R)];
    double r[Z(C::R)];
};

template <class S, class C>
__device__ __forceinline__ bool compute_shur(Shur<C> &s, const double (&Y)[S::template LY<C>()],
                                             const double (&H)[S::template LH<C>()], const double (&g)[S::template Lg<C>()])
{
    constexpr int R = C::R, W = C::W;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        s.r[i] = 0.0;
#pragma unroll
        for (int j = i; j < R; ++j) s.S[i][j] = 0.0;
    }
    bool ok = true;
    if constexpr (!S::GINV || S::HDIAG) {
        // stream Y column by column: S += y_j h_j y_jᵀ, r += y_j h_j g_j  (h = 1/H_jj)
#pragma unroll
        for (int j = 0; j < ((LQRX_FIL_ABL & 2) ? 1 : W); ++j) {
            double v[R], vh[R];
#pragma unroll
            for (int i = 0; i < R; ++i) v[i] = Y[i + j * R];
            if constexpr (S::GINV) {
                const double h = rcp_nr2(H[j]);               // block_cholesky.jl:86 inv
                const double gh = g[j];
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    vh[i] = v[i] * h;
                    s.r[i] = fma(vh[i], gh, s.r[i]);
                }
            } else {
#pragma unroll
                for (int i = 0; i < R; ++i) vh[i] = v[i];
            }
#pragma unroll
            for (int i = 0; i < R; ++i)
#pragma unroll
                for (int i2 = i; i2 < R; ++i2) s.S[i][i2] = fma(vh[i], v[i2], s.S[i][i2]);
        }
    } else {
        // dense / block-diagonal H (block_cholesky.jl:55-77): potrf, then Wt = H⁻¹Yᵀ row by row
        double U[W][W];
#pragma unroll
        for (int j = 0; j < W; ++j)
#pragma unroll
            for (int i = 0; i <= j; ++i) U[i][j] = H[i + j * W];
        ok = potrf_inv<W>(U);
        double Wt[R][W];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            double x[W];
#pragma unroll
            for (int j = 0; j < W; ++j) x[j] = Y[i + j * R];
            trsv_t<W>(U, x);
            trsv_n<W>(U, x);
#pragma unroll
            for (int j = 0; j < W; ++j) Wt[i][j] = x[j];
        }
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const double gj = g[j];
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const double y = Y[i + j * R];
                s.r[i] = fma(Wt[i][j], gj, s.r[i]);
#pragma unroll
                for (int i2 = i; i2 < R; ++i2) s.S[i][i2] = fma(y, Wt[i2][j], s.S[i][i2]);
            }
        }
    }
    return ok;
}

// ------------------------------------------------------------------ forward step
// Carried between knots: Ua = C̃_{k-1} (factor, inverse diagonal) and λ_{k-1} (forward).
template <class S> struct Carry {
    double Ua[Z(S::NX)][Z(S::NX)];
    double lprev[Z(S::NX)];
};

// slab: wave-major [k][field][64 lanes] doubles (coalesced; 32-bit offsets per wave)
template <class S> __device__ __forceinline__ uint32_t slab_so(int k, int f)
{
    return (uint32_t)((k * S::SLOT + f) * 64 * 8);
}

// cholesky! + forward_substitution! of knot k (class C), given its Schur pieces sc, y_k
// (yc), and the Schur pieces of knot k+1 (sn, class Cn; NoCls at the last knot).
// Returns the number of slab stores issued (all single doubles).
template <class S, class C, class Cn>
__device__ __forceinline__ void factor_knot(int k, const Shur<C> &sc, const double (&yc)[Z(C::PS + C::P2)],
                                            const Shur<Cn> &sn, Carry<S> &cy, const Ctx<S> &c, int &info)
{
    constexpr int p1 = C::P1, ps = C::PS, p2 = C::P2;
    constexpr int O1 = C::O1, OS = C::OS, O2 = C::O2;
    static_assert(Cn::none || Cn::P1 == p2, "n1[k+1] == n2[k]");
    double D[Z(p1)][Z(ps)], Bm[Z(ps)][Z(ps)], E[Z(ps)][Z(p2)], F[Z(p1)][Z(p2)], Cm[Z(p2)][Z(p2)];
    double cc[Z(ps)], d[Z(p2)];
#pragma unroll
    for (int i = 0; i < p1; ++i) {
#pragma unroll
        for (int j = 0; j < ps; ++j) D[i][j] = sc.S[O1 + i][OS + j];
#pragma unroll
        for (int j = 0; j < p2; ++j) F[i][j] = sc.S[O1 + i][O2 + j];
    }
#pragma unroll
    for (int i = 0; i < ps; ++i) {
#pragma unroll
        for (int j = i; j < ps; ++j) Bm[i][j] = sc.S[OS + i][OS + j];
#pragma unroll
        for (int j = 0; j < p2; ++j) E[i][j] = sc.S[OS + i][O2 + j];
        cc[i] = sc.r[OS + i] - yc[i];                             // copy_shur! :284
    }
#pragma unroll
    for (int i = 0; i < p2; ++i) {
#pragma unroll
        for (int j = i; j < p2; ++j) {
            double v = sc.S[O2 + i][O2 + j];
            if constexpr (!Cn::none) v += sn.S[i][j];             // A_{k+1} ≡ C_k  (:166, :277)
            Cm[i][j] = v;
        }
        double dv = sc.r[O2 + i] - yc[ps + i];                    // :285
        if constexpr (!Cn::none) dv += sn.r[i];                   // d .+= r_D2 of k+1  (:251)
        d[i] = dv;
    }
    // cholesky!(U[k], F[k])  cholesky_solve.jl:47-67
    if constexpr (p1 > 0) {
        if constexpr (ps > 0) trsm_t<p1, ps>(cy.Ua, D);              // :49  D̃ = A⁻ᵀD
        if constexpr (p2 > 0) trsm_t<p1, p2>(cy.Ua, F);              // :57  F̃ = A⁻ᵀF
    }
    if constexpr (ps > 0) {
#pragma unroll
        for (int i = 0; i < ps; ++i)
#pragma unroll
            for (int j = i; j < ps; ++j) {
                double v = Bm[i][j];
#pragma unroll
                for (int q = 0; q < p1; ++q) v = fma(-D[q][i], D[q][j], v);   // :50-53
                Bm[i][j] = v;
            }
        if (!potrf_inv<ps>(Bm) && info == 0) info = k + 1;
#pragma unroll
        for (int i = 0; i < ps; ++i)
#pragma unroll
            for (int j = 0; j < p2; ++j) {
                double v = E[i][j];
#pragma unroll
                for (int q = 0; q < p1; ++q) v = fma(-D[q][i], F[q][j], v);   // :59
                E[i][j] = v;
            }
        if constexpr (p2 > 0) trsm_t<ps, p2>(Bm, E);                   // :60
    }
    if constexpr (p2 > 0) {
#pragma unroll
        for (int i = 0; i < p2; ++i)
#pragma unroll
            for (int j = i; j < p2; ++j) {
                double v = Cm[i][j];
#pragma unroll
                for (int q = 0; q < p1; ++q) v = fma(-F[q][i], F[q][j], v);   // :61-62
#pragma unroll
                for (int q = 0; q < ps; ++q) v = fma(-E[q][i], E[q][j], v);
                Cm[i][j] = v;
            }
        if (!potrf_inv<p2>(Cm) && info == 0) info = k + 1;
    }
    // forward_substitution!  cholesky_solve.jl:93-117
    double mu[Z(ps)], la[Z(p2)];
#pragma unroll
    for (int i = 0; i < ps; ++i) {
        double v = cc[i];
#pragma unroll
        for (int q = 0; q < p1; ++q) v = fma(-D[q][i], cy.lprev[q], v);
        mu[i] = v;
    }
    if constexpr (ps > 0) trsv_t<ps>(Bm, mu);
#pragma unroll
    for (int i = 0; i < p2; ++i) {
        double v = d[i];
#pragma unroll
        for (int q = 0; q < p1; ++q) v = fma(-F[q][i], cy.lprev[q], v);
#pragma unroll
        for (int q = 0; q < ps; ++q) v = fma(-E[q][i], mu[q], v);
        la[i] = v;
    }
    if constexpr (p2 > 0) trsv_t<p2>(Cm, la);
    // slab (batch-fastest, coalesced): B̃ | C̃ | D̃ | Ẽ | μ | λ  (F̃: recomputed, see Shape)
    int f = 0;
#pragma unroll
    for (int i = 0; i < ps; ++i)
#pragma unroll
        for (int j = i; j < ps; ++j) sstore(Bm[i][j], make_rsrc(c.bS), c.vS, slab_so<S>(k, f++));
#pragma unroll
    for (int i = 0; i < p2; ++i)
#pragma unroll
        for (int j = i; j < p2; ++j) sstore(Cm[i][j], make_rsrc(c.bS), c.vS, slab_so<S>(k, f++));
#pragma unroll
    for (int i = 0; i < p1; ++i)
#pragma unroll
        for (int j = 0; j < ps; ++j) sstore(D[i][j], make_rsrc(c.bS), c.vS, slab_so<S>(k, f++));
#pragma unroll
    for (int i = 0; i < ps; ++i)
#pragma unroll
        for (int j = 0; j < p2; ++j) sstore(E[i][j], make_rsrc(c.bS), c.vS, slab_so<S>(k, f++));
#pragma unroll
    for (int i = 0; i < ps; ++i) sstore(mu[i], make_rsrc(c.bS), c.vS, slab_so<S>(k, f++));
#pragma unroll
    for (int i = 0; i < p2; ++i) sstore(la[i], make_rsrc(c.bS), c.vS, slab_so<S>(k, f++));
    // carry C̃_k, λ_k to knot k+1
    if constexpr (p2 > 0) {
#pragma unroll
        for (int i = 0; i < p2; ++i) {
            cy.lprev[i] = la[i];
#pragma unroll
            for (int j = i; j < p2; ++j) cy.Ua[i][j] = Cm[i][j];
        }
    }
}

// forward step k (class C; next class Cn, class after next Cnn for the DMA issued here)
template <class S, class C, class Cn, class Cnn, bool FIRST = false>
__device__ __forceinline__ void fwd_step(const KktArgs &a, const Ctx<S> &c, int k, double *stg,
                                         Shur<C> &sc, double (&yc)[Z(C::PS + C::P2)], Shur<Cn> &sn,
                                         double (&yn)[Z(Cn::PS + Cn::P2)], Carry<S> &cy, int &info)
{
    if constexpr (!Cn::none) {
        Buf<S> b{stg + ((k + 1) % 3) * S::BUF};
        double Yv[S::template LY<Cn>()], Hv[S::template LH<Cn>()], gv[S::template Lg<Cn>()];
        b.template ld_Y<Cn>(c.lane, Yv);
        b.template ld_H<Cn>(c.lane, Hv);
        b.template ld_g<Cn>(c.lane, gv);
        const bool ok = compute_shur<S, Cn>(sn, Yv, Hv, gv);
        if (!ok && info == 0) info = -(k + 2);
        const auto yk = b.template y<S::template Ly<Cn>()>(c.lane);
#pragma unroll
        for (int i = 0; i < Cn::PS + Cn::P2; ++i) yn[i] = yk[i];
    }
    factor_knot<S, C, Cn>(k, sc, yc, sn, cy, c, info);
}

// ------------------------------------------------------------------ backward step
template <class C> struct SlabV {        // slab contents of one knot, in registers
    double Bm[Z(C::PS)][Z(C::PS)], Cm[Z(C::P2)][Z(C::P2)], D[Z(C::P1)][Z(C::PS)], E[Z(C::PS)][Z(C::P2)],
        F[Z(C::P1)][Z(C::P2)], mu[Z(C::PS)], la[Z(C::P2)];
};

template <class S, class C>
__device__ __forceinline__ void slab_load(SlabV<C> &v, const Ctx<S> &c, int k)
{
    constexpr int p1 = C::P1, ps = C::PS, p2 = C::P2;
    int f = 0;
    auto at = [&](int ff) { return bload(make_rsrc(c.bS), c.vS, slab_so<S>(k, ff)); };
#pragma unroll
    for (int i = 0; i < ps; ++i)
#pragma unroll
        for (int j = i; j < ps; ++j) v.Bm[i][j] = at(f++);
#pragma unroll
    for (int i = 0; i < p2; ++i)
#pragma unroll
        for (int j = i; j < p2; ++j) v.Cm[i][j] = at(f++);
#pragma unroll
    for (int i = 0; i < p1; ++i)
#pragma unroll
        for (int j = 0; j < ps; ++j) v.D[i][j] = at(f++);
#pragma unroll
    for (int i = 0; i < ps; ++i)
#pragma unroll
        for (int j = 0; j < p2; ++j) v.E[i][j] = at(f++);
#pragma unroll
    for (int i = 0; i < ps; ++i) v.mu[i] = at(f++);
#pragma unroll
    for (int i = 0; i < p2; ++i) v.la[i] = at(f++);
}

// Backward slab ring: interior / last knots' slab chunks come back by LDS-DMA (16-B pieces;
// the wave-major chunk [field][64 lanes] of a knot is contiguous, so piece p = 16·p bytes and
// the LDS image is the same [field][64] layout), issued two steps before use like the knot
// data.  Register loads (slab_load) would be tracked by the compiler, whose wait for them also
// drains every DMA issued after them (it does not count the asm DMA), i.e. one-step prefetch.
template <class S> constexpr int slab_ring_fields()
{
    return S::template slab<typename S::I>() > S::template slab<typename S::L>() ? S::template slab<typename S::I>()
                                                                                 : S::template slab<typename S::L>();
}
template <class S> constexpr int slab_dma_instrs() { return (slab_ring_fields<S>() + 1) / 2; }
template <class S> constexpr int SLB = slab_dma_instrs<S>() * 128;     // doubles per ring slot
// DMA instructions that stage one knot's slab chunk of class C (two fields per instruction)
template <class S, class C> constexpr int slab_dma_of() { return (S::template slab<C>() + 1) / 2; }

// slab k into its ring slot (k mod 3); k < 1: the same DMA, from slab 1, into the slot a slab k
// would take — a slot nothing reads again (the backward sweep's last steps), so every step
// issues the same number of DMAs and the hand-counted waits hold on every compiled path
template <class S, class C>
__device__ __forceinline__ void stage_slab(const Ctx<S> &c, int k, double *ring)
{
    const u4_t r = make_rsrc4(c.bS);
    const uint32_t so = slab_so<S>(k < 1 ? 1 : k, 0), l0 = lds_addr(ring + ((k + 3) % 3) * SLB<S>);
#pragma unroll
    for (int i = 0; i < slab_dma_of<S, C>(); ++i) dma_lds<16>(r, 2u * c.vS, so + 1024u * i, l0 + 1024u * i);
}

// F̃ of knot k+1 (class Cn, p1 × p2) for the backward sweep, recomputed with the forward's
// exact operation order (compute_shur's F block of the Schur pieces, then factor_knot's
// trsm by the previous knot's C̃ factor Ua = C̃_k, inverse diagonal) — bit-identical to the
// value the forward used.
template <class S, class Cn>
__device__ __forceinline__ void recompute_Ft(double (&Fo)[Z(Cn::P1)][Z(Cn::P2)], const double (&Ua)[Z(Cn::P1)][Z(Cn::P1)],
                                             const double (&Y)[S::template LY<Cn>()],
                                             const double (&H)[S::template LH<Cn>()])
{
    constexpr int R = Cn::R, W = Cn::W, p1 = Cn::P1, p2 = Cn::P2, O1 = Cn::O1, O2 = Cn::O2;
    if constexpr ((LQRX_FIL_ABL & 4) && p1 > 0 && p2 > 0) {
#pragma unroll
        for (int i = 0; i < p1; ++i)
#pragma unroll
            for (int i2 = 0; i2 < p2; ++i2) Fo[i][i2] = Y[i + i2] * Ua[0][0];
    } else if constexpr (p1 > 0 && p2 > 0) {
#pragma unroll
        for (int i = 0; i < p1; ++i)
#pragma unroll
            for (int i2 = 0; i2 < p2; ++i2) Fo[i][i2] = 0.0;
        if constexpr (!S::GINV || S::HDIAG) {
#pragma unroll
            for (int j = 0; j < W; ++j) {
                double vh[p1];
                if constexpr (S::GINV) {
                    const double h = rcp_nr2(H[j]);
#pragma unroll
                    for (int i = 0; i < p1; ++i) vh[i] = Y[(O1 + i) + j * R] * h;
                } else {
#pragma unroll
                    for (int i = 0; i < p1; ++i) vh[i] = Y[(O1 + i) + j * R];
                }
#pragma unroll
                for (int i = 0; i < p1; ++i)
#pragma unroll
                    for (int i2 = 0; i2 < p2; ++i2) Fo[i][i2] = fma(vh[i], Y[(O2 + i2) + j * R], Fo[i][i2]);
            }
        } else {
            double U[W][W];
#pragma unroll
            for (int j = 0; j < W; ++j)
#pragma unroll
                for (int i = 0; i <= j; ++i) U[i][j] = H[i + j * W];
            (void)potrf_inv<W>(U);
            double Wt[p2][W];
#pragma unroll
            for (int i2 = 0; i2 < p2; ++i2) {
                double x[W];
#pragma unroll
                for (int j = 0; j < W; ++j) x[j] = Y[(O2 + i2) + j * R];
                trsv_t<W>(U, x);
                trsv_n<W>(U, x);
#pragma unroll
                for (int j = 0; j < W; ++j) Wt[i2][j] = x[j];
            }
#pragma unroll
            for (int j = 0; j < W; ++j)
#pragma unroll
                for (int i = 0; i < p1; ++i)
#pragma unroll
                    for (int i2 = 0; i2 < p2; ++i2) Fo[i][i2] = fma(Y[(O1 + i) + j * R], Wt[i2][j], Fo[i][i2]);
        }
        trsm_t<p1, p2>(Ua, Fo);                                   // cholesky_solve.jl:57
    }
}

template <class S, class C>
__device__ __forceinline__ void slab_read(SlabV<C> &v, const Ctx<S> &c, int k, const double *ring)
{
    static_assert(S::template slab<C>() <= slab_ring_fields<S>(), "slab chunk fits a ring slot");
    constexpr int p1 = C::P1, ps = C::PS, p2 = C::P2;
    const double *b = ring + (k % 3) * SLB<S> + c.lane;
    int f = 0;
#pragma unroll
    for (int i = 0; i < ps; ++i)
#pragma unroll
        for (int j = i; j < ps; ++j) v.Bm[i][j] = b[64 * f++];
#pragma unroll
    for (int i = 0; i < p2; ++i)
#pragma unroll
        for (int j = i; j < p2; ++j) v.Cm[i][j] = b[64 * f++];
#pragma unroll
    for (int i = 0; i < p1; ++i)
#pragma unroll
        for (int j = 0; j < ps; ++j) v.D[i][j] = b[64 * f++];
#pragma unroll
    for (int i = 0; i < ps; ++i)
#pragma unroll
        for (int j = 0; j < p2; ++j) v.E[i][j] = b[64 * f++];
#pragma unroll
    for (int i = 0; i < ps; ++i) v.mu[i] = b[64 * f++];
#pragma unroll
    for (int i = 0; i < p2; ++i) v.la[i] = b[64 * f++];
}

// final multipliers of knot k (class C) from its slab and knot k+1's (class Cn, final μ, λ
// already in vn.mu / vn.la).  backward_substitution!, cholesky_solve.jl:119-143.
template <class C, class Cn>
__device__ __forceinline__ void bwd_knot(SlabV<C> &v, const SlabV<Cn> &vn)
{
    constexpr int ps = C::PS, p2 = C::P2;
    if constexpr (!Cn::none) {
#pragma unroll
        for (int i = 0; i < p2; ++i) {                            // λ += D' μ' + F' λ'
            double s = v.la[i];
#pragma unroll
            for (int q = 0; q < Cn::PS; ++q) s = fma(vn.D[i][q], vn.mu[q], s);
#pragma unroll
            for (int q = 0; q < Cn::P2; ++q) s = fma(vn.F[i][q], vn.la[q], s);
            v.la[i] = s;
        }
        if constexpr (p2 > 0) trsv_n<p2>(v.Cm, v.la);
#pragma unroll
        for (int i = 0; i < ps; ++i) {                            // μ -= E λ
            double s = v.mu[i];
#pragma unroll
            for (int q = 0; q < p2; ++q) s = fma(-v.E[i][q], v.la[q], s);
            v.mu[i] = s;
        }
        if constexpr (ps > 0) trsv_n<ps>(v.Bm, v.mu);
#pragma unroll
        for (int i = 0; i < p2; ++i) v.la[i] = -v.la[i];
#pragma unroll
        for (int i = 0; i < ps; ++i) v.mu[i] = -v.mu[i];
    } else {                                                       // terminal :139-143
        if constexpr (ps > 0) trsv_n<ps>(v.Bm, v.mu);
#pragma unroll
        for (int i = 0; i < ps; ++i) v.mu[i] = -v.mu[i];
    }
}

// calc_residual! + calc_primals! of knot k (class C): needs λ_{k-1} (lp, class Cp's λ),
// μ_k, λ_k (v).  cholesky_solver.jl:195-236 (SOC: :263-266).
template <class S, class C> struct KnotIn {      // a staged knot's Y, H, g in registers
    double Y[S::template LY<C>()], H[S::template LH<C>()], g[S::template Lg<C>()];
    __device__ __forceinline__ void load(const Buf<S> &b, int lane)
    {
        b.template ld_Y<C>(lane, Y);
        if constexpr (S::GINV) {
            b.template ld_H<C>(lane, H);
            b.template ld_g<C>(lane, g);
        }
    }
};

template <class S, class C, int NLP>
__device__ __forceinline__ void primal_knot(const Ctx<S> &c, int k, const SlabV<C> &v, const double (&lp)[Z(NLP)],
                                            const KnotIn<S, C> &in, uint32_t ring = 0)
{
    constexpr int R = C::R, W = C::W;
    static_assert(NLP == C::P1, "λ_{k-1} has n1[k] entries");
    const auto &Y = in.Y;
    double z[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
        double s = 0.0;
        if constexpr (LQRX_FIL_ABL & 8) {
            z[j] = Y[j] * (C::P2 ? v.la[0] : 1.0);
            continue;
        }
#pragma unroll
        for (int i = 0; i < C::P2; ++i) s = fma(Y[(C::O2 + i) + j * R], v.la[i], s);   // D1ᵀλ_k
#pragma unroll
        for (int i = 0; i < C::PS; ++i) s = fma(Y[(C::OS + i) + j * R], v.mu[i], s);   // Cᵀμ_k
#pragma unroll
        for (int i = 0; i < C::P1; ++i) s = fma(Y[(C::O1 + i) + j * R], lp[i], s);     // D2ᵀλ_{k-1}
        z[j] = s;
    }
    if constexpr (S::GINV) {
        const auto &g = in.g;
        const auto &H = in.H;
#pragma unroll
        for (int j = 0; j < W; ++j) z[j] += g[j];                                     // add_gradient!
        if constexpr (S::HDIAG) {
#pragma unroll
            for (int j = 0; j < W; ++j) z[j] *= rcp_nr2(H[j]);
        } else {
            double U[W][W];
#pragma unroll
            for (int j = 0; j < W; ++j)
#pragma unroll
                for (int i = 0; i <= j; ++i) U[i][j] = H[i + j * W];
            (void)potrf_inv<W>(U);
            trsv_t<W>(U, z);
            trsv_n<W>(U, z);
        }
    }
    if constexpr ((LQRX_FIL_ABL & 64) != 0) return;
    if constexpr (S::SOA) {                                       // coalesced 512-B rows
        // every lane stores (a dead lane's offset is past the buffer's range: dropped), so no
        // exec branch changes the count of vector-memory ops the hand-placed vmcnt bounds rely on
        const uint32_t vo = c.live ? c.vdz : 0xFFFFFF00u;
#pragma unroll
        for (int j = 0; j < W; ++j) bstore(-z[j], make_rsrc(c.bdz), vo, (uint32_t)(Off<S>::g(k) + j) * c.rowb);
    } else {                                                      // dense image, every lane
        double nz[W];
#pragma unroll
        for (int j = 0; j < W; ++j) nz[j] = -z[j];
        if (ring) {                                               // output ring (layout 0, interior)
#pragma unroll
            for (int j = 0; j < W; ++j) *(lds_dw *)(size_t)(ring + 8u * j) = nz[j];
        } else if constexpr (S::PAD) {
            const Rt rt = c.rt.fresh();
            const int lr = std::is_same<C, typename S::L>::value ? rt.nx : (int)rt.Lg;
            c.template out_store_pad<W, std::is_same<C, typename S::I>::value>(
                nz, c.ozb, (const StPat<W> *)(const void *)&c.pz, c.sgz, c.bdz, rt.og(k), lr,
                [&](int j) { return rt.template col<S, C>(j); });
        } else {
            c.template out_store<W, S::I::W>(nz, c.ozi, c.pz, c.sgz, c.bdz, Off<S>::g(k));
        }
    }
}

template <class S, class C>
__device__ __forceinline__ void store_lam(const Ctx<S> &c, int k, const SlabV<C> &v, uint32_t ring = 0)
{
    if constexpr ((LQRX_FIL_ABL & 64) != 0) return;
    if constexpr (S::SOA) {                                       // (dead lanes: out of range)
        const uint32_t r0 = (uint32_t)Off<S>::y(k), vo = c.live ? c.vlam : 0xFFFFFF00u;
#pragma unroll
        for (int i = 0; i < C::PS; ++i) bstore(v.mu[i], make_rsrc(c.blam), vo, (r0 + i) * c.rowb);
#pragma unroll
        for (int i = 0; i < C::P2; ++i) bstore(v.la[i], make_rsrc(c.blam), vo, (r0 + C::PS + i) * c.rowb);
        return;
    } else {                                                      // [μ_k; λ_k], dense image
        constexpr int LL = C::PS + C::P2;
        if constexpr (LL > 0) {
            double lv[LL];
#pragma unroll
            for (int i = 0; i < C::PS; ++i) lv[i] = v.mu[i];
#pragma unroll
            for (int i = 0; i < C::P2; ++i) lv[C::PS + i] = v.la[i];
            if (ring) {
#pragma unroll
                for (int i = 0; i < LL; ++i) *(lds_dw *)(size_t)(ring + 8u * i) = lv[i];
            } else if constexpr (S::PAD) {
                const Rt rt = c.rt.fresh();
                int p1, ps, p2;
                rt.template cls<S, C>(p1, ps, p2);
                c.template out_store_pad<LL, std::is_same<C, typename S::I>::value>(
                    lv, c.olb, (const StPat<LL> *)(const void *)&c.pl, c.slz, c.blam, rt.oy(k), ps + p2,
                    [&](int i) { return rt.template lrow<S, C>(i); });
            } else {
                c.template out_store<LL, Z(S::I::PS + S::I::P2)>(lv, c.oli, c.pl, c.slz, c.blam, Off<S>::y(k));
            }
        }
    }
}

// Start of forward step k (class C; Cnn = class of knot k+2): knot k+1 must have landed.
// After its DMA (issued at step k-2) came the slab stores of step k-2 (not counted:
// conservative), the DMA of knot k+2 (≥ Dmin<Cnn> instructions) and the slab stores of
// step k-1 (single-double stores, ≥ the smaller of the F / C slab sizes).  Step 0 has no
// stores before it.  Then knot k+3 is restaged into knot k's (consumed) buffer.  G: knot k+1's
// group counted from the most recent (2 while a step restages knot k+3; 1 after the last one).
template <class S, class C, class Cnn, bool FIRST, int G = 2>
__device__ __forceinline__ void fwd_wait()
{
    constexpr int sF = S::template slab<typename S::F>(), sC = S::template slab<C>();
    constexpr int Sprev = FIRST ? 0 : (sF < sC ? sF : sC);
    vm_wait<S::template Dmin<Cnn>() + Sprev, G>();
}

// ------------------------------------------------------------------ layout-0 output ring
// The layout-0 δz / λ chunks of one knot are 40-B pieces 4 KB apart (one per trajectory); L2
// writes their lines back partially before the neighbouring knots fill them.  Interior steps of
// the staged kernel instead put their chunks into an LDS image of a group of OR_G knots —
// per trajectory the group's δz run ([t][OR_G·W]) and λ run ([t][OR_G·L]), in memory order — and
// the image of the previous group leaves during the next group's steps, W + L store instructions
// per step (exactly the count of the direct stores it replaces, so the hand-counted vmcnt bounds
// are unchanged; the first group's steps issue out-of-range stores).  Instruction f moves
// the image's doubles 64f … 64f + 63: consecutive lanes write consecutive doubles of one
// trajectory's OR_G-knot run.
constexpr int OR_G = 4;
template <class S> constexpr int or_w() { return S::I::W; }
template <class S> constexpr int or_l() { return S::I::PS + S::I::P2; }
template <class S> constexpr int or_doubles() { return OR_G * 64 * (or_w<S>() + or_l<S>()); }   // one group image
// flush instructions f ∈ [f0, f0 + NF) of the group image at LDS byte address img whose δz run
// starts at element offset oz and λ run at ol; valid = false: out-of-range stores (dropped)
template <class S, int NF>
__device__ __forceinline__ void or_flush(const Ctx<S> &c, uint32_t img, int f0, int64_t oz, int64_t ol, bool valid)
{
    constexpr int RZ = OR_G * or_w<S>(), RL = OR_G * or_l<S>();
    const rsrc_t rz = make_rsrc(c.bdz), rl = make_rsrc(c.blam);
#pragma unroll
    for (int u = 0; u < NF; ++u) {
        const int f = f0 + u;
        const bool isz = f < RZ;
        const uint32_t p = 64u * (uint32_t)(isz ? f : f - RZ) + (uint32_t)c.lane;
        const uint32_t run = isz ? (uint32_t)RZ : (uint32_t)RL;
        const uint32_t tr = p / run, e = p - tr * run;
        const double v = *(lds_dw *)(size_t)(img + 8u * (isz ? p : 64u * RZ + p));
        const uint32_t vo = (valid && tr < (uint32_t)c.nlive)
                                ? tr * (uint32_t)((isz ? c.sgz : c.slz) * 8) + 8u * e : 0xFFFFFF00u;
        bstore(v, isz ? rz : rl, vo, (uint32_t)((isz ? oz : ol) * 8));
    }
}

// ------------------------------------------------------------------ the kernel
template <class S>
__global__ __launch_bounds__(64) void kkt_fil_kernel(const KktArgs a, double *__restrict__ scratch)
{
    using F = typename S::F;
    using I = typename S::I;
    using L = typename S::L;
    __shared__ __attribute__((aligned(16))) double stg[3 * S::BUF];
    __shared__ __attribute__((aligned(16))) double sl[3 * SLB<S>];
    __shared__ __attribute__((aligned(16))) double ost[S::SOA ? 1 : 64 * (S::WOUT + S::LOUT)];
    // the layout-0 output ring (two group images), where the static LDS allows it
    __shared__ __attribute__((aligned(16))) uint32_t dpad[64];   // stage_fill's target
    constexpr bool RING = !S::SOA && LQRX_FIL_RING &&
                          (3 * S::BUF + 3 * SLB<S> + 64 * (S::WOUT + S::LOUT) + 2 * or_doubles<S>()) * 8 + 256 <=
                              160 * 1024;
    __shared__ __attribute__((aligned(16))) double oring[RING ? 2 * or_doubles<S>() : 1];
    const int N = a.N;                                          // ≥ 4 (host-checked)
    const int64_t t0 = (int64_t)blockIdx.x * 64;
    Ctx<S> c;
    c.lane = threadIdx.x;
    c.lpad = lds_addr(dpad);
    // a.sel (layout 0): wave w solves the trajectories sel[64w ..) of the *nsel selected ones
    // (the SQP's second-order-correction subset); waves past the end leave at once (uniform)
    const int64_t nb = (!S::SOA && a.sel) ? (int64_t)*a.nsel : a.batch;
    if (t0 >= nb) return;
    c.nlive = (int)(nb - t0 < 64 ? nb - t0 : 64);
    c.live = c.lane < c.nlive;
    c.bS = scratch + (int64_t)blockIdx.x * N * S::SLOT * 64;
    c.vS = 8u * c.lane;
    if constexpr (!S::SOA) {
        if (a.sel) c.sel = a.sel + t0;
    }
    if constexpr (S::SOA) {
        // wave bases at trajectory t0 of element row 0; a lane past the batch end reads the
        // next row's first trajectories (or past the array: buffer bounds return 0) — its
        // results are never stored
        c.bY = a.Y + t0;
        c.by = a.y + t0;
        c.bH = a.H + t0;
        c.bg = a.g + t0;
        c.bdz = a.dz + t0;
        c.blam = a.lam + t0;
        c.rowb = (uint32_t)(a.batch * 8);
        c.limY = (uint32_t)((a.sY * a.batch - t0) * 8);
        c.limy = (uint32_t)((a.sy * a.batch - t0) * 8);
        c.limH = (uint32_t)((a.sH * a.batch - t0) * 8);
        c.limg = (uint32_t)((a.sg * a.batch - t0) * 8);
        c.vsoa = (uint32_t)(((c.lane >> 5) * a.batch + 2 * (c.lane & 31)) * 8);
        c.vdz = c.vlam = 8u * c.lane;
    } else {
        const int64_t tb = c.sel ? 0 : t0;                 // base trajectory of the wave's arrays
        const int64_t tl = c.sel ? (int64_t)c.sel[c.live ? c.lane : c.nlive - 1] : c.lane;
        c.bY = a.Y + tb * a.sY;
        c.by = a.y + tb * a.sy;
        c.bH = a.H + tb * a.sH;
        c.bg = a.g + tb * a.sg;
        c.bdz = a.dz + tb * a.sg;
        c.blam = a.lam + tb * a.sl;
        c.vdz = (uint32_t)(tl * a.sg * 8);
        c.vlam = (uint32_t)(tl * a.sl * 8);
        c.pY.init(a.sY, c.lane, c.nlive, c.sel);
        c.py.init(a.sy, c.lane, c.nlive, c.sel);
        c.pH.init(a.sH, c.lane, c.nlive, c.sel);
        c.pg.init(a.sg, c.lane, c.nlive, c.sel);
        c.init_out(a, ost);
    }
    int info = 0;

    // ---------------- forward ----------------
    dma_group();
    c.stage_any(a, 0, stg, true);
    dma_group();
    c.stage_I(1, stg + S::BUF, true);
    dma_group();
    c.stage_I(2, stg + 2 * S::BUF, true);               // N ≥ 4: knot 2 is interior
    vm_wait<S::template Dmin<I>() * 2, 3>();            // knot 0
    Shur<F> s0;
    double y0[Z(F::PS + F::P2)];
    {
        Buf<S> b{stg};
        double Yv[S::template LY<F>()], Hv[S::template LH<F>()], gv[S::template Lg<F>()];
        b.template ld_Y<F>(c.lane, Yv);
        b.template ld_H<F>(c.lane, Hv);
        b.template ld_g<F>(c.lane, gv);
        if (!compute_shur<S, F>(s0, Yv, Hv, gv) && info == 0)
            info = -1;
        const auto yk = b.template y<S::template Ly<F>()>(c.lane);
#pragma unroll
        for (int i = 0; i < F::PS + F::P2; ++i) y0[i] = yk[i];
    }
    Carry<S> cy;
#pragma unroll
    for (int i = 0; i < S::NX; ++i) {
        cy.lprev[i] = 0.0;
#pragma unroll
        for (int j = 0; j < S::NX; ++j) cy.Ua[i][j] = 0.0;
    }
    Shur<I> sI;
    double yI[Z(I::PS + I::P2)];
    fwd_wait<S, F, I, true>();
    dma_group();
    c.stage_any(a, 3, stg, true);
    fwd_step<S, F, I, I, true>(a, c, 0, stg, s0, y0, sI, yI, cy, info);
    for (int k = 1; k <= N - 3; ++k) {
        Shur<I> sn;
        double yn[Z(I::PS + I::P2)];
        if (k == N - 3) {
            fwd_wait<S, I, L, false>();                         // (no restage: k+3 = N)
            fwd_step<S, I, I, L>(a, c, k, stg, sI, yI, sn, yn, cy, info);
        } else {
            fwd_wait<S, I, I, false>();
            dma_group();
            c.stage_any(a, k + 3, stg, true);
            fwd_step<S, I, I, I>(a, c, k, stg, sI, yI, sn, yn, cy, info);
        }
        sI = sn;
#pragma unroll
        for (int i = 0; i < I::PS + I::P2; ++i) yI[i] = yn[i];
    }
    Shur<L> sL;
    double yL[Z(L::PS + L::P2)];
    fwd_wait<S, I, NoCls, false, 1>();
    fwd_step<S, I, L, NoCls>(a, c, N - 2, stg, sI, yI, sL, yL, cy, info);
    {
        Shur<NoCls> none;
        factor_knot<S, L, NoCls>(N - 1, sL, yL, none, cy, c, info);
    }

#if LQRX_FIL_ABL & 1
    // ablation (tools only): forward sweep alone
    if (a.info && c.live) a.info[c.sel ? (int64_t)c.sel[c.lane] : t0 + c.lane] = info;
    return;
#endif
    // ---------------- backward + primal recovery ----------------
    // Step j finalises μ_j, λ_j (slab j) and recovers δz_{j+1} (staged knot j+1); it issues
    // the slab of j-2 and knot j-1, both consumed two steps later.  Stores per step: λ/μ of
    // knot j and δz of knot j+1; all of them count in vmcnt like the DMA (lower bounds below).
    // nS: slab DMAs of an interior knot (the L-class chunk of knot N-1 is larger: lower bounds
    // stay valid since it is staged first)
    constexpr int nS = slab_dma_of<S, I>(), nK = S::template Dbwd<I>();
    constexpr int stL = L::PS + L::P2, stI = I::PS + I::P2;             // store_lam
    vm_wait<0>();                                               // forward slab stores landed
    dma_group();
    stage_slab<S, L>(c, N - 1, sl);
    dma_group();
    stage_slab<S, I>(c, N - 2, sl);
    c.stage_any(a, N - 1, stg, false);
    vm_wait<nS + S::template Dbwd<L>(), 2>();                   // slab N-1
    SlabV<L> vL;
    slab_read<S, L>(vL, c, N - 1, sl);
    dma_group();
    stage_slab<S, I>(c, N - 3, sl);                             // N-3 ≥ 1: interior
    c.stage_I(N - 2, stg + ((N - 2) % 3) * S::BUF, false);
    SlabV<NoCls> vnone;
    bwd_knot<L, NoCls>(vL, vnone);                              // step N-1 (no primal)
    store_lam<S, L>(c, N - 1, vL);
    // step N-2: slab N-2, knot N-1 (issued before step N-1's DMA and stores)
    vm_wait<nS + nK + stL, 2>();
    SlabV<I> vI;
    slab_read<S, I>(vI, c, N - 2, sl);
    dma_group();
    stage_slab<S, I>(c, N - 4, sl);                             // (N = 4: the k < 1 filler)
    c.stage_I(N - 3, stg + ((N - 3) % 3) * S::BUF, false);
    bwd_knot<I, L>(vI, vL);                                     // class L: no F̃ (p2 = 0)
    {
        KnotIn<S, L> in;
        in.load(Buf<S>{stg + ((N - 1) % 3) * S::BUF}, c.lane);
        primal_knot<S, L, L::P1>(c, N - 1, vL, vI.la, in);
    }
    store_lam<S, I>(c, N - 2, vI);
    // output ring: interior steps q = N−3−j in whole groups of OR_G (q < nq) write to the ring; a
    // trailing partial group stores directly; the last group image leaves after the loop
    const bool ring_on = RING && !c.sel;
    const int nq = ring_on ? ((N - 3) / OR_G) * OR_G : 0;
    const uint32_t rbase = (uint32_t)(size_t)(lptr_t)oring;
    constexpr uint32_t RB = (uint32_t)or_doubles<S>() * 8u;            // bytes per group image
    constexpr int RZ = OR_G * or_w<S>(), RL = OR_G * or_l<S>();
    for (int j = N - 3; j >= 1; --j) {
        // slab j, knot j+1 were issued at step j+2; after them: stores of step j+2, the DMA
        // of step j+1 (slab j-1 — the filler when j < 2 — and knot j) and its stores.
        constexpr int stp = stI + I::W;                         // stores of an interior step
        // (target: the group of step j+2, the second most recent; every group carries a slab
        // DMA — stage_slab's k < 1 filler at the last steps).  At j = N−3 the ops after it are
        // stL + nS + nK + L::W + stI, at j = N−4 L::W + stI + nS + nK + stp, later stp + nS + nK
        // + stp: ONE wait at the smallest of the three (it waits for a few more of step j+2's
        // stores in the steady state) — one bound per loop, so it holds on every compiled path,
        // also those a static check cannot rule out (the loop entering at a later case)
        constexpr int b0 = stL + nS + nK + L::W + stI, b1 = L::W + stI + nS + nK + stp, b2 = stp + nS + nK + stp;
        constexpr int bw = b0 < b1 ? (b0 < b2 ? b0 : b2) : (b1 < b2 ? b1 : b2);
        vm_wait<bw, 2>();
        SlabV<I> v;
        slab_read<S, I>(v, c, j, sl);
        KnotIn<S, I> in;                                        // knot j+1: F̃_{j+1} and δz_{j+1}
        in.load(Buf<S>{stg + ((j + 1) % 3) * S::BUF}, c.lane);
        dma_group();
        stage_slab<S, I>(c, j - 2, sl);                         // (j − 2 < 1: the filler)
        if (j - 1 >= 1) c.stage_I(j - 1, stg + ((j - 1) % 3) * S::BUF, false);
        else c.stage_any(a, 0, stg, false);
        recompute_Ft<S, I>(vI.F, v.Cm, in.Y, in.H);
        bwd_knot<I, I>(v, vI);
        const int q = N - 3 - j;
        if (q < nq) {
            const int g = q / OR_G, sl_ = q % OR_G;
            // 1/OR_G of the previous group's image leaves (group g−1: δz of knots kz … kz+OR_G−1,
            // λ of knots kz−1 …, lowest first in memory)
            const uint32_t prev = rbase + (uint32_t)((g + 1) & 1) * RB;
            const int kz = N - 1 - OR_G * g, kl = kz - 1;
            or_flush<S, or_w<S>() + or_l<S>()>(c, prev, sl_ * (or_w<S>() + or_l<S>()), Off<S>::g(kz), Off<S>::y(kl), g > 0);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t cur = rbase + (uint32_t)(g & 1) * RB;
            const int pos = OR_G - 1 - sl_;                    // this step's knots in memory order
            primal_knot<S, I, I::P1>(c, j + 1, vI, v.la, in, cur + 8u * (uint32_t)(c.lane * RZ + pos * or_w<S>()));
            store_lam<S, I>(c, j, v, cur + 8u * (uint32_t)(64 * RZ + c.lane * RL + pos * or_l<S>()));
        } else {
            primal_knot<S, I, I::P1>(c, j + 1, vI, v.la, in);
            store_lam<S, I>(c, j, v);
        }
        vI = v;
    }
    if (nq > 0) {
        // the last ring group leaves whole
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int gl = nq / OR_G - 1;
        const int kz = N - 2 - OR_G * gl - (OR_G - 1), kl = kz - 1;
        or_flush<S, RZ + RL>(c, rbase + (uint32_t)(gl & 1) * RB, 0, Off<S>::g(kz), Off<S>::y(kl), true);
    }
    {
        // step 0: multipliers of knot 0 (its class-F slab is the wider one: a register load,
        // once), primal of knot 1, then primal of knot 0
        SlabV<F> v0;
        slab_load<S, F>(v0, c, 0);
        vm_wait<0>();
        KnotIn<S, I> in1;
        in1.load(Buf<S>{stg + (1 % 3) * S::BUF}, c.lane);
        recompute_Ft<S, I>(vI.F, v0.Cm, in1.Y, in1.H);
        bwd_knot<F, I>(v0, vI);
        primal_knot<S, I, I::P1>(c, 1, vI, v0.la, in1);
        store_lam<S, F>(c, 0, v0);
        KnotIn<S, F> in0;
        in0.load(Buf<S>{stg}, c.lane);
        double none[1] = {0.0};
        primal_knot<S, F, 0>(c, 0, v0, none, in0);
    }
    if (a.info && c.live) a.info[t0 + c.lane] = info;
}

// ------------------------------------------------------------------ the direct variant
// Shapes whose knot images do not fit the three-deep LDS ring (e.g. DoubleIntegrator(3):
// 13×9 Y blocks, 60 KB per staged knot image of 64 trajectories) run the same per-knot code
// with each lane reading its own trajectory's Y/H/g/y straight from HBM (compile-time
// offsets, no LDS): a lane streams a contiguous chunk per knot, its 64 neighbours the chunks
// of the next trajectories; L2 absorbs the partial lines.  Same operation order as the staged
// kernel, so the two agree bit for bit on a shape both serve.
// element e of trajectory t's packed array (length len) starting at offset off: layout 0
// [t·len + off + e], layout 1 [(off + e)·batch + t] — one coalesced 512-B row per element for
// the wave, loaded with the row offset in the scalar offset (32-bit, uniform) and the lane's
// trajectory in the vector offset (dead lanes hold the last live trajectory: always in range)
template <class S>
__device__ __forceinline__ double gld(const double *base, int64_t t, int64_t len, int64_t off, int e, int64_t batch)
{
    if constexpr (S::SOA) {
        const int64_t t0 = (int64_t)blockIdx.x * 64;
        return bload(make_rsrc(base + t0), (uint32_t)(t - t0) * 8u, (uint32_t)((off + e) * batch * 8));
    } else {
        return base[t * len + off + e];
    }
}

// padded shapes (S::PAD): element (i, j) of knot k's Y (class C), H's diagonal, g, y — 0
// (H: 1) at padded positions; uniform branches, the real entries at the structure's offsets
// A column's rows come as one scalar offset per row segment plus the row in the instruction's
// immediate offset (a knot needs a few scalar registers, not one per element).  First and
// interior knots (OVER): a padded row past a segment's real rows reads the real data that
// follows it — the next segment, column or knot of the same trajectory, always inside the
// array — and the value is discarded by a uniform select (no branch: the loads stay one
// cluster).  The last knot has nothing after it: its padded rows are not read (uniform
// branches).  A padded column reads the knot's first column, discarded the same way.
template <int S0, int LS, bool OVER>
__device__ __forceinline__ void pad_seg(double *v, rsrc_t r, uint32_t vo, int64_t base, int ls, bool real)
{
    const uint32_t so = (uint32_t)(base * 8);
#pragma unroll
    for (int i = 0; i < LS; ++i) {
        const bool keep = real && i < ls;
        if constexpr (OVER) {
            const double x = bload(r, vo + 8u * (uint32_t)i, so);
            v[S0 + i] = keep ? x : 0.0;
        } else {
            double x = 0.0;
            if (keep) x = bload(r, vo + 8u * (uint32_t)i, so);
            v[S0 + i] = x;
        }
    }
}
// rows [0, NR) of padded column j of knot k's Y (class C): NR = C::R, or C::P1 for the head
template <class S, class C, int NR>
__device__ __forceinline__ void pad_Ycol(const Rt &rt, int k, int j, double *v)
{
    int p1, ps, p2;
    rt.cls<S, C>(p1, ps, p2);
    const int cj = rt.col<S, C>(j);
    const bool real = cj >= 0;
    const int64_t cb = rt.oY(k) + (real ? (int64_t)cj * (p1 + ps + p2) : 0);
    const rsrc_t r = make_rsrc(rt.bY);
    constexpr bool OVER = !std::is_same<C, typename S::L>::value;
    pad_seg<0, (NR < C::P1 ? NR : C::P1), OVER>(v, r, rt.vY, cb, p1, real);
    if constexpr (NR > C::P1) {
        pad_seg<C::P1, C::PS, OVER>(v, r, rt.vY, cb + p1, ps, real);
        pad_seg<C::P1 + C::PS, C::P2, OVER>(v, r, rt.vY, cb + p1 + ps, p2, real);
    }
}
// H, g: a padded column reads the knot's first column (every knot has one) and discards it
template <class S, class C>
__device__ __forceinline__ double pad_H(const KktArgs &, const Rt &rt, int64_t, int k, int j)
{
    const int cj = rt.col<S, C>(j);
    const double x = bload(make_rsrc(rt.bH), rt.vH, (uint32_t)((rt.og(k) + (cj < 0 ? 0 : cj)) * 8));
    return cj < 0 ? 1.0 : x;
}
template <class S, class C>
__device__ __forceinline__ double pad_g(const KktArgs &, const Rt &rt, int64_t, int k, int j)
{
    const int cj = rt.col<S, C>(j);
    const double x = bload(make_rsrc(rt.bg), rt.vg, (uint32_t)((rt.og(k) + (cj < 0 ? 0 : cj)) * 8));
    return cj < 0 ? 0.0 : x;
}
// y: a padded row of a first / interior knot reads the chunk's first element (non-empty: it
// holds the knot's D1 rows); the last knot's chunk can be empty, so its padded rows are skipped
template <class S, class C>
__device__ __forceinline__ double pad_y(const KktArgs &, const Rt &rt, int64_t, int k, int i)
{
    const int ri = rt.lrow<S, C>(i);
    if constexpr (std::is_same<C, typename S::L>::value) {
        double x = 0.0;
        if (ri >= 0) x = bload(make_rsrc(rt.by), rt.vy, (uint32_t)((rt.oy(k) + ri) * 8));
        return x;
    } else {
        const double x = bload(make_rsrc(rt.by), rt.vy, (uint32_t)((rt.oy(k) + (ri < 0 ? 0 : ri)) * 8));
        return ri < 0 ? 0.0 : x;
    }
}

template <class S, class C> struct GIn {          // knot k's inputs (class C) of one trajectory
    double Y[S::template LY<C>()], H[S::template LH<C>()], g[S::template Lg<C>()];
    __device__ __forceinline__ void load(const KktArgs &a, const Rt &rt0, int64_t t, int k)
    {
        using O = Off<S>;
        if constexpr (S::PAD) {
            const Rt rt = rt0.fresh();
#pragma unroll
            for (int j = 0; j < C::W; ++j) pad_Ycol<S, C, C::R>(rt, k, j, Y + j * C::R);
            if constexpr (S::GINV) {
#pragma unroll
                for (int e = 0; e < S::template LH<C>(); ++e) H[e] = pad_H<S, C>(a, rt, t, k, e);
#pragma unroll
                for (int e = 0; e < S::template Lg<C>(); ++e) g[e] = pad_g<S, C>(a, rt, t, k, e);
            }
            return;
        }
#pragma unroll
        for (int e = 0; e < S::template LY<C>(); ++e) Y[e] = gld<S>(a.Y, t, a.sY, O::Y(k), e, a.batch);
        if constexpr (S::GINV) {
#pragma unroll
            for (int e = 0; e < S::template LH<C>(); ++e) H[e] = gld<S>(a.H, t, a.sH, O::H(k), e, a.batch);
#pragma unroll
            for (int e = 0; e < S::template Lg<C>(); ++e) g[e] = gld<S>(a.g, t, a.sg, O::g(k), e, a.batch);
        }
    }
    __device__ __forceinline__ const KnotIn<S, C> &as_in() const { return *reinterpret_cast<const KnotIn<S, C> *>(this); }
};

// Schur pieces of knot k (class C, diagonal H or the SOC variant) in two parts, each streamed
// from HBM column by column, same per-entry operation order as compute_shur:
//   HEAD: the D2×D2 block S[O1..][O1..] and r[O1..] — all that knot k−1's factor needs
//         (added to its C̃ block, copy_shur! :166, :277), computed one knot ahead;
//   REST: everything knot k's own factor reads (the D2×(C, D1) rows and the C, D1 rows).
// Only one full Schur image is live at a time (plus the p1×p1 head of the next knot).
template <class S, class C, bool HEAD>
__device__ __forceinline__ void shur_part(Shur<C> &sc, const KktArgs &a, const Rt &rt0, int64_t t, int k)
{
    const Rt rt = S::PAD ? rt0.fresh() : rt0;
    static_assert(!S::GINV || S::HDIAG, "direct kernel: diagonal H or the SOC variant");
    constexpr int R = C::R, W = C::W, p1 = C::P1;
    constexpr int lo = 0, hi = HEAD ? p1 : R;                     // rows i in [lo, hi)
    auto Yp = [&](int e) { return gld<S>(a.Y, t, a.sY, Off<S>::Y(k), e, a.batch); };
    auto Hp = [&](int e) {
        if constexpr (S::PAD) return pad_H<S, C>(a, rt, t, k, e);
        else return gld<S>(a.H, t, a.sH, Off<S>::H(k), e, a.batch);
    };
    auto gp = [&](int e) {
        if constexpr (S::PAD) return pad_g<S, C>(a, rt, t, k, e);
        else return gld<S>(a.g, t, a.sg, Off<S>::g(k), e, a.batch);
    };
    auto want = [](int i, int i2) { return HEAD ? (i < p1 && i2 < p1) : !(i < p1 && i2 < p1); };
#pragma unroll
    for (int i = lo; i < hi; ++i) {
        if (HEAD || i >= p1) sc.r[i] = 0.0;
#pragma unroll
        for (int i2 = i; i2 < R; ++i2)
            if (want(i, i2)) sc.S[i][i2] = 0.0;
        // a padded constraint row of this knot's C or D1 block: unit pivot (its row and column
        // stay exact zeros); padded D2 rows are the previous knot's D1 rows, pivoted there
        if constexpr (S::PAD && !HEAD)
            if (i >= p1 && rt.row<S, C>(i) < 0) sc.S[i][i] = 1.0;
    }
#pragma unroll
    for (int j = 0; j < W; ++j) {
        double v[R], vh[R];
        if constexpr (S::PAD) {
            pad_Ycol<S, C, HEAD ? p1 : R>(rt, k, j, v);
        } else {
#pragma unroll
            for (int i = 0; i < R; ++i)
                if (!HEAD || i < p1) v[i] = Yp(i + j * R);
        }
        if constexpr (S::GINV) {
            const double h = rcp_nr2(Hp(j));                      // block_cholesky.jl:86 inv
            const double gh = gp(j);
#pragma unroll
            for (int i = lo; i < hi; ++i) {
                vh[i] = v[i] * h;
                if (HEAD || i >= p1) sc.r[i] = fma(vh[i], gh, sc.r[i]);
            }
        } else {
#pragma unroll
            for (int i = lo; i < hi; ++i) vh[i] = v[i];
        }
#pragma unroll
        for (int i = lo; i < hi; ++i)
#pragma unroll
            for (int i2 = i; i2 < R; ++i2)
                if (want(i, i2)) sc.S[i][i2] = fma(vh[i], v[i2], sc.S[i][i2]);
    }
}

template <class S, class C>
__device__ __forceinline__ void y_direct(double (&yc)[Z(C::PS + C::P2)], const KktArgs &a, const Rt &rt0, int64_t t, int k)
{
    const Rt rt = S::PAD ? rt0.fresh() : rt0;
#pragma unroll
    for (int i = 0; i < C::PS + C::P2; ++i) {
        if constexpr (S::PAD) yc[i] = pad_y<S, C>(a, rt, t, k, i);
        else yc[i] = gld<S>(a.y, t, a.sy, Off<S>::y(k), i, a.batch);
    }
}

template <class S>
__global__ __launch_bounds__(64) void kkt_fild_kernel(const KktArgs a, double *__restrict__ scratch)
{
    using F = typename S::F;
    using I = typename S::I;
    using L = typename S::L;
    __shared__ __attribute__((aligned(16))) double ost[S::SOA ? 1 : 64 * (S::WOUT + S::LOUT)];
    const int N = a.N;                                          // ≥ 4 (host-checked)
    // LPW live trajectories per wave (fild_lpw: 32 on small layout-0 batches, the other lanes
    // shadow the last live one); layout 1 keeps 64 (gld's row base)
    const int LPW = S::SOA ? 64 : a.lpw;
    const int64_t t0 = (int64_t)blockIdx.x * LPW;
    Ctx<S> c;
    c.lane = threadIdx.x;
    c.nlive = (int)(a.batch - t0 < LPW ? a.batch - t0 : LPW);
    c.live = c.lane < c.nlive;
    const int64_t t = t0 + (c.live ? c.lane : c.nlive - 1);     // dead lanes re-read a live one
    c.bS = scratch + (int64_t)blockIdx.x * N * S::SLOT * 64;
    c.vS = 8u * c.lane;
    if constexpr (S::SOA) {
        c.bdz = a.dz + t0;
        c.blam = a.lam + t0;
        c.rowb = (uint32_t)(a.batch * 8);
        c.vdz = c.vlam = 8u * c.lane;
    } else {
        c.bdz = a.dz + t0 * a.sg;
        c.blam = a.lam + t0 * a.sl;
        c.vdz = (uint32_t)(c.lane * a.sg * 8);
        c.vlam = (uint32_t)(c.lane * a.sl * 8);
        if constexpr (S::PAD) {
            c.rt.init(a);
            c.rt.lanes(a, t0, t);
        }
        c.init_out(a, ost);
    }
    int info = 0;

    // ---------------- forward ----------------
    // (diagonal H has no factor to fail: compute_shur's ok is always true on this path)
    Carry<S> cy;
#pragma unroll
    for (int i = 0; i < S::NX; ++i) {
        cy.lprev[i] = 0.0;
#pragma unroll
        for (int j = 0; j < S::NX; ++j) cy.Ua[i][j] = 0.0;
    }
    {
        Shur<F> s0;
        double y0[Z(F::PS + F::P2)];
        shur_part<S, F, false>(s0, a, c.rt, t, 0);                    // F: p1 = 0, REST = all
        y_direct<S, F>(y0, a, c.rt, t, 0);
        Shur<I> h1;
        shur_part<S, I, true>(h1, a, c.rt, t, 1);
        factor_knot<S, F, I>(0, s0, y0, h1, cy, c, info);
    }
    for (int k = 1; k <= N - 3; ++k) {
        Shur<I> sk;
        double yk[Z(I::PS + I::P2)];
        shur_part<S, I, false>(sk, a, c.rt, t, k);
        y_direct<S, I>(yk, a, c.rt, t, k);
        Shur<I> hn;
        shur_part<S, I, true>(hn, a, c.rt, t, k + 1);
        factor_knot<S, I, I>(k, sk, yk, hn, cy, c, info);   // (knot k's own HEAD went to k−1)
    }
    Shur<L> sL;
    double yL[Z(L::PS + L::P2)];
    {
        Shur<I> sk;
        double yk[Z(I::PS + I::P2)];
        shur_part<S, I, false>(sk, a, c.rt, t, N - 2);
        y_direct<S, I>(yk, a, c.rt, t, N - 2);
        shur_part<S, L, true>(sL, a, c.rt, t, N - 1);
        factor_knot<S, I, L>(N - 2, sk, yk, sL, cy, c, info);
    }
    shur_part<S, L, false>(sL, a, c.rt, t, N - 1);
    y_direct<S, L>(yL, a, c.rt, t, N - 1);
    {
        Shur<NoCls> none;
        factor_knot<S, L, NoCls>(N - 1, sL, yL, none, cy, c, info);
    }

    // ---------------- backward + primal recovery ----------------
    SlabV<L> vL;
    slab_load<S, L>(vL, c, N - 1);
    SlabV<NoCls> vnone;
    bwd_knot<L, NoCls>(vL, vnone);
    store_lam<S, L>(c, N - 1, vL);
    SlabV<I> vI;
    slab_load<S, I>(vI, c, N - 2);
    bwd_knot<I, L>(vI, vL);
    {
        GIn<S, L> in;
        in.load(a, c.rt, t, N - 1);
        primal_knot<S, L, L::P1>(c, N - 1, vL, vI.la, in.as_in());
    }
    store_lam<S, I>(c, N - 2, vI);
    for (int j = N - 3; j >= 1; --j) {
        SlabV<I> v;
        slab_load<S, I>(v, c, j);
        GIn<S, I> in;                                            // knot j+1: F̃_{j+1} and δz_{j+1}
        in.load(a, c.rt, t, j + 1);
        recompute_Ft<S, I>(vI.F, v.Cm, in.Y, in.H);
        bwd_knot<I, I>(v, vI);
        primal_knot<S, I, I::P1>(c, j + 1, vI, v.la, in.as_in());
        store_lam<S, I>(c, j, v);
        vI = v;
    }
    {
        SlabV<F> v0;
        slab_load<S, F>(v0, c, 0);
        GIn<S, I> in1;
        in1.load(a, c.rt, t, 1);
        recompute_Ft<S, I>(vI.F, v0.Cm, in1.Y, in1.H);
        bwd_knot<F, I>(v0, vI);
        primal_knot<S, I, I::P1>(c, 1, vI, v0.la, in1.as_in());
        store_lam<S, F>(c, 0, v0);
        GIn<S, F> in0;
        in0.load(a, c.rt, t, 0);
        double none[1] = {0.0};
        primal_knot<S, F, 0>(c, 0, v0, none, in0.as_in());
    }
    if (a.info && c.live) a.info[t0 + c.lane] = info;
}

// live trajectories per wave of the direct kernel.  A/B (LQRX_FILD_LPW=32: a layout-0 batch
// ≤ 32768 runs 32 per wave, twice the waves) measured slower at B = 16384 — (6,2,101) 2.24 →
// 2.60 ms, (8,4,101) 6.24 → 7.75, (5,2,101) 1.38 → 1.54, DoubleIntegrator(3) 2.64 → 2.91
// (profiles/r05/r): the kernel is bound by its waves' instruction issue, not by loads in flight
#ifndef LQRX_FILD_LPW
#define LQRX_FILD_LPW 64
#endif
template <class S> int fild_lpw(const KktArgs &a)
{
    return (!S::SOA && a.batch <= 32768) ? LQRX_FILD_LPW : 64;
}
template <class S> size_t slab_bytes(const KktArgs &a)
{
    const int lpw = fild_lpw<S>(a);   // (also the LDS-ring kernel's bound at 64: ≥ its need)
    const size_t Bp = (((size_t)a.batch + lpw - 1) / lpw) * 64;   // wave-major slab, 64 lanes/wave
    // (+1 KiB: the backward slab DMA of the last knot may read up to 512 B past its chunk)
    return Bp * (size_t)a.N * S::SLOT * sizeof(double) + 1024;
}

template <class S, bool DIRECT = false>
hipError_t launch(const KktArgs &a, hipStream_t s)
{
    Scratch sc;
    hipError_t e = sc.get(a, slab_bytes<S>(a), s);
    if (e != hipSuccess) return e;
    if constexpr (DIRECT) {
        KktArgs b = a;
        b.lpw = fild_lpw<S>(a);
        dim3 grid((unsigned)((a.batch + b.lpw - 1) / b.lpw)), block(64);
        hipLaunchKernelGGL((kkt_fild_kernel<S>), grid, block, 0, s, b, (double *)sc.p);
    } else {
        dim3 grid((unsigned)((a.batch + 63) / 64)), block(64);
        hipLaunchKernelGGL((kkt_fil_kernel<S>), grid, block, 0, s, a, (double *)sc.p);
    }
    e = hipGetLastError();
    hipError_t ef = sc.release(s);
    return e != hipSuccess ? e : ef;
}

// Explicit instantiations of every dispatched shape: this compiler has dropped the host stub
// of an implicitly instantiated kernel template launched from a conditional (link error).
#define LQRX_FIL_INST1(NX, M, A0, AK, AN, SOA)                                                          \
    template __global__ void kkt_fil_kernel<Shape<NX, M, A0, AK, AN, true, true, SOA>>(const KktArgs, double *__restrict__);  \
    template __global__ void kkt_fil_kernel<Shape<NX, M, A0, AK, AN, false, true, SOA>>(const KktArgs, double *__restrict__); \
    template __global__ void kkt_fil_kernel<Shape<NX, M, A0, AK, AN, true, false, SOA>>(const KktArgs, double *__restrict__);
#define LQRX_FIL_INST(NX, M, A0, AK, AN) LQRX_FIL_INST1(NX, M, A0, AK, AN, false) LQRX_FIL_INST1(NX, M, A0, AK, AN, true)
// diagonal-H variants only (the dense-H staging ring of these shapes exceeds 160 KB of LDS)
#define LQRX_FIL_INST_DIAG1(NX, M, A0, AK, AN, SOA)                                                     \
    template __global__ void kkt_fil_kernel<Shape<NX, M, A0, AK, AN, true, true, SOA>>(const KktArgs, double *__restrict__);  \
    template __global__ void kkt_fil_kernel<Shape<NX, M, A0, AK, AN, true, false, SOA>>(const KktArgs, double *__restrict__);
#define LQRX_FIL_INST_DIAG(NX, M, A0, AK, AN) LQRX_FIL_INST_DIAG1(NX, M, A0, AK, AN, false) LQRX_FIL_INST_DIAG1(NX, M, A0, AK, AN, true)
// direct (no LDS staging) variants, diagonal H
#define LQRX_FILD_INST1(NX, M, A0, AK, AN, SOA)                                                          \
    template __global__ void kkt_fild_kernel<Shape<NX, M, A0, AK, AN, true, true, SOA>>(const KktArgs, double *__restrict__);  \
    template __global__ void kkt_fild_kernel<Shape<NX, M, A0, AK, AN, true, false, SOA>>(const KktArgs, double *__restrict__);
#define LQRX_FILD_INST(NX, M, A0, AK, AN) LQRX_FILD_INST1(NX, M, A0, AK, AN, false) LQRX_FILD_INST1(NX, M, A0, AK, AN, true)
LQRX_FIL_INST(3, 2, 3, 0, 3)
LQRX_FIL_INST_DIAG(4, 1, 4, 0, 4)
LQRX_FILD_INST(6, 3, 6, 1, 6)
LQRX_FILD_INST(4, 2, 4, 1, 4)
LQRX_FILD_INST(5, 2, 5, 0, 5)
LQRX_FILD_INST(7, 3, 7, 0, 7)
LQRX_FILD_INST(6, 2, 6, 0, 6)
LQRX_FILD_INST(8, 4, 8, 0, 8)
// padded direct variants (layout 0, diagonal H and SOC): every smaller trajectory structure
#define LQRX_FILP_INST(NX, M, A0, AK, AN)                                                                 \
    template __global__ void kkt_fild_kernel<Shape<NX, M, A0, AK, AN, true, true, false, true>>(const KktArgs, double *__restrict__); \
    template __global__ void kkt_fild_kernel<Shape<NX, M, A0, AK, AN, true, false, false, true>>(const KktArgs, double *__restrict__);
LQRX_FILP_INST(4, 2, 4, 1, 4)
LQRX_FILP_INST(6, 3, 6, 1, 6)
LQRX_FILP_INST(8, 4, 8, 1, 8)
#undef LQRX_FILP_INST
#undef LQRX_FIL_INST
#undef LQRX_FIL_INST1
#undef LQRX_FIL_INST_DIAG
#undef LQRX_FIL_INST_DIAG1
#undef LQRX_FILD_INST
#undef LQRX_FILD_INST1

// ------------------------------------------------------------------ dense / block-diagonal H
// (BlockCholesky modes 0/1, block_cholesky.jl:55-77) on the diagonal-H kernels: with H_k = UᵀU,
// Z = Y U⁻¹ and gz = U⁻ᵀg the KKT system is the same with H = I (S = ZZᵀ = Y H⁻¹ Yᵀ, r = Z gz
// = Y H⁻¹ g, λ unchanged) and δz = U⁻¹δz'.  The pre-pass (kkt_hz_kernel) writes Z (Y's
// packing) one row per thread, gz (g's packing), a unit diagonal H and U (packed upper, inverse
// diagonal); the diagonal-H kernel solves;
// the post-pass applies U⁻¹ to δz in place and merges `info` in the order the dense-H sweep
// reports it (H_k is factored one step before knot k−1's pivots: a non-SPD H_k, −(k+1), wins
// over a pivot failure at knot ≥ k−1).  One thread per (trajectory, knot), w ≤ WM.
// One thread per (trajectory, knot, row of Y): the rows of a knot are consecutive threads, so
// their Y loads and Z stores are one contiguous run per column and their H loads the same
// addresses; every thread factors H_k = UᵀU itself (w ≤ 10: cheaper than a pass that stores U
// for the others to re-read), forms z = y U⁻¹ of its row, and the knot's row-0 thread also
// writes gz = U⁻ᵀg, the unit diagonal, the packed U for the post-pass and the H-failure knot.
// The trajectory form's row counts give the knot in closed form.
template <int WM>
__global__ __launch_bounds__(256) void kkt_hz_kernel(const KktArgs a, double *__restrict__ Z, double *__restrict__ gz,
                                                    double *__restrict__ ones, double *__restrict__ Up,
                                                    int32_t *__restrict__ infoh, int64_t sU)
{
    const int N = a.N;
    const int R0 = a.meta[0] + a.meta[1] + a.meta[2], R1 = a.meta[8] + a.meta[9] + a.meta[10];
    const int RL = a.meta[8 * (N - 1)] + a.meta[8 * (N - 1) + 1] + a.meta[8 * (N - 1) + 2];
    const int64_t Rt = (int64_t)R0 + (int64_t)(N - 2) * R1 + RL;     // Y rows per trajectory
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.batch * Rt) return;
    const int64_t t = i / Rt;
    int j = (int)(i - t * Rt), k;
    if (j < R0) {
        k = 0;
    } else if (j < R0 + (N - 2) * R1) {
        j -= R0;
        k = 1 + j / R1;
        j -= (k - 1) * R1;
    } else {
        j -= R0 + (N - 2) * R1;
        k = N - 1;
    }
    const int32_t *m = a.meta + 8 * k;
    const int rows = m[0] + m[1] + m[2], w = m[3];
    const double *H = a.H + t * a.sH + m[6];
    double U[WM][WM];
#pragma unroll
    for (int c = 0; c < WM; ++c)
#pragma unroll
        for (int r = 0; r <= c; ++r) U[r][c] = (c < w) ? H[r + (int64_t)c * w] : (r == c ? 1.0 : 0.0);
    const bool ok = potrf_inv<WM>(U);
    const double *Y = a.Y + t * a.sY + m[4] + j;
    double x[WM];
#pragma unroll
    for (int c = 0; c < WM; ++c) x[c] = c < w ? Y[(int64_t)c * rows] : 0.0;
    trsv_t<WM>(U, x);
    double *Zt = Z + t * a.sY + m[4] + j;
#pragma unroll
    for (int c = 0; c < WM; ++c)
        if (c < w) Zt[(int64_t)c * rows] = x[c];
    if (j == 0) {
        if (!ok) atomicMin(&infoh[t], k);             // first non-SPD knot (pre-set to N)
        const int64_t og = m[7];
        const double *g = a.g + t * a.sg + og;
#pragma unroll
        for (int c = 0; c < WM; ++c) x[c] = c < w ? g[c] : 0.0;
        trsv_t<WM>(U, x);
        double *gzt = gz + t * a.sg + og, *on = ones + t * a.sg + og;
#pragma unroll
        for (int c = 0; c < WM; ++c)
            if (c < w) {
                gzt[c] = x[c];
                on[c] = 1.0;
            }
        // packed-U offset of knot k: every knot before the last has knot 0's w (trajectory form)
        const int w0 = a.meta[3];
        double *Ut = Up + t * sU + (int64_t)k * (w0 * (w0 + 1) / 2);
        int e = 0;
#pragma unroll
        for (int c = 0; c < WM; ++c)
#pragma unroll
            for (int r = 0; r <= c; ++r)
                if (c < w) Ut[e++] = U[r][c];
    }
}

template <int WM>
__global__ __launch_bounds__(256) void kkt_hpost_kernel(const KktArgs a, const double *__restrict__ Up,
                                                       const int32_t *__restrict__ infoh, int64_t sU)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.batch * a.N) return;
    const int64_t t = i / a.N;
    const int k = (int)(i - t * a.N);
    const int32_t *m = a.meta + 8 * k;
    const int w = m[3];
    const int64_t og = m[7];
    // packed-U offset of knot k: every knot before the last has knot 0's w (trajectory form)
    const int w0 = a.meta[3];
    const int64_t oU = (int64_t)k * (w0 * (w0 + 1) / 2);
    const double *Ut = Up + t * sU + oU;
    double U[WM][WM];
    int e = 0;
#pragma unroll
    for (int c = 0; c < WM; ++c)
#pragma unroll
        for (int r = 0; r <= c; ++r) U[r][c] = (c < w) ? Ut[e++] : (r == c ? 1.0 : 0.0);
    double x[WM];
    double *dz = a.dz + t * a.sg + og;
#pragma unroll
    for (int c = 0; c < WM; ++c) x[c] = c < w ? dz[c] : 0.0;
    trsv_n<WM>(U, x);
#pragma unroll
    for (int c = 0; c < WM; ++c)
        if (c < w) dz[c] = x[c];
    if (k == 0 && a.info) {
        // a non-SPD H_k wins over any Schur pivot failure, as in the reference order (every
        // H_k is factored in shur! before cholesky! sees a pivot) and the oracle / the other routes
        const int kh = infoh[t];                      // first non-SPD H knot, or N
        if (kh < a.N) a.info[t] = -(kh + 1);
    }
}

} // namespace fil

// LQRX_KKT_PAD=0 turns off the padded shapes and the dense-H passes (those structures then go
// to the large-block kernels, as before round 4): A/B and cross-checks
static bool fil_ext_on()
{
    static const bool on = [] { const char *e = std::getenv("LQRX_KKT_PAD"); return !(e && *e == '0'); }();
    return on;
}

// Dispatch: the FIL kernel serves a structure iff every knot matches one of the
// instantiated (n̄, m, P0, PK, PN) shapes; otherwise the generic kernel (lqrx_kkt.hip) runs.
// F is called with the matching Shape (diag-H/Ginv, dense-H/Ginv, or SOC) as a value tag.
template <class Fn>
static bool fil_dispatch(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                         const int32_t *w, Fn &&fn)
{
    const int N = a.N;
    if (N < 4) return false;
    const int nx = n2[0], m = w[0] - nx, P0 = p[0], PK = p[1], PN = p[N - 1];
    if (n1[0] != 0 || w[N - 1] != nx || n2[N - 1] != 0 || n1[N - 1] != nx) return false;
    for (int k = 1; k < N - 1; ++k)
        if (n1[k] != nx || n2[k] != nx || p[k] != PK || w[k] != nx + m) return false;
    const bool diag = a.h_mode == 2, ginv = a.ginv != 0, soa = a.layout == 1;
#define LQRX_FIL_SEL(NX, M, A0, AK, AN, SOA)                                                             \
    if (diag && ginv) fn(fil::Shape<NX, M, A0, AK, AN, true, true, SOA>{}, std::false_type{}, a);        \
    else if (ginv) fn(fil::Shape<NX, M, A0, AK, AN, false, true, SOA>{}, std::false_type{}, a);          \
    else fn(fil::Shape<NX, M, A0, AK, AN, true, false, SOA>{}, std::false_type{}, a);
#define LQRX_FIL(NX, M, A0, AK, AN)                                                                      \
    if (nx == NX && m == M && P0 == A0 && PK == AK && PN == AN) {                                        \
        if (soa) { LQRX_FIL_SEL(NX, M, A0, AK, AN, true) }                                               \
        else { LQRX_FIL_SEL(NX, M, A0, AK, AN, false) }                                                  \
        return true;                                                                                     \
    }
#define LQRX_FIL_DIAG(NX, M, A0, AK, AN)                                                                 \
    if (nx == NX && m == M && P0 == A0 && PK == AK && PN == AN && (diag || !ginv)) {                     \
        if (soa) {                                                                                       \
            if (ginv) fn(fil::Shape<NX, M, A0, AK, AN, true, true, true>{}, std::false_type{}, a);       \
            else fn(fil::Shape<NX, M, A0, AK, AN, true, false, true>{}, std::false_type{}, a);           \
        } else {                                                                                         \
            if (ginv) fn(fil::Shape<NX, M, A0, AK, AN, true, true>{}, std::false_type{}, a);             \
            else fn(fil::Shape<NX, M, A0, AK, AN, true, false>{}, std::false_type{}, a);                 \
        }                                                                                                \
        return true;                                                                                     \
    }
#define LQRX_FILD(NX, M, A0, AK, AN)                                                                     \
    if (nx == NX && m == M && P0 == A0 && PK == AK && PN == AN && (diag || !ginv)) {                     \
        if (soa) {                                                                                       \
            if (ginv) fn(fil::Shape<NX, M, A0, AK, AN, true, true, true>{}, std::true_type{}, a);        \
            else fn(fil::Shape<NX, M, A0, AK, AN, true, false, true>{}, std::true_type{}, a);            \
        } else {                                                                                         \
            if (ginv) fn(fil::Shape<NX, M, A0, AK, AN, true, true>{}, std::true_type{}, a);              \
            else fn(fil::Shape<NX, M, A0, AK, AN, true, false>{}, std::true_type{}, a);                  \
        }                                                                                                \
        return true;                                                                                     \
    }
    LQRX_FIL(3, 2, 3, 0, 3)        // Dubins car (BASELINE cfg3), test/dubins.jl
    LQRX_FIL_DIAG(4, 1, 4, 0, 4)   // cartpole trajectory problem (test/problems.jl:58-88, device SQP)
    LQRX_FILD(6, 3, 6, 1, 6)       // DoubleIntegrator(3) (test/problems.jl:14-56, test/cholesky_solve.jl)
    LQRX_FILD(4, 2, 4, 1, 4)       // DoubleIntegrator(2)
    LQRX_FILD(5, 2, 5, 0, 5)       // trajectory_structure(5, 2, N), diagonal H (the SQP problems' shape)
    LQRX_FILD(7, 3, 7, 0, 7)       // trajectory_structure(7, 3, N), diagonal H
    LQRX_FILD(6, 2, 6, 0, 6)       // trajectory_structure(6, 2, N) (round 5)
    LQRX_FILD(8, 4, 8, 0, 8)       // trajectory_structure(8, 4, N) (round 5)
    // any other trajectory structure up to a padded bin (layout 0; layout 1 is staged): the
    // smallest bin that holds it, its own sizes at run time (Shape PAD, Rt).  LQRX_KKT_PAD=0
    // sends them to the large-block kernels instead (A/B)
    // (per-lane byte offsets from a wave's base are 32-bit and the buffer range 2 GiB: 64
    // trajectories of every array must span less)
    const int64_t smax = std::max(std::max(a.sY, a.sy), std::max(a.sH, a.sg));
    if (fil_ext_on() && !soa && (diag || !ginv) && nx >= 1 && m >= 0 && P0 >= 0 && PK >= 0 && PN >= 0 &&
        smax * 8 * 64 < (int64_t)INT32_MAX) {
        KktArgs b = a;
        b.rt[0] = nx; b.rt[1] = m; b.rt[2] = P0; b.rt[3] = PK; b.rt[4] = PN;
#define LQRX_FILP(NX, M, A0, AK, AN)                                                                     \
        if (nx <= NX && m <= M && P0 <= A0 && PK <= AK && PN <= AN) {                                    \
            if (ginv) fn(fil::Shape<NX, M, A0, AK, AN, true, true, false, true>{}, std::true_type{}, b);  \
            else fn(fil::Shape<NX, M, A0, AK, AN, true, false, false, true>{}, std::true_type{}, b);     \
            return true;                                                                                 \
        }
        LQRX_FILP(4, 2, 4, 1, 4)
        LQRX_FILP(6, 3, 6, 1, 6)
        LQRX_FILP(8, 4, 8, 1, 8)
#undef LQRX_FILP
    }
#undef LQRX_FIL
#undef LQRX_FIL_SEL
#undef LQRX_FIL_DIAG
#undef LQRX_FILD
    return false;
}

// Dense / block-diagonal H (ginv, layout 0) on a structure whose diagonal-H form a FIL shape
// serves: the pre-pass / diagonal kernel / post-pass of fil::kkt_hz_kernel.  Scratch: Z | gz |
// unit H | packed U | H-failure knots | the diagonal kernel's slab.
namespace {
constexpr int FILH_WM = 10;                           // w ≤ 10: every FIL shape and padded bin
struct FilH {
    int64_t sU = 0;
    size_t oZ = 0, ogz = 0, oon = 0, oU = 0, oinf = 0, oslab = 0, slab = 0, total = 0;
};
bool filh_plan(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2, const int32_t *w,
               KktArgs &b, FilH &P)
{
    // (not for a trajectory subset: the pre/post passes cover the whole batch)
    if (!fil_ext_on() || a.h_mode == 2 || !a.ginv || a.layout != 0 || a.maxw > FILH_WM || a.batch <= 0 || a.sel)
        return false;
    b = a;
    b.h_mode = 2;
    b.sH = a.sg;                                      // unit diagonal H, g's packing
    size_t sb = 0;
    if (!fil_dispatch(b, n1, p, n2, w, [&](auto shape, auto, const KktArgs &c) { sb = fil::slab_bytes<decltype(shape)>(c); }))
        return false;
    for (int k = 0; k < a.N; ++k) P.sU += (int64_t)w[k] * (w[k] + 1) / 2;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t B = (size_t)a.batch;
    P.oZ = 0;
    P.ogz = P.oZ + al(B * (size_t)a.sY * 8);
    P.oon = P.ogz + al(B * (size_t)a.sg * 8);
    P.oU = P.oon + al(B * (size_t)a.sg * 8);
    P.oinf = P.oU + al(B * (size_t)P.sU * 8);
    P.oslab = P.oinf + al(B * 4);
    P.slab = sb;
    P.total = P.oslab + sb;
    return true;
}
} // namespace

bool kkt_fil_launch(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                    const int32_t *w, hipStream_t s, hipError_t *err)
{
    if (fil_dispatch(a, n1, p, n2, w, [&](auto shape, auto direct, const KktArgs &b) {
            *err = fil::launch<decltype(shape), decltype(direct)::value>(b, s);
        }))
        return true;
    KktArgs b;
    FilH P;
    if (!filh_plan(a, n1, p, n2, w, b, P)) return false;
    Scratch sc;
    hipError_t e = sc.get(a, P.total, s);
    if (e != hipSuccess) {
        *err = e;
        return true;
    }
    char *base = (char *)sc.p;
    double *Z = (double *)(base + P.oZ), *gz = (double *)(base + P.ogz), *on = (double *)(base + P.oon),
           *Up = (double *)(base + P.oU);
    int32_t *infoh = (int32_t *)(base + P.oinf);
    const int64_t nt = a.batch * a.N;
    const unsigned grid = (unsigned)((nt + 255) / 256);
    // H-failure knots start at N ("none"): 0x7f7f7f7f ≥ N for every accepted structure
    e = hipMemsetAsync(infoh, 0x7f, (size_t)a.batch * 4, s);
    if (e == hipSuccess) {
        int64_t Rt = 0;
        for (int k = 0; k < a.N; ++k) Rt += n1[k] + p[k] + n2[k];
        hipLaunchKernelGGL((fil::kkt_hz_kernel<FILH_WM>), dim3((unsigned)((a.batch * Rt + 255) / 256)), dim3(256), 0, s,
                           a, Z, gz, on, Up, infoh, P.sU);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        b.Y = Z; b.g = gz; b.H = on;
        b.ws = base + P.oslab;
        b.ws_bytes = P.slab;
        hipError_t e2 = hipSuccess;
        (void)fil_dispatch(b, n1, p, n2, w, [&](auto shape, auto direct, const KktArgs &c) {
            e2 = fil::launch<decltype(shape), decltype(direct)::value>(c, s);
        });
        e = e2;
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL((fil::kkt_hpost_kernel<FILH_WM>), dim3(grid), dim3(256), 0, s, a, Up, infoh, P.sU);
        e = hipGetLastError();
    }
    hipError_t er = sc.release(s);
    *err = e != hipSuccess ? e : er;
    return true;
}

bool kkt_fil_scratch_bytes(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                           const int32_t *w, size_t *bytes)
{
    if (fil_dispatch(a, n1, p, n2, w, [&](auto shape, auto, const KktArgs &b) { *bytes = fil::slab_bytes<decltype(shape)>(b); }))
        return true;
    KktArgs b;
    FilH P;
    if (!filh_plan(a, n1, p, n2, w, b, P)) return false;
    *bytes = P.total;
    return true;
}

} // namespace lqrx
