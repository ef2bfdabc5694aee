// lqrx_stage.h — coalesced LDS-DMA staging of per-trajectory packed knot blocks
// (global_load_lds), shared by the KKT kernels.  The ABI's KKT inputs are packed per
// trajectory (batch slowest), so one knot's block of the 64 trajectories of a wave is 64
// chunks of L doubles at stride s: the DMA walks them as one dense [t][L] image, 16-byte
// pieces when every chunk is 16-B aligned, dwords otherwise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lqrx {

using gptr_t = const __attribute__((address_space(1))) void *;
using lptr_t = __attribute__((address_space(3))) void *;

// stage L doubles at element offset `off` of each of the wave's 64 trajectories (stride s
// elements) into lds[t*L + e].  16-byte pieces when every chunk is 16-B aligned, else dwords.
__device__ __forceinline__ void stage_chunk(const double *X, int64_t s, int64_t off, int L,
                                            int64_t t0, int64_t batch, double *lds, int lane)
{
    if (L <= 0) return;
    const bool wide = ((s | off | L) & 1) == 0;                 // uniform
    const int unit = wide ? 16 : 4;
    const int per = L * 8 / unit;                               // pieces per trajectory
    const int q = 64 / per, r = 64 - q * per;                   // uniform
    int tl = lane / per, e = lane - tl * per;
    const bool full = t0 + 64 <= batch;                         // uniform: no clamp needed
    // running byte address; advancing by (q trajectories, r pieces) per instruction
    const int64_t sb = s * 8;
    const char *gp = (const char *)X + (t0 + tl) * sb + off * 8 + (int64_t)e * unit;
    const int64_t step = q * sb + (int64_t)r * unit, wrap = sb - (int64_t)per * unit;
    for (int i = 0; i < 64 * per; i += 64) {
        const char *src = gp;
        if (!full && t0 + tl >= batch)
            src = (const char *)X + (batch - 1) * sb + off * 8 + (int64_t)e * unit;
        char *lp = (char *)lds + (int64_t)i * unit;
        if (wide)
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lp, 16, 0, 0);
        else
            __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lp, 4, 0, 0);
        tl += q;
        e += r;
        gp += step;
        if (e >= per) {
            e -= per;
            tl += 1;
            gp += wrap;
        }
    }
}


// a raw buffer descriptor (stride 0, full 31-bit range, gfx9 dword-3 format bits) as four
// SGPRs, for the inline-asm LDS-DMA below
typedef uint32_t u4_t __attribute__((ext_vector_type(4)));
// raw buffer resource with an explicit size: loads at offsets ≥ bytes return 0 (no access)
__device__ __forceinline__ u4_t make_rsrc4n(const void *base, uint32_t bytes)
{
    const uint64_t a = (uint64_t)base;
    u4_t r;
    r.x = (uint32_t)a;
    r.y = (uint32_t)(a >> 32) & 0xffffu;
    r.z = bytes;
    r.w = 0x00020000u;
    return r;
}
__device__ __forceinline__ u4_t make_rsrc4(const void *base)
{
    const uint64_t a = (uint64_t)base;
    u4_t r;
    r.x = (uint32_t)a;
    r.y = (uint32_t)(a >> 32) & 0xffffu;
    r.z = 0x7fffffffu;
    r.w = 0x00020000u;
    return r;
}

// One LDS-DMA instruction (buffer_load_dword{,x3,x4} … lds; M0 = the wave's LDS destination,
// each lane's piece lands at M0 + lane·slot).  Issued as inline asm ON PURPOSE: the compiler's
// wait-count pass cannot tell which LDS bytes a DMA writes, so after a DMA issued through the
// builtin it makes EVERY later LDS read wait for it (vmcnt(0) before the first read of the
// knot staged two steps earlier) — which defeats the ring's prefetch entirely.  Issued here the
// DMA is invisible to that pass: completion is tracked by hand (vm_wait<N>, which counts these
// like any vector-memory op) and the "memory" clobber keeps LDS accesses from moving across it.
// M0 is set and NOT restored: M0 is reserved (a clobber of it is not honoured), and the
// kernels including this header leave it unused outside these blocks — which
// tests/test_isa_guards.py checks on the compiled gfx950 assembly (the round-1 save/restore
// pair per DMA cost 4–8 % of the KKT kernel in its latency-bound regimes).
template <int BYTES>
__device__ __forceinline__ void dma_lds(u4_t r, uint32_t vo, uint32_t so, uint32_t lds)
{
    if constexpr (BYTES == 16)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, %3 offen lds" ::"v"(vo), "s"(lds),
                     "s"(r), "s"(so)
                     : "memory");
    else if constexpr (BYTES == 12)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx3 %0, %2, %3 offen lds" ::"v"(vo), "s"(lds),
                     "s"(r), "s"(so)
                     : "memory");
    else {
        static_assert(BYTES == 4, "LDS-DMA piece of 4, 12 or 16 bytes");
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %0, %2, %3 offen lds" ::"v"(vo), "s"(lds),
                     "s"(r), "s"(so)
                     : "memory");
    }
}
__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(size_t)(lptr_t)p; }

// Source marker (an assembly comment, no instruction): the LDS-DMA issued from here up to the
// next marker form one group — the unit a hand-placed wait names as its target
// (`s_waitcnt vmcnt(N) … ; lqrx.wait g=G`: the G-th most recent group must have landed).
// tests/isa_vmcnt.py checks every such bound against the compiled gfx950 instruction stream:
// at least N vector-memory instructions issued after the target group's last DMA, on every path.
__device__ __forceinline__ void dma_group() { asm volatile("; lqrx.grp"); }

// number of DMA instructions stage_chunk issues for a chunk of L doubles (same rule)
__host__ __device__ constexpr int stage_instrs(int L, bool wide) { return L <= 0 ? 0 : (wide ? L / 2 : 2 * L); }

} // namespace lqrx
