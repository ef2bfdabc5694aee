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


// number of DMA instructions stage_chunk issues for a chunk of L doubles (same rule)
__host__ __device__ constexpr int stage_instrs(int L, bool wide) { return L <= 0 ? 0 : (wide ? L / 2 : 2 * L); }

} // namespace lqrx
