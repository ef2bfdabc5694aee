// Probe: LDS layout written by buffer_load_dwordx3 ... lds (12-byte LDS-DMA) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
using lptr_t = __attribute__((address_space(3))) void *;
__global__ void k(const unsigned *X, unsigned *out)
{
    __shared__ unsigned lds[64 * 4 + 64];
    for (int i = threadIdx.x; i < 64 * 5; i += 64) lds[i] = 0xdeadbeef;
    __syncthreads();
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)X, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr_t)lds, 12, threadIdx.x * 12, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 5; i += 64) out[i] = lds[i];
}
int main()
{
    unsigned h[64 * 4], *d, *o, ho[64 * 5];
    for (int i = 0; i < 64 * 4; ++i) h[i] = i;
    hipMalloc(&d, sizeof h); hipMalloc(&o, sizeof ho);
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
    hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
    for (int i = 0; i < 40; ++i) printf("%x ", ho[i]);
    printf("\n... [190..200): ");
    for (int i = 190; i < 200; ++i) printf("%x ", ho[i]);
    printf("\n");
    return 0;
}
