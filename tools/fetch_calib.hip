// fetch_calib.hip — calibration of the PMC FETCH_SIZE counter for the load widths the kernels use
// (MI355X_MICROARCH.md's ×2 correction is stated for wide coalesced reads; the KKT kernels also
// read 4-B and 8-B scalars per lane).  Each kernel streams the same 1 GiB buffer exactly once,
// fully coalesced, with one load width; the rocprofv3 FETCH_SIZE per dispatch divided by 1 GiB
// is the counter's scale for that width.  Run:
//   rocprofv3 --pmc FETCH_SIZE -d out -o fc --output-format csv -- ./tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename V>
__global__ __launch_bounds__(256) void stream_sum(const V *__restrict__ x, size_t n, float *__restrict__ out)
{
    float s = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const V v = x[i];
        const float *f = (const float *)&v;
#pragma unroll
        for (int e = 0; e < (int)(sizeof(V) / 4); ++e) s += f[e];
    }
    if (s == 123.456f) out[0] = s;            // keeps the loads; never true for the zero buffer
}

int main()
{
    const size_t bytes = (size_t)1 << 30;
    void *buf = nullptr;
    float *out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc((void **)&out, 4) != hipSuccess) return 1;
    if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
    const dim3 grid(256 * 8 * 4), block(256);
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef float f4 __attribute__((ext_vector_type(4)));
    hipLaunchKernelGGL(stream_sum<float>, grid, block, 0, 0, (const float *)buf, bytes / 4, out);
    hipLaunchKernelGGL(stream_sum<f2>, grid, block, 0, 0, (const f2 *)buf, bytes / 8, out);
    hipLaunchKernelGGL(stream_sum<f4>, grid, block, 0, 0, (const f4 *)buf, bytes / 16, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("fetch_calib: 3 dispatches (4, 8, 16 B per lane), %zu bytes each\n", bytes);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
