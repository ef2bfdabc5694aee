// mfma_probe.hip — measure fp64 MFMA / VALU throughput on gfx950 (diagnostic only).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int ACC>
__global__ void mfma_f64(double* out, int iters) {
  d4 acc[ACC];
  for (int i = 0; i < ACC; ++i) acc[i] = d4{0,0,0,0};
  double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0,0,0);
  }
  double s = 0; for (int i = 0; i < ACC; ++i) s += acc[i][0]+acc[i][1]+acc[i][2]+acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void valu_f64(double* out, int iters) {
  double x0 = threadIdx.x, x1 = x0+1, x2 = x0+2, x3 = x0+3, x4=x0+4,x5=x0+5,x6=x0+6,x7=x0+7;
  const double a = 0.999999, b = 1e-7;
  for (int it = 0; it < iters; ++it) {
    x0 = fma(x0, a, b); x1 = fma(x1, a, b); x2 = fma(x2, a, b); x3 = fma(x3, a, b);
    x4 = fma(x4, a, b); x5 = fma(x5, a, b); x6 = fma(x6, a, b); x7 = fma(x7, a, b);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0+x1+x2+x3+x4+x5+x6+x7;
}
int main() {
  double* out; hipMalloc(&out, 1 << 24);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int iters = 4096;
  for (int wpb : {1, 2, 4}) {
    int blocks = 256 * 4 * wpb / wpb;  // one block per SIMD-slot
    dim3 g(256 * 4 * wpb / 1), bl(64);
    (void)blocks;
    hipLaunchKernelGGL(mfma_f64<4>, g, bl, 0, 0, out, 16); hipDeviceSynchronize();
    hipEventRecord(e0); hipLaunchKernelGGL(mfma_f64<4>, g, bl, 0, 0, out, iters); hipEventRecord(e1);
    hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1);
    double fl = (double)g.x * iters * 4 * 2048.0;
    printf("mfma_f64_16x16x4 waves=%d (%d/SIMD) : %.2f TFLOP/s (%.3f ms)\n", g.x, wpb, fl / ms / 1e9, ms);
  }
  for (int wps : {1, 2, 4, 8}) {
    dim3 g(256 * 4 * wps), bl(64);
    hipLaunchKernelGGL(valu_f64, g, bl, 0, 0, out, 16); hipDeviceSynchronize();
    hipEventRecord(e0); hipLaunchKernelGGL(valu_f64, g, bl, 0, 0, out, iters); hipEventRecord(e1);
    hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1);
    double fl = (double)g.x * 64 * iters * 8 * 2.0;
    printf("valu v_fma_f64 waves/SIMD=%d : %.2f TFLOP/s\n", wps, fl / ms / 1e9);
  }
  return 0;
}
