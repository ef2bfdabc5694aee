// overlap_probe.hip — does fp64 VALU / v_readlane work of one wave overlap fp64 MFMA of the
// partner wave on the same SIMD?  512-thread workgroups: waves 0-3 (one per SIMD) run the
// MFMA loop, waves 4-7 run a VALU loop.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int MODE>  // bit0: MFMA waves active, bit1: VALU f64 waves active, bit2: readlane waves, bit3: f32 valu
__global__ __launch_bounds__(512) void k(double* out, int iters) {
  int w = threadIdx.x >> 6;
  double res = 0;
  if (w < 4) {
    if (MODE & 1) {
      d4 acc[4]; for (int i = 0; i < 4; ++i) acc[i] = d4{0,0,0,0};
      double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
      for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0,0,0);
      for (int i = 0; i < 4; ++i) res += acc[i][0];
    }
  } else {
    if (MODE & 2) {
      double x0 = threadIdx.x, x1 = x0+1, x2 = x0+2, x3 = x0+3;
      for (int it = 0; it < iters * 8; ++it) { x0 = fma(x0, 0.9999, 1e-7); x1 = fma(x1, 0.9999, 1e-7); x2 = fma(x2, 0.9999, 1e-7); x3 = fma(x3, 0.9999, 1e-7); }
      res = x0 + x1 + x2 + x3;
    }
    if (MODE & 4) {
      int v = threadIdx.x; int acc = 0;
      for (int it = 0; it < iters * 8; ++it) {
        acc += __builtin_amdgcn_readlane(v, it & 63); acc ^= __builtin_amdgcn_readlane(v + acc, 5);
        acc += __builtin_amdgcn_readlane(v ^ acc, 7); acc ^= __builtin_amdgcn_readlane(v + 3, 9);
      }
      res = acc;
    }
    if (MODE & 8) {
      float x0 = threadIdx.x, x1 = x0+1, x2 = x0+2, x3 = x0+3;
      for (int it = 0; it < iters * 8; ++it) { x0 = fmaf(x0, 0.9999f, 1e-7f); x1 = fmaf(x1, 0.9999f, 1e-7f); x2 = fmaf(x2, 0.9999f, 1e-7f); x3 = fmaf(x3, 0.9999f, 1e-7f); }
      res = x0 + x1 + x2 + x3;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = res;
}
template <int MODE> float t(double* out, int iters) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(512), 0, 0, out, 8); hipDeviceSynchronize();
  float best = 1e9;
  for (int r = 0; r < 3; ++r) {
    hipEventRecord(e0); hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(512), 0, 0, out, iters); hipEventRecord(e1);
    hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
  }
  return best;
}
int main() {
  double* out; hipMalloc(&out, 256 * 512 * 8);
  int it = 2048;
  printf("mfma only          %.3f ms\n", t<1>(out, it));
  printf("valu f64 only      %.3f ms\n", t<2>(out, it));
  printf("mfma + valu f64    %.3f ms\n", t<3>(out, it));
  printf("readlane only      %.3f ms\n", t<4>(out, it));
  printf("mfma + readlane    %.3f ms\n", t<5>(out, it));
  printf("valu f32 only      %.3f ms\n", t<8>(out, it));
  printf("mfma + valu f32    %.3f ms\n", t<9>(out, it));
  return 0;
}
