// lat_probe.hip — dependent-chain latency (cycles, s_memtime) of fp64 VALU ops, v_readlane,
// MFMA f64, and the accuracy of v_rcp_f64 / v_rsq_f64.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ inline long long clk() { long long t; asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory"); return t; }
__global__ void lat(double* out, long long* cyc, double seed) {
  double x = seed + threadIdx.x * 1e-9;
  const int N = 256;
  long long t0, t1;
  // fma chain
  t0 = clk();
#pragma unroll 16
  for (int i = 0; i < N; ++i) x = fma(x, 0.99999, 1e-9);
  t1 = clk(); cyc[0] = (t1 - t0); out[0] = x;
  // mul chain
  t0 = clk();
#pragma unroll 16
  for (int i = 0; i < N; ++i) x = x * 1.0000001;
  t1 = clk(); cyc[1] = (t1 - t0); out[1] = x;
  // rcp chain
  t0 = clk();
#pragma unroll 16
  for (int i = 0; i < N; ++i) x = __builtin_amdgcn_rcp(x);
  t1 = clk(); cyc[2] = (t1 - t0); out[2] = x;
  // readlane chain (f64 via 2x b32)
  t0 = clk();
  long long bits = __double_as_longlong(x);
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    int lo = __builtin_amdgcn_readlane((int)bits, 3), hi = __builtin_amdgcn_readlane((int)(bits >> 32), 3);
    bits = (((long long)hi << 32) | (unsigned)lo) + threadIdx.x;
  }
  t1 = clk(); cyc[3] = (t1 - t0); out[3] = (double)bits;
  // readlane -> fma chain (SGPR operand)
  t0 = clk();
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    long long b = __double_as_longlong(x);
    int lo = __builtin_amdgcn_readlane((int)b, 3), hi = __builtin_amdgcn_readlane((int)(b >> 32), 3);
    double s = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
    x = fma(s, 0.99999, x * 1e-9);
  }
  t1 = clk(); cyc[4] = (t1 - t0); out[4] = x;
  // mfma dependent chain
  d4 acc = {x, 0, 0, 0};
  t0 = clk();
#pragma unroll 16
  for (int i = 0; i < N; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, 1e-3, acc, 0, 0, 0);
  t1 = clk(); cyc[5] = (t1 - t0); out[5] = acc[0] + acc[3];
  // ds (LDS) write->read roundtrip chain
  __shared__ double sh[64];
  t0 = clk();
  for (int i = 0; i < N; ++i) { sh[threadIdx.x] = x; __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); x = sh[(threadIdx.x + 1) & 63] + 1e-9; }
  t1 = clk(); cyc[6] = (t1 - t0); out[6] = x;
  // sqrt chain
  t0 = clk();
#pragma unroll 16
  for (int i = 0; i < N; ++i) x = __builtin_amdgcn_sqrt(x) + 1.0;
  t1 = clk(); cyc[7] = (t1 - t0); out[7] = x;
}
__global__ void acc(const double* in, double* rc, double* rs, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x; if (i >= n) return;
  double a = in[i];
  rc[i] = __builtin_amdgcn_rcp(a); rs[i] = __builtin_amdgcn_rsq(a);
}
int main() {
  double* out; long long* cyc; hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 64 * 8);
  hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, out, cyc, 1.5);
  long long h[8]; hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost);
  const char* nm[] = {"fma f64", "mul f64", "rcp f64", "readlane b32x2", "readlane->fma", "mfma f64 16x16x4 (dep)", "lds wr->rd", "sqrt f64 + add"};
  for (int i = 0; i < 8; ++i) printf("%-26s %6.1f cycles/op (s_memtime units)\n", nm[i], h[i] / 256.0);
  int n = 1 << 20; double *d, *rc, *rs; hipMalloc(&d, n * 8); hipMalloc(&rc, n * 8); hipMalloc(&rs, n * 8);
  double* hd = new double[n]; for (int i = 0; i < n; ++i) hd[i] = std::ldexp(1.0 + (i * 0.6180339887) - (long)(i * 0.6180339887), (i % 61) - 30);
  hipMemcpy(d, hd, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(acc, dim3(n / 256), dim3(256), 0, 0, d, rc, rs, n);
  double* hc = new double[n]; double* hs = new double[n];
  hipMemcpy(hc, rc, n * 8, hipMemcpyDeviceToHost); hipMemcpy(hs, rs, n * 8, hipMemcpyDeviceToHost);
  double mc = 0, ms = 0; for (int i = 0; i < n; ++i) { mc = fmax(mc, fabs(hc[i] * hd[i] - 1)); ms = fmax(ms, fabs(hs[i] * hs[i] * hd[i] - 1)); }
  printf("v_rcp_f64 max rel err %.3e   v_rsq_f64 max rel err (via r^2 a - 1) %.3e   (eps %.3e)\n", mc, ms, 2.2e-16);
  return 0;
}
