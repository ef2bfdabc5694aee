// dp_ablate.hip — diagnostic A/B of Riccati kernel variants, interleaved in one process
// (cdna_hip_programming.md §5.4 rule 24).  Not part of the product library.
#include "../lqr.jl_amd/csrc/lqrx_dp.hip"
#include "../include/lqrx.h"
#include <cstdio>
#include <vector>
#include <string>
using namespace lqrx;

template <int W, int VAR> float run(const DpArgs &a, hipEvent_t e0, hipEvent_t e1) {
    dim3 grid((unsigned)a.batch), block(64);
    hipEventRecord(e0);
    hipLaunchKernelGGL((dp_riccati_kernel<double, 2, 1, W, VAR, true>), grid, block, 0, 0, a);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main(int argc, char **argv) {
    size_t n = 32, m = 16, N = 256; size_t B = argc > 1 ? atol(argv[1]) : 65536;
    size_t nn = n * n, nm = n * m, mm = m * m;
    std::vector<double> hA(B * nn), hB(B * nm), hQ(B * nn), hR(B * mm), hQf(B * nn), hx(B * n);
    lqrx_make_random_dp((int)n, (int)m, (long)B, 0, 20260104, 0, hA.data(), hB.data(), hQ.data(), hR.data(), hQf.data(), hx.data());
    DpArgs a{};
    void *p[10];
    size_t sz[10] = {B * nn, B * nm, B * nn, B * mm, B * nn, B * n, B * (N - 1) * nm, B * nn, B * N * n, B * (N - 1) * m};
    const double *src[6] = {hA.data(), hB.data(), hQ.data(), hR.data(), hQf.data(), hx.data()};
    for (int i = 0; i < 10; ++i) { hipMalloc(&p[i], sz[i] * 8); if (i < 6) hipMemcpy(p[i], src[i], sz[i] * 8, hipMemcpyHostToDevice); }
    int32_t *info; hipMalloc(&info, B * 4);
    a.A = p[0]; a.B = p[1]; a.Q = p[2]; a.R = p[3]; a.Qf = p[4]; a.x0 = p[5];
    a.K = p[6]; a.P = p[7]; a.X = p[8]; a.U = p[9]; a.info = info;
    a.n = (int)n; a.m = (int)m; a.N = (int)N; a.dtype = 0; a.p_all = 0; a.batch = B;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const char *names[] = {"W2 fast", "W3 fast", "W2 fast (rep)", "W3 fast (rep)", "W3 nosolve", "W3 noroll",
                           "W3 nosolve+noroll", "W3 noKstore", "W2 noroll", "W2 sweeponly"};
    std::vector<std::vector<float>> t(10);
    for (int rep = 0; rep < 4; ++rep) {
        t[0].push_back(run<2, 0>(a, e0, e1));
        t[1].push_back(run<3, 0>(a, e0, e1));
        t[2].push_back(run<2, 0>(a, e0, e1));
        t[3].push_back(run<3, 0>(a, e0, e1));
        t[4].push_back(run<3, VAR_NOSOLVE>(a, e0, e1));
        t[5].push_back(run<3, VAR_NOROLL>(a, e0, e1));
        t[6].push_back(run<3, VAR_NOSOLVE | VAR_NOROLL>(a, e0, e1));
        t[7].push_back(run<3, VAR_NOKSTORE | VAR_NOROLL>(a, e0, e1));
        t[8].push_back(run<2, VAR_NOROLL>(a, e0, e1));
        t[9].push_back(run<2, VAR_SWEEPONLY>(a, e0, e1));
    }
    double fl = (double)B * (N - 1) * (4.0*n*n*n + 8.0*n*n*m + 4.0*n*m*m + m*m*m/3.0 + 2.0*n*n + 2.0*m*m + 2.0*n*n + 4.0*n*m);
    for (int v = 0; v < 10; ++v) {
        float best = 1e30f; for (int r = 1; r < 4; ++r) best = std::min(best, t[v][r]);
        printf("%-22s best %8.3f ms   %7.0f traj/s   %5.1f TF(alg)\n", names[v], best, B / (best * 1e-3), fl / (best * 1e-3) / 1e12);
    }
    hipError_t e = hipGetLastError(); printf("last error: %s\n", hipGetErrorString(e));
    return 0;
}
