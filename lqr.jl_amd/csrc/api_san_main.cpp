// api_san_main.cpp — host-side sanitizer driver for the C ABI (SURVEY §5 "race detection /
// sanitizers").  Built by `make -C lqr.jl_amd/csrc asan`: lqrx_api.cpp compiled with
// AddressSanitizer + UBSan on the HOST side only (-Xarch_host; the kernels are the normal
// objects, GPU sanitizers are not available on this pool), linked into this program and run
// by tests/test_sanitizers.py on the CPU.  It drives everything the ABI does on the host
// without a GPU: argument validation of every entry point (LAPACK-style codes), the KKT
// block-structure layout / packing arithmetic (lqrx_kkt_sizes, workspace sizes), the
// counter-based problem generator (shard consistency), LS sizing, and the last-error
// buffer truncation.  With no device the device-touching paths must fail cleanly with
// LQRX_ERR_HIP / LQRX_ERR_NODEVICE rather than touch memory they do not own.
#include "../../include/lqrx.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

static int fails = 0;
#define CHECK(cond)                                                                              \
    do {                                                                                         \
        if (!(cond)) {                                                                           \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s (last error: %s)\n", __FILE__, __LINE__, \
                         #cond, lqrx_last_error());                                              \
            ++fails;                                                                             \
        }                                                                                        \
    } while (0)

static void dubins(int N, std::vector<int32_t> &n1, std::vector<int32_t> &p, std::vector<int32_t> &n2,
                   std::vector<int32_t> &w)
{
    n1.assign(N, 3); p.assign(N, 0); n2.assign(N, 3); w.assign(N, 5);
    n1[0] = 0; p[0] = 3; p[N - 1] = 3; n2[N - 1] = 0; w[N - 1] = 3;
}

int main()
{
    CHECK(lqrx_abi_version() == LQRX_ABI_VERSION);
    const int have_gpu = lqrx_device_available();

    // ---- DP validation ----
    double dummy[64] = {0};
    int32_t info[4] = {0};
    lqrx_dp_desc d{};
    d.n = 32; d.m = 16; d.N = 256; d.dtype = LQRX_F64; d.batch = 4;
    CHECK(lqrx_dp_solve(nullptr, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr) == -1);
    lqrx_dp_desc b = d; b.n = 0;
    CHECK(lqrx_dp_solve(&b, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr) == -1);
    b = d; b.N = 1;
    CHECK(lqrx_dp_solve_host(&b, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info) == -1);
    b = d; b.dtype = 7;
    CHECK(lqrx_dp_solve(&b, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr) == -1);
    b = d; b.p_mode = 2;
    CHECK(lqrx_dp_solve(&b, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr) == -1);
    b = d; b.knot_stride_AB = 5;
    CHECK(lqrx_dp_solve(&b, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr) == -1);
    b = d; b.n = 513;                  // past the workgroup kernel's 512
    CHECK(lqrx_dp_solve(&b, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr) == LQRX_ERR_UNSUPPORTED);
    b = d; b.layout = 9;
    CHECK(lqrx_dp_solve(&b, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr) < 0);
    CHECK(lqrx_dp_solve(&d, dummy, nullptr, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr) == -3);
    CHECK(lqrx_dp_solve(&d, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, nullptr, dummy, info, nullptr) == -10);
    // linear cost terms: lin (argument 8) and its pointers validated before any device work
    CHECK(lqrx_dp_solve_linear(&d, dummy, dummy, dummy, dummy, dummy, dummy, nullptr, dummy, dummy, dummy, dummy, info, nullptr) == -8);
    {
        lqrx_dp_linear ln{dummy, dummy, nullptr, dummy, dummy};
        CHECK(lqrx_dp_solve_linear(&d, dummy, dummy, dummy, dummy, dummy, dummy, &ln, dummy, dummy, dummy, dummy, info, nullptr) == -8);
        CHECK(lqrx_dp_solve_linear_host(&d, dummy, dummy, dummy, dummy, dummy, dummy, nullptr, dummy, dummy, dummy, dummy, info) == -8);
        ln.qf = dummy;
        CHECK(lqrx_dp_solve_linear(&d, dummy, dummy, dummy, dummy, dummy, dummy, &ln, dummy, nullptr, dummy, dummy, info, nullptr) == -10);
    }
    b = d; b.batch = 0;                                          // empty batch: nothing to do
    CHECK(lqrx_dp_solve(&b, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == 0);
    if (!have_gpu) {                                             // valid call, no device: clean failure
        b = d; b.n = 4; b.m = 1; b.N = 5; b.batch = 1;
        CHECK(lqrx_dp_solve_host(&b, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info) <= LQRX_ERR_HIP + 0);
    }

    // ---- last-error buffer ----
    b = d; b.m = -3;
    (void)lqrx_dp_solve(&b, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr);
    const int len = lqrx_get_last_error(nullptr, 0);
    CHECK(len > 10);
    char small[6];
    CHECK(lqrx_get_last_error(small, sizeof small) == len && std::strlen(small) == 5);
    char one[1] = {'x'};
    CHECK(lqrx_get_last_error(one, 1) == len && one[0] == '\0');
    std::vector<char> big(len + 1);
    CHECK(lqrx_get_last_error(big.data(), big.size()) == len && std::strcmp(big.data(), lqrx_last_error()) == 0);

    // ---- KKT structure layout ----
    std::vector<int32_t> n1, p, n2, w;
    dubins(101, n1, p, n2, w);
    lqrx_kkt_desc k{};
    k.N = 101; k.dtype = LQRX_F64; k.batch = 16384; k.n1 = n1.data(); k.p = p.data(); k.n2 = n2.data(); k.w = w.data();
    k.h_mode = 2; k.ginv = 1;
    int64_t nY = 0, ny = 0, nH = 0, ng = 0, nl = 0;
    CHECK(lqrx_kkt_sizes(&k, &nY, &ny, &nH, &ng, &nl) == 0);
    CHECK(nY == 6 * 5 + 99 * 30 + 6 * 3 && ny == 6 + 99 * 3 + 3 && nH == 100 * 5 + 3 && ng == nH && nl == ny);
    k.h_mode = 0;
    CHECK(lqrx_kkt_sizes(&k, nullptr, nullptr, &nH, nullptr, nullptr) == 0 && nH == 100 * 25 + 9);
    size_t ws = 0;
    CHECK(lqrx_kkt_workspace_size(&k, &ws) == 0 && ws > 0);
    CHECK(lqrx_kkt_workspace_size(&k, nullptr) == -2);
    lqrx_kkt_desc kb = k; kb.h_mode = 3;
    CHECK(lqrx_kkt_sizes(&kb, &nY, nullptr, nullptr, nullptr, nullptr) == -1);
    kb = k; kb.dtype = LQRX_F32;                               // fp32: the large-block kernels
    CHECK(lqrx_kkt_sizes(&kb, &nY, nullptr, nullptr, nullptr, nullptr) == 0);
    CHECK(lqrx_kkt_workspace_size(&kb, &ws) == 0 && ws > 0);
    kb = k; kb.dtype = 7;
    CHECK(lqrx_kkt_sizes(&kb, &nY, nullptr, nullptr, nullptr, nullptr) == -1);
    std::vector<int32_t> bad = n1;
    bad[7] = 2;                                                 // n1[k] != n2[k-1]
    kb = k; kb.n1 = bad.data();
    CHECK(lqrx_kkt_sizes(&kb, &nY, nullptr, nullptr, nullptr, nullptr) == -1);
    std::vector<int32_t> badn2 = n2;
    badn2[100] = 1;                                             // last knot must have n2 == 0
    kb = k; kb.n2 = badn2.data();
    CHECK(lqrx_kkt_sizes(&kb, &nY, nullptr, nullptr, nullptr, nullptr) == -1);
    std::vector<int32_t> bigp = p;
    bigp[50] = 600;                                             // block rows > 512
    kb = k; kb.p = bigp.data();
    CHECK(lqrx_kkt_sizes(&kb, &nY, nullptr, nullptr, nullptr, nullptr) == LQRX_ERR_UNSUPPORTED);
    kb = k; kb.w = nullptr;
    CHECK(lqrx_kkt_sizes(&kb, &nY, nullptr, nullptr, nullptr, nullptr) == -1);
    CHECK(lqrx_kkt_solve(&k, nullptr, dummy, dummy, dummy, dummy, dummy, info, nullptr) == -2);
    CHECK(lqrx_kkt_solve_ws(&k, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr, 0, nullptr) == -9);

    // ---- generator: a shard equals the matching slice of the whole batch ----
    for (int dt = 0; dt < 2; ++dt) {
        const int n = 5, m = 3, B = 6, s = dt ? 4 : 8;
        std::vector<unsigned char> A(B * n * n * s), Bm(B * n * m * s), Q(B * n * n * s), R(B * m * m * s),
            Qf(B * n * n * s), x0(B * n * s);
        CHECK(lqrx_make_random_dp(n, m, B, 0, 7, dt, A.data(), Bm.data(), Q.data(), R.data(), Qf.data(), x0.data()) == 0);
        std::vector<unsigned char> A2(2 * n * n * s), B2(2 * n * m * s), Q2(2 * n * n * s), R2(2 * m * m * s),
            Qf2(2 * n * n * s), x2(2 * n * s);
        CHECK(lqrx_make_random_dp(n, m, 2, 3, 7, dt, A2.data(), B2.data(), Q2.data(), R2.data(), Qf2.data(), x2.data()) == 0);
        CHECK(std::memcmp(A2.data(), A.data() + 3 * n * n * s, A2.size()) == 0);
        CHECK(std::memcmp(R2.data(), R.data() + 3 * m * m * s, R2.size()) == 0);
        CHECK(std::memcmp(x2.data(), x0.data() + 3 * n * s, x2.size()) == 0);
        if (!dt) {
            const double *q = (const double *)Q.data(), *f = (const double *)Qf.data();
            for (int i = 0; i < n; ++i)
                for (int j = 0; j < n; ++j) CHECK(q[i + j * n] == q[j + i * n] && f[i + j * n] == 10.0 * q[i + j * n]);
        }
    }
    CHECK(lqrx_make_random_dp(0, 1, 1, 0, 1, 0, dummy, dummy, dummy, dummy, dummy, dummy) < 0);

    // ---- LS / SQP validation ----
    CHECK(lqrx_ls_lds_bytes(4, 1, 101) > 0 && lqrx_ls_lds_bytes(4, 1, 101) <= 163840);
    CHECK(lqrx_ls_lds_bytes(6, 3, 101) <= 163840);   // Nm = 300: the global-H path
    lqrx_ls_desc ls{4, 1, 101, 5, 8};
    CHECK(lqrx_ls_solve(&ls, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info, nullptr, nullptr, nullptr) < 0);
    ls.hu_mode = 0; ls.N = 1026; ls.m = 1;                      // (N-1)m = 1025 > 1024
    CHECK(lqrx_ls_solve_host(&ls, dummy, dummy, dummy, dummy, dummy, dummy, dummy, dummy, info) == LQRX_ERR_UNSUPPORTED);
    lqrx_dubins_sqp_desc q{};
    q.N = 1; q.max_iters = 10; q.batch = 1; q.dt = 0.1;
    CHECK(lqrx_dubins_sqp_solve(&q, dummy, dummy, dummy, dummy, info, info, nullptr) < 0);
    lqrx_sqp_desc g{};
    g.model = LQRX_MODEL_CARTPOLE; g.N = 21; g.max_iters = 10; g.batch = 2; g.dt = 0.25; g.mu = 1.0;
    for (int i = 0; i < 4; ++i) g.Q[i] = 0.01, g.Qf[i] = 100.0;
    g.R[0] = 0.1;
    g.params[0] = 1.0; g.params[1] = 0.2; g.params[2] = 0.5; g.params[3] = 9.81;
    lqrx_sqp_desc gb = g; gb.model = 5;
    CHECK(lqrx_sqp_solve(&gb, dummy, dummy, dummy, dummy, info, info, nullptr) == -1);
    gb = g; gb.params[2] = 0.0;
    CHECK(lqrx_sqp_solve(&gb, dummy, dummy, dummy, dummy, info, info, nullptr) == -1);
    gb = g; gb.R[0] = 0.0;
    CHECK(lqrx_sqp_solve_host(&gb, dummy, dummy, dummy, dummy, info, info) == -1);
    CHECK(lqrx_sqp_solve(&g, nullptr, dummy, dummy, dummy, info, info, nullptr) == -2);
    int32_t nx = 0, nu = 0;
    CHECK(lqrx_sqp_model_dims(LQRX_MODEL_CARTPOLE, &nx, &nu) == 0 && nx == 4 && nu == 1);
    CHECK(lqrx_sqp_model_dims(-1, &nx, &nu) == -1 && lqrx_sqp_model_dims(5, &nx, &nu) == -1);
    CHECK(lqrx_sqp_model_dims(LQRX_MODEL_DOUBLE_INTEGRATOR3, &nx, &nu) == 0 && nx == 6 && nu == 3);
    gb = g; gb.stage_rows = 3;
    CHECK(lqrx_sqp_solve(&gb, dummy, dummy, dummy, dummy, info, info, nullptr) == -1);
    if (!have_gpu) {
        std::vector<double> Zh(2 * (21 * 4 + 20)), x0h(8), lamh(2 * 22 * 4);
        CHECK(lqrx_sqp_solve_host(&g, Zh.data(), x0h.data(), x0h.data(), lamh.data(), info, info) <= LQRX_ERR_HIP + 0);
    }

    std::printf("api sanitizer run: %s (%d failed checks, device %d)\n", fails ? "FAILED" : "ok", fails, have_gpu);
    return fails ? 1 : 0;
}
