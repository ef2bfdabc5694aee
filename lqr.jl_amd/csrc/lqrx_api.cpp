// lqrx_api.cpp — the C ABI (include/lqrx.h): argument validation, stream-ordered scratch,
// host-pointer convenience wrappers, the synthetic-problem generator.
#include "../../include/lqrx.h"
#include "lqrx_internal.h"
#define LQRX_STR2(x) #x
#define LQRX_STR(x) LQRX_STR2(x)

#include <hip/hip_runtime.h>
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <map>
#include <mutex>
#include <vector>

namespace {

thread_local std::string g_err;

int set_err(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int set_err(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_err(hipError_t e, const char *what)
{
    return set_err(LQRX_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

size_t dsize(int dtype) { return dtype == LQRX_F32 ? 4 : 8; }

// ---- stream-ordered device buffers (for the *_host wrappers) ----
struct DevBuf {
    void *p = nullptr;
    ~DevBuf()
    {
        if (p) (void)hipFree(p);
    }
};

int dev_alloc(DevBuf &b, size_t bytes, const char *name)
{
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) return hip_err(e, name);
    return 0;
}

int validate_dp(const lqrx_dp_desc *d)
{
    if (!d) return set_err(-1, "desc is NULL");
    if (d->n < 1) return set_err(-1, "desc.n must be >= 1 (got %d)", d->n);
    if (d->m < 1) return set_err(-1, "desc.m must be >= 1 (got %d)", d->m);
    if (d->N < 2) return set_err(-1, "desc.N must be >= 2 (got %d)", d->N);
    if (d->dtype != LQRX_F64 && d->dtype != LQRX_F32)
        return set_err(-1, "desc.dtype must be LQRX_F64 or LQRX_F32 (got %d)", d->dtype);
    if (d->batch < 0) return set_err(-1, "desc.batch must be >= 0");
    if (d->layout != 0 && d->layout != 1)
        return set_err(-1, "desc.layout must be 0 (batch slowest) or 1 (batch fastest, SoA) (got %d)", d->layout);
    if (d->p_mode != 0 && d->p_mode != 1) return set_err(-1, "desc.p_mode must be 0 or 1");
    if (d->knot_stride_AB != 0 && d->knot_stride_AB != 1)
        return set_err(-1, "desc.knot_stride_AB must be 0 (time-invariant) or 1 (per knot)");
    if (d->knot_stride_QR != 0 && d->knot_stride_QR != 1)
        return set_err(-1, "desc.knot_stride_QR must be 0 (time-invariant) or 1 (per knot)");
    const bool tv = d->knot_stride_AB != 0 || d->knot_stride_QR != 0;
    if (!lqrx::dp_supported(d->dtype, d->n, d->m, tv))
        return set_err(LQRX_ERR_UNSUPPORTED, "no kernel instantiated for n=%d m=%d%s", d->n, d->m,
                       tv ? " (time-varying)" : "");
    return 0;
}

} // namespace

namespace lqrx {
// The device a stream belongs to (the null stream: the calling thread's current device).
// Library state below is keyed on it, not on hipGetDevice(), so a call on a stream of
// device d works whatever device the calling thread has current.
hipError_t stream_device(hipStream_t s, int *dev)
{
    if (!s) return hipGetDevice(dev);
    hipDevice_t d = 0;
    hipError_t e = hipStreamGetDevice(s, &d);
    if (e == hipSuccess) *dev = (int)d;
    return e;
}

// Process-wide state (mutex-guarded, created on first use): one memory pool per device for
// stream-ordered scratch; freed blocks stay mapped (release threshold ∞), so steady-state
// calls allocate nothing from the driver.
static std::mutex pool_mu;
static std::map<int, hipMemPool_t> pools;
hipError_t scratch_alloc(void **p, size_t bytes, hipStream_t s)
{
    auto &mu = pool_mu;
    int dev = 0;
    hipError_t e = stream_device(s, &dev);
    if (e != hipSuccess) return e;
    hipMemPool_t pool = nullptr;
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = pools.find(dev);
        if (it == pools.end()) {
            hipMemPoolProps props{};
            props.allocType = hipMemAllocationTypePinned;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            if ((e = hipMemPoolCreate(&pool, &props)) != hipSuccess) return e;
            uint64_t keep = UINT64_MAX;                     // never trim freed blocks
            if ((e = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep)) != hipSuccess) return e;
            pools.emplace(dev, pool);
        } else {
            pool = it->second;
        }
    }
    return hipMallocFromPoolAsync(p, bytes, pool, s);
}
hipError_t scratch_free(void *p, hipStream_t s) { return hipFreeAsync(p, s); }
hipError_t scratch_trim(int device, size_t keep)
{
    std::lock_guard<std::mutex> lock(pool_mu);
    for (auto &kv : pools)
        if (device < 0 || kv.first == device) {
            hipError_t e = hipMemPoolTrimTo(kv.second, keep);
            if (e != hipSuccess) return e;
        }
    return hipSuccess;
}
} // namespace lqrx

namespace {
// Layout 1 on the MFMA kernel (one trajectory per wave, contiguous blocks wanted): the SoA
// inputs are transposed to layout 0 in one stream-ordered scratch block, solved, and the
// outputs transposed back into the caller's SoA buffers.  Extra HBM traffic: one read + one
// write of every input and output (2× the algorithmic bytes); the n ≤ 4 kernels read SoA
// natively instead.
hipError_t dp_launch_soa_staged(const lqrx::DpArgs &a, hipStream_t s)
{
    const int64_t B = a.batch, n = a.n, m = a.m, N = a.N, es = dsize(a.dtype);
    const int64_t kAB = a.tv_AB ? N - 1 : 1, kQR = a.tv_QR ? N - 1 : 1;
    // inputs A B Q R Qf x0 [q r qf], outputs K P X U [d p]
    const int nin = a.lin ? 9 : 6, nout = a.lin ? 6 : 4;
    const int64_t S_in[9] = {n * n * kAB, n * m * kAB, n * n * kQR, m * m * kQR, n * n, n,
                             n * kQR, m * kQR, n};
    const int64_t S_out[6] = {m * n * (N - 1), a.p_all ? n * n * N : n * n, n * N, m * (N - 1),
                              m * (N - 1), a.p_all ? n * N : n};
    const void *in[9] = {a.A, a.B, a.Q, a.R, a.Qf, a.x0, a.q, a.r, a.qf};
    void *out[6] = {a.K, a.P, a.X, a.U, a.d, a.p};
    size_t off[15], total = 0;
    for (int i = 0; i < nin + nout; ++i) {
        off[i] = total;
        total += ((size_t)(i < nin ? S_in[i] : S_out[i - nin]) * B * es + 255) & ~(size_t)255;
    }
    void *blk = nullptr;
    hipError_t e = lqrx::scratch_alloc(&blk, total, s);
    if (e != hipSuccess) return e;
    char *base = (char *)blk;
    lqrx::DpArgs a0 = a;
    a0.layout = 0;
    const void **pin[9] = {&a0.A, &a0.B, &a0.Q, &a0.R, &a0.Qf, &a0.x0, &a0.q, &a0.r, &a0.qf};
    void **pout[6] = {&a0.K, &a0.P, &a0.X, &a0.U, &a0.d, &a0.p};
    for (int i = 0; i < nin && e == hipSuccess; ++i) {        // [S][B] → [B][S]
        *pin[i] = base + off[i];
        e = lqrx::batch_transpose(in[i], base + off[i], S_in[i], B, (int)es, s);
    }
    for (int i = 0; i < nout; ++i) *pout[i] = base + off[nin + i];
    if (e == hipSuccess) e = lqrx::dp_launch(a0, s);
    for (int i = 0; i < nout && e == hipSuccess; ++i)         // [B][S] → [S][B]
        e = lqrx::batch_transpose(base + off[nin + i], out[i], B, S_out[i], (int)es, s);
    hipError_t ef = lqrx::scratch_free(blk, s);
    return e != hipSuccess ? e : ef;
}
} // namespace

extern "C" {

int lqrx_abi_version(void) { return LQRX_ABI_VERSION; }
#ifndef LQRX_SRC_HASH
#define LQRX_SRC_HASH "unknown"
#endif
const char *lqrx_build_info(void)
{
    return "src_sha256=" LQRX_SRC_HASH " abi=" LQRX_STR(LQRX_ABI_VERSION) " arch=gfx950 built=" __DATE__ " " __TIME__;
}
int lqrx_scratch_trim(int32_t device, size_t keep_bytes)
{
    const hipError_t e = lqrx::scratch_trim(device, keep_bytes);
    return e == hipSuccess ? 0 : hip_err(e, "hipMemPoolTrimTo");
}

const char *lqrx_last_error(void) { return g_err.c_str(); }

int lqrx_get_last_error(char *buf, size_t len)
{
    if (buf && len > 0) {
        const size_t k = std::min(len - 1, g_err.size());
        std::memcpy(buf, g_err.data(), k);
        buf[k] = '\0';
    }
    return (int)g_err.size();
}

int lqrx_device_available(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 0;
    hipDeviceProp_t prop;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

}   // extern "C"

namespace {
// lqrx_dp_solve and lqrx_dp_solve_linear (lin != NULL); argument numbers in error codes
// follow the calling entry point's signature
int dp_solve_impl(const lqrx_dp_desc *d, const void *A, const void *B, const void *Q,
                  const void *R, const void *Qf, const void *x0, const lqrx_dp_linear *lin,
                  void *K, void *P, void *X, void *U, int32_t *info, void *stream)
{
    int st = validate_dp(d);
    if (st) return st;
    if (d->batch == 0) return 0;
    const int o = lin ? 1 : 0;   // lqrx_dp_solve_linear: lin is argument 8, outputs shift by one
    const void *in[6] = {A, B, Q, R, Qf, x0};
    for (int i = 0; i < 6; ++i)
        if (!in[i]) return set_err(-(i + 2), "input pointer %d is NULL", i + 2);
    if (lin) {
        const void *lp[5] = {lin->q, lin->r, lin->qf, lin->d, lin->p};
        static const char *nm[5] = {"q", "r", "qf", "d", "p"};
        for (int i = 0; i < 5; ++i)
            if (!lp[i]) return set_err(-8, "lin->%s is NULL", nm[i]);
    }
    void *out[4] = {K, P, X, U};
    for (int i = 0; i < 4; ++i)
        if (!out[i]) return set_err(-(i + 8 + o), "output pointer %d is NULL", i + 8 + o);

    lqrx::DpArgs a{};
    if (lin) {
        a.lin = 1;
        a.q = lin->q; a.r = lin->r; a.qf = lin->qf; a.d = lin->d; a.p = lin->p;
    }
    a.A = A; a.B = B; a.Q = Q; a.R = R; a.Qf = Qf; a.x0 = x0;
    a.K = K; a.P = P; a.X = X; a.U = U; a.info = info;
    a.n = d->n; a.m = d->m; a.N = d->N; a.dtype = d->dtype; a.p_all = d->p_mode;
    a.batch = d->batch;
    a.tv_AB = (int)d->knot_stride_AB; a.tv_QR = (int)d->knot_stride_QR;
    a.layout = d->layout;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (d->layout == 1 && !lqrx::dp_lane_supported(d->n, d->m))
        e = dp_launch_soa_staged(a, s);           // MFMA kernel: convert, solve, convert back
    else
        e = lqrx::dp_launch(a, s);
    if (e == hipErrorNotSupported)
        return set_err(LQRX_ERR_UNSUPPORTED, "no kernel for n=%d m=%d", d->n, d->m);
    if (e != hipSuccess) return hip_err(e, "dp kernel launch");
    if (stream == nullptr) {
        e = hipStreamSynchronize(nullptr);
        if (e != hipSuccess) return hip_err(e, "dp kernel");
        if (info) {
            std::vector<int32_t> h((size_t)d->batch);
            e = hipMemcpy(h.data(), info, h.size() * 4, hipMemcpyDeviceToHost);
            if (e != hipSuccess) return hip_err(e, "info D2H");
            for (int32_t v : h)
                if (v) return 1;
        }
    }
    return 0;
}

int dp_solve_host_impl(const lqrx_dp_desc *d, const void *A, const void *B, const void *Q,
                       const void *R, const void *Qf, const void *x0, const lqrx_dp_linear *lin,
                       void *K, void *P, void *X, void *U, int32_t *info)
{
    int st = validate_dp(d);
    if (st) return st;
    if (d->batch == 0) return 0;
    const int o = lin ? 1 : 0;
    const size_t s = dsize(d->dtype), bt = (size_t)d->batch;
    const size_t n = d->n, m = d->m, N = d->N;
    const size_t kAB = d->knot_stride_AB ? N - 1 : 1, kQR = d->knot_stride_QR ? N - 1 : 1;
    const int nin = lin ? 9 : 6, nout = lin ? 6 : 4;
    const size_t szin[9] = {n * n * kAB, n * m * kAB, n * n * kQR, m * m * kQR, n * n, n,
                            n * kQR, m * kQR, n};
    const void *hin[9] = {A, B, Q, R, Qf, x0, lin ? lin->q : nullptr, lin ? lin->r : nullptr,
                          lin ? lin->qf : nullptr};
    const size_t szout[6] = {m * n * (N - 1), d->p_mode ? n * n * N : n * n, n * N, m * (N - 1),
                             m * (N - 1), d->p_mode ? n * N : n};
    void *hout[6] = {K, P, X, U, lin ? lin->d : nullptr, lin ? lin->p : nullptr};
    DevBuf din[9], dout[6], dinfo;
    for (int i = 0; i < nin; ++i) {
        if (!hin[i]) return set_err(i < 6 ? -(i + 2) : -8, "input pointer %s is NULL",
                                    i < 6 ? "" : "in lin");
        if ((st = dev_alloc(din[i], szin[i] * s * bt, "hipMalloc input"))) return st;
        hipError_t e = hipMemcpy(din[i].p, hin[i], szin[i] * s * bt, hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_err(e, "H2D");
    }
    for (int i = 0; i < nout; ++i) {
        if (!hout[i]) return set_err(i < 4 ? -(i + 8 + o) : -8, "output pointer %s is NULL",
                                     i < 4 ? "" : "in lin");
        if ((st = dev_alloc(dout[i], szout[i] * s * bt, "hipMalloc output"))) return st;
    }
    if ((st = dev_alloc(dinfo, 4 * bt, "hipMalloc info"))) return st;
    lqrx_dp_linear dl{};
    if (lin) {
        dl.q = din[6].p; dl.r = din[7].p; dl.qf = din[8].p; dl.d = dout[4].p; dl.p = dout[5].p;
    }
    st = dp_solve_impl(d, din[0].p, din[1].p, din[2].p, din[3].p, din[4].p, din[5].p,
                       lin ? &dl : nullptr, dout[0].p, dout[1].p, dout[2].p, dout[3].p,
                       (int32_t *)dinfo.p, nullptr);
    if (st < 0) return st;
    for (int i = 0; i < nout; ++i) {
        hipError_t e = hipMemcpy(hout[i], dout[i].p, szout[i] * s * bt, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_err(e, "D2H");
    }
    if (info) {
        hipError_t e = hipMemcpy(info, dinfo.p, 4 * bt, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_err(e, "D2H info");
    }
    return st;
}
} // namespace

extern "C" {

int lqrx_dp_solve(const lqrx_dp_desc *d, const void *A, const void *B, const void *Q,
                  const void *R, const void *Qf, const void *x0, void *K, void *P, void *X,
                  void *U, int32_t *info, void *stream)
{
    return dp_solve_impl(d, A, B, Q, R, Qf, x0, nullptr, K, P, X, U, info, stream);
}

int lqrx_dp_solve_host(const lqrx_dp_desc *d, const void *A, const void *B, const void *Q,
                       const void *R, const void *Qf, const void *x0, void *K, void *P,
                       void *X, void *U, int32_t *info)
{
    return dp_solve_host_impl(d, A, B, Q, R, Qf, x0, nullptr, K, P, X, U, info);
}

// compute_ctg!(K, solver, prob) / compute_gain!(K, solver, prob) for a batch
// (dynamic_programming.jl:34-52): one backward knot from P = solver.P.  It is exactly the
// first backward step of a 2-knot solve with Qf = P, so it runs the same kernel family on a
// 2-knot descriptor; the rollout's X, U and a zero x0 live in stream-ordered scratch.
int lqrx_dp_compute_ctg(const lqrx_dp_desc *d, const void *A, const void *B, const void *Q,
                        const void *R, const void *P, void *K, void *P_, int32_t *info, void *stream)
{
    if (!d) return set_err(-1, "desc is NULL");
    lqrx_dp_desc d2 = *d;
    d2.N = 2;
    d2.p_mode = 0;
    d2.knot_stride_AB = d2.knot_stride_QR = 0;
    int st = validate_dp(&d2);
    if (st) return st;
    if (d2.batch == 0) return 0;
    const void *in[5] = {A, B, Q, R, P};
    for (int i = 0; i < 5; ++i)
        if (!in[i]) return set_err(-(i + 2), "input pointer %d is NULL", i + 2);
    if (!K) return set_err(-7, "K is NULL");
    const size_t es = dsize(d2.dtype), bt = (size_t)d2.batch, n = d2.n, m = d2.m;
    // scratch: x0 (zeros) | X (2n) | U (m) | P_ when the caller passed none (compute_gain!)
    const size_t ox = 0, oX = ox + ((n * bt * es + 255) & ~(size_t)255);
    const size_t oU = oX + ((2 * n * bt * es + 255) & ~(size_t)255);
    const size_t oP = oU + ((m * bt * es + 255) & ~(size_t)255);
    const size_t tot = oP + (P_ ? 0 : n * n * bt * es);
    hipStream_t s = (hipStream_t)stream;
    void *blk = nullptr;
    hipError_t e = lqrx::scratch_alloc(&blk, tot, s);
    if (e != hipSuccess) return hip_err(e, "compute_ctg scratch");
    char *b = (char *)blk;
    e = hipMemsetAsync(b + ox, 0, n * bt * es, s);
    if (e != hipSuccess) {
        (void)lqrx::scratch_free(blk, s);
        return hip_err(e, "compute_ctg x0");
    }
    st = dp_solve_impl(&d2, A, B, Q, R, P, b + ox, nullptr, K, P_ ? P_ : (void *)(b + oP), b + oX, b + oU,
                       info, stream);
    e = lqrx::scratch_free(blk, s);
    if (st) return st;
    return e == hipSuccess ? 0 : hip_err(e, "compute_ctg scratch free");
}

int lqrx_dp_compute_ctg_host(const lqrx_dp_desc *d, const void *A, const void *B, const void *Q,
                             const void *R, const void *P, void *K, void *P_, int32_t *info)
{
    if (!d) return set_err(-1, "desc is NULL");
    lqrx_dp_desc d2 = *d;
    d2.N = 2;
    d2.p_mode = 0;
    d2.knot_stride_AB = d2.knot_stride_QR = 0;
    int st = validate_dp(&d2);
    if (st) return st;
    if (d2.batch == 0) return 0;
    const void *hin[5] = {A, B, Q, R, P};
    const size_t es = dsize(d2.dtype), bt = (size_t)d2.batch, n = d2.n, m = d2.m;
    const size_t szin[5] = {n * n, n * m, n * n, m * m, n * n};
    DevBuf din[5], dK, dP, dinfo;
    for (int i = 0; i < 5; ++i) {
        if (!hin[i]) return set_err(-(i + 2), "input pointer %d is NULL", i + 2);
        if ((st = dev_alloc(din[i], szin[i] * es * bt, "hipMalloc input"))) return st;
        const hipError_t e = hipMemcpy(din[i].p, hin[i], szin[i] * es * bt, hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_err(e, "H2D");
    }
    if (!K) return set_err(-7, "K is NULL");
    if ((st = dev_alloc(dK, m * n * es * bt, "hipMalloc K"))) return st;
    if (P_ && (st = dev_alloc(dP, n * n * es * bt, "hipMalloc P_"))) return st;
    if ((st = dev_alloc(dinfo, 4 * bt, "hipMalloc info"))) return st;
    st = lqrx_dp_compute_ctg(&d2, din[0].p, din[1].p, din[2].p, din[3].p, din[4].p, dK.p, P_ ? dP.p : nullptr,
                             (int32_t *)dinfo.p, nullptr);
    if (st < 0) return st;
    hipError_t e = hipMemcpy(K, dK.p, m * n * es * bt, hipMemcpyDeviceToHost);
    if (e == hipSuccess && P_) e = hipMemcpy(P_, dP.p, n * n * es * bt, hipMemcpyDeviceToHost);
    if (e == hipSuccess && info) e = hipMemcpy(info, dinfo.p, 4 * bt, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_err(e, "D2H");
    return st;
}

int lqrx_dp_solve_linear(const lqrx_dp_desc *d, const void *A, const void *B, const void *Q,
                         const void *R, const void *Qf, const void *x0,
                         const lqrx_dp_linear *lin, void *K, void *P, void *X, void *U,
                         int32_t *info, void *stream)
{
    if (!lin) return set_err(-8, "lin is NULL");
    return dp_solve_impl(d, A, B, Q, R, Qf, x0, lin, K, P, X, U, info, stream);
}

int lqrx_dp_solve_linear_host(const lqrx_dp_desc *d, const void *A, const void *B,
                              const void *Q, const void *R, const void *Qf, const void *x0,
                              const lqrx_dp_linear *lin, void *K, void *P, void *X, void *U,
                              int32_t *info)
{
    if (!lin) return set_err(-8, "lin is NULL");
    return dp_solve_host_impl(d, A, B, Q, R, Qf, x0, lin, K, P, X, U, info);
}


// ------------------------------------------------------------------ KKT
namespace {
struct KktLayout {
    std::vector<int32_t> meta; // per knot: n1, p, n2, w, oY, oy, oH, og
    int64_t sY = 0, sy = 0, sH = 0, sg = 0;
    int maxw = 0, maxrows = 0, max_p1 = 0, max_ps = 0, max_p2 = 0;
};

int kkt_layout(const lqrx_kkt_desc *d, KktLayout &L)
{
    if (!d) return set_err(-1, "desc is NULL");
    if (d->N < 1) return set_err(-1, "desc.N must be >= 1");
    if (d->dtype != LQRX_F64 && d->dtype != LQRX_F32)
        return set_err(-1, "desc.dtype must be LQRX_F64 or LQRX_F32 (got %d)", d->dtype);
    if (d->batch < 0) return set_err(-1, "desc.batch must be >= 0");
    if (!d->n1 || !d->p || !d->n2 || !d->w) return set_err(-1, "block-size arrays are NULL");
    if (d->h_mode < 0 || d->h_mode > 2) return set_err(-1, "desc.h_mode must be 0, 1 or 2");
    if (d->ginv != 0 && d->ginv != 1) return set_err(-1, "desc.ginv must be 0 or 1");
    if (d->layout != 0 && d->layout != 1)
        return set_err(-1, "desc.layout must be 0 (per trajectory) or 1 (batch fastest) (got %d)", d->layout);
    L.meta.assign((size_t)d->N * 8, 0);
    for (int k = 0; k < d->N; ++k) {
        int n1 = d->n1[k], p = d->p[k], n2 = d->n2[k], w = d->w[k];
        if (n1 < 0 || p < 0 || n2 < 0 || w < 1)
            return set_err(-1, "knot %d: negative block size or w < 1", k);
        if (k == 0 && n1 != 0) return set_err(-1, "knot 0 must have n1 == 0");
        if (k > 0 && n1 != d->n2[k - 1])
            return set_err(-1, "knot %d: n1 (%d) != n2 of knot %d (%d)", k, n1, k - 1, d->n2[k - 1]);
        if (k == d->N - 1 && n2 != 0) return set_err(-1, "last knot must have n2 == 0");
        int rows = n1 + p + n2;
        if (n1 > lqrx::KW_MAX_BLOCK || p > lqrx::KW_MAX_BLOCK || n2 > lqrx::KW_MAX_BLOCK || w > lqrx::KW_MAX_W)
            return set_err(LQRX_ERR_UNSUPPORTED, "knot %d: block (n1 %d, p %d, n2 %d, w %d) past %d rows per "
                                                 "part / %d columns", k, n1, p, n2, w, lqrx::KW_MAX_BLOCK,
                           lqrx::KW_MAX_W);
        int32_t *m = &L.meta[(size_t)k * 8];
        m[0] = n1; m[1] = p; m[2] = n2; m[3] = w;
        m[4] = (int32_t)L.sY; m[5] = (int32_t)L.sy; m[6] = (int32_t)L.sH; m[7] = (int32_t)L.sg;
        L.sY += (int64_t)rows * w;
        L.sy += p + n2;
        L.sH += d->h_mode == 2 ? w : (int64_t)w * w;
        L.sg += w;
        L.maxw = std::max(L.maxw, w);
        L.maxrows = std::max(L.maxrows, rows);
        L.max_p1 = std::max(L.max_p1, n1);
        L.max_ps = std::max(L.max_ps, p);
        L.max_p2 = std::max(L.max_p2, n2);
    }
    if (L.sY > INT32_MAX) return set_err(LQRX_ERR_UNSUPPORTED, "trajectory too large");
    // layout 1: every array's element rows are addressed with 32-bit byte offsets
    if (d->layout == 1 && std::max(std::max(L.sY, L.sy), std::max(L.sH, L.sg)) * d->batch * 8 > INT32_MAX)
        return set_err(LQRX_ERR_UNSUPPORTED, "layout 1: arrays above 2 GiB (split the batch)");
    return 0;
}
// Per-device cache of uploaded structure tables (process-wide, mutex-guarded), keyed on the
// stream's device.  A structure's table is uploaded by a blocking copy on its first use;
// afterwards a solve issues no host→device traffic besides the launch.  (A per-call
// stream-ordered alloc + pageable async copy was observed to leave the device table stale on
// repeated calls with alternating structures.)  The cache holds at most meta_cache_cap() tables
// and never evicts (nothing is freed under work in flight on another stream); structures
// beyond that get a per-call table from the stream-ordered pool, copied and waited for on
// the CALL's stream only (*tmp set: the caller frees it, stream-ordered, after the launch).
size_t meta_cache_cap()   // LQRX_META_CACHE overrides 4096 (tests exercise the overflow path)
{
    static const size_t v = [] { const char *e = std::getenv("LQRX_META_CACHE"); return e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)4096; }();
    return v;
}
int device_meta(const std::vector<int32_t> &meta, hipStream_t s, const int32_t **out, void **tmp)
{
    static std::mutex mu;
    static std::map<std::pair<int, std::vector<int32_t>>, int32_t *> cache;
    *tmp = nullptr;
    int dev = 0;
    hipError_t e = lqrx::stream_device(s, &dev);
    if (e != hipSuccess) return hip_err(e, "stream device");
    const size_t bytes = meta.size() * sizeof(int32_t);
    std::lock_guard<std::mutex> lock(mu);
    auto key = std::make_pair(dev, meta);
    auto it = cache.find(key);
    if (it != cache.end()) {
        *out = it->second;
        return 0;
    }
    if (cache.size() >= meta_cache_cap()) {
        if ((e = lqrx::scratch_alloc(tmp, bytes, s)) != hipSuccess) return hip_err(e, "meta scratch");
        if ((e = hipMemcpyAsync(*tmp, meta.data(), bytes, hipMemcpyHostToDevice, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess) {
            (void)lqrx::scratch_free(*tmp, s);
            *tmp = nullptr;
            return hip_err(e, "meta H2D");
        }
        *out = (const int32_t *)*tmp;
        return 0;
    }
    int prev = -1;
    if ((e = hipGetDevice(&prev)) != hipSuccess) return hip_err(e, "hipGetDevice");
    if (prev != dev && (e = hipSetDevice(dev)) != hipSuccess) return hip_err(e, "hipSetDevice");
    int32_t *d = nullptr;
    e = hipMalloc((void **)&d, bytes);
    if (e == hipSuccess && (e = hipMemcpy(d, meta.data(), bytes, hipMemcpyHostToDevice)) != hipSuccess) {
        (void)hipFree(d);
        d = nullptr;
    }
    if (prev != dev) (void)hipSetDevice(prev);
    if (e != hipSuccess) return hip_err(e, "meta upload");
    cache.emplace(std::move(key), d);
    *out = d;
    return 0;
}
} // namespace

extern "C" int lqrx_kkt_sizes(const lqrx_kkt_desc *d, int64_t *nY, int64_t *ny, int64_t *nH,
                              int64_t *ng, int64_t *nlam)
{
    KktLayout L;
    int st = kkt_layout(d, L);
    if (st) return st;
    if (nY) *nY = L.sY;
    if (ny) *ny = L.sy;
    if (nH) *nH = L.sH;
    if (ng) *ng = L.sg;
    if (nlam) *nlam = L.sy;
    return 0;
}

namespace {
bool kkt_force_generic();
// kernel arguments of one KKT call (no device pointers yet)
lqrx::KktArgs kkt_args(const lqrx_kkt_desc *d, const KktLayout &L)
{
    lqrx::KktArgs a{};
    a.N = d->N; a.h_mode = d->h_mode; a.ginv = d->ginv; a.batch = d->batch;
    a.sY = L.sY; a.sy = L.sy; a.sH = L.sH; a.sg = L.sg; a.sl = L.sy;
    a.maxw = L.maxw; a.maxrows = L.maxrows;
    a.max_p1 = L.max_p1; a.max_ps = L.max_ps; a.max_p2 = L.max_p2;
    static const int force_lane = [] { const char *v = std::getenv("LQRX_KKT_FORCE_LANE"); return v && *v == '1'; }();
    a.force_lane = force_lane;
    a.layout = d->layout;
    a.dtype = d->dtype == LQRX_F32 ? 1 : 0;
    return a;
}
// Kernel family for a call.  fp32: the large-block MFMA kernels, past them the
// workgroup-per-trajectory kernel.  fp64: the compile-time shapes (FIL) first, then the
// LDS-staged / small lane generic kernels, then the large-block kernels (which also replace the
// scratch-spilling lane<8,8,8,12,16> kernel), then the workgroup-per-trajectory kernel (blocks
// past 64 rows / w past 128).  LQRX_KKT_BIG=1 forces the large-block kernels wherever they
// apply, =0 never uses them; LQRX_KKT_WG=1 forces the workgroup kernel (layout 0; A/B tests).
enum { KK_NONE = 0, KK_FIL, KK_GENERIC, KK_BIG, KK_WG };
int kkt_big_env()
{
    static const int v = [] { const char *e = std::getenv("LQRX_KKT_BIG"); return e && *e ? std::atoi(e) : -1; }();
    return v;
}
int kkt_wg_env()
{
    static const int v = [] { const char *e = std::getenv("LQRX_KKT_WG"); return e && *e == '1' ? 1 : 0; }();
    return v;
}
int kkt_route(const lqrx_kkt_desc *d, const lqrx::KktArgs &a)
{
    if (a.layout == 1) {   // SoA read natively by the compile-time shapes (fp64); else staged
        size_t b = 0;
        const bool fil = d->dtype == LQRX_F64 && !a.force_lane && !kkt_force_generic() &&
                         lqrx::kkt_fil_scratch_bytes(a, d->n1, d->p, d->n2, d->w, &b);
        return fil ? KK_FIL : KK_NONE;
    }
    const bool wgk = lqrx::kkt_wg_supported(a, d->n1, d->p, d->n2, d->w);
    if (kkt_wg_env() && wgk) return KK_WG;
    const bool big = kkt_big_env() != 0 && lqrx::kkt_big_supported(a, d->n1, d->p, d->n2, d->w);
    if (d->dtype == LQRX_F32) return big ? KK_BIG : wgk ? KK_WG : KK_NONE;
    if (kkt_big_env() == 1 && big) return KK_BIG;
    size_t b = 0;
    const bool fil = !a.force_lane && !kkt_force_generic() && lqrx::kkt_fil_scratch_bytes(a, d->n1, d->p, d->n2, d->w, &b);
    if (fil) return KK_FIL;
    const int gc = lqrx::kkt_generic_class(a);
    if (gc == 1 || gc == 2 || (gc == 3 && (!big || a.force_lane))) return KK_GENERIC;
    return big ? KK_BIG : wgk ? KK_WG : KK_NONE;
}
// LQRX_KKT_GENERIC=1 forces the generic (runtime-shaped) kernel, for A/B checks
bool kkt_force_generic()
{
    static const bool v = [] { const char *e = std::getenv("LQRX_KKT_GENERIC"); return e && *e == '1'; }();
    return v;
}
// workspace bytes of the kernel family `route` (kkt_route of the same call: sizing and launch
// use one routing decision)
size_t kkt_ws_bytes(const lqrx_kkt_desc *d, const lqrx::KktArgs &a, int route)
{
    size_t b = 0;
    switch (route) {
    case KK_FIL: (void)lqrx::kkt_fil_scratch_bytes(a, d->n1, d->p, d->n2, d->w, &b); return b;
    case KK_BIG: return lqrx::kkt_big_scratch_bytes(a, d->n1, d->p, d->n2, d->w);
    case KK_WG: return lqrx::kkt_wg_scratch_bytes(a, d->n1, d->p, d->n2, d->w);
    case KK_GENERIC: return lqrx::kkt_scratch_bytes(a);
    default: return 0;
    }
}
// a layout-1 call staged through layout 0: the six transposed arrays (Y y H g | dz λ), each
// 256-B aligned — part of the call's workspace (lqrx_kkt_workspace_size counts them)
size_t kkt_stage_bytes(const lqrx_kkt_desc *d, const KktLayout &L, size_t soff[6] = nullptr)
{
    const size_t es = d->dtype == LQRX_F32 ? 4 : 8, B = (size_t)d->batch;
    const int64_t S[6] = {L.sY, L.sy, L.sH, L.sg, L.sg, L.sy};
    size_t tot = 0;
    for (int i = 0; i < 6; ++i) {
        if (soff) soff[i] = tot;
        tot += ((size_t)S[i] * B * es + 255) & ~(size_t)255;
    }
    return tot;
}
int kkt_solve_impl(const lqrx_kkt_desc *d, const void *Y, const void *y, const void *H, const void *g,
                   void *dz, void *lam, int32_t *info, void *ws, size_t ws_bytes, void *stream,
                   bool null_sync = true, const int32_t *sel = nullptr, const int32_t *nsel = nullptr);
} // namespace

extern "C" int lqrx_kkt_workspace_size(const lqrx_kkt_desc *d, size_t *bytes)
{
    KktLayout L;
    int st = kkt_layout(d, L);
    if (st) return st;
    if (!bytes) return set_err(-2, "bytes is NULL");
    if (d->batch) {
        lqrx::KktArgs a = kkt_args(d, L);
        int route = kkt_route(d, a);
        size_t stage = 0;
        if (route == KK_NONE && a.layout == 1) {   // staged through layout 0 (kkt_solve_impl)
            a.layout = 0;
            route = kkt_route(d, a);
            if (route != KK_NONE) stage = kkt_stage_bytes(d, L);
        }
        *bytes = stage + kkt_ws_bytes(d, a, route);
    } else {
        *bytes = 0;
    }
    return 0;
}

extern "C" int lqrx_kkt_solve(const lqrx_kkt_desc *d, const void *Y, const void *y, const void *H,
                              const void *g, void *dz, void *lam, int32_t *info, void *stream)
{
    return kkt_solve_impl(d, Y, y, H, g, dz, lam, info, nullptr, 0, stream);
}

extern "C" int lqrx_kkt_solve_ws(const lqrx_kkt_desc *d, const void *Y, const void *y, const void *H,
                                 const void *g, void *dz, void *lam, int32_t *info, void *workspace,
                                 size_t workspace_bytes, void *stream)
{
    if (!workspace) return set_err(-9, "workspace is NULL");
    return kkt_solve_impl(d, Y, y, H, g, dz, lam, info, workspace, workspace_bytes, stream);
}

namespace {
int kkt_solve_impl(const lqrx_kkt_desc *d, const void *Y, const void *y, const void *H, const void *g,
                   void *dz, void *lam, int32_t *info, void *ws, size_t ws_bytes, void *stream, bool null_sync,
                   const int32_t *sel, const int32_t *nsel)
{
    KktLayout L;
    int st = kkt_layout(d, L);
    if (st) return st;
    if (d->batch == 0) return 0;
    const void *in[4] = {Y, y, H, g};
    for (int i = 0; i < 4; ++i)
        if (!in[i]) return set_err(-(i + 2), "input pointer %d is NULL", i + 2);
    if (!dz) return set_err(-6, "dz is NULL");
    if (!lam) return set_err(-7, "lam is NULL");
    hipStream_t s = (hipStream_t)stream;
    // device copy of the block-structure table, uploaded once per distinct structure
    const int32_t *dmeta = nullptr;
    void *meta_tmp = nullptr;
    if ((st = device_meta(L.meta, s, &dmeta, &meta_tmp))) return st;
    hipError_t e;
    lqrx::KktArgs a = kkt_args(d, L);
    a.Y = (const double *)Y; a.y = (const double *)y; a.H = (const double *)H; a.g = (const double *)g;
    a.dz = (double *)dz; a.lam = (double *)lam; a.info = info; a.meta = dmeta;
    // a trajectory subset (internal, SQP): per-lane offsets of the selected trajectories are
    // 32-bit in the layout-0 kernel
    if (sel && nsel && d->layout == 0 &&
        std::max(std::max(L.sY, L.sy), std::max(L.sH, L.sg)) * d->batch * 8 <= INT32_MAX) {
        a.sel = sel;
        a.nsel = nsel;
    }
    // one routing decision per call (the large-block plan is an O(N) pass over the structure)
    int route = kkt_route(d, a);
    // layout 1 without a compile-time shape: the SoA arrays are transposed to layout 0 in a
    // stream-ordered scratch block, solved by the layout-0 kernel family, and dz / λ transposed
    // back (one extra read + write of every array)
    bool staged = false;
    if (route == KK_NONE && a.layout == 1) {
        a.layout = 0;
        route = kkt_route(d, a);
        staged = route != KK_NONE;
        if (!staged) a.layout = 1;
    }
    // the staged arrays: at the front of the caller's workspace (counted by
    // lqrx_kkt_workspace_size: a _ws call draws nothing from the pool), else from the pool
    size_t soff[6];
    const size_t stot = staged ? kkt_stage_bytes(d, L, soff) : 0;
    if (ws) {
        const size_t need = stot + kkt_ws_bytes(d, a, route);
        if (ws_bytes < need) {
            if (meta_tmp) (void)lqrx::scratch_free(meta_tmp, s);
            return set_err(-10, "workspace of %zu bytes < %zu (lqrx_kkt_workspace_size)", ws_bytes, need);
        }
        a.ws = (char *)ws + stot;
        a.ws_bytes = ws_bytes - stot;
    }
    static const int debug_meta = [] { const char *v = std::getenv("LQRX_DEBUG_META"); return v && *v == '1'; }();
    if (route == KK_NONE) {
        if (meta_tmp) (void)lqrx::scratch_free(meta_tmp, s);
        return set_err(LQRX_ERR_UNSUPPORTED, "no KKT kernel for this structure / options (%s; layout 0 serves "
                                             "every structure with blocks <= %d rows and w <= %d, every h_mode "
                                             "and ginv)",
                       d->dtype == LQRX_F32 ? "fp32" : "fp64", lqrx::KW_MAX_BLOCK, lqrx::KW_MAX_W);
    }
    void *stage = nullptr, *pooled = nullptr;
    const int64_t es = d->dtype == LQRX_F32 ? 4 : 8, B = d->batch;
    const int64_t S[6] = {L.sY, L.sy, L.sH, L.sg, L.sg, L.sy};   // Y y H g | dz lam
    if (staged) {
        if (ws) {
            stage = ws;
            e = hipSuccess;
        } else {
            e = lqrx::scratch_alloc(&pooled, stot, s);
            stage = pooled;
        }
        const void *src[4] = {Y, y, H, g};
        const double **dst[4] = {&a.Y, &a.y, &a.H, &a.g};
        for (int i = 0; i < 4 && e == hipSuccess; ++i) {      // [S][B] → [B][S]
            *dst[i] = (const double *)((char *)stage + soff[i]);
            e = lqrx::batch_transpose(src[i], (char *)stage + soff[i], S[i], B, (int)es, s);
        }
        a.dz = (double *)((char *)stage + soff[4]);
        a.lam = (double *)((char *)stage + soff[5]);
        a.sel = nullptr;
        a.nsel = nullptr;
    } else {
        e = hipSuccess;
    }
    if (e != hipSuccess) {
    } else if (route == KK_BIG) e = lqrx::kkt_big_launch(a, d->n1, d->p, d->n2, d->w, s);
    else if (route == KK_WG) e = lqrx::kkt_wg_launch(a, d->n1, d->p, d->n2, d->w, s);
    else if (route == KK_GENERIC || !lqrx::kkt_fil_launch(a, d->n1, d->p, d->n2, d->w, s, &e))
        e = lqrx::kkt_launch(a, s);
    if (staged && e == hipSuccess) {                          // [B][S] → [S][B]
        e = lqrx::batch_transpose(a.dz, dz, B, S[4], (int)es, s);
        if (e == hipSuccess) e = lqrx::batch_transpose(a.lam, lam, B, S[5], (int)es, s);
    }
    if (pooled) {
        const hipError_t ef = lqrx::scratch_free(pooled, s);
        if (e == hipSuccess) e = ef;
    }
    if (debug_meta) {   // read the table back before a per-call table is released
        std::vector<int32_t> back(L.meta.size());
        (void)hipStreamSynchronize(s);
        (void)hipMemcpy(back.data(), dmeta, L.meta.size() * sizeof(int32_t), hipMemcpyDeviceToHost);
        if (back != L.meta) std::fprintf(stderr, "LQRX_DEBUG_META: device meta differs from host\n");
    }
    if (meta_tmp) (void)lqrx::scratch_free(meta_tmp, s);   // stream-ordered after the launch
    if (e == hipErrorNotSupported) return set_err(LQRX_ERR_UNSUPPORTED, "KKT kernel unavailable");
    if (e != hipSuccess) return hip_err(e, "kkt kernel launch");
    if (stream == nullptr && null_sync) {
        e = hipStreamSynchronize(nullptr);
        if (e != hipSuccess) return hip_err(e, "kkt kernel");
        if (info) {
            std::vector<int32_t> h((size_t)d->batch);
            e = hipMemcpy(h.data(), info, h.size() * 4, hipMemcpyDeviceToHost);
            if (e != hipSuccess) return hip_err(e, "info D2H");
            for (int32_t v : h)
                if (v) return 1;
        }
    }
    return 0;
}
} // namespace

extern "C" int lqrx_kkt_solve_host(const lqrx_kkt_desc *d, const void *Y, const void *y,
                                   const void *H, const void *g, void *dz, void *lam,
                                   int32_t *info)
{
    KktLayout L;
    int st = kkt_layout(d, L);
    if (st) return st;
    if (d->batch == 0) return 0;
    const size_t bt = (size_t)d->batch, es = d->dtype == LQRX_F32 ? 4 : 8;
    const size_t szin[4] = {(size_t)L.sY, (size_t)L.sy, (size_t)L.sH, (size_t)L.sg};
    const void *hin[4] = {Y, y, H, g};
    DevBuf din[4], ddz, dlam, dinfo;
    for (int i = 0; i < 4; ++i) {
        if (!hin[i]) return set_err(-(i + 2), "input pointer %d is NULL", i + 2);
        if ((st = dev_alloc(din[i], szin[i] * es * bt, "hipMalloc input"))) return st;
        hipError_t e = hipMemcpy(din[i].p, hin[i], szin[i] * es * bt, hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_err(e, "H2D");
    }
    if (!dz) return set_err(-6, "dz is NULL");
    if (!lam) return set_err(-7, "lam is NULL");
    if ((st = dev_alloc(ddz, (size_t)L.sg * es * bt, "hipMalloc dz"))) return st;
    if ((st = dev_alloc(dlam, (size_t)L.sy * es * bt, "hipMalloc lam"))) return st;
    if ((st = dev_alloc(dinfo, 4 * bt, "hipMalloc info"))) return st;
    st = lqrx_kkt_solve(d, din[0].p, din[1].p, din[2].p, din[3].p, ddz.p, dlam.p,
                        (int32_t *)dinfo.p, nullptr);
    if (st < 0) return st;
    hipError_t e = hipMemcpy(dz, ddz.p, (size_t)L.sg * es * bt, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(lam, dlam.p, (size_t)L.sy * es * bt, hipMemcpyDeviceToHost);
    if (e == hipSuccess && info) e = hipMemcpy(info, dinfo.p, 4 * bt, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_err(e, "D2H");
    return st;
}

// ------------------------------------------------------------------ generator
static inline uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static inline double gauss(uint64_t seed, uint64_t traj, uint64_t field, uint64_t elem)
{
    uint64_t h = splitmix64(seed ^ splitmix64(traj ^ splitmix64((field << 40) ^ elem)));
    uint64_t h2 = splitmix64(h);
    double u1 = ((h >> 11) + 1.0) * (1.0 / 9007199254740992.0); // (0, 1]
    double u2 = (h2 >> 11) * (1.0 / 9007199254740992.0);        // [0, 1)
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

static void gen_one(int n, int m, uint64_t seed, uint64_t t, double *A, double *B, double *Q,
                    double *R, double *Qf, double *x0, std::vector<double> &G)
{
    const double sn = std::sqrt((double)n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i)
            A[i + j * n] = (i == j ? 1.0 : 0.0) + (0.1 / sn) * gauss(seed, t, 0, i + j * n);
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < n; ++i) B[i + j * n] = gauss(seed, t, 1, i + j * n) / sn;
    G.resize((size_t)n * n);
    for (int e = 0; e < n * n; ++e) G[e] = gauss(seed, t, 2, e);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            double s = 0.0;
            for (int p = 0; p < n; ++p) s += G[p + i * n] * G[p + j * n];
            Q[i + j * n] = (i == j ? 1.0 : 0.0) + s / n;
        }
    G.resize((size_t)m * m);
    for (int e = 0; e < m * m; ++e) G[e] = gauss(seed, t, 3, e);
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            for (int p = 0; p < m; ++p) s += G[p + i * m] * G[p + j * m];
            R[i + j * m] = (i == j ? 1.0 : 0.0) + s / m;
        }
    for (int e = 0; e < n * n; ++e) Qf[e] = 10.0 * Q[e];
    for (int i = 0; i < n; ++i) x0[i] = gauss(seed, t, 4, i);
}

int lqrx_make_random_dp(int32_t n, int32_t m, int64_t batch, int64_t traj0, uint64_t seed,
                        int32_t dtype, void *A, void *B, void *Q, void *R, void *Qf, void *x0)
{
    if (n < 1) return set_err(-1, "n must be >= 1");
    if (m < 1) return set_err(-2, "m must be >= 1");
    if (batch < 0) return set_err(-3, "batch must be >= 0");
    if (dtype != LQRX_F64 && dtype != LQRX_F32) return set_err(-6, "bad dtype");
    void *outs[6] = {A, B, Q, R, Qf, x0};
    for (int i = 0; i < 6; ++i)
        if (!outs[i]) return set_err(-(7 + i), "output pointer is NULL");
    const size_t nn = (size_t)n * n, nm = (size_t)n * m, mm = (size_t)m * m;
    unsigned nth = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
    if ((int64_t)nth > batch) nth = (unsigned)std::max<int64_t>(1, batch);
    auto work = [&](unsigned tid) {
        std::vector<double> a(nn), b(nm), q(nn), r(mm), qf(nn), x(n), G;
        for (int64_t t = tid; t < batch; t += nth) {
            gen_one(n, m, seed, (uint64_t)(traj0 + t), a.data(), b.data(), q.data(), r.data(),
                    qf.data(), x.data(), G);
            auto put = [&](void *dst, const std::vector<double> &src, size_t cnt) {
                if (dtype == LQRX_F64)
                    std::memcpy((double *)dst + t * cnt, src.data(), cnt * 8);
                else
                    for (size_t e = 0; e < cnt; ++e) ((float *)dst)[t * cnt + e] = (float)src[e];
            };
            put(A, a, nn); put(B, b, nm); put(Q, q, nn); put(R, r, mm); put(Qf, qf, nn);
            put(x0, x, n);
        }
    };
    std::vector<std::thread> th;
    for (unsigned i = 1; i < nth; ++i) th.emplace_back(work, i);
    work(0);
    for (auto &t : th) t.join();
    return 0;
}

} // extern "C"

// ------------------------------------------------------------------ multi-device host entries
// SURVEY §8(e) through the drop-in boundary: the batch split into contiguous shards, one per
// entry of devices[] (repeats allowed: two shards on one GPU), each shard on its own thread with
// its own non-blocking stream on its device — H2D of its slice, the single-device solve, D2H into
// the caller's arrays at the shard's offset.  Every trajectory is solved exactly as by the
// single-device call (one wave / lane / workgroup per trajectory, no cross-trajectory
// arithmetic), so the outputs are bit-identical whenever the shards select the same kernel as
// the whole batch (the n ≤ 4 quad/lane choice depends on the batch, see dp_lane.hip use_quad).
namespace {
struct Shard {
    int64_t b0 = 0, nb = 0;
    int dev = 0;
    int st = 0;
    std::string err;
};

// shard boundaries: contiguous, the first (B mod ndev) shards one trajectory longer
std::vector<Shard> make_shards(int64_t B, const int32_t *devices, int32_t ndev)
{
    std::vector<Shard> sh((size_t)ndev);
    const int64_t q = B / ndev, r = B % ndev;
    int64_t b0 = 0;
    for (int i = 0; i < ndev; ++i) {
        sh[i].b0 = b0;
        sh[i].nb = q + (i < r ? 1 : 0);
        sh[i].dev = devices[i];
        b0 += sh[i].nb;
    }
    return sh;
}

int check_devices(const int32_t *devices, int32_t ndev, int ai_dev, int ai_ndev)
{
    if (ndev < 1) return set_err(-ai_ndev, "ndev must be >= 1 (got %d)", ndev);
    if (!devices) return set_err(-ai_dev, "devices is NULL");
    int cnt = 0;
    const hipError_t e = hipGetDeviceCount(&cnt);
    if (e != hipSuccess) return set_err(LQRX_ERR_NODEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
    for (int i = 0; i < ndev; ++i)
        if (devices[i] < 0 || devices[i] >= cnt)
            return set_err(-ai_dev, "devices[%d] = %d is not a device (0..%d)", i, devices[i], cnt - 1);
    return 0;
}

// one host array of S elements per trajectory: the shard's slice ↔ a packed device buffer of
// nb trajectories in the same layout (layout 0: one contiguous run; layout 1: S rows of nb
// elements at pitch B)
hipError_t shard_h2d(void *dst, const void *src, size_t S, size_t es, const Shard &sh, int64_t B, int layout,
                     hipStream_t s)
{
    if (layout == 0)
        return hipMemcpyAsync(dst, (const char *)src + (size_t)sh.b0 * S * es, (size_t)sh.nb * S * es,
                              hipMemcpyHostToDevice, s);
    return hipMemcpy2DAsync(dst, (size_t)sh.nb * es, (const char *)src + (size_t)sh.b0 * es, (size_t)B * es,
                            (size_t)sh.nb * es, S, hipMemcpyHostToDevice, s);
}
hipError_t shard_d2h(void *dst, const void *src, size_t S, size_t es, const Shard &sh, int64_t B, int layout,
                     hipStream_t s)
{
    if (layout == 0)
        return hipMemcpyAsync((char *)dst + (size_t)sh.b0 * S * es, src, (size_t)sh.nb * S * es,
                              hipMemcpyDeviceToHost, s);
    return hipMemcpy2DAsync((char *)dst + (size_t)sh.b0 * es, (size_t)B * es, src, (size_t)sh.nb * es,
                            (size_t)sh.nb * es, S, hipMemcpyDeviceToHost, s);
}

// a shard's device buffers and stream, released on its own device
struct ShardCtx {
    hipStream_t s = nullptr;
    std::vector<void *> bufs;
    ~ShardCtx()
    {
        if (s) (void)hipStreamSynchronize(s);
        for (void *p : bufs) (void)hipFree(p);
        if (s) (void)hipStreamDestroy(s);
    }
    int alloc(void **p, size_t bytes)
    {
        hipError_t e = hipMalloc(p, bytes ? bytes : 16);
        if (e != hipSuccess) return hip_err(e, "hipMalloc shard");
        bufs.push_back(*p);
        return 0;
    }
};

// run fn(shard) for every non-empty shard concurrently, each on its device; the first failing
// shard's status and message become the call's; else 1 if any trajectory has info != 0
template <typename F> int run_shards(std::vector<Shard> &sh, const int32_t *info, int64_t B, F fn)
{
    std::vector<std::thread> th;
    for (auto &x : sh) {
        if (x.nb == 0) continue;
        th.emplace_back([&x, &fn] {
            hipError_t e = hipSetDevice(x.dev);
            x.st = e != hipSuccess ? hip_err(e, "hipSetDevice") : fn(x);
            if (x.st < 0) x.err = g_err;
        });
    }
    for (auto &t : th) t.join();
    for (auto &x : sh)
        if (x.st < 0) return set_err(x.st, "shard on device %d (trajectories %lld..%lld): %s", x.dev,
                                     (long long)x.b0, (long long)(x.b0 + x.nb - 1), x.err.c_str());
    if (info)
        for (int64_t b = 0; b < B; ++b)
            if (info[b]) return 1;
    return 0;
}

int dp_solve_host_devices_impl(const lqrx_dp_desc *d, const void *A, const void *B, const void *Q,
                               const void *R, const void *Qf, const void *x0, const lqrx_dp_linear *lin,
                               void *K, void *P, void *X, void *U, int32_t *info, const int32_t *devices,
                               int32_t ndev)
{
    int st = validate_dp(d);
    if (st) return st;
    const int o = lin ? 1 : 0;
    if ((st = check_devices(devices, ndev, 13 + o, 14 + o))) return st;
    if (d->batch == 0) return 0;
    const size_t es = dsize(d->dtype), n = d->n, m = d->m, N = d->N;
    const size_t kAB = d->knot_stride_AB ? N - 1 : 1, kQR = d->knot_stride_QR ? N - 1 : 1;
    const int nin = lin ? 9 : 6, nout = lin ? 6 : 4;
    const size_t szin[9] = {n * n * kAB, n * m * kAB, n * n * kQR, m * m * kQR, n * n, n, n * kQR, m * kQR, n};
    const void *hin[9] = {A, B, Q, R, Qf, x0, lin ? lin->q : nullptr, lin ? lin->r : nullptr,
                          lin ? lin->qf : nullptr};
    const size_t szout[6] = {m * n * (N - 1), d->p_mode ? n * n * N : n * n, n * N, m * (N - 1),
                             m * (N - 1), d->p_mode ? n * N : n};
    void *hout[6] = {K, P, X, U, lin ? lin->d : nullptr, lin ? lin->p : nullptr};
    for (int i = 0; i < nin; ++i)
        if (!hin[i]) return set_err(i < 6 ? -(i + 2) : -8, "input pointer %d is NULL", i < 6 ? i + 2 : 8);
    for (int i = 0; i < nout; ++i)
        if (!hout[i]) return set_err(i < 4 ? -(i + 8 + o) : -8, "output pointer %d is NULL", i < 4 ? i + 8 + o : 8);
    std::vector<Shard> sh = make_shards(d->batch, devices, ndev);
    const int64_t Bt = d->batch;
    const int lay = d->layout;
    return run_shards(sh, info, Bt, [&](Shard &x) -> int {
        ShardCtx c;
        hipError_t e = hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking);
        if (e != hipSuccess) return hip_err(e, "hipStreamCreate");
        void *din[9] = {}, *dout[6] = {}, *dinfo = nullptr;
        int r;
        for (int i = 0; i < nin; ++i) {
            if ((r = c.alloc(&din[i], szin[i] * es * x.nb))) return r;
            if ((e = shard_h2d(din[i], hin[i], szin[i], es, x, Bt, lay, c.s)) != hipSuccess) return hip_err(e, "H2D");
        }
        for (int i = 0; i < nout; ++i)
            if ((r = c.alloc(&dout[i], szout[i] * es * x.nb))) return r;
        if ((r = c.alloc(&dinfo, 4 * x.nb))) return r;
        lqrx_dp_desc ds = *d;
        ds.batch = x.nb;
        lqrx_dp_linear dl{};
        if (lin) {
            dl.q = din[6]; dl.r = din[7]; dl.qf = din[8]; dl.d = dout[4]; dl.p = dout[5];
        }
        if ((r = dp_solve_impl(&ds, din[0], din[1], din[2], din[3], din[4], din[5], lin ? &dl : nullptr, dout[0],
                               dout[1], dout[2], dout[3], (int32_t *)dinfo, c.s)) < 0)
            return r;
        for (int i = 0; i < nout; ++i)
            if ((e = shard_d2h(hout[i], dout[i], szout[i], es, x, Bt, lay, c.s)) != hipSuccess) return hip_err(e, "D2H");
        if (info && (e = hipMemcpyAsync(info + x.b0, dinfo, 4 * x.nb, hipMemcpyDeviceToHost, c.s)) != hipSuccess)
            return hip_err(e, "D2H info");
        if ((e = hipStreamSynchronize(c.s)) != hipSuccess) return hip_err(e, "dp shard");
        return 0;
    });
}
} // namespace

extern "C" int lqrx_dp_solve_host_devices(const lqrx_dp_desc *d, const void *A, const void *B, const void *Q,
                                          const void *R, const void *Qf, const void *x0, void *K, void *P, void *X,
                                          void *U, int32_t *info, const int32_t *devices, int32_t ndev)
{
    return dp_solve_host_devices_impl(d, A, B, Q, R, Qf, x0, nullptr, K, P, X, U, info, devices, ndev);
}

extern "C" int lqrx_dp_solve_linear_host_devices(const lqrx_dp_desc *d, const void *A, const void *B,
                                                 const void *Q, const void *R, const void *Qf, const void *x0,
                                                 const lqrx_dp_linear *lin, void *K, void *P, void *X, void *U,
                                                 int32_t *info, const int32_t *devices, int32_t ndev)
{
    if (!lin) return set_err(-8, "lin is NULL");
    return dp_solve_host_devices_impl(d, A, B, Q, R, Qf, x0, lin, K, P, X, U, info, devices, ndev);
}

extern "C" int lqrx_kkt_solve_host_devices(const lqrx_kkt_desc *d, const void *Y, const void *y, const void *H,
                                           const void *g, void *dz, void *lam, int32_t *info,
                                           const int32_t *devices, int32_t ndev)
{
    KktLayout L;
    int st = kkt_layout(d, L);
    if (st) return st;
    if ((st = check_devices(devices, ndev, 9, 10))) return st;
    if (d->batch == 0) return 0;
    const void *hin[4] = {Y, y, H, g};
    for (int i = 0; i < 4; ++i)
        if (!hin[i]) return set_err(-(i + 2), "input pointer %d is NULL", i + 2);
    if (!dz) return set_err(-6, "dz is NULL");
    if (!lam) return set_err(-7, "lam is NULL");
    const size_t es = d->dtype == LQRX_F32 ? 4 : 8;
    const size_t szin[4] = {(size_t)L.sY, (size_t)L.sy, (size_t)L.sH, (size_t)L.sg};
    std::vector<Shard> sh = make_shards(d->batch, devices, ndev);
    const int64_t Bt = d->batch;
    const int lay = d->layout;
    return run_shards(sh, info, Bt, [&](Shard &x) -> int {
        ShardCtx c;
        hipError_t e = hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking);
        if (e != hipSuccess) return hip_err(e, "hipStreamCreate");
        void *din[4] = {}, *ddz = nullptr, *dlam = nullptr, *dinfo = nullptr;
        int r;
        for (int i = 0; i < 4; ++i) {
            if ((r = c.alloc(&din[i], szin[i] * es * x.nb))) return r;
            if ((e = shard_h2d(din[i], hin[i], szin[i], es, x, Bt, lay, c.s)) != hipSuccess) return hip_err(e, "H2D");
        }
        if ((r = c.alloc(&ddz, (size_t)L.sg * es * x.nb)) || (r = c.alloc(&dlam, (size_t)L.sy * es * x.nb)) ||
            (r = c.alloc(&dinfo, 4 * x.nb)))
            return r;
        lqrx_kkt_desc ds = *d;
        ds.batch = x.nb;
        if ((r = kkt_solve_impl(&ds, din[0], din[1], din[2], din[3], ddz, dlam, (int32_t *)dinfo, nullptr, 0, c.s)) < 0)
            return r;
        if ((e = shard_d2h(dz, ddz, (size_t)L.sg, es, x, Bt, lay, c.s)) != hipSuccess ||
            (e = shard_d2h(lam, dlam, (size_t)L.sy, es, x, Bt, lay, c.s)) != hipSuccess)
            return hip_err(e, "D2H");
        if (info && (e = hipMemcpyAsync(info + x.b0, dinfo, 4 * x.nb, hipMemcpyDeviceToHost, c.s)) != hipSuccess)
            return hip_err(e, "D2H info");
        if ((e = hipStreamSynchronize(c.s)) != hipSuccess) return hip_err(e, "kkt shard");
        return 0;
    });
}

// ------------------------------------------------------------------ batched trajectory SQP
namespace {
int validate_sqp(const lqrx_sqp_desc *d, int *nx, int *nu)
{
    if (!d) return set_err(-1, "desc is NULL");
    if (!lqrx::sqp_model_dims(d->model, nx, nu)) return set_err(-1, "desc.model %d is not a known model", d->model);
    if (d->N < 2) return set_err(-1, "desc.N must be >= 2 (got %d)", d->N);
    if (d->batch < 0) return set_err(-1, "desc.batch must be >= 0");
    if (d->max_iters < 0) return set_err(-1, "desc.max_iters must be >= 0");
    if (d->stage_rows < 0 || d->stage_rows > 2 || d->stage_rows * *nx > 32)
        return set_err(-1, "desc.stage_rows must be 0..2 with stage_rows·nx <= 32 (got %d)", d->stage_rows);
    for (int i = 0; i < d->stage_rows * *nx; ++i)
        if (!std::isfinite(d->stage_A[i])) return set_err(-1, "desc.stage_A must be finite");
    for (int i = 0; i < d->stage_rows; ++i)
        if (!std::isfinite(d->stage_b[i])) return set_err(-1, "desc.stage_b must be finite");
    if (!(d->dt > 0)) return set_err(-1, "desc.dt must be > 0");
    for (int i = 0; i < *nx; ++i)
        if (!(d->Q[i] > 0) || !(d->Qf[i] > 0)) return set_err(-1, "desc.Q / desc.Qf must be positive");
    for (int i = 0; i < *nu; ++i)
        if (!(d->R[i] > 0)) return set_err(-1, "desc.R must be positive");
    if (d->model == LQRX_MODEL_CARTPOLE)
        for (int i = 0; i < 4; ++i)
            if (!(d->params[i] > 0) || !std::isfinite(d->params[i]))
                return set_err(-1, "desc.params (mc, mp, l, g) must be positive and finite");
    if (!(d->mu >= 0) || !(d->tol_p >= 0) || !(d->tol_d >= 0))
        return set_err(-1, "desc.mu / tol_p / tol_d must be >= 0");
    return 0;
}

lqrx_sqp_desc from_dubins(const lqrx_dubins_sqp_desc *d)
{
    lqrx_sqp_desc q{};
    q.model = LQRX_MODEL_DUBINS;
    q.N = d->N; q.max_iters = d->max_iters; q.batch = d->batch; q.dt = d->dt;
    for (int i = 0; i < 3; ++i) q.Q[i] = d->Q[i], q.Qf[i] = d->Qf[i];
    for (int i = 0; i < 2; ++i) q.R[i] = d->R[i];
    q.mu = d->mu; q.tol_p = d->tol_p; q.tol_d = d->tol_d;
    return q;
}

struct SqpKkt {
    lqrx_kkt_desc kd;
    std::vector<int32_t> n1, p, n2, w;
    const double *Y, *y, *H, *g;
    double *lamn, *lams;
    int32_t *info;
    void *ws;
    size_t ws_bytes;
    hipStream_t s;
};

int sqp_kkt(void *ctx, int ginv, double *dz, const int32_t *sel, const int32_t *nsel)
{
    SqpKkt &c = *(SqpKkt *)ctx;
    c.kd.ginv = ginv;
    return kkt_solve_impl(&c.kd, c.Y, c.y, c.H, c.g, dz, ginv ? c.lamn : c.lams, c.info, c.ws, c.ws_bytes, c.s,
                          /*null_sync=*/false, sel, nsel);
}
} // namespace

extern "C" int lqrx_sqp_model_dims(int32_t model, int32_t *nx, int32_t *nu)
{
    int a = 0, b = 0;
    if (!lqrx::sqp_model_dims(model, &a, &b)) return set_err(-1, "model %d is not a known model", model);
    if (nx) *nx = a;
    if (nu) *nu = b;
    return 0;
}

extern "C" int lqrx_sqp_solve(const lqrx_sqp_desc *d, double *Z, const double *x0, const double *xf, double *lam,
                              int32_t *iters, int32_t *status, void *stream)
{
    int nx = 0, nu = 0;
    int st = validate_sqp(d, &nx, &nu);
    if (st) return st;
    if (d->batch == 0) return 0;
    if (!Z) return set_err(-2, "Z is NULL");
    if (!x0) return set_err(-3, "x0 is NULL");
    if (!xf) return set_err(-4, "xf is NULL");
    if (!lam) return set_err(-5, "lam is NULL");
    if (!iters) return set_err(-6, "iters is NULL");
    if (!status) return set_err(-7, "status is NULL");
    const int N = d->N;
    const int pk = d->stage_rows;
    const int64_t B = d->batch, NN = (int64_t)N * nx + (int64_t)(N - 1) * nu,
                  P = (int64_t)(N + 1) * nx + (int64_t)(N - 2) * pk;
    hipStream_t s = (hipStream_t)stream;
    SqpKkt c{};
    lqrx::sqp_structure(nx, nu, pk, N, c.n1, c.p, c.n2, c.w);
    c.kd.N = N; c.kd.dtype = LQRX_F64; c.kd.batch = B;
    c.kd.n1 = c.n1.data(); c.kd.p = c.p.data(); c.kd.n2 = c.n2.data(); c.kd.w = c.w.data();
    c.kd.h_mode = 2; c.kd.ginv = 1; c.kd.layout = 0;
    int64_t sY = 0, sy = 0, sH = 0, sg = 0;
    if ((st = lqrx_kkt_sizes(&c.kd, &sY, &sy, &sH, &sg, nullptr))) return st;
    size_t ws1 = 0, ws0 = 0;
    if ((st = lqrx_kkt_workspace_size(&c.kd, &ws1))) return st;
    c.kd.ginv = 0;
    if ((st = lqrx_kkt_workspace_size(&c.kd, &ws0))) return st;
    // one stream-ordered block, carved (256-B aligned pieces)
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    const size_t oY = take(B * sY * 8), oy = take(B * sy * 8), oH = take(B * sH * 8), og = take(B * sg * 8),
                 odz = take(B * NN * 8), olamn = take(B * P * 8), odzs = take(B * NN * 8), olams = take(B * P * 8),
                 ophi = take(B * 8), odphi = take(B * 8), osoc = take(B * 4),
                 oact = take(4), oinfo = take(B * 4), ows = take(std::max(ws0, ws1)),
                 osel = take(B * 4), onsel = take(4);
    void *blk = nullptr;
    hipError_t e = lqrx::scratch_alloc(&blk, off, s);
    if (e != hipSuccess) return hip_err(e, "sqp scratch");
    char *b = (char *)blk;
    lqrx::SqpArgs A{};
    A.model = d->model; A.N = N; A.B = B; A.dt = d->dt; A.mu = d->mu; A.tol_p = d->tol_p; A.tol_d = d->tol_d;
    for (int i = 0; i < 8; ++i) A.Q[i] = d->Q[i], A.Qf[i] = d->Qf[i], A.R[i] = d->R[i];
    for (int i = 0; i < 4; ++i) A.par[i] = d->params[i];
    A.stage_rows = pk;
    for (int i = 0; i < 32; ++i) A.SA[i] = d->stage_A[i];
    for (int i = 0; i < 4; ++i) A.Sb[i] = d->stage_b[i];
    A.x0 = x0; A.xf = xf; A.Z = Z; A.lam = lam; A.iters = iters; A.status = status;
    A.Y = (double *)(b + oY); A.y = (double *)(b + oy); A.H = (double *)(b + oH); A.g = (double *)(b + og);
    A.dz = (double *)(b + odz); A.lamn = (double *)(b + olamn); A.dzs = (double *)(b + odzs);
    A.phi0 = (double *)(b + ophi); A.dphi = (double *)(b + odphi);
    A.need_soc = (int32_t *)(b + osoc); A.n_active = (int32_t *)(b + oact);
    A.sel = (int32_t *)(b + osel); A.nsel = (int32_t *)(b + onsel);
    c.Y = A.Y; c.y = A.y; c.H = A.H; c.g = A.g; c.lamn = A.lamn; c.lams = (double *)(b + olams);
    c.info = (int32_t *)(b + oinfo); c.ws = b + ows; c.ws_bytes = std::max(ws0, ws1); c.s = s;
    int kkt_rc = 0;
    e = lqrx::sqp_run(A, d->max_iters, s, sqp_kkt, &c, &kkt_rc);
    hipError_t ef = lqrx::scratch_free(blk, s);
    if (kkt_rc < 0) return kkt_rc;
    if (e != hipSuccess) return hip_err(e, "sqp");
    if (ef != hipSuccess) return hip_err(ef, "sqp scratch free");
    if (stream == nullptr && (e = hipStreamSynchronize(nullptr)) != hipSuccess) return hip_err(e, "sqp");
    return 0;
}

extern "C" int lqrx_sqp_solve_host(const lqrx_sqp_desc *d, double *Z, const double *x0, const double *xf,
                                   double *lam, int32_t *iters, int32_t *status)
{
    int nx = 0, nu = 0;
    int st = validate_sqp(d, &nx, &nu);
    if (st) return st;
    if (d->batch == 0) return 0;
    if (!Z || !x0 || !xf || !lam || !iters || !status) return set_err(-2, "NULL host pointer");
    const int64_t B = d->batch, NN = (int64_t)d->N * nx + (int64_t)(d->N - 1) * nu,
                  P = (int64_t)(d->N + 1) * nx + (int64_t)(d->N - 2) * d->stage_rows;
    DevBuf dZ, dx0, dxf, dlam, dit, dst;
    if ((st = dev_alloc(dZ, B * NN * 8, "Z")) || (st = dev_alloc(dx0, B * nx * 8, "x0")) ||
        (st = dev_alloc(dxf, B * nx * 8, "xf")) || (st = dev_alloc(dlam, B * P * 8, "lam")) ||
        (st = dev_alloc(dit, B * 4, "iters")) || (st = dev_alloc(dst, B * 4, "status")))
        return st;
    hipError_t e;
    if ((e = hipMemcpy(dZ.p, Z, B * NN * 8, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(dx0.p, x0, B * nx * 8, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(dxf.p, xf, B * nx * 8, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_err(e, "sqp H2D");
    if ((st = lqrx_sqp_solve(d, (double *)dZ.p, (const double *)dx0.p, (const double *)dxf.p, (double *)dlam.p,
                             (int32_t *)dit.p, (int32_t *)dst.p, nullptr)))
        return st;
    if ((e = hipMemcpy(Z, dZ.p, B * NN * 8, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(lam, dlam.p, B * P * 8, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(iters, dit.p, B * 4, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(status, dst.p, B * 4, hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_err(e, "sqp D2H");
    return 0;
}

extern "C" int lqrx_dubins_sqp_solve(const lqrx_dubins_sqp_desc *d, double *Z, const double *x0, const double *xf,
                                     double *lam, int32_t *iters, int32_t *status, void *stream)
{
    if (!d) return set_err(-1, "desc is NULL");
    const lqrx_sqp_desc q = from_dubins(d);
    return lqrx_sqp_solve(&q, Z, x0, xf, lam, iters, status, stream);
}

extern "C" int lqrx_dubins_sqp_solve_host(const lqrx_dubins_sqp_desc *d, double *Z, const double *x0,
                                          const double *xf, double *lam, int32_t *iters, int32_t *status)
{
    if (!d) return set_err(-1, "desc is NULL");
    const lqrx_sqp_desc q = from_dubins(d);
    return lqrx_sqp_solve_host(&q, Z, x0, xf, lam, iters, status);
}


// ------------------------------------------------------------------ condensed least squares
namespace {
constexpr size_t LS_LDS_MAX = 163840;

int validate_ls(const lqrx_ls_desc *d)
{
    if (!d) return set_err(-1, "desc is NULL");
    if (d->n < 1 || d->m < 1) return set_err(-1, "desc.n, desc.m must be >= 1 (got %d, %d)", d->n, d->m);
    if (d->N < 2) return set_err(-1, "desc.N must be >= 2 (got %d)", d->N);
    if (d->hu_mode < 0 || d->hu_mode > 2) return set_err(-1, "desc.hu_mode must be 0, 1 or 2");
    if (d->batch < 0 || d->batch > 0x7fffffff) return set_err(-1, "desc.batch must be in [0, 2^31)");
    if ((int64_t)(d->N - 1) * d->m > lqrx::ls_max_nm())
        return set_err(LQRX_ERR_UNSUPPORTED, "(N-1)*m = %lld > %d", (long long)(d->N - 1) * d->m, lqrx::ls_max_nm());
    const size_t lds = lqrx::ls_lds_bytes(d->n, d->m, d->N);
    if (lds > LS_LDS_MAX)
        return set_err(LQRX_ERR_UNSUPPORTED, "n=%d m=%d N=%d needs %zu B of LDS (> %zu)", d->n, d->m, d->N, lds,
                       LS_LDS_MAX);
    return 0;
}
} // namespace

extern "C" size_t lqrx_ls_lds_bytes(int32_t n, int32_t m, int32_t N)
{
    if (n < 1 || m < 1 || N < 2) return 0;
    return lqrx::ls_lds_bytes(n, m, N);
}

extern "C" int lqrx_ls_solve(const lqrx_ls_desc *d, const double *A, const double *B, const double *Q,
                             const double *R, const double *Qf, const double *x0, double *U, double *X,
                             int32_t *info, double *Abar, double *bbar, void *stream)
{
    int st = validate_ls(d);
    if (st) return st;
    if (d->batch == 0) return 0;
    const double *in[6] = {A, B, Q, R, Qf, x0};
    for (int i = 0; i < 6; ++i)
        if (!in[i]) return set_err(-(i + 2), "input pointer %d is NULL", i + 2);
    if (!U) return set_err(-8, "U is NULL");
    if (!X) return set_err(-9, "X is NULL");
    lqrx::LsArgs a{};
    a.A = A; a.B = B; a.Q = Q; a.R = R; a.Qf = Qf; a.x0 = x0;
    a.U = U; a.X = X; a.info = info; a.Ab = Abar; a.bb = bbar;
    a.n = d->n; a.m = d->m; a.N = d->N; a.hu_mode = d->hu_mode; a.batch = d->batch;
    hipError_t e = lqrx::ls_launch(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_err(e, "ls kernel launch");
    if (stream == nullptr) {
        if ((e = hipStreamSynchronize(nullptr)) != hipSuccess) return hip_err(e, "ls kernel");
        if (info) {
            std::vector<int32_t> h((size_t)d->batch);
            if ((e = hipMemcpy(h.data(), info, h.size() * 4, hipMemcpyDeviceToHost)) != hipSuccess)
                return hip_err(e, "info D2H");
            for (int32_t v : h)
                if (v) return 1;
        }
    }
    return 0;
}

extern "C" int lqrx_ls_solve_host(const lqrx_ls_desc *d, const double *A, const double *B, const double *Q,
                                  const double *R, const double *Qf, const double *x0, double *U, double *X,
                                  int32_t *info)
{
    int st = validate_ls(d);
    if (st) return st;
    if (d->batch == 0) return 0;
    const size_t bt = (size_t)d->batch, n = d->n, m = d->m, N = d->N;
    const size_t szin[6] = {n * n, n * m, n * n, m * m, n * n, n};
    const double *hin[6] = {A, B, Q, R, Qf, x0};
    DevBuf din[6], dU, dX, dinfo;
    for (int i = 0; i < 6; ++i) {
        if (!hin[i]) return set_err(-(i + 2), "input pointer %d is NULL", i + 2);
        if ((st = dev_alloc(din[i], szin[i] * 8 * bt, "hipMalloc input"))) return st;
        hipError_t e = hipMemcpy(din[i].p, hin[i], szin[i] * 8 * bt, hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_err(e, "H2D");
    }
    if (!U) return set_err(-8, "U is NULL");
    if (!X) return set_err(-9, "X is NULL");
    if ((st = dev_alloc(dU, (N - 1) * m * 8 * bt, "hipMalloc U"))) return st;
    if ((st = dev_alloc(dX, N * n * 8 * bt, "hipMalloc X"))) return st;
    if ((st = dev_alloc(dinfo, 4 * bt, "hipMalloc info"))) return st;
    st = lqrx_ls_solve(d, (const double *)din[0].p, (const double *)din[1].p, (const double *)din[2].p,
                       (const double *)din[3].p, (const double *)din[4].p, (const double *)din[5].p,
                       (double *)dU.p, (double *)dX.p, (int32_t *)dinfo.p, nullptr, nullptr, nullptr);
    if (st < 0) return st;
    hipError_t e;
    if ((e = hipMemcpy(U, dU.p, (N - 1) * m * 8 * bt, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(X, dX.p, N * n * 8 * bt, hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_err(e, "D2H");
    if (info && (e = hipMemcpy(info, dinfo.p, 4 * bt, hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_err(e, "D2H info");
    return st;
}
