// lqrx_internal.h — kernel argument blocks shared by the launchers and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <vector>
#include <stdint.h>

namespace lqrx {

struct DpArgs {
    const void *A, *B, *Q, *R, *Qf, *x0; // device inputs, layout 0
    void *K, *P, *X, *U;                 // device outputs
    int32_t *info;                       // device [batch] or null
    int n, m, N;
    int dtype; // 0 f64, 1 f32
    int p_all;
    int64_t batch;
    int tv_AB, tv_QR; // 1 = per-knot A_k,B_k / Q_k,R_k (N−1 knots per trajectory), 0 = time-invariant
    int layout;       // 0 = per-trajectory blocks, batch slowest; 1 = batch fastest (SoA):
                      // element e of trajectory b at [e·batch + b] (e = the layout-0 offset
                      // within the trajectory) — native in the n ≤ 4 kernels
    // linear cost terms (lqrx_dp_solve_linear; lin = 0: the plain reference problem):
    // q, r per knot with tv_QR (knot stride n / m), qf; outputs d (m per knot), p (n, or
    // n per knot with p_all)
    int lin;
    const void *q, *r, *qf;
    void *d, *p;
    // tests only (LQRX_DP_NS_OFF=1, read by dp_launch): no Newton–Schulz step, every knot takes the
    // exact LDLᵀ sweep — exercises the sweep / verdict paths of the MFMA kernels at every knot
    int ns_off;
};

hipError_t dp_launch(const DpArgs &a, hipStream_t s);
// out = inᵀ for a rows × cols row-major matrix of 4- or 8-byte elements (lqrx_layout.hip):
// layout 1 (SoA, [S][batch]) ↔ layout 0 ([batch][S]) for the kernels that need layout 0
hipError_t batch_transpose(const void *in, void *out, int64_t rows, int64_t cols, int elem_bytes, hipStream_t s);
bool dp_supported(int dtype, int n, int m, bool tv);
// lane-per-trajectory kernel for n ≤ 4, m ≤ 4 (lqrx_dp_lane.hip)
hipError_t dp_lane_launch(const DpArgs &a, hipStream_t s);
bool dp_lane_supported(int n, int m);
// workgroup-per-trajectory kernel for shapes past the register tiles (lqrx_dp_big.hip):
// n > 64 or m > 32, up to 512 each
hipError_t dp_big_launch(const DpArgs &a, hipStream_t s);
bool dp_big_supported(int n, int m);

struct KktArgs {
    const double *Y, *y, *H, *g; // device, packed per trajectory
    double *dz, *lam;
    int32_t *info;
    const int32_t *meta; // device: per knot {n1, p, n2, w, oY, oy, oH, og(=oz), ol}
    int N;
    int h_mode, ginv;
    int64_t batch;
    int64_t sY, sy, sH, sg, sl; // per-trajectory strides (elements)
    int maxw, maxrows, max_p1, max_ps, max_p2;
    int force_lane; // debug: LQRX_KKT_FORCE_LANE=1 selects the register-only kernel
    int layout;     // 0 per-trajectory packed; 1 batch fastest (compile-time shapes only)
    int dtype;      // 0 f64; 1 f32 (the big-block kernels only: Y..lam then point at floats)
    // internal (SQP): solve only the trajectories sel[0 .. *nsel) (device arrays; layout-0
    // LDS-staged kernel only — the other kernels solve the whole batch, which is also correct)
    const int32_t *sel, *nsel;
    void *ws;         // caller's device workspace (lqrx_kkt_solve_ws) or NULL: library pool
    size_t ws_bytes;
    // runtime (n̄, m, P0, PK, PN) of a trajectory-form structure solved on a padded compile-time
    // shape (lqrx_kkt_fil.hip, Shape<…, PAD>); unused otherwise
    int32_t rt[5];
    // live trajectories per 64-lane wave of the direct FIL kernel (lqrx_kkt_fil.hip kkt_fild_kernel,
    // layout 0; set by its launcher): 64, or 32 on small batches so that twice the waves run
    int32_t lpw;
};

hipError_t kkt_launch(const KktArgs &a, hipStream_t s);
// which generic (runtime-shaped, fp64) kernel kkt_launch would pick: 0 none, 1 LDS-staged
// ≤ (3,3,3,5,6), 2 lane ≤ (4,4,4,8,8), 3 lane ≤ (8,8,8,12,16) (runtime-indexed arrays in scratch)
int kkt_generic_class(const KktArgs &a);

// Stream-ordered scratch from a library-owned memory pool (one per device) whose release
// threshold keeps freed blocks mapped: a per-call hipMallocAsync/hipFreeAsync pair then
// costs no page-table work after the first call (the default pool returns memory at every
// synchronisation — measured +0.26 ms per 357 MB KKT slab).  Reentrant: blocks are
// stream-ordered, never shared between calls.  (lqrx_api.cpp)
hipError_t scratch_alloc(void **p, size_t bytes, hipStream_t s);
hipError_t scratch_free(void *p, hipStream_t s);
hipError_t scratch_trim(int device, size_t keep);   // lqrx_scratch_trim
// a launch's slab: the caller's workspace when one was passed, else a pool block
struct Scratch {
    void *p = nullptr;
    bool owned = false;
    hipError_t get(const KktArgs &a, size_t bytes, hipStream_t s)
    {
        if (a.ws) {
            if (a.ws_bytes < bytes) return hipErrorInvalidValue;
            p = a.ws;
            return hipSuccess;
        }
        owned = true;
        return scratch_alloc(&p, bytes, s);
    }
    hipError_t release(hipStream_t s) { return owned ? scratch_free(p, s) : hipSuccess; }
};
// slab bytes the generic kernels need (mirrors kkt_launch's selection; 0 = unsupported)
size_t kkt_scratch_bytes(const KktArgs &a);
// compile-time-shaped kernel for first/interior/last structures (lqrx_kkt_fil.hip); returns
// false (and launches nothing) when the structure has no instantiation
bool kkt_fil_launch(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                    const int32_t *w, hipStream_t s, hipError_t *err);
// slab bytes of the FIL kernel for this structure; false when no FIL shape serves it
bool kkt_fil_scratch_bytes(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                           const int32_t *w, size_t *bytes);

// large-block MFMA kernels (lqrx_kkt_big.hip): any structure with n1, p, n2 ≤ 64, padded
// rows ≤ 128, w ≤ 128, diagonal H or the SOC variant, layout 0, fp64 or fp32
bool kkt_big_supported(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2, const int32_t *w);
size_t kkt_big_scratch_bytes(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                             const int32_t *w);
hipError_t kkt_big_launch(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                          const int32_t *w, hipStream_t s);

// workgroup-per-trajectory KKT kernel (lqrx_kkt_wg.hip): the structures past the large-block
// kernels (any block > 64 rows or w > 128), every h_mode / ginv, layout 0, fp64 or fp32
constexpr int KW_MAX_BLOCK = 512, KW_MAX_W = 1024;
bool kkt_wg_supported(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2, const int32_t *w);
size_t kkt_wg_scratch_bytes(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                            const int32_t *w);
hipError_t kkt_wg_launch(const KktArgs &a, const int32_t *n1, const int32_t *p, const int32_t *n2,
                         const int32_t *w, hipStream_t s);

// ---- batched trajectory SQP (lqrx_sqp.hip) ----
enum { SQP_DUBINS = 0, SQP_CARTPOLE = 1, SQP_DI1 = 2, SQP_DI2 = 3, SQP_DI3 = 4 };   // = LQRX_MODEL_*
struct SqpArgs {
    int model, N, stage_rows;         // stage_rows: PK of the interior-knot linear constraint
    double SA[32], Sb[4];             // A_s (PK × NX, column-major), b_s
    int64_t B;
    double dt, mu, tol_p, tol_d;
    double Q[8], R[8], Qf[8];         // diagonal weights, first NX / NU used
    double par[4];                    // model parameters (cartpole: mc, mp, l, g)
    const double *x0, *xf;            // B×NX
    double *Z;                        // B×NN, in/out
    double *lam;                      // B×P: multipliers of the last accepted Newton step
    int32_t *iters, *status;          // B
    double *Y, *y, *H, *g;            // KKT inputs, ABI layout (internal)
    double *dz, *lamn, *dzs;          // Newton step + its multipliers, SOC step
    double *phi0, *dphi;              // B
    int32_t *need_soc;                // B
    int32_t *n_active;                // 1
    int32_t *sel, *nsel;              // B, 1: the trajectories the next KKT solve needs
};
// kkt(ctx, ginv, dz, sel, nsel): one KKT solve of the trajectories sel[0 .. *nsel)
hipError_t sqp_run(const SqpArgs &A, int max_iters, hipStream_t s,
                   int (*kkt)(void *ctx, int ginv, double *dz, const int32_t *sel, const int32_t *nsel), void *ctx,
                   int *kkt_rc);
void sqp_structure(int nx, int nu, int pk, int N, std::vector<int32_t> &n1, std::vector<int32_t> &p,
                   std::vector<int32_t> &n2, std::vector<int32_t> &w);
bool sqp_model_dims(int model, int *nx, int *nu);

// ---- condensed least-squares LQR (lqrx_ls.hip) ----
struct LsArgs {
    const double *A, *B, *Q, *R, *Qf, *x0;
    double *U, *X, *Ab, *bb;
    int32_t *info;
    int n, m, N, hu_mode;
    int64_t batch;
};
size_t ls_lds_bytes(int n, int m, int N);
int ls_max_nm();          // (N−1)·m cap (the big, global-H path)
hipError_t ls_launch(const LsArgs &a, hipStream_t s);

} // namespace lqrx
