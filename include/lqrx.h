/*
 * lqrx.h — C ABI of the MI355X-native batched LQR / block-tridiagonal-KKT solver.
 *
 * Drop-in boundary for the hot path of bjack205/LQR.jl.  The reference has no FFI: its
 * only native boundary is Julia stdlib `ccall`s into LAPACK/BLAS, one call per knot-op
 * (SURVEY.md §1, §2 "native arithmetic" table).  This ABI replaces those calls at batch
 * grain — one call per batch of independent problems — and is what a Julia `ccall` shim
 * binds (INTEGRATION.md shows the shim).
 *
 * Conventions (all entry points):
 *   - plain C types only; `extern "C"`; no exceptions cross the boundary;
 *   - the caller owns every buffer; the library never frees or retains caller pointers;
 *   - layout 0 = Julia column-major with the batch index slowest, i.e. exactly the memory
 *     of Array{T,3}(r,c,batch) / Array{T,4}(r,c,knots,batch) — no copy from Julia;
 *   - return 0 on success; -i if argument i (1-based) is invalid (LAPACK convention);
 *     1 if the call completed synchronously and at least one trajectory has info != 0;
 *     LQRX_ERR_* (< -99) for runtime failures; lqrx_last_error() describes the last error
 *     of the calling thread;
 *   - `stream` is a hipStream_t: NULL = synchronous (like the reference's solve!), else the
 *     work is enqueued and the call returns immediately (check info[] after syncing);
 *   - reentrant and thread-safe.  Mutable library state, all of it process-wide and
 *     mutex-guarded: the calling thread's last-error string (thread-local); one HIP
 *     memory pool per device for stream-ordered scratch (created on first use, blocks kept
 *     mapped); a cache of uploaded KKT block-structure tables (≤ 4096 distinct structures,
 *     never evicted — each is uploaded once, with a blocking copy, on its first use; calls
 *     with further structures upload a per-call table on their own stream and wait for that
 *     stream only); environment switches read once.  All of it is keyed on the device of
 *     the call's `stream`, not on the thread's current device.  No call synchronises the
 *     whole device.
 */
#ifndef LQRX_H
#define LQRX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LQRX_ABI_VERSION 5   /* 2: layout 1 (DP, KKT), lqrx_sqp_* (models, stage constraints);
                                3: lqrx_dp_solve_linear[_host] (linear cost terms), and
                                   dtype LQRX_F32 on the KKT path (large-block kernels);
                                4: lqrx_scratch_trim (release the library's pooled scratch);
                                   KKT blocks past 64 rows (up to 512, w up to 1024);
                                   KKT layout 1 for every structure (staged);
                                   lqrx_dp_compute_ctg[_host] (per-knot surface);
                                5: lqrx_*_host_devices (one call sharded over GPUs) */

#define LQRX_F64 0
#define LQRX_F32 1

#define LQRX_ERR_HIP (-100)         /* HIP runtime error (see lqrx_last_error)          */
#define LQRX_ERR_UNSUPPORTED (-101) /* valid but not (yet) supported shape / option    */
#define LQRX_ERR_NODEVICE (-102)    /* no gfx950 device / HIP runtime unavailable        */

/* ------------------------------------------------------------------------------------
 * DP path: Riccati backward pass + forward rollout.
 * Replaces solve!(sol::LQRSolution, solver::DPSolver, prob::LQRProblem)
 *   /root/reference/src/dynamic_programming.jl:54-72
 * including compute_gain!/compute_ctg!/chol_solve! (:28-52) and the DPSolver scratch
 * (:2-23: owned by the library, stream-ordered).  Problem data = LQRProblem fields
 * (/root/reference/src/lqr_problem.jl:1-11): time-invariant A (n×n), B (n×m), Q (n×n),
 * R (m×m), Qf (n×n), x0 (n), horizon N knots.
 *
 * Buffers (layout 0, element type per dtype):
 *   A  n·n·batch     B  n·m·batch    Q  n·n·batch    R  m·m·batch    Qf n·n·batch
 *      (×(N-1) per trajectory for time-varying fields, see knot_stride_*; the
 *       time-varying path is SURVEY §8(f) rank 1; every supported n, m)
 *   x0 n·batch
 *   K  m·n·(N-1)·batch     sol.K[k], k = 1..N-1  (LQRSolution.K)
 *   P  n·n·batch  (p_mode 0: P_1 = solver.P on return, :63)
 *      n·n·N·batch (p_mode 1: P_k for k = 1..N, P_N = Qf)
 *   X  n·N·batch           sol.X
 *   U  m·(N-1)·batch       sol.U
 *   info int32·batch : 0, or the knot k (1-based) of the first E = R + BᵀPB found not
 *        positive definite in the backward sweep (the reference discards potrf's info,
 *        dynamic_programming.jl:29; the solve still runs to completion, as there).
 * ------------------------------------------------------------------------------------ */
typedef struct lqrx_dp_desc {
    int32_t n, m, N;        /* state dim, control dim, knots (N >= 2); 1 <= n, m <= 512
                               (n <= 4: lane kernels; n <= 64, m <= 32: register-tiled
                               MFMA kernel; beyond: workgroup-per-trajectory kernel)      */
    int32_t dtype;          /* LQRX_F64 (reference precision) or LQRX_F32            */
    int64_t batch;          /* number of independent problems                          */
    int32_t layout;         /* 0 = column-major blocks, batch slowest (Julia Array{T,3});
                               1 = batch fastest (SoA): element e of trajectory b at
                               [e·batch + b], e = its layout-0 offset within the
                               trajectory (Julia permutedims(X, (3,1,2)), Python [S][batch]);
                               every array of the call (inputs and outputs) uses it.  Native
                               in the n ≤ 4 kernels (coalesced per element); n ≥ 5 converts
                               to layout 0 in stream-ordered scratch and back (2× traffic) */
    int32_t p_mode;         /* 0 = P_1 only (reference-observable), 1 = all P_k        */
    int64_t knot_stride_AB; /* 0 = time-invariant A, B (reference LQRProblem);
                               1 = per knot: A n·n·(N-1)·batch, B n·m·(N-1)·batch, knot k
                               at index k-1 (LCRProblem.A/.B, constrained_problem.jl:3-4) */
    int64_t knot_stride_QR; /* 0 = time-invariant Q, R; 1 = per knot: Q n·n·(N-1)·batch,
                               R m·m·(N-1)·batch (Qf stays the terminal cost)            */
} lqrx_dp_desc;

/* device pointers (hipMalloc'd or torch CUDA/HIP tensors) */
int lqrx_dp_solve(const lqrx_dp_desc *desc, const void *A, const void *B, const void *Q,
                  const void *R, const void *Qf, const void *x0, void *K, void *P, void *X,
                  void *U, int32_t *info, void *stream);

/* host pointers: H2D, solve, D2H, synchronous (what the Julia shim calls by default) */
int lqrx_dp_solve_host(const lqrx_dp_desc *desc, const void *A, const void *B, const void *Q,
                       const void *R, const void *Qf, const void *x0, void *K, void *P,
                       void *X, void *U, int32_t *info);

/* Per-knot DP surface — compute_ctg!(K, solver, prob) (dynamic_programming.jl:45-52, which
 * runs compute_gain! :34-43 first) for a batch of problems, from P = solver.P (P_{k+1}):
 *   K  = E⁻¹BᵀPA  with E = R + BᵀPB   (m·n·batch, sol.K[k])
 *   P_ = Q + AᵀPA − APB·K               (n·n·batch, solver.P_; NULL = compute_gain! only)
 * A, B, Q, R, P as lqrx_dp_solve's A, B, Q, R, Qf (time-invariant; desc.N, p_mode and the
 * knot strides are ignored); info as lqrx_dp_solve (1 = E not positive definite).  The same
 * kernels as lqrx_dp_solve (a 2-knot solve with Qf = P).
 * Precondition: P and Q symmetric, as every cost-to-go and cost Hessian of the recursion is.
 * The n ≥ 5 and n ≤ 4 kernel families use the symmetric fast form (P_ = Q + AᵀPA − GᵀK on the
 * lower triangle, mirrored), the n > 64 workgroup kernel the reference's operation order, so
 * for a non-symmetric P or Q the result depends on the family.  The host wrappers (Python
 * lqrx.compute_ctg*, Julia compute_ctg!) reject P or Q whose asymmetry exceeds
 * max(1e-10, 100 ulp of the dtype) of the matrix's largest entry (Q only when P_ is asked). */
int lqrx_dp_compute_ctg(const lqrx_dp_desc *desc, const void *A, const void *B, const void *Q,
                        const void *R, const void *P, void *K, void *P_, int32_t *info, void *stream);
int lqrx_dp_compute_ctg_host(const lqrx_dp_desc *desc, const void *A, const void *B, const void *Q,
                             const void *R, const void *P, void *K, void *P_, int32_t *info);

/* ------------------------------------------------------------------------------------
 * DP path with linear cost terms — SURVEY §8(f) rank 1 ("time-varying LQR … and cost
 * linear terms"), an extension of the reference LQRProblem (lqr_problem.jl:1-11 has no
 * linear terms).  Stage cost ½xᵀQx + qᵀx + ½uᵀRu + rᵀu, terminal ½xᵀQf x + qfᵀx; the
 * value function gains a linear part V_k(x) = ½xᵀP_k x + p_kᵀx and the policy a
 * feedforward: u_k = −K_k x_k − d_k.  In the reference's op order (oracle/lqr_oracle.c
 * oracle_dp_solve_one_lin): d_k = E⁻¹(r_k + Bᵀp_{k+1}) is one more right-hand side of
 * chol_solve! (dynamic_programming.jl:42), p_k = q_k + Aᵀp_{k+1} − APB·d_k follows :51.
 * Same descriptor, inputs and outputs as lqrx_dp_solve plus:
 *   q   n·batch, or n·(N−1)·batch when knot_stride_QR = 1 (knot k at k−1, like Q)
 *   r   m·batch, or m·(N−1)·batch when knot_stride_QR = 1
 *   qf  n·batch
 *   d   out: m·(N−1)·batch   feedforward d_k, k = 1..N−1
 *   p   out: n·batch (p_mode 0: p_1) or n·N·batch (p_mode 1: p_k, p_N = qf)
 * layout 1 applies to these arrays as well.  All zero q, r, qf give the lqrx_dp_solve
 * results (with d = 0, p = 0).
 * ------------------------------------------------------------------------------------ */
typedef struct lqrx_dp_linear {
    const void *q, *r, *qf; /* linear cost terms (inputs)        */
    void *d, *p;            /* feedforward, linear cost-to-go (outputs) */
} lqrx_dp_linear;

int lqrx_dp_solve_linear(const lqrx_dp_desc *desc, const void *A, const void *B,
                         const void *Q, const void *R, const void *Qf, const void *x0,
                         const lqrx_dp_linear *lin, void *K, void *P, void *X, void *U,
                         int32_t *info, void *stream);

/* host pointers in lin and everywhere else: H2D, solve, D2H, synchronous */
int lqrx_dp_solve_linear_host(const lqrx_dp_desc *desc, const void *A, const void *B,
                              const void *Q, const void *R, const void *Qf, const void *x0,
                              const lqrx_dp_linear *lin, void *K, void *P, void *X, void *U,
                              int32_t *info);

/* ------------------------------------------------------------------------------------
 * KKT path: one inner solve of CholeskySolver._solve!(solver)
 *   /root/reference/src/cholesky_solver.jl:166-182
 * = calculate_shur_factors! (jacobian_blocks.jl:220-286) → cholesky!(chol, shur)
 *   (cholesky_solve.jl:47-67) → forward_/backward_substitution! (:93-143) →
 *   calculate_primals! (cholesky_solver.jl:185-236); ginv = 0 gives the
 *   second_order_correction! variant (cholesky_solver.jl:254-273): δẑ = −Dᵀ(DDᵀ)⁻¹d.
 *
 * Block structure (shared by the whole batch) = ConstraintBlocks (conblocks.jl:403-425):
 * knot k (0-based here) has n1[k] previous-dynamics rows D2, p[k] stage rows C, n2[k]
 * dynamics rows D1 and width w[k] (= n̄ + m for k < N-1, n̄ at the last knot).
 * Packed per-trajectory inputs, each block column-major, concatenated over k:
 *   Y  (n1+p+n2)×w   Y = [D2; C; D1]   (ConstraintBlock.Y)
 *   y  p+n2          y = [c; d]        (ConstraintBlock.y)
 *   H  h_mode 0/1: w×w cost Hessian (dense / block-diagonal Q,R; BlockCholesky modes,
 *      block_cholesky.jl:55-77);  h_mode 2: the w diagonal entries (:82-91)
 *   g  w             gradient [q; r]  (InvertedQuadratic gradient, block_cholesky.jl:126)
 * Outputs:
 *   dz  w per knot  (δZ, get_step ordering [x1;u1;…;xN])
 *   lam p+n2 per knot  [μ_k; λ_k]  (get_multipliers ordering)
 *   info int32·batch: 0 ok; k+1 if a Schur diagonal block at knot k was not SPD;
 *        −(k+1) if H_k was not SPD.
 * ------------------------------------------------------------------------------------ */
typedef struct lqrx_kkt_desc {
    int32_t N;          /* knots                                                  */
    int32_t dtype;      /* LQRX_F64 (every KKT kernel: the compile-time shapes, the
                           padded bins for trajectory structures up to n̄ <= 8, m <= 4
                           — dense / block-diagonal H on both through an H = UᵀU
                           pre/post pass — then the large-block and workgroup kernels)
                           or LQRX_F32 (layout 0: the
                           large-block MFMA kernels for n1, p, n2 <= 64, padded rows
                           <= 128, w <= 128, and the workgroup-per-trajectory kernel
                           past them; every h_mode and ginv; else
                           LQRX_ERR_UNSUPPORTED).  Every knot: n1, p, n2 <= 512 and
                           w <= 1024 (LQRX_ERR_UNSUPPORTED past that)               */
    int64_t batch;
    const int32_t *n1;  /* [N] host arrays describing the block structure           */
    const int32_t *p;   /* [N]                                                      */
    const int32_t *n2;  /* [N]                                                      */
    const int32_t *w;   /* [N]                                                      */
    int32_t h_mode;     /* 0 dense, 1 block-diagonal, 2 diagonal                    */
    int32_t ginv;       /* 1 = _solve!;  0 = second-order-correction variant        */
    int32_t layout;     /* 0 = per-trajectory packed, batch slowest: element e of
                           trajectory t's packed array (Y, y, H, g, dz, lam) at
                           [t·len + e];  1 = batch fastest (SoA) at [e·batch + t] —
                           a wave's 64 trajectories read each element as one 512-B
                           row.  Layout 1 is read natively by the compile-time shapes,
                           (n̄, m, p_first, p_interior, p_last) = Dubins (3,2,3,0,3) every
                           h_mode; cartpole (4,1,4,0,4), DoubleIntegrator(2)/(3)
                           (4,2,4,1,4)/(6,3,6,1,6), trajectory_structure(5,2,N) /
                           (7,3,N) (5,2,5,0,5)/(7,3,7,0,7) with diagonal H or ginv = 0;
                           fp64; N >= 4.  Every other layout-1 call is staged: the
                           arrays are transposed to layout 0 in library scratch, solved
                           by the layout-0 kernels and dz / lam transposed back (2x
                           the bytes).  Layout 1 arrays < 2 GiB.                      */
    int32_t reserved;
} lqrx_kkt_desc;

int lqrx_kkt_solve(const lqrx_kkt_desc *desc, const void *Y, const void *y, const void *H,
                   const void *g, void *dz, void *lam, int32_t *info, void *stream);
int lqrx_kkt_solve_host(const lqrx_kkt_desc *desc, const void *Y, const void *y,
                        const void *H, const void *g, void *dz, void *lam, int32_t *info);
/* Caller-provided workspace (the factor slab): no allocation inside the call — the form a
 * serving loop or a captured hipGraph wants.  lqrx_kkt_workspace_size gives the bytes this
 * structure and batch need (0 for batch 0); lqrx_kkt_solve_ws returns -10 if
 * workspace_bytes is smaller.  One workspace must not be shared by calls in flight on
 * different streams (lqrx_kkt_solve draws stream-ordered scratch from a library pool).
 * Large blocks: the slab (+ Schur images) is sized for the batch but capped at
 * LQRX_KKT_BIG_SLAB_MB (default 40 GiB); a larger batch runs in chunks through it.  Without
 * a caller workspace that scratch comes from the library pool, whose freed blocks stay
 * reserved for the next call (up to the cap) until lqrx_scratch_trim; an out-of-memory pool
 * allocation retries with halved chunks.  A layout-1 call whose structure has no native SoA
 * kernel is staged through layout 0: its six transposed arrays (Y y H g, δz λ) are part of
 * the workspace too (counted by lqrx_kkt_workspace_size, carved from its front), so a _ws call
 * draws no pool scratch in any layout. */
int lqrx_kkt_workspace_size(const lqrx_kkt_desc *desc, size_t *bytes);
int lqrx_kkt_solve_ws(const lqrx_kkt_desc *desc, const void *Y, const void *y, const void *H,
                      const void *g, void *dz, void *lam, int32_t *info, void *workspace,
                      size_t workspace_bytes, void *stream);
/* sizes (elements per trajectory) of the packed KKT buffers, for allocation */
int lqrx_kkt_sizes(const lqrx_kkt_desc *desc, int64_t *nY, int64_t *ny, int64_t *nH,
                   int64_t *ng, int64_t *nlam);

/* ------------------------------------------------------------------------------------
 * Multi-device host entries — SURVEY.md §8(e): "the batch of independent problems shards
 * embarrassingly across the 8 GPUs of one node".  Same arguments and results as the *_host
 * call they extend (lqrx_dp_solve_host, lqrx_dp_solve_linear_host, lqrx_kkt_solve_host; the
 * reference's solve! per shard, dynamic_programming.jl:54-72 / cholesky_solver.jl:166-182),
 * plus devices[ndev]: HIP device ordinals, repeats allowed (two shards on one GPU).  The batch
 * is split into ndev contiguous shards (trajectories [b0, b0 + nb), the first batch mod ndev
 * shards one longer); each runs concurrently on its own thread and non-blocking stream on its
 * device: its slice of every input is copied in (layout 1: the strided slice of every element
 * row), solved by the single-device path, and K/P/X/U (δz/λ) and info land in the caller's
 * host arrays at the shard's offset.  No collective and no peer traffic: the gather IS the
 * D2H into the caller's arrays.  Every trajectory is solved exactly as by the single-device
 * call, so results are bit-identical (n ≤ 4 DP: when the shard batches pick the same quad /
 * lane kernel as the whole batch, ≤ 16384 trajectories per shard or > 16384 in both).
 * Returns -13 / -14 (dp), -14 / -15 (dp linear), -9 / -10 (kkt) for a NULL devices / an
 * entry that is not a device, and ndev < 1; a failing shard's status, with its device and
 * trajectory range in lqrx_last_error; 1 if any trajectory has info != 0. */
int lqrx_dp_solve_host_devices(const lqrx_dp_desc *desc, const void *A, const void *B, const void *Q,
                               const void *R, const void *Qf, const void *x0, void *K, void *P,
                               void *X, void *U, int32_t *info, const int32_t *devices, int32_t ndev);
int lqrx_dp_solve_linear_host_devices(const lqrx_dp_desc *desc, const void *A, const void *B,
                                      const void *Q, const void *R, const void *Qf, const void *x0,
                                      const lqrx_dp_linear *lin, void *K, void *P, void *X, void *U,
                                      int32_t *info, const int32_t *devices, int32_t ndev);
int lqrx_kkt_solve_host_devices(const lqrx_kkt_desc *desc, const void *Y, const void *y,
                                const void *H, const void *g, void *dz, void *lam, int32_t *info,
                                const int32_t *devices, int32_t ndev);

/* ------------------------------------------------------------------------------------
 * Batched trajectory-optimisation SQP around the KKT path: per
 * trajectory, the outer loop of CholeskySolver.solve!/step! (/root/reference/src/
 * cholesky_solver.jl:109-153) with the KKT inputs assembled on the device (update!, :155-164:
 * RK3 dynamics Jacobians, diagonal LQRObjective expansion), _solve! (:166-182), and the
 * L1-merit backtracking line search with second-order correction of test/dubins_sqp.jl:58-97
 * (SOC = second_order_correction!, cholesky_solver.jl:254-273).
 *
 * Models (continuous dynamics, integrated with RobotDynamics' RK3 at step dt; Jacobians by
 * forward-mode dual numbers on the device, as ForwardDiff does in the reference):
 *   LQRX_MODEL_DUBINS   nx 3, nu 2: RobotZoo.DubinsCar ẋ = [v cosθ, v sinθ, ω]
 *                       (test/dubins_sqp.jl); params unused
 *   LQRX_MODEL_CARTPOLE nx 4, nu 1: RobotZoo.Cartpole, x = [x, θ, ẋ, θ̇],
 *                       params = {mc, mp, l, g} (RobotZoo defaults 1, 0.2, 0.5, 9.81;
 *                       test/problems.jl:58-88 Cartpole())
 *   LQRX_MODEL_DOUBLE_INTEGRATOR{1,2,3}  nx 2D, nu D: RobotZoo.DoubleIntegrator(D),
 *                       ẋ = [q̇; u] (test/problems.jl:14-56 DoubleIntegrator(D)); params unused
 * Problem: min Σ_{k<N} ½(x_k−xf)ᵀQ(x_k−xf) + ½u_kᵀRu_k + ½(x_N−xf)ᵀQf(x_N−xf)
 *          s.t. x_1 = x0, x_{k+1} = rk3(x_k, u_k), x_N = xf      (Q, R, Qf diagonal)
 *          and, when stage_rows > 0, A_s x_k = b_s on the interior knots k = 2..N−1 (the
 *          LinearConstraint DoubleIntegrator() adds on 2:N−1; A_s shared by the batch)
 * Buffers (device; layout 0, batch slowest), nx / nu of the model:
 *   Z      (N·nx + (N−1)·nu)·batch in/out: z = [x_1; u_1; …; x_{N−1}; u_{N−1}; x_N]
 *          (the KKT δz order)
 *   x0, xf nx·batch
 *   lam    (nx(N+1) + stage_rows(N−2))·batch out: multipliers of the last accepted Newton
 *          step (KKT λ order)
 *   iters  int32·batch out: accepted steps
 *   status int32·batch out: 0 converged (‖c‖∞ < tol_p and ‖∇f+∇cᵀλ‖₂ < tol_d before a
 *          step), 1 max_iters reached, 2 line search failed (iterate left unchanged)
 * ------------------------------------------------------------------------------------ */
enum {
    LQRX_MODEL_DUBINS = 0,
    LQRX_MODEL_CARTPOLE = 1,
    LQRX_MODEL_DOUBLE_INTEGRATOR1 = 2,
    LQRX_MODEL_DOUBLE_INTEGRATOR2 = 3,
    LQRX_MODEL_DOUBLE_INTEGRATOR3 = 4
};

typedef struct lqrx_sqp_desc {
    int32_t model;          /* LQRX_MODEL_*                                            */
    int32_t N;              /* knots (>= 2)                                            */
    int32_t max_iters;      /* CholeskySolver.solve!: 10                               */
    int32_t stage_rows;     /* rows of the interior linear constraint, 0..2 (nx·rows ≤ 32) */
    int64_t batch;
    double dt;              /* tf / (N−1)                                              */
    double Q[8], R[8], Qf[8]; /* diagonal cost weights (> 0), first nx / nu used         */
    double params[4];       /* model parameters (see above)                            */
    double mu;              /* L1 merit weight (dubins_sqp.jl:59 uses 1)               */
    double tol_p, tol_d;    /* 1e-5, 1e-5 (cholesky_solver.jl:131-132)                 */
    double stage_A[32];     /* A_s, stage_rows × nx column-major                        */
    double stage_b[4];      /* b_s                                                      */
} lqrx_sqp_desc;

/* state / control dimension of a model; -1 for an unknown model */
int lqrx_sqp_model_dims(int32_t model, int32_t *nx, int32_t *nu);
int lqrx_sqp_solve(const lqrx_sqp_desc *desc, double *Z, const double *x0, const double *xf,
                   double *lam, int32_t *iters, int32_t *status, void *stream);
int lqrx_sqp_solve_host(const lqrx_sqp_desc *desc, double *Z, const double *x0, const double *xf,
                        double *lam, int32_t *iters, int32_t *status);

/* The round-1 Dubins-only entry points (model fixed to LQRX_MODEL_DUBINS); they forward to
 * lqrx_sqp_solve[_host]. */
typedef struct lqrx_dubins_sqp_desc {
    int32_t N;
    int32_t max_iters;
    int64_t batch;
    double dt;
    double Q[3], R[2], Qf[3];
    double mu;
    double tol_p, tol_d;
} lqrx_dubins_sqp_desc;

int lqrx_dubins_sqp_solve(const lqrx_dubins_sqp_desc *desc, double *Z, const double *x0,
                          const double *xf, double *lam, int32_t *iters, int32_t *status,
                          void *stream);
int lqrx_dubins_sqp_solve_host(const lqrx_dubins_sqp_desc *desc, double *Z, const double *x0,
                               const double *xf, double *lam, int32_t *iters, int32_t *status);

/* ------------------------------------------------------------------------------------
 * Condensed least-squares LQR: replaces
 * solve!(sol, ::LeastSquaresSolver, prob) (/root/reference/src/least_squares.jl:158-192)
 * with opts :solve_type => :cholesky — Ā/b̄ as buildAb! builds them (:58-103),
 * H = ĀᵀĀ + Hu, y = −Āᵀb̄ (:171-173), potrf/potrs 'U' (:181-182), rollout! (:197-202).
 * One workgroup per trajectory.  (N−1)·m ≤ 192 and lqrx_ls_lds_bytes(n, m, N) <= 163840
 * (e.g. n=4, m=1: N ≤ 189; n=3, m=2: N ≤ 97): the whole problem in LDS.  Larger problems up to
 * (N−1)·m ≤ 1024 keep H in stream-ordered global scratch (Nm(Nm+1)/2 doubles per trajectory)
 * with a blocked factor — e.g. the reference's own LS test problem, DoubleIntegrator()
 * n=6, m=3, N=101 (Nm = 300); lqrx_ls_lds_bytes reports the LDS of the path taken.
 *   hu_mode 0: Hu = 0 — a fresh LeastSquaresSolver (:44), the reference default; the
 *              solve then carries no control cost
 *           1: Hu = blkdiag(chol(R).U) — what build_least_squares! leaves (:121)
 *           2: Hu = blkdiag(R) — the LQR cost; U then equals the DP rollout (extension)
 * Inputs (device, layout 0, batch slowest, time-invariant): A n×n, B n×m, Q n×n, R m×m,
 * Qf n×n, x0 n.  Outputs: U (N−1)·m per trajectory (sol.U_), X N·n (sol.X);
 * Abar (N·n)×((N−1)·m) col-major and bbar N·n per trajectory when non-NULL (buildAb!'s Ā,
 * b̄, for checks).  info[b]: 0 ok, j > 0 = potrf pivot j of H not positive, −1 = Q, Qf
 * (or R for hu_mode 1) not positive definite (cholesky() throws there, :50-52).
 * Return: 0 ok, 1 some info ≠ 0 (synchronous calls only), < 0 as above.
 * ------------------------------------------------------------------------------------ */
typedef struct lqrx_ls_desc {
    int32_t n, m, N;
    int32_t hu_mode;
    int64_t batch;
} lqrx_ls_desc;

size_t lqrx_ls_lds_bytes(int32_t n, int32_t m, int32_t N);
int lqrx_ls_solve(const lqrx_ls_desc *desc, const double *A, const double *B, const double *Q,
                  const double *R, const double *Qf, const double *x0, double *U, double *X,
                  int32_t *info, double *Abar, double *bbar, void *stream);
int lqrx_ls_solve_host(const lqrx_ls_desc *desc, const double *A, const double *B,
                       const double *Q, const double *R, const double *Qf, const double *x0,
                       double *U, double *X, int32_t *info);

/* ------------------------------------------------------------------------------------
 * Utilities
 * ------------------------------------------------------------------------------------ */
int lqrx_abi_version(void);
/* "src_sha256=<SHA-256 of the library's sources> abi=<n> arch=gfx950 built=<date time>": the
 * hash covers lqr.jl_amd/csrc/{*.hip,*.h,*.cpp} (sorted by name) then include/lqrx.h, so a
 * caller can check that the loaded binary was built from the sources beside it */
const char *lqrx_build_info(void);
const char *lqrx_last_error(void);
/* copy the calling thread's last error message into buf (NUL-terminated, truncated to
 * len-1 bytes); returns the full message length.  For bindings that cannot hold a
 * pointer into library memory (SURVEY.md §8(b) lqrx_get_last_error). */
int lqrx_get_last_error(char *buf, size_t len);
/* 1 if the HIP runtime sees a gfx950 device, else 0 (no compute; safe without a GPU) */
int lqrx_device_available(void);
/* Return the library pool's unused stream-ordered scratch of `device` (-1: every device
 * the library has used) to the driver, keeping at most keep_bytes reserved.  Blocks still in
 * use by enqueued work are not affected.  Returns 0, or LQRX_ERR_HIP. */
int lqrx_scratch_trim(int32_t device, size_t keep_bytes);

/* Deterministic synthetic random-dense LQR batch: counter-based
 * splitmix64 + Box–Muller keyed by (seed, trajectory, field, element); host memory,
 * multi-threaded.  A = I + (0.1/√n)G, B = G/√n, Q = I + GᵀG/n, R = I + GᵀG/m, Qf = 10Q,
 * x0 ~ N(0,1).  traj0 offsets the trajectory index (to generate one shard of a batch). */
int lqrx_make_random_dp(int32_t n, int32_t m, int64_t batch, int64_t traj0, uint64_t seed,
                        int32_t dtype, void *A, void *B, void *Q, void *R, void *Qf,
                        void *x0);

#ifdef __cplusplus
}
#endif
#endif /* LQRX_H */
