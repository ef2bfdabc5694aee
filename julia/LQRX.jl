# LQRX.jl — the reference-side binding a LQR.jl maintainer would add to route the hot path
# through liblqrx.so (include/lqrx.h).  Text only: Julia is not installed in this image, so
# this file is not executed by the test-suite; the same C ABI is exercised from Python
# (ctypes, lqr.jl_amd/lqrx/_lib.py) and by the GPU parity tests.
#
# It keeps the reference surface:
#   LQRProblem / DPSolver / solve!(sol, solver, prob)   src/lqr_problem.jl:1-11,
#                                                        src/dynamic_programming.jl:2-72
#   LQRSolution (exported by src/LQR.jl:19 but never defined upstream; fields K, X, U)
# and adds batched forms over Array{T,3}/Array{T,4}, whose column-major memory with the
# batch index last is exactly the ABI's layout 0 (no copies).
module LQRX

using LinearAlgebra

const liblqrx = get(ENV, "LQRX_LIB", joinpath(@__DIR__, "..", "lqr.jl_amd", "lqrx", "liblqrx.so"))

# ---- lqrx_dp_desc (include/lqrx.h) ----
struct DpDesc
    n::Int32; m::Int32; N::Int32; dtype::Int32
    batch::Int64
    layout::Int32; p_mode::Int32
    knot_stride_AB::Int64; knot_stride_QR::Int64
end

lasterror() = unsafe_string(ccall((:lqrx_last_error, liblqrx), Cstring, ()))

function check(rc::Cint)
    rc < 0 && error("lqrx error $rc: $(lasterror())")
    return rc
end

dtypecode(::Type{Float64}) = Int32(0)
dtypecode(::Type{Float32}) = Int32(1)

"""
    LQRSolution(n, m, N, batch=1; T=Float64, all_P=false)
    LQRSolution(prob::LQRProblem)

The output container src/LQR.jl:19 exports but never defines, with the fields
src/dynamic_programming.jl touches: `sol.K[k]` (the m×n gain of knot k, :62, :68),
`sol.X[k]` (:66-69), `sol.U[k]` (:68-69) — for one problem these are Vectors of views (a
batch gives Matrices of views, `sol.K[k, b]`) into the column-major batch arrays Kdata
(m, n, N-1, batch), Xdata (n, N, batch), Udata (m, N-1, batch) that the C ABI writes in place
(layout 0, no copies); P = P₁ (or all P_k) and info (first non-SPD knot, 0 = ok).
"""
struct LQRSolution{T,VK,VX,VU}
    K::VK
    X::VX
    U::VU
    Kdata::Array{T,4}
    P::Array{T}
    Xdata::Array{T,3}
    Udata::Array{T,3}
    info::Vector{Int32}
end
function LQRSolution(n, m, N, batch=1; T=Float64, all_P=false)
    Kd = zeros(T, m, n, N - 1, batch)
    Xd = zeros(T, n, N, batch)
    Ud = zeros(T, m, N - 1, batch)
    P = all_P ? zeros(T, n, n, N, batch) : zeros(T, n, n, batch)
    if batch == 1
        K = [view(Kd, :, :, k, 1) for k in 1:N-1]
        X = [view(Xd, :, k, 1) for k in 1:N]
        U = [view(Ud, :, k, 1) for k in 1:N-1]
    else
        K = [view(Kd, :, :, k, b) for k in 1:N-1, b in 1:batch]
        X = [view(Xd, :, k, b) for k in 1:N, b in 1:batch]
        U = [view(Ud, :, k, b) for k in 1:N-1, b in 1:batch]
    end
    LQRSolution{T,typeof(K),typeof(X),typeof(U)}(K, X, U, Kd, P, Xd, Ud, zeros(Int32, batch))
end

"""
    LQRBatch(A, B, Q, R, Qf, x0, N)   A: n×n×batch, B: n×m×batch, …, x0: n×batch
"""
struct LQRBatch{T}
    A::Array{T,3}; B::Array{T,3}; Q::Array{T,3}; R::Array{T,3}; Qf::Array{T,3}
    x0::Matrix{T}; N::Int
end

"DPSolver(prob): the Julia struct owned the per-knot scratch; here it lives in registers/LDS."
struct DPSolver{T}
    n::Int; m::Int; N::Int
    P::Matrix{T}      # solver.P  — the cost-to-go compute_gain!/compute_ctg! start from (zero, as upstream)
    P_::Matrix{T}     # solver.P_ — what compute_ctg! produces
end
DPSolver{T}(n::Integer, m::Integer, N::Integer) where T = DPSolver{T}(n, m, N, zeros(T, n, n), zeros(T, n, n))
DPSolver(b::LQRBatch{T}) where T = DPSolver{T}(size(b.B, 1), size(b.B, 2), b.N)

"""
    solve!(sol, solver, prob::LQRBatch; devices=nothing)

Batched Riccati backward pass + forward rollout on the GPU (host arrays in, host arrays
out; lqrx_dp_solve_host).  Same outputs as src/dynamic_programming.jl:54-72 for every
problem in the batch; returns 1 if some trajectory had a non-SPD R + BᵀPB (see sol.info).
`devices = 0:7` shards the batch over those GPUs in the same call (lqrx_dp_solve_host_devices:
contiguous shards, one thread + stream per device, results bit-identical to one device).
"""
function solve!(sol::LQRSolution{T}, solver::DPSolver{T}, prob::LQRBatch{T};
                devices::Union{Nothing,AbstractVector{<:Integer}}=nothing) where T
    n, m, N = solver.n, solver.m, solver.N
    batch = size(prob.A, 3)
    all_P = ndims(sol.P) == 4
    d = Ref(DpDesc(n, m, N, dtypecode(T), batch, 0, all_P ? 1 : 0, 0, 0))
    if devices === nothing
        GC.@preserve prob sol begin
            rc = ccall((:lqrx_dp_solve_host, liblqrx), Cint,
                       (Ref{DpDesc}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T},
                        Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{Int32}),
                       d, prob.A, prob.B, prob.Q, prob.R, prob.Qf, prob.x0,
                       sol.Kdata, sol.P, sol.Xdata, sol.Udata, sol.info)
        end
    else
        dv = Vector{Int32}(devices)
        GC.@preserve prob sol dv begin
            rc = ccall((:lqrx_dp_solve_host_devices, liblqrx), Cint,
                       (Ref{DpDesc}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T},
                        Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{Int32}, Ptr{Int32}, Int32),
                       d, prob.A, prob.B, prob.Q, prob.R, prob.Qf, prob.x0,
                       sol.Kdata, sol.P, sol.Xdata, sol.Udata, sol.info, dv, Int32(length(dv)))
        end
    end
    return check(rc)
end

# ---- the reference's own single-problem surface (src/lqr_problem.jl:1-11) -------------
# LQRProblem{n,m,T,TQ,TR} with the reference's field order; Q/Qf/R may be Diagonal (TQ, TR)
# and A/B SizedMatrix — anything AbstractMatrix: solve! densifies them into the ABI buffers.
# With it the reference's three lines (test/dp.jl:14-20) run unchanged through the C ABI:
#     sol = LQRSolution(prob); solver = DPSolver(prob); solve!(sol, solver, prob)
struct LQRProblem{n,m,T,TQ,TR}
    Qf::TQ
    Q::TQ
    R::TR
    A::AbstractMatrix{T}
    B::AbstractMatrix{T}
    x0::AbstractVector{T}
    u0::AbstractVector{T}
    tf::T
    N::Int
end
LQRProblem(Qf::TQ, Q::TQ, R::TR, A::AbstractMatrix{T}, B::AbstractMatrix{T}, x0::AbstractVector,
           u0::AbstractVector, tf::Real, N::Integer) where {T,TQ,TR} =
    LQRProblem{size(B, 1),size(B, 2),T,TQ,TR}(Qf, Q, R, A, B, x0, u0, T(tf), Int(N))
Base.size(prob::LQRProblem{n,m}) where {n,m} = n, m, prob.N                    # lqr_problem.jl:21
num_vars(prob::LQRProblem{n,m}) where {n,m} = prob.N * n + (prob.N - 1) * m     # :22-25

LQRSolution(prob::LQRProblem{n,m,T}) where {n,m,T} = LQRSolution(n, m, prob.N, 1; T=T)
DPSolver(prob::LQRProblem{n,m,T}) where {n,m,T} = DPSolver{T}(n, m, prob.N)

"""
    solve!(sol, solver::DPSolver, prob::LQRProblem)

The reference's solve! (src/dynamic_programming.jl:54-72) for one problem: the
LQRProblem fields (Diagonal / Sized / dense) densified column-major into a batch of one,
lqrx_dp_solve_host, results written through sol.K[k], sol.X[k], sol.U[k] (views of
sol.Kdata …) and sol.P = solver.P₁.
"""
function solve!(sol::LQRSolution{T}, solver::DPSolver{T}, prob::LQRProblem{n,m,T}) where {n,m,T}
    dense3(M, r, c) = reshape(Matrix{T}(M), r, c, 1)      # Diagonal(q) → n×n, SizedMatrix → Matrix
    b = LQRBatch{T}(dense3(prob.A, n, n), dense3(prob.B, n, m), dense3(prob.Q, n, n),
                    dense3(prob.R, m, m), dense3(prob.Qf, n, n), reshape(Vector{T}(prob.x0), n, 1), prob.N)
    return solve!(sol, solver, b)
end
solve!(sol::LQRSolution{T}, prob::LQRProblem{n,m,T}) where {n,m,T} = solve!(sol, DPSolver(prob), prob)

"""
    compute_gain!(K, solver, prob);  compute_ctg!(K, solver, prob)

The reference's per-knot surface (src/dynamic_programming.jl:34-52, called by test/dp.jl:16-17
on `sol.K[1]`): K = (R + BᵀPB)⁻¹BᵀPA from P = solver.P, and for compute_ctg! also
solver.P_ = Q + AᵀPA − AᵀPB·K — lqrx_dp_compute_ctg_host (the same kernels as solve!, on a
2-knot problem with Qf = P).  P = solver.P and Q must be symmetric (the kernels' symmetric
fast form, include/lqrx.h): an asymmetry above max(1e-10, 100 eps(T)) of the largest entry
throws (Q is not checked by compute_gain!, where it never enters K).
"""
function compute_ctg!(K::AbstractMatrix{T}, solver::DPSolver{T}, prob::LQRProblem{n,m,T};
                      gain_only::Bool=false) where {n,m,T}
    dense(M, r, c) = reshape(Matrix{T}(M), r, c)
    A, B, Q, R = dense(prob.A, n, n), dense(prob.B, n, m), dense(prob.Q, n, n), dense(prob.R, m, m)
    rtol = max(1e-10, 100 * eps(T))            # never tighter than 100 ulp of T (fp32 AᵀPA)
    for (nm, M) in (gain_only ? (("P", solver.P),) : (("P", solver.P), ("Q", Q)))
        maximum(abs, M - transpose(M); init=zero(T)) > rtol * max(maximum(abs, M; init=zero(T)), floatmin(T)) &&
            throw(ArgumentError("compute_ctg!: $nm must be symmetric (lqrx_dp_compute_ctg precondition)"))
    end
    Kd = Matrix{T}(undef, m, n)
    info = Int32[0]
    d = Ref(DpDesc(n, m, 2, dtypecode(T), 1, 0, 0, 0, 0))
    GC.@preserve A B Q R solver Kd info begin
        rc = ccall((:lqrx_dp_compute_ctg_host, liblqrx), Cint,
                   (Ref{DpDesc}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{Int32}),
                   d, A, B, Q, R, solver.P, Kd, gain_only ? Ptr{T}(C_NULL) : pointer(solver.P_), info)
    end
    check(rc)
    K .= Kd
    return K
end
compute_gain!(K::AbstractMatrix{T}, solver::DPSolver{T}, prob::LQRProblem{n,m,T}) where {n,m,T} =
    compute_ctg!(K, solver, prob; gain_only=true)

# ---- linear cost terms (lqrx_dp_linear; SURVEY §8(f) rank 1, no upstream counterpart) ----
struct DpLinear
    q::Ptr{Cvoid}; r::Ptr{Cvoid}; qf::Ptr{Cvoid}
    d::Ptr{Cvoid}; p::Ptr{Cvoid}
end

"""
    solve_linear!(sol, d, p, solver, prob, q, r, qf)

Batched DP with stage cost ½xᵀQx + qᵀx + ½uᵀRu + rᵀu and terminal ½xᵀQf x + qfᵀx
(q: n×batch, r: m×batch, qf: n×batch).  Outputs as solve! plus the feedforward
d (m×(N-1)×batch, u_k = −K_k x_k − d_k) and the linear cost-to-go p (n×batch = p₁, or
n×N×batch with all_P).  lqrx_dp_solve_linear_host.
"""
function solve_linear!(sol::LQRSolution{T}, d::Array{T,3}, p::Array{T}, solver::DPSolver{T},
                       prob::LQRBatch{T}, q::Matrix{T}, r::Matrix{T}, qf::Matrix{T}) where T
    n, m, N = solver.n, solver.m, solver.N
    batch = size(prob.A, 3)
    all_P = ndims(sol.P) == 4
    desc = Ref(DpDesc(n, m, N, dtypecode(T), batch, 0, all_P ? 1 : 0, 0, 0))
    GC.@preserve prob sol d p q r qf begin
        lin = Ref(DpLinear(pointer(q), pointer(r), pointer(qf), pointer(d), pointer(p)))
        rc = ccall((:lqrx_dp_solve_linear_host, liblqrx), Cint,
                   (Ref{DpDesc}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ref{DpLinear},
                    Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{Int32}),
                   desc, prob.A, prob.B, prob.Q, prob.R, prob.Qf, prob.x0, lin,
                   sol.Kdata, sol.P, sol.Xdata, sol.Udata, sol.info)
    end
    return check(rc)
end

# ---- KKT: lqrx_kkt_desc ----
struct KktDesc
    N::Int32; dtype::Int32
    batch::Int64
    n1::Ptr{Int32}; p::Ptr{Int32}; n2::Ptr{Int32}; w::Ptr{Int32}
    h_mode::Int32; ginv::Int32; layout::Int32; reserved::Int32
end

"""
    kkt_solve!(dz, lam, info, n1, p, n2, w, Y, y, H, g; h_mode=2, ginv=1)

One CholeskySolver._solve! (src/cholesky_solver.jl:166-182) per trajectory: Y, y, H, g are
the per-knot ConstraintBlock.Y / .y, cost Hessian and gradient, packed (column-major
blocks, concatenated over knots) with the batch as the last dimension.  ginv=0 is the
second_order_correction! variant (:254-273).  `devices = 0:7` shards the batch over those GPUs
in the same call (lqrx_kkt_solve_host_devices).
"""
function kkt_solve!(dz::Matrix{T}, lam::Matrix{T}, info::Vector{Int32},
                    n1::Vector{Int32}, p::Vector{Int32}, n2::Vector{Int32}, w::Vector{Int32},
                    Y::Matrix{T}, y::Matrix{T}, H::Matrix{T}, g::Matrix{T};
                    h_mode::Integer=2, ginv::Integer=1,
                    devices::Union{Nothing,AbstractVector{<:Integer}}=nothing) where {T<:Union{Float64,Float32}}
    # Float32 runs the large-block MFMA kernels (blocks up to 64 rows, w up to 128 —
    # BASELINE configs[4]'s banded KKT) and the workgroup-per-trajectory kernel past them;
    # every H mode and ginv, blocks up to 512 rows and w up to 1024 in either precision
    batch = size(Y, 2)
    GC.@preserve n1 p n2 w Y y H g dz lam info begin
        d = Ref(KktDesc(length(n1), dtypecode(T), batch, pointer(n1), pointer(p), pointer(n2), pointer(w),
                        h_mode, ginv, 0, 0))
        if devices === nothing
            rc = ccall((:lqrx_kkt_solve_host, liblqrx), Cint,
                       (Ref{KktDesc}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{Int32}),
                       d, Y, y, H, g, dz, lam, info)
        else
            dv = Vector{Int32}(devices)
            rc = GC.@preserve dv ccall((:lqrx_kkt_solve_host_devices, liblqrx), Cint,
                       (Ref{KktDesc}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{T}, Ptr{Int32}, Ptr{Int32}, Int32),
                       d, Y, y, H, g, dz, lam, info, dv, Int32(length(dv)))
        end
    end
    return check(rc)
end

# ---- condensed least squares: lqrx_ls_desc ----
struct LsDesc
    n::Int32; m::Int32; N::Int32; hu_mode::Int32
    batch::Int64
end

"""
    ls_solve!(U, X, info, A, B, Q, R, Qf, x0, N; hu_mode=0)

solve!(sol, ::LeastSquaresSolver, prob) (src/least_squares.jl:158-192) for a batch:
A (n,n,batch), B (n,m,batch), Q, R, Qf, x0 (n,batch) → U ((N-1)m, batch) = sol.U_,
X (nN, batch).  hu_mode 0 = a fresh solver (Hu = 0, :44), 1 = after build_least_squares!
(Hu = chol(R).U blocks, :121), 2 = R blocks (the LQR cost).
"""
function ls_solve!(U::Matrix{Float64}, X::Matrix{Float64}, info::Vector{Int32},
                   A::Array{Float64,3}, B::Array{Float64,3}, Q::Array{Float64,3},
                   R::Array{Float64,3}, Qf::Array{Float64,3}, x0::Matrix{Float64}, N::Integer;
                   hu_mode::Integer=0)
    n, m, batch = size(B)
    d = Ref(LsDesc(n, m, N, hu_mode, batch))
    GC.@preserve A B Q R Qf x0 U X info begin
        rc = ccall((:lqrx_ls_solve_host, liblqrx), Cint,
                   (Ref{LsDesc}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                    Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int32}),
                   d, A, B, Q, R, Qf, x0, U, X, info)
    end
    return check(rc)
end

# ---- trajectory SQP: lqrx_sqp_desc ----
struct SqpDesc
    model::Int32; N::Int32; max_iters::Int32; stage_rows::Int32
    batch::Int64
    dt::Float64
    Q::NTuple{8,Float64}; R::NTuple{8,Float64}; Qf::NTuple{8,Float64}; params::NTuple{4,Float64}
    mu::Float64; tol_p::Float64; tol_d::Float64
    stage_A::NTuple{32,Float64}; stage_b::NTuple{4,Float64}
end
const MODEL_DUBINS, MODEL_CARTPOLE = Int32(0), Int32(1)
model_double_integrator(D) = Int32(1 + D)
pad(v, n) = ntuple(i -> i <= length(v) ? Float64(v[i]) : 0.0, n)

"""
    sqp_solve!(Z, lam, iters, status, x0, xf; model, N, dt, Q, R, Qf, params=(), mu=1,
               max_iters=10, tol_p=1e-5, tol_d=1e-5, stage_A=zeros(0,0), stage_b=Float64[])

CholeskySolver.solve! (src/cholesky_solver.jl:109-164) with the L1-merit line search of
test/dubins_sqp.jl:74-97 for a batch of trajectory problems of one model (Dubins car,
cartpole, DoubleIntegrator(D)); Z (N·n + (N−1)·m, batch) in/out, x0/xf (n, batch),
Q/R/Qf the diagonals of the LQRObjective, stage_A/stage_b the LinearConstraint of
DoubleIntegrator() on knots 2:N−1 (test/problems.jl:40-44).
"""
function sqp_solve!(Z::Matrix{Float64}, lam::Matrix{Float64}, iters::Vector{Int32},
                    status::Vector{Int32}, x0::Matrix{Float64}, xf::Matrix{Float64};
                    model::Integer, N::Integer, dt::Real, Q, R, Qf, params=(), mu::Real=1.0,
                    max_iters::Integer=10, tol_p::Real=1e-5, tol_d::Real=1e-5,
                    stage_A::Matrix{Float64}=zeros(0, 0), stage_b::Vector{Float64}=Float64[])
    d = Ref(SqpDesc(model, N, max_iters, length(stage_b), size(Z, 2), dt, pad(Q, 8), pad(R, 8),
                    pad(Qf, 8), pad(params, 4), mu, tol_p, tol_d, pad(vec(stage_A), 32),
                    pad(stage_b, 4)))
    GC.@preserve Z lam iters status x0 xf begin
        rc = ccall((:lqrx_sqp_solve_host, liblqrx), Cint,
                   (Ref{SqpDesc}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                    Ptr{Int32}, Ptr{Int32}),
                   d, Z, x0, xf, lam, iters, status)
    end
    return check(rc)
end

export LQRProblem, LQRSolution, LQRBatch, DPSolver, solve!, solve_linear!, kkt_solve!, ls_solve!,
       compute_gain!, compute_ctg!,
       sqp_solve!, num_vars

end # module
