# ENFHip.jl -- Julia ccall binding of libenf.so (include/enf.h) for bat/EuclidianNormalizingFlows.jl.
#
# NOT EXECUTED IN THIS PIPELINE: Julia is not installed in the build image nor on the GPU boxes
# (SURVEY.md §0). This file is the reference-side binding a maintainer adds; it mirrors
# include/enf.h one to one and is reviewed against the Python host mirror
# (euclidiannormalizingflows.jl_amd/trafos.py), which exercises the same C ABI in tests/.
#
# It adds methods (no type piracy: they dispatch on the package-owned HipMatrix) to the generic
# functions the reference extends (src/EuclidianNormalizingFlows.jl:38-40):
#     (f)(X::HipMatrix), ChangesOfVariables.with_logabsdet_jacobian(f, X::HipMatrix)
# for f any of ScaleShiftTrafo, CenterStretch, CenterContract, JohnsonTrafo, JohnsonTrafoInv,
# HouseholderTrafo, or a ComposedFunction of them -- a composition is flattened into ONE
# enf_flow_apply call (one fused kernel launch). InverseFunctions.inverse stays the reference's.
module ENFHip

using ChangesOfVariables, InverseFunctions
import ChangesOfVariables: with_logabsdet_jacobian
using EuclidianNormalizingFlows: ScaleShiftTrafo, CenterStretch, CenterContract, JohnsonTrafo,
                                 JohnsonTrafoInv, HouseholderTrafo

const libenf = get(ENV, "ENF_LIBRARY", "libenf.so")

const ENF_F32, ENF_F64 = Cint(0), Cint(1)
const OP_SCALESHIFT, OP_CENTER_STRETCH, OP_CENTER_CONTRACT = Int32(0), Int32(1), Int32(2)
const OP_JOHNSON, OP_JOHNSON_INV, OP_HOUSEHOLDER = Int32(3), Int32(4), Int32(5)

# enf_layer (include/enf.h)
struct EnfLayer
    op::Int32
    k::Int32
    p::NTuple{4,Ptr{Cvoid}}
end

# --- device memory owned by this module -------------------------------------------------------
mutable struct HipBuffer
    ptr::Ptr{Cvoid}
    bytes::Int
    function HipBuffer(bytes::Integer)
        r = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:enf_malloc, libenf), Cint, (Ref{Ptr{Cvoid}}, Csize_t), r, bytes))
        b = new(r[], bytes)
        finalizer(b -> ccall((:enf_free, libenf), Cint, (Ptr{Cvoid},), b.ptr), b)
        b
    end
end

"""Column-major D x N matrix resident on the GPU (Julia's sample-per-column convention)."""
struct HipMatrix{T<:Union{Float32,Float64}}
    buf::HipBuffer
    D::Int
    N::Int
end
HipMatrix{T}(D::Integer, N::Integer) where {T} = HipMatrix{T}(HipBuffer(max(D * N, 1) * sizeof(T)), D, N)
Base.size(X::HipMatrix) = (X.D, X.N)
Base.eltype(::HipMatrix{T}) where {T} = T

function HipMatrix(A::AbstractMatrix{T}) where {T<:Union{Float32,Float64}}
    X = HipMatrix{T}(size(A)...)
    Ac = Matrix{T}(A)
    check(ccall((:enf_memcpy, libenf), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Int32, Ptr{Cvoid}),
                X.buf.ptr, Ac, sizeof(Ac), 0, C_NULL))
    check(ccall((:enf_stream_synchronize, libenf), Cint, (Ptr{Cvoid},), C_NULL))
    X
end

function Base.Array(X::HipMatrix{T}) where {T}
    A = Matrix{T}(undef, X.D, X.N)
    check(ccall((:enf_memcpy, libenf), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Int32, Ptr{Cvoid}),
                A, X.buf.ptr, sizeof(A), 1, C_NULL))
    check(ccall((:enf_stream_synchronize, libenf), Cint, (Ptr{Cvoid},), C_NULL))
    A
end

function check(status::Cint)
    status == 0 && return nothing
    msg = unsafe_string(ccall((:enf_last_error, libenf), Cstring, ()))
    error("libenf error $status: $msg")
end

# --- flattening: layer list, innermost first; params uploaded as length-D device vectors -------
_vec(p::Real, D, ::Type{T}) where {T} = fill(T(p), D)
_vec(p::AbstractVector, D, ::Type{T}) where {T} = (length(p) == D || throw(DimensionMismatch()); Vector{T}(p))

_leaves(f::ComposedFunction) = vcat(_leaves(f.inner), _leaves(f.outer))
_leaves(f) = Any[f]

_op(::ScaleShiftTrafo) = (OP_SCALESHIFT, (:a, :b))
_op(::CenterStretch) = (OP_CENTER_STRETCH, (:a, :b, :c))
_op(::CenterContract) = (OP_CENTER_CONTRACT, (:a, :b, :c))
_op(::JohnsonTrafo) = (OP_JOHNSON, (:gamma, :delta, :xi, :lambda))
_op(::JohnsonTrafoInv) = (OP_JOHNSON_INV, (:gamma, :delta, :xi, :lambda))
_op(::HouseholderTrafo) = (OP_HOUSEHOLDER, (:V,))

function _layers(fs, D, ::Type{T}) where {T}
    keep = HipMatrix[]
    layers = EnfLayer[]
    for f in fs
        op, names = _op(f)
        ptrs = Ptr{Cvoid}[C_NULL, C_NULL, C_NULL, C_NULL]
        k = 0
        for (q, nm) in enumerate(names)
            p = getfield(f, nm)
            A = op == OP_HOUSEHOLDER ? Matrix{T}(reshape(p, D, :)) : reshape(_vec(p, D, T), D, 1)
            op == OP_HOUSEHOLDER && (k = size(A, 2))
            M = HipMatrix(A)
            push!(keep, M)
            ptrs[q] = M.buf.ptr
        end
        push!(layers, EnfLayer(op, Int32(k), Tuple(ptrs)))
    end
    layers, keep
end

const _Supported = Union{ScaleShiftTrafo,CenterStretch,CenterContract,JohnsonTrafo,JohnsonTrafoInv,
                         HouseholderTrafo,ComposedFunction}

function _apply(f, X::HipMatrix{T}, want_ladj::Bool) where {T}
    fs = _leaves(f)
    layers, keep = _layers(fs, X.D, T)
    Y = HipMatrix{T}(X.D, X.N)
    ladj = want_ladj ? HipMatrix{T}(1, X.N) : nothing
    check(ccall((:enf_flow_apply, libenf), Cint,
                (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int32,
                 Ptr{EnfLayer}, Int32, Ptr{Cvoid}),
                T === Float64 ? ENF_F64 : ENF_F32, X.D, X.N, X.buf.ptr, X.D, Y.buf.ptr, X.D,
                want_ladj ? ladj.buf.ptr : C_NULL, 0, layers, length(layers), C_NULL))
    GC.@preserve keep nothing
    Y, ladj
end

# (f)(X) and with_logabsdet_jacobian(f, X): one fused launch; ladj is a 1 x N HipMatrix (Julia's
# Adjoint row, src/abstract_trafo.jl:9)
(f::ScaleShiftTrafo)(X::HipMatrix) = _apply(f, X, false)[1]
(f::CenterStretch)(X::HipMatrix) = _apply(f, X, false)[1]
(f::CenterContract)(X::HipMatrix) = _apply(f, X, false)[1]
(f::JohnsonTrafo)(X::HipMatrix) = _apply(f, X, false)[1]
(f::JohnsonTrafoInv)(X::HipMatrix) = _apply(f, X, false)[1]
(f::HouseholderTrafo)(X::HipMatrix) = _apply(f, X, false)[1]

with_logabsdet_jacobian(f::_Supported, X::HipMatrix) = _apply(f, X, true)

# mvnormal_negll_trafograd (src/optimize_whitening.jl:18-22) for a flow over a HipMatrix batch:
# (negll, flat gradient in the enf_flow_param_count layout: layer by layer, field by field).
# Device sums over the batch, normalised here by the batch size; a data-parallel caller sums the
# unnormalised buffer across ranks first (enf_allreduce_sum) and divides by the global size.
function mvnormal_negll_trafograd(f::_Supported, X::HipMatrix{T}) where {T}
    layers, keep = _layers(_leaves(f), X.D, T)
    dt = T === Float64 ? ENF_F64 : ENF_F32
    np = Ref{Int64}(0)
    check(ccall((:enf_flow_param_count, libenf), Cint, (Int64, Ptr{EnfLayer}, Int32, Ref{Int64}),
                X.D, layers, length(layers), np))
    wsb = Ref{Csize_t}(0)
    check(ccall((:enf_flow_negll_grad_workspace, libenf), Cint,
                (Cint, Int64, Int64, Ptr{EnfLayer}, Int32, Ref{Csize_t}),
                dt, X.D, X.N, layers, length(layers), wsb))
    out = HipMatrix(zeros(T, 1 + np[], 1))
    ws = HipBuffer(max(Int(wsb[]), 1))
    check(ccall((:enf_flow_negll_grad, libenf), Cint,
                (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{EnfLayer}, Int32, Ptr{Cvoid}, Ptr{Cvoid},
                 Csize_t, Ptr{Cvoid}),
                dt, X.D, X.N, X.buf.ptr, X.D, layers, length(layers), out.buf.ptr, ws.ptr, wsb[], C_NULL))
    GC.@preserve keep nothing
    g = Array(out)[:, 1] ./ X.N
    g[1], g[2:end]
end

# optimize_whitening (src/optimize_whitening.jl:25-45) over a device-resident sample matrix: one
# enf_whitening_step per minibatch (gradient, negll, the Optimisers ADAGrad update and the
# HouseholderTrafo re-normalisation, three launches) on one flat device parameter vector theta in
# the enf_flow_param_count layout, the layer pointers pointing into theta. Array fields are
# trainable, as Optimisers treats them; scalar fields are broadcast for the kernels and kept.
# Minibatches as the reference's: batchsize = round(Int, N/nbatches), Iterators.partition over the
# columns, the last one possibly shorter. optimizer_state is the device pair (theta, acc). A method
# of the reference's own generic function (dispatch on the shim's HipMatrix, no type piracy).
import Optimisers
import EuclidianNormalizingFlows: optimize_whitening

_fieldvec(p, D, ::Type{T}) where {T} = p isa AbstractArray ? _vec(vec(p), D, T) : fill(T(p), D)

function optimize_whitening(smpls::HipMatrix{T}, initial_trafo::Function, optimizer::Optimisers.ADAGrad;
                            nbatches::Integer = 100, nepochs::Integer = 100,
                            negll_history = Vector{Float64}()) where {T}
    D, N = smpls.D, smpls.N
    fs = _leaves(initial_trafo)
    host, offs, runs, hb = T[], Int[], Int64[], Int64[]
    for f in fs
        op, names = _op(f)
        for nm in names
            p = getfield(f, nm)
            v = op == OP_HOUSEHOLDER ? vec(Matrix{T}(reshape(p, D, :))) : _fieldvec(p, D, T)
            o = length(host)
            push!(offs, o)
            append!(host, v)
            p isa AbstractArray && append!(runs, (o, o + length(v)))      # [start, end) of theta
            op == OP_HOUSEHOLDER && append!(hb, (o, length(v) ÷ D, D))    # (offset, columns, stride)
        end
    end
    theta = HipMatrix(reshape(host, :, 1))
    acc = HipMatrix(fill(T(optimizer.epsilon), length(host), 1))  # Optimisers.init(ADAGrad, x)
    layers = EnfLayer[]
    i = 0
    for f in fs
        op, names = _op(f)
        ptrs = Ptr{Cvoid}[C_NULL, C_NULL, C_NULL, C_NULL]
        for q in eachindex(names)
            i += 1
            ptrs[q] = theta.buf.ptr + offs[i] * sizeof(T)
        end
        k = op == OP_HOUSEHOLDER ? Int32(length(getfield(f, :V)) ÷ D) : Int32(0)
        push!(layers, EnfLayer(op, k, Tuple(ptrs)))
    end
    dt = T === Float64 ? ENF_F64 : ENF_F32
    batchsize = max(round(Int, N / nbatches), 1)
    starts = 0:batchsize:N-1
    wsb = Ref{Csize_t}(0)
    check(ccall((:enf_flow_negll_grad_workspace, libenf), Cint,
                (Cint, Int64, Int64, Ptr{EnfLayer}, Int32, Ref{Csize_t}),
                dt, D, batchsize, layers, length(layers), wsb))
    ws = HipBuffer(max(Int(wsb[]), 1))
    hist = HipMatrix{Float64}(1, nepochs * length(starts))
    s = 0
    for _ in 1:nepochs, b0 in starts
        B = min(b0 + batchsize, N) - b0
        check(ccall((:enf_whitening_step, libenf), Cint,
                    (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{EnfLayer}, Int32, Ptr{Cvoid}, Ptr{Cvoid},
                     Ptr{Int64}, Int32, Ptr{Int64}, Int32, Cdouble, Cdouble, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t,
                     Ptr{Cvoid}),
                    dt, D, B, smpls.buf.ptr + b0 * D * sizeof(T), D, layers, length(layers), theta.buf.ptr,
                    acc.buf.ptr, runs, length(runs) ÷ 2, hb, length(hb) ÷ 3, optimizer.eta, optimizer.epsilon,
                    hist.buf.ptr + s * sizeof(Float64), ws.ptr, wsb[], C_NULL))
        s += 1
    end
    # Functors-style reconstruction of the trained flow from theta
    th = vec(Array(theta))
    i = 0
    rebuilt = map(fs) do f
        op, names = _op(f)
        vals = map(names) do nm
            i += 1
            p = getfield(f, nm)
            p isa AbstractArray || return p
            reshape(eltype(p).(th[offs[i]+1:offs[i]+length(p)]), size(p))
        end
        typeof(f).name.wrapper(vals...)
    end
    trafo = foldl((acc_, f) -> f ∘ acc_, rebuilt[2:end]; init = rebuilt[1])
    (result = trafo, optimizer_state = (theta = theta, acc = acc),
     negll_history = vcat(negll_history, vec(Array(hist))))
end

# JohnsonSU (src/johnson_trafo.jl:120-129) over a 1 x n HipMatrix of values: pdf.(d, X) etc. on the
# device (enf_johnsonsu_eval), rand(d, n) as quantile of a Philox4x32-10 stream (enf_johnsonsu_sample).
using EuclidianNormalizingFlows: JohnsonSU
import Distributions

const ENF_JSU_PDF, ENF_JSU_LOGPDF, ENF_JSU_CDF, ENF_JSU_LOGCDF = Int32(0), Int32(1), Int32(2), Int32(3)
const ENF_JSU_CCDF, ENF_JSU_LOGCCDF, ENF_JSU_QUANTILE = Int32(4), Int32(5), Int32(6)

function _jsu(fn::Int32, d::JohnsonSU, X::HipMatrix{T}) where {T}
    out = HipMatrix{T}(X.D, X.N)
    check(ccall((:enf_johnsonsu_eval, libenf), Cint,
                (Cint, Int32, Int64, Ptr{Cvoid}, Ptr{Cvoid}, Cdouble, Cdouble, Cdouble, Cdouble, Ptr{Cvoid}),
                T === Float64 ? ENF_F64 : ENF_F32, fn, X.D * X.N, X.buf.ptr, out.buf.ptr,
                d.gamma, d.delta, d.xi, d.lambda, C_NULL))
    out
end

jsu_pdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_PDF, d, X)
jsu_logpdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_LOGPDF, d, X)
jsu_cdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_CDF, d, X)
jsu_logcdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_LOGCDF, d, X)
jsu_ccdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_CCDF, d, X)
jsu_logccdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_LOGCCDF, d, X)
jsu_quantile(d::JohnsonSU, P::HipMatrix) = _jsu(ENF_JSU_QUANTILE, d, P)

function jsu_rand(d::JohnsonSU, ::Type{T}, n::Integer; seed::UInt64 = UInt64(0), offset::UInt64 = UInt64(0)) where {T}
    out = HipMatrix{T}(1, n)
    check(ccall((:enf_johnsonsu_sample, libenf), Cint,
                (Cint, Int64, Ptr{Cvoid}, Cdouble, Cdouble, Cdouble, Cdouble, UInt64, UInt64, Ptr{Cvoid}),
                T === Float64 ? ENF_F64 : ENF_F32, n, out.buf.ptr, d.gamma, d.delta, d.xi, d.lambda,
                seed, offset, C_NULL))
    out
end

export HipMatrix, mvnormal_negll_trafograd, optimize_whitening, jsu_pdf, jsu_logpdf, jsu_cdf, jsu_logcdf, jsu_ccdf,
       jsu_logccdf, jsu_quantile, jsu_rand

end # module
