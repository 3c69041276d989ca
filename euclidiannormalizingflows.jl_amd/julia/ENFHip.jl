# ENFHip.jl -- Julia ccall binding of libenf.so (include/enf.h) for bat/EuclidianNormalizingFlows.jl.
#
# NOT EXECUTED IN THIS PIPELINE: Julia is not installed in the build image nor on the GPU boxes
# (SURVEY.md §0), so no line of this file has been run. What IS checked, on every CPU test run
# (tests/test_julia_binding.py): every ccall's symbol, return type, argument types and argument count
# against the prototypes of include/enf.h, the EnfLayer layout against enf_layer, and the constants
# against the header's enums. The semantics it implements are those of the Python host mirror
# (euclidiannormalizingflows.jl_amd/trafos.py, train.py, jsu.py), which runs the same C ABI in tests/.
#
# It adds methods -- dispatching on the shim's own HipMatrix, so no type piracy -- to the reference's
# generic functions:
#     (f)(X::HipMatrix), ChangesOfVariables.with_logabsdet_jacobian(f, X::HipMatrix)
#         for f any of ScaleShiftTrafo, CenterStretch, CenterContract, JohnsonTrafo, JohnsonTrafoInv,
#         HouseholderTrafo, or a ComposedFunction of them (src/EuclidianNormalizingFlows.jl:38-40);
#     EuclidianNormalizingFlows.mvnormal_negll_trafo / mvnormal_negll_trafograd
#         (src/optimize_whitening.jl:7-22), EuclidianNormalizingFlows.optimize_whitening (:25-45);
#     Distributions.pdf / logpdf / cdf / logcdf / ccdf / logccdf, Statistics.quantile and rand for
#         JohnsonSU over a HipMatrix (src/johnson_trafo.jl:120-129).
# A composition runs as ONE enf_flow_apply call (one fused kernel launch) per run of equal promoted
# element type. InverseFunctions.inverse stays the reference's (host-side parameter algebra).
module ENFHip

using ChangesOfVariables, InverseFunctions
import ChangesOfVariables: with_logabsdet_jacobian
import EuclidianNormalizingFlows: mvnormal_negll_trafo, mvnormal_negll_trafograd, optimize_whitening
using EuclidianNormalizingFlows: ScaleShiftTrafo, CenterStretch, CenterContract, JohnsonTrafo,
                                 JohnsonTrafoInv, HouseholderTrafo, JohnsonSU
import Distributions, Statistics, Random, Optimisers

const libenf = get(ENV, "ENF_LIBRARY", "libenf.so")

# enums of include/enf.h (checked against the header by tests/test_julia_binding.py)
const ENF_F32, ENF_F64 = Cint(0), Cint(1)
# dtype flag of the training calls (include/enf.h): the loss reported is the one the reference records under
# Zygote -- rrule(similar_fill) makes every ScaleShiftTrafo's primal ladj zero (src/abstract_trafo.jl:30-33)
const ENF_NEGLL_ZYGOTE = Cint(0x100)
const OP_SCALESHIFT, OP_CENTER_STRETCH, OP_CENTER_CONTRACT = Int32(0), Int32(1), Int32(2)
const OP_JOHNSON, OP_JOHNSON_INV, OP_HOUSEHOLDER = Int32(3), Int32(4), Int32(5)
const ENF_JSU_PDF, ENF_JSU_LOGPDF, ENF_JSU_CDF, ENF_JSU_LOGCDF = Int32(0), Int32(1), Int32(2), Int32(3)
const ENF_JSU_CCDF, ENF_JSU_LOGCCDF, ENF_JSU_QUANTILE = Int32(4), Int32(5), Int32(6)
const ENF_UNIQUE_ID_BYTES = 128
const MEMCPY_H2D, MEMCPY_D2H, MEMCPY_D2D = Int32(0), Int32(1), Int32(2)

# enf_layer (include/enf.h)
struct EnfLayer
    op::Int32
    k::Int32
    p::NTuple{4,Ptr{Cvoid}}
end

_dt(::Type{Float32}) = ENF_F32
_dt(::Type{Float64}) = ENF_F64

function check(status::Cint)
    status == 0 && return nothing
    msg = unsafe_string(ccall((:enf_last_error, libenf), Cstring, ()))
    error("libenf error $status: $msg")
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

function _memcpy(dst::Ptr{Cvoid}, src::Ptr{Cvoid}, bytes::Integer, kind::Int32)
    check(ccall((:enf_memcpy, libenf), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Int32, Ptr{Cvoid}),
                dst, src, bytes, kind, C_NULL))
    check(ccall((:enf_stream_synchronize, libenf), Cint, (Ptr{Cvoid},), C_NULL))
end

function HipMatrix(A::AbstractMatrix{T}) where {T<:Union{Float32,Float64}}
    X = HipMatrix{T}(size(A)...)
    Ac = Matrix{T}(A)
    GC.@preserve X Ac _memcpy(X.buf.ptr, Ptr{Cvoid}(pointer(Ac)), sizeof(Ac), MEMCPY_H2D)
    X
end

function Base.Array(X::HipMatrix{T}) where {T}
    A = Matrix{T}(undef, X.D, X.N)
    GC.@preserve X A _memcpy(Ptr{Cvoid}(pointer(A)), X.buf.ptr, sizeof(A), MEMCPY_D2H)
    A
end

Base.copy(X::HipMatrix{T}) where {T} = (Y = HipMatrix{T}(X.D, X.N);
                                        GC.@preserve X Y _memcpy(Y.buf.ptr, X.buf.ptr, X.D * X.N * sizeof(T), MEMCPY_D2D);
                                        Y)

# element-type conversion of a device matrix (host round trip: only mixed-precision flows need it)
_convert(X::HipMatrix{T}, ::Type{T}) where {T} = X
_convert(X::HipMatrix, ::Type{R}) where {R} = HipMatrix(R.(Array(X)))

# --- flattening: layer list, innermost first; params uploaded as length-D device vectors -------
# A scalar field and a length-1 vector field are broadcast to D rows (the reference's broadcasting
# of muladd.(x, a, b) etc.); any other length must be D.
function _vec(p, D, ::Type{T}) where {T}
    p isa Real && return fill(T(p), D)
    length(p) == D && return Vector{T}(vec(p))
    length(p) == 1 && return fill(T(first(p)), D)
    throw(DimensionMismatch("parameter of length $(length(p)) for D = $D"))
end

_leaves(f::ComposedFunction) = vcat(_leaves(f.inner), _leaves(f.outer))
_leaves(f) = Any[f]

_op(::ScaleShiftTrafo) = (OP_SCALESHIFT, (:a, :b))
_op(::CenterStretch) = (OP_CENTER_STRETCH, (:a, :b, :c))
_op(::CenterContract) = (OP_CENTER_CONTRACT, (:a, :b, :c))
_op(::JohnsonTrafo) = (OP_JOHNSON, (:gamma, :delta, :xi, :lambda))
_op(::JohnsonTrafoInv) = (OP_JOHNSON_INV, (:gamma, :delta, :xi, :lambda))
_op(::HouseholderTrafo) = (OP_HOUSEHOLDER, (:V,))

_ptype(p::AbstractArray) = eltype(p)
_ptype(p::Real) = typeof(p)
_paramtypes(f) = map(nm -> _ptype(getfield(f, nm)), _op(f)[2])

# float(promote_type(...)) layer by layer, as the reference's elementwise functions compute
# (src/johnson_trafo.jl:30, src/center_stretch.jl:5): the running type only widens, so a flow is at
# most a Float32 run followed by a Float64 run.
function _promoted(::Type{T}, f) where {T}
    R = float(promote_type(T, _paramtypes(f)...))
    R === Float32 || R === Float64 || throw(ArgumentError("libenf computes in Float32/Float64, not $R"))
    R
end

function _segments(fs, ::Type{T}) where {T}
    segs = Tuple{DataType,Vector{Any}}[]
    cur = T
    for f in fs
        R = _promoted(cur, f)
        if !isempty(segs) && segs[end][1] === R
            push!(segs[end][2], f)
        else
            push!(segs, (R, Any[f]))
        end
        cur = R
    end
    segs
end

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
        # ScaleShiftTrafo with a length-1 vector `a`: k = 1, its ladj constant log|a[1]| counts once
        # (src/scale_shift_trafo.jl:22; enf_layer.k in include/enf.h)
        op == OP_SCALESHIFT && f.a isa AbstractVector && length(f.a) == 1 && (k = 1)
        push!(layers, EnfLayer(op, Int32(k), Tuple(ptrs)))
    end
    layers, keep
end

const _Supported = Union{ScaleShiftTrafo,CenterStretch,CenterContract,JohnsonTrafo,JohnsonTrafoInv,
                         HouseholderTrafo,ComposedFunction}

function _apply(f, X::HipMatrix{T}, want_ladj::Bool) where {T}
    Y = X
    L = nothing
    for (R, fs) in _segments(_leaves(f), T)
        Xs = _convert(Y, R)
        Ys = HipMatrix{R}(Xs.D, Xs.N)
        accumulate = L !== nothing
        L = want_ladj ? (accumulate ? _convert(L, R) : HipMatrix{R}(1, Xs.N)) : nothing
        layers, keep = _layers(fs, Xs.D, R)
        GC.@preserve Xs Ys L layers keep begin
            check(ccall((:enf_flow_apply, libenf), Cint,
                        (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int32,
                         Ptr{EnfLayer}, Int32, Ptr{Cvoid}),
                        _dt(R), Xs.D, Xs.N, Xs.buf.ptr, Xs.D, Ys.buf.ptr, Xs.D,
                        want_ladj ? L.buf.ptr : C_NULL, accumulate ? 1 : 0, layers, length(layers), C_NULL))
        end
        Y = Ys
    end
    Y, L
end

# (f)(X) and with_logabsdet_jacobian(f, X): one fused launch per dtype run; ladj is a 1 x N
# HipMatrix (Julia's Adjoint row, src/abstract_trafo.jl:9)
(f::ScaleShiftTrafo)(X::HipMatrix) = _apply(f, X, false)[1]
(f::CenterStretch)(X::HipMatrix) = _apply(f, X, false)[1]
(f::CenterContract)(X::HipMatrix) = _apply(f, X, false)[1]
(f::JohnsonTrafo)(X::HipMatrix) = _apply(f, X, false)[1]
(f::JohnsonTrafoInv)(X::HipMatrix) = _apply(f, X, false)[1]
(f::HouseholderTrafo)(X::HipMatrix) = _apply(f, X, false)[1]

with_logabsdet_jacobian(f::_Supported, X::HipMatrix) = _apply(f, X, true)

# Host-resident batch (enf_flow_apply_host): X, Y, ladj in host memory, chunks streamed through the
# device. Not a method of a reference generic (Matrix is not the shim's type).
function stream_with_logabsdet_jacobian(f::_Supported, X::Matrix{T}; chunk_cols::Integer = 0,
                                        want_ladj::Bool = true) where {T<:Union{Float32,Float64}}
    segs = _segments(_leaves(f), T)
    length(segs) == 1 && segs[1][1] === T ||
        throw(ArgumentError("stream_with_logabsdet_jacobian: parameters would promote X's element type"))
    D, N = size(X)
    Y = similar(X)
    L = want_ladj ? zeros(T, 1, N) : nothing
    layers, keep = _layers(segs[1][2], D, T)
    GC.@preserve X Y L layers keep begin
        check(ccall((:enf_flow_apply_host, libenf), Cint,
                    (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int32,
                     Ptr{EnfLayer}, Int32, Int64, Ptr{Cvoid}),
                    _dt(T), D, N, Ptr{Cvoid}(pointer(X)), D, Ptr{Cvoid}(pointer(Y)), D,
                    want_ladj ? Ptr{Cvoid}(pointer(L)) : C_NULL, 0, layers, length(layers), chunk_cols, C_NULL))
    end
    Y, L
end

# --- mvnormal_negll_trafo / mvnormal_negll_trafograd (src/optimize_whitening.jl:7-22) ----------

# negll = -(sum(std_normal_logpdf.(Y)) + sum(ladj)) / n (:12), the flow and both sums on the device
# (enf_flow_negll: one deterministic double reduction of (y^2 + log 2pi)/2 - ladj); only the scalar is
# copied back. The flow runs in its promoted element type R, as mvnormal_negll_trafograd's.
function mvnormal_negll_trafo(trafo::_Supported, X::HipMatrix{T}) where {T}
    fs = _leaves(trafo)
    R = _flow_eltype(fs, T)
    Xr = _convert(X, R)
    layers, keep = _layers(fs, Xr.D, R)
    wsb = Ref{Csize_t}(0)
    GC.@preserve wsb begin
        check(ccall((:enf_flow_negll_workspace, libenf), Cint, (Cint, Int64, Int64, Ref{Csize_t}),
                    _dt(R), Xr.D, Xr.N, wsb))
    end
    ws = HipBuffer(max(Int(wsb[]), 1))
    out = HipMatrix(zeros(R, 1, 1))
    GC.@preserve Xr layers keep ws out begin
        check(ccall((:enf_flow_negll, libenf), Cint,
                    (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{EnfLayer}, Int32, Ptr{Cvoid}, Ptr{Cvoid},
                     Csize_t, Ptr{Cvoid}),
                    _dt(R), Xr.D, Xr.N, Xr.buf.ptr, Xr.D, layers, length(layers), out.buf.ptr, ws.ptr, ws.bytes,
                    C_NULL))
    end
    Array(out)[1] / Xr.N
end

_flow_eltype(fs, ::Type{T}) where {T} = foldl((R, f) -> _promoted(R, f), fs; init = float(T))

function _param_count(layers, D)
    np = Ref{Int64}(0)
    GC.@preserve layers begin
        check(ccall((:enf_flow_param_count, libenf), Cint, (Int64, Ptr{EnfLayer}, Int32, Ref{Int64}),
                    D, layers, length(layers), np))
    end
    Int(np[])
end

function _grad_workspace(::Type{R}, D, N, layers) where {R}
    wsb = Ref{Csize_t}(0)
    GC.@preserve layers begin
        check(ccall((:enf_flow_negll_grad_workspace, libenf), Cint,
                    (Cint, Int64, Int64, Ptr{EnfLayer}, Int32, Ref{Csize_t}),
                    _dt(R), D, N, layers, length(layers), wsb))
    end
    HipBuffer(max(Int(wsb[]), 1))
end

# unnormalised sums: out[1] += N * negll, out[2:end] += its gradient (enf_flow_negll_grad)
function _negll_grad_sums!(out::HipMatrix{R}, X::HipMatrix{R}, col0::Integer, ncols::Integer, layers,
                           ws::HipBuffer; zygote::Bool = false) where {R}
    GC.@preserve out X layers ws begin
        check(ccall((:enf_flow_negll_grad, libenf), Cint,
                    (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{EnfLayer}, Int32, Ptr{Cvoid}, Ptr{Cvoid},
                     Csize_t, Ptr{Cvoid}),
                    _dt(R) | (zygote ? ENF_NEGLL_ZYGOTE : Cint(0)), X.D, ncols, X.buf.ptr + col0 * X.D * sizeof(R), X.D, layers, length(layers),
                    out.buf.ptr, ws.ptr, ws.bytes, C_NULL))
    end
    out
end

# The Zygote tangent of the flow (src/optimize_whitening.jl:20): NamedTuples of the fields, nested
# (outer = ..., inner = ...) for a ComposedFunction; a scalar field's gradient is the sum over its
# broadcast rows, a length-1 vector field's the same sum as a length-1 vector.
function _tangent(f::ComposedFunction, g, pos, D)
    ti, pos = _tangent(f.inner, g, pos, D)
    to, pos = _tangent(f.outer, g, pos, D)
    (outer = to, inner = ti), pos
end
function _tangent(f, g, pos, D)
    op, names = _op(f)
    vals = map(names) do nm
        p = getfield(f, nm)
        n = op == OP_HOUSEHOLDER ? length(p) : D
        gs = g[pos+1:pos+n]
        pos += n
        p isa Real ? sum(gs) : (length(p) == n ? reshape(gs, size(p)) : fill(sum(gs), size(p)))
    end
    NamedTuple{names}(Tuple(vals)), pos
end

# negll as the reference returns it (under Zygote, ScaleShiftTrafo's primal ladj zero: + sum log|a|);
# similar_fill_quirk = false returns the true negll. The gradient is the same either way.
function mvnormal_negll_trafograd(trafo::_Supported, X::HipMatrix{T}; similar_fill_quirk::Bool = true) where {T}
    fs = _leaves(trafo)
    R = _flow_eltype(fs, T)
    Xr = _convert(X, R)
    layers, keep = _layers(fs, Xr.D, R)
    np = _param_count(layers, Xr.D)
    ws = _grad_workspace(R, Xr.D, Xr.N, layers)
    out = HipMatrix(zeros(R, 1 + np, 1))
    GC.@preserve keep _negll_grad_sums!(out, Xr, 0, Xr.N, layers, ws; zygote = similar_fill_quirk)
    g = Array(out)[:, 1] ./ Xr.N
    d_trafo, _ = _tangent(trafo, g, 1, Xr.D)
    g[1], d_trafo
end

# --- input / parameter VJP (enf_flow_vjp) ---------------------------------------------------------
# The pullback of (Y, ladj) = with_logabsdet_jacobian(f, X) that Zygote builds from the reference's
# rrules (householder_trafo_pullback_x, chained_householder_trafo_pullback_x, src/householder_trafo.jl:
# 43-54,105-124) and broadcast AD: dX = J' dY + dladj .* grad_x(ladj) per sample, and with
# params = true the parameter cotangent (Zygote-shaped, as mvnormal_negll_trafograd's) summed over the
# samples. dladj = nothing is a zero ladj cotangent. All arguments share one element type.
function flow_vjp(f::_Supported, X::HipMatrix{T}, dY::HipMatrix{T}, dladj::Union{Nothing,HipMatrix{T}} = nothing;
                  params::Bool = false) where {T}
    size(dY) == size(X) || throw(DimensionMismatch("dY must be $(size(X))"))
    dladj === nothing || dladj.D * dladj.N == X.N || throw(DimensionMismatch("dladj must have N entries"))
    fs = _leaves(f)
    _flow_eltype(fs, T) === T || throw(ArgumentError("flow_vjp: parameters would promote the element type"))
    layers, keep = _layers(fs, X.D, T)
    dX = HipMatrix{T}(X.D, X.N)
    np = params ? _param_count(layers, X.D) : 0
    dp = params ? HipMatrix(zeros(T, np, 1)) : nothing
    ws = _grad_workspace(T, X.D, X.N, layers)  # (a flow beyond one gradient launch's bounds: checkpoints)
    GC.@preserve X dY dladj layers keep dX dp ws begin
        check(ccall((:enf_flow_vjp, libenf), Cint,
                    (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{EnfLayer}, Int32,
                     Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
                    _dt(T), X.D, X.N, X.buf.ptr, X.D, dY.buf.ptr, X.D, dladj === nothing ? C_NULL : dladj.buf.ptr,
                    layers, length(layers), dX.buf.ptr, X.D, params ? dp.buf.ptr : C_NULL,
                    ws.ptr, ws.bytes, C_NULL))
    end
    params || return dX, nothing
    g = vcat(zero(T), Array(dp)[:, 1])
    dX, _tangent(f, g, 1, X.D)[1]
end

# --- RCCL communicator (enf_comm_*) for data-parallel optimize_whitening ------------------------
mutable struct EnfComm
    h::Ptr{Cvoid}
    nranks::Int
    rank::Int
    function EnfComm(nranks::Integer, rank::Integer, id::AbstractVector{UInt8})
        length(id) == ENF_UNIQUE_ID_BYTES || throw(ArgumentError("unique id must be $ENF_UNIQUE_ID_BYTES bytes"))
        idv = Vector{UInt8}(id)
        r = Ref{Ptr{Cvoid}}(C_NULL)
        GC.@preserve idv begin
            check(ccall((:enf_comm_init, libenf), Cint, (Ref{Ptr{Cvoid}}, Int32, Ptr{UInt8}, Int32),
                        r, nranks, idv, rank))
        end
        c = new(r[], Int(nranks), Int(rank))
        finalizer(c -> ccall((:enf_comm_destroy, libenf), Cint, (Ptr{Cvoid},), c.h), c)
        c
    end
end

"""A fresh RCCL unique id; rank 0 creates it and ships it to the other ranks out of band (MPI.jl ...)."""
function comm_unique_id()
    id = zeros(UInt8, ENF_UNIQUE_ID_BYTES)
    check(ccall((:enf_comm_unique_id, libenf), Cint, (Ptr{UInt8},), id))
    id
end

function allreduce_sum!(c::EnfComm, X::HipMatrix{T}) where {T}
    GC.@preserve c X begin
        check(ccall((:enf_allreduce_sum, libenf), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}),
                    c.h, X.buf.ptr, X.D * X.N, _dt(T), C_NULL))
    end
    X
end

# --- optimize_whitening (src/optimize_whitening.jl:25-45) over a device-resident sample matrix -------
# One flat device parameter vector theta in the enf_flow_param_count layout, the layer pointers
# pointing into it. Array fields are trainable, as Optimisers treats them (a length-1 vector field is
# ONE trainable broadcast over D rows: its D gradient entries are summed); scalar fields are broadcast
# for the kernels and kept. Minibatches as the reference's: batchsize = round(Int, N/nbatches),
# Iterators.partition over the columns, the last one possibly shorter.
#
# optimizer_state = (theta, acc, rule): the device parameters, the ADAGrad accumulator and the rule.
# optstate continues a previous run as the reference does (state = deepcopy(optstate), trafo =
# deepcopy(initial_trafo), :28-29): the parameters come from initial_trafo, the accumulator is a COPY
# of optstate.acc and the rule is optstate.rule (Optimisers.update uses the rule stored in the state).
#
# comm: an EnfComm for data-parallel training; every rank holds the same smpls and processes its
# contiguous share [B*rank/world, B*(rank+1)/world) of each minibatch; the unnormalised sums are
# all-reduced and every rank applies the same update: enf_whitening_step_dp (gradient, RCCL sum of the
# kernels' double slice totals, one tail launch), or with tied fields the separate sums + enf_whitening_apply.
function _flatten(fs, D, ::Type{T}) where {T}
    host, offs, runs, hb, tied = T[], Int[], Int64[], Int64[], Tuple{Int,Int}[]
    for f in fs
        op, names = _op(f)
        for nm in names
            p = getfield(f, nm)
            v = op == OP_HOUSEHOLDER ? vec(Matrix{T}(reshape(p, D, :))) : _vec(p, D, T)
            o = length(host)
            push!(offs, o)
            append!(host, v)
            if p isa AbstractArray
                append!(runs, (o, o + length(v)))
                op != OP_HOUSEHOLDER && length(p) == 1 && D > 1 && push!(tied, (o, o + length(v)))
            end
            op == OP_HOUSEHOLDER && append!(hb, (o, length(v) ÷ D, D))
        end
    end
    host, offs, runs, hb, tied
end

function optimize_whitening(smpls::HipMatrix{T}, initial_trafo::Function, optimizer::Optimisers.ADAGrad;
                            nbatches::Integer = 100, nepochs::Integer = 100, optstate = nothing,
                            negll_history = Vector{Float64}(), comm::Union{Nothing,EnfComm} = nothing,
                            similar_fill_quirk::Bool = true) where {T}
    fs = _leaves(initial_trafo)
    R = _flow_eltype(fs, T)
    X = _convert(smpls, R)
    D, N = X.D, X.N
    host, offs, runs, hb, tied = _flatten(fs, D, R)
    theta = HipMatrix(reshape(host, :, 1))
    if optstate === nothing  # Optimisers.setup(optimizer, deepcopy(initial_trafo)): acc = epsilon
        rule = optimizer
        acc = HipMatrix(fill(R(optimizer.epsilon), length(host), 1))
    else
        (optstate.acc isa HipMatrix{R} && size(optstate.acc) == (length(host), 1)) ||
            throw(ArgumentError("optstate does not match the flow's parameter layout / element type"))
        rule = optstate.rule
        acc = copy(optstate.acc)
    end
    layers = EnfLayer[]
    i = 0
    for f in fs
        op, names = _op(f)
        ptrs = Ptr{Cvoid}[C_NULL, C_NULL, C_NULL, C_NULL]
        for q in eachindex(names)
            i += 1
            ptrs[q] = theta.buf.ptr + offs[i] * sizeof(R)
        end
        k = op == OP_HOUSEHOLDER ? Int32(length(getfield(f, :V)) ÷ D) :
            (op == OP_SCALESHIFT && f.a isa AbstractVector && length(f.a) == 1) ? Int32(1) : Int32(0)
        push!(layers, EnfLayer(op, k, Tuple(ptrs)))
    end
    world, rank = comm === nothing ? (1, 0) : (comm.nranks, comm.rank)
    # the training calls' dtype: negll_history as the reference records it (ENF_NEGLL_ZYGOTE) unless
    # similar_fill_quirk = false
    dtq = _dt(R) | (similar_fill_quirk ? ENF_NEGLL_ZYGOTE : Cint(0))
    batchsize = max(round(Int, N / nbatches), 1)
    starts = 0:batchsize:N-1
    ws = _grad_workspace(R, D, batchsize, layers)
    hist = HipMatrix{Float64}(1, nepochs * length(starts))
    np = length(host)
    out = HipMatrix{R}(1 + np, 1)
    zero_out = zeros(R, 1 + np, 1)
    # the one-launch update takes at most 64 trainable runs and 16 Householder batches (enf_whitening_step /
    # _step_dp / _apply: ENF_ERR_UNSUPPORTED beyond); past that the update runs as the separate calls
    limits_ok = length(runs) ÷ 2 <= 64 && length(hb) ÷ 3 <= 16
    fused = world == 1 && isempty(tied) && limits_ok
    s = 0
    GC.@preserve X theta acc layers runs hb ws hist out zero_out begin
        if fused  # one rank: each epoch in ONE call (enf_whitening_epoch: one launch for one-block minibatches)
            for _ in 1:nepochs
                loss_ptr = Ptr{Cdouble}(hist.buf.ptr + s * sizeof(Float64))
                check(ccall((:enf_whitening_epoch, libenf), Cint,
                            (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Int64, Ptr{EnfLayer}, Int32, Ptr{Cvoid}, Ptr{Cvoid},
                             Ptr{Int64}, Int32, Ptr{Int64}, Int32, Cdouble, Cdouble, Ptr{Cdouble}, Ptr{Cvoid},
                             Csize_t, Ptr{Cvoid}),
                            dtq, D, N, X.buf.ptr, D, batchsize, layers, length(layers), theta.buf.ptr,
                            acc.buf.ptr, runs, length(runs) ÷ 2, hb, length(hb) ÷ 3, rule.eta, rule.epsilon,
                            loss_ptr, ws.ptr, ws.bytes, C_NULL))
                s += length(starts)
            end
        end
        for _ in 1:(fused ? 0 : nepochs), b0 in starts
            B = min(b0 + batchsize, N) - b0
            lo, hi = b0 + (B * rank) ÷ world, b0 + (B * (rank + 1)) ÷ world
            loss_ptr = Ptr{Cdouble}(hist.buf.ptr + s * sizeof(Float64))
            if fused  # gradient, negll, ADAGrad and re-normalisation: three launches
                check(ccall((:enf_whitening_step, libenf), Cint,
                            (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{EnfLayer}, Int32, Ptr{Cvoid}, Ptr{Cvoid},
                             Ptr{Int64}, Int32, Ptr{Int64}, Int32, Cdouble, Cdouble, Ptr{Cdouble}, Ptr{Cvoid},
                             Csize_t, Ptr{Cvoid}),
                            dtq, D, B, X.buf.ptr + b0 * D * sizeof(R), D, layers, length(layers), theta.buf.ptr,
                            acc.buf.ptr, runs, length(runs) ÷ 2, hb, length(hb) ÷ 3, rule.eta, rule.epsilon,
                            loss_ptr, ws.ptr, ws.bytes, C_NULL))
            elseif isempty(tied) && limits_ok  # data-parallel: gradient, RCCL sum of the rank's totals, update (enf_whitening_step_dp)
                check(ccall((:enf_whitening_step_dp, libenf), Cint,
                            (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{EnfLayer}, Int32, Ptr{Cvoid}, Ptr{Cvoid},
                             Ptr{Int64}, Int32, Ptr{Int64}, Int32, Cdouble, Cdouble, Int64, Ptr{Cdouble}, Ptr{Cvoid},
                             Ptr{Cvoid}, Csize_t, Ptr{Cvoid}),
                            dtq, D, hi - lo, X.buf.ptr + lo * D * sizeof(R), D, layers, length(layers), theta.buf.ptr,
                            acc.buf.ptr, runs, length(runs) ÷ 2, hb, length(hb) ÷ 3, rule.eta, rule.epsilon, B,
                            loss_ptr, comm === nothing ? C_NULL : comm.h, ws.ptr, ws.bytes, C_NULL))
            else      # local sums, cross-rank sum, tied-field sums, then the update on every rank
                _memcpy(out.buf.ptr, Ptr{Cvoid}(pointer(zero_out)), sizeof(zero_out), MEMCPY_H2D)
                hi > lo && _negll_grad_sums!(out, X, lo, hi - lo, layers, ws; zygote = similar_fill_quirk)
                comm === nothing || allreduce_sum!(comm, out)
                if !isempty(tied)  # the (1 + P) sums are small: fix them up on the host
                    g = Array(out)
                    for (a, b) in tied
                        g[2+a:1+b] .= sum(g[2+a:1+b])
                    end
                    GC.@preserve g _memcpy(out.buf.ptr, Ptr{Cvoid}(pointer(g)), sizeof(g), MEMCPY_H2D)
                end
                if limits_ok
                    check(ccall((:enf_whitening_apply, libenf), Cint,
                                (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Int64}, Int32,
                                 Ptr{Int64}, Int32, Cdouble, Cdouble, Ptr{Cdouble}, Ptr{Cvoid}),
                                _dt(R), D, np, out.buf.ptr, B, theta.buf.ptr, acc.buf.ptr, runs, length(runs) ÷ 2,
                                hb, length(hb) ÷ 3, rule.eta, rule.epsilon, loss_ptr, C_NULL))
                else  # the separate calls: loss, ADAGrad per run, re-normalisation per batch (same arithmetic)
                    g = Array(out)
                    lossv = Float64[Float64(g[1] / R(B))]
                    GC.@preserve lossv _memcpy(Ptr{Cvoid}(loss_ptr), Ptr{Cvoid}(pointer(lossv)), sizeof(lossv), MEMCPY_H2D)
                    for q in 1:2:length(runs)
                        a0, a1 = runs[q], runs[q+1]
                        check(ccall((:enf_adagrad_step, libenf), Cint,
                                    (Cint, Int64, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cdouble, Cdouble, Cdouble, Ptr{Cvoid}),
                                    _dt(R), a1 - a0, theta.buf.ptr + a0 * sizeof(R), acc.buf.ptr + a0 * sizeof(R),
                                    out.buf.ptr + (1 + a0) * sizeof(R), 1.0 / B, rule.eta, rule.epsilon, C_NULL))
                    end
                    for q in 1:3:length(hb)
                        check(ccall((:enf_householder_normalize_strided, libenf), Cint,
                                    (Cint, Int64, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}),
                                    _dt(R), D, hb[q+1], theta.buf.ptr + hb[q] * sizeof(R), hb[q+2], C_NULL))
                    end
                end
            end
            s += 1
        end
    end
    # Functors-style reconstruction of the trained flow from theta (scalar fields kept)
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
    (result = trafo, optimizer_state = (theta = theta, acc = acc, rule = rule),
     negll_history = vcat(negll_history, vec(Array(hist))))
end

# --- JohnsonSU (src/johnson_trafo.jl:120-129) over a HipMatrix of values ---------------------------
# pdf.(d, X) etc. as methods of the Distributions / Statistics generics on the shim's HipMatrix; the
# result element type is float(promote_type(eltype(X), params)), as the reference's johnsontrafo.
function _jsu(fn::Int32, d::JohnsonSU, X::HipMatrix{T}) where {T}
    R = float(promote_type(T, typeof(d.gamma), typeof(d.delta), typeof(d.xi), typeof(d.lambda)))
    Xr = _convert(X, R)
    out = HipMatrix{R}(Xr.D, Xr.N)
    GC.@preserve Xr out begin
        check(ccall((:enf_johnsonsu_eval, libenf), Cint,
                    (Cint, Int32, Int64, Ptr{Cvoid}, Ptr{Cvoid}, Cdouble, Cdouble, Cdouble, Cdouble, Ptr{Cvoid}),
                    _dt(R), fn, Xr.D * Xr.N, Xr.buf.ptr, out.buf.ptr, d.gamma, d.delta, d.xi, d.lambda, C_NULL))
    end
    out
end

Distributions.pdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_PDF, d, X)
Distributions.logpdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_LOGPDF, d, X)
Distributions.cdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_CDF, d, X)
Distributions.logcdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_LOGCDF, d, X)
Distributions.ccdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_CCDF, d, X)
Distributions.logccdf(d::JohnsonSU, X::HipMatrix) = _jsu(ENF_JSU_LOGCCDF, d, X)
Statistics.quantile(d::JohnsonSU, P::HipMatrix) = _jsu(ENF_JSU_QUANTILE, d, P)

"""rand(d, HipMatrix{T}, n): n JohnsonSU samples as a 1 x n HipMatrix, quantile of a Philox4x32-10
stream (key = seed, counter = offset + ...): Distributions' inverse-CDF sampling on the device."""
function Random.rand(d::JohnsonSU, ::Type{HipMatrix{T}}, n::Integer; seed::UInt64 = UInt64(0),
                     offset::UInt64 = UInt64(0)) where {T<:Union{Float32,Float64}}
    out = HipMatrix{T}(1, n)
    GC.@preserve out begin
        check(ccall((:enf_johnsonsu_sample, libenf), Cint,
                    (Cint, Int64, Ptr{Cvoid}, Cdouble, Cdouble, Cdouble, Cdouble, UInt64, UInt64, Ptr{Cvoid}),
                    _dt(T), n, out.buf.ptr, d.gamma, d.delta, d.xi, d.lambda, seed, offset, C_NULL))
    end
    out
end

export HipMatrix, EnfComm, comm_unique_id, allreduce_sum!, stream_with_logabsdet_jacobian, flow_vjp

end # module
