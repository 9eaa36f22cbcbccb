# DLRMHip.jl — the Julia side of the drop-in boundary (ccall shim over include/dlrm_hip.h).
#
# NOT EXECUTED IN THIS REPOSITORY: the image has no Julia toolchain, and the package this shim
# extends (EmbeddingTables 0.1.0, `path = "../EmbeddingTables"`, Manifest.toml:246-250) is
# un-vendored.  The method signatures below are those of the reference's call sites:
#
#   maplookup(strategy, tables, sparse)                        src/model/model.jl:161
#   (dot::DotInteraction)(x, ys) + rrule(dot, X, Y)            src/model/interact.jl:394-447
#   EmbeddingTables.update!(opt, tables, grads, indexers; ...) src/train/train.jl:283-290
#
# A model switches by constructor keywords only (src/model/model.jl:173-192,
# src/data/criteo.jl:408-433):
#
#   ctx   = DLRMHip.Context(0)
#   model = kaggle_dlrm(; embedding_constructor = x -> DLRMHip.HipEmbedding(ctx, x),
#                         interaction = DLRMHip.HipDotInteraction(ctx))
#
# and `_Train.train!` / `DLRMModel` stay unchanged.  Dense inputs x (bottom-MLP output) and the
# interaction output cross PCIe here because the MLPs stay on the CPU in the reference; the
# embedding tables, the gathered rows and every kernel's scratch stay in HBM.
module DLRMHip

using ChainRulesCore
import EmbeddingTables
import EmbeddingTables: maplookup, DefaultStrategy, PreallocationStrategy, SparseEmbeddingUpdate, Static
import OneDNN   # the bottom MLP's output / the top MLP's cotangent arrive as OneDNN.Memory

const libdlrm = joinpath(@__DIR__, "..", "lib", "libdlrm_hip.so")

const DLRM_F32, DLRM_BF16 = Cint(0), Cint(1)
const DLRM_I32, DLRM_I64 = Cint(0), Cint(1)
const DLRM_E_INDEX = Cint(-3)

struct DLRMError <: Exception
    code::Cint
    msg::String
end

#####
##### Context: one device + one stream (dlrm_ctx_create, include/dlrm_hip.h)
#####

mutable struct Context
    ptr::Ptr{Cvoid}
    # fused = true: maplookup on this context's HipEmbeddings returns a HipLookup and the operator
    # chain runs on the training-step kernels (see "The unchanged operator chain" below); lr: the
    # Descent η of the update! that follows (lets the pullback step the once-hit rows itself)
    fused::Bool
    lr::Union{Nothing,Float32}
    # defer_update (fused, lr known): update! leaves its apply launch to the next maplookup, which runs
    # it with that batch's indexer build -- no host synchronisation per step (bounds: see poll_bounds!)
    defer::Bool
    function Context(device::Integer; stream::Ptr{Cvoid} = C_NULL, fused::Bool = false, lr = nothing,
                     defer_update::Bool = true)
        out = Ref{Ptr{Cvoid}}(C_NULL)
        rc = ccall((:dlrm_ctx_create, libdlrm), Cint, (Cint, Ptr{Cvoid}, Ref{Ptr{Cvoid}}), device, stream, out)
        rc == 0 || throw(DLRMError(rc, "dlrm_ctx_create"))
        ctx = new(out[], fused, lr === nothing ? nothing : Float32(lr), defer_update)
        finalizer(c -> ccall((:dlrm_ctx_destroy, libdlrm), Cint, (Ptr{Cvoid},), c.ptr), ctx)
        return ctx
    end
end

function check(ctx::Context, rc::Cint)
    rc == 0 && return nothing
    msg = unsafe_string(ccall((:dlrm_last_error, libdlrm), Cstring, (Ptr{Cvoid},), ctx.ptr))
    # out-of-range indices: the reference's gather throws BoundsError
    rc == DLRM_E_INDEX && throw(BoundsError(msg))
    throw(DLRMError(rc, msg))
end

synchronize(ctx::Context) = check(ctx, ccall((:dlrm_sync, libdlrm), Cint, (Ptr{Cvoid},), ctx.ptr))
check_bounds(ctx::Context) = check(ctx, ccall((:dlrm_check_bounds, libdlrm), Cint, (Ptr{Cvoid},), ctx.ptr))
# the last copy of the device bounds flag that has reached host memory (no GPU call; the step
# backward stores it, dlrm_error_snapshot queues one)
function error_peek(ctx::Context)
    w = Ref{Cuint}(0)
    check(ctx, ccall((:dlrm_error_peek, libdlrm), Cint, (Ptr{Cvoid}, Ref{Cuint}), ctx.ptr, w))
    return w[]
end
error_snapshot(ctx::Context) = check(ctx, ccall((:dlrm_error_snapshot, libdlrm), Cint, (Ptr{Cvoid},), ctx.ptr))

#####
##### Device buffers owned from Julia (dlrm_malloc / dlrm_free / dlrm_memcpy_*)
#####

mutable struct DeviceMatrix{T} <: AbstractMatrix{T}
    ctx::Context
    ptr::Ptr{Cvoid}
    dims::Tuple{Int,Int}          # Julia (rows, cols) = C [cols][rows]
    function DeviceMatrix{T}(ctx::Context, rows::Integer, cols::Integer) where {T}
        p = Ref{Ptr{Cvoid}}(C_NULL)
        check(ctx, ccall((:dlrm_malloc, libdlrm), Cint, (Ptr{Cvoid}, Csize_t, Ref{Ptr{Cvoid}}),
                         ctx.ptr, max(1, rows * cols) * sizeof(T), p))
        m = new{T}(ctx, p[], (Int(rows), Int(cols)))
        finalizer(x -> ccall((:dlrm_free, libdlrm), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), x.ctx.ptr, x.ptr), m)
        return m
    end
end
Base.size(m::DeviceMatrix) = m.dims
Base.getindex(::DeviceMatrix, ::Int...) = error("DeviceMatrix lives in HBM; copy it with Array(m)")
function upload!(m::DeviceMatrix{T}, src::AbstractMatrix{T}) where {T}
    @assert size(src) == size(m)
    src = Matrix(src)
    check(m.ctx, ccall((:dlrm_memcpy_h2d, libdlrm), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{T}, Csize_t),
                       m.ctx.ptr, m.ptr, src, sizeof(src)))
    return m
end
function Base.Array(m::DeviceMatrix{T}) where {T}
    # a host read of any buffer of the context (e.g. Array(tables[t].data)) sees every update! made
    # so far: deferred apply launches of its table sets run first (update! writes the tables in
    # place before it returns in the reference, train.jl:283-290)
    flush_ctx!(m.ctx)
    dst = Matrix{T}(undef, size(m))
    check(m.ctx, ccall((:dlrm_memcpy_d2h, libdlrm), Cint, (Ptr{Cvoid}, Ptr{T}, Ptr{Cvoid}, Csize_t),
                       m.ctx.ptr, dst, m.ptr, sizeof(dst)))
    return dst
end

dtype_code(::Type{Float32}) = DLRM_F32
dtype_code(::Type{T}) where {T} = sizeof(T) == 2 ? DLRM_BF16 : throw(ArgumentError("dtype $T"))

#####
##### HipEmbedding{Static{D}}: the SimpleEmbedding{Static{D}} replacement
#####

"""
    HipEmbedding(ctx, data::AbstractMatrix)

`D × N` embedding table resident in HBM (C `[N][D]`, rows contiguous), the drop-in for
`SimpleEmbedding{Static{D}}(data)` (src/data/criteo.jl:490, src/model/model.jl:185).
"""
struct HipEmbedding{S,T} <: EmbeddingTables.AbstractEmbeddingTable{S,T}
    data::DeviceMatrix{T}
end
function HipEmbedding(ctx::Context, data::AbstractMatrix{T}) where {T}
    D, N = size(data)
    return HipEmbedding{Static{D},T}(upload!(DeviceMatrix{T}(ctx, D, N), data))
end
featuresize(::HipEmbedding{Static{D}}) where {D} = D
Base.size(e::HipEmbedding) = size(e.data)

# dlrm_tables handle of one Vector{HipEmbedding} (registered once, reused every step)
const TABLESETS = IdDict{Any,Ptr{Cvoid}}()
function tableset(tables::AbstractVector{<:HipEmbedding{Static{D},T}}) where {D,T}
    get!(TABLESETS, tables) do
        ctx = first(tables).data.ctx
        ptrs = [t.data.ptr for t in tables]
        rows = Int64[size(t, 2) for t in tables]
        out = Ref{Ptr{Cvoid}}(C_NULL)
        check(ctx, ccall((:dlrm_tables_create, libdlrm), Cint,
                         (Ptr{Cvoid}, Cint, Cint, Cint, Ptr{Ptr{Cvoid}}, Ptr{Int64}, Ref{Ptr{Cvoid}}),
                         ctx.ptr, length(tables), D, dtype_code(T), ptrs, rows, out))
        out[]
    end
end

#####
##### Sparse inputs: packed [T][B*L] device indices, 1-based (index_base = 1)
#####

struct PackedIndices
    data::DeviceMatrix{Int32}    # (B*L) × T  ==  C [T][B*L]
    batch::Int
    lookups::Int
end
"""
    pack(ctx, sparse)

`sparse` as DLRM.jl hands it over: a `Matrix{UInt32}(B, T)` from `DACLoader`
(src/data/criteo.jl:324), a `Vector{Vector{Int}}` (one-hot) or a `Vector{Matrix}` of `L × B`
sample-major index matrices (src/data/criteo.jl:551-557).  All become one device buffer.
"""
function pack(ctx::Context, sparse::AbstractMatrix{<:Integer})
    B, T = size(sparse)
    return PackedIndices(upload!(DeviceMatrix{Int32}(ctx, B, T), Int32.(sparse)), B, 1)
end
function pack(ctx::Context, sparse::AbstractVector)
    L = first(sparse) isa AbstractMatrix ? size(first(sparse), 1) : 1
    B = length(first(sparse)) ÷ L
    host = reduce(hcat, [Int32.(vec(s)) for s in sparse])          # (B*L) × T
    return PackedIndices(upload!(DeviceMatrix{Int32}(ctx, B * L, length(sparse)), host), B, L)
end

#####
##### maplookup (src/model/model.jl:161) + its pullback
#####

# Rows reserved for x at the top of every output column: PreallocationStrategy(P) (DLRM.jl
# builds it as PreallocationStrategy{Float32}(feature_size), src/DLRM.jl:95; the package is
# un-vendored, so its one integer field is read without naming it).
prealloc_rows(s::PreallocationStrategy) =
    something((getfield(s, f) for f in fieldnames(typeof(s)) if getfield(s, f) isa Integer)..., 0)

function _maplookup(tables::AbstractVector{<:HipEmbedding{Static{D},T}}, sparse, P::Integer) where {D,T}
    ctx = first(tables).data.ctx
    idx = sparse isa PackedIndices ? sparse : pack(ctx, sparse)
    # every entry point that reads the tables applies a deferred update! first (the DefaultStrategy
    # method, HipLookup's DeviceMatrix, the unfused rrule), as _fused_maplookup does
    poll_bounds!(tables)
    flush!(tables)
    ys = DeviceMatrix{T}(ctx, P + D * length(tables), idx.batch)
    check(ctx, ccall((:dlrm_maplookup, libdlrm), Cint,
                     (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Cint, Ptr{Cvoid}, Int64, Int64),
                     ctx.ptr, tableset(tables), idx.data.ptr, DLRM_I32, idx.batch * idx.lookups, 1,
                     idx.batch, idx.lookups, ys.ptr, size(ys, 1), P))
    return ys, idx
end

EmbeddingTables.maplookup(s::PreallocationStrategy, tables::AbstractVector{<:HipEmbedding}, sparse) =
    first(tables).data.ctx.fused ? _fused_maplookup(tables, sparse, prealloc_rows(s)) :
                                   first(_maplookup(tables, sparse, prealloc_rows(s)))

# DefaultStrategy: one D x B matrix per table (test/model/embedding_update.jl:31, model.jl:155)
function EmbeddingTables.maplookup(::DefaultStrategy, tables::AbstractVector{<:HipEmbedding{Static{D}}}, sparse) where {D}
    ys = Array(first(_maplookup(tables, sparse, 0)))
    return [ys[(D * (t - 1) + 1):(D * t), :] for t in eachindex(tables)]
end

# The maplookup pullback hands update! one SparseEmbeddingUpdate per table (DLRMGrads.embeddings
# is a Vector{SparseEmbeddingUpdate}, src/train/train.jl:141-145, filled by append!, :183).  Its
# delta is a (D x B) row block of the dt the interaction backward left in HBM and its indices
# are the table's row of the packed device indices -- views, no copies -- built with the same
# constructor DLRM.jl uses (SparseEmbeddingUpdate{Static{D}}(delta, indices), src/playground.jl:44).
struct HipDelta <: AbstractMatrix{Float32}
    dt::DeviceMatrix{Float32}
    offset::Int      # first row of this table's block in every dt column (0-based)
    D::Int
end
Base.size(d::HipDelta) = (d.D, size(d.dt, 2))
Base.getindex(::HipDelta, ::Int...) = error("HipDelta lives in HBM; EmbeddingTables.uncompress copies it")

struct HipIndices <: AbstractMatrix{Int32}
    idx::PackedIndices
    table::Int       # 1-based
end
Base.size(i::HipIndices) = (i.idx.lookups, i.idx.batch)      # L x B, sample-major (criteo.jl:551-557)
Base.getindex(::HipIndices, ::Int...) = error("HipIndices live in HBM")

const HipUpdate{D} = SparseEmbeddingUpdate{Static{D},HipDelta,HipIndices}
hip_delta(u::SparseEmbeddingUpdate) = u.delta::HipDelta        # EmbeddingTables' field names
hip_indices(u::SparseEmbeddingUpdate) = u.indices::HipIndices

function _rrule_maplookup(strategy::PreallocationStrategy, tables::AbstractVector{<:HipEmbedding{Static{D}}},
                          sparse) where {D}
    P = prealloc_rows(strategy)
    ys, idx = _maplookup(tables, sparse, P)
    function maplookup_pullback(dt)
        dt isa DeviceMatrix{Float32} || throw(ArgumentError("the cotangent of ys is the dt of HipDotInteraction's pullback"))
        ups = [SparseEmbeddingUpdate{Static{D}}(HipDelta(dt, P + (t - 1) * D, D), HipIndices(idx, t))
               for t in eachindex(tables)]
        return (NoTangent(), NoTangent(), ups, NoTangent())
    end
    return ys, maplookup_pullback
end

# uncompress(update, nrows) (test/train/backprop.jl:156): the dense D x N gradient, as
# update!(Descent(-1)) of one zero table with the same deterministic kernel.
function EmbeddingTables.uncompress(u::SparseEmbeddingUpdate{Static{D},HipDelta,HipIndices}, nrows::Integer) where {D}
    δ, ix = hip_delta(u), hip_indices(u)
    ctx = δ.dt.ctx
    table = HipEmbedding(ctx, zeros(Float32, D, nrows))
    L, B = ix.idx.lookups, ix.idx.batch
    indexer = HipIndexer(ctx, 1, B * L)
    row0 = Ptr{Int32}(ix.idx.data.ptr) + sizeof(Int32) * B * L * (ix.table - 1)   # this table's index row
    check(ctx, ccall((:dlrm_sgd_update, libdlrm), Cint,
                     (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cuint, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Cint,
                      Ptr{Cvoid}, Cint, Int64, Int64, Cfloat),
                     ctx.ptr, tableset([table]), indexer.ptr, Cuint(0), row0, DLRM_I32, B * L, 1, B, L,
                     δ.dt.ptr, DLRM_F32, size(δ.dt, 1), δ.offset, -1.0f0))
    check_bounds(ctx)
    return Array(table.data)
end

#####
##### HipDotInteraction: (dot)(x, ys) and its rrule (src/model/interact.jl:394-447)
#####

struct HipDotInteraction
    ctx::Context
    pad_to::Int      # POST_INTERACTION_PAD_TO_MUL (src/model/model.jl:32)
end
HipDotInteraction(ctx::Context) = HipDotInteraction(ctx, 1)

function interaction_sizes(d, F, pad_to)
    width = d + F * (F - 1) ÷ 2
    padded = cld(width, pad_to) * pad_to
    return padded, padded - width
end

function _interact(dot::HipDotInteraction, x::AbstractMatrix{T}, ys::DeviceMatrix{T}) where {T}
    d, B = size(x)
    F = size(ys, 1) ÷ d
    xd = x isa DeviceMatrix ? x : upload!(DeviceMatrix{T}(dot.ctx, d, B), Matrix{T}(x))   # bottom MLP output
    width, padding = interaction_sizes(d, F, dot.pad_to)
    out = DeviceMatrix{T}(dot.ctx, width, B)
    check(dot.ctx, ccall((:dlrm_interact_fwd, libdlrm), Cint,
                         (Ptr{Cvoid}, Cint, Cint, Cint, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cint),
                         dot.ctx.ptr, dtype_code(T), d, F, B, xd.ptr, d, ys.ptr, size(ys, 1), out.ptr, width, padding))
    return Array(out), padding                                     # the top MLP runs on the CPU
end

# (dot::DotInteraction)(x, ys; return_t) (src/model/interact.jl:394-411): `out`, or with
# return_t = true `(out, T, padding)` -- T is ys itself (x copied into its top rows).
function (dot::HipDotInteraction)(x::AbstractMatrix{T}, ys::DeviceMatrix{T}; return_t = false) where {T}
    out, padding = _interact(dot, x, ys)
    return return_t ? (out, ys, padding) : out
end
# the bottom MLP's output is a OneDNN.Memory (interact.jl:390-392)
(dot::HipDotInteraction)(x::OneDNN.Memory, ys::DeviceMatrix; kw...) = dot(OneDNN.materialize(x), ys; kw...)

function ChainRulesCore.rrule(dot::HipDotInteraction, X, ys::DeviceMatrix{T}) where {T}
    x = X isa OneDNN.Memory ? OneDNN.materialize(X) : X
    out, padding = _interact(dot, x, ys)
    d, B = size(x)
    F = size(ys, 1) ÷ d
    function dot_pullback(Δ)
        Δh = Δ isa OneDNN.Memory ? OneDNN.materialize(Δ) : Δ
        Δd = upload!(DeviceMatrix{T}(dot.ctx, size(Δh)...), Matrix{T}(Δh))
        dx = DeviceMatrix{Float32}(dot.ctx, d, B)
        dt = DeviceMatrix{Float32}(dot.ctx, F * d, B)               # x rows included, as dot_back
        check(dot.ctx, ccall((:dlrm_interact_bwd, libdlrm), Cint,
                             (Ptr{Cvoid}, Cint, Cint, Cint, Cint, Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64,
                              Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64),
                             dot.ctx.ptr, dtype_code(T), d, F, B, Δd.ptr, size(Δh, 1), padding, ys.ptr, size(ys, 1),
                             dx.ptr, d, dt.ptr, F * d))
        return (NoTangent(), Array(dx), dt)
    end
    return out, dot_pullback
end

#####
##### update!(Descent(lr), tables, grads, indexers) (src/train/train.jl:283-290)
#####

"""
    HipIndexer(ctx, num_tables, max_lookups)

Device-side `Vector{SparseIndexer}` (src/train/train.jl:276-281): per-table grouping of the
lookup positions by row, rebuilt every step inside `update!`.
"""
mutable struct HipIndexer
    ctx::Context
    ptr::Ptr{Cvoid}
    function HipIndexer(ctx::Context, num_tables::Integer, max_lookups::Integer)
        out = Ref{Ptr{Cvoid}}(C_NULL)
        check(ctx, ccall((:dlrm_indexer_create, libdlrm), Cint, (Ptr{Cvoid}, Cint, Int64, Ref{Ptr{Cvoid}}),
                         ctx.ptr, num_tables, max_lookups, out))
        ix = new(ctx, out[])
        finalizer(x -> ccall((:dlrm_indexer_destroy, libdlrm), Cint, (Ptr{Cvoid},), x.ptr), ix)
        return ix
    end
end

"Re-carves the indexer for wave builds of `batch` positions per table now (before capturing a graph)."
reserve!(ix::HipIndexer, batch::Integer) =
    check(ix.ctx, ccall((:dlrm_indexer_reserve, libdlrm), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Cint), ix.ctx.ptr, ix.ptr, batch))
"The wave build's chunk limit for the indexer's later builds (16 or 32; deterministic either way)."
set_chunk!(ix::HipIndexer, max_positions::Integer) =
    check(ix.ctx, ccall((:dlrm_indexer_set_chunk, libdlrm), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Cint), ix.ctx.ptr, ix.ptr,
                        max_positions))
"Parts per table of the indexer's later wave builds of <= 2048 positions (0 = 16, 32 or 64; same segments)."
set_parts!(ix::HipIndexer, parts::Integer) =
    check(ix.ctx, ccall((:dlrm_indexer_set_parts, libdlrm), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Cint), ix.ctx.ptr, ix.ptr,
                        parts))
"Device bytes the indexer holds."
function nbytes(ix::HipIndexer)
    b = Ref{Int64}(0)
    rc = ccall((:dlrm_indexer_bytes, libdlrm), Cint, (Ptr{Cvoid}, Ref{Int64}), ix.ptr, b)
    rc == 0 || throw(DLRMError(rc, "dlrm_indexer_bytes"))
    return Int(b[])
end

const INDEXERS = IdDict{Any,HipIndexer}()

# `num_splits` / `nthreads` tune the CPU scatter; the GPU kernel has its own decomposition.
# Dispatch is on the table type: `custom_update!` (src/train/train.jl:283-290) passes the
# Vector{SparseEmbeddingUpdate} that DLRMGrads gathered.
function EmbeddingTables.update!(
    opt, tables::AbstractVector{<:HipEmbedding{Static{D}}}, grads::AbstractVector{<:SparseEmbeddingUpdate},
    indexers; num_splits = 8, nthreads = Threads.nthreads()
) where {D}
    length(grads) == length(tables) || throw(ArgumentError("one SparseEmbeddingUpdate per table"))
    δ1, ix1 = hip_delta(first(grads)), hip_indices(first(grads))
    # one dt buffer and one packed index set serve every table: table t's block sits D rows after t-1's
    for (t, g) in enumerate(grads)
        δ, ix = hip_delta(g), hip_indices(g)
        (δ.dt === δ1.dt && δ.offset == δ1.offset + (t - 1) * D && ix.idx === ix1.idx && ix.table == t) ||
            throw(ArgumentError("update! expects the per-table views of one maplookup pullback"))
    end
    ctx, idx = δ1.dt.ctx, ix1.idx
    if ctx.fused && haskey(CHAIN_STEPS, tables) && haskey(CHAIN_STEPS[tables], idx.batch)
        st = CHAIN_STEPS[tables][idx.batch]
        st.dt === δ1.dt && return _fused_update!(opt, st, tables)
    end
    ix = get!(() -> HipIndexer(ctx, length(tables), idx.batch * idx.lookups), INDEXERS, indexers)
    check(ctx, ccall((:dlrm_sgd_update, libdlrm), Cint,
                     (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cuint, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Cint,
                      Ptr{Cvoid}, Cint, Int64, Int64, Cfloat),
                     ctx.ptr, tableset(tables), ix.ptr, Cuint(0), idx.data.ptr, DLRM_I32, idx.batch * idx.lookups, 1,
                     idx.batch, idx.lookups, δ1.dt.ptr, DLRM_F32, size(δ1.dt, 1), δ1.offset, opt.eta))
    check_bounds(ctx)     # BoundsError, as the reference's gather throws (no row was written)
    return nothing
end

#####
##### Optional fast path: the sparse half of one train! iteration as the training-step pair
##### (dlrm_step_fwd / dlrm_step_bwd): identical results to maplookup -> interaction ->
##### dot_back -> update!, three launches instead of five.
#####

"""
    HipTrainStep(ctx, tables, batch; lr)

Buffers of one training step (out, dx, dt) and the step's indexer.  `train_step_fwd!` returns
the interaction output for the top MLP; `train_step_bwd!` takes dLoss/d(out) and returns dx,
updating the tables in place (rows hit once by the backward, the rest by the apply).
"""
mutable struct HipTrainStep{T}
    ctx::Context
    tables::Vector{HipEmbedding}
    ix::HipIndexer
    out::DeviceMatrix{T}
    dx::DeviceMatrix{Float32}
    dt::DeviceMatrix{Float32}
    idx::Union{Nothing,PackedIndices}
    x::Union{Nothing,DeviceMatrix{T}}
    padding::Int
    lr::Float32
    spare::Union{Nothing,HipIndexer}     # pipelined steps: the indexer the next batch is built into
    pending::Any                         # (next sparse => its packed indices) after train_step_bwd!(; next)
    bwd::Symbol                          # operator chain: :none, :once_hit_applied, :all_dt, :done
    delta::Union{Nothing,DeviceMatrix{T}}  # operator chain: the uploaded Δ of the pullback
end
function HipTrainStep(ctx::Context, tables::AbstractVector{<:HipEmbedding{Static{D},T}}, batch::Integer;
                      lr = 0.01, pad_to = 1) where {D,T}
    F = length(tables) + 1
    width, padding = interaction_sizes(D, F, pad_to)
    return HipTrainStep{T}(ctx, collect(tables), HipIndexer(ctx, length(tables), batch),
                           DeviceMatrix{T}(ctx, width, batch), DeviceMatrix{Float32}(ctx, D, batch),
                           DeviceMatrix{Float32}(ctx, F * D, batch), nothing, nothing, padding, Float32(lr),
                           nothing, nothing, :none, nothing)
end

function train_step_fwd!(st::HipTrainStep{T}, x::AbstractMatrix{T}, sparse) where {T}
    d, B = size(x)
    if st.pending !== nothing && first(st.pending) === sparse
        st.idx = last(st.pending)        # indexer already built by the previous step's apply
    else
        st.idx = sparse isa PackedIndices ? sparse : pack(st.ctx, sparse)
    end
    st.pending = nothing
    st.x = x isa DeviceMatrix ? x : upload!(DeviceMatrix{T}(st.ctx, d, B), x)
    check(st.ctx, ccall((:dlrm_step_fwd, libdlrm), Cint,
                        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Ptr{Cvoid}, Int64,
                         Ptr{Cvoid}, Int64, Cint),
                        st.ctx.ptr, tableset(st.tables), st.ix.ptr, st.idx.data.ptr, DLRM_I32, st.idx.batch, 1, B,
                        st.x.ptr, d, st.out.ptr, size(st.out, 1), st.padding))
    return x isa DeviceMatrix ? st.out : Array(st.out)   # device-resident when the caller's x is
end

"""
    train_step_bwd!(st, Δ; next = nothing)

With `next` (the next batch's sparse features) the step's apply launch also builds the next
batch's indexer (dlrm_step_bwd_prepare), so `train_step_fwd!(st, x_next, next)` only gathers.
Results are identical either way.  A `DeviceMatrix` Δ is read in place and `dx` comes back as
the step's `DeviceMatrix` (no PCIe copy either way); a host Δ is uploaded and `dx` downloaded.
"""
function train_step_bwd!(st::HipTrainStep{T}, Δ::AbstractMatrix{T}; next = nothing) where {T}
    d, B = size(st.x)
    Δd = Δ isa DeviceMatrix ? Δ : upload!(DeviceMatrix{T}(st.ctx, size(Δ)...), Matrix{T}(Δ))
    if next !== nothing
        nidx = next isa PackedIndices ? next : pack(st.ctx, next)
        nidx.batch == st.idx.batch || throw(DimensionMismatch("the next batch must have the same size"))
        nix = st.spare === nothing ? HipIndexer(st.ctx, length(st.tables), B) : st.spare
        check(st.ctx, ccall((:dlrm_step_bwd_prepare, libdlrm), Cint,
                            (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Ptr{Cvoid},
                             Int64, Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cfloat,
                             Ptr{Cvoid}, Ptr{Cvoid}, Cuint),
                            st.ctx.ptr, tableset(st.tables), st.ix.ptr, st.idx.data.ptr, DLRM_I32, st.idx.batch, 1,
                            B, st.x.ptr, d, Δd.ptr, size(Δ, 1), st.padding, st.dx.ptr, d, st.dt.ptr,
                            size(st.dt, 1), st.lr, nix.ptr, nidx.data.ptr, Cuint(0)))
        st.spare, st.ix = st.ix, nix
        st.pending = next => nidx
        return Δ isa DeviceMatrix ? st.dx : Array(st.dx)
    end
    check(st.ctx, ccall((:dlrm_step_bwd, libdlrm), Cint,
                        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Ptr{Cvoid}, Int64,
                         Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cfloat, Cuint),
                        st.ctx.ptr, tableset(st.tables), st.ix.ptr, st.idx.data.ptr, DLRM_I32, st.idx.batch, 1, B,
                        st.x.ptr, d, Δd.ptr, size(Δ, 1), st.padding, st.dx.ptr, d, st.dt.ptr, size(st.dt, 1),
                        st.lr, Cuint(0)))
    return Δ isa DeviceMatrix ? st.dx : Array(st.dx)
end

#####
##### The unchanged operator chain on the step kernels (Python mirror: dlrm.jl_amd/lazy.py)
#####
# With `Context(dev; fused = true, lr = η)` the four calls an unchanged train! makes
#   ys = maplookup(PreallocationStrategy(d), tables, sparse)      model.jl:161
#   out = interaction(x, ys)  (+ its rrule pullback)                model.jl:163, interact.jl:438-447
#   update!(Descent(η), tables, grads, indexers)                    train.jl:283-290
# run the training-step pair: maplookup returns a HipLookup (nothing launched, ys never written),
# the interaction on it is dlrm_step_fwd (gather + interaction + the update's indexer, one launch),
# its pullback dlrm_step_bwd(DLRM_STEP_BWD_ONLY) (once-hit rows stepped with η there; without lr,
# dlrm_interact_bwd_gather writes every dt row), and update! the apply launch.  Results are those of
# the five-launch chain above, bit for bit (tests/test_gpu_parity.py, through the same ABI).
# With lr known and `defer_update` (the Context default), update! returns at once and the next
# maplookup runs its apply launch together with that batch's indexer build (flush!), so the next
# forward only gathers and no call synchronises: out-of-range indices surface as BoundsError at a
# later maplookup (poll_bounds!, from the flag the step backward copies to host memory) or at
# check_bounds(tables), with no row of the failing step written (Python mirror: HipTables).

const STEP_BWD_ONLY, STEP_APPLY_ONLY, UPDATE_PREBUILT = Cuint(1), Cuint(2), Cuint(2)

"""
    HipLookup

`maplookup(PreallocationStrategy(P), tables, sparse)` on a fused context: the (P + D·T) × B lookup
output, not materialized.  `DeviceMatrix(ys)` gathers it (dlrm_maplookup) for any other consumer.
"""
struct HipLookup{T} <: AbstractMatrix{T}
    tables::AbstractVector          # the model's own Vector{HipEmbedding} (keys the step state)
    idx::PackedIndices
    P::Int
end
Base.size(ys::HipLookup) = (ys.P + featuresize(first(ys.tables)) * length(ys.tables), ys.idx.batch)
Base.getindex(::HipLookup, ::Int...) = error("HipLookup is not materialized; DeviceMatrix(ys) gathers it")
DeviceMatrix(ys::HipLookup) = first(_maplookup(ys.tables, ys.idx, ys.P))

# one preallocated step state per (table set, batch size): out, dx, dt and the step's indexer
const CHAIN_STEPS = IdDict{Any,Dict{Int,Any}}()
chain_step(tables, B::Int) =
    get!(() -> HipTrainStep(first(tables).data.ctx, tables, B; lr = something(first(tables).data.ctx.lr, 0f0)),
         get!(() -> Dict{Int,Any}(), CHAIN_STEPS, tables), B)

# Deferred update!: tables => the HipTrainStep whose apply launch the next maplookup runs, and the
# table sets with deferred steps whose bounds flag has not been checked yet.
const CHAIN_PENDING = IdDict{Any,Any}()
const CHAIN_UNCHECKED = IdDict{Any,Bool}()

"""
    flush!(tables; next = nothing)

Runs a deferred `update!`'s apply launch.  With `next` (the next maplookup's `PackedIndices`, same
batch size) the same launch builds their split indexer (dlrm_step_bwd_prepare), so the next
forward only gathers.  The step stays pending if the call fails.
"""
function flush!(tables; next = nothing)
    st = get(CHAIN_PENDING, tables, nothing)
    st === nothing && return nothing
    ctx = st.ctx
    d, B = size(st.x)
    if next !== nothing && next.batch == st.idx.batch && next.lookups == 1
        nix = st.spare === nothing ? HipIndexer(ctx, length(st.tables), B) : st.spare
        check(ctx, ccall((:dlrm_step_bwd_prepare, libdlrm), Cint,
                         (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Ptr{Cvoid},
                          Int64, Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cfloat,
                          Ptr{Cvoid}, Ptr{Cvoid}, Cuint),
                         ctx.ptr, tableset(st.tables), st.ix.ptr, st.idx.data.ptr, DLRM_I32, st.idx.batch, 1, B,
                         st.x.ptr, d, st.delta.ptr, size(st.delta, 1), st.padding, st.dx.ptr, d, st.dt.ptr,
                         size(st.dt, 1), ctx.lr, nix.ptr, next.data.ptr, STEP_APPLY_ONLY))
        st.spare, st.ix = st.ix, nix
        st.pending = next => next          # train_step_fwd! finds this batch's indexer prepared
    else
        check(ctx, ccall((:dlrm_step_bwd, libdlrm), Cint,
                         (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Ptr{Cvoid}, Int64,
                          Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cfloat, Cuint),
                         ctx.ptr, tableset(st.tables), st.ix.ptr, st.idx.data.ptr, DLRM_I32, st.idx.batch, 1, B,
                         st.x.ptr, d, st.delta.ptr, size(st.delta, 1), st.padding, st.dx.ptr, d, st.dt.ptr,
                         size(st.dt, 1), ctx.lr, STEP_APPLY_ONLY))
    end
    delete!(CHAIN_PENDING, tables)
    return nothing
end

# every deferred update! whose tables live on ctx (a host-visible read point: Array of any of its
# buffers)
function flush_ctx!(ctx::Context)
    for (tables, st) in collect(CHAIN_PENDING)
        st.ctx === ctx && flush!(tables)
    end
    return nothing
end

"""
    poll_bounds!(tables)

No GPU call: throws `BoundsError` if a deferred step had an out-of-range index, as far as the copy of
the device flag that has reached host memory shows (the step backward stores it).  Every kernel
skips its table writes once the flag is set, so the tables hold the state before the failing step;
the pending apply of that step is dropped.
"""
function poll_bounds!(tables)
    get(CHAIN_UNCHECKED, tables, false) || return nothing
    ctx = first(tables).data.ctx
    error_peek(ctx) == 0 && return nothing
    delete!(CHAIN_PENDING, tables)
    delete!(CHAIN_UNCHECKED, tables)
    check_bounds(ctx)                     # synchronises, clears the flag, throws BoundsError
    return nothing
end

"""
    check_bounds(tables::AbstractVector{<:HipEmbedding})

A host-visible point for a table set trained through the deferred chain: runs a pending update,
synchronises and throws `BoundsError` if any step since the last check had an out-of-range index.
Call it before reading the tables back (e.g. `Array(tables[t].data)`).
"""
function check_bounds(tables::AbstractVector{<:HipEmbedding})
    flush!(tables)
    delete!(CHAIN_UNCHECKED, tables)
    check_bounds(first(tables).data.ctx)
end

function _fused_maplookup(tables::AbstractVector{<:HipEmbedding{Static{D},T}}, sparse, P::Integer) where {D,T}
    ctx = first(tables).data.ctx
    idx = sparse isa PackedIndices ? sparse : pack(ctx, sparse)
    poll_bounds!(tables)                  # a deferred step's BoundsError (no GPU call)
    flush!(tables; next = idx)            # its apply launch, with this batch's indexer build
    return HipLookup{T}(tables, idx, Int(P))
end

function _fused_interact(dot::HipDotInteraction, x::AbstractMatrix{T}, ys::HipLookup{T}) where {T}
    d, B = size(x)
    d == ys.P || throw(DimensionMismatch("x has $d rows, maplookup reserved $(ys.P)"))
    flush!(ys.tables)                     # (an update! deferred after this lookup was made runs first)
    st = chain_step(ys.tables, B)
    train_step_fwd!(st, x isa DeviceMatrix ? x : Matrix{T}(x), ys.idx)   # dlrm_step_fwd
    st.bwd = :none
    return st
end

# (a DeviceMatrix x -- the bottom MLP on the GPU -- gets the DeviceMatrix out: no PCIe copy)
(dot::HipDotInteraction)(x::AbstractMatrix{T}, ys::HipLookup{T}; return_t = false) where {T} =
    return_t ? dot(x, DeviceMatrix(ys); return_t) :
    (x isa DeviceMatrix ? _fused_interact(dot, x, ys).out : Array(_fused_interact(dot, x, ys).out))
(dot::HipDotInteraction)(x::OneDNN.Memory, ys::HipLookup; kw...) = dot(OneDNN.materialize(x), ys; kw...)

function ChainRulesCore.rrule(dot::HipDotInteraction, X, ys::HipLookup{T}) where {T}
    x = X isa OneDNN.Memory ? OneDNN.materialize(X) : X
    st = _fused_interact(dot, x, ys)
    function dot_pullback(Δ)
        Δh = Δ isa OneDNN.Memory ? OneDNN.materialize(Δ) : Δ
        d, B = size(st.x)
        # a DeviceMatrix Δ (the top MLP on the GPU) is read in place; a host one is uploaded
        st.delta = Δh isa DeviceMatrix ? Δh : upload!(DeviceMatrix{T}(st.ctx, size(Δh)...), Matrix{T}(Δh))
        if st.ctx.lr !== nothing   # once-hit rows stepped here, the others' dt rows left for update!
            check(st.ctx, ccall((:dlrm_step_bwd, libdlrm), Cint,
                                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Ptr{Cvoid},
                                 Int64, Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cfloat, Cuint),
                                st.ctx.ptr, tableset(st.tables), st.ix.ptr, st.idx.data.ptr, DLRM_I32, st.idx.batch,
                                1, B, st.x.ptr, d, st.delta.ptr, size(Δh, 1), st.padding, st.dx.ptr, d, st.dt.ptr,
                                size(st.dt, 1), st.ctx.lr, STEP_BWD_ONLY))
            st.bwd = :once_hit_applied
        else                       # every dt row written (T re-gathered, no ys)
            check(st.ctx, ccall((:dlrm_interact_bwd_gather, libdlrm), Cint,
                                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Cint,
                                 Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64),
                                st.ctx.ptr, tableset(st.tables), C_NULL, st.idx.data.ptr, DLRM_I32, st.idx.batch, 1,
                                B, 1, st.x.ptr, d, st.delta.ptr, size(Δh, 1), st.padding, st.dx.ptr, d, st.dt.ptr,
                                size(st.dt, 1)))
            st.bwd = :all_dt
        end
        return (NoTangent(), Δh isa DeviceMatrix ? st.dx : Array(st.dx), st.dt)
    end
    return (x isa DeviceMatrix ? st.out : Array(st.out)), dot_pullback
end

function ChainRulesCore.rrule(
    ::typeof(maplookup), strategy::PreallocationStrategy, tables::AbstractVector{<:HipEmbedding{Static{D}}}, sparse
) where {D}
    first(tables).data.ctx.fused || return _rrule_maplookup(strategy, tables, sparse)
    P = prealloc_rows(strategy)
    ys = _fused_maplookup(tables, sparse, P)
    function maplookup_pullback(dt)
        dt isa DeviceMatrix{Float32} || throw(ArgumentError("the cotangent of ys is the dt of HipDotInteraction's pullback"))
        ups = [SparseEmbeddingUpdate{Static{D}}(HipDelta(dt, P + (t - 1) * D, D), HipIndices(ys.idx, t))
               for t in eachindex(tables)]
        return (NoTangent(), NoTangent(), ups, NoTangent())
    end
    return ys, maplookup_pullback
end

# update! of a fused step: the apply launch (the grads are views of that step's dt)
function _fused_update!(opt, st, tables)
    ctx = st.ctx
    d, B = size(st.x)
    if st.bwd === :once_hit_applied && ctx.defer
        opt.eta == ctx.lr || throw(ArgumentError("the pullback stepped the once-hit rows with η = $(ctx.lr), update! got $(opt.eta)"))
        # the apply launch runs in the next maplookup (flush!); bounds surface there (poll_bounds!)
        # or at check_bounds(tables): no host synchronisation here
        CHAIN_PENDING[tables] = st
        CHAIN_UNCHECKED[tables] = true
        st.bwd = :done
        return nothing
    elseif st.bwd === :once_hit_applied
        opt.eta == ctx.lr || throw(ArgumentError("the pullback stepped the once-hit rows with η = $(ctx.lr), update! got $(opt.eta)"))
        check(ctx, ccall((:dlrm_step_bwd, libdlrm), Cint,
                         (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Ptr{Cvoid}, Int64,
                          Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cfloat, Cuint),
                         ctx.ptr, tableset(st.tables), st.ix.ptr, st.idx.data.ptr, DLRM_I32, st.idx.batch, 1, B,
                         st.x.ptr, d, st.delta.ptr, size(st.delta, 1), st.padding, st.dx.ptr, d, st.dt.ptr,
                         size(st.dt, 1), ctx.lr, STEP_APPLY_ONLY))
    elseif st.bwd === :all_dt         # the forward's split indexer: once-hit rows as singles items
        check(ctx, ccall((:dlrm_sgd_update, libdlrm), Cint,
                         (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cuint, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Cint,
                          Ptr{Cvoid}, Cint, Int64, Int64, Cfloat),
                         ctx.ptr, tableset(st.tables), st.ix.ptr, UPDATE_PREBUILT, st.idx.data.ptr, DLRM_I32,
                         st.idx.batch, 1, st.idx.batch, 1, st.dt.ptr, DLRM_F32, size(st.dt, 1), d, opt.eta))
    else
        throw(ArgumentError("update! before the interaction's pullback ran"))
    end
    st.bwd = :done
    check_bounds(ctx)
    return nothing
end

#####
##### Table-sharded exchange (one Julia process per GPU): dlrm_comm_* + dlrm_alltoall_fwd / _bwd
#####

"""
    Comm(ctx, id::Vector{UInt8}, rank, nranks)

An RCCL communicator over the node's GPUs.  `comm_unique_id()` on one rank gives the 128-byte
`id` every rank passes in (distribute it with `Distributed` / MPI / a file).  `alltoall_fwd!`
sends this rank's looked-up vectors of every rank's samples (`send`: [nranks][T_me][B][D]) and
receives every owner's vectors of its own samples (`recv`: [src][T_src][B][D]); `alltoall_bwd!`
returns the fp32 gradient rows to the tables' owners.  Both run on the ctx stream.
"""
mutable struct Comm
    ctx::Context
    ptr::Ptr{Cvoid}
    counts::Vector{Cint}     # tables owned by each rank
    function Comm(ctx::Context, id::Vector{UInt8}, rank::Integer, nranks::Integer, counts::AbstractVector{<:Integer})
        length(id) == 128 || throw(ArgumentError("a communicator id has 128 bytes"))
        out = Ref{Ptr{Cvoid}}(C_NULL)
        check(ctx, ccall((:dlrm_comm_init, libdlrm), Cint, (Ptr{Cvoid}, Ptr{UInt8}, Cint, Cint, Ref{Ptr{Cvoid}}),
                         ctx.ptr, id, rank, nranks, out))
        c = new(ctx, out[], Cint.(counts))
        finalizer(x -> ccall((:dlrm_comm_destroy, libdlrm), Cint, (Ptr{Cvoid},), x.ptr), c)
        return c
    end
end
function comm_unique_id()
    id = zeros(UInt8, 128)
    rc = ccall((:dlrm_comm_unique_id, libdlrm), Cint, (Ptr{UInt8},), id)
    rc == 0 || throw(DLRMError(rc, "dlrm_comm_unique_id"))
    return id
end
"The rank count RCCL reports for the communicator (ncclCommCount)."
function nranks(c::Comm)
    n = Ref{Cint}(0)
    rc = ccall((:dlrm_comm_count, libdlrm), Cint, (Ptr{Cvoid}, Ref{Cint}), c.ptr, n)
    rc == 0 || throw(DLRMError(rc, "dlrm_comm_count"))
    return Int(n[])
end
alltoall_fwd!(c::Comm, send::DeviceMatrix{T}, recv::DeviceMatrix{T}, D::Integer, B::Integer) where {T} =
    check(c.ctx, ccall((:dlrm_alltoall_fwd, libdlrm), Cint,
                       (Ptr{Cvoid}, Ptr{Cvoid}, Cint, Cint, Cint, Ptr{Cint}, Ptr{Cvoid}, Ptr{Cvoid}),
                       c.ctx.ptr, c.ptr, dtype_code(T), D, B, c.counts, send.ptr, recv.ptr))
alltoall_bwd!(c::Comm, gsend::DeviceMatrix{Float32}, grecv::DeviceMatrix{Float32}, D::Integer, B::Integer) =
    check(c.ctx, ccall((:dlrm_alltoall_bwd, libdlrm), Cint,
                       (Ptr{Cvoid}, Ptr{Cvoid}, Cint, Cint, Ptr{Cint}, Ptr{Cvoid}, Ptr{Cvoid}),
                       c.ctx.ptr, c.ptr, D, B, c.counts, gsend.ptr, grecv.ptr))

#####
##### DACLoader replacement (src/data/criteo.jl:309-340): records uploaded raw, load! on the GPU
#####

"""
    HipDACLoader(ctx, dataset::Vector{DACRecord}, batchsize)

Iterates like `DACLoader` (whole batches only, `length = div(length(dataset), batchsize)`) and
yields `(; labels, dense, sparse)` in HBM: `labels` 1 × B Float32, `dense` 13 × B Float32 and
`sparse` a `PackedIndices` over the `Matrix{UInt32}(B, 26)` layout (1-based ids), ready for
`maplookup` / `train_step_fwd!`.  `DACRecord` is bit-compatible with `dlrm_dac_record` (160 B),
so each batch is one upload of the mmap'd records and one `dlrm_dac_decode` launch.
"""
struct HipDACLoader{V}
    ctx::Context
    dataset::V
    batchsize::Int
    raw::DeviceMatrix{UInt8}
    labels::DeviceMatrix{Float32}
    dense::DeviceMatrix{Float32}
    sparse::DeviceMatrix{Int32}
end
function HipDACLoader(ctx::Context, dataset::AbstractVector, batchsize::Integer)
    @assert sizeof(eltype(dataset)) == 160 "DACRecord is 160 bytes (criteo.jl:91-95)"
    B = Int(batchsize)
    return HipDACLoader(ctx, dataset, B, DeviceMatrix{UInt8}(ctx, 160, B), DeviceMatrix{Float32}(ctx, 1, B),
                        DeviceMatrix{Float32}(ctx, 13, B), DeviceMatrix{Int32}(ctx, B, 26))
end
Base.length(l::HipDACLoader) = div(length(l.dataset), l.batchsize)
function Base.iterate(l::HipDACLoader, i = 1)
    i > length(l) && return nothing
    B = l.batchsize
    recs = view(l.dataset, (B * (i - 1) + 1):(B * i))
    GC.@preserve recs begin
        check(l.ctx, ccall((:dlrm_memcpy_h2d, libdlrm), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t),
                           l.ctx.ptr, l.raw.ptr, pointer(recs), 160 * B))
    end
    check(l.ctx, ccall((:dlrm_dac_decode, libdlrm), Cint,
                       (Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Cint, Int64),
                       l.ctx.ptr, l.raw.ptr, B, l.labels.ptr, l.dense.ptr, 13, l.sparse.ptr, DLRM_I32, B))
    return (; labels = l.labels, dense = l.dense, sparse = PackedIndices(l.sparse, B, 1)), i + 1
end

end # module
