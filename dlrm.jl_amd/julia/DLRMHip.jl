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
import EmbeddingTables: maplookup, PreallocationStrategy, SparseEmbeddingUpdate, Static

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
    function Context(device::Integer; stream::Ptr{Cvoid} = C_NULL)
        out = Ref{Ptr{Cvoid}}(C_NULL)
        rc = ccall((:dlrm_ctx_create, libdlrm), Cint, (Cint, Ptr{Cvoid}, Ref{Ptr{Cvoid}}), device, stream, out)
        rc == 0 || throw(DLRMError(rc, "dlrm_ctx_create"))
        ctx = new(out[])
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

function _maplookup(tables::AbstractVector{<:HipEmbedding{Static{D},T}}, sparse) where {D,T}
    ctx = first(tables).data.ctx
    idx = sparse isa PackedIndices ? sparse : pack(ctx, sparse)
    P = D                                                           # rows 1:P reserved for x
    ys = DeviceMatrix{T}(ctx, P + D * length(tables), idx.batch)
    check(ctx, ccall((:dlrm_maplookup, libdlrm), Cint,
                     (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Cint, Ptr{Cvoid}, Int64, Int64),
                     ctx.ptr, tableset(tables), idx.data.ptr, DLRM_I32, idx.batch * idx.lookups, 1,
                     idx.batch, idx.lookups, ys.ptr, size(ys, 1), P))
    return ys, idx
end

EmbeddingTables.maplookup(::PreallocationStrategy, tables::AbstractVector{<:HipEmbedding}, sparse) =
    first(_maplookup(tables, sparse))

# The gradient of the lookup is the dt the interaction backward wrote; SparseEmbeddingUpdate
# just names (dt, its row offset, the indices) so update! can hand them to the kernel.
struct HipEmbeddingUpdate
    dt::DeviceMatrix{Float32}
    offset::Int
    indices::PackedIndices
end

function ChainRulesCore.rrule(
    ::typeof(maplookup), strategy::PreallocationStrategy, tables::AbstractVector{<:HipEmbedding}, sparse
)
    ys, idx = _maplookup(tables, sparse)
    D = featuresize(first(tables))
    # one entry per table (grads.embeddings is a Vector, src/train/train.jl:144); all of them
    # view the same dt: table t's rows sit at offset D + (t-1)*D of every dt column
    pullback(dt) = (NoTangent(), NoTangent(), [HipEmbeddingUpdate(dt, D, idx) for _ in tables], NoTangent())
    return ys, pullback
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

function (dot::HipDotInteraction)(x::AbstractMatrix{T}, ys::DeviceMatrix{T}) where {T}
    d, B = size(x)
    F = size(ys, 1) ÷ d
    xd = x isa DeviceMatrix ? x : upload!(DeviceMatrix{T}(dot.ctx, d, B), x)   # bottom MLP output
    width, padding = interaction_sizes(d, F, dot.pad_to)
    out = DeviceMatrix{T}(dot.ctx, width, B)
    check(dot.ctx, ccall((:dlrm_interact_fwd, libdlrm), Cint,
                         (Ptr{Cvoid}, Cint, Cint, Cint, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cint),
                         dot.ctx.ptr, dtype_code(T), d, F, B, xd.ptr, d, ys.ptr, size(ys, 1), out.ptr, width, padding))
    return Array(out), padding                                     # the top MLP runs on the CPU
end

function ChainRulesCore.rrule(dot::HipDotInteraction, x::AbstractMatrix{T}, ys::DeviceMatrix{T}) where {T}
    out, padding = dot(x, ys)
    d, B = size(x)
    F = size(ys, 1) ÷ d
    function dot_pullback(Δ)
        Δd = upload!(DeviceMatrix{T}(dot.ctx, size(Δ)...), Matrix{T}(Δ))
        dx = DeviceMatrix{Float32}(dot.ctx, d, B)
        dt = DeviceMatrix{Float32}(dot.ctx, F * d, B)               # x rows included, as dot_back
        check(dot.ctx, ccall((:dlrm_interact_bwd, libdlrm), Cint,
                             (Ptr{Cvoid}, Cint, Cint, Cint, Cint, Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64,
                              Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64),
                             dot.ctx.ptr, dtype_code(T), d, F, B, Δd.ptr, size(Δ, 1), padding, ys.ptr, size(ys, 1),
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

const INDEXERS = IdDict{Any,HipIndexer}()

# `num_splits` / `nthreads` tune the CPU scatter; the GPU kernel has its own decomposition.
function EmbeddingTables.update!(
    opt, tables::AbstractVector{<:HipEmbedding{Static{D}}}, grads::AbstractVector{HipEmbeddingUpdate},
    indexers; num_splits = 8, nthreads = Threads.nthreads()
) where {D}
    g = first(grads)           # one dt buffer and one packed index set serve every table
    ctx = g.dt.ctx
    idx = g.indices
    ix = get!(() -> HipIndexer(ctx, length(tables), idx.batch * idx.lookups), INDEXERS, indexers)
    check(ctx, ccall((:dlrm_sgd_update, libdlrm), Cint,
                     (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cuint, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Cint,
                      Ptr{Cvoid}, Cint, Int64, Int64, Cfloat),
                     ctx.ptr, tableset(tables), ix.ptr, 0, idx.data.ptr, DLRM_I32, idx.batch * idx.lookups, 1,
                     idx.batch, idx.lookups, g.dt.ptr, DLRM_F32, size(g.dt, 1), g.offset, opt.eta))
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
end
function HipTrainStep(ctx::Context, tables::AbstractVector{<:HipEmbedding{Static{D},T}}, batch::Integer;
                      lr = 0.01, pad_to = 1) where {D,T}
    F = length(tables) + 1
    width, padding = interaction_sizes(D, F, pad_to)
    return HipTrainStep{T}(ctx, collect(tables), HipIndexer(ctx, length(tables), batch),
                           DeviceMatrix{T}(ctx, width, batch), DeviceMatrix{Float32}(ctx, D, batch),
                           DeviceMatrix{Float32}(ctx, F * D, batch), nothing, nothing, padding, Float32(lr))
end

function train_step_fwd!(st::HipTrainStep{T}, x::AbstractMatrix{T}, sparse) where {T}
    d, B = size(x)
    st.idx = sparse isa PackedIndices ? sparse : pack(st.ctx, sparse)
    st.x = x isa DeviceMatrix ? x : upload!(DeviceMatrix{T}(st.ctx, d, B), x)
    check(st.ctx, ccall((:dlrm_step_fwd, libdlrm), Cint,
                        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Ptr{Cvoid}, Int64,
                         Ptr{Cvoid}, Int64, Cint),
                        st.ctx.ptr, tableset(st.tables), st.ix.ptr, st.idx.data.ptr, DLRM_I32, st.idx.batch, 1, B,
                        st.x.ptr, d, st.out.ptr, size(st.out, 1), st.padding))
    return Array(st.out)
end

function train_step_bwd!(st::HipTrainStep{T}, Δ::AbstractMatrix{T}) where {T}
    d, B = size(st.x)
    Δd = upload!(DeviceMatrix{T}(st.ctx, size(Δ)...), Matrix{T}(Δ))
    check(st.ctx, ccall((:dlrm_step_bwd, libdlrm), Cint,
                        (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Int64, Cint, Cint, Ptr{Cvoid}, Int64,
                         Ptr{Cvoid}, Int64, Cint, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Int64, Cfloat, Cuint),
                        st.ctx.ptr, tableset(st.tables), st.ix.ptr, st.idx.data.ptr, DLRM_I32, st.idx.batch, 1, B,
                        st.x.ptr, d, Δd.ptr, size(Δ, 1), st.padding, st.dx.ptr, d, st.dt.ptr, size(st.dt, 1),
                        st.lr, Cuint(0)))
    return Array(st.dx)
end

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
