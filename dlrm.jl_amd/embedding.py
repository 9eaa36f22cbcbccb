"""Embedding tables and `maplookup` — the forward gather of the DLRM hot path.

Mirrors the operator interface DLRM.jl uses from its (un-vendored) EmbeddingTables
dependency: `SimpleEmbedding{Static{D}}(data)`, `maplookup(strategy, tables, sparse)`,
`lookup(table, idx)`, `PreallocationStrategy(P)` / `DefaultStrategy()`
(call sites: src/model/model.jl:155-161, src/data/criteo.jl:484-492, test/integration.jl:10-11,
test/model/embedding_update.jl:23-33).

Layout: Julia is column-major, so a Julia (D, N) table is a row-major torch tensor [N][D],
and the preallocated lookup output (P + D*T) x B is a torch tensor [B][P + D*T] whose
columns [0, P) are left for the dense vector x (interact.jl:264-270).
Indices follow Julia semantics by default (index_base=1); pass index_base=0 for PyTorch /
HDF5 indices.
"""
import ctypes

import torch

from . import _lib
from .runtime import context, dtype_code, itype_code, ptr, require_device


class SimpleEmbedding:
    """SimpleEmbedding{Static{D}}: one dense table, stored [nrows][D] in HBM."""

    def __init__(self, data):
        if not isinstance(data, torch.Tensor) or data.dim() != 2:
            raise TypeError("SimpleEmbedding expects a 2-D torch tensor [nrows][D]")
        if not data.is_cuda:
            raise ValueError("SimpleEmbedding data must live on the GPU")
        dtype_code(data.dtype)
        self.data = data.contiguous()

    @property
    def featuresize(self):
        return self.data.shape[1]

    def __len__(self):
        return self.data.shape[0]

    def __repr__(self):
        return f"SimpleEmbedding{{Static{{{self.featuresize}}}}}({len(self)} rows, {self.data.dtype})"


class EmbeddingTableSet:
    """A Vector{SimpleEmbedding{Static{D}}} registered with the HIP library (one dlrm_tables).

    All tables share D and dtype, as in every DLRM.jl model (dlrm(), model.jl:173-233)."""

    def __init__(self, tables):
        tables = [t if isinstance(t, SimpleEmbedding) else SimpleEmbedding(t) for t in tables]
        if not tables:
            raise ValueError("EmbeddingTableSet needs at least one table")
        D = tables[0].featuresize
        dt = tables[0].data.dtype
        dev = tables[0].data.device
        for t in tables:
            if t.featuresize != D or t.data.dtype != dt or t.data.device != dev:
                raise ValueError("all tables must share feature size, dtype and device")
        self.tables = tables
        self.D = D
        self.dtype = dt
        self.device = dev
        self.ctx = context(dev)
        T = len(tables)
        ptrs = (ctypes.c_void_p * T)(*[t.data.data_ptr() for t in tables])
        nrows = (ctypes.c_int64 * T)(*[len(t) for t in tables])
        h = ctypes.c_void_p()
        self.ctx.check(self.ctx.lib.dlrm_tables_create(self.ctx.bind(), T, D, dtype_code(dt), ptrs, nrows,
                                                       ctypes.byref(h)))
        self.handle = h

    def __len__(self):
        return len(self.tables)

    def __getitem__(self, i):
        return self.tables[i]

    def __iter__(self):
        return iter(self.tables)

    def nrows(self):
        return [len(t) for t in self.tables]

    def __del__(self):
        try:
            if self.handle:
                self.ctx.lib.dlrm_tables_destroy(self.handle)
        except Exception:
            pass


def as_table_set(tables):
    return tables if isinstance(tables, EmbeddingTableSet) else EmbeddingTableSet(list(tables))


class PreallocationStrategy:
    """PreallocationStrategy{T}(P): one (P + D*T) x B output, rows 1:P left for x."""

    def __init__(self, prealloc=0, dtype=None):
        if prealloc < 0:
            raise ValueError("PreallocationStrategy: negative preallocation")
        self.prealloc = int(prealloc)
        self.dtype = dtype

    def __repr__(self):
        return f"PreallocationStrategy({self.prealloc})"


class DefaultStrategy:
    """DefaultStrategy(): one D x B result per table."""

    def __repr__(self):
        return "DefaultStrategy()"


class PackedIndices:
    """Index arrays of all tables as one device tensor [T][B*L] (sample-major per table).

    Accepts the reference's forms: a list of per-table [B] vectors (Vector{Vector{Int}}),
    a list of per-table [B][L] tensors (the C view of Julia's L x B matrices, criteo.jl:551-557),
    or one [T][B] / [T][B][L] tensor (DACLoader's per-table-contiguous sparse matrix)."""

    def __init__(self, sparse, device=None, dtype=None):
        if isinstance(sparse, PackedIndices):
            self.__dict__.update(sparse.__dict__)
            if device is not None and self.data.device != torch.device(device):
                self.data = self.data.to(device)
            return
        if isinstance(sparse, torch.Tensor):
            if sparse.dim() == 2:
                T, B = sparse.shape
                L = 1
            elif sparse.dim() == 3:
                T, B, L = sparse.shape
            else:
                raise ValueError("packed indices must be [T][B] or [T][B][L]")
            data = sparse.reshape(T, B * L)
        else:
            sparse = list(sparse)
            if not sparse:
                raise ValueError("no index arrays")
            shapes = {tuple(s.shape) for s in sparse}
            if len(shapes) != 1:
                raise ValueError(f"all tables need the same batch/lookups shape, got {shapes}")
            shp = shapes.pop()
            B = shp[0]
            L = shp[1] if len(shp) == 2 else 1
            T = len(sparse)
            data = torch.stack([torch.as_tensor(s).reshape(B * L) for s in sparse])
        if device is not None and data.device != torch.device(device):
            data = data.to(device)
        if dtype is not None and data.dtype != dtype:
            data = data.to(dtype)
        if data.dtype not in (torch.int32, torch.int64):
            data = data.to(torch.int64)
        self.data = data.contiguous()
        self.T, self.B, self.L = int(T), int(B), int(L)

    @classmethod
    def columns(cls, packed, b0, b1):
        """Samples [b0, b1) of every table as a view (no copy): data [T][(b1-b0)*L] with the
        parent's table stride (the micro-batch slices of the sharded step)."""
        v = cls.__new__(cls)
        L = packed.L
        v.data = packed.data[:, b0 * L:b1 * L]
        v.T, v.B, v.L = packed.T, int(b1 - b0), L
        return v

    def on(self, device):
        """This index set on `device` (self if already there)."""
        return self if self.data.device == torch.device(device) else PackedIndices(self, device=device)

    @property
    def stride(self):
        return self.data.stride(0) if self.T > 0 else 0

    @property
    def itype(self):
        return itype_code(self.data.dtype)


def maplookup(strategy, tables, sparse, *, index_base=None, out=None, check_bounds=True):
    """maplookup(strategy, tables, sparse) (EmbeddingTables; model.jl:161).

    PreallocationStrategy(P): returns [B][P + D*T]; row b holds [<untouched P> | e_1 | ... | e_T]
    where e_t = sum_k table_t[idx_t[b, k]] (sum pooling for multi-hot bags).
    DefaultStrategy(): returns a list of per-table [B][D] tensors.
    Raises BoundsError on an out-of-range index when check_bounds (synchronises).
    index_base: 1 (Julia) unless given.
    With `HipTables` (lazy.py): a LazyLookup, gathered by the interaction's fused kernel; the
    tables carry the index base (a different `index_base` raises) and `out` is not taken."""
    from .lazy import HipTables, maplookup_lazy
    if isinstance(tables, HipTables):
        tables.check_index_base(index_base, "maplookup")
        if out is not None:
            raise ValueError("maplookup on HipTables defers the gather into the interaction: no `out` buffer "
                             "(materialize the LazyLookup, or pass the plain table set)")
        return maplookup_lazy(strategy, tables, sparse, check_bounds=check_bounds)
    index_base = 1 if index_base is None else int(index_base)
    ts = as_table_set(tables)
    idx = PackedIndices(sparse, device=ts.device)
    require_device(idx.data, ts.device, "indices")
    if idx.T != len(ts):
        raise ValueError(f"{idx.T} index arrays for {len(ts)} tables")
    P = strategy.prealloc if isinstance(strategy, PreallocationStrategy) else 0
    width = P + ts.D * len(ts)
    if out is None:
        out = torch.empty((idx.B, width), dtype=ts.dtype, device=ts.device)
    elif out.shape[0] != idx.B or out.shape[1] < width or out.stride(1) != 1 or out.dtype != ts.dtype:
        raise ValueError("maplookup: `out` has the wrong shape/dtype/layout")
    require_device(out, ts.device, "out")
    ctx = ts.ctx
    ctx.check(ctx.lib.dlrm_maplookup(ctx.bind(), ts.handle, ptr(idx.data), idx.itype, idx.stride, index_base,
                                     idx.B, idx.L, ptr(out), out.stride(0), P))
    if check_bounds:
        ctx.check_bounds()
    if isinstance(strategy, PreallocationStrategy):
        return out
    return [out[:, t * ts.D:(t + 1) * ts.D] for t in range(len(ts))]


def lookup(table, idx, *, index_base=1, check_bounds=True):
    """lookup(table, idx): table[:, idx] in Julia terms -> [B][D] (sum over L for [B][L] bags)."""
    idx = torch.as_tensor(idx)
    return maplookup(DefaultStrategy(), [table], [idx], index_base=index_base, check_bounds=check_bounds)[0]
