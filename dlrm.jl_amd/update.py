"""Sparse embedding gradients and the SGD scatter update.

Mirrors EmbeddingTables' training API as DLRM.jl calls it:
  * the maplookup pullback -> one `SparseEmbeddingUpdate(delta, indices)` per table
    (test/model/embedding_update.jl:35-40, test/train/backprop.jl:147-158);
  * `SparseIndexer()` per table (src/train/train.jl:276-281);
  * `update!(Descent(lr), tables, grads, indexers; num_splits, nthreads)`
    (src/train/train.jl:283-290) -> `update_` here (Python has no `!`).
The deterministic GPU path dedupes each table's indices with a stable sort and writes every
touched row once; `deterministic=False` uses float atomics instead.
"""
import ctypes

import torch

from . import _lib
from .embedding import EmbeddingTableSet, PackedIndices, as_table_set
from .runtime import context, dtype_code, ptr, require_device


class Descent:
    """Flux.Descent(η): plain SGD, w .-= η * g (default η = 0.1 as in Flux)."""

    def __init__(self, eta=0.1):
        self.eta = float(eta)

    def __repr__(self):
        return f"Descent({self.eta})"


class SparseEmbeddingUpdate:
    """SparseEmbeddingUpdate{Static{D}}(delta, indices): the gradient of one table.

    `delta` is a [B][D] view (column block of the interaction's dt); `grad`, `grad_offset`
    keep the parent matrix so that all tables can be updated in one launch."""

    def __init__(self, grad, grad_offset, featuresize, indices, table_index):
        self.grad = grad
        self.grad_offset = int(grad_offset)
        self.featuresize = int(featuresize)
        self.indices = indices  # PackedIndices of ALL tables (row `table_index` is this table's)
        self.table_index = int(table_index)

    @property
    def delta(self):
        return self.grad[:, self.grad_offset:self.grad_offset + self.featuresize]

    def uncompress(self, nrows, *, index_base=1):
        """uncompress(update, nrows) (test/train/backprop.jl:156): the dense [nrows][D] gradient,
        Σ of delta rows per index (pooled bags: a bag's row counts once per lookup).  It is
        update!(Descent(-1)) into a zero table -- the same deterministic HIP indexer + apply, so the
        sum per row runs in ascending position order, fp32."""
        if self.indices.data.device.type != "cuda":
            raise ValueError("uncompress runs on the GPU (the indices must be device tensors)")
        dev = self.indices.data.device
        out = torch.zeros((nrows, self.featuresize), dtype=torch.float32, device=dev)
        ts = EmbeddingTableSet([out])
        one = PackedIndices(self.indices.data[self.table_index:self.table_index + 1].reshape(
            1, self.indices.B, self.indices.L))
        g = self.grad
        if g.stride(1) != 1:
            raise ValueError("gradient rows must be contiguous")
        require_device(g, dev, "gradient")
        ix = SparseIndexer(1, one.B * one.L, dev)
        ctx = ts.ctx
        ctx.check(ctx.lib.dlrm_sgd_update(ctx.bind(), ts.handle, ix.handle, 0, ptr(one.data), one.itype, one.stride,
                                          index_base, one.B, one.L, ptr(g), dtype_code(g.dtype), g.stride(0),
                                          self.grad_offset, -1.0))
        ctx.check_bounds()
        return out


def maplookup_pullback(strategy_prealloc, tables, sparse, dy):
    """Pullback of maplookup(PreallocationStrategy(P), tables, sparse) given dy [B][P + D*T]
    (e.g. dt_reshaped from dot_back): views, no arithmetic (the rows 1:P belong to x).
    HipTables + the LazyGrad of the fused interaction's pullback: DeferredUpdate views (lazy.py)."""
    from .lazy import HipTables, LazyGrad, pullback_lazy
    if isinstance(tables, HipTables) and isinstance(dy, LazyGrad):
        return pullback_lazy(strategy_prealloc, tables, dy)
    if isinstance(tables, HipTables):
        tables = tables.ts
    ts = as_table_set(tables)
    idx = PackedIndices(sparse, device=ts.device)
    return [SparseEmbeddingUpdate(dy, strategy_prealloc + t * ts.D, ts.D, idx, t) for t in range(len(ts))]


class SparseIndexer:
    """SparseIndexer(): dedupe state for `update_`.  One object serves a whole table set (the
    reference keeps one per table); sized for `capacity` lookups per table."""

    def __init__(self, num_tables, capacity, device=None):
        self.ctx = context(device)
        self.num_tables = int(num_tables)
        self.capacity = int(capacity)
        h = ctypes.c_void_p()
        self.ctx.check(self.ctx.lib.dlrm_indexer_create(self.ctx.bind(), self.num_tables, self.capacity,
                                                        ctypes.byref(h)))
        self.handle = h
        self._built_from = None

    def build(self, tables, indices, *, index_base=1):
        """Dedupes `indices` (asynchronous).  May run on a side stream during the forward pass;
        pass prebuilt=True to update_ afterwards."""
        ts = as_table_set(tables)
        idx = PackedIndices(indices, device=ts.device)
        require_device(idx.data, ts.device, "indices")
        if idx.B * idx.L > self.capacity or idx.T != self.num_tables:
            raise ValueError("SparseIndexer: indices exceed the capacity / table count it was created for")
        self.ctx.check(self.ctx.lib.dlrm_indexer_build(self.ctx.bind(), self.handle, ts.handle, ptr(idx.data),
                                                       idx.itype, idx.stride, index_base, idx.B, idx.L))
        self._built_from = idx
        return self

    def prepare(self, tables, indices, *, index_base=1):
        """The training step's split build of `indices` (one-hot, <= 32768 positions per table) as its
        own launch (dlrm_indexer_prepare: the wave build): a following dlrm_step_fwd of
        these indices only gathers, and update_ / dlrm_sgd_update(PREBUILT) take its once-hit
        positions as well.  Returns False where the wave build does not apply (use build())."""
        ts = as_table_set(tables)
        idx = PackedIndices(indices, device=ts.device)
        require_device(idx.data, ts.device, "indices")
        if idx.L != 1 or idx.B > self.capacity or idx.T != self.num_tables:
            return False
        rc = self.ctx.lib.dlrm_indexer_prepare(self.ctx.bind(), self.handle, ts.handle, ptr(idx.data), idx.itype,
                                               idx.stride, index_base, idx.B)
        if rc == _lib.E_UNSUPPORTED:
            return False
        self.ctx.check(rc)
        self._built_from = idx
        return True

    def reserve(self, batch):
        """dlrm_indexer_reserve: a no-op since round 6 (the wave builds' packed layout needs no
        re-carving before a graph capture); kept for round-5 callers."""
        self.ctx.check(self.ctx.lib.dlrm_indexer_reserve(self.ctx.bind(), self.handle, int(batch)))
        return self

    def set_chunk(self, max_positions):
        """The wave build's chunk limit for later builds (16 or 32; dlrm_indexer_set_chunk)."""
        self.ctx.check(self.ctx.lib.dlrm_indexer_set_chunk(self.ctx.bind(), self.handle, int(max_positions)))
        return self

    def set_parts(self, parts):
        """Parts per table of later wave builds of <= 2048 positions (0 / 16, 32 or 64;
        dlrm_indexer_set_parts): the same segments whatever the setting."""
        self.ctx.check(self.ctx.lib.dlrm_indexer_set_parts(self.ctx.bind(), self.handle, int(parts)))
        return self

    def nbytes(self):
        """Device bytes held (dlrm_indexer_bytes: all allocated at creation, never grown)."""
        b = ctypes.c_int64()
        self.ctx.check(self.ctx.lib.dlrm_indexer_bytes(self.handle, ctypes.byref(b)))
        return b.value

    def state(self):
        """Host-side state of the last build: a mask of _lib.IX_* bits (no GPU call)."""
        st = ctypes.c_uint()
        self.ctx.check(self.ctx.lib.dlrm_indexer_state(self.handle, ctypes.byref(st)))
        return st.value

    def unique_rows(self, table):
        """0-based unique rows touched in `table` by the last build, in segment order (synchronises)."""
        n = ctypes.c_int64()
        cap = self.capacity
        rows = (ctypes.c_int64 * max(cap, 1))()
        self.ctx.check(self.ctx.lib.dlrm_indexer_read(self.ctx.bind(), self.handle, table, ctypes.byref(n), rows,
                                                      None, None, cap))
        return list(rows[: n.value])

    def segments(self, table):
        """(unique_rows, positions, seg_start) of `table`: positions grouped by row (one segment per
        row, segment order unspecified), ascending within a row."""
        n = ctypes.c_int64()
        cap = self.capacity
        rows = (ctypes.c_int64 * max(cap, 1))()
        pos = (ctypes.c_int64 * max(cap, 1))()
        seg = (ctypes.c_int64 * (cap + 1))()
        self.ctx.check(self.ctx.lib.dlrm_indexer_read(self.ctx.bind(), self.handle, table, ctypes.byref(n), rows, pos,
                                                      seg, cap))
        U = n.value
        segs = list(seg[: U + 1])
        nv = segs[U] if U >= 0 else 0
        return list(rows[:U]), list(pos[:nv]), segs

    def __del__(self):
        try:
            if self.handle:
                self.ctx.lib.dlrm_indexer_destroy(self.handle)
        except Exception:
            pass


def update_(opt, tables, grads, indexers=None, *, num_splits=8, nthreads=12, index_base=None, deterministic=True,
            prebuilt=False, check_bounds=None):
    """EmbeddingTables.update!(opt, tables, grads, indexers; num_splits, nthreads).

    `grads` are the SparseEmbeddingUpdates of maplookup_pullback (they share one gradient
    matrix and one PackedIndices, so all tables update in one launch).  num_splits/nthreads
    are accepted for signature parity; the GPU decomposition is chunk-based.
    index_base: 1 (Julia) unless given; HipTables carry their own (a different one raises).
    Tables are mutated in place.  check_bounds (not a reference keyword): None = the default --
    synchronise and raise BoundsError for plain tables; HipTables follow their own policy (a
    deferred apply whose bounds surface at the next maplookup, lazy.py)."""
    del num_splits, nthreads
    from .lazy import DeferredUpdate, HipTables, update_lazy
    if isinstance(tables, HipTables) and grads and isinstance(grads[0], DeferredUpdate):
        tables.check_index_base(index_base, "update_")
        if not deterministic:
            raise ValueError("update_ on HipTables is the deterministic step apply (deterministic=False is not "
                             "available on the fused path)")
        # (indexers: accepted for the reference's signature; the step carries its own SparseIndexer)
        return update_lazy(opt, tables, grads, check_bounds=check_bounds)
    index_base = 1 if index_base is None else int(index_base)
    if isinstance(tables, HipTables):
        tables = tables.ts
    if not isinstance(opt, Descent):
        raise TypeError("update_ implements Descent (plain SGD), the optimizer DLRM.jl trains with")
    ts = as_table_set(tables)
    if len(grads) != len(ts):
        raise ValueError(f"{len(grads)} gradients for {len(ts)} tables")
    g0 = grads[0]
    for t, g in enumerate(grads):
        if (g.grad.data_ptr() != g0.grad.data_ptr() or g.indices is not g0.indices or g.table_index != t or
                g.grad_offset != g0.grad_offset + t * ts.D):
            raise ValueError("update_ expects the per-table views produced by maplookup_pullback")
    grad = g0.grad
    if grad.stride(1) != 1:
        raise ValueError("gradient rows must be contiguous")
    require_device(grad, ts.device, "gradient")
    idx = g0.indices.on(ts.device)
    if grad.shape[0] != idx.B:
        raise ValueError(f"gradient has {grad.shape[0]} rows for a batch of {idx.B}")
    flags = 0
    ix = None
    if deterministic:
        if indexers is None:
            indexers = SparseIndexer(len(ts), idx.B * idx.L, ts.device)
        ix = indexers
        if ix.num_tables != len(ts) or ix.capacity < idx.B * idx.L:
            raise ValueError("SparseIndexer too small for this batch / table set")
        if prebuilt:
            flags |= _lib.UPDATE_PREBUILT
    else:
        flags |= _lib.UPDATE_ATOMIC
    ctx = ts.ctx
    ctx.check(ctx.lib.dlrm_sgd_update(ctx.bind(), ts.handle, ix.handle if ix is not None else None, flags,
                                      ptr(idx.data), idx.itype, idx.stride, index_base, idx.B, idx.L, ptr(grad),
                                      dtype_code(grad.dtype), grad.stride(0), g0.grad_offset, opt.eta))
    if check_bounds or check_bounds is None:
        ctx.check_bounds()
    return tables
