"""The reference's operator chain on the fused training-step kernels.

An unchanged `train!` (src/train/train.jl:215-227, :283-290) drives the hot path as four operators:

    ys = maplookup(PreallocationStrategy(d), tables, sparse)     model.jl:161
    out, back = rrule(interaction, x, ys)                          model.jl:163, interact.jl:438-447
    _, dx, dy = back(Δ)                                            (Zygote pullback)
    update!(Descent(η), tables, maplookup_pullback(dy), indexers)  train.jl:283-290

Run literally, that is five launches with ys written to and read back from HBM.  `HipTables` is
the table type whose methods make the same four calls hit the fused kernels (the Python mirror of
DLRMHip.jl's lazy `maplookup` for `HipEmbedding`):

  maplookup            -> a `LazyLookup` (indices + tables; nothing launched, ys never written)
  DotInteraction(x, ys)-> dlrm_step_fwd: the gather, the interaction and the update's indexer in
                          one launch (the gather-only forward)
  its pullback         -> dlrm_step_bwd(DLRM_STEP_BWD_ONLY): dot_back on re-gathered rows; with the
                          learning rate known up front (`HipTables(..., lr=η)`) the rows hit once in
                          the batch get their SGD step right there, else every dt row is written
  maplookup_pullback   -> `DeferredUpdate` views of that dt
  update!              -> dlrm_step_bwd(DLRM_STEP_APPLY_ONLY) (the repeated rows), or, without a
                          known η, dlrm_sgd_update(PREBUILT) with the forward's split indexer

Three launches per step, bit for bit the result of `HotPath.step` and of the five-launch chain.

With the learning rate known, `update!` is deferred by default (`HipTables(..., defer_update=True)`, a
property of the tables, so the reference's own call `update!(opt, tables, grads, indexers; num_splits,
nthreads)` defers unchanged): its apply launch runs in the next `maplookup` on these tables, together
with the build of that batch's indexer (dlrm_step_bwd_prepare with STEP_APPLY_ONLY), so the forward
that follows only gathers -- the pipelined step's three launches, with no host synchronisation.
Bounds errors keep the reference's outcome (BoundsError, and no row of the failing step written):
the kernels skip every table write once the device flag is set, the step backward copies the flag
into host memory (one thread's store), and the next `maplookup` reads that copy without touching
the GPU (dlrm_error_peek) and raises BoundsError when it is set -- one step or more after
the failing one, the tables still in the state before it.  `check_bounds()` and every read of the
tables through `HipTables` (`ts`, indexing, iteration) run a pending update and synchronise.
Anything else that reads ys gets it materialized (`LazyLookup.materialize`).  `out`, `dx` and the
gradient live in per-batch-size buffers reused by the next step, as the reference's own
preallocated scratch (`DotInteraction`'s per-thread scratchpads) is.
"""
from . import _lib
from .embedding import EmbeddingTableSet, PackedIndices, PreallocationStrategy, as_table_set
from .update import Descent, SparseEmbeddingUpdate


class HipTables:
    """Vector{HipEmbedding{Static{D}}}: embedding tables whose lookup is deferred into the
    interaction.  lr: the Descent η the following update! will use (lets the backward apply the
    once-hit rows itself, the fastest form); None: update! applies every row.  defer_update: with
    lr known, update! leaves its apply launch to the next maplookup (bounds errors surface there,
    from a snapshot of the device flag, or at check_bounds / a read of the tables); False: update!
    runs it at once and synchronises to check bounds, as the reference's update! returns with the
    tables written."""

    def __init__(self, tables, *, lr=None, index_base=1, defer_update=True):
        self._ts = as_table_set(tables) if not isinstance(tables, EmbeddingTableSet) else tables
        self.lr = None if lr is None else float(lr)
        self.index_base = int(index_base)  # 1: Julia's, as maplookup / update_ default to
        self.defer_update = bool(defer_update)
        self._hp = {}
        self._spare = {}      # batch -> the second indexer of the pipelined form
        self._pending = None  # the LazyGrad whose apply launch is deferred to the next maplookup
        self._unchecked = False  # deferred steps whose bounds flag has not been checked yet

    @property
    def ts(self):
        """The EmbeddingTableSet, with any deferred update applied and its bounds checked (a read of
        the tables is a host-visible point: BoundsError here if a deferred step had a bad index)."""
        self.check_bounds()
        return self._ts

    def check_bounds(self):
        """Runs a deferred update, synchronises and raises BoundsError if any step since the last
        check skipped an out-of-range index (its rows, and those of every later step, unwritten)."""
        self.flush()
        self._unchecked = False
        self._ts.ctx.check_bounds()

    def poll_bounds(self):
        """No GPU call: raises BoundsError if the last error-flag snapshot that has landed is set.
        A pending update of a failed step is dropped (the kernels skipped its writes anyway)."""
        if self._unchecked and self._ts.ctx.error_peek():
            self._pending = None
            self._unchecked = False
            self._ts.ctx.check_bounds()  # synchronises, clears the flag, raises

    def flush(self, next_idx=None):
        """Runs a deferred update!'s apply launch.  next_idx (the next maplookup's PackedIndices):
        the same launch builds their split indexer, so the next forward only gathers."""
        lz = self._pending
        if lz is None:
            return
        hp = lz.hp
        if (next_idx is not None and next_idx.L == 1 and next_idx.B == lz.idx.B and
                (next_idx.itype, next_idx.stride) == (lz.idx.itype, lz.idx.stride)):
            nix = self._spare.get(hp.B)
            if nix is None:
                from .update import SparseIndexer
                nix = self._spare[hp.B] = SparseIndexer(hp.T, hp.B, hp.ts.device)
            hp.step_bwd(lz.delta, x=lz.x, idx=lz.idx, flags=_lib.STEP_APPLY_ONLY, prepare=(nix, next_idx))
            self._spare[hp.B], hp.indexer = hp.indexer, nix  # the next forward reads the prepared one
        else:
            hp.step_bwd(lz.delta, x=lz.x, idx=lz.idx, flags=_lib.STEP_APPLY_ONLY)
        self._pending = None  # (only once the apply launch was queued: a failed call keeps it pending)

    def check_index_base(self, index_base, op):
        """A caller-passed index base must be the tables' own (None: the tables')."""
        if index_base is not None and int(index_base) != self.index_base:
            raise ValueError(f"{op}: index_base={index_base}, but these HipTables were built with "
                             f"index_base={self.index_base}")

    def __len__(self):
        return len(self._ts)

    def __iter__(self):
        return iter(self.ts)

    def __getitem__(self, i):
        return self.ts[i]

    @property
    def D(self):
        return self._ts.D

    def hotpath(self, batch):
        """The preallocated step state of one batch size (buffers, indexer)."""
        from .hotpath import HotPath
        hp = self._hp.get(batch)
        if hp is None:
            hp = HotPath(self._ts, batch, 1, lr=0.0 if self.lr is None else self.lr, index_base=self.index_base)
            if not hp.step_api:
                raise ValueError("HipTables: this table set has no training-step kernels (deterministic, one-hot)")
            self._hp[batch] = hp
        return hp


class LazyLookup:
    """maplookup(PreallocationStrategy(P), ::HipTables, sparse) before anything is gathered."""

    def __init__(self, tables, idx, prealloc, check_bounds=True):
        self.tables, self.idx, self.prealloc = tables, idx, int(prealloc)
        self.check_bounds = bool(check_bounds)  # materialize()'s default

    @property
    def shape(self):
        return (self.idx.B, self.prealloc + self.tables.D * len(self.tables))

    @property
    def dtype(self):
        return self.tables._ts.dtype

    @property
    def device(self):
        return self.tables._ts.device

    def materialize(self, check_bounds=None):
        """The ys the reference's maplookup returns (one dlrm_maplookup launch)."""
        from .embedding import maplookup
        cb = self.check_bounds if check_bounds is None else check_bounds
        return maplookup(PreallocationStrategy(self.prealloc), self.tables.ts, self.idx,
                         index_base=self.tables.index_base, check_bounds=cb)

    # -- the interaction on it: dlrm_step_fwd
    def interact(self, x):
        if x.shape[1] != self.prealloc:
            raise ValueError(f"the interaction's x has {x.shape[1]} columns, maplookup reserved {self.prealloc}")
        # an update! deferred after this lookup was made (out of the train! order) runs first: the
        # forward must read the updated tables, and it rebuilds the indexer that update reads
        self.tables.flush()
        hp = self.tables.hotpath(self.idx.B)
        hp.validate(x, self.idx)
        hp.step_fwd(x, self.idx)
        return hp


class LazyGrad:
    """The cotangent of a LazyLookup: the step backward's dt ([B][F*D] fp32, x rows first) and
    whether the once-hit rows were already stepped (then only the repeated rows' dt rows exist)."""

    def __init__(self, hp, idx, x, delta, applied_once_hit):
        self.hp, self.idx, self.x, self.delta, self.applied = hp, idx, x, delta, applied_once_hit

    @property
    def dt(self):
        return self.hp.dt


class DeferredUpdate(SparseEmbeddingUpdate):
    """One table's SparseEmbeddingUpdate from a LazyGrad: a view of dt like maplookup_pullback's,
    plus the step state update! finishes."""

    def __init__(self, lazy, table_index, prealloc):
        hp = lazy.hp
        super().__init__(hp.dt, prealloc + table_index * hp.D, hp.D, lazy.idx, table_index)
        self.lazy = lazy

    def uncompress(self, nrows, *, index_base=1):
        if self.lazy.applied:
            raise ValueError("the pullback stepped the once-hit rows itself (HipTables(lr=...)): dt holds only the "
                             "repeated rows; build HipTables without lr to read the full gradient")
        return super().uncompress(nrows, index_base=index_base)


def maplookup_lazy(strategy, tables, sparse, check_bounds=True):
    """(Bounds of a LazyLookup's indices are raised by the fused forward's flag: at update_ with
    check_bounds, or at the next check_bounds.)"""
    idx = PackedIndices(sparse, device=tables._ts.device)
    if idx.T != len(tables):
        raise ValueError(f"{idx.T} index arrays for {len(tables)} tables")
    if isinstance(strategy, PreallocationStrategy) and idx.L == 1:
        tables.poll_bounds()  # a deferred step's BoundsError, from the flag snapshot (no GPU call)
        tables.flush(next_idx=idx)  # a deferred update's apply, with this batch's indexer build
        return LazyLookup(tables, idx, strategy.prealloc, check_bounds)
    # pooled bags / DefaultStrategy: the plain operator (no fused step form)
    from .embedding import maplookup
    return maplookup(strategy, tables.ts, idx, index_base=tables.index_base, check_bounds=check_bounds)


def rrule_lazy(x, ys):
    """rrule(::DotInteraction, x, ::LazyLookup) -> (out, pullback)."""
    hp = ys.interact(x)
    tables, idx = ys.tables, ys.idx

    def dot_pullback(delta):
        if tables.lr is not None:  # once-hit rows stepped here (w = fmaf(-η, g, w)), the rest left in dt
            # (a second pullback on this forward is refused by the library: it would step them twice)
            hp.step_bwd(delta, x=x, idx=idx, flags=_lib.STEP_BWD_ONLY)
        else:                      # every dt row written; update! steps every row
            hp.interact_bwd(delta, x=x, idx=idx)
        # applied: the split backward ran (a shape without it writes every dt row, as above)
        applied = bool(hp.indexer.state() & _lib.IX_SINGLES_DONE)
        return None, hp.dx, LazyGrad(hp, idx, x, delta, applied)

    return hp.out, dot_pullback


def pullback_lazy(strategy_prealloc, tables, dy):
    if dy.hp is not tables.hotpath(dy.idx.B):
        raise ValueError("the gradient belongs to another table set")
    return [DeferredUpdate(dy, t, strategy_prealloc) for t in range(len(tables))]


def update_lazy(opt, tables, grads, *, check_bounds=None):
    """update!(Descent(η), ::HipTables, grads): the apply launch of the step.  check_bounds: None
    (the reference's call): the tables' policy -- deferred apply + flag snapshot when they defer,
    else the launch and a synchronising check; True: run it now and check; False: no check."""
    if not isinstance(opt, Descent):
        raise TypeError("update_ implements Descent (plain SGD), the optimizer DLRM.jl trains with")
    lz = grads[0].lazy
    if len(grads) != len(tables) or any(g.lazy is not lz or g.table_index != t for t, g in enumerate(grads)):
        raise ValueError("update_ expects the per-table views of one maplookup pullback")
    hp = lz.hp
    tables.flush()
    if lz.applied:
        if opt.eta != tables.lr:
            raise ValueError(f"the pullback stepped the once-hit rows with η = {tables.lr}; update! got {opt.eta}")
        if tables.defer_update and not check_bounds:
            tables._pending = lz  # applied by the next maplookup's launch (or any read of the tables)
            # (the step backward that ran in the pullback already copied the bounds flag as of this
            # step's forward into host memory, for poll_bounds: no launch, no synchronisation here)
            tables._unchecked = tables._unchecked or check_bounds is None
            return tables
        hp.step_bwd(lz.delta, x=lz.x, idx=lz.idx, flags=_lib.STEP_APPLY_ONLY)
    else:
        hp.lr = opt.eta
        hp.sgd_update(lz.idx, prebuilt=True)  # the forward's split indexer: once-hit rows as singles items
    if check_bounds or check_bounds is None:
        tables._unchecked = False
        hp.check_bounds()
    return tables
