"""The hot path as one preallocated training-step engine.

One `HotPath.step(x, indices, dout)` = what DLRM.jl's train! loop (src/train/train.jl:215-227)
does for the sparse half of the model on one batch:

    ys  = maplookup(PreallocationStrategy(d), tables, sparse)      model.jl:161
    out = interaction(x, ys)                                       model.jl:163
    (top MLP + loss produce dout = dLoss/dout: out of scope, supplied by the caller)
    dx, dt = dot_back(dot, dout, T, d, padding)                    interact.jl:442-445
    update!(Descent(lr), tables, maplookup_pullback(dt), indexers) train.jl:283-290

All buffers are allocated once; a step issues 3 kernel launches on the current stream
(default: dlrm_step_fwd = lookup + interaction + indexer sort; dlrm_step_bwd = interaction
bwd with the SGD step of once-hit rows, then the apply of repeated rows) with no host
synchronisation, so the whole step can be captured in a torch.cuda graph (`fused=False`
runs maplookup and the interaction as two launches, like the reference).  With
`overlap_indexer=True` (the default where ys is kept and the indexer is the hash build,
B*L > 4096) the indexer (which depends only on the indices) runs on a side stream
concurrently with the lookup and the interaction.

`materialize_ys` (default: off wherever it applies, i.e. fused forward and one-hot lookups):
the reference keeps the lookup output ys (= the interaction's T) for dot_back.  Off, the
forward writes only `out` and the backward rebuilds T from x and the gathered table rows
(dlrm_interact_bwd_gather) -- the same values, bit for bit, since the tables change only in
the update that follows -- which saves ys's write and keeps the step's HBM traffic at what
the math needs.  Turn it on to read `ys` (e.g. for parity checks against maplookup).
"""
import torch

from . import _lib
from .embedding import EmbeddingTableSet, PackedIndices
from .interact import interaction_sizes
from .runtime import dtype_code, ptr, require_device
from .shapes import APPLY_MAX_N
from .update import SparseIndexer


class HotPath:
    def __init__(self, tables, batch, lookups=1, *, lr=0.1, index_base=0, deterministic=True,
                 overlap_indexer=None, pad_to=1, fused=True, materialize_ys=None, pipeline=False, chunk=None,
                 parts=None):
        self.ts = tables if isinstance(tables, EmbeddingTableSet) else EmbeddingTableSet(tables)
        self.B, self.L = int(batch), int(lookups)
        self.T, self.D = len(self.ts), self.ts.D
        self.d = self.D  # dense vector length == feature size (model.jl:220)
        self.F = self.T + 1
        self.lr = float(lr)
        self.index_base = int(index_base)
        self.deterministic = deterministic
        self.fused = fused
        _, self.width, self.padding = interaction_sizes(self.d, self.F, pad_to)
        dev, dt = self.ts.device, self.ts.dtype
        can_skip = fused and self.L == 1
        if materialize_ys is None:
            materialize_ys = not can_skip
        if not materialize_ys and not can_skip:
            raise ValueError("materialize_ys=False needs the fused forward and one-hot lookups (lookups=1)")
        self.materialize_ys = bool(materialize_ys)
        self.ys = torch.empty((self.B, self.F * self.D), dtype=dt, device=dev) if self.materialize_ys else None
        self._fwd_x = self._fwd_idx = None
        self.out = torch.empty((self.B, self.width), dtype=dt, device=dev)
        self.dx = torch.empty((self.B, self.d), dtype=torch.float32, device=dev)
        self.dt = torch.empty((self.B, self.F * self.d), dtype=torch.float32, device=dev)
        self.indexer = SparseIndexer(self.T, self.B * self.L, dev) if deterministic else None
        # the wave build's chunk limit (None: the library's 32; shapes.step_chunk picks per workload)
        self.chunk = chunk
        if chunk is not None and self.indexer is not None:
            self.indexer.set_chunk(chunk)
        # parts per table of the wave builds of <= 2048 positions (None: the library's 16;
        # shapes.step_parts picks per workload)
        self.parts = parts
        if parts is not None and self.indexer is not None:
            self.indexer.set_parts(parts)
        self.ctx = self.ts.ctx
        self.lib = self.ctx.lib
        self.dcode = dtype_code(dt)
        if overlap_indexer is None:
            # default: a hash-built indexer (B*L > 4096 positions per table) of the operator path
            # runs on a side stream beside the forward (the step API forks it inside dlrm_step_fwd)
            overlap_indexer = self.materialize_ys and self.B * self.L > 4096
        self.overlap_indexer = bool(overlap_indexer) and deterministic
        self._side = torch.cuda.Stream(device=dev) if self.overlap_indexer else None
        self._indexer_done = None
        # the training-step pair (dlrm_step_fwd / dlrm_step_bwd): indexer built inside the forward's
        # launch, once-hit rows updated inside the backward's, the rest by the apply launch
        self.step_api = (not self.materialize_ys) and self.indexer is not None and not self.overlap_indexer
        # pipelined steps: the NEXT batch's split indexer is built during this step, so the
        # step's forward launch only gathers; two indexers alternate.
        #   "apply" (`step_prep`): by extra workgroups of this step's apply launch
        #           (dlrm_step_bwd_prepare) -- the indexer's latency hides behind the apply's;
        #   "side"  (`step_next`): by its own launch on a side stream (measured slower: a replayed
        #           hipGraph runs the branch concurrently, but it slows the kernels beside it and each
        #           step pays two cross-queue hops of ~3.7 us: DESIGN.md §6).
        mode = {False: None, 0: None, None: None, True: "side", 1: "side", 2: "apply"}.get(pipeline, pipeline)
        if mode not in (None, "side", "apply"):
            raise ValueError(f"pipeline must be None, 'side' or 'apply', not {pipeline!r}")
        # (pooled bags: "side" only -- the next batch's build beside this step's apply, `step_next`)
        self.pipeline = mode if (mode and ((self.step_api and self.L == 1) or (mode == "side" and self.L > 1))) else None
        self._prepare_ok = None  # build_split: None untried, False the wave build does not take it
        if self.pipeline:
            self._ixs = [self.indexer, SparseIndexer(self.T, self.B * self.L, dev)]
            if chunk is not None:
                self._ixs[1].set_chunk(chunk)
            if parts is not None:
                self._ixs[1].set_parts(parts)
            if self.pipeline == "apply" and self.B > 2048:  # (the in-apply wave build's parts, before any capture)
                for ix in self._ixs:
                    ix.reserve(self.B)
            self._ix_of = [None, None]  # the PackedIndices each indexer was last built from
            self._cur = 0
            self._pside = torch.cuda.Stream(device=dev)
            self._pev = torch.cuda.Event()

    # -- pieces --------------------------------------------------------------------------
    def _check(self, rc):
        if rc != _lib.OK:
            self.ctx.check(rc)

    def lookup(self, idx):
        h = self.ctx.bind()
        self._check(self.lib.dlrm_maplookup(h, self.ts.handle, ptr(idx.data), idx.itype, idx.stride, self.index_base,
                                            self.B, self.L, ptr(self.ys), self.ys.stride(0), self.d))

    def interact_fwd(self, x):
        h = self.ctx.bind()
        self._check(self.lib.dlrm_interact_fwd(h, self.dcode, self.d, self.F, self.B, ptr(x), x.stride(0),
                                               ptr(self.ys), self.ys.stride(0), ptr(self.out), self.out.stride(0),
                                               self.padding))

    def lookup_interact_fwd(self, x, idx):
        h = self.ctx.bind()
        ys, ys_ld = (ptr(self.ys), self.ys.stride(0)) if self.materialize_ys else (None, 0)
        self._check(self.lib.dlrm_lookup_interact_fwd(h, self.ts.handle, ptr(idx.data), idx.itype, idx.stride,
                                                      self.index_base, self.B, self.L, ptr(x), x.stride(0), ys,
                                                      ys_ld, ptr(self.out), self.out.stride(0), self.padding))
        self._fwd_x, self._fwd_idx = x, idx

    def build_indexer(self, idx):
        h = self.ctx.bind()
        self._check(self.lib.dlrm_indexer_build(h, self.indexer.handle, self.ts.handle, ptr(idx.data), idx.itype,
                                                idx.stride, self.index_base, self.B, self.L))

    def interact_bwd(self, dout, x=None, idx=None, build_indexer=False):
        """dot_back.  Without a materialized ys, T is rebuilt from x and the indices of the
        forward (the last forward's unless given); build_indexer: the same launch also builds
        the update's indexer from those indices."""
        h = self.ctx.bind()
        if self.materialize_ys:
            self._check(self.lib.dlrm_interact_bwd(h, self.dcode, self.d, self.F, self.B, ptr(dout), dout.stride(0),
                                                   self.padding, ptr(self.ys), self.ys.stride(0), ptr(self.dx),
                                                   self.dx.stride(0), ptr(self.dt), self.dt.stride(0)))
            return
        x = self._fwd_x if x is None else x
        idx = self._fwd_idx if idx is None else idx
        if x is None or idx is None:
            raise RuntimeError("interact_bwd without a materialized ys needs the forward's x and indices")
        ixh = self.indexer.handle if (build_indexer and self.indexer is not None) else None
        self._check(self.lib.dlrm_interact_bwd_gather(h, self.ts.handle, ixh, ptr(idx.data), idx.itype, idx.stride,
                                                      self.index_base, self.B, self.L, ptr(x), x.stride(0),
                                                      ptr(dout), dout.stride(0), self.padding, ptr(self.dx),
                                                      self.dx.stride(0), ptr(self.dt), self.dt.stride(0)))

    def sgd_update(self, idx, prebuilt):
        h = self.ctx.bind()
        flags = 0 if self.deterministic else _lib.UPDATE_ATOMIC
        if prebuilt:
            flags |= _lib.UPDATE_PREBUILT
        self._check(self.lib.dlrm_sgd_update(h, self.ts.handle, self.indexer.handle if self.indexer else None, flags,
                                             ptr(idx.data), idx.itype, idx.stride, self.index_base, self.B, self.L,
                                             ptr(self.dt), _lib.F32, self.dt.stride(0), self.d, self.lr))

    def step_fwd(self, x, idx):
        """dlrm_step_fwd: lookup + interaction (no ys) + the split indexer, one launch."""
        h = self.ctx.bind()
        self._check(self.lib.dlrm_step_fwd(h, self.ts.handle, self.indexer.handle, ptr(idx.data), idx.itype,
                                           idx.stride, self.index_base, self.B, ptr(x), x.stride(0), ptr(self.out),
                                           self.out.stride(0), self.padding))
        self._fwd_x, self._fwd_idx = x, idx

    def step_bwd(self, dout, x=None, idx=None, flags=0, prepare=None):
        """dlrm_step_bwd: dot_back + update!(Descent(lr)) with the indexer of step_fwd
        (flags: _lib.STEP_BWD_ONLY / STEP_APPLY_ONLY run one of its two launches)."""
        h = self.ctx.bind()
        x = self._fwd_x if x is None else x
        idx = self._fwd_idx if idx is None else idx
        if prepare is not None:  # (next indexer, next indices): built by this step's apply launch
            nix, nidx = prepare
            if (nidx.itype, nidx.stride, nidx.B, nidx.L) != (idx.itype, idx.stride, idx.B, idx.L):
                raise ValueError("the next batch's indices must have this batch's layout")
            self._check(self.lib.dlrm_step_bwd_prepare(h, self.ts.handle, self.indexer.handle, ptr(idx.data),
                                                       idx.itype, idx.stride, self.index_base, self.B, ptr(x),
                                                       x.stride(0), ptr(dout), dout.stride(0), self.padding,
                                                       ptr(self.dx), self.dx.stride(0), ptr(self.dt),
                                                       self.dt.stride(0), self.lr, nix.handle, ptr(nidx.data), flags))
            return
        self._check(self.lib.dlrm_step_bwd(h, self.ts.handle, self.indexer.handle, ptr(idx.data), idx.itype,
                                           idx.stride, self.index_base, self.B, ptr(x), x.stride(0), ptr(dout),
                                           dout.stride(0), self.padding, ptr(self.dx), self.dx.stride(0),
                                           ptr(self.dt), self.dt.stride(0), self.lr, flags))

    def build_split(self, indexer, idx):
        """The indexer form dlrm_step_bwd consumes: the wave build (dlrm_indexer_prepare) for one-hot
        batches of <= shapes.APPLY_MAX_N positions per table, else dlrm_indexer_build_split (the
        in-LDS parts build up to 8192 positions, the hash build above: beside a step of B = 8192 the
        parts build's 104 workgroups cost the step less than the wave build's 416)."""
        h = self.ctx.bind()
        if idx.L == 1 and self.B <= APPLY_MAX_N and self._prepare_ok is not False:
            rc = self.lib.dlrm_indexer_prepare(h, indexer.handle, self.ts.handle, ptr(idx.data), idx.itype,
                                               idx.stride, self.index_base, self.B)
            if rc == _lib.OK:
                self._prepare_ok = True
                return
            if rc != _lib.E_UNSUPPORTED:
                self._check(rc)
            self._prepare_ok = False
        self._check(self.lib.dlrm_indexer_build_split(h, indexer.handle, self.ts.handle, ptr(idx.data), idx.itype,
                                                      idx.stride, self.index_base, self.B))

    def prime(self, idx, x=None, dout=None, prev=None):
        """Readies the indexer of the batch the next `step_next` / `step_prep` call will process:
        "side": builds it; "apply": runs one pipelined step of batch `prev` (x, dout) that
        prepares `idx` in indexer 0, so the next `step_prep` starts from indexer 0."""
        if self.pipeline == "apply":
            self._cur, self._ix_of = 1, [None, None]
            self.step_prep(x, prev, dout, idx)
            return
        if self.L > 1:  # pooled bags: dlrm_indexer_build (the bag build)
            home, self.indexer = self.indexer, self._ixs[self._cur]
            self.build_indexer(idx)
            self.indexer = home
        else:
            self.build_split(self._ixs[self._cur], idx)
        self._ix_of[self._cur] = idx

    def step_prep(self, x, idx, dout, next_idx):
        """One training step of batch `idx` (same math as `step`, bit for bit) whose apply launch
        also builds batch `next_idx`'s split indexer (dlrm_step_bwd_prepare): when `idx` was
        prepared by the previous call, this step's forward launch only gathers."""
        cur, nxt = self._cur, 1 - self._cur
        self.indexer = self._ixs[cur]
        self.step_fwd(x, idx)  # gather-only when this indexer holds idx, prepared (the library checks)
        self.step_bwd(dout, x=x, idx=idx, prepare=(self._ixs[nxt], next_idx))
        self._ix_of[nxt] = next_idx
        self._cur = nxt
        return self.dx

    def step_next(self, x, idx, dout, next_idx):
        """One training step of batch `idx` (same math as `step`, bit for bit) that also builds
        batch `next_idx`'s indexer on a side stream: exactly one indexer build per step, off the
        step's critical path (it depends only on the indices).  The side stream first waits for
        everything queued so far (the previous step's apply read the buffer it rebuilds) and is
        joined at the end of the step."""
        cur, nxt = self._cur, 1 - self._cur
        if self._ix_of[cur] is not idx:  # out of sequence (first call, or a different batch)
            self.prime(idx)
        main = torch.cuda.current_stream(self.ts.device)
        if self.L > 1:
            return self._step_bags_next(main, x, idx, dout, next_idx, cur, nxt)
        self._pside.wait_stream(main)
        with torch.cuda.stream(self._pside):
            self.build_split(self._ixs[nxt], next_idx)
            self._pev.record(self._pside)
        self._ix_of[nxt] = next_idx
        self.lookup_interact_fwd(x, idx)  # ys not materialized: the fused forward alone
        self.indexer = self._ixs[cur]
        self.step_bwd(dout, x=x, idx=idx)
        main.wait_event(self._pev)
        self._cur = nxt
        return self.dx

    def _step_bags_next(self, main, x, idx, dout, next_idx, cur, nxt):
        """step_next for pooled bags (configs[4]): forward and backward on the main stream, then the
        apply of batch `idx` with its prebuilt indexer while batch `next_idx`'s bag build runs on the
        side stream beside it, forked when the backward is queued and joined at the end of the step.
        The apply (hundreds of us of latency-bound items) hides the build; beside the gather-heavy
        forward (the unpipelined form) the build's kernels and the forward's slowed each other and
        the step paid the build's length."""
        if self.fused:  # (not self.forward: that forks this batch's own build)
            self.lookup_interact_fwd(x, idx)
        else:
            self.lookup(idx)
            self.interact_fwd(x)
        self.interact_bwd(dout, x=x, idx=idx)
        self._pside.wait_stream(main)  # (also: the apply that last read indexer nxt is done)
        with torch.cuda.stream(self._pside):
            home, self.indexer = self.indexer, self._ixs[nxt]
            self.build_indexer(next_idx)
            self.indexer = home
            self._pev.record(self._pside)
        self._ix_of[nxt] = next_idx
        home, self.indexer = self.indexer, self._ixs[cur]
        self.sgd_update(idx, True)
        self.indexer = home
        main.wait_event(self._pev)
        self._cur = nxt
        return self.dx

    # -- step --------------------------------------------------------------------------
    def validate(self, x, idx, dout=None):
        """Host-side shape/device checks (call once per new buffer set; the step itself does not)."""
        dev = self.ts.device
        require_device(x, dev, "x")
        require_device(idx.data, dev, "indices")
        if x.shape != (self.B, self.d) or x.dtype != self.ts.dtype or x.stride(1) != 1:
            raise ValueError(f"x must be [{self.B}][{self.d}] {self.ts.dtype}")
        if (idx.T, idx.B, idx.L) != (self.T, self.B, self.L):
            raise ValueError("indices do not match the engine's (tables, batch, lookups)")
        if dout is not None:
            require_device(dout, dev, "dout")
            if dout.shape != (self.B, self.width) or dout.dtype != self.ts.dtype or dout.stride(1) != 1:
                raise ValueError(f"dout must be [{self.B}][{self.width}] {self.ts.dtype}")

    def forward(self, x, idx):
        if self.step_api:
            self.step_fwd(x, idx)
            return self.out
        if self.overlap_indexer:
            main = torch.cuda.current_stream(self.ts.device)
            self._side.wait_stream(main)
            with torch.cuda.stream(self._side):
                self.build_indexer(idx)
                self._indexer_done = torch.cuda.Event()
                self._indexer_done.record(self._side)
        if self.fused:
            self.lookup_interact_fwd(x, idx)
        else:
            self.lookup(idx)
            self.interact_fwd(x)
        return self.out

    def backward(self, idx, dout):
        if self.step_api:
            self.step_bwd(dout, idx=idx)
            return self.dx
        # without ys (and deterministic), the indexer is built inside the backward's launch
        in_bwd = not self.materialize_ys and self.indexer is not None and not self.overlap_indexer
        self.interact_bwd(dout, idx=idx, build_indexer=in_bwd)
        prebuilt = in_bwd
        if self.overlap_indexer and self._indexer_done is not None:
            torch.cuda.current_stream(self.ts.device).wait_event(self._indexer_done)
            prebuilt = True
        self.sgd_update(idx, prebuilt)
        return self.dx

    def step(self, x, idx, dout):
        self.forward(x, idx)
        return self.backward(idx, dout)

    def check_bounds(self):
        self.ctx.check_bounds()


def packed(indices_tensor):
    """[T][B] or [T][B][L] int32/int64 device tensor -> PackedIndices (no copy)."""
    return PackedIndices(indices_tensor)
