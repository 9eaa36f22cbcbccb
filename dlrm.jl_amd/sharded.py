"""Table-sharded (model-parallel) hot path across the GPUs of one node.

The reference has no distributed code; this is the MI355X extension the
north star asks for: embedding tables shard BY TABLE across ranks, and one all-to-all each
way moves the looked-up vectors to the ranks that own the samples, and their gradients back.

  rank r owns the tables tables(r) (a TablePartition) and B samples of the global batch
  Bg = world * B (weak scaling: B per GPU fixed; strong scaling: Bg fixed, B = Bg / world).
  The step runs as M micro-batches of Bm = B / M samples per rank, so the all-to-all of one
  micro-batch overlaps the compute of the next on a second stream.  Micro-batch m of the global
  batch is its samples [m*world*Bm, (m+1)*world*Bm), in rank order: rank r's local sample b is
  global sample  global_index(r, b) = (b // Bm) * world * Bm + r * Bm + b % Bm
  (M = 1: r * B + b), so each micro-batch's index columns, exchange blocks and gradient rows are
  contiguous, and the update sees the global batch in global order.

  forward : maplookup of r's T_r tables for all Bg samples, written straight into the
            exchange layout (dlrm_maplookup_blocked)        -> send [world][T_r][B][D]
            all-to-all (block j -> rank j)                  -> recv = [src j][T_j][B][D]
            every table's B vectors for r's samples are now one contiguous [B][D] block of
            recv, i.e. a B-row table whose row b is sample b: the fused lookup+interaction
            kernel runs on these T "received tables" with identity indices (no ys copy)
  backward: dot_back re-gathers T from the received tables and stores each table's gradient
            rows straight into the send layout (dlrm_interact_bwd_blocked; other ops: dt
            [B][F*D], then dlrm_scatter_rows)                -> gsend [dst j][B][T_j][D]
            all-to-all                                      -> grecv [src i][B][T_r][D]
                                                               = grad [Bg][T_r*D]
            update!(Descent) of r's tables with r's indices for all Bg samples; the
            SparseIndexer (positions grouped by row: a hash build over the whole chip for
            Bg*L > 4096) depends on the indices only and is built on a side stream while
            the forward runs

Per rank and step: lookup(m) for every m on the compute stream; exchange_fwd(m) on the comm stream
as soon as lookup(m) is done; interaction fwd + bwd of m once its vectors arrived; exchange_bwd(m) on
the comm stream; the update when the last gradient block arrived.  Exposed: the first forward and
the last backward exchange (1/M of each direction) -- DESIGN.md §6.  M = 1 (the default): lookup,
exchange, interaction, exchange and update in stream order on the compute stream, the index build
alone on the side stream.

All compute goes through a `ShardOps` object: `HipShardOps` (the product: the C-ABI kernels)
or, in the CPU gloo tests, a test-only CPU checker.  torch.distributed (backend "nccl"
= RCCL over xGMI on MI355X) carries the two all-to-alls (uneven table counts per rank: the
split-size form of all_to_all_single), or, with exchange="abi", the library's own RCCL
communicator (dlrm_alltoall_fwd / _bwd, dlrm.jl_amd/comm.py).  The bench replays each whole step,
collectives included, as one hipGraph (`capture_full`, `--shard-graph full`, the default); where the
backend's collectives cannot be captured (gloo), the compute between them (`capture`) with the
collectives launched eagerly.  A graph holding RCCL work keeps a reference on its communicator, so
`close()` (graphs first, then the communicator) must run before the communicator is destroyed.
"""
import os

import torch
import torch.distributed as dist

from . import _lib
from .embedding import EmbeddingTableSet, PackedIndices
from .interact import interaction_sizes
from .runtime import context, dtype_code, ptr
from .shapes import PREPARE_MAX_N, zipf_perm, zipf_rows
from .update import SparseIndexer


class TablePartition:
    """Assignment of T tables to `world` ranks.

    Default: contiguous, count-balanced blocks (every table costs Bg*L lookups per step
    whatever its size, so equal counts balance the gather, the exchange and the update).
    `TablePartition.fitting(rows, world, row_bytes, capacity)` keeps that when every block
    fits in `capacity` bytes and otherwise assigns tables largest-first to the rank with the
    fewest bytes (ties: fewest tables) -- e.g. Criteo-Terabyte fp32 on 2 GPUs, whose
    contiguous halves are 185 and 267 GB (criteo.jl:379-406)."""

    def __init__(self, T, world, owners=None):
        self.T, self.world = T, world
        if owners is None:
            base, extra = divmod(T, world)
            counts = [base + (1 if r < extra else 0) for r in range(world)]
            starts = [sum(counts[:r]) for r in range(world)]
            owners = [list(range(starts[r], starts[r] + counts[r])) for r in range(world)]
        if sorted(t for o in owners for t in o) != list(range(T)) or len(owners) != world:
            raise ValueError("every table must be owned by exactly one rank")
        self.owners = [list(o) for o in owners]
        self.counts = [len(o) for o in self.owners]
        self.order = [t for o in self.owners for t in o]  # tables in exchange-block order
        self.contiguous = self.order == list(range(T)) and all(
            o == list(range(o[0], o[0] + len(o))) for o in self.owners if o)

    @classmethod
    def fitting(cls, rows, world, row_bytes, capacity):
        p = cls(len(rows), world)
        if max(sum(rows[t] for t in o) * row_bytes for o in p.owners) <= capacity:
            return p
        load = [0] * world
        owners = [[] for _ in range(world)]
        for t in sorted(range(len(rows)), key=lambda t: -rows[t]):
            r = min(range(world), key=lambda r: (load[r], len(owners[r])))
            owners[r].append(t)
            load[r] += rows[t]
        if max(load) * row_bytes > capacity:
            raise ValueError(f"no table partition over {world} ranks fits {capacity} bytes per rank: the greedy "
                             f"assignment needs {[l * row_bytes for l in load]} bytes per rank")
        return cls(len(rows), world, [sorted(o) for o in owners])

    def tables(self, r):
        return self.owners[r]

    def range(self, r):
        """[t0, t1) of rank r (contiguous partitions only)."""
        if not self.contiguous:
            raise ValueError("range(): this partition is not contiguous; use tables(r)")
        o = self.owners[r]
        return (o[0], o[0] + len(o)) if o else (sum(self.counts[:r]), sum(self.counts[:r]))

    def bytes_per_rank(self, rows, row_bytes):
        return [sum(rows[t] for t in o) * row_bytes for o in self.owners]


class HipShardOps:
    """The product ops: the HIP kernels behind include/dlrm_hip.h (no host syncs)."""

    def __init__(self, tables, batch_global, lookups, lr, index_base=0, device=None):
        tables = list(tables)
        self.ts = EmbeddingTableSet(tables) if tables else None
        self.device = self.ts.device if self.ts else torch.device(device)
        self.ctx = self.ts.ctx if self.ts else context(self.device)
        self.lib = self.ctx.lib
        self.Bg, self.L, self.lr, self.base = batch_global, lookups, lr, index_base
        self.indexer = SparseIndexer(len(tables), batch_global * lookups, self.device) if tables else None
        if self.indexer is not None and lookups == 1 and batch_global <= PREPARE_MAX_N:
            self.indexer.reserve(batch_global)  # (the wave build's parts layout, before any capture)
        self.rts = self.ident = None
        self._prepare = None  # None: not tried yet; False: the wave build does not take this shape

    def _ok(self, rc):
        if rc != _lib.OK:
            self.ctx.check(rc)

    def bind_recv(self, tabs_per_mb):
        """tabs_per_mb[m]: micro-batch m's T received [Bm][D] blocks in global table order (views of
        its receive buffer); each block is a Bm-row table read in place with identity indices."""
        self.rts = [EmbeddingTableSet(tabs) for tabs in tabs_per_mb]
        T, Bm = len(tabs_per_mb[0]), tabs_per_mb[0][0].shape[0]
        ar = torch.arange(Bm, dtype=torch.int32, device=self.device)
        self.ident = PackedIndices(ar.repeat(T, 1).reshape(T, Bm, 1))

    def build_indexer(self, idx):
        """The update's split indexer over the global batch: the wave build (dlrm_indexer_prepare:
        16 parts per 2048 positions per table, one wave each; above 2048 positions the scan build,
        csrc/indexer.hpp wave_build_group_scan) for one-hot global batches of <= shapes.PREPARE_MAX_N
        positions per table (world 8 at the metric config, 16384: 13.4 us against the hash build's
        40 us; configs[3] at global batch 2048: 11 us against the in-LDS build's 22 us), else
        dlrm_indexer_build (in-LDS or hash build)."""
        if idx.L == 1 and idx.B <= PREPARE_MAX_N and self._prepare is not False:
            rc = self.lib.dlrm_indexer_prepare(self.ctx.bind(), self.indexer.handle, self.ts.handle, ptr(idx.data),
                                               idx.itype, idx.stride, self.base, idx.B)
            if rc == _lib.OK:
                self._prepare = True
                return
            if rc != _lib.E_UNSUPPORTED:
                self.ctx.check(rc)
            self._prepare = False
        self._ok(self.lib.dlrm_indexer_build(self.ctx.bind(), self.indexer.handle, self.ts.handle, ptr(idx.data),
                                             idx.itype, idx.stride, self.base, idx.B, idx.L))

    def lookup_blocked(self, idx, out, ld, tstride, brows, bstride):
        self._ok(self.lib.dlrm_maplookup_blocked(self.ctx.bind(), self.ts.handle, ptr(idx.data), idx.itype,
                                                 idx.stride, self.base, idx.B, idx.L, ptr(out), ld, 0, tstride, brows,
                                                 bstride))

    def scatter_rows(self, src, src_ld, src_off, dst, dbase, dld, T, B, D):
        self._ok(self.lib.dlrm_scatter_rows(self.ctx.bind(), src.element_size(), T, B, D, ptr(src), src_ld, src_off,
                                            ptr(dst), ptr(dbase), ptr(dld)))

    def interact_fwd_recv(self, x, out, padding, m=0):
        i = self.ident
        self._ok(self.lib.dlrm_lookup_interact_fwd(self.ctx.bind(), self.rts[m].handle, ptr(i.data), i.itype,
                                                   i.stride, 0, i.B, 1, ptr(x), x.stride(0), None, 0, ptr(out),
                                                   out.stride(0), padding))

    def interact_bwd_recv(self, dout, x, dx, dt, padding, m=0):
        i = self.ident
        self._ok(self.lib.dlrm_interact_bwd_gather(self.ctx.bind(), self.rts[m].handle, None, ptr(i.data), i.itype,
                                                   i.stride, 0, i.B, 1, ptr(x), x.stride(0), ptr(dout),
                                                   dout.stride(0), padding, ptr(dx), dx.stride(0), ptr(dt),
                                                   dt.stride(0)))

    def interact_bwd_send(self, dout, x, dx, gsend, dbase, dld, padding, m=0):
        """dot_back on micro-batch m's received tables with every table's dt rows stored straight
        into the exchange's send layout (one launch: dlrm_interact_bwd_blocked).  False: shape not
        supported by the fused kernel (the caller repacks dt instead)."""
        i = self.ident
        rc = self.lib.dlrm_interact_bwd_blocked(self.ctx.bind(), self.rts[m].handle, ptr(i.data), i.itype, i.stride,
                                                0, i.B, ptr(x), x.stride(0), ptr(dout), dout.stride(0), padding,
                                                ptr(dx), dx.stride(0), ptr(gsend), ptr(dbase), ptr(dld))
        if rc == _lib.E_UNSUPPORTED:
            return False
        self._ok(rc)
        return True

    def update(self, idx, grad, prebuilt=False):
        flags = _lib.UPDATE_PREBUILT if prebuilt else 0
        self._ok(self.lib.dlrm_sgd_update(self.ctx.bind(), self.ts.handle, self.indexer.handle, flags, ptr(idx.data),
                                          idx.itype, idx.stride, self.base, idx.B, idx.L, ptr(grad),
                                          dtype_code(grad.dtype), grad.stride(0), 0, self.lr))

    def check_bounds(self):
        self.ctx.check_bounds()


class ShardedHotPath:
    """One step of the table-sharded hot path on this rank, as `micro` micro-batches (see the
    module docstring)."""

    def __init__(self, ops, partition, rank, batch_local, dim, lookups, dtype, device, group=None, exchange=None,
                 micro=1):
        self.ops, self.part, self.rank = ops, partition, rank
        self.world = partition.world
        self.B, self.D, self.L = batch_local, dim, lookups
        if micro < 1 or batch_local % micro:
            raise ValueError(f"{micro} micro-batches do not divide {batch_local} samples per rank")
        self.M = micro
        self.Bm = batch_local // micro
        self.Bg = batch_local * self.world
        self.T = partition.T
        self.F = self.T + 1
        self.mine = partition.tables(rank)
        self.Tr = len(self.mine)
        self.group = group
        _, self.width, self.padding = interaction_sizes(dim, self.F)
        dev = device
        D, B, Bm, T, Tr, W, M = dim, batch_local, self.Bm, self.T, self.Tr, self.world, micro
        # per micro-batch exchange buffers (forward: send [peer][T_r][Bm][D] -> recv [src][T_j][Bm][D];
        # backward: gsend [owner][Bm][T_j][D] -> rows [m*W*Bm, (m+1)*W*Bm) of grad [Bg][T_r*D])
        self.send = torch.empty((M, W * Tr * Bm * D), dtype=dtype, device=dev)
        self.recv = torch.empty((M, T * Bm * D), dtype=dtype, device=dev)
        self.out = torch.empty((B, self.width), dtype=dtype, device=dev)
        self.dx = torch.empty((B, D), dtype=torch.float32, device=dev)
        self.dt = None  # [Bm][F*D] fp32, only where the backward cannot store into gsend directly
        self.gsend = torch.empty((M, T * Bm * D), dtype=torch.float32, device=dev)
        self.grecv = torch.empty((W * Tr * B * D,), dtype=torch.float32, device=dev)
        self.grad = self.grecv.view(self.Bg, Tr * D) if Tr else None
        # element counts of each peer's block (flat all_to_all_single splits), per micro-batch
        self.fwd_in_splits = [Tr * Bm * D] * W
        self.fwd_out_splits = [c * Bm * D for c in partition.counts]
        self.bwd_in_splits = self.fwd_out_splits
        self.bwd_out_splits = self.fwd_in_splits
        # received block of global table t: position of t in the exchange order
        slot = {t: i for i, t in enumerate(partition.order)}
        self.recv_tables = [[self.recv[m, slot[t] * Bm * D:(slot[t] + 1) * Bm * D].view(Bm, D) for t in range(T)]
                            for m in range(M)]
        # gsend block of owner j = [Bm][T_j][D]: table t (k-th of its owner) at base + b * T_j * D
        base, ld, off = [0] * T, [0] * T, 0
        for j, tabs in enumerate(partition.owners):
            for k, t in enumerate(tabs):
                base[t], ld[t] = off + k * D, len(tabs) * D
            off += len(tabs) * Bm * D
        self.gs_base = torch.tensor(base, dtype=torch.int64, device=dev)
        self.gs_ld = torch.tensor(ld, dtype=torch.int64, device=dev)
        ops.bind_recv(self.recv_tables)
        # the exchange: torch.distributed (default; backend "nccl" = RCCL) or the library's own RCCL
        # communicator (exchange="abi" / DLRM_EXCHANGE=abi: dlrm_alltoall_fwd / _bwd, as a Julia
        # process per GPU would drive it)
        exchange = exchange or os.environ.get("DLRM_EXCHANGE", "torch")
        self.comm = None
        if exchange == "abi":
            from .comm import CommExchange
            self.comm = CommExchange(rank, self.world, dev, group=group)
        elif exchange != "torch":
            raise ValueError(f"exchange must be 'torch' or 'abi', not {exchange!r}")
        self._graphs = None
        self._full = None  # capture_full: one graph per index batch, collectives inside
        self._fused_bwd = None  # None: not tried yet; False: the ops cannot (repack instead)
        cuda = dev.type == "cuda"
        self._side = torch.cuda.Stream(device=dev) if cuda else None   # the indexer build
        self._cstream = torch.cuda.Stream(device=dev) if cuda else None  # the exchanges
        self._ev = ([[torch.cuda.Event() for _ in range(M)] for _ in range(4)] if cuda else None)
        self._ix_done = torch.cuda.Event() if cuda else None

    def global_index(self, b, rank=None):
        """The global-batch sample of local sample b (this rank, or `rank`)."""
        r = self.rank if rank is None else rank
        return (b // self.Bm) * self.world * self.Bm + r * self.Bm + b % self.Bm

    def rows(self, m):
        return slice(m * self.Bm, (m + 1) * self.Bm)

    # ---- exchange (pure data movement; identical for every ShardOps)
    def _a2a(self, out, inp, out_splits, in_splits):
        if out.is_cuda and dist.get_backend(self.group) == "gloo":
            # gloo has no device all-to-all: stage through host memory (tests / 1-GPU rehearsals;
            # the product backend is "nccl" = RCCL, which moves device memory over xGMI)
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def grad_rows(self, m):
        """Micro-batch m's gradient rows of grad [Bg][T_r*D] (flat)."""
        n = self.world * self.Bm * self.Tr * self.D
        return self.grecv[m * n:(m + 1) * n]

    def exchange_fwd(self, m=0):
        if self.comm is not None:
            self.comm.alltoall_fwd(self.send[m], self.recv[m], self.D, self.Bm, self.part.counts)
            return
        self._a2a(self.recv[m], self.send[m], self.fwd_out_splits, self.fwd_in_splits)

    def pack_grad(self, m=0):
        """dt's table columns -> gsend[m] [owner j][Bm][T_j][D] (one launch)."""
        self.ops.scatter_rows(self.dt, self.F * self.D, self.D, self.gsend[m], self.gs_base, self.gs_ld, self.T,
                              self.Bm, self.D)

    def exchange_bwd(self, m=0):
        if self.comm is not None:
            self.comm.alltoall_bwd(self.gsend[m], self.grad_rows(m), self.D, self.Bm, self.part.counts)
            return
        self._a2a(self.grad_rows(m), self.gsend[m], self.bwd_out_splits, self.bwd_in_splits)

    # ---- the step's compute segments
    def seg_index(self, idx):
        """The update's SparseIndexer (depends on the indices only)."""
        if self.Tr:
            self.ops.build_indexer(idx)

    def seg_lookup(self, idx, m=0):
        """idx: PackedIndices of this rank's tables for the GLOBAL batch ([T_r][Bg*L], global order);
        micro-batch m's columns are gathered into its exchange layout send[m] [world][T_r][Bm][D]."""
        if self.Tr:
            Bm, D, Tr, n = self.Bm, self.D, self.Tr, self.world * self.Bm
            sub = idx if self.M == 1 else PackedIndices.columns(idx, m * n, (m + 1) * n)
            self.ops.lookup_blocked(sub, self.send[m], D, Bm * D, Bm, Tr * Bm * D)

    def seg_interact(self, x, dout, m=0):
        r = self.rows(m)
        self.ops.interact_fwd_recv(x[r], self.out[r], self.padding, m)
        self.interact_bwd(dout, x, m)

    def interact_bwd(self, dout, x, m=0):
        """dot_back of micro-batch m, its table gradients in the exchange layout: one launch where the
        ops offer it (the backward's stores go straight to gsend[m]), else dt + the repack."""
        r = self.rows(m)
        send = getattr(self.ops, "interact_bwd_send", None)
        if send is not None and self._fused_bwd is not False:
            self._fused_bwd = send(dout[r], x[r], self.dx[r], self.gsend[m], self.gs_base, self.gs_ld, self.padding, m)
            if self._fused_bwd:
                return
        if self.dt is None:
            self.dt = torch.empty((self.Bm, self.F * self.D), dtype=torch.float32, device=self.dx.device)
        self.ops.interact_bwd_recv(dout[r], x[r], self.dx[r], self.dt, self.padding, m)
        self.pack_grad(m)

    def seg_update(self, idx):
        if self.Tr:
            self.ops.update(idx, self.grad, prebuilt=True)

    def forward(self, x, idx):
        self.seg_index(idx)
        for m in range(self.M):
            self.seg_lookup(idx, m)
            self.exchange_fwd(m)
            r = self.rows(m)
            self.ops.interact_fwd_recv(x[r], self.out[r], self.padding, m)
        return self.out

    def backward(self, idx, dout, x):
        for m in range(self.M):
            self.interact_bwd(dout, x, m)
            self.exchange_bwd(m)
        self.seg_update(idx)
        return self.dx

    # ---- one step: compute on the current stream, exchanges on the comm stream
    def _run(self, idx, lookup, interact, update, index):
        """The step's schedule with the segments as callables (eager launches or graph replays)."""
        M = self.M
        if self._cstream is None:  # CPU (gloo tests): the same order, one stream
            index()
            for m in range(M):
                lookup(m)
                self.exchange_fwd(m)
            for m in range(M):
                interact(m)
                self.exchange_bwd(m)
            update()
            return
        main, cs = torch.cuda.current_stream(), self._cstream
        ev_look, ev_recv, ev_bwd, _ = self._ev
        self._side.wait_stream(main)  # the previous step's update read the indexer it rebuilds
        with torch.cuda.stream(self._side):
            index()
            self._ix_done.record(self._side)
        if M == 1:
            # nothing to overlap the exchanges with: they run in stream order on the compute
            # stream (each cross-stream event hop costs a few us of dependency latency:
            # tools/shard_sim.py, step 140 us against 68 us of main-stream work with four hops)
            lookup(0)
            self.exchange_fwd(0)
            interact(0)
            self.exchange_bwd(0)
            main.wait_event(self._ix_done)
            update()
            return
        # M > 1: every exchange on the step's own stream (the capture's origin stream under graph
        # capture), the compute that overlaps them on the second stream.  (The other way round --
        # exchanges on the second stream -- captured fine but segfaulted in graph instantiation,
        # for the library's and torch's RCCL exchange alike: tools/capture_diag.py)
        #   main: lookup(0) | a2a_fwd(0) | a2a_fwd(1) ... | a2a_bwd(0) ... | update
        #   cs  :   lookup(1..M-1) | interact(0) | interact(1) ...
        lookup(0)
        cs.wait_stream(main)
        with torch.cuda.stream(cs):
            for m in range(1, M):
                lookup(m)
                ev_look[m].record(cs)
        for m in range(M):
            if m:
                main.wait_event(ev_look[m])
            self.exchange_fwd(m)
            ev_recv[m].record(main)
            cs.wait_event(ev_recv[m])
            with torch.cuda.stream(cs):
                interact(m)
                ev_bwd[m].record(cs)
        for m in range(M):
            main.wait_event(ev_bwd[m])
            self.exchange_bwd(m)
        main.wait_event(self._ix_done)
        update()

    def step(self, x, idx, dout):
        self._run(idx, lambda m: self.seg_lookup(idx, m), lambda m: self.seg_interact(x, dout, m),
                  lambda: self.seg_update(idx), lambda: self.seg_index(idx))
        return self.dx

    # ---- hipGraph replay of the compute segments (collectives stay eager)
    def capture(self, x, idx_list, dout):
        """Captures seg_index / seg_lookup(m) / seg_update per index batch and seg_interact(m) once."""
        s = torch.cuda.Stream(device=self.out.device)
        s.wait_stream(torch.cuda.current_stream())
        look, upd, ixg = [], [], []

        def graph(fn):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                fn()
            return g
        with torch.cuda.stream(s):
            for idx in idx_list:
                ixg.append(graph(lambda: self.seg_index(idx)))
                look.append([graph(lambda: self.seg_lookup(idx, m)) for m in range(self.M)])
                upd.append(graph(lambda: self.seg_update(idx)))
            mid = [graph(lambda: self.seg_interact(x, dout, m)) for m in range(self.M)]
        torch.cuda.current_stream().wait_stream(s)
        self._graphs = (look, mid, upd, ixg)

    def step_graphed(self, k):
        """One step of index batch k from the captured graphs (same schedule as `step`)."""
        if self._full is not None:
            self._full[k].replay()
            return
        look, mid, upd, ixg = self._graphs
        self._run(None, lambda m: look[k][m].replay(), lambda m: mid[m].replay(), lambda: upd[k].replay(),
                  lambda: ixg[k].replay())

    def capture_full(self, x, idx_list, dout):
        """One hipGraph per index batch holding the WHOLE step: the side-stream index build, the
        lookup, both all-to-alls (RCCL: torch.distributed "nccl" or the library's communicator,
        captured on the step's streams), the interaction and the update -- one replay per step, so
        M > 1 micro-batch overlap is not launch-bound.  Raises if the backend cannot
        be captured (gloo); the caller falls back to `capture` (collectives eager)."""
        if dist.is_initialized() and dist.get_backend(self.group) != "nccl":
            raise RuntimeError(f"{dist.get_backend(self.group)} collectives cannot be captured")
        s = torch.cuda.Stream(device=self.out.device)
        s.wait_stream(torch.cuda.current_stream())
        graphs = []
        with torch.cuda.stream(s):
            for idx in idx_list:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    self.step(x, idx, dout)
                graphs.append(g)
        torch.cuda.current_stream().wait_stream(s)
        self._full = graphs
        if self.comm is not None:
            self.comm.retain_graphs(graphs)

    def release_graphs(self):
        """Drops every captured graph.  A graph holding RCCL work keeps a reference on its
        communicator, and destroying the communicator (dist.destroy_process_group(), or the library
        communicator's close) waits for that reference: release the graphs first (close() does)."""
        for g in (self._full or []):
            g.reset()
        if self._graphs is not None:
            look, mid, upd, ixg = self._graphs
            for g in [g for gs in look for g in gs] + mid + upd + ixg:
                g.reset()
        self._full = self._graphs = None

    def close(self):
        """Releases the graphs, then the library communicator (exchange="abi").  Call before
        dist.destroy_process_group() when the step was captured with the torch exchange."""
        self.release_graphs()
        if self.comm is not None:
            self.comm.close()
            self.comm = None


def make_bench_engine(pkg, w, batch_local, device, rank, world, lr, seed=51234, capacity=None, nbatch=8,
                      micro=None):
    """Bench setup for one rank: local tables (full size) and nbatch index batches for the
    global batch; returns (engine, step(k) closure, prepare_graphs() closure).  batch_local =
    global batch / world for strong scaling.  micro: micro-batches per step (default 1: with the
    whole step in one graph the parallel branches overlap but pay a cross-queue hop each (~3.7 us) --
    tools/shard_sim.py at world 8 with stand-in exchanges: 167 us with 2 against 157 us with 1 --
    and with per-segment graphs two micro-batches are launch-bound: 198 us vs 162 us)."""
    import numpy as np
    if micro is None:
        micro = 1
    rows = w["rows"]
    D, L = w["dim"], w["lookups"]
    E = 4 if w["dtype"] == "f32" else 2
    if capacity is None:
        capacity = int(torch.cuda.get_device_properties(device).total_memory * 0.85)
    part = TablePartition.fitting(rows, world, D * E, capacity)
    mine = part.tables(rank)
    dt = torch.float32 if w["dtype"] == "f32" else torch.bfloat16
    g = torch.Generator(device=device).manual_seed(seed + rank)
    tables = []
    for t in mine:
        n = rows[t]
        s = 1.0 / float(np.sqrt(n))
        tables.append(torch.empty((n, D), dtype=dt, device=device).uniform_(-s, s, generator=g))
    Bg = batch_local * world
    ops = HipShardOps(tables, Bg, L, lr, device=device)
    eng = ShardedHotPath(ops, part, rank, batch_local, D, L, dt, device, micro=micro)
    nb = nbatch
    packs = []
    zipf = w.get("zipf")
    rng = np.random.default_rng(seed + rank)
    perms = {t: zipf_perm(rng, rows[t]) for t in mine} if zipf else None  # the same rows stay hot
    for _ in range(nb):
        if zipf:
            cols = [torch.from_numpy(zipf_rows(rng, rows[t], Bg * L, zipf, perms[t])).to(device) for t in mine]
        else:
            cols = [torch.randint(0, rows[t], (Bg * L,), device=device, generator=g,
                                  dtype=torch.int64).to(torch.int32) for t in mine]
        data = torch.stack(cols) if cols else torch.zeros((0, Bg * L), dtype=torch.int32, device=device)
        packs.append(PackedIndices(data.reshape(len(cols), Bg, L)))
    x = torch.randn((batch_local, D), device=device, generator=g).to(dt)
    dout = (torch.randn((batch_local, eng.width), device=device, generator=g) * 1e-3).to(dt)
    eng.bench_packs = packs  # the index batches (tools/bench_full_step.py drives the full step with them)
    eng._bench_x, eng._bench_dout = x, dout

    def step(k):
        if eng._graphs is not None or eng._full is not None:
            eng.step_graphed(k % nb)
        else:
            eng.step(x, packs[k % nb], dout)

    def prepare_graphs(full=True):
        """full: the whole step per graph, collectives included (capture_full); else (or if that
        capture is refused) the compute segments between eager collectives.  Returns the form."""
        if full:
            try:
                eng.capture_full(x, packs, dout)
                return "full"
            except Exception as e:  # (a backend whose collectives cannot be captured)
                eng._full = None
                import sys
                print(f"note: whole-step capture refused ({e!r}); graphing the compute segments", file=sys.stderr)
        eng.capture(x, packs, dout)
        return "segments"

    return eng, step, prepare_graphs
