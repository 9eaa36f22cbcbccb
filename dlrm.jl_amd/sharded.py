"""Table-sharded (model-parallel) hot path across the GPUs of one node.

The reference has no distributed code; this is the MI355X extension the
north star asks for: embedding tables shard BY TABLE across ranks, and one all-to-all each
way moves the looked-up vectors to the ranks that own the samples, and their gradients back.

  rank r owns tables [t0_r, t1_r) (contiguous, balanced count) and samples
  [r*B, (r+1)*B) of the global batch Bg = world * B (weak scaling: B per GPU is fixed).

  forward : lookup of r's tables for all Bg samples -> send [Bg][T_r*D]
            all-to-all (row block j -> rank j)      -> recv_j [B][T_j*D] from every rank j
            scatter into ys [B][F*D] columns D + t0_j*D ...   (x goes in columns 0..D)
            DotInteraction(x, ys) on the local batch
  backward: dot_back -> dt [B][F*D]
            gather dt column blocks per owner -> all-to-all -> grad [Bg][T_r*D]
            update!(Descent) of r's tables with r's indices for all Bg samples

All compute goes through a `ShardOps` object: `HipShardOps` (the product: the C-ABI kernels)
or, in the CPU gloo tests, a test-only CPU checker.  torch.distributed (backend "nccl"
= RCCL over xGMI on MI355X) carries the two all-to-alls; uneven table counts per rank use
the split-size form of all_to_all_single.
"""
import torch
import torch.distributed as dist

from . import _lib
from .embedding import EmbeddingTableSet, PackedIndices
from .interact import interaction_sizes
from .runtime import dtype_code, ptr
from .update import SparseIndexer


class TablePartition:
    """Contiguous, count-balanced assignment of T tables to `world` ranks
    (every table costs Bg lookups per step whatever its size; Kaggle's largest table is
    5.2 GB at D=128 fp32, far below one GPU's 288 GB, so count balance is what matters)."""

    def __init__(self, T, world):
        base, extra = divmod(T, world)
        self.counts = [base + (1 if r < extra else 0) for r in range(world)]
        self.starts = [sum(self.counts[:r]) for r in range(world)]
        self.T, self.world = T, world

    def range(self, r):
        return self.starts[r], self.starts[r] + self.counts[r]


class HipShardOps:
    """The product ops: the HIP kernels behind include/dlrm_hip.h (no host syncs)."""

    def __init__(self, tables, batch_global, lookups, lr, index_base=0):
        self.ts = tables if isinstance(tables, EmbeddingTableSet) else EmbeddingTableSet(tables)
        self.ctx = self.ts.ctx
        self.lib = self.ctx.lib
        self.Bg, self.L, self.lr, self.base = batch_global, lookups, lr, index_base
        self.indexer = SparseIndexer(len(self.ts), batch_global * lookups, self.ts.device)

    def _ok(self, rc):
        if rc != _lib.OK:
            self.ctx.check(rc)

    def lookup(self, idx, send):
        self._ok(self.lib.dlrm_maplookup(self.ctx.bind(), self.ts.handle, ptr(idx.data), idx.itype, idx.stride,
                                         self.base, idx.B, idx.L, ptr(send), send.stride(0), 0))

    def interact_fwd(self, x, ys, out, padding):
        d = x.shape[1]
        self._ok(self.lib.dlrm_interact_fwd(self.ctx.bind(), dtype_code(x.dtype), d, ys.shape[1] // d, x.shape[0],
                                            ptr(x), x.stride(0), ptr(ys), ys.stride(0), ptr(out), out.stride(0),
                                            padding))

    def interact_bwd(self, dout, ys, dx, dt, padding):
        d = dx.shape[1]
        self._ok(self.lib.dlrm_interact_bwd(self.ctx.bind(), dtype_code(dout.dtype), d, ys.shape[1] // d,
                                            dout.shape[0], ptr(dout), dout.stride(0), padding, ptr(ys), ys.stride(0),
                                            ptr(dx), dx.stride(0), ptr(dt), dt.stride(0)))

    def update(self, idx, grad):
        self._ok(self.lib.dlrm_sgd_update(self.ctx.bind(), self.ts.handle, self.indexer.handle, 0, ptr(idx.data),
                                          idx.itype, idx.stride, self.base, idx.B, idx.L, ptr(grad),
                                          dtype_code(grad.dtype), grad.stride(0), 0, self.lr))


class ShardedHotPath:
    """One step of the table-sharded hot path on this rank (see module docstring)."""

    def __init__(self, ops, partition, rank, batch_local, dim, lookups, dtype, device, group=None):
        self.ops, self.part, self.rank = ops, partition, rank
        self.world = partition.world
        self.B, self.D, self.L = batch_local, dim, lookups
        self.Bg = batch_local * self.world
        self.T = partition.T
        self.F = self.T + 1
        self.t0, self.t1 = partition.range(rank)
        self.Tr = self.t1 - self.t0
        self.group = group
        _, self.width, self.padding = interaction_sizes(dim, self.F)
        dev = device
        D, B = dim, batch_local
        self.send = torch.empty((self.Bg, max(self.Tr, 1) * D), dtype=dtype, device=dev)
        self.recv = torch.empty((sum(c * B * D for c in partition.counts),), dtype=dtype, device=dev)
        self.ys = torch.zeros((B, self.F * D), dtype=dtype, device=dev)
        self.out = torch.empty((B, self.width), dtype=dtype, device=dev)
        self.dx = torch.empty((B, D), dtype=torch.float32, device=dev)
        self.dt = torch.empty((B, self.F * D), dtype=torch.float32, device=dev)
        self.gsend = torch.empty((sum(c * B * D for c in partition.counts),), dtype=torch.float32, device=dev)
        self.grecv = torch.empty((self.Bg, max(self.Tr, 1) * D), dtype=torch.float32, device=dev)
        # element counts of each peer's block (flat all_to_all_single splits)
        self.fwd_in_splits = [B * self.Tr * D] * self.world
        self.fwd_out_splits = [B * c * D for c in partition.counts]
        self.bwd_in_splits = self.fwd_out_splits
        self.bwd_out_splits = self.fwd_in_splits
        self.offsets = [sum(self.fwd_out_splits[:j]) for j in range(self.world)]

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

    def exchange_fwd(self):
        self._a2a(self.recv, self.send.reshape(-1)[: self.Bg * self.Tr * self.D], self.fwd_out_splits,
                  self.fwd_in_splits)
        D, B = self.D, self.B
        for j in range(self.world):
            c = self.part.counts[j]
            if c == 0:
                continue
            t0, _ = self.part.range(j)
            blk = self.recv[self.offsets[j]: self.offsets[j] + B * c * D].view(B, c * D)
            self.ys[:, D + t0 * D: D + (t0 + c) * D].copy_(blk)

    def exchange_bwd(self):
        D, B = self.D, self.B
        for j in range(self.world):
            c = self.part.counts[j]
            if c == 0:
                continue
            t0, _ = self.part.range(j)
            self.gsend[self.offsets[j]: self.offsets[j] + B * c * D].view(B, c * D).copy_(
                self.dt[:, D + t0 * D: D + (t0 + c) * D])
        self._a2a(self.grecv.reshape(-1)[: self.Bg * self.Tr * self.D], self.gsend, self.bwd_out_splits,
                  self.bwd_in_splits)

    # ---- the step
    def forward(self, x, idx):
        """idx: PackedIndices of this rank's tables for the GLOBAL batch ([T_r][Bg*L])."""
        if self.Tr:
            self.ops.lookup(idx, self.send)
        self.exchange_fwd()
        self.ops.interact_fwd(x, self.ys, self.out, self.padding)
        return self.out

    def backward(self, idx, dout):
        self.ops.interact_bwd(dout, self.ys, self.dx, self.dt, self.padding)
        self.exchange_bwd()
        if self.Tr:
            self.ops.update(idx, self.grecv)
        return self.dx

    def step(self, x, idx, dout):
        self.forward(x, idx)
        return self.backward(idx, dout)


def make_bench_engine(pkg, w, batch_local, device, rank, world, lr, seed=51234):
    """Bench setup for one rank: local tables (full size) and NBATCH index batches for the
    global batch; returns (engine, step(k) closure)."""
    import numpy as np
    rows = w["rows"]
    D, L = w["dim"], w["lookups"]
    part = TablePartition(len(rows), world)
    t0, t1 = part.range(rank)
    dt = torch.float32 if w["dtype"] == "f32" else torch.bfloat16
    g = torch.Generator(device=device).manual_seed(seed + rank)
    tables = []
    for n in rows[t0:t1]:
        s = 1.0 / float(np.sqrt(n))
        t = torch.empty((n, D), dtype=torch.float32, device=device).uniform_(-s, s, generator=g)
        tables.append(t.to(dt))
    Bg = batch_local * world
    ops = HipShardOps(tables, Bg, L, lr) if tables else None
    eng = ShardedHotPath(ops, part, rank, batch_local, D, L, dt, device)
    nb = 8
    packs = []
    for _ in range(nb):
        cols = [torch.randint(0, n, (Bg * L,), device=device, generator=g, dtype=torch.int64).to(torch.int32)
                for n in rows[t0:t1]]
        data = torch.stack(cols) if cols else torch.zeros((0, Bg * L), dtype=torch.int32, device=device)
        packs.append(PackedIndices(data.reshape(len(cols), Bg, L)))
    x = torch.randn((batch_local, D), device=device, generator=g).to(dt)
    dout = (torch.randn((batch_local, eng.width), device=device, generator=g) * 1e-3).to(dt)

    def step(k):
        eng.step(x, packs[k % nb], dout)

    return eng, step
