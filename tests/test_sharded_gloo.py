"""Table-sharded multi-rank path (dlrm.jl_amd/sharded.py) on CPU: world_size 2 and 3, gloo.

The exchange logic (partition, uneven all-to-all splits, column scatter/gather) is the
product code; local compute is supplied by the CPU oracle (test-only ShardOps), and the
result must equal — bit for bit — one process running the same step on the global batch.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OracleShardOps:
    """CPU checker with the ShardOps interface (tables: list of numpy arrays)."""

    def __init__(self, tables, lr):
        import oracle
        self.o = oracle
        self.tables = tables
        self.lr = lr

    def bind_recv(self, tabs_per_mb):
        self.recv_tables = tabs_per_mb

    def build_indexer(self, idx):
        pass

    def lookup_blocked(self, idx, out, ld, tstride, brows, bstride):
        T, Bg, D = len(self.tables), idx.B, self.tables[0].shape[1]
        tmp = np.zeros((Bg, T * D), dtype=np.float32)
        self.o.maplookup(self.tables, idx.data.numpy().astype(np.int64), 0, Bg, idx.L, tmp, 0)
        b = np.arange(Bg)[:, None, None]
        t = np.arange(T)[None, :, None]
        c = np.arange(D)[None, None, :]
        dst = (b // brows) * bstride + (b % brows) * ld + t * tstride + c
        out.view(-1).numpy()[dst.reshape(-1)] = tmp.reshape(-1)

    def scatter_rows(self, src, src_ld, src_off, dst, dbase, dld, T, B, D):
        b = np.arange(B)[:, None, None]
        t = np.arange(T)[None, :, None]
        c = np.arange(D)[None, None, :]
        s_ = (b * src_ld + src_off + t * D + c).reshape(-1)
        d_ = (dbase.numpy()[None, :, None] + b * dld.numpy()[None, :, None] + c).reshape(-1)
        dst.view(-1).numpy()[d_] = src.reshape(-1).numpy()[s_]

    def _ys(self, x, m):
        return torch.cat([x] + list(self.recv_tables[m]), dim=1).numpy()

    def interact_fwd_recv(self, x, out, padding, m=0):
        ys = self._ys(x, m)
        res = self.o.interact_fwd(x.contiguous().numpy(), ys, len(self.recv_tables[m]) + 1, padding)
        out.copy_(torch.from_numpy(res))

    def interact_bwd_recv(self, dout, x, dx, dt, padding, m=0):
        d = dx.shape[1]
        rdx, rdt = self.o.interact_bwd(dout.contiguous().numpy(), self._ys(x, m), d, len(self.recv_tables[m]) + 1,
                                       padding)
        dx.copy_(torch.from_numpy(rdx))
        dt.copy_(torch.from_numpy(rdt))

    def update(self, idx, grad, prebuilt=False):
        self.o.sgd_update(self.tables, idx.data.numpy().astype(np.int64), 0, idx.B, idx.L, grad.numpy(), 0, self.lr)


def _problem(T, rows, D, B, world, L, seed=3):
    rng = np.random.default_rng(seed)
    tables = [rng.uniform(-1, 1, size=(rows[t], D)).astype(np.float32) for t in range(T)]
    Bg = B * world
    idx = np.stack([rng.integers(0, rows[t], size=Bg * L) for t in range(T)]).astype(np.int64)
    x = rng.standard_normal((Bg, D)).astype(np.float32)
    F = T + 1
    dout = rng.standard_normal((Bg, D + F * (F - 1) // 2)).astype(np.float32)
    return tables, idx, x, dout


def _worker(rank, world, port, cfg, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import dlrm_pkg
    pkg = dlrm_pkg.load()
    from dlrm_jl_amd.sharded import ShardedHotPath, TablePartition
    T, rows, D, B, L, lr, owners, micro = cfg
    tables, idx, x, dout = _problem(T, rows, D, B, world, L)
    part = TablePartition(T, world, owners)
    mine = part.tables(rank)
    ops = OracleShardOps([tables[t].copy() for t in mine], lr)
    eng = ShardedHotPath(ops, part, rank, B, D, L, torch.float32, torch.device("cpu"), micro=micro)
    p = pkg.PackedIndices(torch.from_numpy(idx[mine]).reshape(len(mine), B * world, L))
    sl = [eng.global_index(b) for b in range(B)]  # this rank's samples of the global batch
    eng.step(torch.from_numpy(x[sl]).contiguous(), p, torch.from_numpy(dout[sl]).contiguous())
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), out=eng.out.numpy(), dx=eng.dx.numpy(),
             **{f"table{t}": ops.tables[k] for k, t in enumerate(mine)})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,T,L,owners,micro,G", [
    (2, 5, 1, None, 1, 0), (2, 7, 3, None, 1, 0), (3, 4, 1, None, 1, 0), (3, 2, 2, None, 1, 0),
    (2, 5, 1, [[4, 0, 2], [1, 3]], 1, 0), (3, 6, 2, [[5], [0, 2, 3, 4], [1]], 1, 0),
    (2, 5, 1, None, 2, 0), (3, 6, 2, [[5], [0, 2, 3, 4], [1]], 2, 0), (2, 7, 1, None, 4, 0),
    # strong scaling (bench.py --global-batch): one global batch of 12 over 2 and 3 ranks
    (2, 5, 1, None, 1, 12), (3, 5, 1, None, 1, 12), (3, 5, 1, None, 2, 12), (2, 6, 2, None, 3, 12)])
def test_sharded_step_equals_single_process(tmp_path, pkg, world, T, L, owners, micro, G):
    """owners: explicit (non-contiguous) table assignment, as TablePartition.fitting makes.
    micro: micro-batches per step (rank r's local sample b is global sample global_index(r, b)).
    G: a fixed global batch split over the ranks (strong scaling); 0: 4 samples per rank (weak)."""
    import oracle
    rows = [3, 50, 1000, 7, 400, 12, 90][:T]
    D, B, lr = 16, (G // world if G else 4), 0.5
    cfg = (T, rows, D, B, L, lr, owners, micro)
    mp.start_processes(_worker, args=(world, _free_port(), cfg, str(tmp_path)), nprocs=world, start_method="spawn")
    # single process on the global batch
    tables, idx, x, dout = _problem(T, rows, D, B, world, L)
    Bg = B * world
    F = T + 1
    ys = np.zeros((Bg, F * D), dtype=np.float32)
    oracle.maplookup(tables, idx, 0, Bg, L, ys, D)
    out = oracle.interact_fwd(x, ys, F)
    dx, dt = oracle.interact_bwd(dout, ys, D, F)
    oracle.sgd_update(tables, idx, 0, Bg, L, dt, D, lr)
    from dlrm_jl_amd.sharded import TablePartition
    part = TablePartition(T, world, owners)
    Bm = B // micro
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        sl = [(b // Bm) * world * Bm + r * Bm + b % Bm for b in range(B)]
        assert np.array_equal(z["out"], out[sl])
        assert np.array_equal(z["dx"], dx[sl])
        for t in part.tables(r):
            assert np.array_equal(z[f"table{t}"], tables[t]), (r, t)


def test_table_partition_is_balanced_and_contiguous():
    import dlrm_pkg
    dlrm_pkg.load()
    from dlrm_jl_amd.sharded import TablePartition
    for T, W in [(26, 8), (26, 4), (26, 2), (26, 1), (3, 8), (64, 8)]:
        p = TablePartition(T, W)
        assert sum(p.counts) == T and max(p.counts) - min(p.counts) <= 1
        covered = [t for r in range(W) for t in range(*p.range(r))]
        assert covered == list(range(T))


def test_partition_fits_terabyte_tables():
    """Criteo-Terabyte (criteo.jl:379-406) at D=128 fp32: the contiguous blocks fit 288 GB at 4
    and 8 GPUs; at 2 GPUs (267 GB block) the byte-balanced assignment is used instead."""
    import dlrm_pkg
    pkg = dlrm_pkg.load()
    from dlrm_jl_amd.sharded import TablePartition
    rows = pkg.TERABYTE_EMBEDDING_SIZES
    rb, cap = 128 * 4, int(288e9 * 0.85)
    for W in (2, 4, 8):
        p = TablePartition.fitting(rows, W, rb, cap)
        per = p.bytes_per_rank(rows, rb)
        assert max(per) <= cap and sorted(p.order) == list(range(26))
        assert p.contiguous == (W != 2)
    p2 = TablePartition.fitting(rows, 2, rb, cap)
    assert max(p2.bytes_per_rank(rows, rb)) < 240e9
    with pytest.raises(ValueError):
        TablePartition(3, 2, [[0, 1], [1, 2]])
    with pytest.raises(ValueError, match="bytes per rank"):  # 452 GB fp32 cannot fit one 288 GB GPU
        TablePartition.fitting(rows, 1, rb, cap)


# ---- the full training step, data-parallel MLPs + sharded tables (SURVEY §8 rows f1 + f3) ------

def _full_problem(T, rows, D, B, world, seed=11):
    rng = np.random.default_rng(seed)
    tables = [rng.uniform(-0.5, 0.5, size=(rows[t], D)).astype(np.float32) for t in range(T)]
    Bg = B * world
    idx = np.stack([rng.integers(0, rows[t], size=Bg) for t in range(T)]).astype(np.int64)
    dense = rng.standard_normal((Bg, 13)).astype(np.float32)
    labels = (rng.random(Bg) < 0.4).astype(np.float32)
    F = T + 1
    bsz = [13, 32, D]
    tsz = [D + F * (F - 1) // 2, 24, 1]

    def mlp(sizes):
        return ([rng.standard_normal((o, i)).astype(np.float32) * np.float32((2.0 / (i + o)) ** 0.5)
                 for i, o in zip(sizes[:-1], sizes[1:])],
                [rng.standard_normal(o).astype(np.float32) * np.float32(0.1) for o in sizes[1:]])
    return tables, idx, dense, labels, mlp(bsz), mlp(tsz)


def _full_worker(rank, world, port, cfg, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import dlrm_pkg
    pkg = dlrm_pkg.load()
    from dlrm_jl_amd.sharded import ShardedHotPath, TablePartition
    T, rows, D, B, lr = cfg
    tables, idx, dense, labels, (bW, bb), (tW, tb) = _full_problem(T, rows, D, B, world)
    part = TablePartition(T, world)
    mine = part.tables(rank)
    ops = OracleShardOps([tables[t].copy() for t in mine], lr)
    eng = ShardedHotPath(ops, part, rank, B, D, 1, torch.float32, torch.device("cpu"))
    t_ = lambda a: [torch.from_numpy(v) for v in a]  # noqa: E731
    model = pkg.ShardedDLRMModel(pkg.DenseMLP(t_(bW), t_(bb)), pkg.DenseMLP(t_(tW), t_(tb), sigmoid_last=True),
                                 eng, lr)
    p = pkg.PackedIndices(torch.from_numpy(idx[mine]).reshape(len(mine), B * world, 1))
    sl = slice(rank * B, (rank + 1) * B)
    loss = model.step(torch.from_numpy(dense[sl]).contiguous(), p, torch.from_numpy(labels[sl]).contiguous())
    arrs = {f"table{t}": ops.tables[k] for k, t in enumerate(mine)}
    for name, m in (("bot", model.bottom), ("top", model.top)):
        for i in range(len(m.W)):
            arrs[f"{name}_W{i}"] = m.W[i].numpy()
            arrs[f"{name}_b{i}"] = m.b[i].numpy()
    np.savez(os.path.join(outdir, f"full{rank}.npz"), loss=float(loss), **arrs)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_full_step_equals_single_process(tmp_path, pkg, world):
    """Data-parallel MLPs (gradients all-reduced over gloo) + table-sharded hot path == one
    process running the full step on the global batch: loss, every MLP parameter, every table."""
    import oracle
    from helpers import assert_close
    T, D, B, lr = 5, 8, 6, 0.3
    rows = [3, 50, 200, 7, 40]
    mp.start_processes(_full_worker, args=(world, _free_port(), (T, rows, D, B, lr), str(tmp_path)), nprocs=world,
                       start_method="spawn")
    tables, idx, dense, labels, (bW, bb), (tW, tb) = _full_problem(T, rows, D, B, world)
    Bg, F = B * world, T + 1
    t_ = lambda a: [torch.from_numpy(v.copy()) for v in a]  # noqa: E731
    bottom = pkg.DenseMLP(t_(bW), t_(bb))
    top = pkg.DenseMLP(t_(tW), t_(tb), sigmoid_last=True)
    x = bottom.forward(torch.from_numpy(dense)).numpy()
    ys = np.zeros((Bg, F * D), dtype=np.float32)
    oracle.maplookup(tables, idx, 0, Bg, 1, ys, D)
    out = oracle.interact_fwd(x, ys, F)
    pr = top.forward(torch.from_numpy(out)).reshape(-1)
    lab = torch.from_numpy(labels)
    want_loss = float(pkg.bce_loss(pr, lab))
    dout = top.backward(pkg.bce_loss_back(pr, lab).reshape(-1, 1)).numpy()
    dx, dt = oracle.interact_bwd(np.ascontiguousarray(dout), ys, D, F)
    oracle.sgd_update(tables, idx, 0, Bg, 1, dt, D, lr)
    bottom.backward(torch.from_numpy(dx), need_dx=False)
    top.sgd_(lr)
    bottom.sgd_(lr)
    from dlrm_jl_amd.sharded import TablePartition
    part = TablePartition(T, world)
    for r in range(world):
        z = np.load(tmp_path / f"full{r}.npz")
        assert abs(float(z["loss"]) - want_loss) <= 1e-6 * abs(want_loss)
        for name, m in (("bot", bottom), ("top", top)):
            for i in range(len(m.W)):
                assert_close(z[f"{name}_W{i}"], m.W[i].numpy(), rtol=1e-5, what=f"rank {r} {name} W{i}")
                assert_close(z[f"{name}_b{i}"], m.b[i].numpy(), rtol=1e-5, what=f"rank {r} {name} b{i}")
        for t in part.tables(r):
            assert_close(z[f"table{t}"], tables[t], rtol=1e-5, what=f"rank {r} table {t}")
