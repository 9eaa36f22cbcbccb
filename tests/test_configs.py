"""Parity at the BASELINE.json configurations the metric test does not cover.

  configs[2]  26 Criteo-Kaggle tables x 128 bf16, B = 8192 (the hash-built indexer, MFMA bf16)
  configs[3]  Criteo-Terabyte rows (882.8M, 226 GB bf16 on one GPU), Zipf(1.05) hot rows
  configs[4]  pooled bags: 64 tables x 256 fp32, L = 10, Zipf(1.2) hot rows

The C oracle (oracle/dlrm_oracle.c) cannot hold 9-226 GB of tables, but a training step reads
and writes only the rows its indices touch: `compact()` copies those rows out of the device
tables, renumbers the indices, and the oracle runs the same step on the compact tables.  The
forward output, dx and every touched row after the update are compared; untouched rows are
checked to be unchanged on the device.  Where even that is too large, size-independent
properties are used: row-encoded gathers (bit-exact), exact integer-gradient updates.
Reference semantics: sum pooling, sample-major bags (src/data/criteo.jl:551-557); table sizes
src/data/criteo.jl:350-406."""
import numpy as np
import pytest
import torch

import oracle
from helpers import assert_close

pytestmark = pytest.mark.gpu


def bf16_bits(t):
    return t.contiguous().view(torch.int16).cpu().numpy().view(np.uint16)


def host_rows(t, rows):
    """rows of a device table as a host array (float32, or bf16 bit patterns)."""
    sel = t.index_select(0, torch.from_numpy(rows).to(t.device))
    return sel.cpu().numpy() if t.dtype == torch.float32 else bf16_bits(sel)


def compact(tables, idx_list):
    """(unique rows per table, compact host tables, per batch the renumbered indices [T][N] int64):
    the rows every batch of idx_list touches, renumbered consistently across the batches."""
    uniq, comp = [], []
    ridx = [np.empty_like(i, dtype=np.int64) for i in idx_list]
    for t, tab in enumerate(tables):
        u = np.unique(np.concatenate([i[t] for i in idx_list]))
        uniq.append(u)
        comp.append(host_rows(tab, u))
        for k, i in enumerate(idx_list):
            ridx[k][t] = np.searchsorted(u, i[t])
    return uniq, comp, ridx


def to_f32(a):
    return oracle.bf16_to_f32(a) if a.dtype == np.uint16 else a


def zipf_indices(pkg, rng, rows, n, s, perms=None):
    perms = perms or [pkg.zipf_perm(rng, r) for r in rows]
    return np.stack([pkg.zipf_rows(rng, r, n, s, p) for r, p in zip(rows, perms)]).astype(np.int64)


def run_step_vs_oracle(pkg, gpu, tables, idx_np, B, L, lr, dtype, seed, hot_kw=None, pipeline=None):
    """Training steps on the device tables, in the form bench.py times (`pipeline`, from
    pkg.step_pipeline: None = indexer in the forward's launch, "side" = the next batch's indexer on
    a side stream, "apply" = built by the previous step's apply launch), against the oracle's
    steps on the rows they touch.  idx_np: one [T][B*L] batch, or a list of two consecutive batches
    (a pipelined step then consumes the indexer the previous step prepared).  Asserts the last
    step's out and dx, every touched row after all steps, and that untouched rows are unchanged."""
    T, D = len(tables), tables[0].shape[1]
    F = T + 1
    batches = idx_np if isinstance(idx_np, list) else [idx_np]
    uniq, comp, ridx = compact(tables, batches)
    before = [t.clone() for t in tables] if sum(t.numel() for t in tables) * 2 < 40e9 else None
    rng = np.random.default_rng(seed)
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(dtype).to(gpu)
    ts = pkg.EmbeddingTableSet(tables)
    hp = pkg.HotPath(ts, B, L, lr=lr, index_base=0, pipeline=pipeline, **(hot_kw or {}))
    assert hp.pipeline == pipeline, (hp.pipeline, pipeline)
    dout = torch.from_numpy((rng.standard_normal((B, hp.width)) * 1e-2).astype(np.float32)).to(dtype).to(gpu)
    P = [pkg.PackedIndices(torch.from_numpy(i).to(torch.int32).to(gpu).reshape(T, B, L)) for i in batches]
    for p in P:
        hp.validate(x, p, dout)
    n = len(P)
    if pipeline == "apply":  # prime = one step of the last batch, preparing batch 0
        hp.prime(P[0], x=x, dout=dout, prev=P[-1])
        for k in range(n):
            hp.step_prep(x, P[k], dout, P[(k + 1) % n])
        order = [n - 1] + list(range(n))
    elif pipeline == "side":
        hp.prime(P[0])
        for k in range(n):
            hp.step_next(x, P[k], dout, P[(k + 1) % n])
        order = list(range(n))
    else:
        for k in range(n):
            hp.step(x, P[k], dout)
        order = list(range(n))
    torch.cuda.synchronize()
    hp.check_bounds()
    # the oracle's steps on the compact tables
    xh = x.cpu().numpy() if dtype == torch.float32 else bf16_bits(x)
    dh = dout.cpu().numpy() if dtype == torch.float32 else bf16_bits(dout)
    bf = dtype == torch.bfloat16
    for k in order:
        ys = np.zeros((B, F * D), dtype=xh.dtype)
        oracle.maplookup(comp, ridx[k], 0, B, L, ys, D)
        out = oracle.interact_fwd(xh, ys, F, hp.padding)
        if bf:  # the interaction of |x|, |rows|: sum |products| per entry, the scale of its rounding
            out_abs = to_f32(oracle.interact_fwd(xh & 0x7fff, ys & 0x7fff, F, hp.padding))
        dx, dt = oracle.interact_bwd(dh, ys, D, F, hp.padding)
        oracle.sgd_update(comp, ridx[k], 0, B, L, dt, D, lr)
    got_out = hp.out.float().cpu().numpy()
    nsteps = len(order)
    if bf:  # one bf16 rounding of an fp32 sum that may differ in order, of products whose bf16 factors
        # earlier steps rounded on each side (1 ulp apart per step): relative to the sum of |products|
        err = np.abs(got_out - to_f32(out))
        bound = 2.0 ** -7 * np.abs(to_f32(out)) + 2.0 ** -7 * (nsteps - 1) * out_abs + 2.0 ** -12 * out_abs + 1e-6
        assert (err <= bound).all(), ("out", err.max(), (err / (out_abs + 1e-30)).max())
    else:
        assert_close(got_out, out, rtol=1e-5, scale=np.abs(out).max(), what="out")
    assert_close(hp.dx.cpu().numpy(), dx, rtol=1e-4 * nsteps if bf else 1e-5, scale=np.abs(dx).max(), what="dx")
    for t, tab in enumerate(tables):
        got = to_f32(host_rows(tab, uniq[t]))
        want = to_f32(comp[t])
        if bf:  # the same fp32 update, each side rounded once to bf16 per step: 1 ulp (2^-7 relative) per
            # step of the values involved (the row before the steps and after them)
            err = np.abs(got - want)
            scale = np.abs(want) + (np.abs(to_f32(host_rows(before[t], uniq[t]))) if before is not None else 0)
            assert (err <= 2.0 ** -7 * nsteps * scale + 1e-30).all(), (t, err.max())
        else:
            g = np.abs(to_f32(host_rows(before[t], uniq[t])) - want) if before is not None else np.abs(want)
            assert_close(got, want, rtol=1e-5, scale=g.max() + 1e-6, what=f"table {t} rows")
        if before is not None:  # every other row unchanged
            mask = torch.ones(tab.shape[0], dtype=torch.bool, device=gpu)
            mask[torch.from_numpy(uniq[t]).to(gpu)] = False
            assert torch.equal(tab[mask], before[t][mask]), f"table {t}: an untouched row changed"
    return hp


# ------------------------------------------------------- the bench's exact forms, full size
def kaggle_tables(pkg, gpu, D, dtype, seed):
    g = torch.Generator(device=gpu).manual_seed(seed)
    return [torch.empty((n, D), dtype=dtype, device=gpu).uniform_(-n ** -0.5, n ** -0.5, generator=g)
            for n in pkg.KAGGLE_EMBEDDING_SIZES]


@pytest.mark.parametrize("workload", ["kaggle-d128-b2048", "kaggle-d16-b2048", "kaggle-d128-b8192-bf16"])
def test_bench_form_vs_oracle(pkg, gpu, workload):
    """The exact step form bench.py times for each Kaggle-row workload (pkg.step_pipeline: B <= 2048,
    the metric config and D = 16, build the next batch's indexer in the previous step's apply
    launch; bf16 B = 8192 on a side stream), over two consecutive batches so the prepared indexer is
    consumed, at full table size, against the oracle on the touched rows (validation.jl:125-146)."""
    w = pkg.WORKLOADS[workload]
    D, B = w["dim"], w["batch"]
    dtype = torch.float32 if w["dtype"] == "f32" else torch.bfloat16
    tables = kaggle_tables(pkg, gpu, D, dtype, seed=D + B)
    rng = np.random.default_rng(B + D)
    batches = [np.stack([rng.integers(0, n, size=B) for n in w["rows"]]).astype(np.int64) for _ in range(2)]
    pipeline = pkg.step_pipeline(w)
    hp = run_step_vs_oracle(pkg, gpu, tables, batches, B, 1, 0.05, dtype, seed=B, pipeline=pipeline,
                            hot_kw={"chunk": pkg.step_chunk(w), "parts": pkg.step_parts(w)})
    assert hp.step_api and hp.chunk == pkg.step_chunk(w) and hp.parts == pkg.step_parts(w)


# ---------------------------------------------------------------------------- configs[2]
def test_kaggle_bf16_b8192_step_vs_oracle(pkg, gpu):
    """configs[2]: the full Kaggle tables (33.8M rows x 128 bf16 = 8.6 GB), B = 8192, uniform
    indices: the step (hash indexer on the side stream, bf16 MFMA interaction, once-hit rows
    updated in the backward) against the oracle on the touched rows."""
    rows = pkg.KAGGLE_EMBEDDING_SIZES
    D, B = 128, 8192
    g = torch.Generator(device=gpu).manual_seed(11)
    tables = [torch.empty((n, D), dtype=torch.bfloat16, device=gpu).uniform_(-n ** -0.5, n ** -0.5, generator=g)
              for n in rows]
    rng = np.random.default_rng(12)
    idx = np.stack([rng.integers(0, n, size=B) for n in rows]).astype(np.int64)
    hp = run_step_vs_oracle(pkg, gpu, tables, idx, B, 1, 0.05, torch.bfloat16, seed=13)
    assert hp.step_api  # the bench's step form


# ---------------------------------------------------------------------------- configs[4]
def test_pooled_64x256_l10_zipf_step_vs_oracle(pkg, gpu):
    """configs[4] at 100k rows per table (the oracle's size): 64 tables x 256 fp32, L = 10 sum-pooled
    bags, Zipf(1.2) hot rows, B = 2048 -- the bench's pooled path (many-wave pooled gather, the
    interaction at d = 256 / F = 65, the bag build on a side stream, the hot-segment apply) over two
    consecutive batches, against the oracle; and the pipelined form (the next batch's bag build
    beside the apply, HotPath.step_next) the same way."""
    rows = [100_000] * 64
    D, B, L = 256, 2048, 10
    g = torch.Generator(device=gpu).manual_seed(21)
    tables = [torch.empty((n, D), device=gpu).uniform_(-n ** -0.5, n ** -0.5, generator=g) for n in rows]
    rng = np.random.default_rng(22)
    idx = [zipf_indices(pkg, rng, rows, B * L, 1.2) for _ in range(2)]
    pipeline = pkg.step_pipeline(pkg.WORKLOADS["pooled-64x256-l10"])
    keep = [t.clone() for t in tables]
    hp = run_step_vs_oracle(pkg, gpu, tables, idx, B, L, 0.05, torch.float32, seed=23, pipeline=pipeline)
    assert hp.materialize_ys and pipeline is None  # pooled bags keep ys (the bench's form)
    del hp
    hp = run_step_vs_oracle(pkg, gpu, keep, idx, B, L, 0.05, torch.float32, seed=23, pipeline="side")
    assert hp.pipeline == "side"


def test_pooled_full_size_properties(pkg, gpu):
    """configs[4] at full size (64 x 1M x 256 fp32 = 65.5 GB): the pooled gather of row-encoded
    tables is exact (a bag's L encoded rows sum without rounding), and an integer-gradient
    update on zeroed tables equals the closed-form scatter-add bit for bit (each bag's gradient
    counted once per lookup, duplicates within a bag included)."""
    T, N, D, B, L = 64, 1_000_000, 256, 2048, 10
    rng = np.random.default_rng(31)
    idx = torch.from_numpy(zipf_indices(pkg, rng, [N] * T, B * L, 1.2)).to(torch.int32).to(gpu)
    col = torch.arange(D, device=gpu, dtype=torch.float32)[None, :] / 256.0
    tables = []
    for t in range(T):  # value = (row mod 1021) + c/256 (+ nothing per table: sums stay < 2^14)
        r = torch.arange(N, device=gpu, dtype=torch.float32).remainder_(1021.0)
        tables.append((r[:, None] + col).contiguous())
    ts = pkg.EmbeddingTableSet(tables)
    p = pkg.PackedIndices(idx.reshape(T, B, L))
    ys = pkg.maplookup(pkg.PreallocationStrategy(D), ts, p, index_base=0)
    want = idx.to(torch.float32).remainder(1021.0).reshape(T, B, L).sum(dim=2)  # [T][B], exact
    want = want.T[:, :, None] + L * col[None, :, :]
    assert torch.equal(ys[:, D:].reshape(B, T, D), want)
    del ys
    for t in tables:
        t.zero_()
    gi = torch.from_numpy(rng.integers(-4, 5, size=(B, T * D)).astype(np.float32)).to(gpu)
    pkg.update_(pkg.Descent(1.0), ts, pkg.maplookup_pullback(0, ts, p, gi), index_base=0)
    for t in (0, 17, 63):
        rows_t = idx[t].long()
        u = torch.unique(rows_t)
        ref = torch.zeros((N, D), dtype=torch.float64, device=gpu)
        ref.index_add_(0, rows_t, gi[:, t * D:(t + 1) * D].double().repeat_interleave(L, dim=0))
        assert torch.equal(tables[t][u], (-ref[u]).float())
        nz = tables[t].abs().sum(dim=1) != 0
        touched = torch.zeros(N, dtype=torch.bool, device=gpu)
        touched[u] = True
        assert not (nz & ~touched).any(), "a row no index touched was written"


# ---------------------------------------------------------------------------- configs[3]
def test_terabyte_bf16_full_size(pkg, gpu):
    """configs[3] on one GPU: the 26 Criteo-Terabyte tables (882.8M rows x 128 bf16 = 226 GB,
    criteo.jl:379-406).  (1) Row-encoded gather: columns 0-3 of row r hold its four bytes and
    column 4 the table, so every gathered row identifies itself exactly (bf16 holds 0-255).
    (2) The bench's pipelined step form over two Zipf(1.05) batches against the oracle on their touched rows.
    (3) An integer-gradient update on zeroed tables == the closed form, bit for bit."""
    rows = pkg.TERABYTE_EMBEDDING_SIZES
    T, D, B = len(rows), 128, 2048
    if torch.cuda.get_device_properties(gpu).total_memory < sum(rows) * D * 2 + 20e9:
        pytest.skip("needs a 288 GB MI355X")
    tables = [torch.empty((n, D), dtype=torch.bfloat16, device=gpu) for n in rows]
    chunk = 1 << 24
    for t, (tab, n) in enumerate(zip(tables, rows)):
        tab[:, 5:] = 1.0
        for r0 in range(0, n, chunk):
            r = torch.arange(r0, min(n, r0 + chunk), device=gpu, dtype=torch.int64)
            for k in range(4):
                tab[r0:r0 + len(r), k] = ((r >> (8 * k)) & 255).to(torch.bfloat16)
            tab[r0:r0 + len(r), 4] = float(t)
    rng = np.random.default_rng(41)
    perms = [pkg.zipf_perm(rng, r) for r in rows]  # the same rows stay hot across batches
    idx_np = zipf_indices(pkg, rng, rows, B, 1.05, perms)
    idx2_np = zipf_indices(pkg, rng, rows, B, 1.05, perms)
    idx = torch.from_numpy(idx_np).to(torch.int32).to(gpu)
    ts = pkg.EmbeddingTableSet(tables)
    ys = pkg.maplookup(pkg.PreallocationStrategy(D), ts, pkg.PackedIndices(idx), index_base=0)
    got = ys[:, D:].reshape(B, T, D).float()
    dec = sum(got[:, :, k].to(torch.int64) << (8 * k) for k in range(4))  # [B][T]
    assert torch.equal(dec, idx.T.to(torch.int64))
    assert torch.equal(got[:, :, 4], torch.arange(T, device=gpu, dtype=torch.float32)[None, :].expand(B, T))
    del ys, got
    # (2) the bench's step form (pkg.step_pipeline: the indexer built by the previous step's apply
    # launch, 8 parts per table) over two consecutive batches vs the oracle (fresh random rows where
    # the steps read and write)
    g = torch.Generator(device=gpu).manual_seed(42)
    idx2 = torch.from_numpy(idx2_np).to(torch.int32).to(gpu)
    for t, tab in enumerate(tables):
        u = torch.unique(torch.cat([idx[t], idx2[t]]).long())
        tab[u] = torch.empty((len(u), D), device=gpu).uniform_(-0.05, 0.05, generator=g).to(torch.bfloat16)
    pipeline = pkg.step_pipeline(pkg.WORKLOADS["terabyte-d128-bf16-zipf"])
    assert pipeline == "apply"
    w = pkg.WORKLOADS["terabyte-d128-bf16-zipf"]
    hp = run_step_vs_oracle(pkg, gpu, tables, [idx_np, idx2_np], B, 1, 0.05, torch.bfloat16, seed=43,
                            pipeline=pipeline, hot_kw={"chunk": pkg.step_chunk(w), "parts": pkg.step_parts(w)})
    assert hp.parts == 32  # (the bench's form: 256-B rows)
    del hp
    # (3) exact integer-gradient update on zeroed tables
    for tab in tables:
        tab.zero_()
    gi = torch.from_numpy(rng.integers(-4, 5, size=(B, T * D)).astype(np.float32)).to(gpu)
    p = pkg.PackedIndices(idx)
    pkg.update_(pkg.Descent(1.0), ts, pkg.maplookup_pullback(0, ts, p, gi), index_base=0)
    for t in (0, 5, 19, 25):  # 227.6M, 3, 292.8M (the largest) and 36 rows
        rows_t = idx[t].long()
        u = torch.unique(rows_t)
        ref = torch.zeros((len(u), D), dtype=torch.float64, device=gpu)
        ref.index_add_(0, torch.searchsorted(u, rows_t), gi[:, t * D:(t + 1) * D].double())
        assert torch.equal(tables[t][u].float(), (-ref).float().to(torch.bfloat16).float())
        nz = (tables[t] != 0).any(dim=1).nonzero().flatten()
        assert torch.isin(nz, u).all(), "a row no index touched was written"


@pytest.mark.parametrize("rank", [5, 0])
def test_terabyte_fp32_shard_of_world8(pkg, gpu, rank):
    """configs[3] in its own form: fp32 Criteo-Terabyte tables sharded by table over 8 GPUs, global
    batch 2048 (256 per GPU).  On this one GPU, rank `rank`'s shard at full size (rank 5: the
    292.8M-row table, 150 GB fp32; rank 0: 116 GB) runs its table-owning half of the sharded step --
    the lookup of its tables for all 2048 samples straight into the exchange's send layout, the split
    indexer over the global batch, and the update from the received gradient rows -- checked against
    a host gather and the closed-form scatter-add on the touched rows (integer gradients on zeroed
    tables: exact), and no untouched row written."""
    from dlrm_jl_amd.sharded import HipShardOps, TablePartition
    rows = pkg.TERABYTE_EMBEDDING_SIZES
    world, Bg, D = 8, 2048, 128
    B = Bg // world
    part = TablePartition.fitting(rows, world, D * 4, int(260e9))
    mine = part.tables(rank)
    need = sum(rows[t] for t in mine) * D * 4
    if torch.cuda.get_device_properties(gpu).total_memory < need + 30e9:
        pytest.skip("needs a 288 GB MI355X")
    Tr = len(mine)
    # row-encoded fp32 tables: columns 0..2 = the row's three 11-bit pieces (exact in fp32), 3 = table
    tables = [torch.empty((rows[t], D), dtype=torch.float32, device=gpu) for t in mine]
    chunk = 1 << 24
    for k, (t, tab) in enumerate(zip(mine, tables)):
        tab[:, 4:] = 0.5
        for r0 in range(0, rows[t], chunk):
            r = torch.arange(r0, min(rows[t], r0 + chunk), device=gpu, dtype=torch.int64)
            for q in range(3):
                tab[r0:r0 + len(r), q] = ((r >> (11 * q)) & 2047).to(torch.float32)
            tab[r0:r0 + len(r), 3] = float(t)
    rng = np.random.default_rng(50 + rank)
    perms = [pkg.zipf_perm(rng, rows[t]) for t in mine]
    idx_np = np.stack([pkg.zipf_rows(rng, rows[t], Bg, 1.05, p) for t, p in zip(mine, perms)]).astype(np.int32)
    idx = torch.from_numpy(idx_np).to(gpu)
    ops = HipShardOps(tables, Bg, 1, 1.0, device=gpu)
    p = pkg.PackedIndices(idx.reshape(Tr, Bg, 1))
    send = torch.empty((world * Tr * B * D,), dtype=torch.float32, device=gpu)
    ops.lookup_blocked(p, send, D, B * D, B, Tr * B * D)
    got = send.view(world, Tr, B, D).permute(1, 0, 2, 3).reshape(Tr, Bg, D)
    dec = sum(got[:, :, q].to(torch.int64) << (11 * q) for q in range(3))
    assert torch.equal(dec, idx.to(torch.int64))
    assert torch.equal(got[:, :, 3], torch.tensor(mine, device=gpu, dtype=torch.float32)[:, None].expand(Tr, Bg))
    del send, got
    for tab in tables:
        tab.zero_()
    ops.build_indexer(p)
    gi = torch.from_numpy(rng.integers(-4, 5, size=(Bg, Tr * D)).astype(np.float32)).to(gpu)
    ops.update(p, gi, prebuilt=True)
    ops.check_bounds()
    for k, t in enumerate(mine):
        rows_t = idx[k].long()
        u = torch.unique(rows_t)
        ref = torch.zeros((len(u), D), dtype=torch.float64, device=gpu)
        ref.index_add_(0, torch.searchsorted(u, rows_t), gi[:, k * D:(k + 1) * D].double())
        assert torch.equal(tables[k][u], (-ref).float()), (rank, t)
        nz = (tables[k] != 0).any(dim=1).nonzero().flatten()
        assert torch.isin(nz, u).all(), "a row no index touched was written"
