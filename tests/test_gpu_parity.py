"""GPU parity: the HIP path (through the C ABI) against the pinned CPU oracle and the goldens.

Bars (see tests/helpers.py): bit-exact for one-hot lookups, pooled lookups (same fp32 add
order as the oracle), unique rows and segment membership; fp32 tolerance for the MFMA
interaction and chunked update sums; one bf16 rounding for bf16 outputs.
"""
import numpy as np
import pytest
import torch

import oracle
from helpers import assert_close, julia_isapprox, rand_indices, rand_tables

pytestmark = pytest.mark.gpu


def dev_tables(tables, device, dtype=torch.float32):
    if dtype == torch.bfloat16:
        return [torch.from_numpy(oracle.bf16_to_f32(oracle.f32_to_bf16(t))).to(device).to(torch.bfloat16)
                for t in tables]
    return [torch.from_numpy(t).to(device) for t in tables]


def to_np_bits(t):
    """device tensor -> numpy (bf16 as uint16 bit patterns, fp32 as float32)"""
    t = t.detach().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def to_np_f32(t):
    return t.detach().float().cpu().numpy()


# ------------------------------------------------------------------ golden (HDF5) vectors
@pytest.mark.parametrize("kind", ["single", "multi"])
def test_golden_full_step(pkg, gpu, golden, kind):
    """test/integration.jl + src/validation.jl on the GPU: lookup -> interaction -> backward ->
    SGD(η=10), against the PyTorch goldens of the reference."""
    g = golden[kind]
    T, N, D = g["emb"].shape
    B, d = g["mlp_bottom"].shape
    L = int(g["L"])
    tables = pkg.EmbeddingTableSet(dev_tables(list(g["emb"]), gpu))
    idx = pkg.PackedIndices(torch.from_numpy(g["idx"]).reshape(T, B, L).to(gpu))
    x = torch.from_numpy(g["mlp_bottom"]).to(gpu)
    strategy = pkg.PreallocationStrategy(d)
    ys = pkg.maplookup(strategy, tables, idx, index_base=0)
    got = to_np_f32(ys[:, d:]).reshape(B, T, D)
    if L == 1:
        assert np.array_equal(got, g["concatenated"][:, 1:, :])
    else:
        assert_close(got, g["concatenated"][:, 1:, :], rtol=1e-6, what="pooled lookup vs PyTorch")
        ref = np.zeros((B, d + T * D), dtype=np.float32)
        oracle.maplookup(list(g["emb"]), g["idx"], 0, B, L, ref, d)
        assert np.array_equal(got, ref[:, d:].reshape(B, T, D))  # same add order: bit-exact
    dot = pkg.DotInteraction()
    out, back = pkg.rrule(dot, x, ys)
    o = to_np_f32(out)
    assert np.array_equal(o[:, :d], g["mlp_bottom"])
    assert_close(o[:, d:], g["zflat"], rtol=1e-5, what="zflat")
    assert julia_isapprox(o, g["output_interaction"])
    dout = torch.from_numpy(g["d_output_interaction"]).to(gpu)
    _, dx, dy = back(dout)
    grads = pkg.maplookup_pullback(d, tables, idx, dy)
    pkg.update_(pkg.Descent(float(g["lr"])), tables, grads, index_base=0)
    for t in range(T):
        rows = g[f"upd_rows_{t}"]
        new = to_np_f32(tables[t].data)
        assert_close(new[rows], g[f"upd_vals_{t}"], rtol=1e-5, what=f"update_emb_{t}")
        untouched = np.setdiff1d(np.arange(N), rows)
        assert np.array_equal(new[untouched], g["emb"][t][untouched])


# ------------------------------------------------------------------ lookup
@pytest.mark.parametrize("dim", [4, 8, 16, 32, 64, 128, 256, 12])
@pytest.mark.parametrize("lookups", [1, 3])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_lookup_vs_oracle(pkg, gpu, dim, lookups, dtype):
    rng = np.random.default_rng(dim * 10 + lookups)
    rows = [5, 1000, 3, 77]
    B = 37
    tabs = rand_tables(rng, rows, dim)
    idx = rand_indices(rng, rows, B, lookups)
    dt = dev_tables(tabs, gpu, dtype)
    P = 8 if dtype == torch.bfloat16 else 4
    out = pkg.maplookup(pkg.PreallocationStrategy(P), dt, torch.from_numpy(idx).reshape(len(rows), B, lookups).to(gpu),
                        index_base=0)
    ref_tabs = [to_np_bits(t) for t in dt]
    ref = np.zeros((B, P + dim * len(rows)), dtype=ref_tabs[0].dtype)
    oracle.maplookup(ref_tabs, idx, 0, B, lookups, ref, P)
    assert np.array_equal(to_np_bits(out)[:, P:], ref[:, P:])


@pytest.mark.parametrize("ntab", [31, 33, 40])
@pytest.mark.parametrize("lookups", [1, 5])
def test_lookup_table_pointer_forms(pkg, gpu, ntab, lookups):
    """<= 32 tables: pointers by value in the kernel arguments; more: descriptor loads (lookup.hip)."""
    rng = np.random.default_rng(ntab * 7 + lookups)
    rows = [int(r) for r in rng.integers(1, 3000, ntab)]
    B = 203
    tabs = rand_tables(rng, rows, 128)
    idx = rand_indices(rng, rows, B, lookups)
    dt = dev_tables(tabs, gpu)
    out = pkg.maplookup(pkg.PreallocationStrategy(128), dt, torch.from_numpy(idx).reshape(ntab, B, lookups).to(gpu),
                        index_base=0)
    ref = np.zeros((B, 128 * (ntab + 1)), dtype=np.float32)
    oracle.maplookup(tabs, idx, 0, B, lookups, ref, 128)
    assert np.array_equal(to_np_f32(out)[:, 128:], ref[:, 128:])
    bad = idx.copy().reshape(ntab, B * lookups)
    bad[ntab - 1, B * lookups // 2] = rows[ntab - 1]  # one out-of-range index in the last table
    with pytest.raises(pkg.BoundsError):
        pkg.maplookup(pkg.PreallocationStrategy(128), dt, torch.from_numpy(bad).reshape(ntab, B, lookups).to(gpu),
                      index_base=0)


@pytest.mark.parametrize("itype", [torch.int32, torch.int64])
@pytest.mark.parametrize("base", [0, 1])
def test_lookup_index_types_and_base(pkg, gpu, itype, base):
    rng = np.random.default_rng(3)
    rows = [50, 60]
    tabs = rand_tables(rng, rows, 16)
    idx = rand_indices(rng, rows, 64, 2)
    out = pkg.maplookup(pkg.PreallocationStrategy(0), dev_tables(tabs, gpu),
                        torch.from_numpy(idx + base).to(itype).reshape(2, 64, 2).to(gpu), index_base=base)
    ref = np.zeros((64, 32), dtype=np.float32)
    oracle.maplookup(tabs, idx, 0, 64, 2, ref, 0)
    assert np.array_equal(to_np_f32(out), ref)


def test_lookup_default_strategy_and_lookup(pkg, gpu):
    rng = np.random.default_rng(11)
    tabs = rand_tables(rng, [9, 10], 8)
    idx = [torch.tensor([1, 9, 3]), torch.tensor([10, 1, 1])]  # Julia 1-based
    res = pkg.maplookup(pkg.DefaultStrategy(), dev_tables(tabs, gpu), idx)
    assert np.array_equal(to_np_f32(res[0]), tabs[0][[0, 8, 2]])
    assert np.array_equal(to_np_f32(res[1]), tabs[1][[9, 0, 0]])
    one = pkg.lookup(dev_tables(tabs, gpu)[0], torch.tensor([2, 2]))
    assert np.array_equal(to_np_f32(one), tabs[0][[1, 1]])


def test_lookup_bounds_error(pkg, gpu):
    tabs = dev_tables([np.ones((5, 16), dtype=np.float32)], gpu)
    for bad in ([0, 6], [1, 7], [-3, 2]):
        with pytest.raises(pkg.BoundsError):
            pkg.maplookup(pkg.DefaultStrategy(), tabs, [torch.tensor(bad)])  # 1-based: 0, 6, 7, -3 invalid
    # the error state is cleared after being reported
    res = pkg.maplookup(pkg.DefaultStrategy(), tabs, [torch.tensor([1, 5])])
    assert np.array_equal(to_np_f32(res[0]), np.ones((2, 16), dtype=np.float32))


def test_lookup_empty_batch(pkg, gpu):
    tabs = dev_tables([np.ones((5, 16), dtype=np.float32)], gpu)
    out = pkg.maplookup(pkg.PreallocationStrategy(16), tabs, [torch.zeros(0, dtype=torch.int64)])
    assert out.shape == (0, 32)


# ------------------------------------------------------------------ interaction
@pytest.mark.parametrize("d,F,B", [(16, 8, 128), (4, 4, 4), (128, 27, 300), (32, 17, 65), (64, 33, 20),
                                   (16, 1, 5), (16, 2, 9), (8, 65, 7), (12, 5, 10), (128, 100, 3),
                                   (128, 50, 33), (256, 65, 19), (64, 96, 5), (256, 40, 7)])
def test_interaction_fwd_bwd_vs_oracle(pkg, gpu, d, F, B):
    rng = np.random.default_rng(d * 1000 + F)
    x = rng.standard_normal((B, d)).astype(np.float32)
    ys = np.zeros((B, F * d), dtype=np.float32)
    ys[:, d:] = rng.standard_normal((B, (F - 1) * d)).astype(np.float32)
    ref_ys = ys.copy()
    ref = oracle.interact_fwd(x, ref_ys, F)
    gys = torch.from_numpy(ys).to(gpu)
    dot = pkg.DotInteraction()
    out, back = pkg.rrule(dot, torch.from_numpy(x).to(gpu), gys)
    assert np.array_equal(to_np_f32(gys), ref_ys)  # fast_vcat
    o = to_np_f32(out)
    assert np.array_equal(o[:, :d], x)
    scale = float(np.abs(ys).max() ** 2 * d)
    assert_close(o, ref, rtol=2e-6, scale=scale, what="interaction fwd")
    dout = rng.standard_normal(ref.shape).astype(np.float32)
    rdx, rdt = oracle.interact_bwd(dout, ref_ys, d, F)
    _, dx, dt = back(torch.from_numpy(dout).to(gpu))
    scale_b = float(np.abs(dout).max() * np.abs(ys).max() * F)
    assert_close(to_np_f32(dt), rdt, rtol=2e-6, scale=scale_b, what="dt")
    assert_close(to_np_f32(dx), rdx, rtol=2e-6, scale=scale_b, what="dx")


@pytest.mark.parametrize("d,F,B", [(128, 27, 64), (16, 8, 33), (32, 17, 9)])
def test_interaction_bf16(pkg, gpu, d, F, B):
    rng = np.random.default_rng(5)
    x = oracle.f32_to_bf16(rng.standard_normal((B, d)).astype(np.float32))
    ys = oracle.f32_to_bf16(rng.standard_normal((B, F * d)).astype(np.float32))
    ref_ys = ys.copy()
    ref = oracle.interact_fwd(x, ref_ys, F)  # fp32 accumulate, one rounding
    tx = torch.from_numpy(x.view(np.int16)).to(gpu).view(torch.bfloat16)
    tys = torch.from_numpy(ys.view(np.int16)).to(gpu).view(torch.bfloat16)
    out, back = pkg.rrule(pkg.DotInteraction(), tx, tys)
    o = oracle.bf16_to_f32(to_np_bits(out))
    r = oracle.bf16_to_f32(ref)
    assert np.array_equal(to_np_bits(out)[:, :d], x)
    assert_close(o, r, rtol=8e-3, scale=float(np.abs(r).max()), what="bf16 fwd")
    dout = oracle.f32_to_bf16(rng.standard_normal(ref.shape).astype(np.float32))
    rdx, rdt = oracle.interact_bwd(dout, ref_ys, d, F)
    tdout = torch.from_numpy(dout.view(np.int16)).to(gpu).view(torch.bfloat16)
    _, dx, dt = back(tdout)
    assert dt.dtype == torch.float32 and dx.dtype == torch.float32  # dot_back returns fp32 (:419-424)
    s = float(np.abs(rdt).max())
    assert_close(to_np_f32(dt), rdt, rtol=2e-6, scale=s, what="bf16 dt")
    assert_close(to_np_f32(dx), rdx, rtol=2e-6, scale=s, what="bf16 dx")


def test_interaction_model_kat(pkg, gpu, kat):
    m = kat["model"]
    x = torch.tensor(m["bottom_mlp_output"], dtype=torch.float32, device=gpu)
    tabs = [torch.tensor(t, dtype=torch.float32, device=gpu) for t in m["tables"]]
    idx = [torch.tensor(i) + 1 for i in m["sparse_idx0"]]  # model.jl:117 adds 1
    ys = pkg.maplookup(pkg.PreallocationStrategy(4), tabs, idx)
    for t in range(3):
        np.testing.assert_allclose(to_np_f32(ys[:, 4 + 4 * t:8 + 4 * t]), np.array(m["embedding_outputs"][t]), atol=1e-6)
    out = pkg.DotInteraction()(x, ys)
    np.testing.assert_allclose(to_np_f32(out), np.array(m["interaction_output"]), atol=1e-4)


# ------------------------------------------------------------------ indexer + update
def _np_segments(idx_row):
    rows = np.unique(idx_row)
    order = np.argsort(idx_row, kind="stable")
    return rows, order


@pytest.mark.parametrize("rows,B,L,zipf", [([3, 4, 10, 1000, 5_000_000], 2048, 1, None), ([1000, 7, 20000], 300, 10, None),
                                           ([2], 1, 1, None), ([100000, 3], 5000, 1, None), ([256, 257, 70000], 2048, 1, None),
                                           ([300, 100000, 5_000_000], 2048, 1, 1.1), ([100000, 1000], 4000, 2, 1.2),
                                           ([0x10000, 0x1000000], 1500, 1, None),
                                           # hash build (N > 4096): all-distinct, tiny, skewed, pooled
                                           ([3, 4, 10, 1000, 5_000_000], 8192, 1, None),
                                           ([1_000_000, 1_000_000, 3], 2048, 10, 1.2),
                                           ([2, 100000, 33_000_000], 16384, 1, None),
                                           ([5000], 4097, 1, 1.05), ([1], 6000, 1, None),
                                           ([64] * 3, 300, 20, None), ([3, 70000, 1000], 8193, 1, 1.1),
                                           ([2, 100000, 33_000_000], 8192, 1, None)])
def test_indexer_segments_bit_exact(pkg, gpu, rows, B, L, zipf):
    """Both sort strategies (1 pass + bucket rank; full LSD radix on skewed rows), LDS and
    global-scratch variants: unique rows and per-row positions must match numpy exactly."""
    rng = np.random.default_rng(B + L)
    idx = rand_indices(rng, rows, B, L, zipf=zipf)
    tabs = pkg.EmbeddingTableSet([torch.zeros((n, 16), device=gpu) for n in rows])
    ix = pkg.SparseIndexer(len(rows), B * L, gpu)
    ix.build(tabs, torch.from_numpy(idx).reshape(len(rows), B, L).to(gpu), index_base=0)
    _assert_segments(ix, idx, B * L)


@pytest.mark.parametrize("rows,B,zipf", [("kaggle", 2048, None), ([300, 100000, 3, 5_000_000], 2048, 1.1),
                                         ([1, 2, 7, 0x1000001], 1000, None), ([5], 1, None)])
def test_step_fwd_indexer_parts(pkg, gpu, rows, B, zipf):
    """The forward launch's indexer sorts each table as parts split by the row's low bits
    (IndexerDev::vshift); read back through dlrm_indexer_read, the parts merge into the same
    segments a whole-table build gives."""
    if rows == "kaggle":
        rows = pkg.KAGGLE_EMBEDDING_SIZES
    D = 32
    rng = np.random.default_rng(B + 17)
    idx = rand_indices(rng, rows, B, 1, zipf=zipf)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(rand_tables(rng, rows, D), gpu)), B, 1, lr=0.1, index_base=0)
    assert hp.step_api
    x = torch.randn((B, D), device=gpu)
    hp.step_fwd(x, pkg.PackedIndices(torch.from_numpy(idx).to(torch.int32).to(gpu)))
    torch.cuda.synchronize()
    _assert_segments(hp.indexer, idx, B)


@pytest.mark.parametrize("rows,B,zipf,case", [
    ("kaggle", 2048, None, ""), ("kaggle", 8192, None, ""),          # tiny tables overflow the pool at 8192
    ([3, 4, 10, 1000, 5_000_000], 16384, None, ""), ([300, 100000, 3, 5_000_000], 6000, 1.1, ""),
    ([500, 2000, 1_000_000], 16384, 1.5, ""),                          # hot rows: multi-row parts in HBM
    ([1], 16384, None, ""), ([0x10000, 0x1000000], 3000, None, ""), ([7, 70000], 2049, None, ""),
    ([1000], 16384, None, "one-part"),                                 # every index in one part: 8 rows
    ([5000, 3], 4100, 1.05, ""),
    ([300, 100000, 3, 5_000_000], 6000, 1.1, "int64"),                # int64 indices: the rounds form
    ([3, 1000, 40, 5_000_000], 32768, None, ""),                      # 256 parts per table (scan, 16 waves)
    ([1_000_000] * 3, 20480, 1.2, ""),                                 # configs[4]'s positions, Zipf hot rows
    ([70000, 9], 30000, 1.05, "int64"),                               # 32768-class rounds form (16 rounds)
    ([1000], 32768, None, "one-part")])                               # every index in one part of 256
def test_wave_prepare_segments(pkg, gpu, rows, B, zipf, case):
    """dlrm_indexer_prepare (the wave build: 16 parts per 2048 positions; above 2048 the scan build --
    int32 indices, N % 4 == 0 -- else rounds of 2048 positions; parts that overflow a workgroup's LDS
    pool sorted in HBM) up to 32768 positions per table: unique rows and per-row positions exactly
    numpy's, every once-hit flag right.  The parts of a table are packed back to back (round 6's
    compact layout: each part's entries at its table's offset + the positions of the parts below it)."""
    if rows == "kaggle":
        rows = pkg.KAGGLE_EMBEDDING_SIZES
    rng = np.random.default_rng(B + len(rows) + 3)
    idx = rand_indices(rng, rows, B, 1, zipf=zipf)
    if case == "one-part":  # rows 5 + P k: all in part 5 of P (128 at 16384, 256 at 32768)
        P = 128 if B <= 16384 else 256
        idx = (5 + P * rng.integers(0, 1000 // P, size=(1, B))).astype(idx.dtype)
    tabs = pkg.EmbeddingTableSet([torch.zeros((n, 16), device=gpu) for n in rows])
    ix = pkg.SparseIndexer(len(rows), B, gpu)
    itype = torch.int64 if case == "int64" else torch.int32
    assert ix.prepare(tabs, torch.from_numpy(idx).to(itype).to(gpu), index_base=0)
    tabs.ctx.check_bounds()
    _assert_segments(ix, idx, B)
    if B <= 2048:  # the same segments with 32 and 64 parts per table (dlrm_indexer_set_parts)
        for parts in (32, 64):
            ix.set_parts(parts)
            assert ix.prepare(tabs, torch.from_numpy(idx).to(itype).to(gpu), index_base=0)
            _assert_segments(ix, idx, B)


@pytest.mark.parametrize("rows,B,table,where,value,itype,zipf", [
    ([3, 5000, 100000], 2048, 1, 77, "over", torch.int32, None),        # one round (N <= 2048)
    ([3, 5000, 100000], 2049, 1, -1, "over", torch.int32, None),        # rounds (N % 4 != 0), last chunk
    ([3, 5000, 100000], 8192, 1, 5000, "negative", torch.int32, None),  # the scan build
    ([3, 5000, 100000], 16384, 1, 0, "over", torch.int32, None),
    ([300, 100000, 3, 5_000_000], 6000, 3, 4321, "over", torch.int64, None),  # int64: the rounds form
    ([3, 5000], 4100, 0, 17, "over", torch.int32, None),               # a tiny table: DIRECT parts
    ([500, 2000, 1_000_000], 16384, 0, 9000, "negative", torch.int32, 1.5),  # hot rows: parts in HBM (G)
])
def test_wave_prepare_bounds(pkg, gpu, rows, B, table, where, value, itype, zipf):
    """dlrm_indexer_prepare with an out-of-range index (past the last row, or negative) in every
    form of the wave build: wave_build_group (one round, rounds, int64), wave_build_group_scan,
    a DIRECT tiny table, a workgroup sorting in HBM (G).  ADVICE r5: the build itself does not
    raise the ctx's flag (it may run beside a step whose kernels read that flag to decide their
    writes); the apply of the prepared indexer (a prebuilt update_) raises BoundsError and writes
    no row.  The word is cleared by the next prepare: a clean batch then updates normally."""
    rng = np.random.default_rng(B + table)
    idx = rand_indices(rng, rows, B, 1, zipf=zipf)
    good = idx.copy()
    idx[table, where] = rows[table] if value == "over" else -1
    D = 16
    tabs = pkg.EmbeddingTableSet([torch.zeros((n, D), device=gpu) for n in rows])
    ix = pkg.SparseIndexer(len(rows), B, gpu)
    tabs.ctx.check_bounds()
    bad = torch.from_numpy(idx).to(itype).to(gpu)
    assert ix.prepare(tabs, bad, index_base=0)
    tabs.ctx.check_bounds()  # (no raise: the build leaves the ctx's flag alone)
    dy = torch.ones((B, len(rows) * D), device=gpu)
    grads = pkg.maplookup_pullback(0, tabs, bad, dy)
    with pytest.raises(pkg.BoundsError):
        pkg.update_(pkg.Descent(0.5), tabs, grads, ix, index_base=0, prebuilt=True)
    for t in tabs:
        assert not t.data.any()  # no row written
    ok = torch.from_numpy(good).to(itype).to(gpu)
    assert ix.prepare(tabs, ok, index_base=0)
    pkg.update_(pkg.Descent(0.5), tabs, pkg.maplookup_pullback(0, tabs, ok, dy), ix, index_base=0, prebuilt=True)
    for t, n in enumerate(rows):
        cnt = np.bincount(good[t], minlength=n).astype(np.float32)
        assert np.array_equal(to_np_f32(tabs[t].data), np.repeat(-0.5 * cnt[:, None], D, axis=1))


def test_step_next_bad_index_in_next_batch_only(pkg, gpu):
    """HotPath.step_next builds the NEXT batch's indexer on a side stream beside the
    current step.  An out-of-range index in that next batch must not freeze the current step (its
    once-hit rows are written by the backward, which reads the ctx's flag): the current step's
    tables equal a plain step bit for bit and no BoundsError is raised yet; the next step raises it
    and writes nothing."""
    rows, D, B = [3, 40, 100000, 7, 2_000_000], 64, 2048
    rng = np.random.default_rng(5)
    tabs = rand_tables(rng, rows, D)
    good_np = rand_indices(rng, rows, B, 1)
    bad_np = rand_indices(rng, rows, B, 1)
    bad_np[2, 1234] = rows[2] + 1
    good = pkg.PackedIndices(torch.from_numpy(good_np).to(torch.int32).to(gpu))
    bad = pkg.PackedIndices(torch.from_numpy(bad_np).to(torch.int32).to(gpu))
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = len(rows) + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32)).to(gpu)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=0.25, index_base=0, pipeline="side")
    hp.step_next(x, good, dout, bad)
    torch.cuda.synchronize()
    hp.check_bounds()  # the bad batch has not been looked up yet
    ref = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=0.25, index_base=0)
    ref.step(x, good, dout)
    torch.cuda.synchronize()
    for a, b in zip(hp.ts, ref.ts):
        assert torch.equal(a.data, b.data)
    before = [t.data.clone() for t in hp.ts]
    hp.step_next(x, bad, dout, good)
    with pytest.raises(pkg.BoundsError):
        hp.check_bounds()
    for a, b in zip(hp.ts, before):
        assert torch.equal(a.data, b)


def test_prepared_step_equals_fresh_step_and_bounds(pkg, gpu):
    """dlrm_indexer_prepare -> dlrm_step_fwd (gather only: the indexer is prepared) ->
    dlrm_step_bwd equals a step whose forward builds its own indexer, bit for bit; an out-of-range
    index in the prepared batch raises BoundsError and leaves every table unchanged."""
    rows, D, B = [3, 40, 100000, 7, 2_000_000], 64, 2048
    rng = np.random.default_rng(61)
    tabs = rand_tables(rng, rows, D)
    idx_np = rand_indices(rng, rows, B, 1)
    p = pkg.PackedIndices(torch.from_numpy(idx_np).to(torch.int32).to(gpu))
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = len(rows) + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32)).to(gpu)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=0.25, index_base=0)
    assert hp.indexer.prepare(hp.ts, p, index_base=0)
    assert hp.indexer.state() & pkg._lib.IX_PREPARED
    hp.step_fwd(x, p)
    hp.step_bwd(dout, x=x, idx=p)
    torch.cuda.synchronize()
    hp.check_bounds()
    ref = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=0.25, index_base=0)
    ref.step(x, p, dout)
    torch.cuda.synchronize()
    assert torch.equal(hp.out, ref.out) and torch.equal(hp.dx, ref.dx)
    for a, b in zip(hp.ts, ref.ts):
        assert torch.equal(a.data, b.data)
    bad_np = idx_np.copy()
    bad_np[2, 77] = rows[2] + 9
    bad = pkg.PackedIndices(torch.from_numpy(bad_np).to(torch.int32).to(gpu))
    hp2 = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=0.25, index_base=0)
    assert hp2.indexer.prepare(hp2.ts, bad, index_base=0)
    hp2.step_fwd(x, bad)
    hp2.step_bwd(dout, x=x, idx=bad)
    with pytest.raises(pkg.BoundsError):
        hp2.check_bounds()
    for t in range(len(rows)):
        assert np.array_equal(to_np_f32(hp2.ts[t].data), tabs[t]), f"table {t} was written on a BoundsError step"


@pytest.mark.parametrize("rows,B,L,zipf,case", [
    ([1_000_000] * 6, 2048, 10, 1.2, ""),          # configs[4]'s bags: 20480 positions per table, Zipf(1.2)
    ([3, 1000, 40, 5_000_000], 3000, 8, None, ""),  # 24000: tiny tables (one row per part), uniform
    ([7, 100_000], 4096, 8, 1.05, ""),              # 32768: the largest wave build
    ([1_000_000] * 2, 1000, 9, 1.2, ""),            # 9000: N % 256 != 0
    ([1_000_000], 2048, 10, None, "two-hot"),       # two hot rows in one part: the general HBM sort
    ([1_000_000], 2048, 10, None, "hot+300")])      # a hot row + ~380 others: LDS counting passes
def test_bag_wave_build_segments(pkg, gpu, rows, B, L, zipf, case):
    """dlrm_indexer_build of pooled bags with 8192 < B L <= 32768 positions per table: the bag build
    (round 6: count, place by part, per-part sort, a streamed hot-row prefix for parts too big for
    LDS; it replaced the hash build for configs[4]) groups the positions p = b L + k exactly as
    numpy does; then a prebuilt update_ (the apply maps p to its bag) equals the closed-form
    scatter-add of integer bag gradients on every touched row, and writes no other row."""
    rng = np.random.default_rng(B * L + len(rows))
    idx = rand_indices(rng, rows, B, L, zipf=zipf)
    if case == "two-hot":  # rows 7 and 7 + 3 * 256: both in part 7 of 256, a third of the positions each
        idx[0, 0::3] = 7
        idx[0, 1::3] = 7 + 3 * 256
    elif case == "hot+300":  # row 9 at a fifth of the positions, 300 more distinct rows of part 9
        idx[0, 0::5] = 9
        idx[0, 1:1501:5] = 9 + 256 * rng.choice(np.arange(1, 3900), size=300, replace=False)
    D = 16
    tabs = pkg.EmbeddingTableSet([torch.zeros((n, D), device=gpu) for n in rows])
    ix = pkg.SparseIndexer(len(rows), B * L, gpu)
    p = pkg.PackedIndices(torch.from_numpy(idx).to(torch.int32).to(gpu).reshape(len(rows), B, L))
    ix.build(tabs, p, index_base=0)
    tabs.ctx.check_bounds()
    _assert_segments(ix, idx, B * L)
    gi = torch.from_numpy(rng.integers(-4, 5, size=(B, len(rows) * D)).astype(np.float32)).to(gpu)
    pkg.update_(pkg.Descent(1.0), tabs, pkg.maplookup_pullback(0, tabs, p, gi), ix, index_base=0, prebuilt=True)
    gh = gi.cpu().numpy()
    for t, n in enumerate(rows):
        ref = np.zeros((n, D), dtype=np.float64)
        np.add.at(ref, idx[t], np.repeat(gh[:, t * D:(t + 1) * D], L, axis=0))
        assert np.array_equal(to_np_f32(tabs[t].data), (-ref).astype(np.float32))


@pytest.mark.parametrize("itype,base", [(torch.int64, 0), (torch.int32, 1)])
def test_bag_build_int64_base_and_bounds(pkg, gpu, itype, base):
    """The bag build (dlrm_indexer_build above 8192 positions per table) with int64 indices and with
    1-based ones (the reference's): segments exactly numpy's; then one index past the end and one
    below the base: the build leaves them out and raises the bounds flag, the prebuilt update writes
    no row and raises BoundsError, as every dlrm_indexer_build does."""
    rows, B, L, D = [3, 70000, 1_000_000], 1100, 9, 16
    rng = np.random.default_rng(41)
    idx = rand_indices(rng, rows, B, L, zipf=1.1)
    tabs = pkg.EmbeddingTableSet([torch.zeros((n, D), device=gpu) for n in rows])
    ix = pkg.SparseIndexer(len(rows), B * L, gpu)
    p = pkg.PackedIndices(torch.from_numpy(idx + base).to(itype).to(gpu).reshape(len(rows), B, L))
    ix.build(tabs, p, index_base=base)
    tabs.ctx.check_bounds()
    _assert_segments(ix, idx, B * L)
    bad = idx + base
    bad[1, 5000] = rows[1] + base
    bad[2, 77] = base - 1
    pb = pkg.PackedIndices(torch.from_numpy(bad).to(itype).to(gpu).reshape(len(rows), B, L))
    ix.build(tabs, pb, index_base=base)
    gi = torch.ones((B, len(rows) * D), device=gpu)
    with pytest.raises(pkg.BoundsError):
        pkg.update_(pkg.Descent(1.0), tabs, pkg.maplookup_pullback(0, tabs, pb, gi), ix, index_base=base,
                    prebuilt=True)
        tabs.ctx.check_bounds()
    for t in tabs:
        assert not t.data.any()  # no row written


def test_indexer_footprint_compact(pkg, gpu):
    """the wave builds' per-part arrays are packed per table (round 6), so an indexer of
    26 tables x 16384 positions holds its 128-part build in a few hundred bytes per position
    (round 5: ~7 GB after the first such build), and it does not grow when that build runs."""
    rows = pkg.KAGGLE_EMBEDDING_SIZES
    N = 16384
    ix = pkg.SparseIndexer(len(rows), N, gpu)
    before = ix.nbytes()
    assert before < len(rows) * N * 600, before
    tabs = pkg.EmbeddingTableSet([torch.zeros((n, 16), device=gpu) for n in rows])
    idx = rand_indices(np.random.default_rng(3), rows, N, 1)
    assert ix.prepare(tabs, torch.from_numpy(idx).to(torch.int32).to(gpu), index_base=0)
    tabs.ctx.check_bounds()
    assert ix.nbytes() == before
    _assert_segments(ix, idx, N)


def _assert_segments(ix, idx, N):
    """One segment per distinct row (segment order unspecified), holding exactly that row's
    positions in ascending order (vectorised: large-N builds have ~N segments per table)."""
    for t in range(idx.shape[0]):
        got_rows, pos, seg = ix.segments(t)
        got_rows, pos, seg = np.asarray(got_rows, dtype=np.int64), np.asarray(pos), np.asarray(seg)
        order = np.argsort(idx[t], kind="stable")
        urows, starts, counts = np.unique(idx[t][order], return_index=True, return_counts=True)
        assert len(got_rows) == len(urows) and seg[-1] == N and len(seg) == len(urows) + 1
        assert np.array_equal(np.sort(got_rows), urows)
        k = np.searchsorted(urows, got_rows)
        assert np.array_equal(np.diff(seg), counts[k])
        want = order[np.repeat(starts[k] - seg[:-1], counts[k]) + np.arange(N)]
        assert np.array_equal(pos, want)


@pytest.mark.parametrize("rows,B,zipf", [([3, 4, 10, 1000, 5_000_000], 2048, None), ([300, 100000, 5_000_000], 2048, 1.1),
                                         ([256, 257, 70000], 2048, None), ([0x10000, 0x1000000], 1500, None),
                                         ([2], 1, None), ("kaggle", 2048, None), ([100000, 3], 5000, None),
                                         ([50] * 40, 512, None)])
def test_backward_built_indexer(pkg, gpu, rows, B, zipf):
    """dlrm_interact_bwd_gather with an indexer: the indexer built in the backward's launch
    (256-thread workgroups beside the backward's; or its own launch where the shape has no
    fused form: N > 2048, F > 32) groups positions exactly, and the backward is unchanged."""
    if rows == "kaggle":
        rows = pkg.KAGGLE_EMBEDDING_SIZES
    rng = np.random.default_rng(B + len(rows))
    D = 16
    idx = rand_indices(rng, rows, B, 1, zipf=zipf)
    tabs = pkg.EmbeddingTableSet([torch.randn((n, D), device=gpu) for n in rows])
    hp = pkg.HotPath(tabs, B, 1, index_base=0)
    assert not hp.materialize_ys
    p = pkg.PackedIndices(torch.from_numpy(idx).to(torch.int32).reshape(len(rows), B, 1).to(gpu))
    x = torch.randn((B, D), device=gpu)
    dout = torch.randn((B, hp.width), device=gpu)
    hp.interact_bwd(dout, x=x, idx=p)
    dx0, dt0 = hp.dx.clone(), hp.dt.clone()
    hp.interact_bwd(dout, x=x, idx=p, build_indexer=True)
    torch.cuda.synchronize()
    hp.check_bounds()
    assert torch.equal(hp.dx, dx0) and torch.equal(hp.dt, dt0)
    _assert_segments(hp.indexer, idx, B)


@pytest.mark.parametrize("dim", [16, 128, 256, 8, 12])
@pytest.mark.parametrize("L", [1, 4])
def test_sgd_update_vs_oracle(pkg, gpu, dim, L):
    rng = np.random.default_rng(dim + 100 * L)
    rows = [3, 4, 27, 1000, 200000]
    B = 1024
    tabs = rand_tables(rng, rows, dim)
    idx = rand_indices(rng, rows, B, L)
    Pd = 16
    grad = rng.standard_normal((B, Pd + dim * len(rows))).astype(np.float32)
    ref = [t.copy() for t in tabs]
    uniq = oracle.sgd_update(ref, idx, 0, B, L, grad, Pd, 0.5)
    ts = pkg.EmbeddingTableSet(dev_tables(tabs, gpu))
    pidx = pkg.PackedIndices(torch.from_numpy(idx).reshape(len(rows), B, L).to(gpu))
    grads = pkg.maplookup_pullback(Pd, ts, pidx, torch.from_numpy(grad).to(gpu))
    ix = pkg.SparseIndexer(len(rows), B * L, gpu)
    pkg.update_(pkg.Descent(0.5), ts, grads, ix, index_base=0)
    for t in range(len(rows)):
        assert len(ix.unique_rows(t)) == uniq[t]
        assert sorted(ix.unique_rows(t)) == np.unique(idx[t]).tolist()
        new = to_np_f32(ts[t].data)
        touched = np.unique(idx[t])
        # hot rows (3-row table: ~340 hits each) are summed in 32-position chunks: tolerance
        scale = 0.5 * np.abs(grad).max() * B * L
        assert_close(new[touched], ref[t][touched], rtol=1e-6, scale=scale, what=f"table {t}")
        untouched = np.setdiff1d(np.arange(rows[t]), touched)
        assert np.array_equal(new[untouched], tabs[t][untouched])


@pytest.mark.parametrize("rows,B,L,zipf", [([3, 1000, 1_000_000], 2048, 10, 1.2), ([7, 200000], 8192, 1, None)])
def test_sgd_update_hash_build_vs_oracle(pkg, gpu, rows, B, L, zipf):
    """update! with B*L > 4096 positions per table (the hash-built indexer) against the oracle."""
    rng = np.random.default_rng(B * L)
    D, Pd = 64, 8
    tabs = rand_tables(rng, rows, D)
    idx = rand_indices(rng, rows, B, L, zipf=zipf)
    grad = rng.standard_normal((B, Pd + D * len(rows))).astype(np.float32)
    ref = [t.copy() for t in tabs]
    uniq = oracle.sgd_update(ref, idx, 0, B, L, grad, Pd, 0.25)
    ts = pkg.EmbeddingTableSet(dev_tables(tabs, gpu))
    pidx = pkg.PackedIndices(torch.from_numpy(idx).reshape(len(rows), B, L).to(gpu))
    ix = pkg.SparseIndexer(len(rows), B * L, gpu)
    pkg.update_(pkg.Descent(0.25), ts, pkg.maplookup_pullback(Pd, ts, pidx, torch.from_numpy(grad).to(gpu)), ix,
                index_base=0)
    torch.cuda.synchronize()
    for t in range(len(rows)):
        assert len(ix.unique_rows(t)) == uniq[t]
        new = to_np_f32(ts[t].data)
        touched = np.unique(idx[t])
        assert_close(new[touched], ref[t][touched], rtol=1e-6, scale=0.25 * np.abs(grad).max() * B * L,
                     what=f"table {t}")
        untouched = np.setdiff1d(np.arange(rows[t]), touched)
        assert np.array_equal(new[untouched], tabs[t][untouched])


@pytest.mark.parametrize("B", [6000, 9000])
def test_hash_build_bounds_error_and_reuse(pkg, gpu, B):
    """Large-N builds (the hash build beyond 4096 positions): an out-of-range index is
    skipped and flagged; the next build with the same indexer (hash slots reset by the
    previous build) is exact again."""
    rows = [10, 50000]
    rng = np.random.default_rng(11)
    idx = rand_indices(rng, rows, B, 1)
    bad = idx.copy()
    bad[1, 17] = rows[1] + 5
    bad[0, 4000] = -1
    tabs = pkg.EmbeddingTableSet([torch.zeros((n, 16), device=gpu) for n in rows])
    ix = pkg.SparseIndexer(len(rows), B, gpu)
    ix.build(tabs, torch.from_numpy(bad).reshape(2, B, 1).to(gpu), index_base=0)
    torch.cuda.synchronize()
    with pytest.raises(pkg.BoundsError):
        tabs.ctx.check_bounds()
    for t, p in ((0, 4000), (1, 17)):
        got_rows, pos, seg = ix.segments(t)
        assert p not in pos and seg[-1] == B - 1
    for k in range(3):
        idx2 = rand_indices(rng, rows, B, 1)
        ix.build(tabs, torch.from_numpy(idx2).reshape(2, B, 1).to(gpu), index_base=0)
        _assert_segments(ix, idx2, B)


def test_sgd_update_bitwise_deterministic_and_atomic_close(pkg, gpu):
    rng = np.random.default_rng(99)
    rows = [3, 10, 100000]
    B, D = 4096, 128
    tabs = rand_tables(rng, rows, D)
    idx = torch.from_numpy(rand_indices(rng, rows, B, 1)).to(gpu)
    grad = torch.from_numpy(rng.standard_normal((B, D * len(rows))).astype(np.float32)).to(gpu)
    results = []
    for mode in ("det", "det", "atomic"):
        ts = pkg.EmbeddingTableSet(dev_tables(tabs, gpu))
        p = pkg.PackedIndices(idx)
        grads = pkg.maplookup_pullback(0, ts, p, grad)
        pkg.update_(pkg.Descent(0.1), ts, grads, index_base=0, deterministic=(mode == "det"))
        results.append([to_np_f32(t.data) for t in ts])
    for a, b in zip(results[0], results[1]):
        assert np.array_equal(a, b)  # bitwise reproducible
    for a, c in zip(results[0], results[2]):
        assert_close(c, a, rtol=1e-6, scale=0.1 * 4.0 * B, what="atomic vs deterministic")


def test_sgd_update_integer_gradients_exact(pkg, gpu):
    """Exactly representable sums: order cannot matter, so GPU == closed form bit for bit."""
    rng = np.random.default_rng(5)
    rows = [3, 50, 10000]
    B, D, L = 2048, 32, 2
    tabs = [np.zeros((n, D), dtype=np.float32) for n in rows]
    idx = rand_indices(rng, rows, B, L)
    grad = rng.integers(-8, 8, size=(B, D * len(rows))).astype(np.float32)
    ts = pkg.EmbeddingTableSet(dev_tables(tabs, gpu))
    p = pkg.PackedIndices(torch.from_numpy(idx).reshape(3, B, L).to(gpu))
    pkg.update_(pkg.Descent(1.0), ts, pkg.maplookup_pullback(0, ts, p, torch.from_numpy(grad).to(gpu)), index_base=0)
    for t, n in enumerate(rows):
        want = np.zeros((n, D))
        np.add.at(want, idx[t], np.repeat(grad[:, t * D:(t + 1) * D], L, axis=0))
        assert np.array_equal(to_np_f32(ts[t].data), (-want).astype(np.float32))


@pytest.mark.parametrize("deterministic", [True, False])
def test_update_bounds_error(pkg, gpu, deterministic):
    """An out-of-range index: Julia's checked gather throws BoundsError at maplookup
    (model.jl:161), before update!, so the tables stay untouched -- not even the valid index's
    row is written.  After the error is reported the flag is clear and updates apply again."""
    ts = pkg.EmbeddingTableSet([torch.zeros((4, 16), device=gpu)])
    p = pkg.PackedIndices([torch.tensor([1, 5])])
    g = torch.ones((2, 16), device=gpu)
    with pytest.raises(pkg.BoundsError):
        pkg.update_(pkg.Descent(1.0), ts, pkg.maplookup_pullback(0, ts, p, g), deterministic=deterministic)
    assert not to_np_f32(ts[0].data).any()
    ok = pkg.PackedIndices([torch.tensor([1, 1])])
    pkg.update_(pkg.Descent(1.0), ts, pkg.maplookup_pullback(0, ts, ok, g), deterministic=deterministic)
    ts.ctx.check_bounds()
    assert to_np_f32(ts[0].data)[0].tolist() == [-2.0] * 16  # index_base 1: row 0, hit twice


@pytest.mark.parametrize("B", [512, 6000])
def test_step_bounds_error_leaves_tables(pkg, gpu, B):
    """The training step (dlrm_step_fwd / dlrm_step_bwd, once-hit rows updated inside the backward)
    with one out-of-range index: BoundsError, and no table row changes (the reference throws in
    maplookup, model.jl:161, before any update!)."""
    rng = np.random.default_rng(9)
    rows = [5, 300, 100000]
    D = 32
    tabs = rand_tables(rng, rows, D)
    idx_np = rand_indices(rng, rows, B, 1)
    idx_np[2, B // 3] = rows[2] + 7  # out of range
    ts = pkg.EmbeddingTableSet(dev_tables(tabs, gpu))
    hp = pkg.HotPath(ts, B, 1, lr=0.1, index_base=0)
    p = pkg.PackedIndices(torch.from_numpy(idx_np).to(torch.int32).to(gpu).reshape(3, B, 1))
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    dout = torch.from_numpy(rng.standard_normal((B, hp.width)).astype(np.float32)).to(gpu)
    hp.step(x, p, dout)
    with pytest.raises(pkg.BoundsError):
        hp.check_bounds()
    for t in range(3):
        assert np.array_equal(to_np_f32(ts[t].data), tabs[t]), f"table {t} was written on a BoundsError step"


# ------------------------------------------------------------------ the engine
@pytest.mark.parametrize("overlap,materialize", [(False, False), (False, True), (True, False), (True, True)])
def test_hotpath_step_matches_operator_sequence(pkg, gpu, overlap, materialize):
    """The engine (fused forward; backward from a materialized ys or re-gathered rows) equals
    the reference-shaped operator sequence bit for bit."""
    rng = np.random.default_rng(1)
    rows = [10, 3000, 7, 100000]
    D, B = 32, 512
    tabs = rand_tables(rng, rows, D)
    idx = torch.from_numpy(rand_indices(rng, rows, B, 1)).to(torch.int32).to(gpu)
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = len(rows) + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32)).to(gpu)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=0.25, index_base=0,
                     overlap_indexer=overlap, materialize_ys=materialize)
    p = pkg.PackedIndices(idx)
    hp.step(x, p, dout)
    torch.cuda.synchronize()
    hp.check_bounds()
    # same thing through the reference-shaped operator API
    ts2 = pkg.EmbeddingTableSet(dev_tables(tabs, gpu))
    ys = pkg.maplookup(pkg.PreallocationStrategy(D), ts2, p, index_base=0)
    out, back = pkg.rrule(pkg.DotInteraction(), x, ys)
    _, dx, dy = back(dout)
    pkg.update_(pkg.Descent(0.25), ts2, pkg.maplookup_pullback(D, ts2, p, dy), index_base=0)
    assert np.array_equal(to_np_f32(hp.out), to_np_f32(out))
    assert np.array_equal(to_np_f32(hp.dx), to_np_f32(dx))
    m = _dt_written_mask(idx.cpu().numpy(), D) if hp.step_api else slice(None)
    assert np.array_equal(to_np_f32(hp.dt)[m], to_np_f32(dy)[m])
    for a, b in zip(hp.ts, ts2):
        assert np.array_equal(to_np_f32(a.data), to_np_f32(b.data))


def _dt_written_mask(idx, D):
    """[B][F*D] bool: the dt entries dlrm_step_bwd must write -- the rows of positions whose table
    row is hit more than once (once-hit rows are updated in place; the x rows' gradient is dx, and
    the split step backward leaves dt's x rows unwritten)."""
    T, B = idx.shape
    keep = np.ones((B, T + 1), dtype=bool)
    keep[:, 0] = False
    for t in range(T):
        _, inv, cnt = np.unique(idx[t], return_inverse=True, return_counts=True)
        keep[:, t + 1] = cnt[inv] > 1
    return np.repeat(keep, D, axis=1)


@pytest.mark.parametrize("rows,D,B,zipf,dtype", [
    ([10, 3000, 7, 100000], 32, 512, None, torch.float32),            # F = 5: one 16-row block
    ("kaggle", 16, 2048, None, torch.float32),                         # F = 27, N = 2048: split form
    ([3, 4, 10, 1000, 5_000_000], 128, 2048, 1.1, torch.float32),      # hot rows (multi-slice segments)
    ([5, 100000, 3, 77] * 6 + [9, 10], 128, 300, None, torch.bfloat16),
    ([300, 100000, 5_000_000], 64, 3000, None, torch.float32),         # N > 2048: unsplit fallback
    ([300, 100000, 3, 5_000_000], 64, 3000, 1.1, torch.float32),       # 2048 < N <= 4096: split in-LDS build
    ([300, 100000, 3, 5_000_000], 64, 6000, 1.1, torch.float32),       # N > 4096: split hash build
    ([5, 100000, 3, 77] * 6 + [9, 10], 128, 8192, None, torch.bfloat16),  # configs[2] shape (bf16, B=8192)
    ([50] * 40, 32, 200, None, torch.float32),                         # F = 41: unsplit fallback
    ([50] * 40, 32, 6000, None, torch.float32),                        # F = 41, N > 4096: unsplit hash build
    ([1], 16, 64, None, torch.float32),                                # every position hits one row
    ([10, 3000, 7, 100000, 3], 256, 512, 1.2, torch.float32),          # 1-KB rows: 4 chunks per lane group
    ([10, 3000, 7, 100000, 3] * 3, 8, 37, 1.1, torch.bfloat16),        # d <= 64: one backward wave per sample
    ([10, 3000, 7, 100000], 4, 101, None, torch.float32),              # d = 4, partial last block
    ([30, 500, 7, 20000] * 5, 48, 77, 1.1, torch.float32)])            # d = 48: 3/4 of the super-block
def test_step_api_matches_operator_sequence(pkg, gpu, rows, D, B, zipf, dtype):
    """dlrm_step_fwd / dlrm_step_bwd (indexer built in the forward's launch, once-hit rows
    updated inside the backward) == maplookup -> DotInteraction -> dot_back -> update!
    bit for bit: out, dx, the updated tables, and every dt row the apply reads."""
    if rows == "kaggle":
        rows = pkg.KAGGLE_EMBEDDING_SIZES
    rng = np.random.default_rng(B + D)
    T = len(rows)
    idx_np = rand_indices(rng, rows, B, 1, zipf=zipf)
    tabs = [rng.uniform(-1, 1, size=(n, D)).astype(np.float32) for n in rows]
    idx = torch.from_numpy(idx_np).to(torch.int32).to(gpu)
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu).to(dtype)
    F = T + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32)).to(gpu).to(dtype)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu, dtype)), B, 1, lr=0.5, index_base=0)
    assert hp.step_api
    p = pkg.PackedIndices(idx)
    for _ in range(2):  # two steps: the second reads rows the first updated
        hp.step(x, p, dout)
    torch.cuda.synchronize()
    hp.check_bounds()
    ts2 = pkg.EmbeddingTableSet(dev_tables(tabs, gpu, dtype))
    for _ in range(2):
        ys = pkg.maplookup(pkg.PreallocationStrategy(D), ts2, p, index_base=0)
        out, back = pkg.rrule(pkg.DotInteraction(), x, ys)
        _, dx, dy = back(dout)
        pkg.update_(pkg.Descent(0.5), ts2, pkg.maplookup_pullback(D, ts2, p, dy), index_base=0)
    torch.cuda.synchronize()
    assert np.array_equal(to_np_bits(hp.out), to_np_bits(out))
    assert np.array_equal(to_np_f32(hp.dx), to_np_f32(dx))
    m = _dt_written_mask(idx_np, D)
    assert np.array_equal(to_np_f32(hp.dt)[m], to_np_f32(dy)[m])
    for a, b in zip(hp.ts, ts2):
        assert np.array_equal(to_np_bits(a.data), to_np_bits(b.data))


def _operator_steps(pkg, tabs, gpu, dtype, D, p, x, dout, lr, nsteps):
    """The reference's operator sequence (maplookup -> DotInteraction -> dot_back -> update!)."""
    ts = pkg.EmbeddingTableSet(dev_tables(tabs, gpu, dtype))
    for _ in range(nsteps):
        ys = pkg.maplookup(pkg.PreallocationStrategy(D), ts, p, index_base=0)
        out, back = pkg.rrule(pkg.DotInteraction(), x, ys)
        _, dx, dy = back(dout)
        pkg.update_(pkg.Descent(lr), ts, pkg.maplookup_pullback(D, ts, p, dy), index_base=0)
    return ts, out, dx


def test_split_backward_then_prebuilt_update_steps_each_row_once(pkg, gpu):
    """dlrm_step_bwd(BWD_ONLY) updates the once-hit rows itself; a following
    dlrm_sgd_update(PREBUILT) with the same split indexer must then apply only the repeated rows
    (it stepped the once-hit rows a second time from dt rows never written)."""
    rows, D, B = [3, 40, 100000, 7, 2_000_000], 128, 512
    rng = np.random.default_rng(11)
    tabs = rand_tables(rng, rows, D)
    idx_np = rand_indices(rng, rows, B, 1)
    p = pkg.PackedIndices(torch.from_numpy(idx_np).to(torch.int32).to(gpu))
    x = torch.randn((B, D), device=gpu)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=0.5, index_base=0)
    dout = torch.randn((B, hp.width), device=gpu)
    hp.dt.fill_(float("nan"))  # once-hit rows' dt entries stay unwritten: reading one poisons the table
    hp.step_fwd(x, p)
    hp.step_bwd(dout, x=x, idx=p, flags=pkg._lib.STEP_BWD_ONLY)
    hp.sgd_update(p, prebuilt=True)
    torch.cuda.synchronize()
    ts_ref, out, dx = _operator_steps(pkg, tabs, gpu, torch.float32, D, p, x, dout, 0.5, 1)
    torch.cuda.synchronize()
    assert np.array_equal(to_np_f32(hp.dx), to_np_f32(dx))
    for a, b in zip(hp.ts, ts_ref):
        assert np.array_equal(to_np_f32(a.data), to_np_f32(b.data))


def test_prepare_with_unaligned_x_updates_once_hit_rows(pkg, gpu):
    """dlrm_step_bwd_prepare after dlrm_indexer_build_split with an x whose rows are not 16-B
    aligned (no split backward for it, so the apply must take the once-hit rows too): every row is
    stepped (the apply launch that carried the next build had no once-hit items; such
    shapes now take the plain step and leave the next build to the next forward)."""
    rows, D, B = [5, 300, 100000, 9, 1_000_000], 16, 256
    rng = np.random.default_rng(12)
    tabs = rand_tables(rng, rows, D)
    batches = [pkg.PackedIndices(torch.from_numpy(rand_indices(rng, rows, B, 1)).to(torch.int32).to(gpu))
               for _ in range(2)]
    xs = torch.randn((B, D + 1), device=gpu)
    x = xs[:, 1:]  # row stride D + 1: not 16-B aligned
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=0.25, index_base=0)
    dout = torch.randn((B, hp.width), device=gpu)
    nxt = pkg.SparseIndexer(len(rows), B, gpu)
    hp.build_split(hp.indexer, batches[0])
    hp.step_bwd(dout, x=x, idx=batches[0], prepare=(nxt, batches[1]))
    torch.cuda.synchronize()
    hp.check_bounds()
    ts = pkg.EmbeddingTableSet(dev_tables(tabs, gpu))
    ys = pkg.maplookup(pkg.PreallocationStrategy(D), ts, batches[0], index_base=0)
    _, back = pkg.rrule(pkg.DotInteraction(), x.contiguous(), ys)
    _, dx, dy = back(dout)
    pkg.update_(pkg.Descent(0.25), ts, pkg.maplookup_pullback(D, ts, batches[0], dy), index_base=0)
    torch.cuda.synchronize()
    np.testing.assert_allclose(to_np_f32(hp.dx), to_np_f32(dx), rtol=1e-5, atol=1e-6)
    for a, b in zip(hp.ts, ts):
        np.testing.assert_allclose(to_np_f32(a.data), to_np_f32(b.data), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("rows,D,B,lr_known", [
    ("kaggle", 128, 2048, True), ("kaggle", 128, 2048, False),   # the BASELINE metric shape
    ([3, 4000, 9, 200000, 12], 16, 512, True), ([3, 4000, 9, 200000, 12], 16, 512, False)])
def test_drop_in_operator_chain_on_step_kernels(pkg, gpu, rows, D, B, lr_known):
    """The reference's unchanged operator chain (maplookup -> rrule(DotInteraction) -> pullback ->
    maplookup_pullback -> update!) on HipTables runs the training-step kernels (3 launches, ys never
    written) and equals HotPath.step bit for bit: out, dx, every table, over two steps.  The small
    cases pass Julia's 1-based indices with every default left alone (HipTables, maplookup and
    update_ all default to index_base = 1); the Kaggle case passes 0-based ones explicitly."""
    base = 0 if rows == "kaggle" else 1
    if rows == "kaggle":
        rows = pkg.KAGGLE_EMBEDDING_SIZES
    rng = np.random.default_rng(B + D)
    T = len(rows)
    tabs = [rng.uniform(-0.05, 0.05, size=(n, D)).astype(np.float32) for n in rows]
    idxs = [pkg.PackedIndices(torch.from_numpy(rand_indices(rng, rows, B, 1) + base).to(torch.int32).to(gpu))
            for _ in range(2)]
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = T + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32) * 1e-2).to(gpu)
    lr = 0.25
    kw = {"index_base": 0} if base == 0 else {}
    ht = pkg.HipTables(dev_tables(tabs, gpu), lr=lr if lr_known else None, **kw)
    dot = pkg.DotInteraction()
    for p in idxs:
        ys = pkg.maplookup(pkg.PreallocationStrategy(D), ht, p, **kw)
        assert isinstance(ys, pkg.LazyLookup) and ys.shape == (B, D + T * D)
        out, back = pkg.rrule(dot, x, ys)
        _, dx, dy = back(dout)
        assert dy.applied == lr_known
        pkg.update_(pkg.Descent(lr), ht, pkg.maplookup_pullback(D, ht, p, dy), **kw)
    torch.cuda.synchronize()
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=lr, index_base=base)
    for p in idxs:
        hp.step(x, p, dout)
    torch.cuda.synchronize()
    assert np.array_equal(to_np_f32(out), to_np_f32(hp.out))
    assert np.array_equal(to_np_f32(dx), to_np_f32(hp.dx))
    for a, b in zip(ht.ts, hp.ts):
        assert np.array_equal(to_np_f32(a.data), to_np_f32(b.data))
    # an index base other than the tables' own is refused, not silently shifted
    with pytest.raises(ValueError):
        pkg.maplookup(pkg.PreallocationStrategy(D), ht, idxs[0], index_base=1 - base)
    if lr_known:  # the pullback stepped the once-hit rows with η: update! must use the same η
        ys = pkg.maplookup(pkg.PreallocationStrategy(D), ht, idxs[0])
        _, back = pkg.rrule(dot, x, ys)
        _, _, dy = back(dout)
        with pytest.raises(ValueError):
            pkg.update_(pkg.Descent(lr * 2), ht, pkg.maplookup_pullback(D, ht, idxs[0], dy), **kw)
        # a second pullback of the same forward would step the once-hit rows twice: refused
        with pytest.raises(pkg.DLRMError) as e:
            back(dout)
        assert e.value.code == pkg._lib.E_STATE


def test_drop_in_chain_deferred_update(pkg, gpu):
    """update!(opt, tables, grads, indexers) -- the reference's own call, no extra keyword -- on
    HipTables with a known η defers its apply launch to the next maplookup, which runs it together
    with the build of its own batch's indexer (the pipelined step): over three steps out, dx and
    every table equal HotPath.step bit for bit, a read of the tables runs the pending update first,
    and the second and third forwards found their indexer prepared."""
    rows, D, B = pkg.KAGGLE_EMBEDDING_SIZES, 128, 2048
    rng = np.random.default_rng(41)
    T = len(rows)
    tabs = [rng.uniform(-0.05, 0.05, size=(n, D)).astype(np.float32) for n in rows]
    idxs = [pkg.PackedIndices(torch.from_numpy(rand_indices(rng, rows, B, 1)).to(torch.int32).to(gpu))
            for _ in range(3)]
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = T + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32) * 1e-2).to(gpu)
    lr = 0.25
    ht = pkg.HipTables(dev_tables(tabs, gpu), lr=lr, index_base=0)
    dot = pkg.DotInteraction()
    used = []
    for p in idxs:
        ys = pkg.maplookup(pkg.PreallocationStrategy(D), ht, p)
        used.append(ht.hotpath(B).indexer)
        out, back = pkg.rrule(dot, x, ys)
        _, dx, dy = back(dout)
        pkg.update_(pkg.Descent(lr), ht, pkg.maplookup_pullback(D, ht, p, dy), pkg.SparseIndexer(T, B, gpu),
                    num_splits=8, nthreads=12)
        assert ht._pending is not None  # deferred
    got = [to_np_f32(t.data) for t in ht.ts]  # the read runs the last pending update
    assert ht._pending is None
    assert used[1] is not used[0] and used[2] is used[0]  # two indexers alternate (prepared forwards)
    torch.cuda.synchronize()
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=lr, index_base=0)
    for p in idxs:
        hp.step(x, p, dout)
    torch.cuda.synchronize()
    assert np.array_equal(to_np_f32(out), to_np_f32(hp.out))
    assert np.array_equal(to_np_f32(dx), to_np_f32(hp.dx))
    for a, b in zip(got, hp.ts):
        assert np.array_equal(a, to_np_f32(b.data))
    ht.hotpath(B).check_bounds()


def test_default_strategy_lookup_after_a_deferred_update(pkg, gpu):
    """a DefaultStrategy maplookup (test/model/embedding_update.jl:31) right after a
    deferred update! must see that update applied, as the reference's update! writes the tables in
    place before it returns (train.jl:283-290).  The Julia shim flushes in _maplookup; the Python
    mirror through HipTables.ts.  Checked against the same steps on HotPath, bit for bit."""
    rows, D, B = [3, 50, 1000, 100000], 16, 256
    rng = np.random.default_rng(7)
    T = len(rows)
    tabs = [rng.uniform(-0.05, 0.05, size=(n, D)).astype(np.float32) for n in rows]
    idxs = [pkg.PackedIndices(torch.from_numpy(rand_indices(rng, rows, B, 1)).to(torch.int32).to(gpu))
            for _ in range(2)]
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = T + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32) * 1e-2).to(gpu)
    lr = 0.5
    ht = pkg.HipTables(dev_tables(tabs, gpu), lr=lr, index_base=0)
    dot = pkg.DotInteraction()
    for p in idxs:
        ys = pkg.maplookup(pkg.PreallocationStrategy(D), ht, p)
        _, back = pkg.rrule(dot, x, ys)
        _, _, dy = back(dout)
        pkg.update_(pkg.Descent(lr), ht, pkg.maplookup_pullback(D, ht, p, dy), pkg.SparseIndexer(T, B, gpu),
                    num_splits=8, nthreads=12)
    assert ht._pending is not None  # deferred
    got = pkg.maplookup(pkg.DefaultStrategy(), ht, idxs[0])
    assert ht._pending is None
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=lr, index_base=0)
    for p in idxs:
        hp.step(x, p, dout)
    torch.cuda.synchronize()
    i0 = idxs[0].data.reshape(T, B).cpu().numpy()
    for t in range(T):
        want = to_np_f32(hp.ts[t].data)[i0[t]]
        assert np.array_equal(to_np_f32(got[t]), want)


@pytest.mark.parametrize("sync_before_next", [True, False])
def test_drop_in_chain_deferred_bounds_error(pkg, gpu, sync_before_next):
    """The deferred update! keeps the reference's bounds outcome without a per-step host sync: a
    batch with one out-of-range index raises BoundsError at a later maplookup (from the flag
    snapshot, no GPU call) or at check_bounds, and no row of that step -- nor of any step queued
    after it -- is written: the tables equal one good step.  After the error the chain trains on."""
    rows, D, B = [3, 40, 100000, 7, 2_000_000], 64, 512
    rng = np.random.default_rng(43)
    T = len(rows)
    tabs = [rng.uniform(-0.05, 0.05, size=(n, D)).astype(np.float32) for n in rows]
    good = rand_indices(rng, rows, B, 1)
    bad = rand_indices(rng, rows, B, 1)
    bad[2, B // 2] = rows[2] + 5
    p_good = pkg.PackedIndices(torch.from_numpy(good).to(torch.int32).to(gpu))
    p_bad = pkg.PackedIndices(torch.from_numpy(bad).to(torch.int32).to(gpu))
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = T + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32) * 1e-2).to(gpu)
    lr = 0.5
    ht = pkg.HipTables(dev_tables(tabs, gpu), lr=lr, index_base=0)
    dot = pkg.DotInteraction()

    def chain(p):
        ys = pkg.maplookup(pkg.PreallocationStrategy(D), ht, p)
        _, back = pkg.rrule(dot, x, ys)
        _, _, dy = back(dout)
        pkg.update_(pkg.Descent(lr), ht, pkg.maplookup_pullback(D, ht, p, dy))

    chain(p_good)
    chain(p_bad)
    assert ht._pending is not None
    if sync_before_next:  # the snapshot has landed: the next maplookup raises without a GPU call
        torch.cuda.synchronize()
    raised = False
    try:  # (without the sync the host may run ahead: the step queues and writes nothing)
        chain(p_good)
    except pkg.BoundsError:
        raised = True
    assert raised or not sync_before_next
    if not raised:
        with pytest.raises(pkg.BoundsError):
            ht.check_bounds()
    assert ht._pending is None
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=lr, index_base=0)
    hp.step(x, p_good, dout)
    torch.cuda.synchronize()
    for a, b in zip(ht.ts, hp.ts):  # (ts: flushed and checked -- clean now)
        assert np.array_equal(to_np_f32(a.data), to_np_f32(b.data)), "a row of a BoundsError step was written"
    chain(p_good)  # the flag is clear: the chain trains again
    hp.step(x, p_good, dout)
    torch.cuda.synchronize()
    for a, b in zip(ht.ts, hp.ts):
        assert np.array_equal(to_np_f32(a.data), to_np_f32(b.data))


def test_lazy_lookup_interacted_after_a_deferred_update(pkg, gpu):
    """a LazyLookup made before a deferred update! and interacted after it reads the
    updated tables (the pending apply runs first) and the update is not lost: two steps in this
    order equal two HotPath steps."""
    rows, D, B = [3, 40, 100000, 7], 32, 256
    rng = np.random.default_rng(44)
    T = len(rows)
    tabs = [rng.uniform(-0.05, 0.05, size=(n, D)).astype(np.float32) for n in rows]
    p0, p1 = (pkg.PackedIndices(torch.from_numpy(rand_indices(rng, rows, B, 1)).to(torch.int32).to(gpu))
              for _ in range(2))
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = T + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32) * 1e-2).to(gpu)
    ht = pkg.HipTables(dev_tables(tabs, gpu), lr=0.5, index_base=0)
    dot = pkg.DotInteraction()
    ys0 = pkg.maplookup(pkg.PreallocationStrategy(D), ht, p0)
    _, back = pkg.rrule(dot, x, ys0)
    _, _, dy = back(dout)
    ys1_early = pkg.LazyLookup(ht, p1, D)  # made while nothing is pending ...
    pkg.update_(pkg.Descent(0.5), ht, pkg.maplookup_pullback(D, ht, p0, dy))
    assert ht._pending is not None  # ... and interacted after the deferred update!
    out1, back = pkg.rrule(dot, x, ys1_early)
    _, dx1, dy = back(dout)
    pkg.update_(pkg.Descent(0.5), ht, pkg.maplookup_pullback(D, ht, p1, dy))
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=0.5, index_base=0)
    hp.step(x, p0, dout)
    hp.step(x, p1, dout)
    torch.cuda.synchronize()
    assert np.array_equal(to_np_f32(out1), to_np_f32(hp.out))
    assert np.array_equal(to_np_f32(dx1), to_np_f32(hp.dx))
    for a, b in zip(ht.ts, hp.ts):
        assert np.array_equal(to_np_f32(a.data), to_np_f32(b.data))


def test_step_api_state_and_bounds(pkg, gpu):
    """The forward's split indexer also drives the plain update (once-hit rows included, bit for
    bit the update of a fresh build); step_bwd needs step_fwd's indices; an out-of-range index
    raises BoundsError and the step still matches the operator sequence on the valid positions."""
    rows, D, B = [100, 7, 5000], 16, 256
    rng = np.random.default_rng(3)
    tabs = rand_tables(rng, rows, D)
    idx_np = rand_indices(rng, rows, B, 1)
    idx = torch.from_numpy(idx_np).to(torch.int32).to(gpu)
    x = torch.randn((B, D), device=gpu)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=1.0, index_base=0)
    dout = torch.randn((B, hp.width), device=gpu)
    p = pkg.PackedIndices(idx)
    hp.step_fwd(x, p)
    g = torch.randn((B, hp.F * D), device=gpu)
    hp.dt.copy_(g)
    hp.sgd_update(p, prebuilt=True)
    ts_ref = pkg.EmbeddingTableSet(dev_tables(tabs, gpu))
    pkg.update_(pkg.Descent(1.0), ts_ref, pkg.maplookup_pullback(D, ts_ref, p, g), index_base=0)
    for a, b in zip(hp.ts, ts_ref):
        assert np.array_equal(to_np_f32(a.data), to_np_f32(b.data))
    other = pkg.PackedIndices(idx.clone())
    with pytest.raises(pkg.DLRMError) as e:
        hp.step_bwd(dout, x=x, idx=other)
    assert e.value.code == pkg._lib.E_STATE
    hp.step_bwd(dout, x=x, idx=p)
    torch.cuda.synchronize()
    hp.check_bounds()
    # out-of-range: flagged; no table row is written (by the step or by the operators: the
    # reference's gather throws before update!), and out / dx agree on the valid positions
    bad_np = idx_np.copy()
    bad_np[1, 5] = rows[1] + 3
    bad = pkg.PackedIndices(torch.from_numpy(bad_np).to(torch.int32).to(gpu))
    hp2 = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, 1, lr=1.0, index_base=0)
    hp2.step(x, bad, dout)
    with pytest.raises(pkg.BoundsError):
        hp2.check_bounds()
    ts2 = pkg.EmbeddingTableSet(dev_tables(tabs, gpu))
    ys = pkg.maplookup(pkg.PreallocationStrategy(D), ts2, bad, index_base=0, check_bounds=False)
    out, back = pkg.rrule(pkg.DotInteraction(), x, ys)
    _, dx, dy = back(dout)
    pkg.update_(pkg.Descent(1.0), ts2, pkg.maplookup_pullback(D, ts2, bad, dy), index_base=0, check_bounds=False)
    with pytest.raises(pkg.BoundsError):  # the operators flagged it too (and this clears the flag)
        ts2.ctx.check_bounds()
    assert np.array_equal(to_np_f32(hp2.out), to_np_f32(out))
    assert np.array_equal(to_np_f32(hp2.dx), to_np_f32(dx))
    for a, b in zip(hp2.ts, ts2):
        assert np.array_equal(to_np_f32(a.data), to_np_f32(b.data))


# ------------------------------------------------------------------ full-size properties
def test_full_size_properties_metric_config(pkg, gpu):
    """BASELINE metric shape (26 Kaggle tables x 128 fp32, B=2048): properties that need no
    CPU oracle at 17 GB — row-encoded gather exactness, the interaction adjoint identity
    <dz, tri(T T')> == 1/2 <dT, T>, and an exact integer-gradient update."""
    rows = pkg.KAGGLE_EMBEDDING_SIZES
    D, B = 128, 2048
    T = len(rows)
    g = torch.Generator(device=gpu).manual_seed(0)
    # encode (table, row) into every element exactly: value = row mod 4093 + 4096 * t + c/128
    tabs = []
    for t, n in enumerate(rows):
        r = torch.arange(n, device=gpu, dtype=torch.float32).remainder_(4093).add_(4096.0 * t)
        tabs.append((r[:, None] + torch.arange(D, device=gpu, dtype=torch.float32)[None, :] / 128.0).contiguous())
    ts = pkg.EmbeddingTableSet(tabs)
    idx = torch.stack([torch.randint(0, n, (B,), device=gpu, generator=g) for n in rows]).to(torch.int32)
    ys = pkg.maplookup(pkg.PreallocationStrategy(D), ts, pkg.PackedIndices(idx), index_base=0)
    want = (idx.to(torch.float32).T.remainder(4093) + 4096.0 * torch.arange(T, device=gpu)[None, :])
    want = want[:, :, None] + torch.arange(D, device=gpu, dtype=torch.float32)[None, None, :] / 128.0
    assert torch.equal(ys[:, D:].reshape(B, T, D), want)
    # interaction adjoint identity on random data
    x = torch.randn((B, D), device=gpu, generator=g)
    ys2 = torch.randn((B, (T + 1) * D), device=gpu, generator=g) * 0.1
    out, back = pkg.rrule(pkg.DotInteraction(), x, ys2)
    dz = torch.randn(out.shape, device=gpu, generator=g)
    dz[:, :D] = 0
    _, dx, dt = back(dz)
    lhs = (dz[:, D:].double() * out[:, D:].double()).sum()
    rhs = 0.5 * (dt.double() * ys2.double()).sum()
    assert abs(lhs - rhs) <= 1e-5 * (dz.abs().double() * out.abs().double()).sum()
    # torch fp32 reference of the interaction at full size
    Tm = ys2.reshape(B, T + 1, D).double()
    Z = Tm @ Tm.transpose(1, 2)
    li, lj = torch.tril_indices(T + 1, T + 1, -1, device=gpu)
    assert torch.allclose(out[:, D:].double(), Z[:, li, lj], rtol=1e-5, atol=1e-5)
    # exact update with integer gradients on zeroed tables
    zt = pkg.EmbeddingTableSet([torch.zeros((n, D), device=gpu) for n in rows])
    gi = torch.randint(-4, 5, (B, D * T), device=gpu, generator=g).to(torch.float32)
    pidx = pkg.PackedIndices(idx)
    pkg.update_(pkg.Descent(1.0), zt, pkg.maplookup_pullback(0, zt, pidx, gi), index_base=0)
    for t in (0, 8, 2, 25):  # a 1460-row, a 3-row, a 10M-row and the last table
        ref = torch.zeros((rows[t], D), device=gpu, dtype=torch.float64)
        ref.index_add_(0, idx[t].long(), gi[:, t * D:(t + 1) * D].double())
        assert torch.equal(zt[t].data, (-ref).float())


# ------------------------------------------------------------------ fused lookup + interaction
@pytest.mark.parametrize("rows,D,B,L,dtype", [
    ([1000] * 7, 16, 128, 1, torch.float32), ([1000] * 7, 16, 128, 10, torch.float32),
    ([5, 100000, 3, 77] * 6 + [9, 10], 128, 300, 1, torch.float32), ([50] * 40, 32, 33, 3, torch.float32),
    ([5, 100000, 3, 77] * 6 + [9, 10], 128, 200, 1, torch.bfloat16), ([60] * 12, 64, 70, 4, torch.bfloat16),
    ([7] * 3, 4, 9, 2, torch.float32)])
def test_fused_lookup_interaction_equals_two_operators(pkg, gpu, rows, D, B, L, dtype):
    rng = np.random.default_rng(len(rows) * D + L)
    tabs = dev_tables(rand_tables(rng, rows, D), gpu, dtype)
    idx = torch.from_numpy(rand_indices(rng, rows, B, L)).reshape(len(rows), B, L).to(torch.int32).to(gpu)
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu).to(dtype)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(tabs), B, L, index_base=0, fused=True, materialize_ys=True)
    p = pkg.PackedIndices(idx)
    hp.validate(x, p)
    hp.forward(x, p)
    ys = pkg.maplookup(pkg.PreallocationStrategy(D), tabs, p, index_base=0)
    out = pkg.DotInteraction()(x, ys)
    torch.cuda.synchronize()
    hp.check_bounds()
    assert torch.equal(hp.ys, ys)    # lookup output + fast_vcat: bit-identical
    assert torch.equal(hp.out, out)  # same MFMA order: bit-identical


@pytest.mark.parametrize("T,D,B,dtype", [(40, 64, 37, torch.float32), (64, 256, 29, torch.float32),
                                         (50, 128, 21, torch.float32), (64, 256, 17, torch.bfloat16),
                                         (90, 64, 11, torch.float32)])
def test_ys_backward_equals_gather_backward(pkg, gpu, T, D, B, dtype):
    """33 <= F <= 96: dlrm_interact_bwd on a materialized ys (the split kernel's load plan, one wave
    per 64-column super-block) gives the bits of the re-gathering backward (bwd_body), whose MFMA
    sums it shares."""
    rng = np.random.default_rng(T * 7 + D)
    rows = [int(r) for r in rng.integers(2, 5000, T)]
    tabs = dev_tables(rand_tables(rng, rows, D), gpu, dtype)
    idx = pkg.PackedIndices(torch.from_numpy(rand_indices(rng, rows, B, 1)).reshape(T, B, 1).to(torch.int32).to(gpu))
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu).to(dtype)
    ts = pkg.EmbeddingTableSet(tabs)
    a = pkg.HotPath(ts, B, 1, index_base=0, fused=True, materialize_ys=True, deterministic=False)
    g = pkg.HotPath(ts, B, 1, index_base=0, fused=True, materialize_ys=False, deterministic=False)
    dout = (torch.randn((B, a.width), device=gpu) * 1e-2).to(dtype)
    a.forward(x, idx)
    g.forward(x, idx)
    a.interact_bwd(dout)
    g.interact_bwd(dout, x=x, idx=idx)
    torch.cuda.synchronize()
    a.check_bounds()
    assert torch.equal(a.out, g.out)
    assert torch.equal(a.dx, g.dx)
    assert torch.equal(a.dt, g.dt)  # x row included


def test_fused_bounds_error(pkg, gpu):
    tabs = [torch.ones((4, 16), device=gpu), torch.ones((4, 16), device=gpu)]
    hp = pkg.HotPath(pkg.EmbeddingTableSet(tabs), 2, 1, index_base=0, materialize_ys=True)
    x = torch.zeros((2, 16), device=gpu)
    hp.forward(x, pkg.PackedIndices(torch.tensor([[0, 1], [2, 4]], dtype=torch.int32, device=gpu)))
    with pytest.raises(pkg.BoundsError):
        hp.check_bounds()
    assert torch.equal(hp.ys[0, 16:], torch.ones(32, device=gpu))  # valid rows still gathered


def test_gather_backward_bounds_error(pkg, gpu):
    """The re-gathering backward validates indices like the forward (BoundsError, no fault)."""
    tabs = [torch.ones((4, 16), device=gpu), torch.ones((4, 16), device=gpu)]
    hp = pkg.HotPath(pkg.EmbeddingTableSet(tabs), 2, 1, index_base=0)
    assert not hp.materialize_ys
    x = torch.zeros((2, 16), device=gpu)
    bad = pkg.PackedIndices(torch.tensor([[0, 1], [2, 7]], dtype=torch.int32, device=gpu))
    hp.interact_bwd(torch.zeros((2, hp.width), device=gpu), x=x, idx=bad)
    with pytest.raises(pkg.BoundsError):
        hp.check_bounds()


def test_host_tensors_are_rejected_before_launch(pkg, gpu):
    x = torch.zeros((4, 16))
    ys = torch.zeros((4, 32), device=gpu)
    with pytest.raises(ValueError):
        pkg.DotInteraction()(x.to(gpu), ys, out=torch.zeros((4, 17)))
    hp = pkg.HotPath(pkg.EmbeddingTableSet([torch.zeros((5, 16), device=gpu)]), 4, 1, index_base=0)
    with pytest.raises(ValueError):
        hp.validate(x, pkg.PackedIndices(torch.zeros((1, 4), dtype=torch.int32)))


# ------------------------------------------------------------------ sharded (2 ranks on one GPU)
SHARD_CASES = {
    "small": dict(rows=[3, 5000, 70, 100000, 11], D=32, B=64, L=2, zipf=None),
    # Criteo-Terabyte's 26 row counts (criteo.jl:379-406) scaled by 1/20000 (floor 3), Zipf(1.05)
    # hot rows, one-hot: TablePartition.fitting at a capacity the contiguous halves exceed
    "terabyte-scaled": dict(rows=[max(3, n // 20000) for n in [
        227605432, 39060, 17295, 7424, 20265, 3, 7122, 1543, 63, 130229467, 3067956, 405282, 10,
        2209, 11938, 155, 4, 976, 14, 292775614, 40790948, 187188510, 590152, 12973, 108, 36]],
        D=32, B=256, L=1, zipf=1.05),
    # d = 128: the backward's send-layout stores from the two-waves-per-sample kernel
    "kaggle-scaled-d128": dict(rows=[1460, 583, 10131, 2202, 305, 24, 12517, 633, 3, 9314, 5683, 8351, 3194, 27,
                                     14992, 5461, 10, 5652, 2173, 4, 7046, 18, 15, 2861, 105, 1425],
                               D=128, B=128, L=1, zipf=None),
    # global batch 4096 (> 2048 positions per table): the sharded update's indexer is the scan wave build
    "kaggle-scaled-b4096": dict(rows=[1460, 583, 10131, 2202, 305, 24, 12517, 633, 3, 9314, 5683, 8351, 3194, 27,
                                      14992, 5461, 10, 5652, 2173, 4, 7046, 18, 15, 2861, 105, 1425],
                                D=32, B=2048, L=1, zipf=1.05),
}


def _shard_inputs(case, world):
    c = SHARD_CASES[case]
    rows, D, B, L = c["rows"], c["D"], c["B"], c["L"]
    T, Bg = len(rows), B * world
    rng = np.random.default_rng(7)
    tabs = rand_tables(rng, rows, D)
    idx = rand_indices(rng, rows, Bg, L, zipf=c["zipf"])
    x = rng.standard_normal((Bg, D)).astype(np.float32)
    F = T + 1
    dout = rng.standard_normal((Bg, D + F * (F - 1) // 2)).astype(np.float32)
    return rows, D, B, L, tabs, idx, x, dout


def _shard_owners(case, owners, world):
    if owners != "fitting":
        return owners
    from dlrm_jl_amd.sharded import TablePartition
    c = SHARD_CASES[case]
    rb = c["D"] * 4
    cap = int(0.56 * sum(c["rows"]) * rb)  # the contiguous halves need ~0.59 of the bytes (as at full size)
    part = TablePartition.fitting(c["rows"], world, rb, cap)
    assert not part.contiguous
    return part.owners


def _gpu_shard_worker(rank, world, port, outdir, owners=None, graphed=False, case="small", micro=1):
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import dlrm_pkg
    pkg = dlrm_pkg.load()
    from dlrm_jl_amd.sharded import HipShardOps, ShardedHotPath, TablePartition
    dev = torch.device("cuda:0")
    rows, D, B, L, tabs, idx, x, dout = _shard_inputs(case, world)
    T, Bg = len(rows), B * world
    part = TablePartition(T, world, _shard_owners(case, owners, world))
    mine = part.tables(rank)
    ops = HipShardOps([torch.from_numpy(tabs[t]).to(dev) for t in mine], Bg, L, 0.25, device=dev)
    eng = ShardedHotPath(ops, part, rank, B, D, L, torch.float32, dev, micro=micro)
    p = pkg.PackedIndices(torch.from_numpy(idx[mine]).to(torch.int32).reshape(len(mine), Bg, L).to(dev))
    sl = [eng.global_index(b) for b in range(B)]  # this rank's samples of the global batch
    xd, dd = torch.from_numpy(x[sl]).to(dev), torch.from_numpy(dout[sl]).to(dev)
    if graphed:  # the bench's form: compute segments replayed as hipGraphs around eager exchanges
        eng.capture(xd, [p], dd)
        eng.step_graphed(0)
    else:
        eng.step(xd, p, dd)
    torch.cuda.synchronize()
    ops.ctx.check_bounds()
    np.savez(os.path.join(outdir, f"g{rank}.npz"), out=eng.out.cpu().numpy(), dx=eng.dx.cpu().numpy(),
             **{f"t{t}": ops.ts[k].data.cpu().numpy() for k, t in enumerate(mine)})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("owners,graphed,case,micro", [
    (None, False, "small", 1), ([[4, 0, 2], [1, 3]], True, "small", 1), ("fitting", True, "terabyte-scaled", 1),
    (None, True, "kaggle-scaled-d128", 1), (None, True, "kaggle-scaled-b4096", 1),
    # micro-batches: exchange of one half overlapping the compute of the other (comm stream)
    (None, False, "small", 2), ([[4, 0, 2], [1, 3]], True, "small", 4), ("fitting", True, "terabyte-scaled", 2),
    (None, True, "kaggle-scaled-d128", 2)])
def test_sharded_two_ranks_equal_single_gpu_step(pkg, gpu, tmp_path, owners, graphed, case, micro):
    """The table-sharded step (HIP kernels, 2 ranks sharing the GPU, gloo exchange; contiguous,
    explicit or TablePartition.fitting's byte-balanced non-contiguous assignment; eager or
    hipGraph-segment launches) equals the single-GPU HotPath on the global batch bit for bit.
    "terabyte-scaled": configs[3]'s row counts (scaled), Zipf hot rows, the partition the
    Terabyte tables need at 2 GPUs."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    mp.start_processes(_gpu_shard_worker, args=(world, port, str(tmp_path), owners, graphed, case, micro),
                       nprocs=world, start_method="spawn")
    rows, D, B, L, tabs, idx, x, dout = _shard_inputs(case, world)
    T, Bg = len(rows), B * world
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), Bg, L, lr=0.25, index_base=0)
    p = pkg.PackedIndices(torch.from_numpy(idx).to(torch.int32).reshape(T, Bg, L).to(gpu))
    hp.step(torch.from_numpy(x).to(gpu), p, torch.from_numpy(dout).to(gpu))
    from dlrm_jl_amd.sharded import TablePartition
    part = TablePartition(T, world, _shard_owners(case, owners, world))
    Bm = B // micro
    for r in range(world):
        z = np.load(tmp_path / f"g{r}.npz")
        sl = [(b // Bm) * world * Bm + r * Bm + b % Bm for b in range(B)]
        assert np.array_equal(z["out"], to_np_f32(hp.out)[sl])
        assert np.array_equal(z["dx"], to_np_f32(hp.dx)[sl])
        for t in part.tables(r):
            assert np.array_equal(z[f"t{t}"], to_np_f32(hp.ts[t].data)), (r, t)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_exchange_layout_kernels(pkg, gpu, dtype):
    """dlrm_maplookup_blocked (lookup written straight into the [peer][table][b][D] send layout)
    == maplookup + the permute; dlrm_scatter_rows == the per-owner column scatter, bit for bit
    (16-B and element paths)."""
    from dlrm_jl_amd.sharded import HipShardOps
    rng = np.random.default_rng(21)
    rows, D, L, W, Bl = [10, 300, 5000], 32, 2, 3, 16
    T, Bg = len(rows), W * Bl
    tabs = rand_tables(rng, rows, D)
    idx = torch.from_numpy(rand_indices(rng, rows, Bg, L)).to(torch.int32).reshape(T, Bg, L).to(gpu)
    ops = HipShardOps(dev_tables(tabs, gpu, dtype), Bg, L, 0.1, device=gpu)
    p = pkg.PackedIndices(idx)
    ref = pkg.maplookup(pkg.PreallocationStrategy(0), ops.ts, p, index_base=0)
    out = torch.zeros(W * T * Bl * D, dtype=dtype, device=gpu)
    ops.lookup_blocked(p, out, D, Bl * D, Bl, T * Bl * D)
    want = ref.reshape(W, Bl, T, D).permute(0, 2, 1, 3).reshape(-1)
    assert np.array_equal(to_np_bits(out), to_np_bits(want))
    # scatter: owners [[2, 0], [1]] -> per-owner [B][T_j][D] blocks, plus an odd (unaligned) layout
    B, F = 24, T + 1
    src = torch.from_numpy(rng.standard_normal((B, F * D)).astype(np.float32)).to(gpu)
    for base, ld in (([D, 2 * B * D, 0], [2 * D, D, 2 * D]), ([1, 3 * B * D + 5, D + 2], [2 * D + 3, D, 2 * D + 3])):
        n = 4 * B * D + 64
        dst = torch.zeros(n, dtype=torch.float32, device=gpu)
        ops.scatter_rows(src, F * D, D, dst, torch.tensor(base, device=gpu), torch.tensor(ld, device=gpu), T, B, D)
        exp = np.zeros(n, dtype=np.float32)
        s_np = src.cpu().numpy()
        for b in range(B):
            for t in range(T):
                exp[base[t] + b * ld[t]: base[t] + b * ld[t] + D] = s_np[b, D + t * D: D + (t + 1) * D]
        assert np.array_equal(dst.cpu().numpy(), exp)


@pytest.mark.parametrize("mode", ["side", "apply"])
@pytest.mark.parametrize("rows,D,B,dtype,parts", [("kaggle", 128, 2048, torch.float32, None),
                                                  ("kaggle", 16, 2048, torch.float32, None),
                                                  ("kaggle", 16, 2048, torch.float32, 32),  # (the bench's D = 16 form)
                                                  ("kaggle", 128, 2048, torch.float32, 64),
                                                  ([300, 100000, 3, 5_000_000], 64, 6000, torch.float32, None),
                                                  # configs[2]'s shape: the in-apply wave build at 8192
                                                  ("kaggle", 128, 8192, torch.bfloat16, None),
                                                  ([3, 500, 100000, 2_000_000], 32, 16384, torch.float32, None),
                                                  ([5, 100000, 3, 77] * 6 + [9, 10], 128, 512, torch.bfloat16, None),
                                                  # Terabyte-shaped bf16 x 128 at B = 2048 (256-B rows: the
                                                  # bench builds 32 parts per table)
                                                  ([3, 200000, 60, 50000, 10, 100000] * 4 + [7, 30000], 128, 2048,
                                                   torch.bfloat16, 32)])
def test_pipelined_steps_match_operator_sequence(pkg, gpu, rows, D, B, dtype, parts, mode):
    """Pipelined steps (the next batch's split indexer built during the step: "side" =
    HotPath.step_next on a side stream, "apply" = HotPath.step_prep inside the apply launch, so
    the next forward only gathers; eager steps, then hipGraph-captured ones) == the operator
    sequence over the same batches, bit for bit; also with 32 and 64 parts per table
    (dlrm_indexer_set_parts: the same segments, so the same bits)."""
    if rows == "kaggle":
        rows = pkg.KAGGLE_EMBEDDING_SIZES
    rng = np.random.default_rng(B + 7)
    T = len(rows)
    tabs = [rng.uniform(-1, 1, size=(n, D)).astype(np.float32) for n in rows]
    packs = [pkg.PackedIndices(torch.from_numpy(rand_indices(rng, rows, B, 1, zipf=1.1)).to(torch.int32).to(gpu))
             for _ in range(3)]
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu).to(dtype)
    F = T + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32)).to(gpu).to(dtype)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu, dtype)), B, 1, lr=0.5, index_base=0, pipeline=mode,
                     parts=parts)
    assert hp.pipeline == mode
    step = hp.step_next if mode == "side" else hp.step_prep
    order = [0, 1, 2, 0]
    step(x, packs[0], dout, packs[1])
    step(x, packs[1], dout, packs[2])
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            step(x, packs[2], dout, packs[0])
            step(x, packs[0], dout, packs[1])
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    hp.check_bounds()
    ts2 = pkg.EmbeddingTableSet(dev_tables(tabs, gpu, dtype))
    for k in order:
        ys = pkg.maplookup(pkg.PreallocationStrategy(D), ts2, packs[k], index_base=0)
        out, back = pkg.rrule(pkg.DotInteraction(), x, ys)
        _, dx, dy = back(dout)
        pkg.update_(pkg.Descent(0.5), ts2, pkg.maplookup_pullback(D, ts2, packs[k], dy), index_base=0)
    torch.cuda.synchronize()
    assert np.array_equal(to_np_bits(hp.out), to_np_bits(out))
    assert np.array_equal(to_np_f32(hp.dx), to_np_f32(dx))
    for a, b in zip(hp.ts, ts2):
        assert np.array_equal(to_np_bits(a.data), to_np_bits(b.data))


# ------------------------------------------------------------------ the C-ABI exchange (RCCL)
def test_comm_abi_world1_exchange_and_sharded_step(pkg, gpu):
    """dlrm_comm_unique_id / dlrm_comm_init / dlrm_alltoall_fwd / _bwd through ctypes on a one-rank
    RCCL communicator (the 1-GPU box has no peers): the exchanges deliver their blocks bit for bit,
    and the sharded step driven through them equals the single-GPU HotPath."""
    from dlrm_jl_amd.comm import CommExchange
    from dlrm_jl_amd.sharded import HipShardOps, ShardedHotPath, TablePartition
    rows, D, B, L = [3, 5000, 70, 100000, 11], 32, 128, 1
    T = len(rows)
    comm = CommExchange(0, 1, gpu)
    send = torch.randn((T * B * D,), device=gpu).to(torch.bfloat16)
    recv = torch.empty_like(send)
    comm.alltoall_fwd(send, recv, D, B, [T])
    g = torch.randn((T * B * D,), device=gpu)
    grecv = torch.empty_like(g)
    comm.alltoall_bwd(g, grecv, D, B, [T])
    torch.cuda.synchronize()
    assert torch.equal(recv, send) and torch.equal(grecv, g)
    with pytest.raises(TypeError):  # the gradient exchange is fp32
        comm.alltoall_bwd(g.to(torch.bfloat16), grecv, D, B, [T])
    import ctypes
    h = ctypes.c_void_p()
    assert comm.lib.dlrm_comm_init(comm.ctx.bind(), comm._uid, 3, 1, ctypes.byref(h)) == pkg._lib.E_ARG  # rank 3 of 1
    comm.close()
    rng = np.random.default_rng(17)
    tabs = rand_tables(rng, rows, D)
    idx = rand_indices(rng, rows, B, L)
    x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
    F = T + 1
    dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32)).to(gpu)
    p = pkg.PackedIndices(torch.from_numpy(idx).to(torch.int32).reshape(T, B, L).to(gpu))
    ops = HipShardOps([torch.from_numpy(t).to(gpu) for t in tabs], B, L, 0.25, device=gpu)
    eng = ShardedHotPath(ops, TablePartition(T, 1), 0, B, D, L, torch.float32, gpu, exchange="abi")
    eng.step(x, p, dout)
    hp = pkg.HotPath(pkg.EmbeddingTableSet(dev_tables(tabs, gpu)), B, L, lr=0.25, index_base=0)
    hp.step(x, p, dout)
    torch.cuda.synchronize()
    ops.ctx.check_bounds()
    assert torch.equal(eng.out, hp.out) and torch.equal(eng.dx, hp.dx)
    for a, b in zip(ops.ts, hp.ts):
        assert torch.equal(a.data, b.data)


@pytest.mark.timeout(90)
@pytest.mark.parametrize("exchange,micro", [("abi", 1), ("torch", 1), ("abi", 2), ("torch", 2)])
def test_sharded_whole_step_graph_world1(pkg, gpu, exchange, micro):
    """capture_full: the whole sharded step -- side-stream index build, lookup, both all-to-alls
    (the library's RCCL communicator, or torch.distributed "nccl" = RCCL), interaction, update --
    captured as one hipGraph per index batch on a one-rank communicator (micro = 2: the exchanges
    on the comm stream, overlapping the other micro-batch's compute), replayed, equals the eager
    step bit for bit (tables, out, dx) over the same sequence of batches; close() then releases the
    graphs before the communicators (the order RCCL needs)."""
    import socket
    import torch.distributed as dist
    from dlrm_jl_amd.sharded import HipShardOps, ShardedHotPath, TablePartition
    rows, D, B, L = [3, 5000, 70, 100000, 11], 32, 128, 1
    T = len(rows)
    own_pg = False
    if exchange == "torch" and not dist.is_initialized():
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=gpu)
        own_pg = True
    try:
        rng = np.random.default_rng(23)
        tabs = rand_tables(rng, rows, D)
        idxs = [pkg.PackedIndices(torch.from_numpy(rand_indices(rng, rows, B, L)).to(torch.int32).reshape(T, B, L)
                                  .to(gpu)) for _ in range(2)]
        x = torch.from_numpy(rng.standard_normal((B, D)).astype(np.float32)).to(gpu)
        F = T + 1
        dout = torch.from_numpy(rng.standard_normal((B, D + F * (F - 1) // 2)).astype(np.float32) * 1e-2).to(gpu)

        def engine():
            ops = HipShardOps([torch.from_numpy(t).to(gpu) for t in tabs], B, L, 0.25, device=gpu)
            return ops, ShardedHotPath(ops, TablePartition(T, 1), 0, B, D, L, torch.float32, gpu, exchange=exchange,
                                       micro=micro)
        ops_e, eng_e = engine()
        for k in (0, 1, 0):
            eng_e.step(x, idxs[k], dout)
        ops_g, eng_g = engine()
        eng_g.step(x, idxs[0], dout)  # eager warm-up (settles the ops' one-time choices), batch 0
        torch.cuda.synchronize()
        eng_g.capture_full(x, idxs, dout)
        eng_g.step_graphed(1)
        eng_g.step_graphed(0)
        torch.cuda.synchronize()
        ops_e.ctx.check_bounds()
        assert torch.equal(eng_g.out, eng_e.out) and torch.equal(eng_g.dx, eng_e.dx)
        for a, b in zip(ops_g.ts, ops_e.ts):
            assert torch.equal(a.data, b.data)
        # the graphs hold RCCL work: released before their communicator is destroyed (round 4's hang
        # was ncclCommDestroy at this test's end, waiting on graphs that were still alive)
        eng_g.close()
        eng_e.close()
    finally:
        if own_pg:
            dist.destroy_process_group()
