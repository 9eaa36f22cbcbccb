"""The Criteo DAC data path (SURVEY §8 rows f2 + f4) against the reference's own dataset fixtures.

Fixtures (data, copied from the reference's test/dataset/): alldays.txt = the first 250 lines of
the DAC dataset, day_{0..4}.gz = the same lines in five gzip shards.  The checks follow
test/data/criteo.jl: record write/read round trip, sharded maps == monolithic maps, and the
reindexed binary == parseline + reindex of every original line.  The checker is
oracle/dac_oracle.py (a line-by-line Python restatement of criteo.jl).
"""
import os

import numpy as np
import pytest
import torch

import dac_oracle
from conftest import GOLDEN

DAC_DIR = os.path.join(GOLDEN, "dac")
ALLDAYS = os.path.join(DAC_DIR, "alldays.txt")
SHARDS = [os.path.join(DAC_DIR, f"day_{i}.gz") for i in range(5)]


@pytest.fixture(scope="module")
def ref_records():
    with open(ALLDAYS) as f:
        return dac_oracle.parse_text(f.read())


def test_record_layout_and_roundtrip(pkg, tmp_path):
    """DACRecord is 160 B; write then read gives the same record (test/data/criteo.jl:19-24)."""
    dac = pkg.dac
    assert dac.DAC_DTYPE.itemsize == 160 and dac.DAC_DTYPE == dac_oracle.DAC_DTYPE
    rng = np.random.default_rng(5)
    r = np.zeros(3, dtype=dac.DAC_DTYPE)
    r["label"] = rng.integers(0, 2, 3)
    r["continuous"] = rng.random((3, 13), dtype=np.float32)
    r["categorical"] = rng.integers(0, 2**32, (3, 26), dtype=np.uint32)
    p = tmp_path / "r.bin"
    r.tofile(p)
    assert os.path.getsize(p) == 480
    assert np.array_equal(dac.load(str(p)), r)


def test_parse_matches_parseline(pkg, ref_records):
    got = pkg.dac.parse_tsv(ALLDAYS)
    assert len(got) == 250
    assert np.array_equal(got["label"], ref_records["label"])
    assert np.array_equal(got["categorical"], ref_records["categorical"])
    # log in Float32 (criteo.jl:55): the C logf and the float64-then-round restatement agree to 1 ulp
    np.testing.assert_array_max_ulp(got["continuous"], ref_records["continuous"], maxulp=1)


def test_parse_gz_shards_concatenate_to_alldays(pkg):
    whole = pkg.dac.parse_tsv(ALLDAYS)
    parts = np.concatenate([pkg.dac.parse_tsv(s) for s in SHARDS])
    assert np.array_equal(parts, whole)


def test_sharded_maps_equal_monolithic(pkg, ref_records):
    """test/data/criteo.jl:38-57: maps built over the five shards == maps over the whole file."""
    dac = pkg.dac
    mono = dac.reindex(dac.parse_tsv(ALLDAYS))
    sharded = dac.reindex([dac.parse_tsv(s) for s in SHARDS])
    want = dac_oracle.reindex_maps([ref_records])
    assert mono.sizes() == sharded.sizes() == [len(m) for m in want]
    with pytest.raises(KeyError):
        mono.lookup(0, 0xFFFFFFFF)
    for j in range(26):
        for v, i in want[j].items():
            assert mono.lookup(j, v) == i == sharded.lookup(j, v)


def test_process_reindexed_binary_equals_parsed_lines(pkg, ref_records, tmp_path):
    """test/data/criteo.jl:63-79: binarize + reindex! of the binary == reindex(parseline(line))."""
    dac = pkg.dac
    binpath = str(tmp_path / "alldays.bin")
    data, maps = dac.process(ALLDAYS, binpath)
    want = dac_oracle.reindex_records(dac_oracle.reindex_maps([ref_records]), ref_records)
    data.flush()
    disk = dac.load(binpath)
    assert os.path.getsize(binpath) == 250 * 160
    assert np.array_equal(disk["categorical"], want["categorical"])
    assert np.array_equal(disk["label"], want["label"])
    np.testing.assert_array_max_ulp(disk["continuous"], want["continuous"], maxulp=1)
    assert disk["categorical"].min() == 1  # 1-based ids (get!(dict, v, length(dict) + 1))


def test_parse_errors_and_unknown_values(pkg):
    dac = pkg.dac
    with pytest.raises(pkg.DLRMError):
        dac.parse_tsv(b"0\t1\t2\n")  # too few fields
    line = open(ALLDAYS, "rb").readline()
    with pytest.raises(pkg.DLRMError):
        dac.parse_tsv(line.replace(b"\t", b"\tzz", 1))  # not a base-10 integer
    label = line.split(b"\t", 1)
    for big in (b"4294967295", b"2147483648", b"-2147483649"):  # parse(Int32, ...) throws OverflowError
        with pytest.raises(pkg.DLRMError):
            dac.parse_tsv(big + b"\t" + label[1])
    assert dac.parse_tsv(b"-2147483648\t" + label[1])["label"][0] == -2147483648
    recs = dac.parse_tsv(line + line)
    assert len(recs) == 2 and np.array_equal(recs[0], recs[1])
    maps = dac.reindex(recs)
    other = dac.parse_tsv(open(ALLDAYS, "rb").read().split(b"\n")[5] + b"\n")
    with pytest.raises(KeyError):
        maps.reindex_(other)  # a value missing from the maps (the reference's KeyError)


# ---- GPU: load! as a decode kernel, the double-buffered DACLoader, a real-data step ----------

@pytest.fixture(scope="module")
def reindexed(pkg, ref_records):
    dac = pkg.dac
    data = dac.parse_tsv(ALLDAYS)
    maps = dac.reindex(data)
    maps.reindex_(data)
    return data, maps


@pytest.mark.gpu
@pytest.mark.parametrize("itype,direct,native", [(torch.int32, False, True), (torch.int64, False, True),
                                                 (torch.int32, True, False), (torch.int32, False, False)])
def test_dac_loader_batches_match_load(pkg, gpu, reindexed, itype, direct, native):
    """native: the C++ prefetch thread; direct: the dataset page-locked, one DMA per batch; else
    pinned staging driven from Python.  Two epochs (the loader restarts), the second one
    abandoned after one batch and then a third run in full."""
    data, _ = reindexed
    loader = pkg.DACLoader(data, 64, gpu, index_dtype=itype, direct=direct, native=native)
    assert loader.direct == direct and loader.native == native
    for b in loader:  # an epoch, then an abandoned one
        pass
    it = iter(loader)
    next(it)
    if native:  # a live iteration holds a batch buffer: a second one must not start over it
        with pytest.raises(RuntimeError):
            next(iter(loader))
    it.close()
    assert len(loader) == 250 // 64  # whole batches only (criteo.jl:326-329)
    seen = 0
    for i, b in enumerate(loader):
        labels, dense, sparse = dac_oracle.load_batch(data[i * 64:(i + 1) * 64])
        assert np.array_equal(b.labels.cpu().numpy(), labels)
        assert np.array_equal(b.dense.cpu().numpy(), dense)
        assert np.array_equal(b.sparse.cpu().numpy(), sparse.astype(np.int64))
        seen += 1
    assert seen == 3
    loader.close()


@pytest.mark.gpu
def test_real_data_training_steps(pkg, gpu, reindexed):
    """A real-data smoke test: the 250-line DAC sample, reindexed, drives the full
    training step (26 tables sized by the maps, D = 16, 1-based ids straight from the loader).
    Every batch passes the bounds check and the loss stays finite; the first batch's forward
    matches a host gather of the same ids."""
    data, maps = reindexed
    sizes = maps.sizes()
    D, B, T = 16, 32, 26
    gen = torch.Generator(device=gpu).manual_seed(3)
    tables = [torch.empty((n, D), device=gpu).uniform_(-n ** -0.5, n ** -0.5, generator=gen) for n in sizes]
    host0 = [t.cpu().numpy() for t in tables]
    bsz, tsz = pkg.kaggle_mlp_sizes(D, T)
    model = pkg.DLRMModel(pkg.random_mlp(bsz, sigmoid_last=False, generator=gen, device=gpu), tables,
                          pkg.random_mlp(tsz, sigmoid_last=True, generator=gen, device=gpu), B, 1, lr=0.05,
                          index_base=1)
    losses = []
    for i, b in enumerate(pkg.DACLoader(data, B, gpu)):
        idx = pkg.PackedIndices(b.sparse.reshape(T, B, 1))
        if i == 0:
            ys = pkg.maplookup(pkg.PreallocationStrategy(0), model.tables, idx, index_base=1)
            want = np.concatenate([host0[t][b.sparse[t].cpu().numpy() - 1] for t in range(T)], axis=1)
            assert np.array_equal(ys.cpu().numpy(), want)
        losses.append(model.step(b.dense, idx, b.labels).clone())
    torch.cuda.synchronize()
    model.hot.check_bounds()
    assert len(losses) == 250 // B and all(np.isfinite(float(l)) for l in losses)
