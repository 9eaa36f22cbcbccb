"""CPU restatement of the reference's Criteo DAC data path — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this (the checker for dlrm.jl_amd/dac.py and the dlrm_dac_* C ABI).
Pinned by the reference's own fixtures: test/dataset/alldays.txt (the first 250 lines of the
DAC dataset) and its five gzip shards day_{0..4}.gz, copied as data under tests/golden/dac/, and
the properties test/data/criteo.jl checks on them (sharded maps == monolithic maps; the
reindexed binary == parse + reindex of each line).
"""
import math

import numpy as np

DAC_DTYPE = np.dtype([("label", "<i4"), ("continuous", "<f4", (13,)), ("categorical", "<u4", (26,))])


def emptyparse(s, base):
    """criteo.jl:41-47: an empty field is zero."""
    return 0 if s == "" else int(s, base)


def logtransform(x):
    """criteo.jl:55: log(max(Float32(x), 0) + 1) in Float32."""
    return np.float32(math.log(float(max(np.float32(x), np.float32(0))) + 1.0))


def parseline(line):
    """criteo.jl:164-176: label, 13 continuous (base 10, logtransformed), 26 categorical (base 16)."""
    f = line.rstrip("\n").split("\t")
    assert len(f) == 40, len(f)
    rec = np.zeros((), dtype=DAC_DTYPE)
    rec["label"] = int(f[0], 10)
    rec["continuous"] = [logtransform(emptyparse(v, 10)) for v in f[1:14]]
    rec["categorical"] = [emptyparse(v, 16) for v in f[14:40]]
    return rec


def parse_text(text):
    lines = [ln for ln in text.split("\n") if ln]
    return np.array([parseline(ln) for ln in lines], dtype=DAC_DTYPE)


def reindex_maps(shards):
    """categorical_values + reindex (criteo.jl:182-249): per feature, first-appearance ids from 1."""
    maps = [dict() for _ in range(26)]
    for recs in shards:
        for r in recs:
            for j in range(26):
                maps[j].setdefault(int(r["categorical"][j]), len(maps[j]) + 1)
    return maps


def reindex_records(maps, recs):
    """reindex!(data, maps) (criteo.jl:251-259)."""
    out = recs.copy()
    for i in range(len(out)):
        out[i]["categorical"] = [maps[j][int(out[i]["categorical"][j])] for j in range(26)]
    return out


def load_batch(recs):
    """load! (criteo.jl:284-307) for one batch: labels f32 [B], dense [B][13] (Julia (13, B)),
    sparse [26][B] (Julia Matrix{UInt32}(B, 26))."""
    return (recs["label"].astype(np.float32), np.ascontiguousarray(recs["continuous"]),
            np.ascontiguousarray(recs["categorical"].T))
