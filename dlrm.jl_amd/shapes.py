"""Workload shapes of the DLRM hot path (BASELINE.json configs).

Table row counts are the reference's own constants (src/data/criteo.jl:350-406).
"""
import os

import numpy as np

# src/data/criteo.jl:350-377
KAGGLE_EMBEDDING_SIZES = [
    1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194, 27,
    14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572,
]

# src/data/criteo.jl:379-406
TERABYTE_EMBEDDING_SIZES = [
    227605432, 39060, 17295, 7424, 20265, 3, 7122, 1543, 63, 130229467, 3067956, 405282, 10,
    2209, 11938, 155, 4, 976, 14, 292775614, 40790948, 187188510, 590152, 12973, 108, 36,
]

# name -> workload description (bench.py's config.workload names one of these)
WORKLOADS = {
    # configs[0]: 7 tables x 1000 x 16 (+ dense = 8 features), B=128 — golden HDF5 (parity only)
    "golden-single": dict(rows=[1000] * 7, dim=16, batch=128, lookups=1, dtype="f32"),
    "golden-multi": dict(rows=[1000] * 7, dim=16, batch=128, lookups=10, dtype="f32"),
    # configs[1]: Criteo-Kaggle shape, dim 16, batch 2048, fp32 (gather/scatter)
    "kaggle-d16-b2048": dict(rows=KAGGLE_EMBEDDING_SIZES, dim=16, batch=2048, lookups=1, dtype="f32"),
    # BASELINE.json metric: 26 tables x 128-dim, bs=2048 (Kaggle rows), fp32, fwd+bwd
    "kaggle-d128-b2048": dict(rows=KAGGLE_EMBEDDING_SIZES, dim=128, batch=2048, lookups=1, dtype="f32"),
    # configs[2]: 26 tables, dim 128, batch 8192, bf16 — MFMA interaction
    "kaggle-d128-b8192-bf16": dict(rows=KAGGLE_EMBEDDING_SIZES, dim=128, batch=8192, lookups=1, dtype="bf16"),
    # configs[3]: Criteo-Terabyte rows (882.8M, Zipf).  fp32 (452 GB) needs >= 2 GPUs (table-sharded,
    # TablePartition.fitting); bf16 (226 GB) fits one MI355X's 288 GB
    "terabyte-d128-zipf": dict(rows=TERABYTE_EMBEDDING_SIZES, dim=128, batch=2048, lookups=1, dtype="f32", zipf=1.05,
                               rows_src="Criteo-Terabyte (criteo.jl:379-406)"),
    "terabyte-d128-bf16-zipf": dict(rows=TERABYTE_EMBEDDING_SIZES, dim=128, batch=2048, lookups=1, dtype="bf16",
                                    zipf=1.05, rows_src="Criteo-Terabyte (criteo.jl:379-406)"),
    # configs[4]: pooled mode, 64 tables x dim 256, hot-row skew (rows per table: 1M)
    "pooled-64x256-l10": dict(rows=[1_000_000] * 64, dim=256, batch=2048, lookups=10, dtype="f32", zipf=1.2,
                              rows_src="64 x 1M synthetic"),
}


WAVE_MAX_N = 32768  # the wave build's positions per table (csrc/common.hpp kWaveMaxN)
# One GPU: the in-apply wave build, and the side stream's wave build, up to APPLY_MAX_N positions per
# table; above, the side stream's in-LDS parts build (configs[2] at 8192: 85.3 M samples/s, against
# 69 M with the scan build in the apply launch and 82 M with it on the side stream, round 5).  The
# sharded update's indexer: the wave build up to PREPARE_MAX_N (the scan build: 13.4 us for 4
# tables x 16384 positions, against 40 us for the hash build).  DLRM_APPLY_MAX_N / DLRM_PREPARE_MAX_N
# override, for A/B runs.
APPLY_MAX_N = int(os.environ.get("DLRM_APPLY_MAX_N", 2048))
PREPARE_MAX_N = int(os.environ.get("DLRM_PREPARE_MAX_N", WAVE_MAX_N))


def step_pipeline(w):
    """Where the training step's split indexer is built for workload `w` (the form bench.py times
    and tests/test_configs.py checks step by step on the CPU checker): "apply" = inside the previous
    step's apply launch (one-hot batches <= 2048: the forward then only gathers; round 3, metric
    config 49.1M vs 43.8M samples/s with the build in the forward's launch), "side" = the next
    batch's build on a side stream (one-hot batches > 2048: the in-LDS parts build; the in-apply wave
    build takes up to 16384 positions per table but measured slower at 8192, APPLY_MAX_N), None =
    pooled bags: the operator path, whose bag build runs on a side stream beside the forward.  (The
    pooled "side" form -- the next batch's bag build beside this step's apply, HotPath.step_next --
    measured the same, 674.6 vs 670 us per step: the stages' sum either way, as the forward and the
    persistent apply fill every CU slot; round 6.)"""
    L, B = w["lookups"], w["batch"]
    if L != 1:  # pooled bags: the operator path (its bag build on a side stream beside the forward)
        return None
    return "apply" if B <= APPLY_MAX_N else "side"


def step_chunk(w):
    """The wave build's chunk limit for workload `w` (HotPath(chunk=...), dlrm_indexer_set_chunk): 16
    for one-hot batches -- the 105-row Kaggle table's 17..32-position segments then run as one-round
    hot-slice items: metric step 36.9 -> 36.4 us, 55.5 -> 56.1 M samples/s in an alternating A/B, D = 16
    unchanged at 16 parts and 85.6 vs 81.5 M at 32 (profiles/r14/chunk16_ab_*, profiles/r15/chunk_sweep)
    -- and for Zipf rows too since they build 32 parts per table (step_parts): Terabyte bf16 58.1 / 58.5
    vs 57.4 / 57.4 M (at 16 parts Zipf rows preferred 32: 52.5 vs 51.8 M, round 6 first session)."""
    if w["lookups"] != 1 or (w.get("zipf") and not step_parts(w)):
        return None
    return 16


def step_parts(w):
    """Parts per table of the step's wave build for workload `w` (HotPath(parts=...),
    dlrm_indexer_set_parts): 32 where a row is <= 256 B -- the apply's items are light and the next
    batch's build is the apply launch's long pole, so shortening its chain (half the positions per
    wave) wins: D = 16 80.8 -> 85.5 M samples/s, Terabyte bf16 rows 52.0 -> 57.7 M (apply 17.5 ->
    11.8 us) -- and the library's 16 at 512-B rows, where the extra build workgroups cost the heavier
    apply more (metric 56.8 -> 55.0 M with 32); round 6, profiles/r15/parts_ab."""
    if w["lookups"] != 1:
        return None
    return 32 if w["dim"] * (2 if w["dtype"] == "bf16" else 4) <= 256 else None


def table_bytes(rows, dim, esize):
    return sum(rows) * dim * esize


def zipf_perm(rng, n):
    """The affine bijection r -> (a*r + c) mod n that places a table's Zipf ranks on its rows.
    Drawn once per table, so the same rows stay hot from batch to batch (hot-row skew)."""
    a = int(rng.integers(1, max(n, 2)))
    while np.gcd(a, n) != 1:
        a += 1
    return a, int(rng.integers(0, n))


def zipf_rows(rng, n, size, s, perm=None):
    """Zipf(s) ranks (rank 0 hottest, tail folded mod n) scattered over the table's rows by an
    affine bijection r -> (a*r + c) mod n, so hot rows sit at random places.
    perm: the table's (a, c) from zipf_perm (fixed across batches); None draws a fresh one."""
    z = (rng.zipf(s, size=size) - 1) % n
    a, c = zipf_perm(rng, n) if perm is None else perm
    return ((z.astype(np.int64) * a + c) % n).astype(np.int32)
