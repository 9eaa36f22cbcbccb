"""Shared test helpers: seeded inputs and comparison criteria.

Tolerances (stated here once, used by every parity test):
  * integer / index / copy work (one-hot lookup, unique rows, segment positions): bit-exact.
  * fp32 reductions in a different order than the checker (interaction MFMA k order,
    chunked hot-row sums): |a - b| <= 1e-5 * (|b| + scale) elementwise, where `scale` is the
    magnitude of the summed terms, AND Julia's isapprox default on the whole array,
    norm(a - b) <= sqrt(eps(Float32)) * max(norm(a), norm(b)) (the reference's own criterion,
    test/integration.jl, src/validation.jl).
  * bf16 outputs: one bf16 rounding (2^-8 relative) of the fp32 result.
"""
import numpy as np

SQRT_EPS_F32 = float(np.sqrt(np.finfo(np.float32).eps))


def julia_isapprox(a, b, rtol=SQRT_EPS_F32):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.linalg.norm(a - b) <= rtol * max(np.linalg.norm(a), np.linalg.norm(b))


def assert_close(a, b, rtol=1e-5, scale=None, what=""):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    s = np.abs(b).max() if scale is None else scale
    s = max(float(s), 1e-30)
    err = np.abs(a - b)
    bound = rtol * (np.abs(b) + s)
    bad = err > bound
    assert not bad.any(), f"{what}: {bad.sum()} elements off, max err {err.max():.3e} (bound rtol={rtol})"
    assert julia_isapprox(a, b), f"{what}: fails Julia isapprox"


def rand_tables(rng, rows, dim, scale=1.0):
    return [(rng.uniform(-scale, scale, size=(n, dim))).astype(np.float32) for n in rows]


def rand_indices(rng, rows, batch, lookups, zipf=None):
    out = np.empty((len(rows), batch * lookups), dtype=np.int64)
    for t, n in enumerate(rows):
        if zipf is None:
            out[t] = rng.integers(0, n, size=batch * lookups)
        else:
            z = rng.zipf(zipf, size=batch * lookups) - 1
            out[t] = np.minimum(z, n - 1)
    return out
