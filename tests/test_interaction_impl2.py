"""Implementation 2 of the interaction (src/model/interact.jl:176-215, :503-554) as GPU operators,
and the maplookup pullback's `uncompress` (test/train/backprop.jl:147-158).

The checkers are the reference's own known-answer vectors (tests/golden/kat_reference_tests.json,
transcribed from test/model/interact.jl:9-32) and float64 numpy restatements of the formulas the
docstrings cite."""
import numpy as np
import pytest
import torch

from helpers import assert_close, rand_indices

pytestmark = pytest.mark.gpu


def upper_pairs(sz):
    """(col, row), row < col, in triangular_slice_kernel! order (interact.jl:64-75)."""
    return [(c, r) for c in range(1, sz) for r in range(c)]


def test_triangular_slice_kat(pkg, gpu, kat):
    k = kat["triangle"]
    x = torch.tensor([k["x_julia_colmajor_as_rows_of_C"]], dtype=torch.float32, device=gpu)  # [1][col][row]
    y = pkg.triangular_slice(x)
    assert y.cpu().numpy()[0].tolist() == k["y"]
    up = pkg.triangular_slice_back(y, 3)  # [1][col][row] = the Julia matrix transposed
    assert up.cpu().numpy()[0].T.tolist() == k["back_upper_julia"]
    sym = pkg.triangular_slice_back(y, 3, symmetric=True)
    assert sym.cpu().numpy()[0].T.tolist() == k["back_fused_symmetric_julia"]


@pytest.mark.parametrize("sz,B,dtype", [(8, 128, torch.float32), (27, 300, torch.float32), (27, 64, torch.bfloat16),
                                        (65, 17, torch.float32), (1, 4, torch.float32)])
def test_triangular_slice_bit_exact(pkg, gpu, sz, B, dtype):
    rng = np.random.default_rng(sz)
    z = torch.from_numpy(rng.standard_normal((B, sz, sz)).astype(np.float32)).to(dtype).to(gpu)
    y = pkg.triangular_slice(z)
    zc = z.float().cpu().numpy()
    want = np.array([[zc[b, c, r] for c, r in upper_pairs(sz)] for b in range(B)], dtype=np.float32).reshape(B, -1)
    assert np.array_equal(y.float().cpu().numpy(), want)
    # the pullback puts every value back where it came from, zeros elsewhere
    for symmetric in (False, True):
        a = pkg.triangular_slice_back(y, sz, symmetric=symmetric).float().cpu().numpy()
        exp = np.zeros((B, sz, sz), dtype=np.float32)
        for c, r in upper_pairs(sz):
            exp[:, c, r] = zc[:, c, r]
            if symmetric:
                exp[:, r, c] = zc[:, c, r]
        assert np.array_equal(a, exp)


@pytest.mark.parametrize("F,d,B,dtype", [(8, 16, 128, torch.float32), (27, 128, 256, torch.float32),
                                         (27, 128, 64, torch.bfloat16), (65, 256, 8, torch.float32),
                                         (5, 100, 33, torch.float32)])
def test_self_batched_mul_and_rrule(pkg, gpu, F, d, B, dtype):
    """self_batched_mul (interact.jl:526-537) and its rrule dT = T (Δ + Δᵀ) (:539-551) against
    float64 restatements, fp32 accumulation tolerance (bf16: one rounding of the output)."""
    rng = np.random.default_rng(F * d)
    t = torch.from_numpy(rng.standard_normal((B, F, d)).astype(np.float32)).to(dtype).to(gpu)
    z, back = pkg.rrule_self_batched_mul(t)
    t64 = t.float().cpu().numpy().astype(np.float64)
    want = t64 @ t64.transpose(0, 2, 1)
    if dtype == torch.float32:
        assert_close(z.float().cpu().numpy(), want, rtol=1e-5, scale=np.sqrt(d), what="self_batched_mul")
    else:  # one bf16 rounding (2^-8 relative) of the fp32-accumulated value
        err = np.abs(z.float().cpu().numpy() - want)
        assert (err <= 2.0 ** -8 * np.abs(want) + 1e-4 * np.sqrt(d)).all(), err.max()
    assert torch.equal(z, z.transpose(1, 2))  # symmetric, bit for bit
    delta = torch.from_numpy(rng.standard_normal((B, F, F)).astype(np.float32)).to(dtype).to(gpu)
    _, dt = back(delta)
    d64 = delta.float().cpu().numpy().astype(np.float64)
    s = d64 + d64.transpose(0, 2, 1)
    assert_close(dt.cpu().numpy(), s @ t64, rtol=1e-5, scale=np.sqrt(F) * 2, what="self_batched_mul_back")


@pytest.mark.parametrize("F,d,B", [(8, 16, 128), (27, 128, 512), (27, 16, 2048)])
def test_dot_interaction_composition_equals_fused(pkg, gpu, F, d, B):
    """dot_interaction (Implementation 2) composed from the pieces == the fused operator
    (DotInteraction / dot_back), forward and backward, within fp32 tolerance; and the fused
    dot_interaction entry == DotInteraction() bit for bit."""
    rng = np.random.default_rng(B + F)
    x = torch.from_numpy(rng.standard_normal((B, d)).astype(np.float32)).to(gpu)
    ys = torch.from_numpy(rng.standard_normal((B, F * d)).astype(np.float32)).to(gpu)
    out, pull = pkg.rrule_dot_interaction(x, ys)
    assert torch.equal(out, pkg.DotInteraction()(x, ys))
    t = ys.reshape(B, F, d)  # x already copied in by the forward (fast_vcat)
    z, zback = pkg.rrule_self_batched_mul(t)
    zflat, sback = pkg.rrule_triangular_slice(z)
    composed = torch.cat([x, zflat], dim=1)
    assert_close(composed.cpu().numpy(), out.cpu().numpy(), rtol=1e-5, scale=np.sqrt(d), what="composed forward")
    delta = torch.from_numpy(rng.standard_normal(out.shape).astype(np.float32) * 1e-2).to(gpu)
    _, dx, dy = pull(delta)
    _, dz = sback(delta[:, d:].contiguous())
    _, dt = zback(dz)
    dt = dt.reshape(B, F * d)
    assert_close(dt.cpu().numpy(), dy.cpu().numpy(), rtol=1e-5, scale=0.05 * np.sqrt(F), what="composed dT")
    assert_close((delta[:, :d] + dt[:, :d]).cpu().numpy(), dx.cpu().numpy(), rtol=1e-5, scale=0.05 * np.sqrt(F),
                 what="composed dx")


@pytest.mark.parametrize("rows,B,L,dtype", [([3, 50, 10000], 512, 1, torch.float32), ([7, 1000], 300, 10, torch.float32),
                                            ([20, 5000], 256, 3, torch.bfloat16)])
def test_uncompress_matches_autodiff(pkg, gpu, rows, B, L, dtype):
    """test/train/backprop.jl:147-158: the maplookup pullback's SparseEmbeddingUpdate, uncompressed
    to a dense [N][D] gradient, equals autodiff of the plain gather `embedding[:, ids]` (sum-pooled
    bags) -- here torch autograd in float64."""
    rng = np.random.default_rng(len(rows) * B + L)
    D, T = 16, len(rows)
    tabs = [rng.standard_normal((n, D)).astype(np.float32) for n in rows]
    idx_np = rand_indices(rng, rows, B, L)
    dy = torch.from_numpy(rng.standard_normal((B, D + T * D)).astype(np.float32)).to(dtype).to(gpu)
    ts = pkg.EmbeddingTableSet([torch.from_numpy(a).to(dtype).to(gpu) for a in tabs])
    p = pkg.PackedIndices(torch.from_numpy(idx_np).to(gpu).reshape(T, B, L))
    grads = pkg.maplookup_pullback(D, ts, p, dy)  # rows 0:D belong to x (PreallocationStrategy(D))
    for t, n in enumerate(rows):
        got = grads[t].uncompress(n, index_base=0).cpu().numpy()
        e = torch.from_numpy(tabs[t].astype(np.float64)).requires_grad_(True)
        bags = e[torch.from_numpy(idx_np[t]).reshape(B, L)].sum(dim=1)  # [B][D]
        (bags * dy[:, D + t * D:D + (t + 1) * D].double().cpu()).sum().backward()
        assert_close(got, e.grad.numpy(), rtol=1e-5, scale=np.sqrt(B * L / n + 1), what=f"uncompress table {t}")
