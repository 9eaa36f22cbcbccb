"""The full training step around the hot path: bottom/top MLPs + BCE + Descent.

Golden: the reference's ref/pytorch_reference_{single,multi}.hdf5 (MLP weights, `mlp_top`, `loss`,
`update_bot_*`, `update_top_*`, `update_emb_*`), extracted by tests/golden/make_fixtures.py and
checked the way src/validation.jl:17-146 checks the Julia model (one Descent(10) step; Julia
isapprox at sqrt(eps(Float32)) on every updated parameter).

CPU tests pin the dense math (dlrm.jl_amd/dense.py on CPU tensors; the interaction's dx, which
the bottom MLP's pullback needs, comes from the oracle).  GPU tests run `DLRMModel.step` whole:
the MLPs on hipBLASLt/rocBLAS via torch, the hot path through the HIP C ABI.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

import oracle
from conftest import GOLDEN
from helpers import assert_close, julia_isapprox


@pytest.fixture(scope="module")
def dense_golden():
    out = {}
    for kind in ("single", "multi"):
        with np.load(os.path.join(GOLDEN, f"pytorch_reference_{kind}_dense.npz"), allow_pickle=False) as z:
            out[kind] = {k: z[k] for k in z.files}
    return out


def _mlp(pkg, g, short, sigmoid_last, device="cpu"):
    n = len([k for k in g if k.startswith(f"{short}_W")])
    Ws = [torch.from_numpy(g[f"{short}_W{i}"]).to(device) for i in range(n)]
    bs = [torch.from_numpy(g[f"{short}_b{i}"]).to(device) for i in range(n)]
    return pkg.DenseMLP(Ws, bs, sigmoid_last=sigmoid_last)


def _check_updates(mlp, g, short):
    n = len(mlp.W)
    for i in range(n):
        for kk, got in (("W", mlp.W[i]), ("b", mlp.b[i])):
            want = g[f"upd_{short}_{kk}{i}"]
            orig = g[f"{short}_{kk}{i}"]
            got = got.detach().cpu().numpy()
            assert not np.array_equal(orig, want)  # the step moved it (validation.jl:97)
            assert julia_isapprox(got, want), f"update_{short}_{2 * i}.{kk}: fails Julia isapprox"
            assert julia_isapprox(orig - got, orig - want), f"{short} layer {i} {kk}: gradient differs"


@pytest.mark.parametrize("kind", ["single", "multi"])
def test_dense_forward_matches_golden(pkg, golden, dense_golden, kind):
    g, gd = golden[kind], dense_golden[kind]
    bottom = _mlp(pkg, gd, "bot", False)
    top = _mlp(pkg, gd, "top", True)
    x = bottom.forward(torch.from_numpy(gd["input_bot"]))
    assert_close(x.numpy(), g["mlp_bottom"], rtol=1e-5, what="mlp_bottom")
    p = top.forward(torch.from_numpy(g["output_interaction"])).reshape(-1)
    assert_close(p.numpy(), gd["mlp_top"], rtol=1e-5, what="mlp_top")
    loss = pkg.bce_loss(p, torch.from_numpy(gd["labels"]))
    assert abs(float(loss) - float(gd["loss"])) <= 1e-5 * abs(float(gd["loss"]))


@pytest.mark.parametrize("kind", ["single", "multi"])
def test_dense_backward_and_descent_match_golden(pkg, golden, dense_golden, kind):
    """validation.jl:74-123 for both MLPs; the interaction pullback between them is the oracle's."""
    g, gd = golden[kind], dense_golden[kind]
    lr = float(g["lr"])
    T, N, D = g["emb"].shape
    B, d = g["mlp_bottom"].shape
    L = int(g["L"])
    bottom = _mlp(pkg, gd, "bot", False)
    top = _mlp(pkg, gd, "top", True)
    bottom.forward(torch.from_numpy(gd["input_bot"]))
    p = top.forward(torch.from_numpy(g["output_interaction"])).reshape(-1)
    labels = torch.from_numpy(gd["labels"])
    dout = top.backward(pkg.bce_loss_back(p, labels).reshape(-1, 1))
    assert_close(dout.numpy(), g["d_output_interaction"], rtol=1e-4, what="dLoss/d(output_interaction)")
    ys = np.zeros((B, (T + 1) * D), dtype=np.float32)
    oracle.maplookup(list(g["emb"]), g["idx"], 0, B, L, ys, d)
    oracle.interact_fwd(g["mlp_bottom"], ys, T + 1)
    dx, _ = oracle.interact_bwd(np.ascontiguousarray(dout.numpy()), ys, d, T + 1)
    bottom.backward(torch.from_numpy(dx), need_dx=False)
    top.sgd_(lr)
    bottom.sgd_(lr)
    _check_updates(top, gd, "top")
    _check_updates(bottom, gd, "bot")


def test_bce_clamps_like_the_reference(pkg):
    """train.jl:36-40: log terms clamped at -100; the pullback adds eps(T) (train.jl:52-58)."""
    p = torch.tensor([0.0, 1.0, 0.5], dtype=torch.float32)
    y = torch.tensor([1.0, 0.0, 1.0], dtype=torch.float32)
    loss = pkg.bce_loss(p, y)
    want = (100.0 + 100.0 + -np.log(0.5)) / 3
    assert abs(float(loss) - want) < 1e-4
    dp = pkg.bce_loss_back(p, y)
    assert torch.isfinite(dp).all()
    eps = np.finfo(np.float32).eps
    assert abs(float(dp[2]) - (1 / 3) * (0.0 / (0.5 + eps) - 1.0 / (0.5 + eps))) < 1e-6


def test_model_rejects_mismatched_mlps(pkg):
    bottom, top = pkg.kaggle_mlp_sizes(16, 26)
    assert bottom == [13, 512, 256, 16]
    assert top == [16 + 27 * 26 // 2, 1024, 1024, 512, 256, 1]  # criteo.jl:408-433
    with pytest.raises(ValueError):
        pkg.DenseMLP([torch.zeros(4, 3), torch.zeros(2, 5)], [torch.zeros(4), torch.zeros(2)])


# ---- GPU: the whole step, HIP hot path + torch MLPs ----------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["single", "multi"])
def test_train_step_matches_pytorch_reference(pkg, gpu, golden, dense_golden, kind):
    """src/validation.jl:17-58 on the GPU: loss, mlp_top, every MLP update and every table update."""
    g, gd = golden[kind], dense_golden[kind]
    T, N, D = g["emb"].shape
    B = g["mlp_bottom"].shape[0]
    L = int(g["L"])
    lr = float(g["lr"])
    bottom = _mlp(pkg, gd, "bot", False, gpu)
    top = _mlp(pkg, gd, "top", True, gpu)
    tables = pkg.EmbeddingTableSet([torch.from_numpy(t).to(gpu) for t in g["emb"]])
    model = pkg.DLRMModel(bottom, tables, top, B, L, lr=lr, index_base=0)
    idx = pkg.PackedIndices(torch.from_numpy(g["idx"]).to(torch.int32).reshape(T, B, L).to(gpu))
    dense = torch.from_numpy(gd["input_bot"]).to(gpu)
    labels = torch.from_numpy(gd["labels"]).to(gpu)
    loss = model.step(dense, idx, labels)
    torch.cuda.synchronize()
    model.hot.check_bounds()
    assert abs(float(loss) - float(gd["loss"])) <= 1e-5 * abs(float(gd["loss"])), (float(loss), float(gd["loss"]))
    assert_close(model.prob.cpu().numpy(), gd["mlp_top"], rtol=1e-5, what="mlp_top")
    _check_updates(top, gd, "top")
    _check_updates(bottom, gd, "bot")
    for t in range(T):
        rows = g[f"upd_rows_{t}"]
        got = tables[t].data.cpu().numpy()
        assert_close(got[rows], g[f"upd_vals_{t}"], rtol=1e-5, what=f"update_emb_{t}")
        untouched = np.setdiff1d(np.arange(N), rows)
        assert np.array_equal(got[untouched], g["emb"][t][untouched])


@pytest.mark.gpu
def test_train_step_graph_replay_equals_eager(pkg, gpu):
    """Kaggle-shaped MLPs (criteo.jl:408-433), 26 small tables, B=512: a captured step replayed
    twice == two eager steps, bit for bit (tables, weights, loss)."""
    torch.manual_seed(0)
    T, D, B = 26, 16, 512
    rows = [1000 + 37 * t for t in range(T)]
    bsz, tsz = pkg.kaggle_mlp_sizes(D, T)

    def make():
        gen = torch.Generator(device=gpu).manual_seed(7)
        tabs = [torch.empty((n, D), device=gpu).uniform_(-0.05, 0.05, generator=gen) for n in rows]
        bottom = pkg.random_mlp(bsz, sigmoid_last=False, generator=gen, device=gpu)
        top = pkg.random_mlp(tsz, sigmoid_last=True, generator=gen, device=gpu)
        return pkg.DLRMModel(bottom, tabs, top, B, 1, lr=0.05, index_base=0)

    gen = torch.Generator(device=gpu).manual_seed(11)
    dense = torch.randn((B, 13), device=gpu, generator=gen)
    labels = (torch.rand((B,), device=gpu, generator=gen) < 0.3).float()
    idx = pkg.PackedIndices(torch.stack([torch.randint(0, n, (B,), device=gpu, generator=gen, dtype=torch.int32)
                                         for n in rows]).reshape(T, B, 1).contiguous())
    a = make()
    la = [float(a.step(dense, idx, labels)) for _ in range(2)]
    b = make()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            b.step(dense, idx, labels)
    torch.cuda.current_stream().wait_stream(s)
    lb = []
    for _ in range(2):
        gr.replay()
        torch.cuda.synchronize()
        lb.append(float(b.loss))
    assert la == lb
    for ta, tb in zip(a.tables, b.tables):
        assert torch.equal(ta.data, tb.data)
    for pa, pb in zip(a.top.params() + a.bottom.params(), b.top.params() + b.bottom.params()):
        assert torch.equal(pa, pb)


@pytest.mark.gpu
@pytest.mark.parametrize("B,N", [(2048, 1024), (128, 16), (1000, 260), (17, 4), (4096, 512)])
def test_relu_bwd_bias_seam(pkg, gpu, B, N):
    """dlrm_relu_bwd_bias == threshold_backward (bit-exact) + column sums (fp32 tolerance), and
    its last-arriver counters leave themselves at 0 (a second launch gives the same bits)."""
    from dlrm_jl_amd.runtime import context, ptr
    gen = torch.Generator(device=gpu).manual_seed(B + N)
    y = torch.randn((B, N), device=gpu, generator=gen).relu_()
    g0 = torch.randn((B, N), device=gpu, generator=gen)
    want_g = torch.ops.aten.threshold_backward(g0, y, 0.0)
    want_b = want_g.double().sum(0)
    ctx = context(gpu)
    nw, nc = ctypes.c_int64(), ctypes.c_int64()
    assert ctx.lib.dlrm_relu_bwd_bias_workspace(B, N, ctypes.byref(nw), ctypes.byref(nc)) == 0
    work = torch.empty(nw.value, device=gpu)
    cnt = torch.zeros(nc.value, dtype=torch.int32, device=gpu)
    outs = []
    for _ in range(2):
        g = g0.clone()
        gb = torch.empty(N, device=gpu)
        ctx.check(ctx.lib.dlrm_relu_bwd_bias(ctx.bind(), B, N, ptr(y), y.stride(0), ptr(g), g.stride(0), ptr(gb),
                                             ptr(work), ptr(cnt)))
        torch.cuda.synchronize()
        assert torch.equal(g, want_g)
        outs.append(gb.clone())
    assert torch.equal(outs[0], outs[1])
    assert int(cnt.abs().sum()) == 0
    assert_close(outs[0].cpu().numpy(), want_b.cpu().numpy(), rtol=1e-5, what="bias gradient")


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 128, 2048, 3001])
def test_bce_head_seam(pkg, gpu, B):
    """dlrm_bce_head == the torch restatement of sigmoid -> bce_loss -> rrule (train.jl:33-64),
    including saturated logits (the -100 clamp)."""
    from dlrm_jl_amd.runtime import context, ptr
    gen = torch.Generator(device=gpu).manual_seed(B)
    z = torch.randn((B, 1), device=gpu, generator=gen) * 4
    z[: min(B, 3), 0] = torch.tensor([120.0, -120.0, 0.0], device=gpu)[: min(B, 3)]
    y = (torch.rand(B, device=gpu, generator=gen) < 0.5).float()
    prob, dz = torch.empty(B, device=gpu), torch.empty((B, 1), device=gpu)
    loss, db = torch.empty((), device=gpu), torch.empty(1, device=gpu)
    ctx = context(gpu)
    ctx.check(ctx.lib.dlrm_bce_head(ctx.bind(), B, ptr(z), z.stride(0), ptr(y), ptr(prob), ptr(dz), ptr(loss),
                                    ptr(db)))
    torch.cuda.synchronize()
    zd = z.double().reshape(-1)
    p = torch.sigmoid(zd)
    assert_close(prob.cpu().numpy(), p.cpu().numpy(), rtol=1e-6, what="prob")
    want_loss = float(pkg.bce_loss(p.float(), y))
    assert abs(float(loss) - want_loss) <= 1e-5 * max(1.0, abs(want_loss))
    # dlogit from the kernel's own prob: near saturation 1 - p is a few ulps, so one ulp of the
    # sigmoid moves (1-p)/(1-p+eps) by O(1) — the reference's formula, not a kernel error
    pk = prob.double()
    want_dz = pkg.bce_loss_back(prob, y).double() * pk * (1 - pk)
    assert_close(dz.reshape(-1).cpu().numpy(), want_dz.cpu().numpy(), rtol=1e-4, what="dlogit")
    assert abs(float(db) - float(dz.double().sum())) <= 1e-5 * max(1e-3, float(dz.abs().sum()))


def _dp_full_worker(rank, world, port, outdir):
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
    tabs, idx, dense, labels, mk = _dp_problem(pkg, dev, world)
    T, B, D = len(tabs), dense.shape[0] // world, tabs[0].shape[1]
    part = TablePartition(T, world)
    mine = part.tables(rank)
    ops = HipShardOps([torch.from_numpy(tabs[t]).to(dev) for t in mine], B * world, 1, 0.2, device=dev)
    eng = ShardedHotPath(ops, part, rank, B, D, 1, torch.float32, dev)
    bottom, top = mk()
    model = pkg.ShardedDLRMModel(bottom, top, eng, 0.2)
    p = pkg.PackedIndices(torch.from_numpy(idx[mine]).to(torch.int32).reshape(len(mine), B * world, 1).to(dev))
    sl = slice(rank * B, (rank + 1) * B)
    loss = model.step(torch.from_numpy(dense[sl]).to(dev), p, torch.from_numpy(labels[sl]).to(dev))
    torch.cuda.synchronize()
    ops.ctx.check_bounds()
    arrs = {f"t{t}": ops.ts[k].data.cpu().numpy() for k, t in enumerate(mine)}
    for name, m in (("bot", bottom), ("top", top)):
        for i in range(len(m.W)):
            arrs[f"{name}_W{i}"] = m.W[i].cpu().numpy()
            arrs[f"{name}_b{i}"] = m.b[i].cpu().numpy()
    np.savez(os.path.join(outdir, f"dp{rank}.npz"), loss=float(loss), **arrs)
    dist.barrier()
    dist.destroy_process_group()


def _dp_problem(pkg, dev, world):
    rng = np.random.default_rng(17)
    rows, D, B = [4, 3000, 90, 60000, 13, 700], 16, 96
    T = len(rows)
    tabs = [rng.uniform(-0.3, 0.3, (n, D)).astype(np.float32) for n in rows]
    idx = np.stack([rng.integers(0, n, B * world) for n in rows]).astype(np.int64)
    dense = rng.standard_normal((B * world, 13)).astype(np.float32)
    labels = (rng.random(B * world) < 0.3).astype(np.float32)
    bsz, tsz = pkg.kaggle_mlp_sizes(D, T)

    def mk():
        gen = torch.Generator(device=dev).manual_seed(99)
        return (pkg.random_mlp(bsz, sigmoid_last=False, generator=gen, device=dev),
                pkg.random_mlp(tsz, sigmoid_last=True, generator=gen, device=dev))
    return tabs, idx, dense, labels, mk


@pytest.mark.gpu
def test_data_parallel_full_step_two_ranks_equals_single_gpu(pkg, gpu, tmp_path):
    """SURVEY rows f1 + f3: two ranks sharing the GPU (gloo; RCCL on a full node) run the full step
    with data-parallel MLPs (bucketed gradient all-reduce) and table-sharded HIP hot path; the
    result equals one GPU's DLRMModel on the global batch (fp32 tolerance: the dense gradients
    are summed in a different order)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    mp.start_processes(_dp_full_worker, args=(world, port, str(tmp_path)), nprocs=world, start_method="spawn")
    tabs, idx, dense, labels, mk = _dp_problem(pkg, gpu, world)
    T, Bg = len(tabs), dense.shape[0]
    bottom, top = mk()
    model = pkg.DLRMModel(bottom, [torch.from_numpy(t).to(gpu) for t in tabs], top, Bg, 1, lr=0.2, index_base=0)
    p = pkg.PackedIndices(torch.from_numpy(idx).to(torch.int32).reshape(T, Bg, 1).to(gpu))
    loss = float(model.step(torch.from_numpy(dense).to(gpu), p, torch.from_numpy(labels).to(gpu)))
    from dlrm_jl_amd.sharded import TablePartition
    part = TablePartition(T, world)
    for r in range(world):
        z = np.load(tmp_path / f"dp{r}.npz")
        assert abs(float(z["loss"]) - loss) <= 1e-5 * abs(loss)
        for name, m in (("bot", bottom), ("top", top)):
            for i in range(len(m.W)):
                assert_close(z[f"{name}_W{i}"], m.W[i].cpu().numpy(), rtol=1e-5, what=f"rank {r} {name} W{i}")
                assert_close(z[f"{name}_b{i}"], m.b[i].cpu().numpy(), rtol=1e-5, what=f"rank {r} {name} b{i}")
        for t in part.tables(r):
            assert_close(z[f"t{t}"], model.tables[t].data.cpu().numpy(), rtol=1e-5, what=f"rank {r} table {t}")


@pytest.mark.gpu
def test_train_step_bf16_tables(pkg, gpu, golden, dense_golden):
    """bf16 tables (SURVEY configs[2]'s storage) under the fp32 MLPs: the hot path computes in bf16
    storage / fp32 accumulation, x and dLoss/dout cross the boundary rounded to bf16.  Loss and
    updated rows agree with the fp32 golden step to bf16 precision."""
    g, gd = golden["single"], dense_golden["single"]
    T, N, D = g["emb"].shape
    B = g["mlp_bottom"].shape[0]
    lr = float(g["lr"])
    tabs = [torch.from_numpy(t).to(gpu).to(torch.bfloat16) for t in g["emb"]]
    start = [t.float().cpu().numpy() for t in tabs]
    model = pkg.DLRMModel(_mlp(pkg, gd, "bot", False, gpu), tabs, _mlp(pkg, gd, "top", True, gpu), B, 1, lr=lr,
                          index_base=0)
    idx = pkg.PackedIndices(torch.from_numpy(g["idx"]).to(torch.int32).reshape(T, B, 1).to(gpu))
    loss = float(model.step(torch.from_numpy(gd["input_bot"]).to(gpu), idx, torch.from_numpy(gd["labels"]).to(gpu)))
    torch.cuda.synchronize()
    model.hot.check_bounds()
    assert abs(loss - float(gd["loss"])) <= 1e-2 * abs(float(gd["loss"]))
    for t in range(T):
        rows = g[f"upd_rows_{t}"]
        got = model.tables[t].data.float().cpu().numpy()
        want_delta = g[f"upd_vals_{t}"] - g["emb"][t][rows]  # the golden step's change of each touched row
        got_delta = got[rows] - start[t][rows]
        # bf16 storage: each row moves by the golden delta up to bf16 rounding of the row values
        tol = 2 * 2.0 ** -8 * np.abs(start[t][rows]).max() + 0.05 * np.abs(want_delta).max()
        assert np.abs(got_delta - want_delta).max() <= tol, t
        untouched = np.setdiff1d(np.arange(N), rows)
        assert np.array_equal(got[untouched], start[t][untouched])
