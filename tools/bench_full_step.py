"""Full DLRM training step on one MI355X: bottom MLP -> hot path (HIP) -> top MLP
-> BCE -> backward -> Descent on every weight and table.  A secondary measurement beside bench.py
(whose `value` stays the hot path the BASELINE metric names).

    python tools/bench_full_step.py [--workload kaggle-d128-b2048] [--steps 48] [--warmup 8]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_full_step.py
        (N ranks: ShardedDLRMModel = data-parallel MLPs with bucketed all-reduce + table-sharded hot
         path, B samples per rank, eager launches; prints the whole-job samples/s)

Model: kaggle_dlrm's MLPs (criteo.jl:408-433: bottom [13, 512, 256, D], top [D+P, 1024, 1024, 512,
256, 1]) with GlorotNormal weights, the workload's tables (ScaledUniform), synthetic N(0,1) dense
features, Bernoulli(0.25) labels, uniform int32 indices; 8 index batches cycled; 8 steps per
hipGraph replay.  Prints one JSON line: the full step, the hot-path-only step and the dense-only
step (the same MLP launches with the hot path's output and dx held fixed), with the dense half's
achieved TFLOP/s against the 157.3 TFLOP/s fp32 matrix peak (MI355X_MICROARCH.md; no xf32 on gfx950).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dlrm_pkg  # noqa: E402

NB = 8
FP32_MATRIX_PEAK_TFLOPS = 157.3


def graph_of(fn, nsteps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for k in range(nsteps):
                fn(k)
    torch.cuda.current_stream().wait_stream(s)
    return g


def timed(g, reps):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / (reps * NB)


def main_sharded(a, pkg):
    """One rank of the multi-GPU full step (SURVEY rows f1 + f3)."""
    import torch.distributed as dist
    from dlrm_jl_amd.sharded import make_bench_engine
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    backend = os.environ.get("DLRM_DIST_BACKEND", "nccl")  # "gloo": 1-GPU rehearsal only
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    w = pkg.WORKLOADS[a.workload]
    D, B, T = w["dim"], w["batch"], len(w["rows"])
    eng, _, _ = make_bench_engine(pkg, w, B, dev, rank, world, a.lr)
    gen = torch.Generator(device=dev).manual_seed(4242)  # identical MLP replicas on every rank
    bsz, tsz = pkg.kaggle_mlp_sizes(D, T)
    bottom = pkg.random_mlp(bsz, sigmoid_last=False, generator=gen, device=dev)
    top = pkg.random_mlp(tsz, sigmoid_last=True, generator=gen, device=dev)
    model = pkg.ShardedDLRMModel(bottom, top, eng, a.lr)
    g2 = torch.Generator(device=dev).manual_seed(51234 + rank)
    dense = [torch.randn((B, 13), device=dev, generator=g2) for _ in range(NB)]
    labels = [(torch.rand((B,), device=dev, generator=g2) < 0.25).float() for _ in range(NB)]
    for k in range(a.warmup):
        model.step(dense[k % NB], eng.bench_packs[k % NB], labels[k % NB])
    torch.cuda.synchronize()
    eng.ops.ctx.check_bounds()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        loss = model.step(dense[k % NB], eng.bench_packs[k % NB], labels[k % NB])
    torch.cuda.synchronize()
    dist.barrier()
    ms = torch.tensor([(time.perf_counter() - t0) * 1e3 / a.steps], device=dev)
    dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({
            "metric": f"DLRM full training step samples/s (MLPs + BCE + hot path + Descent), {world} MI355X",
            "value": round(B * world / (float(ms) * 1e-3), 1), "unit": "samples/s", "ms_per_step": round(float(ms), 4),
            "n_gpus": world, "scaling": "weak", "dtype": w["dtype"] + " tables, f32 MLPs", "loss_last": round(float(loss), 5),
            "config": {"workload": a.workload, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"data-parallel MLPs (all-reduce) + table-sharded x{world} (all-to-all)",
                       "launch": "eager", "backend": backend}}))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="kaggle-d128-b2048")
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--lr", type=float, default=0.01)
    a = ap.parse_args()
    pkg = dlrm_pkg.load()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return main_sharded(a, pkg)
    dev = torch.device("cuda:0")
    w = pkg.WORKLOADS[a.workload]
    if w["lookups"] != 1 or w["dtype"] != "f32":
        raise SystemExit("full-step bench: one-hot fp32 workloads only")
    rows, D, B = w["rows"], w["dim"], w["batch"]
    T = len(rows)
    gen = torch.Generator(device=dev).manual_seed(51234)  # model.jl:193
    tables = [torch.empty((n, D), device=dev).uniform_(-n ** -0.5, n ** -0.5, generator=gen) for n in rows]
    bsz, tsz = pkg.kaggle_mlp_sizes(D, T)
    bottom = pkg.random_mlp(bsz, sigmoid_last=False, generator=gen, device=dev)
    top = pkg.random_mlp(tsz, sigmoid_last=True, generator=gen, device=dev)
    model = pkg.DLRMModel(bottom, tables, top, B, 1, lr=a.lr, index_base=0)
    dense = [torch.randn((B, 13), device=dev, generator=gen) for _ in range(NB)]
    labels = [(torch.rand((B,), device=dev, generator=gen) < 0.25).float() for _ in range(NB)]
    packs = [pkg.PackedIndices(torch.stack([torch.randint(0, n, (B,), device=dev, generator=gen, dtype=torch.int32)
                                            for n in rows]).reshape(T, B, 1).contiguous()) for _ in range(NB)]
    x0 = torch.randn((B, D), device=dev, generator=gen)
    model.hot.validate(x0, packs[0])

    def full(k):
        model.step(dense[k], packs[k], labels[k])

    for k in range(a.warmup):
        full(k % NB)
    torch.cuda.synchronize()
    model.hot.check_bounds()
    l0 = float(model.loss)
    reps = max(1, a.steps // NB)
    ms_full = timed(graph_of(full, NB), reps)

    hot = model.hot
    dout = (torch.randn((B, hot.width), device=dev, generator=gen) * 1e-3)

    def hot_only(k):
        hot.step(x0, packs[k], dout)

    ms_hot = timed(graph_of(hot_only, NB), reps)
    out_fixed = hot.out.clone()
    dx_fixed = hot.dx.clone()

    def dense_only(k):
        bottom.forward(dense[k])
        z = top.forward(out_fixed, logits=True)
        model.head(z, labels[k])
        top.backward(model._dz)
        bottom.backward(dx_fixed, need_dx=False)
        top.sgd_(a.lr)
        bottom.sgd_(a.lr)

    ms_dense = timed(graph_of(dense_only, NB), reps)
    macs = sum(i * o for i, o in zip(bsz[:-1], bsz[1:])) + sum(i * o for i, o in zip(tsz[:-1], tsz[1:]))
    # forward + weight gradient + input gradient (no input gradient for the bottom's first layer)
    flops = B * 2 * (3 * macs - bsz[0] * bsz[1])
    l1 = float(model.loss)
    line = {
        "metric": "DLRM full training step samples/s (MLPs + BCE + hot path + Descent), 1 MI355X",
        "value": round(B / (ms_full * 1e-3), 1), "unit": "samples/s", "ms_per_step": round(ms_full, 4),
        "hot_path_ms": round(ms_hot, 4), "dense_only_ms": round(ms_dense, 4),
        "dense_flop_per_step": flops, "dense_tflops": round(flops / (ms_dense * 1e-3) / 1e12, 2),
        "dense_frac_of_fp32_matrix_peak": round(flops / (ms_dense * 1e-3) / 1e12 / FP32_MATRIX_PEAK_TFLOPS, 4),
        "dtype": "f32", "data": "synthetic (uniform indices, Bernoulli(0.25) labels, N(0,1) dense)",
        "config": {"workload": a.workload, "tables": T, "dim": D, "batch": B, "bottom_mlp": bsz, "top_mlp": tsz,
                   "launch": f"hipGraph replay ({NB} steps per graph)"},
        "loss_first_warmup_to_last": [round(l0, 5), round(l1, 5)],
    }
    print(json.dumps(line))


if __name__ == "__main__":
    main()
