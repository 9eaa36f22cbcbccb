"""Benchmark of the DLRM embedding + interaction hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--no-cpu-baseline]

One step = one training pass of the hot path over one batch (src/train/train.jl:215-227 minus
the dense MLPs): maplookup -> DotInteraction -> dot_back -> update!(Descent) of the tables,
with the dense vector x and dLoss/d(out) supplied as synthetic inputs already in HBM.
Default workload (BASELINE metric): 26 Criteo-Kaggle tables (criteo.jl:350-377) x 128-dim
fp32, 2048 samples per GPU, one-hot int32 indices drawn uniformly per table, 64 distinct
batches cycled (their touched rows far exceed the 256 MiB Infinity Cache, so the timed gathers
read HBM, not a warm MALL).  N > 1 (under torchrun, or without a launcher: bench.py then starts one
process per GPU itself): tables sharded by table across ranks, per-GPU batch fixed
(weak scaling), RCCL all-to-all of the looked-up vectors forward and of their gradients
backward (dlrm.jl_amd/sharded.py).  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import dlrm_pkg  # noqa: E402

METRIC = "DLRM samples/sec (fwd+bwd), 26 tables×128-dim bs=2048; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured float4 copy
NBATCH = 64  # distinct index batches cycled (--nbatch)
CHUNK = 64  # steps per captured hipGraph


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=640)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--graph-steps", type=int, default=CHUNK,
                    help="steps per captured hipGraph, rounded down to whole cycles over the index batches "
                         "(the per-replay launch gap is paid once per graph)")
    ap.add_argument("--workload", default="kaggle-d128-b2048")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: the global batch (split evenly over the ranks; e.g. configs[3]: "
                         "--workload terabyte-d128-zipf --global-batch 2048 = 256 per GPU at 8 GPUs); 0 (default): "
                         "weak scaling, the workload's batch per GPU")
    ap.add_argument("--micro", type=int, default=0,
                    help="multi-GPU: micro-batches per step (the exchange of one overlaps the compute of the next); "
                         "0: 1 -- M = 2 halves every launch and its exchanges must stay on the capture's origin "
                         "stream (RCCL captured on a forked stream crashes hipStreamEndCapture on this HIP), so it "
                         "measured 161 us against 160 us (tools/shard_sim.py, world 8, stand-in exchanges; DESIGN.md §6)")
    ap.add_argument("--shard-graph", choices=["full", "segments"], default="full",
                    help="multi-GPU graph form: 'full' (default) = one hipGraph per step with the RCCL "
                         "all-to-alls inside (falls back to 'segments' where the capture is refused, e.g. gloo); "
                         "'segments' = the compute between eager collectives")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--mode", choices=["auto", "graph", "eager"], default="auto",
                    help="auto: hipGraph replay, except eager launches for pooled bags on one GPU (measured "
                         "2.10M vs 2.00M samples/s: eager lets the side-stream indexer overlap the gather)")
    ap.add_argument("--overlap-indexer", type=int, default=-1, help="-1: the engine's default")
    ap.add_argument("--fused", type=int, default=1)
    ap.add_argument("--chunk", type=int, default=-1,
                    help="the wave build's chunk limit (16 or 32; 0: the library's default 32); -1 (default): "
                         "pkg.step_chunk (16 for uniform one-hot batches, 32 for Zipf rows)")
    ap.add_argument("--parts", type=int, default=-1,
                    help="parts per table of the step's wave build (16, 32 or 64; 0: the library's 16); -1 "
                         "(default): pkg.step_parts (32 for rows <= 256 B)")
    ap.add_argument("--materialize-ys", type=int, default=-1,
                    help="1: forward writes ys and backward reads it (reference data flow); 0: backward "
                         "re-gathers T; -1 (default): 0 where it applies (fused, lookups=1)")
    ap.add_argument("--stage-timing", type=int, default=1, help="0: skip the per-stage telemetry (traces)")
    ap.add_argument("--ceiling", type=int, default=1,
                    help="1: measure this box's stream and 512-B-row gather rates beside the 8 TB/s spec (rank 0)")
    ap.add_argument("--chain", type=int, default=1,
                    help="1: also time the reference's operator chain on HipTables (the drop-in path; one GPU)")
    ap.add_argument("--nbatch", type=int, default=NBATCH, help="distinct index batches cycled")
    ap.add_argument("--sustain", type=float, default=2.0,
                    help="seconds of back-to-back steps timed after the K-step region (reported as 'sustained')")
    ap.add_argument("--probe-region", default="",
                    help="comma-separated step counts: print the timed region's ms per step for each (graph "
                         "launch overhead vs K) and exit")
    ap.add_argument("--pipeline", type=int, default=-1,
                    help="where the step's indexer is built: 0 in the forward's launch; 2 inside the previous "
                         "step's apply launch, so the forward only gathers (step API, batches <= 2048); 1 the next "
                         "batch's indexer on a side stream during the step; -1 (default, pkg.step_pipeline): 2 for "
                         "one-hot batches <= 2048 (round 3: the gather-only forward is shorter than the in-launch "
                         "build; D=128 49.1M vs 43.8M samples/s with 0, D=16 72.6M), 1 for one-hot batches > 2048 "
                         "(configs[2] 73.8M vs 71.7M), 0 for pooled bags")
    return ap.parse_args()


def rank_env(base, rank, world, port):
    """The environment torchrun gives rank `rank` of a one-node job of `world` ranks."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(world, cmd, base_env=None, port=None, poll_s=0.05):
    """`--gpus N` without a launcher (WORLD_SIZE unset): starts N fresh processes of `cmd`, one
    per rank with torchrun's variables (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*; rank r on
    GPU r), before this process touches the GPU, and waits for them.  Returns the job's exit
    code: 0 if every rank exits 0; else the first failing rank's code, after stopping the
    others (a rank that dies leaves its peers blocked in a collective)."""
    import subprocess
    base_env = dict(os.environ if base_env is None else base_env)
    port = port or free_port()
    procs = [subprocess.Popen(cmd, env=rank_env(base_env, r, world, port)) for r in range(world)]
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    for q in live:
                        q.terminate()
            if live:
                time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def algorithmic_bytes(w, B, T, D, L, E, I, uniq, chunks, materialize_ys=True):
    """Per-launch algorithmic HBM bytes of each stage (SURVEY.md §8d formulas)."""
    d, F = D, T + 1
    P = F * (F - 1) // 2
    N = B * L
    ys_w = F * D * E if materialize_ys else 0  # the lookup output, when the forward writes it
    # backward's T: the materialized ys, or x + the T gathered rows (and their indices)
    t_r = F * D * E if materialize_ys else d * E + T * (I + D * E)
    return {
        # fused maplookup + interaction: x, L rows + L indices per table in; (ys and) out written
        "lookup_interact_fwd": B * (d * E + T * L * (I + D * E) + ys_w + (d + P) * E),
        "lookup": T * B * (L * I + L * D * E + D * E),
        "interact_fwd": B * (d * E + (F - 1) * D * E + d * E + (d + P) * E),
        "interact_bwd": B * ((d + P) * E + t_r + F * D * 4 + d * 4),
        "indexer_build": T * N * I + T * N * 4 + uniq * 8 + chunks * 16,
        # positions (perm) + each bag's gradient row once (pooled: shared by its L lookups) +
        # read-modify-write of every touched row + the chunk descriptors
        "sgd_update": T * N * 4 + T * B * D * 4 + uniq * 2 * D * E + chunks * 16,
    }


def step_api_bytes(B, T, D, L, E, I, st, pipelined=False):
    """Per-launch algorithmic HBM bytes of the training-step pair (dlrm_step_fwd / dlrm_step_bwd),
    from the batch's index statistics st: n1 = positions whose row is hit once (updated inside the
    backward), n2 = the other positions, u2 = their distinct rows (one apply chunk each)."""
    d, F = D, T + 1
    P = F * (F - 1) // 2
    N = B * L
    gather = B * (d * E + T * L * (I + D * E))          # x + the indices + the gathered rows
    indexer = T * N * I + T * N * 4 + st["uniq"] * 8 + st["u2"] * 16 + T * N  # + perm, segments, chunks, flags
    return {
        # pipelined: the indexer is its own (side-stream) launch, not part of the forward's
        "lookup_interact_fwd": gather + B * (d + P) * E + (0 if pipelined else indexer),
        "indexer_build": indexer,
        # dout, x, the re-gathered rows, the once-hit flags; dx and dt's x rows, dt rows of repeated
        # positions, once-hit rows written back after their SGD step
        "interact_bwd": B * (d + P) * E + gather + T * N + B * (d * 4 + D * 4) + st["n2"] * D * 4 + st["n1"] * D * E,
        "sgd_update": st["n2"] * (4 + D * 4) + st["u2"] * (2 * D * E + 16),
    }


def index_stats(idx_np):
    """idx_np: [T][N] -> n1 (positions of once-hit rows), n2 (the rest), u2 (distinct repeated rows), uniq."""
    n1 = n2 = u2 = uniq = 0
    for row in idx_np:
        _, cnt = np.unique(row, return_counts=True)
        uniq += len(cnt)
        n1 += int((cnt == 1).sum())
        n2 += int(cnt[cnt > 1].sum())
        u2 += int((cnt > 1).sum())
    return {"n1": n1, "n2": n2, "u2": u2, "uniq": uniq}


def make_inputs(pkg, w, B, dev, rank, T_rows, nbatch):
    """Tables ~ ScaledUniform (model.jl:61-65), x ~ N(0,1), dout ~ N(0, 1e-3)."""
    g = torch.Generator(device=dev).manual_seed(51234 + rank)  # model.jl:193 seed
    dt = torch.float32 if w["dtype"] == "f32" else torch.bfloat16
    D, L = w["dim"], w["lookups"]
    tables = []
    for n in T_rows:
        s = 1.0 / float(np.sqrt(n))
        # drawn in the table dtype directly (a 293M-row Terabyte table has no room for an fp32 copy)
        tables.append(torch.empty((n, D), dtype=dt, device=dev).uniform_(-s, s, generator=g))
    idx = []
    zipf = w.get("zipf")
    rng = np.random.default_rng(51234 + rank)
    perms = [pkg.zipf_perm(rng, n) for n in T_rows] if zipf else None  # the same rows stay hot
    for _ in range(nbatch):
        if zipf:
            cols = [torch.from_numpy(pkg.zipf_rows(rng, n, B * L, zipf, p)) for n, p in zip(T_rows, perms)]
            idx.append(torch.stack(cols).to(dev).contiguous())
            continue
        cols = [torch.randint(0, n, (B * L,), device=dev, generator=g, dtype=torch.int64).to(torch.int32)
                for n in T_rows]
        idx.append(torch.stack(cols).contiguous())
    return tables, idx, g


def cpu_baseline(pkg, w, seconds, threads):
    """Times the C restatement (oracle/, OpenMP) of the same step on the host: full-size
    tables in DRAM, same batch size.  Rank 0, N=1 only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    native = oracle.use_native()  # gcc -march=native on this host (falls back to the x86-64-v3 build)
    model, host_cpus, allowed = oracle.host_cpu()
    rows = w["rows"]
    D, B, L = w["dim"], w["batch"], w["lookups"]
    T = len(rows)
    F = T + 1
    P = F * (F - 1) // 2
    rng = np.random.default_rng(51234)
    tables = []
    for t, n in enumerate(rows):
        a = np.empty((n, D), dtype=np.float32)
        oracle.fill_uniform(a, -1.0 / np.sqrt(n), 1.0 / np.sqrt(n), 1000 + t, threads)
        tables.append(a)
    if w.get("zipf"):
        batches = [np.stack([pkg.zipf_rows(rng, n, B * L, w["zipf"]) for n in rows]).astype(np.int64) for _ in range(4)]
    else:
        batches = [np.stack([rng.integers(0, n, size=B * L) for n in rows]).astype(np.int64) for _ in range(4)]
    x = rng.standard_normal((B, D)).astype(np.float32)
    dout = (rng.standard_normal((B, D + P)) * 1e-3).astype(np.float32)
    ys = np.zeros((B, F * D), dtype=np.float32)

    def step(k):
        idx = batches[k % len(batches)]
        oracle.maplookup(tables, idx, 0, B, L, ys, D, threads)
        oracle.interact_fwd(x, ys, F, 0, threads)
        dx, dt = oracle.interact_bwd(dout, ys, D, F, 0, threads)
        oracle.sgd_update(tables, idx, 0, B, L, dt, D, 0.01, threads)

    step(0)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step(n + 1)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    del tables
    return {"value": B * n / el, "unit": "samples/s", "cores": threads, "kind": "port",
            "cpu_model": model, "host_cpus": host_cpus, "cpus_allowed": allowed,
            "build": "gcc -O3 -march=native -fopenmp" if native else "gcc -O3 -march=x86-64-v3 -fopenmp",
            "sample": f"C/OpenMP restatement of the same step (oracle/dlrm_oracle.c), {T} tables x {D} "
                      f"fp32 in host DRAM ({sum(rows) * D * 4 / 1e9:.1f} GB), B={B}, {n} timed steps "
                      f"({el:.1f} s) after 1 warm-up, {threads} OpenMP threads on {model}; not the Julia "
                      f"reference (no julia toolchain)"}


def measured_ceiling(dev, row_bytes):
    """The HBM rates this box reaches with hand-written gfx950 kernels (tools/bw_probe.hip, built
    into dlrm.jl_amd/lib/libdlrm_probe.so), beside the 8 TB/s spec (report both): a
    1 GiB nontemporal copy (read + write), a 1 GiB read, and reads of 262,144 random line-aligned rows
    of 512 B, of this workload's row size and of 64 B from a 4 GiB buffer (tools/fetch_probe.hip's
    shape) -- each the best of 5 HIP-event-timed launches on the current stream after a warm-up."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "dlrm.jl_amd", "lib", "libdlrm_probe.so"))
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    lib.dlrm_probe_copy.argtypes = [vp, vp, i64, vp]
    lib.dlrm_probe_read.argtypes = [vp, i64, vp, vp]
    lib.dlrm_probe_gather.argtypes = [vp, i64, ctypes.c_int, ctypes.c_int, vp, vp]
    st = vp(torch.cuda.current_stream(dev).cuda_stream)

    def best(fn, nbytes, reps=5):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = []
        for _ in range(reps):
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1) * 1e-3)
        return round(nbytes / min(t) / 1e9, 1)
    out = {}
    try:
        n = 1 << 30
        src = torch.empty(n // 4, dtype=torch.float32, device=dev).fill_(1.0)
        dst = torch.empty_like(src)
        sink = torch.empty(1 << 20, dtype=torch.float32, device=dev)
        p = lambda t: vp(t.data_ptr())  # noqa: E731
        out["stream_copy_GBps"] = best(lambda: lib.dlrm_probe_copy(p(src), p(dst), n, st), 2 * n)
        out["stream_read_GBps"] = best(lambda: lib.dlrm_probe_read(p(src), n, p(sink), st), n)
        del src, dst
        big = torch.empty((4 << 30) // 4, dtype=torch.float32, device=dev).fill_(1.0)
        rows = 262144
        for rb in sorted({512, int(row_bytes), 64}):
            if rb in (64, 128, 256, 512, 1024):
                out[f"gather_{rb}B_GBps"] = best(lambda: lib.dlrm_probe_gather(p(big), 4 << 30, rb, rows, p(sink), st),
                                                 rows * rb)
        out["gather_GBps"] = out.get(f"gather_{int(row_bytes)}B_GBps")
        out["gather_row_bytes"] = int(row_bytes)
        out["method"] = ("tools/bw_probe.hip, best of 5 HIP-event-timed launches: 1 GiB nontemporal copy "
                         "(read+write bytes), 1 GiB read, 262,144 random line-aligned rows read from 4 GiB")
        del big
        torch.cuda.empty_cache()
    except Exception as e:  # (memory / API trouble: reported, never fatal)
        out["error"] = repr(e)
    return out


def load_prof(workload):
    """The committed rocprofv3 summary of this workload (tools/profile.sh -> profiles/pmc_<workload>.json:
    per-stage rocprof average durations, PMC HBM bytes and MFMA busy fractions, with the HEAD it was
    taken at), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            prof = json.load(f)
    except Exception:
        return None
    # a workload whose fused forward is two kernels (pooled bags: maplookup + the interaction on ys)
    # has them as two profiler stages; the bench times them as one (lookup_interact_fwd)
    if "lookup_interact_fwd" not in prof and "lookup" in prof and "interact_fwd" in prof:
        a, b = prof["lookup"], prof["interact_fwd"]
        comb = {"avg_us": a["avg_us"] + b["avg_us"], "kernels": a.get("kernels", []) + b.get("kernels", [])}
        if "hbm_bytes_per_launch" in a and "hbm_bytes_per_launch" in b:
            comb["hbm_bytes_per_launch"] = a["hbm_bytes_per_launch"] + b["hbm_bytes_per_launch"]
        if "mfma_busy" in a or "mfma_busy" in b:
            comb["mfma_busy"] = max(a.get("mfma_busy", 0.0), b.get("mfma_busy", 0.0))
        prof["lookup_interact_fwd"] = comb
    return prof


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no outside launcher: one fresh process per rank, started before anything here touches the
        # GPU (torch.cuda.device_count() does not initialise it on this stack)
        backend = os.environ.get("DLRM_DIST_BACKEND", "nccl")
        if backend == "nccl" and torch.cuda.device_count() < a.gpus:
            raise SystemExit(f"--gpus {a.gpus}: only {torch.cuda.device_count()} GPU(s) visible (RCCL needs one "
                             f"GPU per rank; DLRM_DIST_BACKEND=gloo rehearses ranks sharing one GPU)")
        sys.exit(spawn_ranks(a.gpus, [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]))
    pkg = dlrm_pkg.load()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))  # one rank per GPU on a full node
    torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("DLRM_DIST_BACKEND", "nccl")  # "gloo" only for 1-GPU rehearsals
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    w = dict(pkg.WORKLOADS[a.workload])
    if a.global_batch:
        if a.global_batch % world:
            raise SystemExit(f"--global-batch {a.global_batch} does not split over {world} ranks")
        w["batch"] = a.global_batch // world
    B, D, L = w["batch"], w["dim"], w["lookups"]
    E = 4 if w["dtype"] == "f32" else 2
    if a.pipeline < 0:
        # in-apply build where the forward's gather is shorter than its in-launch indexer: rows of
        # <= 256 B (D=16 fp32; Terabyte bf16 x 128: 45.6M vs 41.9M samples/s, profiles/r5c_*);
        # the same choice tests/test_configs.py checks against the oracle (shapes.step_pipeline)
        a.pipeline = {None: 0, "side": 1, "apply": 2}[pkg.step_pipeline(w)]
    if a.mode == "auto":
        a.mode = "eager" if (L > 1 and world == 1) else "graph"
    rows = w["rows"]
    T = len(rows)
    nb = a.nbatch

    if world == 1:
        tables, idx, g = make_inputs(pkg, w, B, dev, rank, rows, nb)
        ts = pkg.EmbeddingTableSet(tables)
        engine = pkg.HotPath(ts, B, L, lr=a.lr, index_base=0,
                             overlap_indexer=None if a.overlap_indexer < 0 else bool(a.overlap_indexer),
                             fused=bool(a.fused),
                             materialize_ys=None if a.materialize_ys < 0 else bool(a.materialize_ys),
                             pipeline={0: None, 1: "side", 2: "apply"}[a.pipeline],
                             chunk=pkg.step_chunk(w) if a.chunk < 0 else (a.chunk or None),
                             parts=pkg.step_parts(w) if a.parts < 0 else (a.parts or None))
        F = T + 1
        dtp = tables[0].dtype
        x = torch.randn((B, D), device=dev, generator=g).to(dtp)
        dout = (torch.randn((B, engine.width), device=dev, generator=g) * 1e-3).to(dtp)
        packs = [pkg.PackedIndices(i.reshape(T, B, L)) for i in idx]
        for p in packs:
            engine.validate(x, p, dout)

        if engine.pipeline == "apply":
            def step(k):
                engine.step_prep(x, packs[k % nb], dout, packs[(k + 1) % nb])
        elif engine.pipeline:
            def step(k):
                engine.step_next(x, packs[k % nb], dout, packs[(k + 1) % nb])
        else:
            def step(k):
                engine.step(x, packs[k % nb], dout)
    else:
        from dlrm_jl_amd.sharded import make_bench_engine
        micro = a.micro or 1
        engine, step, prepare_graphs = make_bench_engine(pkg, w, B, dev, rank, world, a.lr, nbatch=nb, micro=micro)
        if a.mode == "graph":
            # each whole step (both all-to-alls included) replayed as one hipGraph; where the
            # backend refuses the capture, the compute between eager collectives
            for k in range(max(a.warmup, 1)):
                step(k)
            torch.cuda.synchronize()
            try:
                a.mode = prepare_graphs(full=a.shard_graph == "full")
            except Exception as e:  # capture refused: eager launches (same work)
                print(f"note: graph capture failed ({e!r}); timing eager launches", file=sys.stderr)
                engine._graphs = engine._full = None
                a.mode = "eager"

    # warm-up (also validates indices once)
    for k in range(max(a.warmup, 1)):
        step(k)
    torch.cuda.synchronize()
    if world == 1:
        engine.check_bounds()
    elif engine.ops is not None:
        engine.ops.ctx.check_bounds()

    # hipGraphs: a graph holds up to CHUNK consecutive steps (one index batch each), so the
    # per-replay launch gap (~8 us measured on MI355X) is paid once per graph, not per step.
    # The timed K steps replay graphs of exactly the steps they stand for: full CHUNK-step graphs
    # plus one graph of the remainder (captured once here, outside the timed region).
    nb = a.nbatch
    # (a whole number of cycles over the nb index batches, so every piece starts at batch 0, the
    # state the pipelined indexer is primed to)
    chunk = nb * max(1, a.graph_steps // nb)
    graphs = {}
    def prime():
        """Pipelined steps: the indexer the first step of a run reads holds batch 0 (a run starts
        at batch 0; the graphs were captured from this state)."""
        if world == 1 and engine.pipeline:
            engine.prime(packs[0], x=x, dout=dout, prev=packs[nb - 1])

    prime()

    def capture(start, n):
        prime()  # every piece is captured from the state it is replayed in (indexer primed for batch 0)
        cur = torch.cuda.current_stream()
        s = torch.cuda.Stream()
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                for k in range(start, start + n):
                    step(k)
        cur.wait_stream(s)
        gr.replay()
        return gr

    def plan(n):
        """(start, length) pieces of steps [0, n): whole chunks cycling over the nb batches + a tail."""
        out, k = [], 0
        while n - k >= chunk:
            out.append(((k % nb), chunk))
            k += chunk
        if n > k:
            out.append(((k % nb), n - k))
        return out

    probe = [int(v) for v in a.probe_region.split(",") if v]
    if a.mode == "graph":
        try:
            for piece in set(plan(a.steps)) | set(plan(nb)) | set(plan(a.warmup)) | {p for n in probe for p in plan(n)}:
                if piece not in graphs:
                    graphs[piece] = capture(*piece)
            torch.cuda.synchronize()
        except Exception as e:  # graph capture unsupported: eager
            print(f"note: graph capture failed ({e!r}); timing eager launches", file=sys.stderr)
            graphs = None
    else:
        graphs = None

    def run_steps(n):
        """n consecutive steps starting at batch 0."""
        if graphs is None:
            for k in range(n):
                step(k)
            return
        for piece in plan(n):
            graphs[piece].replay()

    local_ms = [0.0]  # this rank's ms per step in the last timed region

    def timed(n):
        # the W untimed warm-up steps run right before the region (the first warm-up pass above sits
        # behind graph capture and host work, which leave the GPU idle), then the pipelined indexer
        # is re-primed for batch 0
        # (pipelined graphs are valid only from the state they were captured in: every replayed
        # piece starts at batch 0, so the indexer is re-primed before each run)
        if a.warmup > 0:
            prime()
            run_steps(a.warmup)
        prime()  # (outside the timed region)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_steps(n)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        ms = (time.perf_counter() - t0) * 1e3 / n
        local_ms[0] = ms
        if world > 1:
            tt = torch.tensor([ms], device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            ms = float(tt.item())
        return ms

    if probe:
        res = {}
        for rep in range(3):
            for n in probe:
                res.setdefault(n, []).append(round(timed(n), 5))
        if rank == 0:
            print(json.dumps({"probe_region_ms_per_step": {n: v for n, v in res.items()}}))
        return
    ms = timed(a.steps)
    dist_info = None
    if world > 1:
        # what the job ran on, as the collectives saw it: the rank count of an all-reduce over the
        # default group (RCCL for backend "nccl"), the library communicator's own ncclCommCount when
        # it carries the exchange, each rank's step time (value uses the max) and the table partition
        cdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
        one = torch.ones(1, device=cdev)
        dist.all_reduce(one)
        mine = torch.tensor([local_ms[0]], device=cdev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        E_ = 4 if w["dtype"] == "f32" else 2
        dist_info = {"backend": dist.get_backend(), "ranks_in_allreduce": int(one.item()),
                     "exchange": "abi" if engine.comm is not None else "torch.distributed all_to_all_single",
                     "rccl_comm_nranks": engine.comm.nranks() if engine.comm is not None else None,
                     "rank_ms_per_step": [round(float(t.item()), 4) for t in every],
                     "partition": {"tables_per_rank": [list(o) for o in engine.part.owners],
                                   "gb_per_rank": [round(b / 1e9, 2) for b in
                                                   engine.part.bytes_per_rank(rows, D * E_)]}}
    # sustained: >= a.sustain seconds of back-to-back steps (whole cycles over the nb batches), so a
    # short K does not hide clock ramp or cache effects; reported beside value, not instead of it
    sustained = None
    if a.sustain > 0:
        per = chunk // nb  # (whole graphs: every piece of the run was captured)
        cyc = max(1, int(np.ceil(a.sustain * 1e3 / (ms * nb))))
        cyc = per * int(np.ceil(cyc / per))
        if world > 1:  # every rank runs the same number of steps
            tc = torch.tensor([cyc], device=dev)
            dist.all_reduce(tc, op=dist.ReduceOp.MAX)
            cyc = int(tc.item())
        ms_s = timed(cyc * nb)
        sustained = {"steps": cyc * nb, "seconds": round(ms_s * cyc * nb / 1e3, 3), "ms_per_step": round(ms_s, 4),
                     "value": round(B * world / (ms_s / 1e3), 1)}
    value = B * world / (ms / 1e3)

    # ---- the drop-in operator chain (what an unchanged train! drives through the shim:
    # maplookup -> rrule(DotInteraction) -> pullback -> maplookup_pullback -> update!) on HipTables,
    # i.e. the fused step kernels reached through the reference's operator API (dlrm.jl_amd/lazy.py)
    chain = None
    if world == 1 and L == 1 and a.chain and graphs is not None:
        ht = pkg.HipTables(ts, lr=a.lr, index_base=0)
        dot = pkg.DotInteraction()
        strat = pkg.PreallocationStrategy(D)
        indexers = pkg.SparseIndexer(T, B, dev)  # train.jl:279 (accepted; the step carries its own)

        def chain_step(k):
            p = packs[k % nb]
            ys = pkg.maplookup(strat, ht, p)
            _, back = pkg.rrule(dot, x, ys)
            _, _, dy = back(dout)
            # the reference's call, train.jl:283-290 (no extra keyword): deferred by the tables' policy
            pkg.update_(pkg.Descent(a.lr), ht, pkg.maplookup_pullback(D, ht, p, dy), indexers, num_splits=8,
                        nthreads=12)

        try:
            for k in range(2):
                chain_step(k)
            ht.flush()  # (update! is deferred into the next maplookup's launch; a graph piece ends flushed)
            gs = {}
            for piece in set(plan(a.steps)) | set(plan(a.warmup)):
                cur = torch.cuda.current_stream()
                s_ = torch.cuda.Stream()
                s_.wait_stream(cur)
                with torch.cuda.stream(s_):
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr, stream=s_):
                        for k in range(piece[0], piece[0] + piece[1]):
                            chain_step(k)
                        ht.flush()
                cur.wait_stream(s_)
                gs[piece] = gr
            for piece in plan(a.warmup):
                gs[piece].replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for piece in plan(a.steps):
                gs[piece].replay()
            torch.cuda.synchronize()
            ms_c = (time.perf_counter() - t0) * 1e3 / a.steps
            ht.check_bounds()
            chain = {"value": round(B / (ms_c / 1e3), 1), "ms_per_step": round(ms_c, 4),
                     "vs_step": round(ms / ms_c, 3),
                     "form": "maplookup(HipTables) -> rrule(DotInteraction) -> pullback -> maplookup_pullback -> "
                             "update!(Descent(η), tables, grads, indexers; num_splits, nthreads) as train.jl:283-290 "
                             "calls it: dlrm_step_fwd / dlrm_step_bwd(BWD_ONLY, which also copies the bounds flag to "
                             "host memory) / the deferred update!'s apply launch, run by the next maplookup with that "
                             "batch's indexer build (dlrm_step_bwd_prepare(APPLY_ONLY)); no host sync per step; "
                             "hipGraph replay"}
        except Exception as e:
            print(f"note: drop-in chain timing failed ({e!r})", file=sys.stderr)

    # ---- per-kernel timing (HIP events on the launch stream) + roofline, rank 0
    roofline = None
    stages = None
    if rank == 0 and world == 1 and a.stage_timing:
        uniq = chunks = 0
        for k in range(nb):
            engine.build_indexer(packs[k])
            torch.cuda.synchronize()
            for t in range(T):
                uniq += len(engine.indexer.unique_rows(t))
        uniq /= nb
        chunks = uniq  # one chunk per unique row, plus a few for hot rows
        bytes_ = algorithmic_bytes(w, B, T, D, L, E, 4, uniq, chunks, engine.materialize_ys)
        # one prebuilt indexer per index batch, so the update stage can be timed on its own
        indexers = [pkg.SparseIndexer(T, B * L, dev) for _ in range(nb)]  # not the engine's own
        for ix in indexers:
            if engine.chunk:
                ix.set_chunk(engine.chunk)  # (the engine's chunk limit)
            if engine.parts:
                ix.set_parts(engine.parts)
        home = engine.indexer
        for k in range(nb):
            engine.indexer = indexers[k]
            engine.build_indexer(packs[k])
        engine.indexer = home

        def apply_k(k):
            engine.indexer = indexers[k]
            engine.sgd_update(packs[k], prebuilt=True)
            engine.indexer = home

        in_bwd = (engine.fused and not engine.materialize_ys and engine.indexer is not None
                  and not engine.overlap_indexer)
        if engine.step_api:
            sts = [index_stats(packs[k].data.reshape(T, B * L).cpu().numpy()) for k in range(nb)]
            st = {key: sum(v[key] for v in sts) / nb for key in sts[0]}
            bytes_ = step_api_bytes(B, T, D, L, E, 4, st, pipelined=bool(engine.pipeline))
            for k in range(nb):  # batch k's split indexer, built by its own step forward
                engine.indexer = indexers[k]
                engine.step_fwd(x, packs[k])
            engine.indexer = home

            def sbwd_k(k, flags):
                engine.indexer = indexers[k]
                engine.step_bwd(dout, x=x, idx=packs[k], flags=flags)
                engine.indexer = home

        def bwd_index_k(k):
            engine.indexer = indexers[k]
            engine.interact_bwd(dout, x=x, idx=packs[k], build_indexer=True)
            engine.indexer = home

        if engine.pipeline == "apply":  # the next batch's indexer built by the apply launch
            names = ["lookup_interact_fwd", "interact_bwd", "sgd_update"]
            nxt = [pkg.SparseIndexer(T, B * L, dev) for _ in range(2)]
            for ix in nxt:
                if engine.chunk:
                    ix.set_chunk(engine.chunk)
                if engine.parts:
                    ix.set_parts(engine.parts)

            def apply_prep_k(k):
                engine.indexer = indexers[k]
                engine.step_bwd(dout, x=x, idx=packs[k], flags=pkg._lib.STEP_APPLY_ONLY,
                                prepare=(nxt[k % 2], packs[(k + 1) % nb]))
                engine.indexer = home

            fns = [lambda k: engine.lookup_interact_fwd(x, packs[k]), lambda k: sbwd_k(k, pkg._lib.STEP_BWD_ONLY),
                   apply_prep_k]
            bytes_["sgd_update"] += bytes_["indexer_build"]
        elif engine.pipeline and L > 1:  # pooled bags: the next batch's bag build beside the apply
            names = ["lookup_interact_fwd", "interact_bwd", "sgd_update", "indexer_build"]

            def build_k(k):
                engine.indexer = indexers[k]
                engine.build_indexer(packs[k])
                engine.indexer = home

            fns = [lambda k: engine.lookup_interact_fwd(x, packs[k]), lambda k: engine.interact_bwd(dout, x=x, idx=packs[k]),
                   apply_k, build_k]
        elif engine.pipeline:  # indexer on the side stream, built for the next batch
            names = ["lookup_interact_fwd", "interact_bwd", "sgd_update", "indexer_build"]
            fns = [lambda k: engine.lookup_interact_fwd(x, packs[k]), lambda k: sbwd_k(k, pkg._lib.STEP_BWD_ONLY),
                   lambda k: sbwd_k(k, pkg._lib.STEP_APPLY_ONLY),
                   lambda k: engine.build_split(indexers[k], packs[k])]
        elif engine.step_api:  # indexer in the forward's launch; once-hit rows updated by the backward
            names = ["lookup_interact_fwd", "interact_bwd", "sgd_update"]
            fns = [lambda k: engine.step_fwd(x, packs[k]), lambda k: sbwd_k(k, pkg._lib.STEP_BWD_ONLY),
                   lambda k: sbwd_k(k, pkg._lib.STEP_APPLY_ONLY)]
        elif in_bwd:  # the indexer is built inside the backward's launch
            names = ["lookup_interact_fwd", "interact_bwd", "sgd_update"]
            fns = [lambda k: engine.lookup_interact_fwd(x, packs[k]), bwd_index_k, apply_k]
            bytes_["interact_bwd"] += bytes_["indexer_build"]
        elif engine.fused:
            names = ["lookup_interact_fwd", "indexer_build", "interact_bwd", "sgd_update"]
            fns = [lambda k: engine.lookup_interact_fwd(x, packs[k]), lambda k: engine.build_indexer(packs[k]),
                   lambda k: engine.interact_bwd(dout, x=x, idx=packs[k]), apply_k]
        else:
            names = ["lookup", "interact_fwd", "indexer_build", "interact_bwd", "sgd_update"]
            fns = [lambda k: engine.lookup(packs[k]), lambda k: engine.interact_fwd(x),
                   lambda k: engine.build_indexer(packs[k]), lambda k: engine.interact_bwd(dout, x=x, idx=packs[k]),
                   apply_k]
        # Each stage: a hipGraph of its kernel(s) over the nb index batches (the same batches the
        # timed loop cycles, so caches are no warmer than there), replayed REPS times between two HIP
        # events on the launch stream; per-launch time = elapsed / (REPS * nb).  Back-to-back
        # graph nodes carry no event markers, so this agrees with rocprofv3's per-kernel average.
        reps = max(2, min(8, a.steps // nb))
        stages = {}
        cur = torch.cuda.current_stream()
        for n, fn in zip(names, fns):
            gr = None
            if graphs is not None:
                s = torch.cuda.Stream()
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr, stream=s):
                        for k in range(nb):
                            fn(k)
                cur.wait_stream(s)

            def once():
                if gr is not None:
                    gr.replay()
                else:
                    for k in range(nb):
                        fn(k)

            once()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            for _ in range(reps):
                once()
            e1.record(cur)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / (reps * nb)
            stages[n] = {"us": round(us, 2), "alg_bytes": int(bytes_[n]),
                         "GBps": round(bytes_[n] / (us * 1e-6) / 1e9, 1)}
        for n in names:
            stages[n]["frac"] = round(stages[n]["GBps"] / HBM_PEAK_GBS, 4)
        # the dominant kernel of the step's critical path (a side-stream stage overlaps it): the
        # longest launch in the committed rocprofv3 summary of this workload when it has every stage
        # (the same kernels, timed by the profiler), else by the HIP-event timings above
        crit = [n for n in names if not (engine.pipeline == "side" and n == "indexer_build")]
        prof = load_prof(a.workload)
        have = prof is not None and all(n in prof and "avg_us" in prof[n] for n in crit)
        dom = max(crit, key=lambda n: prof[n]["avg_us"] if have else stages[n]["us"])
        ach = stages[dom]["GBps"]
        step_bytes = sum(bytes_[n] for n in names)  # every launch of one step (side-stream work included)
        step_gbs = step_bytes / (ms * 1e-3) / 1e9
        # SURVEY.md §8(d)'s un-fused per-sample bytes (BASELINE.md's denominator: 112.6 KB/sample at the
        # metric config): per (sample, table) the gather L*I + L*D*E + D*E and the scatter-SGD
        # D*E + L*I + 2*D*E (U = B, no dedupe), plus the interaction's fwd F*D*E + (d+P)*E and bwd
        # (d+P)*E + 2*F*D*E + d*E
        Fu, Pu = T + 1, (T + 1) * T // 2
        unfused = B * (T * (2 * L * 4 + L * D * E + 4 * D * E) + Fu * D * E + (D + Pu) * E
                       + (D + Pu) * E + 2 * Fu * D * E + D * E)
        unf_gbs = unfused / (ms * 1e-3) / 1e9
        roofline = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": (prof or {}).get(dom, {}).get("hbm_bytes_per_launch"),
                    "alg_bytes_per_launch": int(bytes_[dom]), "avg_launch_us": stages[dom]["us"],
                    "step": {"alg_bytes": int(step_bytes), "ms": round(ms, 4), "GBps": round(step_gbs, 1),
                             "frac": round(step_gbs / HBM_PEAK_GBS, 4),
                             "bytes_basis": "fused: the algorithmic bytes of this step's own launches (frac); "
                                            "frac_unfused: SURVEY §8(d)'s un-fused per-sample bytes (BASELINE.md)",
                             "unfused_bytes": int(unfused), "frac_unfused": round(unf_gbs / HBM_PEAK_GBS, 4)},
                    "stages": stages}
        if a.ceiling:
            roofline["measured_ceiling"] = measured_ceiling(dev, D * E)
            cg = roofline["measured_ceiling"].get("gather_GBps")
            if cg:
                roofline["frac_of_measured_gather"] = round(ach / cg, 4)
        if prof is not None:
            roofline["profile"] = {"file": f"profiles/pmc_{a.workload}.json", "head": prof.get("head"),
                                   "dominant_by": "rocprofv3 avg duration" if have else "HIP events",
                                   "rocprof_avg_us": {n: round(prof[n]["avg_us"], 2) for n in names
                                                      if n in prof and "avg_us" in prof[n]}}
            # PMC HBM traffic (2 FETCH_SIZE + WRITE_SIZE per launch) beside each stage's algorithmic bytes:
            # a stage whose frac counts cache re-reads (pooled Zipf rows) shows traffic well below them
            for n in names:
                tb = prof.get(n, {}).get("hbm_bytes_per_launch")
                if tb:
                    stages[n]["traffic"] = int(tb)
                    stages[n]["traffic_GBps"] = round(tb / (stages[n]["us"] * 1e-6) / 1e9, 1)
            mf = {n: round(prof[n]["mfma_busy"], 4) for n in names if n in prof and "mfma_busy" in prof[n]}
            if mf:  # north_star: MFMA utilisation of the interaction kernels (SIMD-cycle fraction)
                roofline["mfma"] = mf

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and w["dtype"] == "f32":
        # every CPU this process may run on, capped by the OMP_NUM_THREADS share the host grants a
        # one-GPU job (16 on the GPU box; its machine has more: host_cpus in the line)
        allowed = len(os.sched_getaffinity(0))
        cap = int(os.environ.get("OMP_NUM_THREADS", "0"))
        threads = min(allowed, cap) if cap > 0 else allowed
        try:
            cpu = cpu_baseline(pkg, w, a.cpu_seconds, threads)
        except Exception as e:
            print(f"note: cpu baseline failed: {e!r}", file=sys.stderr)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
            "scaling": "strong" if a.global_batch else "weak",
            "vs_baseline": None, "dtype": w["dtype"],
            "data": (f"synthetic ({'Zipf(%g) over permuted rows' % w['zipf'] if w.get('zipf') else 'uniform'} "
                     "indices, ScaledUniform tables, N(0,1) x, N(0,1e-3) dLoss/dout)"),
            "config": {"workload": a.workload, "tables": T, "dim": D, "batch_per_gpu": B, "global_batch": B * world,
                       "lookups": L, "index_dtype": "int32", "table_rows": w.get("rows_src", "Criteo-Kaggle (criteo.jl:350-377)"),
                       "parallelism": ("single-gpu" if world == 1 else f"table-sharded x{world} + "
                                       + ("RCCL all-to-all" if dist.get_backend() == "nccl" else
                                          f"{dist.get_backend()} all-to-all (host-staged rehearsal)")),
                       "index_batches": nb,
                       **({"chunk_limit": engine.chunk or 32} if world == 1 and engine.step_api else {}),
                       **({"micro_batches": engine.M} if world > 1 else {}),
                       "launch": (f"hipGraph replay (<= {chunk} steps per graph)" if graphs is not None else
                                  "hipGraph replay of each whole step, RCCL all-to-alls captured inside"
                                  if a.mode == "full" else
                                  "hipGraph replay of the compute between eager all-to-alls" if a.mode == "segments"
                                  else "eager"),
                       "ys": ("received blocks read in place (no ys)" if world > 1 else "materialized"
                              if engine.materialize_ys else "not materialized (backward re-gathers T)"),
                       "step": ("3 launches: fused lookup + interaction (gather only) / dlrm_step_bwd_prepare = "
                                "interaction backward with once-hit rows updated + apply of repeated rows, whose launch "
                                "also builds the next batch's indexer"
                                if world == 1 and engine.pipeline == "apply" else
                                "fused forward + dlrm_step_bwd (once-hit rows updated in the backward); the next "
                                "batch's indexer built on a side stream during the step"
                                if world == 1 and engine.pipeline else
                                "dlrm_step_fwd/dlrm_step_bwd (indexer in the forward launch, once-hit rows "
                                "updated in the backward)" if world == 1 and engine.step_api else "operators")},
            **({"distributed": dist_info} if dist_info else {}),
            "sustained": sustained, "drop_in_chain": chain, "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        # captured graphs hold RCCL work and keep a reference on the communicator: release them
        # first, or destroying the process group waits on them forever
        engine.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
