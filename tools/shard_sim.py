"""Compute-side timing of one rank of the table-sharded step, on one GPU.

Builds rank R of a WORLD-rank run of a bench workload (its own tables at full size, the
global-batch indices, the received-table buffer) and times the three compute segments the
bench replays between the two all-to-alls (seg_lookup, seg_interact, seg_update) as
hipGraphs with HIP events.  The exchanges themselves are not run (no peers): their time is
the RCCL all-to-all of the sizes printed.

    python tools/shard_sim.py [--world 8] [--rank 0] [--workload kaggle-d128-b2048] [--micro M]
                              [--global-batch G]   (strong scaling: B = G / world per rank)
Segments are timed summed over the step's micro-batches; "main_stream" = index-free compute of one
step (lookup + interaction + update), what the exchanges overlap with.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--workload", default="kaggle-d128-b2048")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--micro", type=int, default=0, help="0: make_bench_engine's default")
    ap.add_argument("--global-batch", type=int, default=0)
    a = ap.parse_args()
    pkg = dlrm_pkg.load()
    from dlrm_jl_amd import sharded
    dev = torch.device("cuda:0")
    w = dict(pkg.WORKLOADS[a.workload])
    B = a.global_batch // a.world if a.global_batch else w["batch"]

    class NoExchange(sharded.ShardedHotPath):
        def exchange_fwd(self, m=0):
            pass

        def exchange_bwd(self, m=0):
            pass

    sharded.ShardedHotPath = NoExchange
    eng, step, prepare = sharded.make_bench_engine(pkg, w, B, dev, a.rank, a.world, 0.01, micro=a.micro or None)
    M = eng.M
    for k in range(3):
        step(k)
    torch.cuda.synchronize()
    prepare()
    look, mid, upd, ixg = eng._graphs
    res = {}
    for name, fn in (("seg_index", lambda k: ixg[k % 8].replay()),
                     ("seg_lookup", lambda k: [g.replay() for g in look[k % 8]]),
                     ("seg_interact", lambda k: [g.replay() for g in mid]),
                     ("seg_update", lambda k: upd[k % 8].replay()), ("step", lambda k: eng.step_graphed(k % 8))):
        for k in range(5):
            fn(k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        h0 = time.perf_counter()
        for k in range(a.iters):
            fn(k)
        h1 = time.perf_counter()
        e.record()
        torch.cuda.synchronize()
        res[name] = round(s.elapsed_time(e) * 1e3 / a.iters, 2)
        res["host_" + name] = round((h1 - h0) * 1e6 / a.iters, 2)  # launch-side time per replay
    res["main_stream"] = round(res["seg_lookup"] + res["seg_interact"] + res["seg_update"], 2)
    res["micro_batches"], res["batch_per_rank"] = M, B
    E = 4 if w["dtype"] == "f32" else 2
    res["a2a_fwd_bytes_out"] = eng.send.numel() * E
    res["a2a_bwd_bytes_out"] = eng.gsend.numel() * 4
    res["tables_here"] = eng.Tr
    res["world"], res["rank"], res["workload"] = a.world, a.rank, a.workload
    print(json.dumps(res))


if __name__ == "__main__":
    main()
