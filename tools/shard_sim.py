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

--exchange sleep: each all-to-all is stood in for by a spin kernel (torch.cuda._sleep, one wave) as
long as the exchange of that micro-batch would take over xGMI: the bytes this rank sends to its
peers / (7 links x --link-gbs).  With --graph full the whole step (index build, lookups, stand-in
exchanges on the comm stream, interaction, update) is captured as ONE hipGraph per index batch
(capture_full), so M > 1 overlap is measured without per-segment launches; "step" is then the
replayed whole step, and "host_step" its launch-side cost.
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
    ap.add_argument("--exchange", choices=["none", "sleep"], default="none")
    ap.add_argument("--link-gbs", type=float, default=100.0,
                    help="per-link xGMI rate an all-to-all reaches (spec 153 GB/s per direction)")
    ap.add_argument("--graph", choices=["segments", "full"], default="segments")
    a = ap.parse_args()
    pkg = dlrm_pkg.load()
    from dlrm_jl_amd import sharded
    dev = torch.device("cuda:0")
    w = dict(pkg.WORKLOADS[a.workload])
    B = a.global_batch // a.world if a.global_batch else w["batch"]

    cyc_per_us = [0.0]
    if a.exchange == "sleep":  # calibrate the spin kernel (clock64 cycles per microsecond)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1000)
        s.record()
        torch.cuda._sleep(2_000_000)
        e.record()
        torch.cuda.synchronize()
        cyc_per_us[0] = 2_000_000 / (s.elapsed_time(e) * 1e3)

    def spin(nbytes_to_peers):
        us = nbytes_to_peers / (7 * a.link_gbs * 1e3)  # bytes / (7 links x GB/s) in microseconds
        torch.cuda._sleep(max(1, int(us * cyc_per_us[0])))

    class SimExchange(sharded.ShardedHotPath):
        def exchange_fwd(self, m=0):
            if a.exchange == "sleep":
                spin(self.send[m].numel() * self.send.element_size() * (self.world - 1) / self.world)

        def exchange_bwd(self, m=0):
            if a.exchange == "sleep":
                spin(self.gsend[m].numel() * 4 * (self.world - 1) / self.world)

        def capture_full(self, x, idx_list, dout):
            s = torch.cuda.Stream(device=self.out.device)
            s.wait_stream(torch.cuda.current_stream())
            graphs = []
            with torch.cuda.stream(s):
                for idx in idx_list:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=s):
                        self.step(x, idx, dout)
                    graphs.append(g)
            torch.cuda.current_stream().wait_stream(s)
            self._full = graphs

    sharded.ShardedHotPath = SimExchange
    eng, step, prepare = sharded.make_bench_engine(pkg, w, B, dev, a.rank, a.world, 0.01, micro=a.micro or None)
    M = eng.M
    for k in range(3):
        step(k)
    torch.cuda.synchronize()
    prepare(full=False)
    look, mid, upd, ixg = eng._graphs
    full = None
    if a.graph == "full":
        x_, dout_ = eng._bench_x, eng._bench_dout
        eng.capture_full(x_, eng.bench_packs, dout_)
        full = eng._full
    res = {}
    stages = [("seg_index", lambda k: ixg[k % 8].replay()),
              ("seg_lookup", lambda k: [g.replay() for g in look[k % 8]]),
              ("seg_interact", lambda k: [g.replay() for g in mid]),
              ("seg_update", lambda k: upd[k % 8].replay())]
    if full is not None:
        stages.append(("step", lambda k: full[k % 8].replay()))
    else:
        eng._full = None
        stages.append(("step", lambda k: eng.step_graphed(k % 8)))
    for name, fn in stages:
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
    res["exchange"], res["graph"] = a.exchange, a.graph
    if a.exchange == "sleep":
        res["link_gbs"] = a.link_gbs
        res["a2a_fwd_us"] = round(res["a2a_fwd_bytes_out"] * (a.world - 1) / a.world / (7 * a.link_gbs * 1e3), 2)
        res["a2a_bwd_us"] = round(res["a2a_bwd_bytes_out"] * (a.world - 1) / a.world / (7 * a.link_gbs * 1e3), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
