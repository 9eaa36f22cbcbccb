"""Per-operation device times of the hot path's launches on one workload (default: the BASELINE
metric shape, 26 Kaggle tables x 128 fp32, B=2048), each op captured over 8 index batches into a
hipGraph and replayed between two HIP events.  For comparing kernel variants on the GPU box:

    python tools/stage_times.py [--workload NAME] [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlrm_pkg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="kaggle-d128-b2048")
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--zipf", type=float, default=0.0)
a = ap.parse_args()
pkg = dlrm_pkg.load()
dev = torch.device("cuda:0")
w = pkg.WORKLOADS[a.workload]
rows, D, B = w["rows"], w["dim"], w["batch"]
T = len(rows)
NB = 8
dt = torch.float32 if w["dtype"] == "f32" else torch.bfloat16
g = torch.Generator(device=dev).manual_seed(7)
tabs = [torch.empty((n, D), device=dev).uniform_(-0.05, 0.05, generator=g).to(dt) for n in rows]
ts = pkg.EmbeddingTableSet(tabs)
packs = []
for _ in range(NB):
    cols = []
    for n in rows:
        if a.zipf > 0:
            u = torch.rand(B, device=dev, generator=g).double()
            r = torch.floor(torch.exp(torch.log1p(-u) / (1.0 - a.zipf))).clamp_(max=n) - 1  # rough power law
            cols.append(r.clamp_(0, n - 1).to(torch.int32))
        else:
            cols.append(torch.randint(0, n, (B,), device=dev, generator=g, dtype=torch.int32))
    packs.append(pkg.PackedIndices(torch.stack(cols).reshape(T, B, 1).contiguous()))
hp = pkg.HotPath(ts, B, 1, lr=0.01, index_base=0)
x = torch.randn((B, D), device=dev, generator=g).to(dt)
dout = (torch.randn((B, hp.width), device=dev, generator=g) * 1e-3).to(dt)
split_ix = [pkg.SparseIndexer(T, B, dev) for _ in range(NB)]
plain_ix = [pkg.SparseIndexer(T, B, dev) for _ in range(NB)]
home = hp.indexer


def with_ix(ix, fn):
    def f(k):
        hp.indexer = ix[k]
        fn(k)
        hp.indexer = home
    return f


for k in range(NB):
    hp.indexer = split_ix[k]
    hp.step_fwd(x, packs[k])
    hp.indexer = plain_ix[k]
    hp.build_indexer(packs[k])
hp.indexer = home
torch.cuda.synchronize()

ops = {
    "fwd (lookup+interaction, no ys)": lambda k: hp.lookup_interact_fwd(x, packs[k]),
    "step_fwd (fwd + split indexer)": lambda k: hp.step_fwd(x, packs[k]),
    "indexer_build (1024-thread, own launch)": lambda k: hp.build_indexer(packs[k]),
    "bwd_gather (no indexer)": lambda k: hp.interact_bwd(dout, x=x, idx=packs[k]),
    "bwd_gather + indexer (one launch)": with_ix(plain_ix, lambda k: hp.interact_bwd(dout, x=x, idx=packs[k],
                                                                                     build_indexer=True)),
    "step_bwd BWD_ONLY (once-hit SGD inside)": with_ix(split_ix, lambda k: hp.step_bwd(
        dout, x=x, idx=packs[k], flags=pkg._lib.STEP_BWD_ONLY)),
    "step_bwd APPLY_ONLY (repeated rows)": with_ix(split_ix, lambda k: hp.step_bwd(
        dout, x=x, idx=packs[k], flags=pkg._lib.STEP_APPLY_ONLY)),
    "sgd_update (all rows, prebuilt)": with_ix(plain_ix, lambda k: hp.sgd_update(packs[k], prebuilt=True)),
    "full step (HotPath.step)": lambda k: hp.step(x, packs[k], dout),
}
res = {}
cur = torch.cuda.current_stream()
for name, fn in ops.items():
    s = torch.cuda.Stream()
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        for k in range(NB):
            fn(k)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for k in range(NB):
                fn(k)
    cur.wait_stream(s)
    gr.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(cur)
    for _ in range(a.reps):
        gr.replay()
    e1.record(cur)
    torch.cuda.synchronize()
    res[name] = round(e0.elapsed_time(e1) * 1e3 / (a.reps * NB), 2)
    print(f"{name:45s} {res[name]:8.2f} us", flush=True)
print(json.dumps({"workload": a.workload, "zipf": a.zipf, "us": res}))
