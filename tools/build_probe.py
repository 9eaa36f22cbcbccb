"""Where the step's split build costs time (metric config: 26 Kaggle tables x 128 fp32, B = 2048).
HIP-event timings over 64 index batches, each form replayed as one hipGraph:
  build      dlrm_indexer_prepare alone (the wave build + item lists, its own launch)
  fwd        the gather-only forward (dlrm_step_fwd of a prepared indexer)
  fwd||build the build on a side stream beside the forward (fork / join in the graph)
  apply      the apply launch alone (dlrm_step_bwd APPLY_ONLY)
  apply+prep the apply launch with the next batch's build in it (dlrm_step_bwd_prepare)"""
import os
import sys
import json

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlrm_pkg  # noqa: E402

pkg = dlrm_pkg.load()
from dlrm_jl_amd.runtime import ptr  # noqa: E402

dev = torch.device("cuda:0")
D, B, NB = int(os.environ.get("D", "128")), 2048, 64
rows = pkg.KAGGLE_EMBEDDING_SIZES
T = len(rows)
g = torch.Generator(device=dev).manual_seed(3)
tabs = [torch.empty((n, D), device=dev).uniform_(-0.01, 0.01, generator=g) for n in rows]
ts = pkg.EmbeddingTableSet(tabs)
packs = [pkg.PackedIndices(torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in rows])
                           .to(torch.int32)) for _ in range(NB)]
hp = pkg.HotPath(ts, B, 1, lr=0.01, index_base=0, pipeline="apply")
x = torch.randn((B, D), device=dev, generator=g)
dout = torch.randn((B, hp.width), device=dev, generator=g) * 1e-3
ixs = [pkg.SparseIndexer(T, B, dev) for _ in range(NB)]
lib, ctx = ts.ctx.lib, ts.ctx


def prepare(k):
    p = packs[k]
    ctx.check(lib.dlrm_indexer_prepare(ctx.bind(), ixs[k].handle, ts.handle, ptr(p.data), p.itype, p.stride, 0, B))


def fwd(k):
    hp.indexer = ixs[k]
    hp.step_fwd(x, packs[k])


def timed(name, fn, reps=4):
    cur = torch.cuda.current_stream()
    s = torch.cuda.Stream()
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            for k in range(NB):
                fn(k)
    cur.wait_stream(s)
    gr.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * NB)
    out[name] = round(us, 2)


out = {}
for k in range(NB):
    prepare(k)
torch.cuda.synchronize()
timed("build", prepare)
side = torch.cuda.Stream()


def fwd_only(k):
    prepare_state(k)
    fwd(k)


def prepare_state(k):  # (the prepared flag is consumed by the forward: re-arm it on the host only)
    pass


# the forward consumes the prepared state: time prepare+fwd in stream order, then subtract
timed("build+fwd serial", lambda k: (prepare(k), fwd(k)))


def par(k):
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        prepare(k)
    ev = torch.cuda.Event()
    ev.record(side)
    main.wait_event(ev)  # (the forward needs the prepared flag on the host only; the join keeps the graph whole)
    fwd(k)


def par2(k):
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        prepare(k)
    fwd(k)
    ev = torch.cuda.Event()
    ev.record(side)
    main.wait_event(ev)


timed("fwd || build (joined after)", par2)
for k in range(NB):
    hp.indexer = ixs[k]
    hp.step_fwd(x, packs[k])  # builds in the forward launch (not prepared)
torch.cuda.synchronize()
timed("fwd with in-launch build", lambda k: (setattr(hp, "indexer", ixs[k]), hp.step_fwd(x, packs[k])))
print(json.dumps(out))
