"""Does a side-stream branch of a captured hipGraph run concurrently with the main branch?
Times, per iteration over 8 index batches: the fused forward alone; the standalone indexer
alone; both in sequence on one stream; both as parallel graph branches (fork/join per step)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlrm_pkg  # noqa: E402

pkg = dlrm_pkg.load()
dev = torch.device("cuda:0")
rows = pkg.KAGGLE_EMBEDDING_SIZES
B, D, T, NB = 2048, 128, 26, 8
g = torch.Generator(device=dev).manual_seed(3)
ts = pkg.EmbeddingTableSet([torch.empty((n, D), device=dev).uniform_(-0.05, 0.05, generator=g) for n in rows])
packs = [pkg.PackedIndices(torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in rows])
                           .to(torch.int32).reshape(T, B, 1)) for _ in range(NB)]
hp = pkg.HotPath(ts, B, 1, lr=0.01, index_base=0)
x = torch.randn((B, D), device=dev, generator=g)
ixs = [pkg.SparseIndexer(T, B, dev) for _ in range(NB)]


def build(k):
    home = hp.indexer
    hp.indexer = ixs[k]
    hp.build_indexer(packs[k])
    hp.indexer = home


def fwd(k):
    hp.lookup_interact_fwd(x, packs[k])


def time_graph(body, reps=20):
    main = torch.cuda.Stream()
    side = torch.cuda.Stream()
    main.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(main):
        body(main, side)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=main):
            body(main, side)
    torch.cuda.current_stream().wait_stream(main)
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream()
    e0.record(cur)
    for _ in range(reps):
        gr.replay()
    e1.record(cur)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * NB)


def only_fwd(main, side):
    for k in range(NB):
        fwd(k)


def only_ix(main, side):
    for k in range(NB):
        build(k)


def seq(main, side):
    for k in range(NB):
        build((k + 1) % NB)
        fwd(k)


def par(main, side):
    for k in range(NB):
        side.wait_stream(main)
        with torch.cuda.stream(side):
            build((k + 1) % NB)
        fwd(k)
        main.wait_stream(side)


def par_loose(main, side):  # the side branch joins one step later
    for k in range(NB):
        side.wait_stream(main)
        with torch.cuda.stream(side):
            build((k + 1) % NB)
        fwd(k)
        fwd(k)  # stand-in for the rest of the step
        main.wait_stream(side)


want = sys.argv[1].split(",") if len(sys.argv) > 1 else None  # e.g. "parallel" (rocprofv3 timelines)
for name, body in [("fwd", only_fwd), ("indexer", only_ix), ("seq", seq), ("parallel", par),
                   ("fwd x2 + side indexer", par_loose)]:
    if want and name.split()[0] not in want:
        continue
    print(f"{name:28s} {time_graph(body):8.2f} us/iter", flush=True)
    torch.cuda.synchronize()
    import time as _t
    _t.sleep(0.05)  # (a gap in a kernel trace between the configurations)
