"""Hash indexer build time (dlrm_indexer_build, N = 8192 positions per table: the configs[2]
batch) for different table-size mixes: which tables make the build slow?
usage (GPU box): python tools/hix_probe.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlrm_pkg  # noqa: E402

pkg = dlrm_pkg.load()
dev = torch.device("cuda:0")
B = int(os.environ.get("HIX_B", "8192"))
mixes = {
    "kaggle": list(pkg.KAGGLE_EMBEDDING_SIZES),
    "26x3": [3] * 26,
    "26x100": [100] * 26,
    "26x10k": [10_000] * 26,
    "26x10M": [10_000_000] * 26,
    "kaggle-small13": sorted(pkg.KAGGLE_EMBEDDING_SIZES)[:13],
    "kaggle-large13": sorted(pkg.KAGGLE_EMBEDDING_SIZES)[13:],
}
g = torch.Generator(device=dev).manual_seed(1)
for name, rows in mixes.items():
    T = len(rows)
    tabs = pkg.EmbeddingTableSet([torch.zeros((n, 4), device=dev) for n in rows])
    idx = torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in rows]).to(torch.int32)
    idx = idx.reshape(T, B, 1)
    ix = pkg.SparseIndexer(T, B, dev)
    for _ in range(5):
        ix.build(tabs, idx, index_base=0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    a.record()
    for _ in range(reps):
        ix.build(tabs, idx, index_base=0)
    b.record()
    torch.cuda.synchronize()
    print(f"{name:16s} T={T:2d} B={B}: {a.elapsed_time(b) * 1e3 / reps:7.2f} us per build", flush=True)
    del tabs, ix, idx
    torch.cuda.empty_cache()
