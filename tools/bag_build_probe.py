"""Standalone timing of dlrm_indexer_build for pooled-bag shapes (configs[4]: 64 tables x 20480
positions): HIP events around 20 back-to-back builds, per index distribution.  The build form is
the library's default for the shape (the bag build above 8192 positions per table since round 6;
at or below 8192 the in-LDS builds); DLRM_BAG_WAVE=0 in the environment selects the hash build
instead, DLRM_BAG_VS its parts per table, for A/B.
usage: python tools/bag_build_probe.py [T] [N] [ROWS] [DIST: uniform | zipf1.05 | zipf1.2 | all]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlrm_pkg  # noqa: E402

pkg = dlrm_pkg.load()
dev = torch.device("cuda:0")
T = int(sys.argv[1]) if len(sys.argv) > 1 else 64
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20480
R = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
rows = [R] * T if R > 0 else pkg.KAGGLE_EMBEDDING_SIZES[:T]  # (ROWS 0: the Kaggle tables)
ts = pkg.EmbeddingTableSet([torch.zeros((n, 4), device=dev) for n in rows])
ix = pkg.SparseIndexer(T, N, dev)
rng = np.random.default_rng(5)
form = "hash" if os.environ.get("DLRM_BAG_WAVE") == "0" else "bag"
only = sys.argv[4] if len(sys.argv) > 4 else "all"
for dist in [d for d in ("uniform", "zipf1.05", "zipf1.2") if only in ("all", d)]:
    packs = []
    for _ in range(4):  # (one-hot [T][N] unless N is a multiple of 10: [T][N/10][10] bags)
        if dist == "uniform":
            a = np.stack([rng.integers(0, n, size=N) for n in rows])
        else:
            s = float(dist[4:])
            a = np.stack([pkg.zipf_rows(rng, n, N, s) for n in rows])
        packs.append(pkg.PackedIndices(torch.from_numpy(a.astype(np.int32)).to(dev).reshape(T, N // 10, 10)
                                       if N % 10 == 0 else torch.from_numpy(a.astype(np.int32)).to(dev)))
    for k in range(6):
        ix.build(ts, packs[k % 4], index_base=0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(20):
        ix.build(ts, packs[k % 4], index_base=0)
    e1.record()
    torch.cuda.synchronize()
    ts.ctx.check_bounds()
    u = np.mean([len(np.unique(packs[0].data[t].cpu().numpy())) for t in range(min(T, 4))])
    print(f"{form} T={T} N={N} rows={R} {dist}: {e0.elapsed_time(e1) * 1e3 / 20:.1f} us per build "
          f"(~{u:.0f} unique rows per table)", flush=True)
