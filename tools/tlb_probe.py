"""Random-row gather time vs table size (one table, D = 128 fp32, 65536 uniform rows per
lookup launch through dlrm_maplookup): separates the HBM/cache cost of a row from address
translation reach (the Kaggle 10M-row table is 5 GB)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlrm_pkg  # noqa: E402

pkg = dlrm_pkg.load()
dev = torch.device("cuda:0")
D, B = 128, 65536
g = torch.Generator(device=dev).manual_seed(3)
for rows in (1 << 16, 1 << 18, 1 << 20, 1 << 22, 10_000_000, 1 << 25):
    tab = torch.empty((rows, D), device=dev).uniform_(-1, 1, generator=g)
    ts = pkg.EmbeddingTableSet([tab])
    idxs = [pkg.PackedIndices(torch.randint(0, rows, (1, B, 1), device=dev, generator=g, dtype=torch.int64)
                              .to(torch.int32)) for _ in range(16)]
    out = torch.empty((B, D), device=dev)
    for k in range(16):
        pkg.maplookup(pkg.PreallocationStrategy(0), ts, idxs[k], out=out, index_base=0, check_bounds=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(4):
        for k in range(16):
            pkg.maplookup(pkg.PreallocationStrategy(0), ts, idxs[k], out=out, index_base=0, check_bounds=False)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 64
    print(f"rows {rows:>9} ({rows * D * 4 / 2**30:6.2f} GiB): {us:6.2f} us per 65536-row gather = "
          f"{2 * B * D * 4 / us / 1e3:6.0f} GB/s (read + write)", flush=True)
    del tab, ts, idxs, out
    torch.cuda.empty_cache()
