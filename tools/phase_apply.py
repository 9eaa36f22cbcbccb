"""Per-block timing of sgd_apply_kernel (library built with -DDLRM_PHASE, tools/phase_indexer.sh
APPLY=1): Kaggle rows, D=128 fp32, B=2048, uniform indices; prints the span of chunk and hot blocks."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlrm_pkg  # noqa: E402

pkg = dlrm_pkg.load()
lib = pkg._lib.load(os.environ["DLRM_HIP_LIB"])
dev = torch.device("cuda:0")
world = int(sys.argv[1]) if len(sys.argv) > 1 else 1  # > 1: rank 0's update of a WORLD-rank sharded step
rows = pkg.KAGGLE_EMBEDDING_SIZES
B, D = 2048, 128
if world == 1:
    tabs = [torch.zeros((n, D), device=dev) for n in rows]
    ts = pkg.EmbeddingTableSet(tabs)
    g = torch.Generator(device=dev).manual_seed(1)
    idx = torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in rows]).to(torch.int32)
    p = pkg.PackedIndices(idx.reshape(len(rows), B, 1))
    hp = pkg.HotPath(ts, B, 1, lr=0.01, index_base=0)
    x = torch.randn((B, D), device=dev)
    dout = torch.randn((B, hp.width), device=dev)
    run = lambda: hp.step(x, p, dout)  # noqa: E731
else:
    from dlrm_jl_amd import sharded

    class NoExchange(sharded.ShardedHotPath):
        def exchange_fwd(self):
            pass

        def exchange_bwd(self):
            pass

    sharded.ShardedHotPath = NoExchange
    eng, step, _ = sharded.make_bench_engine(pkg, dict(pkg.WORKLOADS["kaggle-d128-b2048"]), B, dev, 0, world, 0.01)
    run = lambda: step(0)  # noqa: E731
for _ in range(3):
    run()
torch.cuda.synchronize()
lib.dlrm_debug_apply_reset()
run()
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (3 * 32768))()
lib.dlrm_debug_apply(buf)
a = np.array(buf, dtype=np.int64).reshape(3, 32768)
used = a[0] > 0
st, en, kind = a[0][used], a[1][used], a[2][used]
t0 = st.min()
for k, name in [(1, "chunk"), (2, "hot"), (3, "singles")]:
    if not (kind == k).any():
        continue
    m = kind == k
    busy = m & (en > 0)
    print(f"{name}: blocks {m.sum()}  start {(st[m].min() - t0) / 100:.2f}..{(st[m].max() - t0) / 100:.2f} us  "
          f"end max {(en[busy].max() - t0) / 100:.2f} us  dur p50/p99/max "
          f"{np.percentile((en[busy] - st[busy]) / 100, 50):.2f}/{np.percentile((en[busy] - st[busy]) / 100, 99):.2f}/"
          f"{((en[busy] - st[busy]) / 100).max():.2f} us")
# the hot blocks that did work: durations sorted
hb = (kind == 2) & (en - st > 100)
print("longest hot blocks us:", np.round(np.sort((en[hb] - st[hb]) / 100)[-12:], 2).tolist())
