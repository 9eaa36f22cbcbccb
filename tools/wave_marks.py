"""Wave-build phase marks (library built with -DDLRM_PHASE: tools/build_variant.sh DIR -DDLRM_PHASE=1)
of the standalone wave build (dlrm_indexer_prepare, one launch, nothing else running) at N positions
per table, plus its HIP-event time.  env: DLRM_HIP_LIB (the marks build), N (2048), ROWS = kaggle |
shard (tables 0-3 of Kaggle, as rank 0 of 8) | big (26 tables of 10M rows)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dlrm_pkg  # noqa: E402

pkg = dlrm_pkg.load()
lib = pkg._lib.load(os.environ["DLRM_HIP_LIB"])
from dlrm_jl_amd.runtime import ptr  # noqa: E402

dev = torch.device("cuda:0")
N = int(os.environ.get("N", "2048"))
kind = os.environ.get("ROWS", "kaggle")
rows = {"kaggle": pkg.KAGGLE_EMBEDDING_SIZES, "shard": pkg.KAGGLE_EMBEDDING_SIZES[:4],
        "big": [10_000_000] * 26}[kind]
T = len(rows)
g = torch.Generator(device=dev).manual_seed(3)
ts = pkg.EmbeddingTableSet([torch.zeros((n, 4), device=dev) for n in rows])
packs = [pkg.PackedIndices(torch.stack([torch.randint(0, n, (N,), device=dev, generator=g) for n in rows])
                           .to(torch.int32)) for _ in range(4)]
ix = pkg.SparseIndexer(T, N, dev)
ctx = ts.ctx


def prep(k):
    p = packs[k % 4]
    ctx.check(lib.dlrm_indexer_prepare(ctx.bind(), ix.handle, ts.handle, ptr(p.data), p.itype, p.stride, 0, N))


for k in range(8):
    prep(k)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for k in range(20):
    prep(k)
e1.record()
torch.cuda.synchronize()
print(f"ROWS={kind} N={N}: {e0.elapsed_time(e1) * 1e3 / 20:.2f} us per build (events, back to back)")
prep(0)
torch.cuda.synchronize()
wb = (ctypes.c_ulonglong * (256 * 4 * 16))()
lib.dlrm_debug_wph(wb)
vs = 4 if N <= 2048 else (5 if N <= 4096 else (6 if N <= 8192 else 7))
ngr = min(256, (T << vs) // 4)
a3 = np.array(wb, dtype=np.int64).reshape(256, 4, 16)[:ngr].reshape(-1, 16)
ok = a3[:, 0] > 0
rel = (a3[ok] - a3[ok][:, :1]) / 100
print("marks over", int(ok.sum()), "waves (us from the wave's mark 0: p50 / max)")
for k in [7, 1, 2, 3, 4, 5, 9, 8, 6]:
    col = a3[ok][:, k]
    if (col > 0).any():
        r = rel[:, k][col > 0]
        print(f"  mark {k:2d}: {np.percentile(r, 50):6.2f} / {r.max():6.2f}")
st = a3[ok][:, 0]
print("wave start spread us:", round((st.max() - st.min()) / 100, 2))
