"""Wave-build phase marks (library built with -DDLRM_PHASE) of the standalone step build
(dlrm_indexer_prepare, one launch, nothing else running), metric config."""
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
D, B = 128, 2048
rows = pkg.KAGGLE_EMBEDDING_SIZES
T = len(rows)
g = torch.Generator(device=dev).manual_seed(3)
ts = pkg.EmbeddingTableSet([torch.zeros((n, 4), device=dev) for n in rows])
packs = [pkg.PackedIndices(torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in rows])
                           .to(torch.int32)) for _ in range(4)]
ix = pkg.SparseIndexer(T, B, dev)
ctx = ts.ctx
for k in range(8):
    p = packs[k % 4]
    ctx.check(lib.dlrm_indexer_prepare(ctx.bind(), ix.handle, ts.handle, ptr(p.data), p.itype, p.stride, 0, B))
torch.cuda.synchronize()
wb = (ctypes.c_ulonglong * (256 * 4 * 16))()
lib.dlrm_debug_wph(wb)
a3 = np.array(wb, dtype=np.int64).reshape(256, 4, 16)[:104].reshape(-1, 16)
ok = a3[:, 0] > 0
rel = (a3[ok] - a3[ok][:, :1]) / 100
print("standalone wave build marks over", int(ok.sum()), "waves (us from mark 0: p50 / max)")
for k in [7, 8, 9, 1, 2, 3, 4, 5, 6]:
    col = a3[ok][:, k]
    if (col > 0).any():
        r = rel[:, k][col > 0]
        print(f"  mark {k:2d}: {np.percentile(r, 50):6.2f} / {r.max():6.2f}")
st = a3[ok][:, 0]
print("wave start spread us:", round((st.max() - st.min()) / 100, 2))
