"""Phase timing of indexer_build_kernel (library built with -DDLRM_PHASE=<block>, see
tools/phase_indexer.sh): Kaggle row counts, B=2048, uniform int32 indices."""
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
rows = pkg.KAGGLE_EMBEDDING_SIZES
B = int(os.environ.get("B", "2048"))
tabs = [torch.zeros((n, 4), device=dev) for n in rows]
ts = pkg.EmbeddingTableSet(tabs)
g = torch.Generator(device=dev).manual_seed(1)
idx = torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in rows]).to(torch.int32)
p = pkg.PackedIndices(idx.reshape(len(rows), B, 1))
ix = pkg.SparseIndexer(len(rows), B, dev)
for _ in range(5):
    ix.build(ts, p, index_base=0)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 576)()
lib.dlrm_debug_phase.restype = ctypes.c_int
lib.dlrm_debug_phase(buf)
ph = np.array(buf[:64], dtype=np.int64)
st, en = np.array(buf[64:320], dtype=np.int64), np.array(buf[320:576], dtype=np.int64)
t0 = ph[0]
print("phase (us since block start):", {k: round((ph[k] - t0) / 100, 2) for k in range(64) if ph[k] >= t0 and ph[k]})
T = len(rows)
s0 = st[:T].min()
print("block start offsets us:", np.round((st[:T] - s0) / 100, 2).tolist())
print("block durations us:", np.round((en[:T] - st[:T]) / 100, 2).tolist())
print("kernel span us:", (en[:T].max() - s0) / 100)
