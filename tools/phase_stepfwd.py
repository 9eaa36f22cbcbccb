"""Phase timing of the split indexer inside dlrm_step_fwd's launch (library built with
-DDLRM_PHASE=<table>, tools/phase_indexer.sh; PHASE_SCRIPT=phase_stepfwd.py): BASELINE metric
shape, uniform int32 indices.  Phases: 1 indices loaded, 2 digit counts, 3 scan, 4 max bucket,
5 scattered, 10 rows ordered, 20 segments, 22 chunks written (us since the block's start)."""
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
B, D = 2048, 128
g = torch.Generator(device=dev).manual_seed(1)
ts = pkg.EmbeddingTableSet([torch.empty((n, D), device=dev).uniform_(-0.05, 0.05, generator=g) for n in rows])
idx = torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in rows]).to(torch.int32)
p = pkg.PackedIndices(idx.reshape(len(rows), B, 1))
hp = pkg.HotPath(ts, B, 1, lr=0.01, index_base=0)
x = torch.randn((B, D), device=dev, generator=g)
for _ in range(5):
    hp.step_fwd(x, p)
torch.cuda.synchronize()
lib.dlrm_debug_phase_fwd_reset()
hp.step_fwd(x, p)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 64)()
lib.dlrm_debug_phase_fwd.restype = ctypes.c_int
lib.dlrm_debug_phase_fwd(buf)
ph = np.array(buf[:64], dtype=np.int64)
t0 = min(ph[60], ph[62])  # the launch's first block
blk = int(os.environ.get("BLK", "0"))
print(f"block {blk} (table {blk >> hp.indexer_vshift if hasattr(hp, 'indexer_vshift') else blk // 4}):",
      {k: round((ph[k] - t0) / 100, 2) for k in range(60) if ph[k]},
      f"| gather blocks {round((ph[60] - t0) / 100, 2)}..{round((ph[61] - t0) / 100, 2)} us,"
      f" indexer blocks {round((ph[62] - t0) / 100, 2)}..{round((ph[63] - t0) / 100, 2)} us")
