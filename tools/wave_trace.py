"""Per-sample wave timelines of the forward and backward bodies (library built with
-DDLRM_WTRACE, tools/wave_trace.sh): BASELINE metric shape, uniform indices.  For each launch
prints, relative to the first wave's start (us): the spread of wave starts, and the p50/p90/max
of each phase.  fwd slots: 0 start, 1 loads+MFMA done, 2 output written.  bwd slots: 0 start,
1 S built, 2 super-block 0 MFMA done, 3 super-block 1 MFMA done, 4 stores issued."""
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
B, D = 2048, int(os.environ.get("DLRM_WT_D", "128"))  # DLRM_WT_D=16: configs[1]
T = len(rows)
g = torch.Generator(device=dev).manual_seed(1)
ts = pkg.EmbeddingTableSet([torch.empty((n, D), device=dev).uniform_(-0.05, 0.05, generator=g) for n in rows])
packs = [pkg.PackedIndices(torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in rows])
                           .to(torch.int32).reshape(T, B, 1)) for _ in range(4)]
hp = pkg.HotPath(ts, B, 1, lr=0.01, index_base=0)
x = torch.randn((B, D), device=dev, generator=g)
dout = torch.randn((B, hp.width), device=dev, generator=g) * 1e-3
buf = (ctypes.c_ulonglong * (2 * 6 * 8192))()
lib.dlrm_debug_wtrace.restype = ctypes.c_int


def show(kind, slots, names):
    lib.dlrm_debug_wtrace(buf)
    a = np.array(buf, dtype=np.int64).reshape(2, 6, 8192)[kind][:, :B]
    t0 = a[0].min()
    rel = (a - t0) / 100.0  # us
    print(f"  start spread: p50 {np.percentile(rel[0], 50):.2f} p90 {np.percentile(rel[0], 90):.2f} max {rel[0].max():.2f}")
    # slots a launch never writes (e.g. super-block 1 when D <= 64) are skipped
    used = [s for s in range(slots) if a[s].max() > 0]
    for prev, s in zip(used, used[1:]):
        d = rel[s] - rel[prev]
        print(f"  {names[s]:28s} dur p50 {np.percentile(d, 50):.2f} p90 {np.percentile(d, 90):.2f} max {d.max():.2f}"
              f" | done at p50 {np.percentile(rel[s], 50):.2f} max {rel[s].max():.2f}")


for mode in sys.argv[1:] or ["ops"]:
    for k in range(6):  # warm
        hp.step(x, packs[k % 4], dout)
    torch.cuda.synchronize()
    if mode == "ops":
        print("fwd (lookup_interact_fwd, no ys):")
        hp.lookup_interact_fwd(x, packs[1]); torch.cuda.synchronize()
        show(0, 3, ["start", "loads+mfma", "out written"])
        print("bwd_gather (no indexer):")
        hp.interact_bwd(dout, x=x, idx=packs[1]); torch.cuda.synchronize()
        show(1, 5, ["start", "S built", "sb0 mfma", "sb1 mfma", "stores"])
        if os.environ.get("DLRM_BWD_SPLIT", "1") != "0":
            print("  (split backward: slots = start, S barrier, MFMA done, stores issued, stores drained)")
    else:
        print("step_fwd:")
        hp.step_fwd(x, packs[2]); torch.cuda.synchronize()
        show(0, 3, ["start", "loads+mfma", "out written"])
        print("step_bwd (BWD_ONLY):")
        hp.step_bwd(dout, x=x, idx=packs[2], flags=pkg._lib.STEP_BWD_ONLY); torch.cuda.synchronize()
        show(1, 5, ["start", "S built", "sb0 mfma", "sb1 mfma", "stores"])
        if os.environ.get("DLRM_BWD_SPLIT", "1") != "0":
            print("  (split backward: slots = start, S barrier, MFMA done, stores issued, stores drained)")
