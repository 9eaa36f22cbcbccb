"""DACLoader throughput: synthetic 160-B DAC records in host memory -> pinned
staging -> HBM -> dlrm_dac_decode, alone and overlapped with the hot-path training step
(Kaggle 26 x 128 fp32, B = 2048) consuming every batch.

    python tools/bench_dac_loader.py [--batches 200]

Prints one JSON line: loader-only records/s, step-only and loader+step samples/s.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dlrm_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=200)
    ap.add_argument("--direct", type=int, default=0, help="1: page-locked dataset, one DMA per batch")
    a = ap.parse_args()
    pkg = dlrm_pkg.load()
    dev = torch.device("cuda:0")
    w = pkg.WORKLOADS["kaggle-d128-b2048"]
    rows, D, B = w["rows"], w["dim"], w["batch"]
    T = len(rows)
    rng = np.random.default_rng(1)
    data = np.zeros(B * a.batches, dtype=pkg.DAC_DTYPE)
    data["label"] = rng.integers(0, 2, len(data))
    data["continuous"] = rng.random((len(data), 13), dtype=np.float32)
    data["categorical"] = np.stack([rng.integers(1, n + 1, len(data)) for n in rows], axis=1).astype(np.uint32)

    loader = pkg.DACLoader(data, B, dev, direct=a.direct == 1)
    for _ in loader:  # warm-up
        pass
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in loader:
        pass
    torch.cuda.synchronize()
    t_load = time.perf_counter() - t0

    gen = torch.Generator(device=dev).manual_seed(51234)
    tables = [torch.empty((n, D), device=dev).uniform_(-n ** -0.5, n ** -0.5, generator=gen) for n in rows]
    hp = pkg.HotPath(pkg.EmbeddingTableSet(tables), B, 1, lr=0.01, index_base=1)
    x = torch.randn((B, D), device=dev, generator=gen)
    dout = torch.randn((B, hp.width), device=dev, generator=gen) * 1e-3
    first = next(iter(loader))
    fixed = pkg.PackedIndices(first.sparse.clone().reshape(T, B, 1))
    for _ in range(5):
        hp.step(x, fixed, dout)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.batches):
        hp.step(x, fixed, dout)
    torch.cuda.synchronize()
    t_step = time.perf_counter() - t0

    t0 = time.perf_counter()
    for b in loader:
        hp.step(x, pkg.PackedIndices(b.sparse.reshape(T, B, 1)), dout)
    torch.cuda.synchronize()
    t_both = time.perf_counter() - t0
    hp.check_bounds()

    # the step captured once per loader slot (its index buffer is fixed), replayed per batch: the
    # loader's slot hand-off orders each replay after that batch's decode
    slots = loader._out
    graphs = []
    for sl in slots:
        pk = pkg.PackedIndices(sl.sparse.reshape(T, B, 1))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                hp.step(x, pk, dout)
        torch.cuda.current_stream().wait_stream(s)
        graphs.append(gr)
    for gr in graphs:  # warm replays
        gr.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(len(loader)):
        graphs[0].replay()
    torch.cuda.synchronize()
    t_step_g = time.perf_counter() - t0
    t0 = time.perf_counter()
    for b in loader:
        graphs[0 if b is slots[0] else 1].replay()
    torch.cuda.synchronize()
    t_both_g = time.perf_counter() - t0
    hp.check_bounds()
    n = len(loader) * B
    print(json.dumps({
        "metric": "DACLoader records/s (host records -> pinned -> HBM -> decode), 1 MI355X",
        "loader_only_records_per_s": round(n / t_load, 1),
        "step_only_samples_per_s_eager": round(n / t_step, 1),
        "loader_plus_step_samples_per_s_eager": round(n / t_both, 1),
        "step_only_samples_per_s_graph": round(n / t_step_g, 1),
        "loader_plus_step_samples_per_s_graph": round(n / t_both_g, 1),
        "batch": B, "batches": len(loader), "record_bytes": 160, "direct_dma": loader.direct,
        "loader_GBps": round(n * 160 / t_load / 1e9, 2),
        "native_prefetch": loader.native,
        "note": "eager: the step launched per batch; graph: the step captured once per loader slot and replayed",
    }))


if __name__ == "__main__":
    main()
