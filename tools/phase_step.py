"""Per-item timeline of the metric step's apply launch (sgd_apply_kernel MODE 2: the next batch's
split-indexer build in its first workgroups, then hot slices, chunk items).  Needs the phase build
of the library (tools/build_variant.sh DIR -DDLRM_PHASE=<build block>; DLRM_HIP_LIB=DIR/...).
Prints, per item kind, the start / end spread in us from the launch's first item, and the phase
marks of one build workgroup (indexer.hpp PHASE(k))."""
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
D = int(os.environ.get("D", "128"))
B = int(os.environ.get("B", "2048"))
# WL=tb: Terabyte-like Zipf(1.05) rows (row counts capped at 2^24 to keep the tables small; the key
# widths stay > 8 bits, so the build takes the same paths)
WL = os.environ.get("WL", "kaggle")
rows = pkg.KAGGLE_EMBEDDING_SIZES if WL == "kaggle" else [min(n, 1 << 24) for n in pkg.TERABYTE_EMBEDDING_SIZES]
tabs = [torch.zeros((n, D), device=dev) for n in rows]
ts = pkg.EmbeddingTableSet(tabs)
g = torch.Generator(device=dev).manual_seed(1)
if WL == "kaggle":
    packs = [pkg.PackedIndices(torch.stack([torch.randint(0, n, (B,), device=dev, generator=g) for n in rows])
                               .to(torch.int32)) for _ in range(4)]
else:
    rng = np.random.default_rng(1)
    perms = [pkg.zipf_perm(rng, n) for n in rows]
    packs = [pkg.PackedIndices(torch.from_numpy(np.stack([pkg.zipf_rows(rng, n, B, 1.05, p) for n, p in zip(rows, perms)]))
                               .to(dev)) for _ in range(4)]
hp = pkg.HotPath(ts, B, 1, lr=0.01, index_base=0, pipeline="apply")
x = torch.randn((B, D), device=dev)
dout = torch.randn((B, hp.width), device=dev) * 1e-3
hp.prime(packs[0], x=x, dout=dout, prev=packs[3])
for k in range(3):
    hp.step_prep(x, packs[k % 4], dout, packs[(k + 1) % 4])
torch.cuda.synchronize()
lib.dlrm_debug_items.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * (3 * 65536))()
lib.dlrm_debug_items(None, 1)
hp.step_prep(x, packs[3], dout, packs[0])
torch.cuda.synchronize()
lib.dlrm_debug_items(buf, 0)
a = np.array(buf, dtype=np.int64).reshape(3, 65536)
used = a[0] > 0
st, en, kind, item = a[0][used], a[1][used], a[2][used] & 255, a[2][used] >> 8
slot = np.nonzero(used)[0]
blk = slot // 16
t0 = st.min()
names = {1: "chunk", 2: "hot slice", 3: "singles", 4: "next-batch build"}
print(f"launch: {len(np.unique(blk))} workgroups logged, last item ends at {(en.max() - t0) / 100:.2f} us")
kslot = slot % 16
for k in sorted(set(kind.tolist())):
  for ks in ([0, 1] if k == 4 and (kslot[kind == 4] == 1).any() else [None]):
    m = (kind == k) if ks is None else ((kind == k) & (kslot == ks))
    d = (en[m] - st[m]) / 100
    print(f"{names.get(k, k) + ('' if ks is None else f' #{ks}'):17s} items {m.sum():5d}  start {(st[m].min() - t0) / 100:6.2f}..{(st[m].max() - t0) / 100:6.2f}"
          f"  end p50 {np.percentile((en[m] - t0) / 100, 50):6.2f} max {(en[m].max() - t0) / 100:6.2f}"
          f"  dur p50/p90/max {np.percentile(d, 50):.2f}/{np.percentile(d, 90):.2f}/{d.max():.2f} us")
# items per workgroup (apply blocks only)
ab = blk[kind != 4]
cnt = np.bincount(ab) if ab.size else np.zeros(1)
print("apply items per workgroup: max", int(cnt.max()), " mean", round(float(cnt[cnt > 0].mean()), 2))
# the last-ending 10 items
o = np.argsort(en)[-10:]
print("last 10 items (kind, item, start, end us):",
      [(names.get(int(kind[i]), int(kind[i])), int(item[i]), round((st[i] - t0) / 100, 2), round((en[i] - t0) / 100, 2))
       for i in o])
ph = (ctypes.c_ulonglong * 576)()
lib.dlrm_debug_phase(ph)
p = np.array(ph[:64], dtype=np.int64)
nz = p[p > 0]
if nz.size:
    print(f"build workgroup {os.environ.get('PHASE_BLOCK', '?')} phases (us from its first mark):",
          {k: round((p[k] - nz.min()) / 100, 2) for k in range(64) if p[k] > 0})

# every build workgroup's phase marks (g_phase2[block][k]): per mark, p50 / max us from the block's mark 0
ph2 = (ctypes.c_ulonglong * (256 * 32))()
lib.dlrm_debug_phase2(ph2)
m = np.array(ph2, dtype=np.int64).reshape(256, 32)
nb = 104 if D > 32 else 208
m = m[:nb]
ok = m[:, 0] > 0
if ok.any():
    rel = (m[ok] - m[ok][:, :1]) / 100
    print("build phase marks over", int(ok.sum()), "workgroups (us from mark 0: p50 / max):")
    for k in range(1, 32):
        col = m[ok][:, k]
        if (col > 0).any():
            r = rel[:, k][col > 0]
            print(f"  mark {k:2d}: {np.percentile(r, 50):6.2f} / {r.max():6.2f}")
    end = (en[kind == 4].max() - t0) / 100
    print("  (build item durations above include the marks' own barriers)")

# wave build marks (g_wph[block][wave][k]): 0 start, 7 index loads issued, 8 landed, 9 validated,
# 1 counted (scans), 2 compacted, 3 first counting pass, 4 sorted, 5 segments written, 6 chunks /
# slices written
if hasattr(lib, "dlrm_debug_wph"):
    wb = (ctypes.c_ulonglong * (256 * 4 * 16))()
    lib.dlrm_debug_wph(wb)
    a3 = np.array(wb, dtype=np.int64).reshape(256, 4, 16)[:int((kind == 4).sum())].reshape(-1, 16)
    ok = a3[:, 0] > 0
    if ok.any():
        rel = (a3[ok] - a3[ok][:, :1]) / 100
        print("wave build marks over", int(ok.sum()), "waves (us from the wave's mark 0: p50 / max):")
        for k in range(1, 16):
            col = a3[ok][:, k]
            if (col > 0).any():
                r = rel[:, k][col > 0]
                print(f"  mark {k:2d}: {np.percentile(r, 50):6.2f} / {r.max():6.2f}")
        # the slowest waves: (group, wave, table rows, per-mark us)
        gw = np.argwhere(np.array(wb, dtype=np.int64).reshape(256, 4, 16)[:int((kind == 4).sum()), :, 0] > 0)
        ends = [(rel[i, 6] if a3[ok][i, 6] > 0 else 0.0, i) for i in range(rel.shape[0])]
        for e, i in sorted(ends)[-8:]:
            g_, w_ = gw[i]
            t_ = int(g_) // 4
            print(f"  slow wave g={int(g_)} w={int(w_)} table {t_} ({rows[t_]} rows):",
                  {k: round(float(rel[i, k]), 2) for k in range(1, 16) if a3[ok][i, k] > 0})
