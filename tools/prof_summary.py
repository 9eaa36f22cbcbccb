"""Summarises rocprofv3 CSV output for the DLRM hot-path kernels.

    python tools/prof_summary.py --kt DIR_WITH_kernel_stats.csv [--fetch DIR] [--write DIR]
                                 [--workload NAME] [--out profiles/NAME]

* kernel stats (--kernel-trace --stats): per-kernel calls / average duration.
* PMC passes (--pmc FETCH_SIZE, --pmc WRITE_SIZE, separate runs): per-dispatch counters in KB.
  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports 1/2 of the bytes of a wide
  coalesced read stream, so HBM read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for
  16-B stores.  hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
* MFMA pass (--pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE, own run): mfma_busy = the MFMA busy
  cycles summed over the chip / (1024 SIMDs x the dispatch's cycles), i.e. the fraction of
  SIMD-cycles the matrix cores were busy (north_star's MFMA utilisation).  rocprofv3 reports
  GRBM_GUI_ACTIVE summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back), so the dispatch's
  cycles are GRBM_GUI_ACTIVE / 8; it reads high on dispatches much shorter than 0.3 ms, so the
  fraction is a lower bound there.
  --refresh FILE.json recomputes mfma_busy of an existing summary and rewrites its .json / .md.
Writes <out>.json (consumed by bench.py for roofline.traffic) and <out>.md.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

STAGES = [  # (regex on the kernel name, stage)
    (r"interact_fwd_kernel<[^,]+, \d+, true|interact_fwd_index_kernel", "lookup_interact_fwd"),
    (r"interact_fwd_kernel<[^,]+, \d+, false|interact_fwd_scalar", "interact_fwd"),
    (r"interact_bwd", "interact_bwd"),  # incl. interact_bwd_index_kernel
    (r"maplookup_", "lookup"),
    (r"indexer_build_kernel|indexer_fast_kernel|hix_|bag_(count|place|sort)_kernel|step_index", "indexer_build"),
    (r"sgd_apply|sgd_chunks", "sgd_update"),
    (r"sgd_hot", "sgd_update"),
    (r"sgd_atomic", "sgd_update"),
]


def stage_of(name):
    for pat, st in STAGES:
        if re.search(pat, name):
            return st
    return None


def short(name):
    m = re.search(r"dlrm::([A-Za-z0-9_]+(<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def one(d, pattern):
    hits = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not hits:
        raise FileNotFoundError(f"{pattern} under {d}")
    return hits[0]


def counters(d, name):
    per = defaultdict(list)
    for r in read_csv(one(d, "*counter_collection.csv")):
        if r["Counter_Name"] != name or "dlrm::" not in r["Kernel_Name"]:
            continue
        per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kt")
    ap.add_argument("--refresh", help="an existing summary .json: recompute mfma_busy, rewrite .json/.md")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--mfma")
    ap.add_argument("--head", default="unknown", help="git HEAD the profiled library was built from")
    ap.add_argument("--workload", default="kaggle-d128-b2048")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.refresh:
        old = json.load(open(a.refresh))
        finish(old["kernels"], old["workload"], old.get("head", "unknown"), a.out or a.refresh[:-len(".json")])
        return
    kernels = {}
    for r in read_csv(one(a.kt, "*kernel_stats.csv")):
        if "dlrm::" not in r["Name"]:
            continue
        kernels[short(r["Name"])] = {"stage": stage_of(r["Name"]), "calls": int(r["Calls"]),
                                     "avg_us": float(r["AverageNs"]) / 1e3, "min_us": float(r["MinNs"]) / 1e3,
                                     "max_us": float(r["MaxNs"]) / 1e3}
    mfma = counters(a.mfma, "SQ_VALU_MFMA_BUSY_CYCLES") if a.mfma else {}
    gui = counters(a.mfma, "GRBM_GUI_ACTIVE") if a.mfma else {}
    fetch = counters(a.fetch, "FETCH_SIZE") if a.fetch else {}
    write = counters(a.write, "WRITE_SIZE") if a.write else {}
    for k, v in kernels.items():
        f = fetch.get(k)
        w = write.get(k)
        if f:
            v["FETCH_SIZE_KB_avg"] = sum(f) / len(f)
        if w:
            v["WRITE_SIZE_KB_avg"] = sum(w) / len(w)
        if f and w:
            v["hbm_bytes_per_launch"] = int(2 * v["FETCH_SIZE_KB_avg"] * 1024 + v["WRITE_SIZE_KB_avg"] * 1024)
        m, g = mfma.get(k), gui.get(k)
        if m and g:
            v["MFMA_BUSY_CYCLES_avg"] = sum(m) / len(m)
            v["GRBM_GUI_ACTIVE_avg"] = sum(g) / len(g)
    finish(kernels, a.workload, a.head, a.out)


def busy(v):
    return v["MFMA_BUSY_CYCLES_avg"] / (1024.0 * v["GRBM_GUI_ACTIVE_avg"] / 8.0)


def finish(kernels, workload, head, out_path):
    for v in kernels.values():
        if "MFMA_BUSY_CYCLES_avg" in v and v.get("GRBM_GUI_ACTIVE_avg"):
            v["mfma_busy"] = busy(v)
    stages = defaultdict(lambda: {"avg_us": 0.0, "kernels": []})
    # a stage's launch = its kernels that run every step: a kernel with fewer than half the calls of
    # the stage's most-called one ran only while priming / capturing (e.g. the step forward that
    # builds the first batch's indexer, before the pipelined steps' gather-only forwards)
    top = defaultdict(int)
    for v in kernels.values():
        if v["stage"] is not None:
            top[v["stage"]] = max(top[v["stage"]], v["calls"])
    for k, v in kernels.items():
        if v["stage"] is None or v["calls"] * 2 < top[v["stage"]]:
            continue
        s = stages[v["stage"]]
        s["avg_us"] += v["avg_us"]
        s["kernels"].append(k)
        if "hbm_bytes_per_launch" in v:
            s["hbm_bytes_per_launch"] = s.get("hbm_bytes_per_launch", 0) + v["hbm_bytes_per_launch"]
        if "mfma_busy" in v:
            s["mfma_busy"] = max(s.get("mfma_busy", 0.0), v["mfma_busy"])
    out = {"workload": workload, "head": head, "kernels": kernels, **{k: dict(v) for k, v in stages.items()}}
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    with open(out_path + ".json", "w") as f:
        json.dump(out, f, indent=1)
    lines = [f"# rocprofv3 summary — {workload} (library built at {head})", "",
             "| kernel | stage | calls | avg µs | min µs | FETCH_SIZE KB | WRITE_SIZE KB | HBM bytes/launch (2·F+W) | MFMA busy |",
             "|---|---|---|---|---|---|---|---|---|"]
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["avg_us"]):
        lines.append(f"| `{k}` | {v['stage']} | {v['calls']} | {v['avg_us']:.2f} | {v['min_us']:.2f} | "
                     f"{v.get('FETCH_SIZE_KB_avg', float('nan')):.0f} | {v.get('WRITE_SIZE_KB_avg', float('nan')):.0f} | "
                     f"{v.get('hbm_bytes_per_launch', '—')} | {v.get('mfma_busy', float('nan')):.3f} |")
    with open(out_path + ".md", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
