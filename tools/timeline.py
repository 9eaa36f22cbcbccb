"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV (dlrm kernels only).

    python tools/timeline.py DIR [--steps 3]
Prints, for the last few steps, each dlrm kernel's start/end relative to the step start and
the gaps between consecutive kernels, to show overlap and launch bubbles.
"""
import csv
import glob
import os
import re
import sys


def main():
    d = sys.argv[1]
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if "dlrm::" not in r["Kernel_Name"]:
                continue
            m = re.search(r"dlrm::([A-Za-z0-9_]+)", r["Kernel_Name"])
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1)))
    rows.sort()
    # a step starts at each fused-forward / lookup kernel
    starts = [i for i, r in enumerate(rows) if r[2] in ("interact_fwd_kernel", "maplookup_vec", "indexer_build_kernel")]
    firsts = []
    for i in starts:
        if not firsts or rows[i][0] - rows[firsts[-1]][0] > 20000:
            firsts.append(i)
    for s in range(max(0, len(firsts) - nsteps - 1), len(firsts) - 1):
        a, b = firsts[s], firsts[s + 1]
        t0 = rows[a][0]
        print(f"--- step (period {(rows[b][0] - t0) / 1e3:.1f} us)")
        for st, en, name in rows[a:b]:
            print(f"  {(st - t0) / 1e3:7.1f} -> {(en - t0) / 1e3:7.1f}  ({(en - st) / 1e3:6.1f})  {name}")


if __name__ == "__main__":
    main()
