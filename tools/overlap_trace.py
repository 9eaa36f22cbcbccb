"""Do kernels of parallel hipGraph branches overlap?  Reads a rocprofv3 --kernel-trace CSV, splits
it into segments at idle gaps (> 5 ms: the probes sleep between configurations) and reports, per
segment: kernels, the union of their busy intervals, the summed durations, and the time during
which >= 2 kernels ran at once (0 = the branches ran in series), with the queue / stream ids the
kernels were dispatched on.

    python tools/overlap_trace.py TRACE_DIR_OR_CSV [--names a,b]"""
import csv
import glob
import os
import re
import sys


def load(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            m = re.search(r"([A-Za-z_][A-Za-z0-9_]*)(?:<|\()", r["Kernel_Name"])
            name = m.group(1) if m else r["Kernel_Name"][:40]
            q = r.get("Queue_Id", r.get("Queue_ID", "?"))
            st = r.get("Stream_Id", r.get("Stream_ID", "?"))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q, st))
    rows.sort()
    return rows


def segments(rows, gap_ns=5_000_000):
    seg, end = [], None
    for r in rows:
        if end is not None and r[0] - end > gap_ns:
            yield seg
            seg = []
        seg.append(r)
        end = r[1] if end is None else max(end, r[1])
    if seg:
        yield seg


def overlap_stats(seg):
    ev = sorted([(s, 1) for s, e, *_ in seg] + [(e, -1) for s, e, *_ in seg])
    busy = multi = 0
    cur, last = 0, ev[0][0]
    for t, d in ev:
        if cur >= 1:
            busy += t - last
        if cur >= 2:
            multi += t - last
        cur += d
        last = t
    total = sum(e - s for s, e, *_ in seg)
    return busy, multi, total


def main():
    rows = load(sys.argv[1])
    for i, seg in enumerate(segments(rows)):
        busy, multi, total = overlap_stats(seg)
        names = {}
        for s, e, n, q, st in seg:
            d = names.setdefault(n, [0, 0, set(), set()])
            d[0] += 1
            d[1] += e - s
            d[2].add(q)
            d[3].add(st)
        span = seg[-1][1] - seg[0][0]
        print(f"segment {i}: {len(seg)} kernels over {span / 1e3:.1f} us; busy (union) {busy / 1e3:.1f} us, "
              f"summed durations {total / 1e3:.1f} us, >= 2 kernels at once {multi / 1e3:.1f} us "
              f"({100.0 * multi / max(busy, 1):.1f} % of busy)")
        for n, (c, t, qs, ss) in sorted(names.items(), key=lambda kv: -kv[1][1]):
            print(f"    {n:40s} x{c:4d}  avg {t / c / 1e3:7.2f} us  queues {sorted(qs)} streams {sorted(ss)}")


if __name__ == "__main__":
    main()
