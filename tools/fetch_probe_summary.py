"""FETCH_SIZE (KB) per launch of tools/fetch_probe.hip's kernels against the bytes each requested.
usage: python tools/fetch_probe_summary.py PMC_DIR REQUESTED_JSON_LINE_FILE"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

pmc, req_file = sys.argv[1], sys.argv[2]
req = json.loads(open(req_file).read().strip().splitlines()[-1])
f = glob.glob(f"{pmc}/**/*counter_collection.csv", recursive=True)[0]
per = defaultdict(list)
for r in csv.DictReader(open(f)):
    if r["Counter_Name"] != "FETCH_SIZE":
        continue
    m = re.search(r"(stream_read|gather_rows<\d+>)", r["Kernel_Name"].replace("gather_rows<", "gather_rows<"))
    if m:
        per[m.group(1)].append(float(r["Counter_Value"]))
out = {}
for k, want in req.items():
    v = per.get(k)
    if not v:
        continue
    kb = sum(v) / len(v)
    out[k] = {"requested_bytes": want, "fetch_size_kb": round(kb, 1),
              "counter_bytes_over_requested": round(kb * 1024 / want, 3)}
print(json.dumps(out, indent=1))
