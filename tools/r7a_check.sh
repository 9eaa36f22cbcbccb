# bf16 B=8192 8-column backward with plain dt stores: bench + WRITE_SIZE pass
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r7a; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --chain 0 --workload kaggle-d128-b8192-bf16 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(round(d['value']/1e6,3), d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 bench.py --workload kaggle-d128-b8192-bf16 --steps 10 --warmup 3 --no-cpu-baseline --sustain 0 --chain 0 > $O/w.log 2>&1 || { tail $O/w.log; exit 1; }
python3 - <<PY
import csv, glob, collections
f = glob.glob("$O/w/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "dlrm::" in r["Kernel_Name"]: acc[r["Kernel_Name"][:80]].append(float(r["Counter_Value"]))
for k, v in acc.items(): print(f"{k:80s} n={len(v):4d} WRITE_KB={sum(v)/len(v):10.0f}")
PY
rm -rf $O/w
