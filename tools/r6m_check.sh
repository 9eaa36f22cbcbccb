# pooled apply with the XCD-contiguous item order: pooled tests, bench, FETCH_SIZE pass
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6m}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pooled or update or lookup_vs" > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 240 python bench.py --no-cpu-baseline --chain 0 --workload pooled-64x256-l10 > $O/pooled.json 2> $O/pooled.err || { tail $O/pooled.err; exit 1; }
python -c "import json; d=json.load(open('$O/pooled.json')); print('pooled', d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --workload pooled-64x256-l10 --steps 10 --warmup 3 --no-cpu-baseline --sustain 0 --chain 0 > $O/fetch.log 2>&1 || { tail $O/fetch.log; exit 1; }
python3 - <<PY
import csv, glob, collections
f = glob.glob("$O/fetch/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:70]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]) / len(kv[1])):
    print(f"{k:70s} n={len(v):4d} FETCH_KB/launch={sum(v)/len(v):12.0f}")
PY
