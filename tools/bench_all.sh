#!/bin/bash
# One bench.py line per BASELINE config into gpurun_out/<tag>_bench_<workload>.json, each step
# under its own time limit; stops at the first failure.  usage: tools/bench_all.sh TAG
set -o pipefail
TAG=${1:?tag}
mkdir -p gpurun_out
for w in kaggle-d128-b2048 kaggle-d16-b2048 kaggle-d128-b8192-bf16 terabyte-d128-bf16-zipf pooled-64x256-l10; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/${TAG}_bench_$w.json || { echo "bench $w failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$w.json'));s=d['sustained'];print('$w',d['value'],s and s['value'],d['ms_per_step'],{k:v['us'] for k,v in d['roofline']['stages'].items()})"
done
