#!/bin/bash
# Bench variants in one GPU session (launch mode x indexer overlap x fused forward).
set -o pipefail
mkdir -p gpurun_out
for mode in graph eager; do
  for ov in 1 0; do
    for fu in 1 0; do
      timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --mode $mode --overlap-indexer $ov --fused $fu \
        > gpurun_out/sweep_${mode}_ov${ov}_fu${fu}.json 2> gpurun_out/sweep_${mode}_ov${ov}_fu${fu}.err || exit $?
      python -c "import json,sys; d=json.load(open('gpurun_out/sweep_${mode}_ov${ov}_fu${fu}.json')); print('$mode ov=$ov fused=$fu', d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
    done
  done
done
