# bf16 B=8192: backward samples-per-block knob
set -o pipefail
O=gpurun_out/r6o; mkdir -p $O
for v in 4 2 8; do
  DLRM_BWD_SPB=$v timeout -k 10 240 python bench.py --no-cpu-baseline --chain 0 --workload kaggle-d128-b8192-bf16 > $O/spb$v.json 2> $O/spb$v.err || { tail $O/spb$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/spb$v.json')); print('spb$v', d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
done
