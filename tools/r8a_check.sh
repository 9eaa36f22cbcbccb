# round 3 (resumed): forward probe (MFMA / output cost), metric bench at HEAD
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8a; mkdir -p $O
timeout -k 10 200 tools/bin/fwd_probe > $O/fwd_probe.txt 2>&1 || { tail -20 $O/fwd_probe.txt; exit 1; }
cat $O/fwd_probe.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(round(d['value']/1e6,3), d['ms_per_step'], d.get('sustained',{}).get('value'), {k: v['us'] for k, v in d['roofline']['stages'].items()}, d.get('drop_in_chain',{}).get('value'))"
