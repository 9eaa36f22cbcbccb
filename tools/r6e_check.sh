# round-3: forward bisect probe, the new GPU tests (drop-in chain, bench forms vs oracle, sharded
# micro-batches, ADVICE fixes), shard_sim at world 8, one default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6e}
mkdir -p $O
timeout -k 10 200 tools/bin/fwd_probe > $O/fwd_probe.txt 2>&1 || { tail -20 $O/fwd_probe.txt; exit 1; }
grep -i "body\|LIBRARY\|2 waves\|bisect" $O/fwd_probe.txt
timeout -k 10 700 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "drop_in or bench_form or sharded_two_ranks or terabyte or split_backward or unaligned" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for m in 1 2; do timeout -k 10 180 python tools/shard_sim.py --world 8 --micro $m > $O/shard_sim_w8_m$m.json 2> $O/shard_sim_w8_m$m.err || { tail $O/shard_sim_w8_m$m.err; exit 1; }; cat $O/shard_sim_w8_m$m.json; done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['sustained']['value'], d['drop_in_chain'], {k: v['us'] for k, v in d['roofline']['stages'].items()}, d['roofline']['step'])"
