# round-3: lookup kernel rework -- lookup/sharded/pooled GPU tests, shard_sim w8, pooled bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6j}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "lookup or pooled or sharded or fused or golden or blocked or comm" > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 120 python tools/shard_sim.py --micro 1 > $O/shard_sim_w8_m1.json 2> $O/shard_sim_w8_m1.err || { tail $O/shard_sim_w8_m1.err; exit 1; }
cat $O/shard_sim_w8_m1.json
timeout -k 10 120 python tools/shard_sim.py --micro 2 > $O/shard_sim_w8_m2.json 2> $O/shard_sim_w8_m2.err || { tail $O/shard_sim_w8_m2.err; exit 1; }
cat $O/shard_sim_w8_m2.json
timeout -k 10 240 python bench.py --no-cpu-baseline --chain 0 --workload pooled-64x256-l10 > $O/pooled.json 2> $O/pooled.err || { tail $O/pooled.err; exit 1; }
python -c "import json; d=json.load(open('$O/pooled.json')); print('pooled', d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
