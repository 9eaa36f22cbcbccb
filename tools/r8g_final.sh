# round-3 final (resumed session, HEAD with the 16-B forward output stores): every BASELINE config's bench line (default flags) + the sharded simulation at world 8
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8g; mkdir -p $O
for w in kaggle-d128-b2048 kaggle-d16-b2048 kaggle-d128-b8192-bf16 terabyte-d128-bf16-zipf pooled-64x256-l10; do
  extra=""; [ $w = kaggle-d128-b2048 ] || extra="--no-cpu-baseline"
  timeout -k 10 400 python bench.py --workload $w $extra > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$w.json'));s=d.get('sustained');print('$w',round(d['value']/1e6,3),s and round(s['value']/1e6,3),d['ms_per_step'],{k:v['us'] for k,v in d['roofline']['stages'].items()}, d.get('drop_in_chain'))"
done
for m in 1 2; do
  timeout -k 10 150 python tools/shard_sim.py --micro $m > $O/shard_sim_w8_m$m.json 2> $O/shard_sim_w8_m$m.err || { tail $O/shard_sim_w8_m$m.err; exit 1; }
  cat $O/shard_sim_w8_m$m.json
done
# A/B: non-temporal 16-B forward output stores (exp/ntout)
for v in "" _ntout; do
  lib=""; [ -n "$v" ] && lib=exp/ntout/libdlrm_hip.so
  env ${lib:+DLRM_HIP_LIB=$lib} timeout -k 10 300 python bench.py --no-cpu-baseline --chain 0 > $O/ab$v.json 2> $O/ab$v.err || { tail $O/ab$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/ab$v.json'));print('ab$v',round(d['value']/1e6,3),d['ms_per_step'],{k:v['us'] for k,v in d['roofline']['stages'].items()})"
done
