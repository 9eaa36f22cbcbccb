# lookup NT-store A/B and the sharded step's launch-side time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6k}
mkdir -p $O
for v in base nt; do
  if [ $v = nt ]; then export DLRM_HIP_LIB=$PWD/tools/bin/libdlrm_nt.so; fi
  timeout -k 10 120 python tools/shard_sim.py --micro 1 > $O/ss_m1_$v.json 2> $O/ss_m1_$v.err || { tail $O/ss_m1_$v.err; exit 1; }
  echo $v; cat $O/ss_m1_$v.json
  timeout -k 10 240 python bench.py --no-cpu-baseline --chain 0 --workload pooled-64x256-l10 > $O/pooled_$v.json 2> $O/pooled_$v.err || { tail $O/pooled_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/pooled_$v.json')); print('pooled', d['value'], d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
done
