# apply launch carrying the next batch's indexer: apply grid shrunk by the build's workgroups (A/B)
set -o pipefail
O=gpurun_out/r6u; mkdir -p $O
run() {  # name, workload, env...
  local n=$1; shift; local wl=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --chain 0 --workload $wl > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,2), round(d['sustained']['value']/1e6,2), d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
}
run d128_base kaggle-d128-b2048 X=1 && run d128_shrink kaggle-d128-b2048 DLRM_APPLY_SHRINK=1 &&
run d16_base kaggle-d16-b2048 X=1 && run d16_shrink kaggle-d16-b2048 DLRM_APPLY_SHRINK=1 &&
run d128_base2 kaggle-d128-b2048 X=1 && run d128_shrink2 kaggle-d128-b2048 DLRM_APPLY_SHRINK=1
