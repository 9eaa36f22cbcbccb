# metric backward block size A/B; Terabyte-rows bf16 bench with the 8-column backward
set -o pipefail
O=gpurun_out/r6s; mkdir -p $O
run() {  # name, workload, env...
  local n=$1; shift; local wl=$1; shift
  env "$@" timeout -k 10 400 python bench.py --no-cpu-baseline --chain 0 --workload $wl > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,2), round(d['sustained']['value']/1e6,2), d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
}
run d128_spb4 kaggle-d128-b2048 X=1 && run d128_spb2 kaggle-d128-b2048 DLRM_BWD_SPB=2 && run d128_spb8 kaggle-d128-b2048 DLRM_BWD_SPB=8 &&
run tb_cpl8 terabyte-d128-bf16-zipf X=1 && run tb_cpl4 terabyte-d128-bf16-zipf DLRM_BWD_CPL=4 DLRM_BWD_SPB=4
