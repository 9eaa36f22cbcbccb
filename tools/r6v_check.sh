# hot-slice size A/B (kHotSlice 128 default, 256, 64) on the metric, D=16, bf16 B=8192 and pooled
set -o pipefail
O=gpurun_out/r6v; mkdir -p $O
run() {  # name, workload, env...
  local n=$1; shift; local wl=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --chain 0 --workload $wl > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,3), round(d['sustained']['value']/1e6,3) if d.get('sustained') else None, d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
}
for wl in kaggle-d128-b2048 kaggle-d16-b2048 kaggle-d128-b8192-bf16; do
  run ${wl}_128 $wl X=1 && run ${wl}_256 $wl DLRM_HIP_LIB=$PWD/tools/bin/libdlrm_hs256.so && run ${wl}_64 $wl DLRM_HIP_LIB=$PWD/tools/bin/libdlrm_hs64.so || exit 1
done
run pooled_128 pooled-64x256-l10 X=1 && run pooled_256 pooled-64x256-l10 DLRM_HIP_LIB=$PWD/tools/bin/libdlrm_hs256.so
