# bf16 one-hot forward at 4 waves per SIMD (default) vs 2 (the old launch bound): bf16 B=8192, Terabyte rows
set -o pipefail
O=gpurun_out/r6x; mkdir -p $O
run() {  # name, workload, env...
  local n=$1; shift; local wl=$1; shift
  env "$@" timeout -k 10 400 python bench.py --no-cpu-baseline --chain 0 --workload $wl > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,3), round(d['sustained']['value']/1e6,3) if d.get('sustained') else None, d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
}
run bf16_w4 kaggle-d128-b8192-bf16 X=1 && run bf16_w2 kaggle-d128-b8192-bf16 DLRM_HIP_LIB=$PWD/tools/bin/libdlrm_fw2.so &&
run tb_w4 terabyte-d128-bf16-zipf X=1 && run tb_w2 terabyte-d128-bf16-zipf DLRM_HIP_LIB=$PWD/tools/bin/libdlrm_fw2.so
