# materialized-ys backward on the split kernel (33 <= F <= 96): tests, pooled bench A/B
set -o pipefail
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "interaction or ys_backward or pooled or fused" > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --chain 0 --workload pooled-64x256-l10 > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,3), d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
}
run ys_split X=1 && run bwd_body DLRM_BWD_YS=0
