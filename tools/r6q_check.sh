# bf16 d=128 split backward with 8 columns per lane: bf16 step tests, then bench A/B (CPL, SPB)
set -o pipefail
O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bf16 or step or bench_form or terabyte or blocked or sharded" > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --chain 0 --workload kaggle-d128-b8192-bf16 > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['value']/1e6,2), d['ms_per_step'], {k: v['us'] for k, v in d['roofline']['stages'].items()})"
}
run cpl4_spb2 DLRM_BWD_CPL=4 DLRM_BWD_SPB=2 && run cpl8_spb4 DLRM_BWD_CPL=8 && run cpl8_spb2 DLRM_BWD_SPB=2 && run cpl8_spb8 DLRM_BWD_SPB=8
