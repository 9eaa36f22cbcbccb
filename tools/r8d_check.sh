# forward: staged output row as 4-element stores (A/B against DLRM_FWD_VEC_OUT=0 in exp/novec)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8d; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fwd or step or lookup_interact or pipelined or bench or interact" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --chain 0 --workload $1 > $O/bench_$1$2.json 2> $O/bench_$1$2.err || { tail $O/bench_$1$2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_$1$2.json')); print('$1$2', round(d['value']/1e6,3), d['ms_per_step'], d.get('sustained',{}).get('value'), {k: v['us'] for k, v in d['roofline']['stages'].items()})"; }
for W in kaggle-d128-b2048 kaggle-d16-b2048 kaggle-d128-b8192-bf16; do
  b $W || exit 1
  DLRM_HIP_LIB=exp/novec/libdlrm_hip.so b $W _novec || exit 1
done
b kaggle-d128-b2048 _again || exit 1
