# backward: packed gradient row as 16-B loads (A/B against DLRM_BWD_VEC_PK=0 in exp/novpk); full GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8e; mkdir -p $O
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --chain 0 --workload $1 > $O/bench_$1$2.json 2> $O/bench_$1$2.err || { tail $O/bench_$1$2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_$1$2.json')); print('$1$2', round(d['value']/1e6,3), d['ms_per_step'], d.get('sustained',{}).get('value'), {k: v['us'] for k, v in d['roofline']['stages'].items()})"; }
for W in kaggle-d128-b2048 kaggle-d16-b2048 terabyte-d128-bf16-zipf; do
  b $W || exit 1
  DLRM_HIP_LIB=exp/novpk/libdlrm_hip.so b $W _novpk || exit 1
done
b kaggle-d128-b2048 _again || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
