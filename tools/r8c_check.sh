# pipelined forward (2 samples per wave) + pipelined step backward (2 samples per wave pair):
# probes, step parity tests, metric / bf16 / Terabyte bench (+ backward A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r8c; mkdir -p $O
timeout -k 10 200 tools/bin/fwd_probe > $O/fwd_probe.txt 2>&1 || { tail -20 $O/fwd_probe.txt; exit 1; }
cat $O/fwd_probe.txt
timeout -k 10 200 tools/bin/bwd_probe > $O/bwd_probe.txt 2>&1 || { tail -20 $O/bwd_probe.txt; exit 1; }
cat $O/bwd_probe.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fwd or step or lookup_interact or pipelined or bench" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --chain 0 --workload $1 > $O/bench_$1$2.json 2> $O/bench_$1$2.err || { tail $O/bench_$1$2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_$1$2.json')); print('$1$2', round(d['value']/1e6,3), d['ms_per_step'], d.get('sustained',{}).get('value'), {k: v['us'] for k, v in d['roofline']['stages'].items()})"; }
b kaggle-d128-b2048 || exit 1
DLRM_BWD_SPW=1 b kaggle-d128-b2048 _bwdspw1 || exit 1
b kaggle-d128-b8192-bf16 || exit 1
b terabyte-d128-bf16-zipf || exit 1
DLRM_BWD_SPW=1 b terabyte-d128-bf16-zipf _bwdspw1 || exit 1
