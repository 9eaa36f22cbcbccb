# round-3 re-entry (re-created container, library rebuilt from HEAD): full GPU suite + smoke + default bench;
# A/B of the step indexer's digit width (DLRM_STEP_DB 8 default vs 9 / 10 in exp/db*)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r9; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --chain 0 --workload $1 > $O/bench_$1$2.json 2> $O/bench_$1$2.err || { tail $O/bench_$1$2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_$1$2.json')); print('$1$2', round(d['value']/1e6,3), d['ms_per_step'], d.get('sustained',{}).get('value'), {k: v['us'] for k, v in d['roofline']['stages'].items()})"; }
for W in kaggle-d128-b2048 kaggle-d16-b2048 terabyte-d128-bf16-zipf; do
  b $W || exit 1
  DLRM_HIP_LIB=exp/db9/libdlrm_hip.so b $W _db9 || exit 1
  DLRM_HIP_LIB=exp/db10/libdlrm_hip.so b $W _db10 || exit 1
done
